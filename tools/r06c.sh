#!/bin/bash
# round 6, lease c: cell-population GPU tests (LOGP_REL 1e-5, DP5 on glibc's pow), smoke, the
# bench's kernel trace (csv)
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06c; mkdir -p $O
export BCM3_PARITY_LOG=$O/parity.jsonl
rc=0
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_cellpop_gpu.py \
  tests/test_cellpop_sync_gpu.py tests/test_cellpop_dp5_gpu.py tests/test_cellpop_lineage_gpu.py tests/test_timecourse_gpu.py \
  tests/test_timepoints_gpu.py tests/test_cellpop_experiments_gpu.py > $O/pytest_cp.log 2>&1 || rc=$?
grep -E "FAILED|passed|failed" $O/pytest_cp.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 40 --warmup 4 --cpu-seconds 0 --throughput-batch 0 --extras 0 --issue-probe 0 --strong-chains 0 > $O/kt.log 2>&1
f=$(find $O/kt -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for r in csv.reader(open('$f')):
    print(r[0][:60], r[1], r[3])
"
exit $rc
