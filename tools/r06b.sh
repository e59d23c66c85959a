#!/bin/bash
# round 6, lease b: C4 run-to-run determinism; the cell-population GPU tests under the measured bar
# (round 6) with the parity log; the PopPK GPU tests (lane-0 stores)
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06b; mkdir -p $O
export BCM3_PARITY_LOG=$O/parity.jsonl
timeout -k 10 200 python tools/c4_determinism.py $O/c4_a.npy > $O/det.txt 2>&1
timeout -k 10 200 python tools/c4_determinism.py $O/c4_b.npy $O/c4_a.npy >> $O/det.txt 2>&1
cat $O/det.txt
rc=0
timeout -k 10 1200 python -u -m pytest -v --timeout 400 --timeout-method thread tests/test_cellpop_gpu.py \
  tests/test_cellpop_sync_gpu.py tests/test_cellpop_dp5_gpu.py tests/test_cellpop_lineage_gpu.py tests/test_timecourse_gpu.py \
  tests/test_timepoints_gpu.py tests/test_cellpop_experiments_gpu.py > $O/pytest_cp.log 2>&1 || rc=$?
tail -30 $O/pytest_cp.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_popk_gpu.py > $O/pytest_popk.log 2>&1 || { tail -40 $O/pytest_popk.log; exit 1; }
tail -3 $O/pytest_popk.log
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ptmh_native_gpu.py tests/test_pt_gpu.py > $O/pytest_pt.log 2>&1 || { tail -40 $O/pytest_pt.log; exit 1; }
tail -3 $O/pytest_pt.log
timeout -k 10 300 python bench.py --steps 60 --warmup 6 --cpu-seconds 0 --extras 0 --throughput-batch 0 --issue-probe 0 --strong-chains 0 > $O/bench_short.json 2> $O/bench_short.err
python3 -c "import json; d=json.load(open('$O/bench_short.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['kernel_share_of_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof -- python3 bench.py --steps 20 --warmup 4 --cpu-seconds 0 --extras 0 --throughput-batch 0 --issue-probe 0 --strong-chains 0 > $O/prof.log 2>&1
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats.csv
python3 -c "
import csv
for r in csv.reader(open('$O/kernel_stats.csv')):
    print(r[0][:70], r[1], r[3])
"
exit $rc
