#!/bin/bash
# round 6, lease d: sampler GPU tests (the scatter folded into the first commit), the bench's kernel
# trace (csv) and a short bench line
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-r06d}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ptmh_native_gpu.py tests/test_pt_gpu.py tests/test_ptmh_multiprocess_gpu.py > $O/pytest_pt.log 2>&1 || { tail -40 $O/pytest_pt.log; exit 1; }
tail -1 $O/pytest_pt.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 40 --warmup 4 --cpu-seconds 0 --throughput-batch 0 --extras 0 --issue-probe 0 --strong-chains 0 > $O/kt.log 2>&1
f=$(find $O/kt -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv
for r in csv.reader(open('$f')):
    print(r[0][:60], r[1], r[3])
"
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 60 --warmup 6 --cpu-seconds 0 --extras 0 --throughput-batch 0 --issue-probe 0 --strong-chains 0 > $O/bench_short$i.json 2> $O/bench_short.err
python3 -c "import json; d=json.load(open('$O/bench_short$i.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['kernel_share_of_step'])"
done
timeout -k 10 200 python -c "
import json, torch, bench
print('circular in sampler', json.dumps(bench.circular_in_sampler(torch.device('cuda', 0), 1)))" > $O/c2_in_sampler.txt 2>&1 || true
tail -1 $O/c2_in_sampler.txt
if [ -f gpuvar/uni_cold.so ]; then
  timeout -k 10 600 python tools/flag_diff.py gpuvar/product.so gpuvar/uni_cold.so > $O/flag_diff.txt 2>&1
  tail -4 $O/flag_diff.txt
fi
if [ -n "$C4P3" ]; then
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 --output-format csv -d $O/c4p3 -o pmc -- python3 tools/cellpop_bench.py 64 2 > $O/c4p3.log 2>&1 || echo "c4 p3 pass failed"
  tail -3 $O/c4p3.log
fi
