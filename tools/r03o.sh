cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ptmh_native_gpu.py -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
grep -E "large_batches|passed|failed" $O/pytest_gpu.log | tail -4
timeout -k 10 300 python bench.py --steps 60 --warmup 6 --cpu-seconds 0 --throughput-batch 0 --extras 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
timeout -k 10 300 python bench.py --chains 512 --steps 30 --warmup 4 --cpu-seconds 0 --throughput-batch 0 --extras 0 > $O/bench512.json 2> $O/bench512.err || { tail -20 $O/bench512.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench512.json')); print('bench512', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['config']['sampler_loop'])"
