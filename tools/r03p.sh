cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
export BCM3_PARITY_LOG=$O/parity.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python tools/variant_timing.py varlib/new_plain.so varlib/simple.so varlib/new_plain.so varlib/simple.so varlib/new_plain.so varlib/simple.so
timeout -k 10 300 python bench.py --steps 60 --warmup 6 --cpu-seconds 0 --throughput-batch 0 --extras 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
