set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
export BCM3_PARITY_LOG=$O/parity.jsonl
timeout -k 10 600 python -u -m pytest tests/test_ptmh_native_gpu.py tests/test_proposal_gpu.py tests/test_popk_gpu.py tests/test_refbind.py -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || true
grep -E "passed|failed" $O/pytest_gpu.log | tail -3
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
timeout -k 10 300 python bench.py --steps 40 --warmup 4 --cpu-seconds 0 --throughput-batch 0 --extras 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
