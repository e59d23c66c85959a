set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
export BCM3_PARITY_LOG=$O/parity.jsonl
timeout -k 10 300 python -u -m pytest tests/test_popk_gpu.py tests/test_pt_gpu.py -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || true
grep -E "passed|failed" $O/pytest_gpu.log | tail -3
cat $O/parity.jsonl | grep -v pk_single
timeout -k 10 400 python tools/spec_sim.py > $O/spec_sim.txt 2>&1 || echo spec_sim failed
cat $O/spec_sim.txt
