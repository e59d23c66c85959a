set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
export BCM3_PARITY_LOG=$O/parity.jsonl
timeout -k 10 600 python -u -m pytest tests/test_ptmh_native_gpu.py tests/test_refbind.py -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || true
grep -E "passed|failed" $O/pytest_gpu.log | tail -3
grep -E "FAILED|ERROR|^E " $O/pytest_gpu.log | head -20
timeout -k 10 400 python tools/spec_sim.py > $O/spec_sim.txt 2>&1 || echo spec_sim failed
tail -12 $O/spec_sim.txt
