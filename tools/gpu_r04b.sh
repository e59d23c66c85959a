set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r04b; mkdir -p $O
export BCM3_PARITY_LOG=$O/parity.jsonl
timeout -k 10 600 python -u -m pytest tests/test_popk_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_popk.log 2>&1 || { tail -30 $O/pytest_popk.log; exit 1; }
tail -3 $O/pytest_popk.log
timeout -k 10 300 python tools/bitexact_probe.py 4096 > $O/bitexact.txt 2>&1; cat $O/bitexact.txt
