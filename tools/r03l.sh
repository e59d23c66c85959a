cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
export BCM3_PARITY_LOG=$O/parity.jsonl
timeout -k 10 900 python -u -m pytest tests/test_cellpop_gpu.py tests/test_cellpop_experiments_gpu.py -v --timeout 600 --timeout-method thread > $O/pytest_cellpop.log 2>&1 || { grep -E "FAILED|Error|error|assert" $O/pytest_cellpop.log | head -30; tail -5 $O/pytest_cellpop.log; exit 1; }
tail -2 $O/pytest_cellpop.log
timeout -k 10 300 python tools/cellpop_bench.py > $O/cellpop_bench.txt 2>&1 || { tail -20 $O/cellpop_bench.txt; exit 1; }
tail -5 $O/cellpop_bench.txt
