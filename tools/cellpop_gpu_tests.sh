# the cell-population GPU tests (single and several experiments)
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-cpt}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cellpop_experiments_gpu.py tests/test_cellpop_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
