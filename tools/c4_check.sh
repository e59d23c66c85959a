# C4 check: cell-population GPU parity tests, the sampler output test, and the C4 timing
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-c4}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_cellpop_gpu.py "tests/test_ptmh_native_gpu.py::test_sample_output_file" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python tools/cellpop_bench.py 64 5 > $O/bench.txt 2>&1
cat $O/bench.txt
BCM3_CP_PHASES=1 timeout -k 10 200 python tools/cellpop_phases.py 16 > $O/phases.txt 2>&1
cat $O/phases.txt
