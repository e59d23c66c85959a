#!/bin/bash
# GPU tests (+ parity summary log) and the default bench line into gpurun_out/$TAG.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r03}
O=gpurun_out/$TAG
mkdir -p $O
export BCM3_PARITY_LOG=$O/parity.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
if [ -z "$NOBENCH" ]; then
  timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
  cat $O/bench.json | head -c 1500
fi
