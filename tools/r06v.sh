#!/bin/bash
# C4 initial-cell launch orders (BCM3_CP_ORDER at the measuring commit: 1 Morton, 2 Hilbert, 3 / 4 by one variability
# dimension, 0 cell order), interleaved; the queue path
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for r in 1 2; do
  for o in 1 2 3 4 0; do
    out=$(BCM3_CP_ORDER=$o timeout -k 10 200 python tools/cellpop_bench.py 64 5 2>/dev/null | tr '\n' ' ')
    echo "round $r [order $o] $out"
  done
done
