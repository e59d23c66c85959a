#!/bin/bash
# C4 generation launches: daughters in their mothers' launch order vs sister pairs shuffled
# (BCM3_CP_SHUFFLE_PAIRS=1): how much the grouping of daughters into wavefronts matters
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for r in 1 2; do
  for sh in 0 1; do
    out=$(BCM3_CP_QUEUE=0 BCM3_CP_SHUFFLE_PAIRS=$sh timeout -k 10 200 python tools/cellpop_bench.py 64 5 2>/dev/null | tr '\n' ' ')
    echo "round $r [shuffle pairs $sh] $out"
  done
  out=$(timeout -k 10 200 python tools/cellpop_bench.py 64 5 2>/dev/null | tr '\n' ' ')
  echo "round $r [queue] $out"
done
