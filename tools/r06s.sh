#!/bin/bash
# C4 work-queue variants (BCM3_CP_OPTS), interleaved, with the queue's packing statistics
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
for r in 1 2; do
  out=$(BCM3_CP_QUEUE=0 timeout -k 10 200 python tools/cellpop_bench.py 64 5 2>/dev/null | tr '\n' ' ')
  echo "round $r [generation launches] $out"
  for v in "" "-DCP_QUEUE_FILL_WAIT=64" "-DCP_QUEUE_FILL_WAIT=1024"; do
    out=$(BCM3_CP_QUEUE_VERBOSE=1 BCM3_CP_OPTS="$v" timeout -k 10 200 python tools/cellpop_bench.py 64 5 2>&1 | grep -E "n=64|checksum|work queue:" | sort | uniq -c | tr '\n' ' ')
    echo "round $r [queue ${v:-product}] $out"
  done
done
