#!/bin/bash
# C4 generation launches: daughters by their mothers' launch order (product) vs along a Morton curve of
# their own variability points (BCM3_CP_DAUGHTER_MORTON=1); kernel time from the trace (host sort excluded)
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06u; mkdir -p $O
for dm in 0 1; do
  BCM3_CP_QUEUE=0 BCM3_CP_DAUGHTER_MORTON=$dm timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/dm$dm -o t -- python3 tools/cellpop_bench.py 64 5 > $O/dm$dm.log 2>&1
  grep -h "n=64\|checksum" $O/dm$dm.log
done
