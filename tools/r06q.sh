#!/bin/bash
# The C4 work queue on the GPU: bit-identity and time against the generation launches, a grid sweep,
# kernel trace of both paths (profiles/r06q_*)
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/r06q${TAG:-}; mkdir -p $O
BCM3_CP_QUEUE_VERBOSE=1 timeout -k 10 200 python -u tools/c4_queue_check.py 64 5 > $O/check.log 2>&1
for g in ${GRIDS:-1024 1536}; do
  BCM3_CP_QUEUE_GRID=$g timeout -k 10 200 python -u tools/c4_queue_check.py 64 3 > $O/grid_$g.log 2>&1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o q -- python3 tools/c4_queue_check.py 64 3 > $O/prof.log 2>&1
