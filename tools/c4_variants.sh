#!/bin/bash
# A/B of hipRTC options of the C4 cell kernel (BCM3_CP_OPTS), interleaved over ROUNDS, each in its own
# process: ms per 64-evaluation batch and the logp checksum (bit-identical variants keep it)
#   VARIANTS="|-DCP_LANE_OPAQUE|..." ROUNDS=2 bash tools/c4_variants.sh    ('' = the product build)
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
IFS='|' read -ra VS <<< "${VARIANTS:-|-DCP_LANE_OPAQUE}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "${VS[@]}"; do
    out=$(BCM3_CP_OPTS="$v" timeout -k 10 200 python tools/cellpop_bench.py 64 5 2>/dev/null | tr '\n' ' ')
    echo "round $r [${v:-product}] $out"
  done
done
