#!/bin/bash
# The C3 bench line (speculative pairs, C++ sampler) with several C3-only library builds swapped in
# for bcm3_amd/lib/libbcm3hip.so (on the GPU box's copy of the tree), interleaved over ROUNDS:
#   ROUNDS=2 bash tools/bench_variants.sh varlib/a.so varlib/b.so ...
set -e
cd "$GRAFT_REPO_ROOT"
cp bcm3_amd/lib/libbcm3hip.so /tmp/libbcm3hip_product.so
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    cp "$lib" bcm3_amd/lib/libbcm3hip.so
    out=$(timeout -k 10 300 python bench.py --steps 60 --warmup 6 --cpu-seconds 0 --extras 0 --throughput-batch 0 \
          --issue-probe 0 --strong-chains 0 2>/dev/null | tail -1)
    python3 -c "import json,sys; d=json.loads(sys.argv[1]); print(f'round $r {sys.argv[2]:24s} value {d[\"value\"]:9.0f} ms/step {d[\"ms_per_step\"]:.4f} kernel {d[\"roofline\"][\"kernel_ms_avg\"]:.4f} ms')" "$out" "$(basename $lib)"
  done
done
cp /tmp/libbcm3hip_product.so bcm3_amd/lib/libbcm3hip.so
