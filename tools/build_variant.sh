#!/bin/bash
# Build a variant of libbcm3hip.so with extra compiler flags into build/var/<name>.so
#   tools/build_variant.sh name [-DFOO ...]      (SRC=<dir>: build from a copy of csrc, e.g. an older revision;
#                                                 NOSKIP=1: without -structurizecfg-skip-uniform-regions)
set -e
name=$1; shift
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT/bcm3_amd/csrc"
make -s ../../build/obj/cellpop_embed.inc
mkdir -p "$ROOT/varlib"
cd "${SRC:-$ROOT/bcm3_amd/csrc}"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -mllvm -simplifycfg-sink-common=false \
  $([ -z "$NOSKIP" ] && echo -mllvm -structurizecfg-skip-uniform-regions) -w -I"$ROOT/build/obj" "$@" -shared -o "$ROOT/varlib/$name.so" \
  popk_kernel.hip expm_pk_kernel.hip analytic_kernel.hip pt_kernels.hip proposal_kernels.hip runtime.hip \
  cellpop_kernels.hip bcm3hip_api.cpp cellpop_rt.cpp libm_tables.cpp -L/opt/rocm/lib -lrccl -lhiprtc
