#!/bin/bash
# Build a variant of libbcm3hip.so with extra compiler flags into build/var/<name>.so
#   tools/build_variant.sh name [-DFOO ...]
set -e
name=$1; shift
cd "$(dirname "$0")/../bcm3_amd/csrc"
mkdir -p ../../varlib
make -s ../../build/obj/cellpop_embed.inc
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -mllvm -simplifycfg-sink-common=false \
  -mllvm -structurizecfg-skip-uniform-regions -w -I../../build/obj "$@" -shared -o ../../varlib/$name.so \
  popk_kernel.hip expm_pk_kernel.hip analytic_kernel.hip pt_kernels.hip proposal_kernels.hip runtime.hip \
  cellpop_kernels.hip bcm3hip_api.cpp cellpop_rt.cpp -L/opt/rocm/lib -lrccl -lhiprtc
