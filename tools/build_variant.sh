#!/bin/bash
# Build a variant of libbcm3hip.so with extra compiler flags into build/var/<name>.so
#   tools/build_variant.sh name [-DFOO ...]
set -e
name=$1; shift
cd "$(dirname "$0")/../bcm3_amd/csrc"
mkdir -p ../../build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -mllvm -simplifycfg-sink-common=false \
  -mllvm -structurizecfg-skip-uniform-regions -w "$@" -shared -o ../../build/var/$name.so \
  popk_kernel.hip analytic_kernel.hip pt_kernels.hip proposal_kernels.hip bcm3hip_api.cpp
