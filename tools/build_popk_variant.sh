#!/bin/bash
# A variant of libbcm3hip.so that differs only in popk_kernel.hip (extra compiler flags or SRC=<dir>
# with another popk_kernel.hip / solver headers), linked with the product's other objects
# (bcm3_amd/csrc/Makefile must have built build/obj first) into varlib/<name>.so:
#   tools/build_popk_variant.sh name [-DFOO | -mllvm -opt=...]     (NOSKIP=1: without
#   -structurizecfg-skip-uniform-regions)
set -e
name=$1; shift
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OBJ="$ROOT/build/obj"
mkdir -p "$ROOT/varlib" "$OBJ/var"
cd "${SRC:-$ROOT/bcm3_amd/csrc}"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -mllvm -simplifycfg-sink-common=false \
  $([ -z "$NOSKIP" ] && echo -mllvm -structurizecfg-skip-uniform-regions) -w "$@" -c -o "$OBJ/var/popk_$name.o" popk_kernel.hip
others=$(ls "$OBJ"/*.o | grep -v '/popk_kernel.hip.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/varlib/$name.so" "$OBJ/var/popk_$name.o" $others \
  -L/opt/rocm/lib -lrccl -lhiprtc
echo "built varlib/$name.so"
