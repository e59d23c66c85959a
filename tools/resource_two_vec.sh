#!/bin/bash
# Register / scratch usage of the C3 kernel (popk_traj_kernel<TWO, VEC, false>) alone, in seconds:
#   tools/resource_two_vec.sh [extra hipcc flags]      (HIPFLAGS as bcm3_amd/csrc/Makefile)
set -e
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "$ROOT/bcm3_amd/csrc"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -mllvm -simplifycfg-sink-common=false \
  ${NOSKIP:+} $([ -z "$NOSKIP" ] && echo -mllvm -structurizecfg-skip-uniform-regions) -w -DBCM3_DEV_TWO_VEC "$@" \
  --offload-device-only -c -Rpass-analysis=kernel-resource-usage -o /tmp/popk_two_vec.o popk_kernel.hip 2>&1 |
  grep -A7 "Function Name: _ZN7bcm3hip16popk_traj_kernelILi1ELi2ELb0E" | grep -E "VGPRs:|SGPRs:|Scratch|Occupancy" | sed 's/.*remark: *//'
