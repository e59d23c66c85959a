#!/bin/bash
# Device assembly of the C3 kernel alone (popk_traj_kernel<TWO, VEC, false>, -DBCM3_DEV_TWO_VEC) with the
# library's flags plus any given, and its spill / register summary:
#   tools/isa_dev.sh out.s [extra hipcc flags]      (SRC=<dir>: another csrc copy)
set -e
out=$1; shift
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
cd "${SRC:-$ROOT/bcm3_amd/csrc}"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -ffp-contract=off \
  -mllvm -simplifycfg-sink-common=false -mllvm -structurizecfg-skip-uniform-regions -w -DBCM3_DEV_TWO_VEC "$@" \
  -o "$out" popk_kernel.hip
python3 - "$out" <<'PY'
import re, sys, collections, os
body, on = [], False
for l in open(sys.argv[1]):
    if re.match(r"^_ZN7bcm3hip16popk_traj_kernelILi1ELi2ELb" + os.environ.get("STATSK", "0") + r"E\S*:", l): on = True; continue
    if on and re.match(r"^\s*\.Lfunc_end", l): break
    if on: body.append(l)
ins = [l.split()[0] for l in body if l.startswith("\t") and not l.strip().startswith((".", ";"))]
c = collections.Counter(ins)
meta = open(sys.argv[1]).read()
m = re.search(r"\.amdhsa_kernel _ZN7bcm3hip16popk_traj_kernelILi1ELi2ELb" + os.environ.get("STATSK", "0") + r"E.*?\.end_amdhsa_kernel", meta, re.S)
kv = dict(re.findall(r"\.amdhsa_(next_free_vgpr|next_free_sgpr|private_segment_fixed_size)\s+(\d+)", m.group(0))) if m else {}
print(f"instr {len(ins)} v_readlane {c['v_readlane_b32']} v_writelane {c['v_writelane_b32']} readfirstlane {c['v_readfirstlane_b32']} "
      f"scratch ops {sum(v for k, v in c.items() if k.startswith('scratch_') or k.startswith('buffer_'))} {kv}")
PY
