"""Static ISA statistics of the BDF kernels (instruction mix, code size) from a device-only -S build.

    python tools/isa_stats.py [pattern]      (default pattern: popk_traj_kernelILi1E = TWO model)
"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "bcm3_amd", "csrc")


def build_asm(out="/tmp/popk_kernel.s"):
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", "-ffp-contract=off", "-mllvm", "-simplifycfg-sink-common=false", "-mllvm", "-structurizecfg-skip-uniform-regions",
                    "-o", out, os.path.join(CSRC, "popk_kernel.hip")], check=True)
    return out


def functions(asm):
    cur, body = None, []
    for line in open(asm):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur and line.strip().startswith(".Lfunc_end"):
            yield cur, body
            cur = None
            continue
        if cur:
            body.append(line)


def stats(body):
    c = collections.Counter()
    nbytes = 0
    for line in body:
        s = line.strip()
        if not s or s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        op = s.split()[0]
        c["total"] += 1
        if op.startswith("v_"):
            c["valu"] += 1
            if "_f64" in op:
                c["valu_f64"] += 1
            if op.startswith("v_cndmask"):
                c["v_cndmask"] += 1
            if op.startswith("v_cmp"):
                c["v_cmp"] += 1
            if "readfirstlane" in op or "readlane" in op:
                c["readlane"] += 1
            if "accvgpr" in op:
                c["accvgpr"] += 1
        elif op.startswith("s_"):
            c["salu_or_ctrl"] += 1
            if op.startswith("s_cbranch"):
                c["s_cbranch"] += 1
            if "saveexec" in op or "exec" in s.split(",")[0]:
                c["exec_ops"] += 1
            if op.startswith("s_waitcnt"):
                c["s_waitcnt"] += 1
            if op.startswith("s_load") or op.startswith("s_buffer_load"):
                c["s_load"] += 1
        elif op.startswith(("global_", "buffer_", "flat_", "scratch_")):
            c["vmem"] += 1
            if op.startswith("scratch_") or "buffer_store" in op and "off" in s:
                c["scratch"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
    return c


def main():
    pat = sys.argv[1] if len(sys.argv) > 1 else "popk_traj_kernelILi1E"
    asm = build_asm()
    for name, body in functions(asm):
        if pat in name:
            c = stats(body)
            print(name[:90])
            print("   " + ", ".join(f"{k}={v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
