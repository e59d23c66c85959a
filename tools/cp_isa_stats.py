"""Static instruction categories of the C4 cell kernel (cp_solve_kernel) by loop depth.

    BCM3_CP_DUMP=/tmp/cp_model.hip <create the C4 likelihood>    (cellpop_rt.cpp writes its program text)
    python tools/cp_isa_stats.py /tmp/cp_model.hip [kernel]    (kernel: cp_solve_kernel, or cp_queue_kernel
                                                                of a BCM3_CP_QUEUE=1 dump)

Compiles the dumped hipRTC program with the runtime's options (hipcc --cuda-device-only -S) and splits
cp_solve_kernel's instructions by the loop depth LLVM annotates (1: the cell driver's step loop, 2: the
attempt loop, 3: the Newton iteration) into: FP64 arithmetic, selects (v_cndmask), moves and DPP
broadcasts, SGPR spill moves (v_readlane / v_writelane into VGPR lanes), compares, other VALU, LDS and
scratch operations. Static counts: which code a step runs is decided at run time (profiles/
r06f_pmc_c4.json has the dynamic totals).
"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def category(op):
    if op in ("v_readlane_b32", "v_writelane_b32"):
        return "sgpr spill moves"
    if re.match(r"v_(add|mul|fma|fmac|div_scale|div_fmas|div_fixup|rcp|rsq|sqrt|ldexp|frexp|max|min|trig|fract)_f64", op):
        return "fp64 arithmetic"
    if op.startswith("v_cndmask"):
        return "selects"
    if op.startswith("v_mov") or op.startswith("v_accvgpr"):
        return "moves / dpp"
    if op.startswith("v_cmp"):
        return "compares"
    if op.startswith("v_"):
        return "other valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("scratch_") or op.startswith("buffer_"):
        return "scratch"
    if op.startswith("s_"):
        return "scalar"
    return "memory / other"


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else "/tmp/cp_model.hip"
    asm = "/tmp/cp_isa_stats.s"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-ffp-contract=off", "-DBCM3_CORRECTLY_ROUNDED", "-I" + os.path.join(ROOT, "bcm3_amd", "csrc"), "-w",
                    "-o", asm, src], check=True)
    lines = open(asm).read().split("\n")
    kernel = sys.argv[2] if len(sys.argv) > 2 else "cp_solve_kernel"
    start = next(i for i, l in enumerate(lines) if l.startswith(kernel + ":"))
    end = next(i for i, l in enumerate(lines) if i > start and l.strip().startswith(".Lfunc_end"))
    depth = 0
    stats = collections.defaultdict(collections.Counter)
    for l in lines[start:end]:
        m = re.match(r"^\.LBB\d+_\d+:\s*;.*Depth=(\d+)", l)
        if m:
            depth = int(m.group(1))
        elif re.match(r"^\.LBB\d+_\d+:", l):
            depth = 0
        if l.startswith("\t") and not l.strip().startswith((".", ";")):
            stats[depth][category(l.split()[0])] += 1
    cats = ["fp64 arithmetic", "selects", "moves / dpp", "sgpr spill moves", "compares", "other valu", "scalar", "lds",
            "scratch", "memory / other"]
    names = {0: "outside loops", 1: "step loop (depth 1)", 2: "attempt loop (depth 2)", 3: "Newton loop (depth 3)"}
    print(f"{'':24s}" + "".join(f"{c[:16]:>17s}" for c in cats) + f"{'total':>8s}")
    allc = collections.Counter()
    for d in sorted(stats):
        tot = sum(stats[d].values())
        allc.update(stats[d])
        print(f"{names.get(d, 'depth ' + str(d)):24s}" + "".join(f"{stats[d][c]:>10d} {100 * stats[d][c] / tot:4.1f}%" for c in cats)
              + f"{tot:>8d}")
    tot = sum(allc.values())
    print(f"{'whole kernel':24s}" + "".join(f"{allc[c]:>10d} {100 * allc[c] / tot:4.1f}%" for c in cats) + f"{tot:>8d}")


if __name__ == "__main__":
    main()
