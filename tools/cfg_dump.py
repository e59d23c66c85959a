"""Basic-block listing of one kernel from a -gline-tables-only -S build: per block the source
lines it came from, its VALU / SALU counts and its branch, to find the hot path by eye.

    hipcc ... --cuda-device-only -S -gline-tables-only -o /tmp/pk_g.s popk_kernel.hip
    python tools/cfg_dump.py /tmp/pk_g.s popk_traj_kernelILi1ELb1E > /tmp/cfg.txt
"""
import re
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    files = {}
    blocks = []
    cur = None
    infn = False
    loc = None
    for line in open(path):
        m = re.match(r"\s*\.file\s+(\d+)\s+\"[^\"]*\"\s+\"([^\"]+)\"", line)
        if m:
            files[m.group(1)] = m.group(2).split("/")[-1].replace(".h", "").replace(".hip", "")
            continue
        if not infn:
            if re.match(r"^_Z\S*" + re.escape(pat) + r"\S*:", line):
                infn = True
                cur = {"label": "entry", "lines": [], "v": 0, "s": 0, "br": [], "n": 0}
                blocks.append(cur)
            continue
        if line.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\S+):", line)
        if m:
            cur = {"label": m.group(1), "lines": [], "v": 0, "s": 0, "br": [], "n": 0}
            blocks.append(cur)
            continue
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
        if m:
            loc = f"{files.get(m.group(1), m.group(1))}:{m.group(2)}"
            if loc != "0" and (not cur["lines"] or cur["lines"][-1] != loc):
                cur["lines"].append(loc)
            continue
        s = line.strip()
        if not s or s.startswith((";", ".", "//")):
            continue
        op = s.split()[0]
        cur["n"] += 1
        if op.startswith("v_"):
            cur["v"] += 1
        elif op.startswith("s_"):
            if op.startswith(("s_cbranch", "s_branch", "s_setpc")):
                cur["br"].append(s.split(";")[0])
            else:
                cur["s"] += 1
    for b in blocks:
        lines = b["lines"]
        if len(lines) > 8:
            lines = lines[:4] + ["..."] + lines[-3:]
        print(f"{b['label']:14s} v{b['v']:4d} s{b['s']:3d}  {' | '.join(b['br']):40s} {' '.join(lines)}")


if __name__ == "__main__":
    main()
