"""Instruction histogram of one plain BDF step of the fast loop (vec::fast_run<Q>, bdf_vec.h), from
the ISA (VERDICT r02 "Next round" 4).

Builds popk_kernel.hip device-only to assembly with -DBCM3_MARKS (bdf_vec.h / bdf_lane.h emit a
"; BDFMARK <phase>" comment at each phase boundary and "; BDFMARK fast_top Q=<q>" at the loop top),
splits the chosen kernel into basic blocks, and walks the control-flow graph from the fast_top block
of each order back to it. A plain step takes, at every branch, the common side: the shortest cycle
in instructions is the step that reuses the BDF coefficients (constant h, no setup, qwait > 1); the
shortest cycle through the set_bdf block is the step that recomputes them. Prints per cycle the
instruction classes and their split over the phases:
  2 predict   3 set_bdf   4 Newton (rhs, matvec, wrms)   5 -> 7 complete head   7 -> 8 eta
  8 -> top    quiet test / loop back

    python tools/step_isa.py [kernel-substring] [--asm existing.s]
        default kernel: popk_traj_kernelILi1ELi2ELb0E (TWO model, VEC solver, no stats)
"""
import collections
import heapq
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "bcm3_amd", "csrc")
CLASSES = ("valu_f64", "valu_other", "v_dpp", "v_readlane", "salu", "s_branch", "s_waitcnt", "lds", "vmem",
           "smem", "other")


def build_asm(out="/tmp/popk_marks.s"):
    # the library's own flags (bcm3_amd/csrc/Makefile HIPFLAGS): without -structurizecfg-skip-uniform-regions
    # every uniform branch would be compiled as an exec-masked region
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                    "-ffp-contract=off", "-mllvm", "-simplifycfg-sink-common=false", "-mllvm",
                    "-structurizecfg-skip-uniform-regions", "-DBCM3_MARKS", "-o", out, os.path.join(CSRC, "popk_kernel.hip")],
                   check=True, stderr=subprocess.DEVNULL)
    return out


def function_lines(asm, pat):
    cur, body = None, []
    for line in open(asm):
        m = re.match(r"^(_Z\S+):", line)
        if m:
            if cur and pat in cur:
                return cur, body
            cur, body = m.group(1), []
            continue
        if cur:
            body.append(line.rstrip("\n"))
    if cur and pat in cur:
        return cur, body
    raise SystemExit(f"no kernel matching {pat}")


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_"):
        if "readlane" in op or "readfirstlane" in op or "writelane" in op:
            return "v_readlane"
        if "dpp" in ins or "row_" in ins or op.startswith("v_mov_b64_dpp"):
            return "v_dpp"
        return "valu_f64" if "_f64" in op else "valu_other"
    if op.startswith("s_"):
        if op.startswith(("s_cbranch", "s_branch", "s_setpc")):
            return "s_branch"
        if op.startswith("s_waitcnt"):
            return "s_waitcnt"
        if op.startswith(("s_load", "s_buffer_load")):
            return "smem"
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


class Block:
    def __init__(self, label):
        self.label = label
        self.items = []  # ("ins", text, phase) | ("mark", text)
        self.succ = []


def blocks_of(body):
    blocks, cur = [], Block("<entry>")
    pending_fall = True
    for line in body:
        s = line.strip()
        if not s:
            continue
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            nb = Block(m.group(1))
            if pending_fall:
                cur.succ.append(nb.label)
            blocks.append(cur)
            cur, pending_fall = nb, True
            continue
        if "BDFMARK" in s:
            cur.items.append(("mark", s.split("BDFMARK", 1)[1].strip()))
            continue
        if s.startswith((";", ".", "//")) or s.endswith(":"):
            continue
        cur.items.append(("ins", s))
        op = s.split()[0]
        if op.startswith(("s_branch", "s_cbranch")):
            tgt = s.split()[-1]
            cur.succ.append(tgt)
            if op.startswith("s_branch"):
                nb = Block(f"<after {tgt} {len(blocks)}>")
                blocks.append(cur)
                cur, pending_fall = nb, False
                continue
            # conditional: fall through into a new block
            nb = Block(f"<fall {len(blocks)}>")
            cur.succ.append(nb.label)
            blocks.append(cur)
            cur, pending_fall = nb, True
        elif op.startswith(("s_endpgm", "s_setpc")):
            blocks.append(cur)
            cur, pending_fall = Block(f"<dead {len(blocks)}>"), False
    blocks.append(cur)
    return {b.label: b for b in blocks}, [b.label for b in blocks]


def ninstr(b):
    return sum(1 for k, *_ in b.items if k == "ins")


def dijkstra(blocks, src, dst, banned=()):
    """shortest block path src -> dst (instructions of every block before dst), not entering banned"""
    dist, prev = {src: 0}, {}
    pq = [(0, src)]
    while pq:
        d, u = heapq.heappop(pq)
        if u == dst:
            break
        if d > dist.get(u, 1 << 60):
            continue
        for v in blocks[u].succ:
            if v not in blocks or (v in banned and v != dst):
                continue
            nd = d + ninstr(blocks[u])
            if nd < dist.get(v, 1 << 60):
                dist[v] = nd
                prev[v] = u
                heapq.heappush(pq, (nd, v))
    if dst not in dist or dst == src:
        return None
    path, x = [dst], dst
    while x != src:
        x = prev[x]
        path.append(x)
    return path[::-1]


def marked(blocks, order, name):
    return [l for l in order if any(k == "mark" and t == name for k, t, *_ in blocks[l].items)]


def step_path(blocks, order, top, seq, set_bdf, avoid=()):
    """Shortest cycle top -> (a block marked seq[0]) -> ... -> top, passing the phase markers in the
    order a plain step passes them. Consecutive markers in one block are one stop. The structurised
    control flow branches on exec (s_cbranch_execz skips a region no lane enters); a wave-uniform
    step enters a region exactly when its condition holds, so the markers pin the regions a plain
    step runs. set_bdf: the step recomputes the BDF coefficients (the region between markers 3 and
    4 is entered) or reuses them (skipped)."""
    banned = {l for l in order if any(k == "mark" and (t.startswith("fast_top") or t in avoid)
                                      for k, t, *_ in blocks[l].items)}
    stops = [[top]]
    for name in seq:
        stops.append(marked(blocks, order, name))
    stops.append([top])
    # DP over stops: best[(i, block)] = (cost, path)
    best = {top: (0, [top])}
    for i in range(1, len(stops)):
        nb = {}
        for b, (c, p) in best.items():
            for cand in stops[i]:
                ban = banned - {top}
                if cand == b:
                    seg = [b]
                elif seq[i - 1:i] == ["4"] and set_bdf:
                    # enter the region the reuse branch skips: leave b by its other successor
                    seg = None
                    for s0 in blocks[b].succ:
                        if s0 != cand and s0 in blocks:
                            t = dijkstra(blocks, s0, cand, ban)
                            if t and (seg is None or len(t) + 1 < len(seg)):
                                seg = [b] + t
                    if seg is None:
                        continue
                else:
                    seg = dijkstra(blocks, b, cand, ban)
                    if seg is None:
                        continue
                    if seq[i - 1:i] == ["4"] and len(seg) > 2:
                        continue  # reuse: the skip edge straight to the Newton block
                cost = c + sum(ninstr(blocks[x]) for x in seg[:-1])
                if cand not in nb or cost < nb[cand][0]:
                    nb[cand] = (cost, p + seg[1:])
        best = nb
        if not best:
            return None
    return best[top][1] if top in best else None


def dump(blocks, path):
    phase = "top"
    for lab in path[:-1]:
        print(f"  -- {lab}")
        for item in blocks[lab].items:
            if item[0] == "mark":
                phase = item[1]
                print(f"  == BDFMARK {phase}")
            else:
                print(f"     {item[1]}")


def histogram(blocks, path):
    """path: list of block labels (first == last == the fast_top block); counts each block once
    except the repeated final one; phases follow the markers in order"""
    h = collections.Counter()
    ph = collections.defaultdict(collections.Counter)
    phase = "top"
    started = False
    for i, lab in enumerate(path[:-1]):
        for item in blocks[lab].items:
            if item[0] == "mark":
                if item[1].startswith("fast_top"):
                    if started:
                        break
                    started = True
                    phase = "top"
                else:
                    phase = item[1]
                continue
            c = classify(item[1])
            h[c] += 1
            ph[phase][c] += 1
    # the part of the start block before its marker (loop back tail) belongs to the step too
    for item in blocks[path[0]].items:
        if item[0] == "mark" and item[1].startswith("fast_top"):
            break
        if item[0] == "ins":
            c = classify(item[1])
            h[c] += 1
            ph["tail"][c] += 1
    return h, ph


# fast_run's markers (bdf_vec.h; the phases build times the same boundaries, tools/phase_probe.py):
# a plain step passes 10 .. 17 in order; the instructions after marker k belong to the next phase
PLAIN = ["10", "11", "12", "13", "14", "15", "16", "17"]
PHASE_NAMES = {"top": "ewt + plain test", "18": "ewt + plain test", "10": "predict", "11": "newton: rhs",
               "12": "newton: solve", "13": "newton: wrms norm", "14": "conv + error test",
               "15": "complete: zn, tau", "16": "complete: eta (root)", "17": "exit test + back edge",
               "general": "rescale", "2": "predict", "3": "set_bdf", "4": "newton",
               "24": "complete: zn, tau", "25": "complete: eta", "26": "exit test + back edge"}


def fmt(c):
    v = sum(c[k] for k in ("valu_f64", "valu_other", "v_dpp", "v_readlane"))
    s = c["salu"] + c["smem"]
    return (f"{sum(c.values()):4d} instr: VALU {v:3d} (f64 {c['valu_f64']}, other {c['valu_other']}, dpp "
            f"{c['v_dpp']}, readlane {c['v_readlane']}), SALU {s:3d}, branch {c['s_branch']:2d}, waitcnt "
            f"{c['s_waitcnt']}, lds {c['lds']}, vmem {c['vmem']}")


def main():
    args = [a for i, a in enumerate(sys.argv[1:], 1) if not a.startswith("--") and sys.argv[i - 1] != "--dump"]
    pat = args[0] if args else "popk_traj_kernelILi1ELi2ELb0E"
    asm = sys.argv[sys.argv.index("--asm") + 1] if "--asm" in sys.argv else build_asm()
    if "--asm" in sys.argv:
        args = [a for a in args if a != asm]
        pat = args[0] if args else "popk_traj_kernelILi1ELi2ELb0E"
    name, body = function_lines(asm, pat)
    blocks, order = blocks_of(body)
    print(name[:100])
    for q in range(1, 6):
        tops = marked(blocks, order, f"fast_top Q={q}")
        if not tops:
            continue
        top = tops[0]
        print(f"Q={q}  fast_top block {top}")
        # fast_run's plain step (one branch on `plain`) and its general attempt ("general" marker:
        # rescale, cvSet, setup and scale tests), the latter with the cvSet region entered
        general = bool(marked(blocks, order, "general"))
        for label, sb, seq, avoid in (
                ("plain step (coefficients held)", False, PLAIN, ("general",)),
                ("general attempt recomputing them (set_bdf)", True,
                 (["general", "2", "3", "4", "24", "25", "26"] if general else ["2", "3", "4", "24", "25", "26"]),
                 ())):
            p = step_path(blocks, order, top, seq, sb, avoid)
            if not p:
                print(f"  {label}: no path")
                continue
            h, ph = histogram(blocks, p)
            if "--dump" in sys.argv and q == int(sys.argv[sys.argv.index("--dump") + 1]):
                dump(blocks, p)
            print(f"  {label} ({len(p) - 1} blocks): {fmt(h)}")
            for k in ("top", "18", "general", "2", "3", "4") + tuple(PLAIN) + ("24", "25", "26", "tail"):
                if k in ph:
                    print(f"     phase {k:>7} {PHASE_NAMES.get(k, ''):24s}: {fmt(ph[k])}")


if __name__ == "__main__":
    main()
