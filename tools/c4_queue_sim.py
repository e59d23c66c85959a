"""What a device-side work queue for the C4 daughters would gain (VERDICT r05 missing item 3), simulated
from the reference solver's own per-cell records: the oracle (the reference's CVODE, oracle/_ref) solves
the bench's first 16 C4 draws; each cell's BDF step count stands for its solve time; cells go four to a
wavefront in launch order (a wavefront lasts as long as its longest cell) onto the wave slots of 16
evaluations' share of the chip (2,048 / 4 = 512). Compared: the product's generation launches (every
generation waits for the previous one) and a wave-level queue (a free slot takes the next four cells
available; daughters become available when their mother ends), next to the work / slots bound.

    python tools/c4_queue_sim.py
"""
import heapq
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("tests", "oracle", os.path.join("tests", "golden"))]
import cellpop as CP  # noqa: E402
import cellpop_helpers as CH  # noqa: E402

SLOTS = 512


def waves_of(items):
    return [max(c[4] for c in items[i:i + 4]) for i in range(0, len(items), 4)]


def sched(durs, slots, t0=0.0):
    h = [t0] * slots
    end = t0
    for d in durs:
        t = heapq.heappop(h)
        heapq.heappush(h, t + d)
        end = max(end, t + d)
    return end


def main():
    prob = CP.load_problem(os.path.join(CH.GOLDEN, "cellpop_likelihood.xml"), CH.PRIOR)
    x = CH.draws(64, 23)[:16]
    r = CP.simulate(prob, x, nthreads=min(16, os.cpu_count() or 1))
    cells = []
    for ev, det in enumerate(r["detail"]):
        if not det["ok"]:
            continue
        gen = {}
        for c in det["cells"]:
            gen[c["index"]] = 0 if c["parent"] < 0 else gen[c["parent"]] + 1
            cells.append((ev, c["index"], c["parent"], gen[c["index"]], c["nsteps"]))
    ngen = max(c[3] for c in cells) + 1
    t = 0.0
    for g in range(ngen):
        t = sched(waves_of([c for c in cells if c[3] == g]), SLOTS, t)
    kids = {}
    for c in cells:
        if c[2] >= 0:
            kids.setdefault((c[0], c[2]), []).append(c)
    pending = [(0.0, i, c) for i, c in enumerate(c for c in cells if c[3] == 0)]
    heapq.heapify(pending)
    slots = [0.0] * SLOTS
    end, cnt = 0.0, 0
    while pending:
        st = heapq.heappop(slots)
        batch = []
        while pending and len(batch) < 4:
            ta, _, c = heapq.heappop(pending)
            batch.append((ta, c))
        te = max(st, max(b[0] for b in batch)) + max(b[1][4] for b in batch)
        end = max(end, te)
        heapq.heappush(slots, te)
        for _, c in batch:
            for k in kids.get((c[0], c[1]), []):
                cnt += 1
                heapq.heappush(pending, (te, 10 ** 9 + cnt, k))
    # daughters first: a free slot takes the daughters already enqueued before the remaining initial
    # cells (the deepest chains start early; initial cells fill the end), initial cells in their order
    lo = [c for c in cells if c[3] == 0]
    lo.reverse()
    hi = []
    slots = [0.0] * SLOTS
    end_p, cnt = 0.0, 0
    while lo or hi:
        st = heapq.heappop(slots)
        batch = []
        while hi and len(batch) < 4 and hi[0][0] <= st:
            ta, _, c = heapq.heappop(hi)
            batch.append((ta, c))
        while lo and len(batch) < 4:
            batch.append((0.0, lo.pop()))
        while hi and len(batch) < 4:
            ta, _, c = heapq.heappop(hi)
            batch.append((ta, c))
        te = max(st, max(b[0] for b in batch)) + max(b[1][4] for b in batch)
        end_p = max(end_p, te)
        heapq.heappush(slots, te)
        for _, c in batch:
            for k in kids.get((c[0], c[1]), []):
                cnt += 1
                heapq.heappush(hi, (te, cnt, k))
    work = sum(waves_of(sorted(cells, key=lambda c: (c[3], c[0], c[1])))) / SLOTS
    print(f"{len(cells)} cells of {len(set(c[0] for c in cells))} finite evaluations, {ngen} generations, {SLOTS} wave slots")
    print(f"generation launches: {t:.0f} step-times; wave-level queue: {end:.0f} ({t / end:.3f}x); work / slots bound: "
          f"{work:.0f} ({t / work:.3f}x); daughters-first queue: {end_p:.0f} ({t / end_p:.3f}x)")


if __name__ == "__main__":
    main()
