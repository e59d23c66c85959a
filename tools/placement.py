"""Where and when the trajectories of one C3 launch run (BCM3HIP_OPT_PLACEMENT_LOG): which SIMD
each wavefront lands on, which trajectories share a SIMD, and what sharing costs the longest ones.

A launch of ~1,300 one-wavefront trajectories (a speculative-pair batch) holds more wavefronts than
the chip's 1,024 SIMDs, and the kernel's registers allow two per SIMD, so every wavefront starts at
once and ~270 SIMDs run two. The launch lasts as long as its slowest trajectory, so what matters is
whether the longest trajectories run alone. This prints, for a batch of chain states of a running
sampler in three dispatch orders (as is, longest first, longest first with the shortest interleaved
into the second round):
  kernel ms, SIMDs used, waves per SIMD, and for the 32 longest trajectories: their steps, wall time,
  us per step, and the share of their lifetime with a second wavefront on their SIMD.

    python tools/placement.py [iterations_warmup]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import numpy as np  # noqa: E402

from bcm3_amd import _hip  # noqa: E402
from bcm3_amd.likelihood import Likelihood  # noqa: E402
from bcm3_amd.ptmh import PTMHNative  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
LIK, PRI = os.path.join(G, "c3_likelihood.xml"), os.path.join(G, "c3_prior.xml")


def decode(hw, xcc):
    """gfx9 HW_ID: WAVE_ID [3:0], SIMD_ID [5:4], CU_ID [11:8], SH_ID [12], SE_ID [15:13]"""
    hw = hw.astype(np.int64)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    slot = hw & 15
    key = ((((xcc.astype(np.int64) & 15) * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    return key, slot


def analyse(label, ctx, x, nst):
    n = len(x)
    ctx.set_option(_hip.OPT_PLACEMENT_LOG, 1)
    ms = []
    for _ in range(3):
        ctx.eval(x)
        ms.append(ctx.last_kernel_ms())
    pl = ctx.placement_log(n)
    ctx.set_option(_hip.OPT_PLACEMENT_LOG, 0)
    key, slot = decode(pl[:, 0] & 0xffffffff, pl[:, 1])
    cyc = (pl[:, 0] >> np.uint64(32)).astype(np.float64)  # shader-clock cycles per trajectory
    t0 = pl[:, 2].astype(np.int64)
    t1 = pl[:, 3].astype(np.int64)
    base = t0.min()
    t0 = (t0 - base) / 100.0  # us
    t1 = (t1 - base) / 100.0
    dur = t1 - t0
    uniq, inv, counts = np.unique(key, return_inverse=True, return_counts=True)
    per = counts[inv]
    # share of each trajectory's lifetime with another wavefront alive on its SIMD
    shared = np.zeros(n)
    for i in np.where(per > 1)[0]:
        others = np.where((key == key[i]) & (np.arange(n) != i))[0]
        ov = 0.0
        for j in others:
            ov += max(0.0, min(t1[i], t1[j]) - max(t0[i], t0[j]))
        shared[i] = min(1.0, ov / max(dur[i], 1e-9))
    order = np.argsort(-nst)
    top = order[:32]
    upstep = dur / np.maximum(nst, 1)
    solo = (per == 1) | (shared < 0.05)
    print(f"[{label}] n={n} kernel {min(ms):.3f} ms (med {np.median(ms):.3f}); makespan {t1.max():.0f} us; "
          f"SIMDs {len(uniq)}, waves/SIMD: " +
          ", ".join(f"{c}:{int((counts == c).sum())}" for c in sorted(set(counts.tolist()))) +
          f"; start spread {t0.max():.1f} us", flush=True)
    print(f"   us/step alone {np.median(upstep[solo]):.3f} (n={int(solo.sum())}), "
          f"sharing >50% {np.median(upstep[shared > 0.5]) if (shared > 0.5).any() else float('nan'):.3f} "
          f"(n={int((shared > 0.5).sum())})")
    ghz = cyc / np.maximum(dur, 1e-9) / 1e3
    print(f"   in-kernel shader clock (s_memtime cycles / wall time): median {np.median(ghz):.3f} GHz, "
          f"longest 32 {np.median(ghz[top]):.3f} GHz, min {ghz.min():.3f} max {ghz.max():.3f}")
    last = int(np.argmax(t1))
    print(f"   last to finish: batch index {last}, steps {nst[last]}, {dur[last]:.0f} us, shared {shared[last]:.2f}, "
          f"start {t0[last]:.1f} us; longest solve: steps {nst[order[0]]}, {dur[order[0]]:.0f} us")
    print("   32 longest: index steps us us/step shared")
    for i in top[:32]:
        print(f"     {i:5d} {nst[i]:5d} {dur[i]:7.0f} {upstep[i]:.3f} {shared[i]:.2f}")
    # which batch positions share a SIMD (the dispatcher's pairing)
    pairs = []
    for u in np.where(counts == 2)[0]:
        ii = np.where(inv == u)[0]
        pairs.append(tuple(sorted(ii.tolist())))
    pairs.sort()
    if pairs:
        print("   first SIMD-sharing pairs (batch positions):", pairs[:12])
    return min(ms)


def main():
    warm = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    ll = Likelihood(LIK, PRI, device=0)
    s = PTMHNative(ll, PRI, 256, seed=20251016, proposal="gaussian_mixture")
    s.iterate(warm)
    states = []
    for _ in range(5):
        s.iterate(1)
        states.append(s.state()["values"].copy())
    s.close()
    x = np.concatenate(states)
    ctx = _hip.Context.from_popk_model(ll.popk_model(), 0)
    nst = ctx.eval(x, detail=True)["stats"]["nst"].reshape(len(x), -1).sum(axis=1)
    lf = np.argsort(-nst, kind="stable")
    analyse("as is", ctx, x, nst)
    analyse("longest first", ctx, np.ascontiguousarray(x[lf]), nst[lf])
    # the 2 x 271 shortest paired among themselves: dispatch the 753 longest first, then the rest
    # interleaved shortest / longest-of-the-rest so the second round lands on SIMDs of the short ones
    ctx.close()
    ll.close()


if __name__ == "__main__":
    main()
