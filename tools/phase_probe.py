"""Per-phase cycle breakdown of the BDF kernel (profiling build lib/libbcm3hip_phases.so).

    make -C bcm3_amd/csrc phases && python tools/phase_probe.py [n] [lpw]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["BCM3HIP_LIB"] = os.path.join(ROOT, "bcm3_amd", "lib", "libbcm3hip_phases.so")
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]

import numpy as np  # noqa: E402

import helpers as H  # noqa: E402
import synthetic as S  # noqa: E402
from bcm3_amd import _hip  # noqa: E402

NAMES = ["driver(out/cb/reinit)", "entry+ewt", "adjust+rescale", "predict", "set_bdf", "newton",
         "errtest/fail", "complete", "eta/next", "tstop/return"]
# the fast loop (vec::fast_run): 10-17 are timed on plain steps (coefficients held), 18 on every
# fast-loop step, 24-26 on recomputing fast-loop steps after their Newton correction; 19/20 whole
# plain / recomputing steps, 21/22 their counts, 23 the marker (bdf_lane.h NPHASES)
FAST = ["ewt + plain test", "predict", "newton: rhs", "newton: solve (I-gJ)^-1", "newton: wrms norm",
        "conv + error test", "complete: zn", "complete: eta"]
GEN = ["conv + error test", "complete: zn, tau", "complete: eta"]
NPH = 32


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    lpw = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    prob = H.c3_problem(1)
    ctx = H.gpu_context(prob, lanes_per_wave=lpw)
    vals = S.prior_draws(1, n, 7)
    g = ctx.eval(vals, detail=True)
    ms = ctx.last_kernel_ms()
    allph = g["traj"].reshape(n, -1)[:, :NPH]
    ph = allph[:, :len(NAMES)]
    nst = g["stats"]["nst"][:, 0].astype(np.float64)
    tot = ph.sum(axis=1)
    imax = int(np.argmax(tot))
    print(f"n={n} lpw={lpw} kernel {ms:.3f} ms; slowest traj {tot[imax]:.3e} cycles, {nst[imax]:.0f} steps "
          f"-> {tot[imax] / nst[imax]:.0f} cycles/step; implied clock {tot[imax] / (ms * 1e-3) / 1e9:.2f} GHz")
    # the slowest trajectory (the one the launch waits for) and the 10 slowest
    slow = np.argsort(-tot)[:10]
    print(f"slowest trajectory: {nst[imax]:.0f} steps, nfe {g['stats']['nfe'][imax, 0]}, netf {g['stats']['netf'][imax, 0]}, "
          f"ncfn {g['stats']['ncfn'][imax, 0]}, nsetups {g['stats']['nsetups'][imax, 0]}; its cycles per step by phase:")
    for k, name in enumerate(NAMES):
        print(f"  {name:24s} {ph[imax, k] / nst[imax]:8.0f}")
    print(f"10 slowest: steps {nst[slow].astype(int).tolist()}, cycles/step {(tot[slow] / nst[slow]).round(0).tolist()}")
    print(f"all: steps mean {nst.mean():.0f}, cycles/step mean {(tot / nst).mean():.0f}; "
          f"corr(steps, cycles/step) {np.corrcoef(nst, tot / nst)[0, 1]:.2f}")
    per = ph.sum(axis=0) / nst.sum()
    print(f"mean cycles per step {per.sum():.0f}:")
    for k, name in enumerate(NAMES):
        print(f"  {name:24s} {per[k]:8.0f}  {100 * per[k] / per.sum():5.1f}%")
    print("stats means:", {k: float(g["stats"][k].mean()) for k in g["stats"].dtype.names})
    qh = g["traj"].reshape(n, -1)[:, NPH:NPH + 5].sum(axis=0)
    print("successful steps by order q=1..5 (UNI solver):", (qh / qh.sum()).round(3).tolist())
    fast_report(allph, nst, ms, tot)


def fast_report(allph, nst, ms, tot):
    """cycles per fast-loop step by phase, the marker's own cost subtracted"""
    mark = allph[:, 23].sum() / (16 * allph.shape[0])
    n_plain, n_gen = allph[:, 21].sum(), allph[:, 22].sum()
    if n_plain == 0:
        print("no fast-loop steps (not the VEC solver?)")
        return
    n_fast = n_plain + n_gen
    c_plain = allph[:, 19].sum() / n_plain
    c_gen = allph[:, 20].sum() / max(n_gen, 1)
    print(f"\nfast loop: {n_fast / nst.sum():.1%} of all steps; plain (coefficients held) {n_plain / n_fast:.1%} of them")
    print(f"marker cost {mark:.0f} cycles (16 back-to-back per trajectory)")
    k_plain, k_gen = 8, 7
    print(f"whole step, loop top to exit test: plain {c_plain:.0f} cycles ({c_plain - k_plain * mark:.0f} without its "
          f"{k_plain} markers), recomputing {c_gen:.0f} ({c_gen - k_gen * mark:.0f} without its {k_gen})")
    rows = [(f"plain: {n}", allph[:, 10 + i].sum() / n_plain) for i, n in enumerate(FAST)]
    rows.append(("exit test + back edge (all)", allph[:, 18].sum() / n_fast))
    print(f"{'plain step phase':34s} {'cycles':>8s} {'- marker':>9s}")
    tot_net = 0.0
    for name, v in rows:
        net = max(v - mark, 0.0)
        tot_net += net
        print(f"  {name:32s} {v:8.0f} {net:9.0f}")
    print(f"  {'sum':32s} {'':8s} {tot_net:9.0f}")
    print(f"{'recomputing step: after Newton':34s}")
    for i, n in enumerate(GEN):
        v = allph[:, 24 + i].sum() / max(n_gen, 1)
        print(f"  {n:32s} {v:8.0f} {max(v - mark, 0.0):9.0f}")
    print(f"etaq roots (step size may grow): {allph[:, 27].sum() / nst.sum():.1%} of steps")
    n_chk, n_skip = allph[:, 28].sum(), allph[:, 29].sum()
    if n_chk:
        print(f"order-change checks: {n_chk / nst.sum():.1%} of steps, screened out {n_skip / n_chk:.1%}; screen "
              f"{allph[:, 30].sum() / n_chk - mark:.0f} cycles per check, exact evaluation "
              f"{allph[:, 31].sum() / max(n_chk - n_skip, 1) - mark:.0f} cycles per evaluation")
    print(f"(phases build: kernel {ms:.3f} ms)")

if __name__ == "__main__":
    main()
