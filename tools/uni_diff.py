"""Diagnose differences between the UNI solver (lanes_per_wave=1) and the lane solver (lpw=64).

    python tools/uni_diff.py [n]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]

import numpy as np  # noqa: E402

import helpers as H  # noqa: E402
import synthetic as S  # noqa: E402
from bcm3_amd import _hip  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    prob = H.c3_problem(1)
    ctx = H.gpu_context(prob, lanes_per_wave=64)
    vals = S.prior_draws(1, n, 12)
    a = ctx.eval(vals, detail=True)
    ctx.set_option(_hip.OPT_LANES_PER_WAVE, 1)
    b = ctx.eval(vals, detail=True)
    same = (a["logp"] == b["logp"]) | (np.isnan(a["logp"]) & np.isnan(b["logp"]))
    print(f"identical logp: {same.mean():.3f} ({(~same).sum()} differ)")
    for k in a["stats"].dtype.names:
        d = a["stats"][k] != b["stats"][k]
        print(f"  stats {k}: {d.mean():.3f} differ")
    bad = np.nonzero(~same)[0][:8]
    for i in bad:
        ta, tb = a["traj"][i, 0], b["traj"][i, 0]
        diff = np.nonzero(~((ta == tb) | (np.isnan(ta) & np.isnan(tb))))
        first_t = diff[1].min() if diff[1].size else -1
        print(f"draw {i}: logp {a['logp'][i]!r} vs {b['logp'][i]!r}; nst {a['stats']['nst'][i,0]} vs "
              f"{b['stats']['nst'][i,0]}; nfe {a['stats']['nfe'][i,0]} vs {b['stats']['nfe'][i,0]}; "
              f"nsetups {a['stats']['nsetups'][i,0]} vs {b['stats']['nsetups'][i,0]}; first traj diff t-index {first_t}; "
              f"max rel {np.nanmax(np.abs(ta - tb) / np.maximum(np.abs(ta), 1e-300)):.3e}")


if __name__ == "__main__":
    main()
