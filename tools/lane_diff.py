"""Diagnostic (not a test): draws whose results differ between the VEC solver (lanes_per_wave 1),
the lane solver (64 per wave) and the UNI solver for a build given by BCM3HIP_LIB; the three must agree bit for bit.

    BCM3HIP_LIB=build/var/X.so python tools/lane_diff.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402

import helpers as H  # noqa: E402

tag = os.path.basename(os.environ.get("BCM3HIP_LIB", "default"))
for pk in ("one", "two", "two_transit"):
    prob, lo, hi = H.make_problem(pk, P=2, T_days=6)
    vals = H.draws(lo, hi, 256, 91)
    out = {}
    for name, lpw, uni in (("vec", 1, 0), ("lane", 64, 0), ("uni", 1, 1)):
        ctx = H.gpu_context(prob, lanes_per_wave=lpw, uni_solver=uni)
        out[name] = ctx.eval(vals, detail=True)
        ctx.close()
    d = np.where(out["vec"]["logp"] != out["lane"]["logp"])[0]
    u = np.where(out["vec"]["logp"] != out["uni"]["logp"])[0]
    print(tag, pk, "differing draws vec/lane:", len(d), "vec/uni:", len(u), flush=True)
