"""Diagnose the one-trajectory-per-wavefront solvers on the two-compartment transit model: status,
logp and solver counters of the UNI / VEC / lane forms on a few draws (BCM3HIP_LIB selects the
library build)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402

import helpers as H  # noqa: E402

pk = sys.argv[1] if len(sys.argv) > 1 else "two_transit"
prob, lo, hi = H.make_problem(pk, P=2, T_days=6)
vals = H.draws(lo, hi, 16, 91)
for lpw, uni in ((1, 0), (1, 1), (64, 0)):
    ctx = H.gpu_context(prob, lanes_per_wave=lpw, uni_solver=uni)
    g = ctx.eval(vals, detail=True)
    ctx.close()
    st = g["stats"]
    print(f"lpw={lpw} uni={uni}: logp {np.array2string(g['logp'][:6], precision=6)} status {g['status'][:6].tolist()}")
    print("   nst", st["nst"][:6, 0].tolist(), "nfe", st["nfe"][:6, 0].tolist(), "netf", st["netf"][:6, 0].tolist())
