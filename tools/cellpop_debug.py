"""Diagnostic (not a test): per-cell comparison of the GPU cell-population path with the oracle.

    python tools/cellpop_debug.py [num_cells] [n_draws]
"""
import math
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import cellpop_helpers as CH  # noqa: E402
import cellpop as CP  # noqa: E402
from bcm3_amd.likelihood import Likelihood  # noqa: E402

nc = int(sys.argv[1]) if len(sys.argv) > 1 else 6
nd = int(sys.argv[2]) if len(sys.argv) > 2 else 6
d = tempfile.mkdtemp()
path = CH.write_likelihood(d, nc, 64)
ll = Likelihood(path, CH.PRIOR, device=0)
prob = CP.load_problem(path, CH.PRIOR)
x = CH.draws(nd, 11)
ref = CP.simulate(prob, x)
lp, st = ll.evaluate_batch(x)
e = prob["experiments"][0]
M, NS = len(e["output_times"]), len(e["model"].ode)
for i in range(nd):
    r = ref["logp"][i]
    print(f"item {i}: gpu {lp[i]:.12g} oracle {r:.12g} diff {lp[i] - r:.3g}")
    det = ref["detail"][i]
    if not det["ok"]:
        continue
    rec, vals, endy = ll.cellpop_cells(i, M, NS)
    cells = det["cells"]
    print(f"   cells gpu {len(rec)} oracle {len(cells)}")
    for k in range(min(len(rec), len(cells))):
        c = cells[k]
        ok = ~np.isnan(c["values"])
        dv = np.max(np.abs(vals[k][ok] - c["values"][ok]) / (np.abs(c["values"][ok]) + 1e-12)) if ok.any() else 0.0
        print(f"   cell {k}: steps {rec['nsteps'][k]} / {c['nsteps']}  div {bool(rec['flags'][k] & 2)} / {c['divided']}  "
              f"sim_end {rec['sim_end'][k]:.10g} / {c['sim_end']:.10g}  values rel {dv:.2e}")
