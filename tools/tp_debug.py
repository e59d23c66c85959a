"""Debug: GPU time-points logp vs the oracle's data likelihood on the GPU's own cells (normal case)."""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import tempfile  # noqa: E402

import cellpop as CP  # noqa: E402
import cellpop_helpers as CH  # noqa: E402
from test_timecourse import tc_likelihood  # noqa: E402
from test_timepoints_gpu import CASES  # noqa: E402

from bcm3_amd.likelihood import Likelihood  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "normal"
data_xml, kw, options = CASES[name]
d = tempfile.mkdtemp()
path = tc_likelihood(d, data_xml, **kw)
only = options.split("=")[1] if options else "-1"
ll = Likelihood(path, CH.PRIOR, device=0, options=options or "")
prob = CP.load_problem(path, CH.PRIOR, use_only_cell_ix=only)
x = CH.draws(8, 3)
lp, status = ll.evaluate_batch(x)
e = prob["experiments"][0]
M, NS = len(e["output_times"]), len(e["model"].ode)
ref = CP.simulate(prob, x)["logp"]
for i in range(len(x)):
    rec, vals, _ = ll.cellpop_cells(i, M, NS)
    tv = [CP.transform(tf, v) for tf, v in zip(prob["transforms"], x[i])]
    tot = 0.0
    for dli, dd in enumerate(e["data"]):
        if dd["kind"] == "time_points":
            part = CP._timepoints_logp(dd, CP.notify_time_points(e, dli, vals), tv)
            print("  dl", dli, "time_points", part)
            tot += part
    print(i, "status", status[i], "gpu", lp[i], "oracle-on-gpu-cells", tot, "oracle-solve", ref[i], "ncells", len(rec))
