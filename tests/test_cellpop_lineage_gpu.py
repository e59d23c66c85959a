"""GPU parity of time courses with an observed lineage (cp_timecourse_kernel's lineage recursion,
cellpop_kernels.hip cp_lineage_likelihood) against the oracle (oracle/cellpop.py _timecourse_logp);
the cases of tests/test_cellpop_lineage.py.

  * on the GPU's own simulated cells and daughters, the oracle's recursion and matching reproduce the
    GPU logp to 1e-12 relative (isolates the data likelihood);
  * against the oracle's own solve: the cell-population envelope (cellpop_helpers.logp_bar) with the -inf
    pattern identical."""
import math

import numpy as np
import pytest

import cellpop_helpers as CH
import cellpop as CP
from test_cellpop_lineage import CASES, lineage_likelihood, only

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=list(CASES))
def lin_case(request, tmp_path_factory):
    from bcm3_amd.likelihood import Likelihood
    name = request.param
    path = lineage_likelihood(tmp_path_factory.mktemp("lineage_gpu"), name)
    opts = f"cellpop.use_only_cell_ix={CASES[name][2]}" if CASES[name][2] else ""
    ll = Likelihood(path, CH.PRIOR, device=0, options=opts)
    prob = CP.load_problem(path, CH.PRIOR, use_only_cell_ix=only(name))
    x = CH.draws(8, 3)
    yield name, ll, prob, x, path
    ll.close()


def test_lineage_on_gpu_values(lin_case):
    name, ll, prob, x, path = lin_case
    lp, status = ll.evaluate_batch(x)
    e = prob["experiments"][0]
    d = e["data"][0]
    M, NS = len(e["output_times"]), len(e["model"].ode)
    for i in range(len(x)):
        if status[i] != 0:
            assert lp[i] == -math.inf
            continue
        rec, vals, _ = ll.cellpop_cells(i, M, NS)
        tv = [CP.transform(tf, v) for tf, v in zip(prob["transforms"], x[i])]
        traj = np.full((e["max_cells"], len(d["times"])), np.nan)
        for k, (tdl, t, ti, six) in enumerate(e["timepoints"]):
            if tdl == 0 and ti >= 0:
                traj[:len(rec), ti] = vals[:, k]
        # the simulated lineage: daughters are numbered after their parents, two at a time, in the
        # order the parents divided (the GPU's creation times identify each daughter's parent)
        nc = len(rec)
        sim_child = [-1] * nc
        parents = [c for c in range(nc) if rec["flags"][c] & 16]
        for k, p in enumerate(parents):
            sim_child[p] = e["num_cells"] + 2 * k
        ok, v = CP._timecourse_logp(d, traj, [c < e["num_cells"] for c in range(nc)], tv, sim_child)
        if v == -math.inf or lp[i] == -math.inf:
            assert v == lp[i], (name, i, v, lp[i])
        else:
            assert abs(lp[i] - v * 1.0) <= 1e-12 * (1 + abs(v)), (name, i, lp[i], v)


def test_lineage_matches_oracle(lin_case):
    name, ll, prob, x, path = lin_case
    lp, _ = ll.evaluate_batch(x)
    ref = CP.simulate(prob, x)["logp"]
    ref_nofma = CP.simulate(CP.load_problem(path, CH.PRIOR, variant="nofma", use_only_cell_ix=only(name)), x)["logp"]
    CH.check_logp(lp, None, ref, ref_nofma, name=f"lineage {name}")
    if name in ("no_division", "t4_missing", "subset"):
        assert np.isfinite(lp).all(), name
    if name == "division":
        assert (lp == -math.inf).all()
