"""GPU parity of the time-points data likelihood (DataLikelihoodTimePoints, cp_timepoints_kernel)
against the oracle (oracle/cellpop.py: notify_time_points + _timepoints_logp over the restated
matching routine, oracle/hungarian.py).

  * on the GPU's own simulated cells, the oracle's Evaluate reproduces the GPU logp to 1e-12
    relative (the matching is index work and exact; the cell likelihoods use the device's log /
    log1p, within an ulp of glibc's) -- this isolates the data likelihood from the ODE solve;
  * against the oracle's own solve (the reference's CVODE per cell) the GPU logp sits in the
    cell-population envelope of test_cellpop_gpu.py, with an identical -inf pattern."""
import math

import numpy as np
import pytest

import cellpop_helpers as CH
import cellpop as CP
from test_timecourse import TC, tc_likelihood
from test_timepoints import TP, _tp

pytestmark = pytest.mark.gpu

DIV = dict(num_cells=4, max_cells=32, experiment_attrs="")

# (data element(s), likelihood kwargs, options)
CASES = {
    "normal": (TP, {}, None),
    "t4_offset_scale": (_tp(error_model="t4", weight="0.5", offset="0.02", scale="1.1", stdev_relative_to_scale="true"),
                        {}, None),
    "columns": (_tp(data_name="pcna_cells_markers", species_name="PCNA_gfp;CycB + PCNA_gfp", stdev="stdev;0.5"), {}, None),
    "relative": (_tp(value_relative_to_timepoint_ix="5", offset="0.01"), {}, None),
    "division": (TP, DIV, "cellpop.use_only_cell_ix=2,7,11"),
    "nondivided": (_tp(use_only_nondivided="true"), DIV, "cellpop.use_only_cell_ix=2,7,11"),
    "late_entry": (_tp(data_name="pcna_cells_late"), dict(entry_time="1.5"), None),
    "early_minus_inf": (TP, dict(entry_time="1.5"), None),
    "one_cell": (_tp(data_name="pcna_cell0_2d"), dict(num_cells=1, max_cells=1), None),
    "with_time_course": (TC + TP.replace('stdev="stdev"', 'stdev="0.2" error_model="t4"'), {}, None),
}


@pytest.fixture(scope="module", params=list(CASES))
def tp_case(request, tmp_path_factory):
    from bcm3_amd.likelihood import Likelihood
    data_xml, kw, options = CASES[request.param]
    d = tmp_path_factory.mktemp("tp_gpu")
    path = tc_likelihood(d, data_xml, **kw)
    only = options.split("=")[1] if options else "-1"
    ll = Likelihood(path, CH.PRIOR, device=0, options=options or "")
    prob = CP.load_problem(path, CH.PRIOR, use_only_cell_ix=only)
    x = CH.draws(8, 3)
    yield request.param, ll, prob, x, (path, only)
    ll.close()


def test_time_points_on_gpu_values(tp_case):
    """the oracle's data likelihoods on the GPU's own simulated cells give the GPU logp"""
    name, ll, prob, x, src = tp_case
    lp, status = ll.evaluate_batch(x)
    e = prob["experiments"][0]
    M, NS = len(e["output_times"]), len(e["model"].ode)
    for i in range(len(x)):
        rec, vals, _ = ll.cellpop_cells(i, M, NS)
        if status[i] != 0:
            assert lp[i] == -math.inf
            continue
        tv = [CP.transform(tf, v) for tf, v in zip(prob["transforms"], x[i])]
        total = 0.0
        for dli, d in enumerate(e["data"]):
            if d["kind"] == "time_points":
                total += CP._timepoints_logp(d, CP.notify_time_points(e, dli, vals), tv)
                continue
            assert d["kind"] == "time_course"
            traj = np.full((e["max_cells"], len(d["times"])), np.nan)
            for k, (tdl, t, ti, six) in enumerate(e["timepoints"]):
                if tdl == dli:
                    traj[:len(rec), ti] = vals[:, k]
            ok, v = CP._timecourse_logp(d, traj, [c < e["num_cells"] for c in range(len(rec))], tv)
            if not ok:
                break
            total += v
        if total == -math.inf or lp[i] == -math.inf:
            assert total == lp[i], (name, i, lp[i], total)
        else:
            assert abs(lp[i] - total) <= 1e-12 * (1 + abs(total)), (name, i, lp[i], total)


def test_time_points_match_oracle(tp_case):
    """against the oracle's own solve: the cell-population envelope, the -inf pattern identical"""
    name, ll, prob, x, src = tp_case
    lp, _ = ll.evaluate_batch(x)
    ref = CP.simulate(prob, x)["logp"]
    ref_nofma = CP.simulate(CP.load_problem(src[0], CH.PRIOR, variant="nofma", use_only_cell_ix=src[1]), x)["logp"]
    CH.check_logp(lp, None, ref, ref_nofma, name=f"time_points {name}")
    if name == "early_minus_inf":
        assert (lp == -math.inf).all()
    if name in ("normal", "late_entry", "columns", "one_cell"):
        assert np.isfinite(lp).all(), (name, lp)
