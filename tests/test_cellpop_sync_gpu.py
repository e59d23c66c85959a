"""GPU parity of synchronised cell-population data (the stored-integration-point cell kernel,
cellpop_solver.h CP_STORED) against the oracle (oracle/cellpop.py + the reference's CVODE in the
stored mode, oracle/cellpop_ref.cpp); the cases of tests/test_cellpop_sync.py.

  * on the GPU's own simulated cell values, the oracle's data likelihoods reproduce the GPU logp to
    1e-12 relative (isolates the data likelihoods from the solve);
  * against the oracle's own solve: the envelope of tests/test_cellpop_gpu.py (logp within
    2e-4 (1 + |logp|), the -inf pattern identical), the same cell counts, division decisions and
    synchronisation-point event times within 1e-3 h."""
import math

import numpy as np
import pytest

import cellpop_helpers as CH
import cellpop as CP
from test_cellpop_sync import CASES, only, sync_likelihood

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=list(CASES))
def sync_case(request, tmp_path_factory):
    from bcm3_amd.likelihood import Likelihood
    name = request.param
    path = sync_likelihood(tmp_path_factory.mktemp("sync_gpu"), name)
    opts = f"cellpop.use_only_cell_ix={CASES[name][2]}" if CASES[name][2] else ""
    ll = Likelihood(path, CH.PRIOR, device=0, options=opts)
    prob = CP.load_problem(path, CH.PRIOR, use_only_cell_ix=only(name))
    x = CH.draws(8, 3)
    yield name, ll, prob, x
    ll.close()


def _oracle_logp_on(e, prob, xrow, rec, vals):
    """the oracle's data likelihoods (Experiment.cpp:346-355) over given cells' entry values"""
    tv = [CP.transform(tf, v) for tf, v in zip(prob["transforms"], xrow)]
    total = 0.0
    for dli, d in enumerate(e["data"]):
        if d["kind"] == "time_points":
            traj = CP.notify_time_points(e, dli, vals)
            total += CP._timepoints_logp(d, traj, tv)
            continue
        traj = np.full((e["max_cells"], len(d["times"])), np.nan)
        avg = np.zeros((len(d["times"]), 1))
        for k, (tdl, t, ti, six) in enumerate(e["timepoints"]):
            if tdl != dli or ti < 0:
                continue
            traj[:len(rec), ti] = vals[:, k]
            if d["kind"] == "time_course_population_average":
                pop = sum(1 for c in range(len(rec)) if 0.0 <= t - rec["creation"][c] <= rec["sim_end"][c])
                for c in range(len(rec)):
                    if vals[c, k] == vals[c, k]:
                        avg[ti, 0] += vals[c, k] / pop
        if d["kind"] == "time_course":
            ok, v = CP._timecourse_logp(d, traj, [c < e["num_cells"] for c in range(len(rec))], tv)
            if not ok:
                break
            total += v
        else:
            total += CP._popavg_logp(d, avg, tv)
    return total


def test_sync_on_gpu_values(sync_case):
    name, ll, prob, x = sync_case
    lp, status = ll.evaluate_batch(x)
    e = prob["experiments"][0]
    M, NS = len(e["output_times"]), len(e["model"].ode)
    checked = 0
    for i in range(len(x)):
        if status[i] != 0:
            assert lp[i] == -math.inf
            continue
        rec, vals, _ = ll.cellpop_cells(i, M, NS)
        total = _oracle_logp_on(e, prob, x[i], rec, vals)
        if total == -math.inf or lp[i] == -math.inf:
            assert total == lp[i], (name, i)
        else:
            assert abs(lp[i] - total) <= 1e-12 * (1 + abs(total)), (name, i, lp[i], total)
            checked += 1
    assert checked > 0, name


def test_sync_matches_oracle(sync_case):
    name, ll, prob, x = sync_case
    lp, status = ll.evaluate_batch(x)
    r = CP.simulate(prob, x)
    ref = r["logp"]
    e = prob["experiments"][0]
    M, NS = len(e["output_times"]), len(e["model"].ode)
    for i in range(len(x)):
        if ref[i] == -math.inf:
            assert lp[i] == -math.inf, (name, i)
        else:
            assert abs(lp[i] - ref[i]) <= 2e-4 * (1.0 + abs(ref[i])), (name, i, lp[i], ref[i])
        if status[i] != 0:
            continue
        cells = r["detail"][i]["cells"] if "detail" in r and isinstance(r["detail"], list) else None
        if cells is None:
            continue
        rec, vals, _ = ll.cellpop_cells(i, M, NS)
        assert len(rec) == len(cells), (name, i)
        for c, oc in enumerate(cells):
            assert bool(rec["flags"][c] & 2) == oc["divided"], (name, i, c)
            assert abs(rec["sim_end"][c] - oc["sim_end"]) <= 1e-3, (name, i, c, rec["sim_end"][c], oc["sim_end"])
            assert abs(rec["creation"][c] - oc["creation"]) <= 1e-3, (name, i, c)
            # every synchronised value exists on both sides or on neither (NaN pattern), and agrees
            gv, ov = vals[c], oc["values"]
            assert (np.isnan(gv) == np.isnan(ov)).all(), (name, i, c)
            fin = ~np.isnan(ov)
            assert np.allclose(gv[fin], ov[fin], rtol=1e-3, atol=1e-6), (name, i, c)
