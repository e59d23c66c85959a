"""GPU parity of synchronised cell-population data (the stored-integration-point cell kernel,
cellpop_solver.h CP_STORED) against the oracle (oracle/cellpop.py + the reference's CVODE in the
stored mode, oracle/cellpop_ref.cpp); the cases of tests/test_cellpop_sync.py.

  * on the GPU's own simulated cell values, the oracle's data likelihoods reproduce the GPU logp to
    1e-12 relative (isolates the data likelihoods from the solve);
  * against the oracle's own solve: the envelope of tests/test_cellpop_gpu.py (cellpop_helpers.logp_bar,
    the -inf pattern identical), the same cell counts, division decisions and
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
    yield name, ll, prob, x, path
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
                # counted at data time + offset (Experiment.cpp:285, 301)
                tt = t + CP._refval(e.get("sync_offset", ("fixed", 0.0)), tv)
                pop = sum(1 for c in range(len(rec)) if 0.0 <= tt - rec["creation"][c] <= rec["sim_end"][c])
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
    name, ll, prob, x, path = sync_case
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
    name, ll, prob, x, path = sync_case
    lp, status = ll.evaluate_batch(x)
    r = CP.simulate(prob, x)
    ref = r["logp"]
    e = prob["experiments"][0]
    M, NS = len(e["output_times"]), len(e["model"].ode)
    ref_nofma = CP.simulate(CP.load_problem(path, CH.PRIOR, variant="nofma", use_only_cell_ix=only(name)), x)["logp"]
    CH.check_logp(lp, None, ref, ref_nofma, name=f"sync {name}")
    for i in range(len(x)):
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


def test_store_grows_and_reruns_the_generation(monkeypatch):
    """the integration-point store starts at a cap below the steps the cells take
    (BCM3_CP_STORE_CAP0=8): every generation overflows, the store doubles and the generation runs
    again -- the logp equals the default store's bit for bit, at two batch sizes (a budget
    cap made the same model fail at one batch size and run at another)"""
    import tempfile
    from bcm3_amd.likelihood import Likelihood
    d = tempfile.mkdtemp()
    path = sync_likelihood(d, "division")
    opts = f"cellpop.use_only_cell_ix={CASES['division'][2]}"
    x = CH.draws(12, 7)
    ll = Likelihood(path, CH.PRIOR, device=0, options=opts)
    want, wst = ll.evaluate_batch(x)
    ll.close()
    monkeypatch.setenv("BCM3_CP_STORE_CAP0", "8")
    ll = Likelihood(path, CH.PRIOR, device=0, options=opts)
    for n in (3, 12):
        got, gst = ll.evaluate_batch(x[:n])
        assert np.array_equal(got, want[:n], equal_nan=True), (n, got, want[:n])
        assert np.array_equal(gst, wst[:n])
    ll.close()
    assert np.isfinite(want).any()
