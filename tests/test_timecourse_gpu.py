"""GPU parity of the time-course data likelihood (DataLikelihoodTimeCourse) against the oracle.

Two layers:
  * the matching (cp_timecourse_kernel's assignment, run alone through bcm3hip_assign_cells) is
    integer/index work on given inputs: bit-exact against oracle/hungarian.py (the restatement of
    the reference's vendored hungarian2 routine) on the same cell-likelihood matrices, including the
    matrices on which that routine is not optimal, -inf and NaN entries, and workspaces in LDS and
    in global memory;
  * the whole likelihood: the GPU's per-cell values fed to the oracle's time-course evaluation give
    the GPU's logp to 1e-12 relative (the cell likelihoods use the device's log / log1p, within an
    ulp of glibc's), and the GPU logp sits in the cell-population envelope of test_cellpop_gpu.py
    against the oracle's own reference-CVODE solve."""
import math

import numpy as np
import pytest

import cellpop_helpers as CH
import cellpop as CP
import hungarian as HG
from test_timecourse import TC, tc_likelihood

pytestmark = pytest.mark.gpu


def _oracle_assign(L):
    """DataLikelihoodTimeCourse::Evaluate's loop (.cpp:287-335) over a given likelihood matrix"""
    R, S = L.shape
    edges = []
    for i in range(R):
        finite = 0
        for j in range(S):
            if math.isnan(L[i, j]):
                return None, -math.inf, 0
            finite += L[i, j] > -math.inf
            edges.append((i, j, -L[i, j]))
        if finite < R:
            return None, -math.inf, 1
    m = HG.min_weight_perfect_matching(max(R, S), S, edges)
    if len(m) != R:
        return None, -math.inf, 1
    lp = 0.0
    for i in range(R):
        lp += L[i, m[i]]
    return m, lp, 1


@pytest.mark.parametrize("R,spread,problems", [(1, 5.0, 8), (2, 0.6, 64), (5, 3.0, 64), (16, 2.0, 64), (16, 40.0, 32),
                                                (64, 3.0, 8), (100, 3.0, 3)])
def test_matching_bit_exact(R, spread, problems):
    """random likelihood matrices: spread ~1 puts many reduced costs below 1 (the routine's int
    truncation), 40 almost none; R = 100 runs from a global-memory workspace"""
    import torch
    from bcm3_amd import _hip
    rng = np.random.default_rng(R * 1000 + problems)
    L = -100.0 + spread * rng.standard_normal((problems, R, R))
    m, s, ok = _hip.assign_cells(torch.tensor(L, device="cuda"))
    for p in range(problems):
        rm, rs, rok = _oracle_assign(L[p])
        assert ok[p] == rok
        assert s[p] == rs, (p, s[p], rs)
        assert list(m[p]) == rm, p


def test_matching_special_entries():
    import torch
    from bcm3_amd import _hip
    L = np.full((6, 4, 4), -10.0)
    L[:, np.arange(4), np.arange(4)] = -1.0
    L[1, 2, 3] = -math.inf               # one -inf: that row has fewer finite entries than rows
    L[2, 3, 0] = math.nan                # NaN: Evaluate fails
    L[3, 0, 1] = math.nan
    L[3, 0, 2] = -math.inf               # the NaN comes first in row 0 -> failure
    L[4, 1, :] = -math.inf
    L[4, 0, 0] = math.nan                # row 0's NaN ends the loop before row 1's -infs
    L[5] = np.array([[0.0, -0.3, -5, -5], [0.0, -0.9, -5, -5], [-5, -5, -1, -1.5], [-5, -5, -1.2, -1.1]])
    m, s, ok = _hip.assign_cells(torch.tensor(L, device="cuda"))
    for p in range(6):
        rm, rs, rok = _oracle_assign(L[p])
        assert (ok[p], s[p]) == (rok, rs), p
        if rm is not None:
            assert list(m[p]) == rm
    assert list(ok) == [1, 1, 0, 0, 0, 1] and s[1] == -math.inf
    assert list(m[5][:2]) == [0, 1]  # the routine's non-optimal pick (0.9 where 0.3 exists)
    # fewer simulated than observed cells: a node without edges, no matching
    m, s, ok = _hip.assign_cells(torch.tensor(np.full((2, 3, 2), -1.0), device="cuda"))
    assert list(s) == [-math.inf] * 2 and list(ok) == [1, 1]


# (data element, likelihood kwargs, options) of the whole-likelihood cases
CASES = {
    "normal": (TC, {}, None),
    "t4_missing": (TC.replace('stdev="stdev"', 'stdev="stdev" error_model="t4" missing_simulation_time_stdev="stdev"'),
                   dict(entry_time="1.5"), None),
    "addprop_weight": (TC.replace('stdev="stdev"', 'stdev="stdev" error_model="additive_proportional_normal" '
                                  'proportional_stdev="0.05" weight="0.5" offset="0.01" scale="1.1" '
                                  'stdev_relative_to_scale="true"'), {}, None),
    "markers_pick": (TC.replace("pcna_cells", "pcna_cells_markers"), dict(num_cells=3, max_cells=3),
                     "cellpop.use_only_cell_ix=4,0,9"),
    "one_cell": (TC.replace("pcna_cells", "pcna_cell0"), dict(num_cells=1, max_cells=1), None),
    "division": (TC, dict(num_cells=4, experiment_attrs=""), None),
    "nan_ends_sum": ('<data type="time_course_population_average" data_name="pcna_mean" species_name="PCNA_gfp" '
                     'stdev="stdev"/><data data_name="pcna_cells" species_name="PCNA_gfp" stdev="stdev" '
                     'error_model="proportional_normal" proportional_stdev="0.1"/>', {}, None),
    "two_time_courses": (TC + TC.replace('stdev="stdev"', 'stdev="0.2" error_model="t4"'), {}, None),
}


@pytest.fixture(scope="module", params=list(CASES))
def tc_case(request, tmp_path_factory):
    from bcm3_amd.likelihood import Likelihood
    data_xml, kw, options = CASES[request.param]
    d = tmp_path_factory.mktemp("tc_gpu")
    path = tc_likelihood(d, data_xml, **kw)
    only = options.split("=")[1] if options else "-1"
    ll = Likelihood(path, CH.PRIOR, device=0, options=options or "")
    prob = CP.load_problem(path, CH.PRIOR, use_only_cell_ix=only)
    x = CH.draws(8, 3)
    yield request.param, ll, prob, x, (path, only)
    ll.close()


def test_time_course_on_gpu_values_is_bit_exact(tc_case):
    """the oracle's DataLikelihoodTimeCourse::Evaluate on the GPU's own simulated cells reproduces
    the GPU logp (the matching exactly, the cell likelihoods to an ulp of log)"""
    name, ll, prob, x, src = tc_case
    lp, status = ll.evaluate_batch(x)
    e = prob["experiments"][0]
    M, NS = len(e["output_times"]), len(e["model"].ode)
    tv_all = [[CP.transform(tf, v) for tf, v in zip(prob["transforms"], row)] for row in x]
    for i in range(len(x)):
        rec, vals, _ = ll.cellpop_cells(i, M, NS)
        if status[i] != 0:  # a failed simulation (a cell's solver, or more cells than max_cells):
            assert lp[i] == -math.inf  # the -inf pattern is checked against the oracle below
            continue
        # the oracle's data likelihood sum over the GPU's cells (Experiment.cpp:346-355)
        total = 0.0
        for dli, d in enumerate(e["data"]):
            traj = np.full((e["max_cells"], len(d["times"])), np.nan)
            for k, (tdl, t, ti, six) in enumerate(e["timepoints"]):
                if tdl == dli:
                    traj[:len(rec), ti] = vals[:, k]
            if d["kind"] == "time_course":
                roots = [c < e["num_cells"] for c in range(len(rec))]
                ok, v = CP._timecourse_logp(d, traj, roots, tv_all[i])
                if not ok:
                    break
                total += v
            else:
                avg = np.zeros((len(d["times"]), 1))
                for k, (tdl, t, ti, six) in enumerate(e["timepoints"]):
                    if tdl == dli:
                        pop = sum(1 for c in range(len(rec)) if 0.0 <= t - rec["creation"][c] <= rec["sim_end"][c])
                        for c in range(len(rec)):
                            if vals[c, k] == vals[c, k]:
                                avg[ti, 0] += vals[c, k] / pop
                total += CP._popavg_logp(d, avg, tv_all[i])
        if total == -math.inf or lp[i] == -math.inf:
            assert total == lp[i], (name, i)
        else:
            assert abs(lp[i] - total) <= 1e-12 * (1 + abs(total)), (name, i, lp[i], total)


def test_time_course_matches_oracle(tc_case):
    """against the oracle's own solve (reference CVODE per cell): the envelope of
    test_cellpop_gpu.py, the -inf pattern identical"""
    name, ll, prob, x, src = tc_case
    lp, _ = ll.evaluate_batch(x)
    ref = CP.simulate(prob, x)["logp"]
    ref_nofma = CP.simulate(CP.load_problem(src[0], CH.PRIOR, variant="nofma", use_only_cell_ix=src[1]), x)["logp"]
    CH.check_logp(lp, None, ref, ref_nofma, name=f"time_course {name}")
    if name == "division":
        assert (lp == -math.inf).all()
    if name == "nan_ends_sum":
        assert np.isfinite(lp).all()
