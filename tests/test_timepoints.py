"""CPU tests of the time-points data likelihood (DataLikelihoodTimePoints,
src/cellpop/DataLikelihoodTimePoints.cpp): the oracle's restatement (oracle/cellpop.py
`_load_time_points`, `notify_time_points`, `_timepoints_logp`) on the reference's rules, and the
product's loader (its options and refusals). The matching routine itself is pinned in
tests/test_timecourse.py. Parity unpinned beyond that: the reference ships no time-points fixture."""
import math

import numpy as np
import pytest

import cellpop_helpers as CH
import cellpop as CP
from test_timecourse import TC, TC_DATA, tc_likelihood, _lik  # noqa: F401

TP = '<data type="time_points" data_name="pcna_cells" species_name="PCNA_gfp" stdev="stdev"/>'


def _tp(**attrs):
    s = TP
    for k, v in attrs.items():
        if k == "data_name":
            s = s.replace('data_name="pcna_cells"', f'data_name="{v}"')
        elif k == "species_name":
            s = s.replace('species_name="PCNA_gfp"', f'species_name="{v}"')
        elif k == "stdev":
            s = s.replace('stdev="stdev"', f'stdev="{v}"')
        else:
            s = s.replace("/>", f' {k}="{v}"/>')
    return s


def test_oracle_loads_columns_and_sums(tmp_path):
    """"a;b+a": two columns, the species registered once each in first-use order, column 1 adds
    both; 3-D data give cells x time points x markers"""
    p = CP.load_problem(tc_likelihood(tmp_path, _tp(data_name="pcna_cells_markers", species_name="PCNA_gfp;CycB + PCNA_gfp",
                                                    stdev="stdev;0.5")), CH.PRIOR)
    e = p["experiments"][0]
    d = e["data"][0]
    m = e["model"]
    assert d["kind"] == "time_points" and d["columns"] == 2 and d["observed"].shape == (16, 21, 2)
    assert d["species_order"] == [m.ode_index("PCNA_gfp"), m.ode_index("CycB")]
    assert d["species_map"] == {m.ode_index("PCNA_gfp"): [0, 1], m.ode_index("CycB"): [1]}
    assert len(e["timepoints"]) == 2 * 21
    r = CP.simulate_experiment(e, p, CH.draws(1, 5)[0])
    assert r["ok"] and math.isfinite(r["logp"])
    traj = r["cell_trajectories"][0]
    assert traj.shape == (16, 21, 2) and not np.isnan(traj).any()
    assert (traj[:, :, 1] >= traj[:, :, 0]).all()  # CycB >= 0 added to PCNA_gfp


def test_oracle_one_cell_is_the_plain_sum(tmp_path):
    """one observed and one simulated cell: no choice in the matching, so the likelihood is the sum
    over time points of LogPdfNormal(observed, simulated) -- the time course's value for the same
    cell (which multiplies by 1 / (2 sigma^2) where LogPdfNormal divides: 1e-12)"""
    kw = dict(num_cells=1, max_cells=1)
    tp = CP.load_problem(tc_likelihood(tmp_path, _tp(data_name="pcna_cell0_2d"), name="tp.xml", **kw), CH.PRIOR)
    tc = CP.load_problem(tc_likelihood(tmp_path, TC.replace("pcna_cells", "pcna_cell0"), name="tc.xml", **kw), CH.PRIOR)
    for v in CH.draws(3, 11):
        a = CP.simulate_experiment(tp["experiments"][0], tp, v)["logp"]
        b = CP.simulate_experiment(tc["experiments"][0], tc, v)["logp"]
        assert math.isfinite(a) and abs(a - b) <= 1e-12 * (1 + abs(b)), (a, b)


def test_oracle_too_few_simulated_cells_is_minus_inf(tmp_path):
    """cells enter at t = 1.5: at t = 0 the 16 observed cells meet no simulated cell (.cpp:241-245);
    with the first two time points' data missing the same problem is finite"""
    p = CP.load_problem(tc_likelihood(tmp_path, TP, entry_time="1.5"), CH.PRIOR)
    assert CP.simulate_experiment(p["experiments"][0], p, CH.draws(1, 5)[0])["logp"] == -math.inf
    p = CP.load_problem(tc_likelihood(tmp_path, _tp(data_name="pcna_cells_late"), entry_time="1.5", name="late.xml"),
                        CH.PRIOR)
    assert math.isfinite(CP.simulate_experiment(p["experiments"][0], p, CH.draws(1, 5)[0])["logp"])


def test_oracle_division_matches_the_first_simulated_cells(tmp_path):
    """with division more cells are alive than observed; the routine keeps edges to right nodes < n
    only (hungarian.cpp:52-84), so the observed cells are matched among the first alive cells"""
    p = CP.load_problem(tc_likelihood(tmp_path, TP, num_cells=4, max_cells=32, experiment_attrs=""), CH.PRIOR,
                        use_only_cell_ix="2,7,11")
    e = p["experiments"][0]
    r = CP.simulate_experiment(e, p, CH.draws(1, 5)[0])
    assert len(r["cells"]) > 4 and math.isfinite(r["logp"])
    nd = CP.load_problem(tc_likelihood(tmp_path, _tp(use_only_nondivided="true"), num_cells=4, max_cells=32,
                                       experiment_attrs="", name="nd.xml"), CH.PRIOR, use_only_cell_ix="2,7,11")
    traj = CP.simulate_experiment(nd["experiments"][0], nd, CH.draws(1, 5)[0])["cell_trajectories"][0]
    assert np.isnan(traj[4:]).all()  # daughters are never notified


def _loader_ok(tmp_path, data_xml, options="backend=none", **kw):
    _lik(tc_likelihood(tmp_path, data_xml, **kw), options).close()


def test_loader_accepts_time_points(tmp_path):
    for data_xml, kw in ((TP, {}), (_tp(error_model="t4", weight="0.5", offset="0.1", scale="stdev"), {}),
                         (_tp(data_name="pcna_cells_markers", species_name="PCNA_gfp; CycB+CycD", stdev="stdev;0.5"), {}),
                         (_tp(value_relative_to_timepoint_ix="3", synchronize="none"), {}),
                         (_tp(use_only_nondivided="true"), dict(num_cells=4, max_cells=32, experiment_attrs="")),
                         (TP + TC, {}), (_tp(synchronize="mitosis"), {}),
                         (_tp(synchronize="anaphase_onset") + TC.replace("/>", ' synchronize="PCNA_gfp_increase"/>'), {})):
        _loader_ok(tmp_path, data_xml, **kw)
    _loader_ok(tmp_path, TP, "backend=none;cellpop.use_only_cell_ix=4,0,9", num_cells=3, max_cells=3)


@pytest.mark.parametrize("data_xml,kw,options", [
    (_tp(error_model="proportional_normal", proportional_stdev="0.1"), {}, None),  # NaN in the reference
    (_tp(synchronize="bogus"), {}, None),
    (_tp(species_name="PCNA_gfp/CycB"), {}, None),                        # division of species
    (_tp(species_name="mitogen_missing"), {}, None),
    (_tp(species_name="PCNA_gfp;CycB"), {}, None),                       # 2 columns on 2-D data
    (TP, dict(num_cells=8, max_cells=8), None),                          # fewer simulated than observed
    (_tp(value_relative_to_timepoint_ix="21"), {}, None),
    (_tp(data_name="pcna_cells_markers"), {}, "backend=none;cellpop.use_only_cell_ix=0"),  # 3-D + pick
    (_tp(data_name="pcna_cell0"), dict(num_cells=1, max_cells=1), None),  # 1-D data
    (TC.replace('data_name=', 'type="duration" data_name='), {}, None),
])
def test_loader_refuses(tmp_path, data_xml, kw, options):
    with pytest.raises(RuntimeError):
        _lik(tc_likelihood(tmp_path, data_xml, **kw), options or "backend=none")
