"""CPU tests of the time-course data likelihood (DataLikelihoodTimeCourse, the cell-population
likelihood's default data type): the oracle's restatement of the vendored matching routine
(oracle/hungarian.py) pinned against that dependency's own test (brute force on integer-cost graphs,
dependencies/hungarian2/test.cpp:45-80) and on the behaviours it keeps, the oracle's time-course
evaluation on the reference's rules, and the product's loader (its options and refusals)."""
import math
import os
import random

import numpy as np
import pytest

import cellpop_helpers as CH
import cellpop as CP
import hungarian as HG

TC_DATA = os.path.join(CH.GOLDEN, "cellpop_tc_data.json")


def _cost(edges, match):
    c = {(l, r): w for l, r, w in edges}
    return sum(c[(i, j)] for i, j in enumerate(match))


def test_matching_agrees_with_brute_force_on_the_dependencys_test_graphs():
    """test.cpp:48-80: n = 10, each left node i joined to (i-2 .. i+1) mod n with costs rand() % 7;
    integer costs make the routine's int truncation exact, so it must reach the optimum"""
    rng = random.Random(1)
    for _ in range(20):
        n = 10
        edges = [(i, (j + n) % n, float(rng.randrange(7))) for i in range(n) for j in range(i - 2, i + 2)]
        truth = HG.brute_force(n, edges)
        got = HG.min_weight_perfect_matching(n, n, edges)
        assert sorted(got) == list(range(n))
        assert _cost(edges, got) == _cost(edges, truth)


def test_matching_on_complete_integer_graphs():
    rng = random.Random(7)
    for n in (1, 2, 3, 5, 6):
        for _ in range(10):
            edges = [(i, j, float(rng.randrange(-20, 20))) for i in range(n) for j in range(n)]
            got = HG.min_weight_perfect_matching(n, n, edges)
            assert _cost(edges, got) == _cost(edges, HG.brute_force(n, edges))


def test_matching_keeps_the_int_truncation_of_the_tight_test():
    """hungarian.cpp:167: a reduced cost below 1 counts as tight, so the greedy start takes it and the
    routine returns a matching that is not the cheapest: costs [[0, 0.3], [0, 0.9]] give 0->0, 1->1
    (0.9) where 0->1, 1->0 costs 0.3"""
    edges = [(0, 0, 0.0), (0, 1, 0.3), (1, 0, 0.0), (1, 1, 0.9)]
    assert HG.min_weight_perfect_matching(2, 2, edges) == [0, 1]
    assert HG.brute_force(2, edges) == [1, 0]
    # scaled by 10 the truncation no longer hides the difference
    edges10 = [(l, r, 10 * c) for l, r, c in edges]
    assert HG.min_weight_perfect_matching(2, 2, edges10) == [1, 0]
    # x86-64 converts out-of-range reduced costs to INT_MIN: tight
    assert HG._tight0(3e9) and HG._tight0(float("nan")) and HG._tight0(0.999) and not HG._tight0(1.0)


def test_matching_without_perfect_matching():
    # a right node without edges (n_right < n), and a left node whose only edge is taken
    assert HG.min_weight_perfect_matching(2, 1, [(0, 0, 1.0), (1, 0, 2.0)]) == []
    assert HG.min_weight_perfect_matching(2, 2, [(0, 0, 1.0), (1, 0, 2.0)]) == []


def tc_likelihood(directory, data_xml, num_cells=16, max_cells=16, name="tc.xml", **kw):
    import make_cellpop_fixtures as F
    path = os.path.join(str(directory), name)
    kw.setdefault("experiment_attrs", ' divide_cells="false"')
    with open(path, "w") as f:
        f.write(F.likelihood_text(num_cells=num_cells, max_cells=max_cells, data_file=TC_DATA,
                                  model_file=os.path.join(CH.GOLDEN, "cellpop_model.xml"), data_xml=data_xml, **kw))
    return path


TC = '<data data_name="pcna_cells" species_name="PCNA_gfp" stdev="stdev"/>'


@pytest.fixture(scope="module")
def tc_problem(tmp_path_factory):
    d = tmp_path_factory.mktemp("tc")
    return CP.load_problem(tc_likelihood(d, TC), CH.PRIOR)


def test_oracle_time_course_is_the_matched_sum(tc_problem):
    """Evaluate's sum: every observed cell's likelihood against the simulated cell the routine gives
    it, in observed-cell order, times the weight; the default type is time_course"""
    e = tc_problem["experiments"][0]
    assert e["data"][0]["kind"] == "time_course" and e["data"][0]["observed"].shape == (16, 21)
    x = CH.draws(3, 5)
    for v in x:
        r = CP.simulate_experiment(e, tc_problem, v)
        assert r["ok"] and len(r["cells"]) == 16 and math.isfinite(r["logp"])
    # at the true parameters the data's own cells are found again better than by chance
    r = CP.simulate_experiment(e, tc_problem, x[0])
    assert r["logp"] > CP.simulate_experiment(e, tc_problem, x[1])["logp"]


def test_oracle_time_course_missing_simulation_penalty(tmp_path):
    """cells created at t = 1.5 have no simulated value at 0 and 1: those observations cost
    LogPdfNormal(distance to the first simulated time point, 0, missing_simulation_time_stdev)"""
    p = CP.load_problem(tc_likelihood(tmp_path, TC.replace("/>", ' missing_simulation_time_stdev="2.5"/>'),
                                      entry_time="1.5"), CH.PRIOR)
    e = p["experiments"][0]
    assert e["data"][0]["missing_stdev"] == ("fixed", 2.5)
    r = CP.simulate_experiment(e, p, CH.draws(1, 5)[0])
    traj = r["cell_trajectories"][0]
    assert np.isnan(traj[:, :2]).all() and not np.isnan(traj[:, 2:]).any()
    assert math.isfinite(r["logp"])


def test_oracle_time_course_division_gives_minus_inf(tmp_path):
    """with division the daughters are simulated cells with a parent: not matchable, so every
    observed cell has fewer finite likelihoods than there are observed cells (.cpp:316-320)"""
    p = CP.load_problem(tc_likelihood(tmp_path, TC, num_cells=4, max_cells=16, experiment_attrs=""), CH.PRIOR)
    r = CP.simulate_experiment(p["experiments"][0], p, CH.draws(1, 5)[0])
    assert r["logp"] == -math.inf


def test_oracle_nan_cell_likelihood_ends_the_sum(tmp_path):
    """proportional_normal on a species that is 0 at t = 0: sigma = 0 and the cell likelihood is
    NaN, Evaluate returns false and Experiment::EvaluateLogProbability keeps the sum of the data
    likelihoods before it (Experiment.cpp:348-355): the population average alone"""
    both = ('<data type="time_course_population_average" data_name="pcna_mean" species_name="PCNA_gfp" stdev="stdev"/>'
            '<data data_name="pcna_cells" species_name="PCNA_gfp" stdev="stdev" error_model="proportional_normal" '
            'proportional_stdev="0.1"/>')
    p = CP.load_problem(tc_likelihood(tmp_path, both), CH.PRIOR)
    popavg = CP.load_problem(tc_likelihood(tmp_path, both.split("<data data_name")[0], name="pa.xml"), CH.PRIOR)
    v = CH.draws(1, 5)[0]
    r = CP.simulate_experiment(p["experiments"][0], p, v)
    assert r["logp"] == CP.simulate_experiment(popavg["experiments"][0], popavg, v)["logp"]
    assert math.isfinite(r["logp"])


def test_oracle_reads_one_and_three_dimensional_data(tmp_path):
    one = CP.load_problem(tc_likelihood(tmp_path, TC.replace("pcna_cells", "pcna_cell0"), num_cells=1, max_cells=1,
                                        name="one.xml"), CH.PRIOR)
    assert one["experiments"][0]["data"][0]["observed"].shape == (1, 21)
    three = CP.load_problem(tc_likelihood(tmp_path, TC.replace("pcna_cells", "pcna_cells_markers"), name="three.xml"),
                            CH.PRIOR)
    two = CP.load_problem(tc_likelihood(tmp_path, TC, name="two.xml"), CH.PRIOR)
    np.testing.assert_array_equal(three["experiments"][0]["data"][0]["observed"], two["experiments"][0]["data"][0]["observed"])
    pick = CP.load_problem(tc_likelihood(tmp_path, TC, num_cells=3, max_cells=3, name="pick.xml"), CH.PRIOR,
                           use_only_cell_ix="4,0,9")
    np.testing.assert_array_equal(pick["experiments"][0]["data"][0]["observed"],
                                  two["experiments"][0]["data"][0]["observed"][[4, 0, 9]])


def _lik(path, options="backend=none"):
    from bcm3_amd.likelihood import Likelihood
    return Likelihood(path, CH.PRIOR, options=options)


def test_loader_accepts_time_course(tmp_path):
    for data_xml, kw in ((TC, {}), (TC.replace("pcna_cells", "pcna_cell0"), dict(num_cells=1, max_cells=1)),
                         (TC.replace("pcna_cells", "pcna_cells_markers"), {}),
                         (TC.replace('stdev="stdev"', 'stdev="stdev" type="time_course" synchronize="none" '
                                     'missing_simulation_time_stdev="stdev" error_model="t4" weight="0.5"'), {}),
                         (TC.replace("/>", ' synchronize="mitosis"/>'), {}),
                         (TC.replace("/>", ' synchronize="DNA_replication_start"/>'),
                          dict(experiment_attrs=' divide_cells="false" synchronization_time_offset="k_D"'))):
        _lik(tc_likelihood(tmp_path, data_xml, **kw)).close()
    _lik(tc_likelihood(tmp_path, TC, num_cells=3, max_cells=3), "backend=none;cellpop.use_only_cell_ix=4,0,9").close()


@pytest.mark.parametrize("data_xml,kw,options", [
    (TC, dict(max_cells=20), None),                                       # more simulated than observed cells
    (TC, dict(max_cells=8, num_cells=8), None),                           # fewer
    (TC.replace("/>", ' synchronize="bogus"/>'), {}, None),
    (TC.replace("/>", ' use_log_ratio="true"/>'), {}, None),
    (TC.replace("/>", ' saturation_scale="2"/>'), {}, None),
    (TC.replace("pcna_cells", "pcna_cell0"), dict(num_cells=1, max_cells=1), "backend=none;cellpop.use_only_cell_ix=0"),
    (TC, dict(num_cells=2, max_cells=2), "backend=none;cellpop.use_only_cell_ix=0,16"),  # out of range
    (TC.replace('data_name=', 'type="duration" data_name='), {}, None),
    (TC.replace('data_name=', 'type="nonsense" data_name='), {}, None),
])
def test_loader_refuses(tmp_path, data_xml, kw, options):
    with pytest.raises(RuntimeError):
        _lik(tc_likelihood(tmp_path, data_xml, **kw), options or "backend=none")
