"""CPU tests of time courses with an observed cell lineage (the data group's "cell_id" / "parent",
DataLikelihoodTimeCourse.cpp:132-167; CalculateCellLikelihood's recursion, :431-563): the oracle's
restatement of the reference's rules on hand-made cases, and the product's loader.

The reference's rules kept (and what they imply):
  * only the observed cells without a parent are matched, against n = max(roots, simulated cells)
    left nodes: any simulated division (more simulated cells than roots) gives -inf;
  * a matched simulated cell without daughters: each observed child's missing-value penalty
    REPLACES the parent's sum (assignment in the loop, .cpp:555-557), so an observed root with
    children scores its last child's subtree penalty only;
  * with simulated daughters: one observed child takes the better daughter, two or more add
    nothing (the #if TODO block), a daughter with no finite child gives -inf.
Parity of these rules is unpinned by reference fixtures (the reference ships none for lineages);
the restatement follows the source line by line."""
import math
import os

import numpy as np
import pytest

import cellpop_helpers as CH
import cellpop as CP

LIN_DATA = os.path.join(CH.GOLDEN, "cellpop_lineage_data.json")
TC = '<data data_name="pcna_cells" species_name="PCNA_gfp" stdev="stdev"/>'

CASES = {
    # 8 roots matched to 8 initial cells that never divide: the finite case
    "no_division": (TC, dict(num_cells=8, max_cells=16, experiment_attrs=' divide_cells="false"'), None),
    "t4_missing": (TC.replace('stdev="stdev"', 'stdev="stdev" error_model="t4" missing_simulation_time_stdev="stdev"'),
                   dict(num_cells=8, max_cells=16, experiment_attrs=' divide_cells="false"'), None),
    # dividing cells: more simulated cells than roots -> -inf (or a failure beyond max_cells)
    "division": (TC, dict(num_cells=8, max_cells=16, experiment_attrs=""), None),
    # a subset of the observed cells: roots 0, 1 and their children 8, 10, 13's parent 8
    "subset": (TC, dict(num_cells=2, max_cells=5, experiment_attrs=' divide_cells="false"'), "0,8,1,10,13"),
}


def lineage_likelihood(directory, name):
    import make_cellpop_fixtures as F
    data_xml, kw, _ = CASES[name]
    path = os.path.join(str(directory), f"lineage_{name}.xml")
    with open(path, "w") as f:
        f.write(F.likelihood_text(data_file=LIN_DATA, model_file=os.path.join(CH.GOLDEN, "cellpop_model.xml"),
                                  data_xml=data_xml, **kw))
    return path


def only(name):
    return CASES[name][2] or "-1"


def test_lineage_loaded_as_the_reference_reads_it(tmp_path):
    e = CP.load_problem(lineage_likelihood(tmp_path, "no_division"), CH.PRIOR)["experiments"][0]
    roots, children = e["data"][0]["lineage"]
    assert roots == list(range(8))
    assert children[0] == [8, 9] and children[8] == [13] and children[1] == [10] and children[13] == []
    e = CP.load_problem(lineage_likelihood(tmp_path, "subset"), CH.PRIOR, use_only_cell_ix=only("subset"))["experiments"][0]
    roots, children = e["data"][0]["lineage"]
    # picked cells 0, 8, 1, 10, 13 -> positions 0..4; 8 is 0's child, 10 is 1's, 13 is 8's
    assert roots == [0, 2] and children == [[1], [4], [3], [], []]


def _tc_inputs(tmp_path, name, nsim_roots):
    e = CP.load_problem(lineage_likelihood(tmp_path, name), CH.PRIOR, use_only_cell_ix=only(name))["experiments"][0]
    d = e["data"][0]
    T = len(d["times"])
    rng = np.random.default_rng(1)
    traj = np.full((e["max_cells"], T), np.nan)
    traj[:nsim_roots] = d["observed"][:nsim_roots] + 0.01 * rng.standard_normal((nsim_roots, T))
    tv = [1.0] * 7
    tv[6] = 0.1  # stdev
    return e, d, traj, tv


def test_root_with_children_scores_its_last_childs_penalty(tmp_path):
    """no simulated daughters: each root's likelihood is the missing-value penalty of its last observed
    child's subtree (assigned, not added), roots without children their own data likelihood"""
    e, d, traj, tv = _tc_inputs(tmp_path, "no_division", 8)
    ok, lp = CP._timecourse_logp(d, traj, [True] * 8, tv, [-1] * 8)
    assert ok and np.isfinite(lp)
    roots, children = d["lineage"]
    times, obs = d["times"], d["observed"]
    msd = 300.0

    def pen(o):
        s = sum(CP._log_pdf_normal(times[k], 0.0, msd) for k in range(len(times)) if not math.isnan(obs[o, k]))
        return s + sum(pen(c) for c in children[o])

    # root 6 and 7 have no children: their row is the plain cell likelihood; root 0 with children
    # 8, 9 takes pen(9) for every simulated cell
    nolin = dict(d, lineage=None)
    _, lp_plain = CP._timecourse_logp(nolin, traj, [True] * 8, tv)
    assert lp != lp_plain
    # the recursion's value for (root 0, any simulated cell) is pen(9): check through a one-root lineage
    one = dict(d, lineage=([0], children), observed=obs)
    ok1, lp1 = CP._timecourse_logp(one, traj[:1], [True], tv, [-1])
    assert ok1 and lp1 == pytest.approx(pen(9) * 1.0, rel=1e-15)


def test_simulated_daughters_rules(tmp_path):
    """with daughters: one observed child takes the better daughter; two children add nothing; the
    extra simulated cells make n > roots -> -inf from the matching"""
    e, d, traj, tv = _tc_inputs(tmp_path, "no_division", 8)
    roots, children = d["lineage"]
    # one root (1, child 10) and one simulated root with daughters 1, 2
    tr = np.full((3, traj.shape[1]), np.nan)
    tr[0] = traj[1]
    tr[1] = d["observed"][10] + 0.02
    tr[2] = d["observed"][10] - 0.5
    one = dict(d, lineage=([1], children))
    ok, lp = CP._timecourse_logp(one, tr, [True, False, False], tv, [1, -1, -1])
    assert ok and lp == -math.inf  # 3 simulated cells > 1 root
    # the recursion itself: root 1 with child 10 against daughter 1 (better) / 2
    own = CP._timecourse_logp(dict(d, lineage=None, observed=d["observed"][[1]]), tr[:1], [True], tv)[1]
    best = CP._timecourse_logp(dict(d, lineage=None, observed=d["observed"][[10]]), tr[1:2], [True], tv)[1]
    worse = CP._timecourse_logp(dict(d, lineage=None, observed=d["observed"][[10]]), tr[2:3], [True], tv)[1]
    assert best > worse
    assert np.isfinite(own + best)


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_builds_agree(tmp_path, name):
    path = lineage_likelihood(tmp_path, name)
    x = CH.draws(3, 5)
    a = CP.simulate(CP.load_problem(path, CH.PRIOR, use_only_cell_ix=only(name)), x)["logp"]
    b = CP.simulate(CP.load_problem(path, CH.PRIOR, variant="nofma", use_only_cell_ix=only(name)), x)["logp"]
    assert ((a == -math.inf) == (b == -math.inf)).all()
    fin = np.isfinite(a)
    assert (np.abs(a[fin] - b[fin]) <= 1e-6 * (1 + np.abs(a[fin]))).all()
    if name in ("no_division", "t4_missing", "subset"):
        assert fin.all(), name
    if name == "division":
        assert not fin.any()


@pytest.mark.parametrize("name", list(CASES))
def test_loader_accepts_lineages(tmp_path, name):
    from bcm3_amd import likelihood
    opts = "backend=none" + (f";cellpop.use_only_cell_ix={CASES[name][2]}" if CASES[name][2] else "")
    likelihood.Likelihood(lineage_likelihood(tmp_path, name), CH.PRIOR, options=opts).close()


def test_loader_refuses_a_missing_parent(tmp_path):
    """a parent outside the picked cells: "Could not find cell ... for parent" (.cpp:153-157)"""
    from bcm3_amd import likelihood
    path = lineage_likelihood(tmp_path, "subset")
    with pytest.raises(RuntimeError):
        likelihood.Likelihood(path, CH.PRIOR, options="backend=none;cellpop.use_only_cell_ix=0,13,1,10,2")
