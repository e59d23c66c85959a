"""Several <experiment>s in one cell_population likelihood (CellPopulationLikelihood::
EvaluateLogProbability, src/cellpop/CellPopulationLikelihood.cpp:82-101): logp is the sum of the
experiments' log-likelihoods in experiment order, -inf when one fails. Checked on MI355X against
the single-experiment likelihoods evaluated separately (each pinned to the oracle by
tests/test_cellpop_gpu.py): the sum must be bit-identical."""
import numpy as np
import pytest

import cellpop_helpers as CH

pytestmark = pytest.mark.gpu


def two_experiments(d):
    a = CH.write_likelihood(d, 6, 64, name="a.xml")
    b = CH.write_likelihood(d, 4, 32, name="b.xml", data_attrs='stdev="stdev" error_model="t4"',
                            experiment_attrs=' divide_cells="false"')
    ta, tb = open(a).read(), open(b).read()
    exp_b = tb[tb.index("<experiment"):tb.index("</experiment>") + len("</experiment>")]
    multi = ta.replace("</bcm_likelihood>", "  " + exp_b + "\n</bcm_likelihood>")
    path = str(d / "ab.xml")
    with open(path, "w") as f:
        f.write(multi)
    return a, b, path


def test_two_experiments_sum(tmp_path):
    from bcm3_amd.likelihood import Likelihood
    a, b, ab = two_experiments(tmp_path)
    x = CH.draws(8, 23)
    out = {}
    for k, p in (("a", a), ("b", b), ("ab", ab)):
        ll = Likelihood(p, CH.PRIOR, device=0)
        out[k] = ll.evaluate_batch(x)
        ll.close()
    (la, sa), (lb, sb), (lab, sab) = out["a"], out["b"], out["ab"]
    assert np.isfinite(la).sum() >= 2 and np.isfinite(lb).sum() >= 2
    expect = np.where(np.isfinite(la) & np.isfinite(lb), la + lb, -np.inf)
    assert np.array_equal(lab, expect), (lab, expect)
    assert np.array_equal(sab != 0, (sa != 0) | (sb != 0))


def test_two_experiments_vs_oracle(tmp_path):
    """the restated CellPopulationLikelihood (oracle/cellpop.py simulate: the experiments' logp
    summed in order) within the envelope of tests/test_cellpop_gpu.py"""
    import cellpop as CP
    from bcm3_amd.likelihood import Likelihood
    _, _, ab = two_experiments(tmp_path)
    x = CH.draws(6, 29)
    ll = Likelihood(ab, CH.PRIOR, device=0)
    lp, _ = ll.evaluate_batch(x)
    ll.close()
    ref = CP.simulate(CP.load_problem(ab, CH.PRIOR), x)["logp"]
    nofma = CP.simulate(CP.load_problem(ab, CH.PRIOR, variant="nofma"), x)["logp"]
    assert np.array_equal(np.isfinite(lp), np.isfinite(ref))
    CH.check_logp(lp, None, ref, nofma, name="two experiments")


def test_dp5_and_synchronised_experiments_sum(tmp_path):
    """one experiment on the DP5 solver, one with synchronised data (the stored-integration-point
    kernel): each experiment compiles its own cell kernel; the sum is bit-identical to the two
    likelihoods evaluated separately"""
    from bcm3_amd.likelihood import Likelihood
    from test_cellpop_dp5 import dp5_likelihood
    from test_cellpop_sync import sync_likelihood
    a = dp5_likelihood(tmp_path, "no_division")
    b = sync_likelihood(tmp_path, "replication")
    ta, tb = open(a).read(), open(b).read()
    exp_b = tb[tb.index("<experiment"):tb.index("</experiment>") + len("</experiment>")]
    ab = str(tmp_path / "dp5_sync.xml")
    with open(ab, "w") as f:
        f.write(ta.replace("</bcm_likelihood>", "  " + exp_b + "\n</bcm_likelihood>"))
    x = CH.draws(6, 31)
    out = {}
    for k, p in (("a", a), ("b", b), ("ab", ab)):
        ll = Likelihood(p, CH.PRIOR, device=0)
        out[k] = ll.evaluate_batch(x)
        ll.close()
    (la, _), (lb, _), (lab, _) = out["a"], out["b"], out["ab"]
    assert np.isfinite(la).sum() >= 2 and np.isfinite(lb).sum() >= 2
    expect = np.where(np.isfinite(la) & np.isfinite(lb), la + lb, -np.inf)
    assert np.array_equal(lab, expect), (lab, expect)
