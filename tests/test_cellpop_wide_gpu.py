"""The cell kernel's one-cell-per-wavefront form (cellpop_solver.h: ROW = 64 when a model has more than 16
ODE species; the four-cell form covers every other cell-population test): the C4 model with six reporter
species appended (cellpop_helpers.write_wide_model, NS = 21) against the oracle -- the reference's
CVODE per cell under the restated Experiment logic -- with the cell-population envelope
(cellpop_helpers.logp_bar), identical cell counts and division decisions; and the work queue forced
onto this form (BCM3_CP_QUEUE=1, one cell per wavefront round) bit-identical to the generation launches
the form runs by default."""
import numpy as np
import pytest

import cellpop as CP
import cellpop_helpers as CH

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wide(tmp_path_factory):
    d = tmp_path_factory.mktemp("wide")
    path = CH.write_wide_likelihood(d, 6, 64)
    prob = CP.load_problem(path, CH.PRIOR)
    e = prob["experiments"][0]
    assert len(e["model"].ode) > 16
    return path, prob, (len(e["output_times"]), len(e["model"].ode))


def test_wide_model_matches_oracle(wide, monkeypatch):
    from bcm3_amd.likelihood import Likelihood
    path, prob, (M, NS) = wide
    monkeypatch.delenv("BCM3_CP_QUEUE", raising=False)
    ll = Likelihood(path, CH.PRIOR, device=0)
    x = CH.draws(8, 11)
    lp, status = ll.evaluate_batch(x)
    ref = CP.simulate(prob, x)
    ref_nofma = CP.simulate(CP.load_problem(path, CH.PRIOR, variant="nofma"), x)
    dev, spread = CH.check_logp(lp, status, ref["logp"], ref_nofma["logp"], name="wide model")
    assert dev and np.median(dev) <= 10.0 * np.median(spread) + 1e-12, (np.median(dev), np.median(spread))
    for i in range(len(x)):
        if not ref["detail"][i]["ok"]:
            continue
        rec, vals, endy = ll.cellpop_cells(i, M, NS)
        cells = ref["detail"][i]["cells"]
        assert len(rec) == len(cells), i
        for k, c in enumerate(cells):
            assert bool(rec["flags"][k] & 2) == c["divided"], (i, k)
            assert abs(rec["creation"][k] - c["creation"]) <= 0.1, (i, k)
    ll.close()


def test_wide_model_queue_bit_identical(wide, monkeypatch):
    from bcm3_amd.likelihood import Likelihood
    path, prob, (M, NS) = wide
    monkeypatch.setenv("BCM3_CP_QUEUE", "0")
    gen = Likelihood(path, CH.PRIOR, device=0)
    monkeypatch.setenv("BCM3_CP_QUEUE", "1")
    que = Likelihood(path, CH.PRIOR, device=0)
    x = CH.draws(8, 11)
    lp_g, st_g = gen.evaluate_batch(x)
    lp_q, st_q = que.evaluate_batch(x)
    np.testing.assert_array_equal(st_q, st_g)
    assert lp_q.tobytes() == lp_g.tobytes()
    for i in np.nonzero(np.isfinite(lp_g))[0]:
        a = gen.cellpop_cells(int(i), M, NS)
        b = que.cellpop_cells(int(i), M, NS)
        assert all(u.tobytes() == v.tobytes() for u, v in zip(a, b)), i
    gen.close()
    que.close()
