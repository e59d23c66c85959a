"""CPU tests: pin the oracle before trusting it (runs without a GPU).

* the C restatement of CVODE BDF (oracle/liboracle.so) equals the vendored CVODE 5.3.0 compiled
  from the reference sources without FMA contraction (oracle/_ref/libbcm3ref_nofma.so) bit for
  bit, for every PK model variant and dosing rule;
* it matches the committed golden outputs of the reference-flags build within the envelope;
* QuantileNormal (Boost erfc_inv restated) agrees with scipy.special.ndtri to a few ulp.
"""
import math
import os

import numpy as np
import pytest

import helpers as H
import oracle as O
import parity

HAVE_REF = os.path.exists(O.LIB_REF) and os.path.exists(O.LIB_REF_NOFMA)
needs_ref = pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built (needs /root/reference)")


@pytest.fixture(scope="module")
def restated():
    return O.Oracle("restated")


def _eval_pair(prob, vals, a, b):
    ra = a.popk_eval(prob, vals, nthreads=4)
    rb = b.popk_eval(prob, vals, nthreads=4)
    return ra, rb


@needs_ref
def test_restated_bit_exact_vs_reference_cvode_c3(restated):
    prob = H.c3_problem(1)
    vals = H.S.prior_draws(1, 1024, 1234)
    a, b = _eval_pair(prob, vals, restated, O.Oracle("ref_nofma"))
    assert np.array_equal(a["traj"], b["traj"], equal_nan=True)
    assert np.array_equal(a["logp"], b["logp"])
    assert np.array_equal(a["stats"], b["stats"])
    assert np.array_equal(a["ok"], b["ok"])


@needs_ref
@pytest.mark.parametrize("pk_type", ["one", "two", "one_biphasic_uptake", "two_biphasic_uptake", "one_transit",
                                     "two_transit"])
@pytest.mark.parametrize("rule", ["daily", "intermittent1", "intermittent2", "intermittent3", "skipped",
                                  "dose_change", "interval12"])
def test_restated_bit_exact_all_models(restated, pk_type, rule):
    kw = dict(P=2, T_days=6)
    if rule.startswith("intermittent"):
        kw["intermittent"] = int(rule[-1])
        kw["T_days"] = 10
    elif rule == "skipped":
        kw["skipped"] = (2, 3)
    elif rule == "dose_change":
        kw["dose_change"] = (500.0, 72.0)
    elif rule == "interval12":
        kw["interval"] = 12.0
    prob, lo, hi = H.make_problem(pk_type, **kw)
    vals = H.draws(lo, hi, 96, 77)
    a, b = _eval_pair(prob, vals, restated, O.Oracle("ref_nofma"))
    assert np.array_equal(a["traj"], b["traj"], equal_nan=True)
    assert np.array_equal(a["logp"], b["logp"])
    assert np.array_equal(a["stats"], b["stats"])


def test_restated_vs_golden_fixture(restated, golden_dir):
    g = np.load(os.path.join(golden_dir, "c3_golden.npz"))
    prob = H.c3_problem(1)
    a = restated.popk_eval(prob, g["values"], nthreads=4)
    e = parity.y1_rel_err(a["traj"][:, 0, 1], g["traj"][:, 0, 1], prob.atol)
    le = parity.llh_err(a["logp"], g["logp"])
    parity.assert_parity(e, le, a["stats"][:, 0, 0], g["stats"][:, 0, 0], a["ok"][:, 0], g["ok"][:, 0])


def test_golden_fixture_self_consistent(golden_dir):
    g = np.load(os.path.join(golden_dir, "c3_golden.npz"))
    assert g["values"].shape == (512, 12)
    assert np.all(np.isfinite(g["logp"][g["ok"][:, 0] == 1]))
    assert np.all(g["logp"][g["ok"][:, 0] == 0] == -np.inf)
    # steps: ~78 per simulated day on the C3 prior
    assert 500 < np.median(g["stats"][:, 0, 0]) < 1500


def test_quantile_normal_vs_scipy(restated):
    sp = pytest.importorskip("scipy.special")
    rng = np.random.default_rng(3)
    ps = np.concatenate([rng.random(2000), 10.0 ** -rng.uniform(1, 15, 500), 1 - 10.0 ** -rng.uniform(1, 15, 500)])
    ours = np.array([restated.lib.orc_quantile_normal(p, 0.0, 1.0) for p in ps])
    ref = sp.ndtri(ps)
    ulp = np.abs(ours - ref) / np.spacing(np.abs(ref))
    assert np.max(ulp) <= 8, np.max(ulp)
    # location-scale form of Boost quantile(normal(mu, sigma), p)
    q = restated.lib.orc_quantile_normal(0.3, -0.5, 0.2)
    assert abs(q - (-0.5 + 0.2 * sp.ndtri(0.3))) < 1e-15


def test_log_pdf_tnu4(restated):
    # Student-t nu=4 log density (ProbabilityDistributions.cpp:216-224) vs the closed form
    for x, mu, s in [(1.0, 0.5, 2.0), (-3.0, 10.0, 0.7), (100.0, 101.0, 5.0)]:
        z = (x - mu) / s
        want = (math.lgamma(2.5) - math.lgamma(2.0) - 0.5 * math.log(4 * math.pi) - 2.5 * math.log1p(z * z / 4)
                - math.log(s))
        assert abs(restated.lib.orc_log_pdf_tnu4(x, mu, s) - want) < 1e-12


def test_transforms(restated):
    t = restated.lib.orc_transform
    assert t(O.TF_NONE, 0.3) == 0.3
    assert abs(t(O.TF_LOG10, 2.0) - 100.0) < 1e-12
    assert abs(t(O.TF_LOG, 1.0) - math.e) < 1e-15
    assert abs(t(O.TF_LOGIT, 0.0) - 0.5) < 1e-16
    assert abs(t(O.TF_LOGIT, 3.0) - 1 / (1 + math.exp(-3.0))) < 1e-16


def test_analytic_oracle_vs_golden(restated, golden_dir):
    g = np.load(os.path.join(golden_dir, "analytic_golden.npz"))
    b = restated.banana(g["banana_values"], 2, 2.0, 1.0)
    c = restated.circular(g["circular_values"], 2, 2.0, 3.5, 0.1)
    assert np.allclose(b, g["banana_logp"], rtol=1e-13, atol=1e-13)
    assert np.allclose(c, g["circular_logp"], rtol=1e-14, atol=1e-14)


def test_simulate_until_rules():
    # LikelihoodPopPKTrajectory.cpp:163-184: skipped day 1 -> simulate only up to t < 24h;
    # first observation later than 15 days -> simulate nothing
    prob, _, _ = H.make_problem("two", P=2, T_days=20, skipped=(1,))
    assert all(prob.time[prob.simulate_until[j] - 1] < 24.0 <= prob.time[prob.simulate_until[j]] for j in range(2))
    pk = H.S.pkdata_skeleton(1)
    pk[H.S.TRIAL]["time"] = [0.0, 100.0, 400.0]
    pk[H.S.TRIAL][H.S.DRUG + "_plasma_concentration"] = [[None, None, 5.0]]
    prob2 = O.build_problem(pk, H.S.TRIAL, H.S.DRUG, "two", H.variables(1))
    assert prob2.simulate_until[0] == 0
