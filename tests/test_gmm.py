"""Proposal adaptation on the host (libbcm3.so: bcm3_gmm_eval, bcm3_adapt_proposals; C++ in
bcm3_amd/csrc/host/GMM.cpp) against the reference's own golden values (tests/stats/GMM.cpp:4-31,
tests/stats/mvn.cpp:17-44) and against the numpy restatement oracle/gmm_oracle.py of
ProposalGaussianMixture::InitializeImpl / GMM::Fit / ProposalGlobalCovariance::InitializeImpl."""
import ctypes as C
import math
import os

import numpy as np
import pytest

import gmm_oracle as G
import helpers as H

torch = pytest.importorskip("torch")


def _lib():
    from bcm3_amd.likelihood import lib
    return lib()


def gmm_eval(weights, means, covs, x):
    w = np.ascontiguousarray(weights, dtype=np.float64)
    K = len(w)
    mu = np.ascontiguousarray(means, dtype=np.float64).reshape(K, -1)
    d = mu.shape[1]
    cv = np.ascontiguousarray(covs, dtype=np.float64).reshape(K, d, d)
    x = np.ascontiguousarray(x, dtype=np.float64).reshape(-1, d)
    lp = np.empty(len(x))
    r = np.empty((len(x), K))
    L = np.empty((K, d, d))
    lc = np.empty(K)
    rc = _lib().bcm3_gmm_eval(K, d, w.ctypes.data, mu.ctypes.data, cv.ctypes.data, len(x), x.ctypes.data,
                              lp.ctypes.data, r.ctypes.data, L.ctypes.data, lc.ctypes.data)
    assert rc == 0
    return lp, r, L, lc


# tests/stats/GMM.cpp:4-31 (BOOST_CHECK_CLOSE tolerance 1e-12 percent)
GMM_W = [0.25, 0.75]
GMM_MU = [[-1.0, -1.0], [2.0, 3.0]]
GMM_COV = [[[2.0, 1.0], [1.0, 1.0]], [[1.0, -0.9], [-0.9, 1.0]]]
GMM_X = [2.0, 2.0]
GMM_LOGPDF = -3.9045912795091535
GMM_RESP = [0.0219370092578219, 0.9780629907421782]
# tests/stats/mvn.cpp:17-44: (mu, sigma, x, pdf, logpdf)
MVN_CASES = [
    ([0.0, 0.0], [[1.0, 0.0], [0.0, 1.0]], [0.0, 0.0], 0.1591549430918953, -1.837877066409345),
    ([0.0, 0.0], [[1.0, 0.0], [0.0, 1.0]], [1.0, 1.0], 0.05854983152431917, -2.837877066409345),
    ([0.0, 0.0], [[1.0, 0.0], [0.0, 1.0]], [-1.0, -1.0], 0.05854983152431917, -2.837877066409345),
    ([1.2e3, 1.2e3], [[234.0, 42.0], [42.0, 786.0]], [1.2e3, 1.2e3], 0.0003729010642586194, -7.894197416778156),
    ([1.2e3, 1.2e3], [[234.0, 42.0], [42.0, 786.0]], [1000.0, 1050.0], 6.617956105689106e-45, -101.726542607819),
]


def test_gmm_golden_values():
    lp, r, _, _ = gmm_eval(GMM_W, GMM_MU, GMM_COV, GMM_X)
    assert abs(lp[0] / GMM_LOGPDF - 1) < 1e-14
    np.testing.assert_allclose(r[0], GMM_RESP, rtol=1e-14)
    g = G.GMM()
    assert g.set(GMM_MU, GMM_COV, GMM_W)
    assert abs(g.log_pdf(np.array(GMM_X)) / GMM_LOGPDF - 1) < 1e-14
    np.testing.assert_allclose(g.responsibilities(np.array(GMM_X)), GMM_RESP, rtol=1e-14)


@pytest.mark.parametrize("case", range(len(MVN_CASES)))
def test_dmvnormal_golden_values(case):
    mu, sigma, x, pdf, logpdf = MVN_CASES[case]
    lp, r, L, lc = gmm_eval([1.0], [mu], [sigma], x)
    assert abs(lp[0] / logpdf - 1) < 1e-13
    assert abs(math.exp(lp[0]) / pdf - 1) < 1e-12
    assert r[0, 0] == 1.0
    np.testing.assert_allclose(L[0] @ L[0].T, sigma, rtol=1e-15)


def test_gmm_eval_rejects_indefinite():
    w = np.ones(1)
    mu = np.zeros(2)
    cov = -np.eye(2)
    assert _lib().bcm3_gmm_eval(1, 2, w.ctypes.data, mu.ctypes.data, cov.ctypes.data, 0, None, None, None, None,
                                None) == -2


def adapt(kind, hist, counts, active, pm, pv, seed=5, adaptation=0, chain0=0, max_hist=2000, adjusted=False,
          kmax=13, nthreads=4):
    C_, Hh, d = hist.shape
    hist = np.ascontiguousarray(hist, dtype=np.float32)
    counts = np.ascontiguousarray(counts, dtype=np.int64)
    active = np.ascontiguousarray(active, dtype=np.uint8)
    pm = np.ascontiguousarray(pm, dtype=np.float64)
    pv = np.ascontiguousarray(pv, dtype=np.float64)
    nc = np.zeros(C_, dtype=np.int32)
    fit = np.zeros(C_, dtype=np.int32)
    w = np.zeros((C_, kmax))
    mu = np.zeros((C_, kmax, d))
    L = np.zeros((C_, kmax, d, d))
    lc = np.zeros((C_, kmax))
    rc = _lib().bcm3_adapt_proposals(kind, int(adjusted), C_, Hh, d, kmax, hist.ctypes.data, counts.ctypes.data,
                                     active.ctypes.data, max_hist, pm.ctypes.data, pv.ctypes.data, seed, adaptation,
                                     chain0, nthreads, nc.ctypes.data, w.ctypes.data, mu.ctypes.data, L.ctypes.data,
                                     lc.ctypes.data, fit.ctypes.data)
    assert rc == 0
    return nc, w, mu, L, lc, fit


def _histories(rng, Hh, d):
    """chain 1: two well separated clusters (AR(1) within each, like an MCMC trace), chain 2: one
    correlated Gaussian, chain 3: a single sample (prior fallback)."""
    hist = np.zeros((4, Hh, d))
    centers = np.array([[-3.0] + [0.0] * (d - 1), [3.0] + [0.0] * (d - 1)])
    z = rng.normal(size=(Hh, d))
    lab = np.cumsum(rng.random(Hh) < 0.05) % 2  # a persistent two-state switching trace
    x = np.zeros((Hh, d))
    for t in range(Hh):
        x[t] = 0.3 * (x[t - 1] if t else 0.0) + 0.5 * z[t]
    hist[1] = x + centers[lab]
    A = rng.normal(size=(d, d)) * 0.3 + np.eye(d)
    hist[2] = rng.normal(size=(Hh, d)) @ A.T + 1.0
    hist[3, 0] = 0.5
    return hist


@pytest.mark.parametrize("d,adjusted", [(2, False), (3, True), (12, False)])
def test_gaussian_mixture_adaptation_matches_restatement(d, adjusted):
    rng = np.random.default_rng(d)
    Hh = 400
    hist = _histories(rng, Hh, d).astype(np.float32)
    counts = np.array([0, Hh, Hh + 60, 1])
    active = np.array([0, 1, 1, 1])
    pm, pv = np.full(d, 0.25), np.full(d, 4.0)
    nc, w, mu, L, lc, fit = adapt(1, hist, counts, active, pm, pv, seed=77, adaptation=1, chain0=8,
                                  adjusted=adjusted)
    assert nc[0] == 0 and not fit[0]  # T == 0: untouched
    for c in (1, 2, 3):
        h = hist[c, :min(counts[c], Hh)].astype(np.float64)
        r = G.CtrRng(77, G.chain_key(8 + c, 1))
        h = G.thin_history(h, 2000, r)
        g, have = G.fit_gaussian_mixture(h, r, pm, pv, adjusted=adjusted)
        K = len(g.means)
        assert nc[c] == K and bool(fit[c]) == have, (c, nc[c], K)
        np.testing.assert_allclose(w[c, :K], g.weights, rtol=1e-8, atol=1e-12)
        for k in range(K):
            np.testing.assert_allclose(mu[c, k], g.means[k], rtol=1e-8, atol=1e-10)
            np.testing.assert_allclose(L[c, k], g.L[k], rtol=1e-7, atol=1e-10)
            assert abs(lc[c, k] - g.logC[k]) <= 1e-8 * (1 + abs(g.logC[k]))
        assert np.all(w[c, K:] == 0.0)
        for k in range(K, 13):
            assert np.array_equal(L[c, k], np.eye(d))
    if d <= 3:
        assert nc[1] >= 2  # the two clusters are found (at d = 12 the ESS guard allows one component)
    assert not fit[3] and np.allclose(L[3, 0], np.diag(np.sqrt(pv)))


def test_history_thinning_and_global_covariance():
    rng = np.random.default_rng(3)
    d, Hh = 4, 300
    hist = rng.normal(size=(3, Hh, d)).astype(np.float32)
    hist[2, :, 1] = 2.0  # a constant column: the 1e-6 prior-variance floor
    counts = np.array([Hh, 1000, Hh])
    active = np.ones(3)
    pm, pv = np.zeros(d), np.full(d, 9.0)
    nc, w, mu, L, lc, fit = adapt(0, hist, counts, active, pm, pv, seed=1, max_hist=120, kmax=1)
    for c in range(3):
        h = hist[c, :min(counts[c], Hh)].astype(np.float64)
        r = G.CtrRng(1, G.chain_key(c, 0))
        h = G.thin_history(h, 120, r)
        assert len(h) == 120
        g, have = G.fit_global_covariance(h, pv)
        np.testing.assert_allclose(L[c, 0] @ L[c, 0].T, g.covs[0], rtol=1e-10, atol=1e-14)
        assert nc[c] == 1 and fit[c]
    assert abs((L[2, 0] @ L[2, 0].T)[1, 1] - 9e-6) < 1e-18


def test_device_proposal_adapt_glue():
    """DeviceProposal.adapt: T == 0 chains keep their state; adapted chains get the fitted mixture
    and a fresh proposal's scales, EMAs and selected component (a new Proposal object per
    adaptation, SamplerPTChain.cpp:428-462)."""
    from bcm3_amd.proposal import DeviceProposal
    from bcm3_amd.sampler import DevicePrior, load_prior
    prior = DevicePrior(load_prior(os.path.join(H.GOLDEN, "circular_prior.xml")), "cpu")
    temps = torch.tensor([0.0, 0.5, 1.0], dtype=torch.float64)
    P = DeviceProposal("gaussian_mixture", prior, temps, kmax=13)
    P.scale.fill_(0.3)
    P.selected.fill_(0)
    rng = np.random.default_rng(4)
    hist = torch.tensor(_histories(rng, 400, 2)[:3], dtype=torch.float32)
    counters = torch.tensor([[400, 0], [400, 0], [400, 0]], dtype=torch.int64)
    chol0 = P.chol.clone()
    P.adapt(hist, counters, seed=9, adaptation=0, chain0=0)
    assert torch.equal(P.chol[0], chol0[0]) and float(P.scale[0, 0]) == 0.3 and int(P.selected[0]) == 0
    assert int(P.ncomp[1]) >= 2
    assert torch.allclose(P.scale[1:], torch.full_like(P.scale[1:], 2.38 / math.sqrt(2)))
    assert (P.selected[1:] == -1).all()
    assert abs(float(P.weights[1, :int(P.ncomp[1])].sum()) - 1.0) < 1e-12
