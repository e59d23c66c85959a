"""GPU parity of the mixture test likelihoods (multimodal_gaussians, truncated_t) and dummy.

The checker is oracle/_ref/libmixref.so: dmvnormal / dmvt / LogPdfT / logsum restated over the
reference's vendored Eigen LLT and triangular solve (oracle/mixture_ref.cpp), itself pinned to the
reference's golden values (tests/test_mixture.py). Tolerance: 1e-12 relative to (1 + |logp|) --
the device factorises with Eigen's unblocked LLT order and solves in index order, while the
checker's Eigen may group the small dot products differently (SSE/AVX packets), and exp / log /
log1p come from two libraries. The posterior runs check the device PT-MH loop on the reference's
example problems against grid integration."""
import ctypes as C
import math
import os

import numpy as np
import pytest

import helpers as H
from test_mixture import mixref

pytestmark = pytest.mark.gpu

TOL = 1e-12


def _ref_eval(kind, weights, means, covs, nus, x):
    L = mixref()
    means = np.ascontiguousarray(means, np.float64)
    K, d = means.shape
    w = np.ascontiguousarray(weights, np.float64)
    cv = np.ascontiguousarray(covs, np.float64)
    nu = np.ascontiguousarray(nus if nus is not None else np.zeros(K), np.float64)
    x = np.ascontiguousarray(x, np.float64)
    out = np.empty(len(x))
    L.mixref_eval(kind, d, K, w.ctypes.data, means.ctypes.data, cv.ctypes.data, nu.ctypes.data, len(x),
                  x.ctypes.data, out.ctypes.data)
    return out


def _check(lp, ref):
    assert np.array_equal(np.isfinite(lp), np.isfinite(ref))
    f = np.isfinite(ref)
    err = np.abs(lp[f] - ref[f]) / (1 + np.abs(ref[f]))
    assert err.max() <= TOL, err.max()


MG_MEANS = np.array([[-5.0, -5.0], [5.0, 5.0]])
MG_COVS = np.array([[[1, -0.9], [-0.9, 1]], [[2, -0.5], [-0.5, 1]]], np.float64)
TT_MEANS = np.array([[0.5, 2.0, 0.0], [4.0, 1.0, 2.0]])
TT_COVS = np.array([[[0.4, -0.3, 0.0], [-0.3, 0.4, 0.0], [0.0, 0.0, 0.2]],
                    [[0.5, 0.2, 0.3], [0.2, 0.3, 0.4], [0.3, 0.4, 0.8]]])
TT_NUS = np.array([3.0, 4.0])
TT_W = np.array([0.3, 0.7])


def _spd(rng, K, d):
    A = rng.normal(size=(K, d, d))
    return A @ A.transpose(0, 2, 1) + d * 0.2 * np.eye(d)


def test_context_multimodal_gaussians():
    from bcm3_amd import _hip
    x = np.random.default_rng(1).uniform(-10, 10, (8192, 2))
    ctx = _hip.Context.mixture(_hip.MIXTURE_NORMAL, np.log([0.5, 0.5]), MG_MEANS, MG_COVS)
    lp, st = ctx.eval(x)
    ctx.close()
    assert np.all(st == 0)
    _check(lp, _ref_eval(1, [0.5, 0.5], MG_MEANS, MG_COVS, None, x))


def test_context_truncated_t_example():
    from bcm3_amd import _hip
    x = np.random.default_rng(2).uniform(-2, 5, (8192, 3))
    ctx = _hip.Context.mixture(_hip.MIXTURE_T, np.log(TT_W / TT_W.sum()), TT_MEANS, TT_COVS, TT_NUS)
    lp, _ = ctx.eval(x)
    ctx.close()
    _check(lp, _ref_eval(2, TT_W, TT_MEANS, TT_COVS, TT_NUS, x))


@pytest.mark.parametrize("K,d", [(1, 1), (3, 1), (3, 5), (5, 16)])
def test_context_t_random_components(K, d):
    from bcm3_amd import _hip
    rng = np.random.default_rng(100 * K + d)
    means = rng.normal(size=(K, d))
    covs = _spd(rng, K, d) if d > 1 else rng.uniform(0.2, 3.0, (K, 1, 1))
    # the upper triangle is never read (Eigen::LLT<Lower>): scramble it
    for k in range(K):
        covs[k][np.triu_indices(d, 1)] += 7.0
    nus = rng.uniform(0.5, 30.0, K)
    if d == 1:
        nus[0] = 2e10  # LogPdfT's normal branch
    w = rng.uniform(0.1, 1.0, K)
    x = rng.normal(scale=3.0, size=(4096, d))
    ctx = _hip.Context.mixture(_hip.MIXTURE_T, np.log(w / w.sum()), means, covs, nus)
    lp, _ = ctx.eval(x)
    ctx.close()
    _check(lp, _ref_eval(2, w, means, covs, nus, x))


@pytest.mark.parametrize("d", [1, 4, 16])
def test_context_normal_random_components(d):
    from bcm3_amd import _hip
    rng = np.random.default_rng(7 + d)
    K = 2
    means = rng.normal(size=(K, d))
    covs = _spd(rng, K, d)
    x = rng.normal(scale=4.0, size=(4096, d))
    ctx = _hip.Context.mixture(_hip.MIXTURE_NORMAL, np.log([0.5, 0.5]), means, covs)
    lp, _ = ctx.eval(x)
    ctx.close()
    # the checker's kind 1 is MultimodalGaussians' two equally weighted components
    _check(lp, _ref_eval(1, [0.5, 0.5], means, covs, None, x))


def test_not_positive_definite_is_refused():
    from bcm3_amd import _hip
    with pytest.raises(Exception):
        _hip.Context.mixture(_hip.MIXTURE_NORMAL, np.log([1.0]), np.zeros((1, 2)), np.array([[[1.0, 2.0], [2.0, 1.0]]]))


def _lik(name, tmp_path=None, text=None, prior=None):
    from bcm3_amd.likelihood import Likelihood
    if text is not None:
        p = tmp_path / "likelihood.xml"
        p.write_text(text)
        lik = str(p)
    else:
        lik = os.path.join(H.GOLDEN, f"{name}_likelihood.xml")
    return Likelihood(lik, prior or os.path.join(H.GOLDEN, f"{name}_prior.xml"), device=0)


def test_example_likelihoods_through_libbcm3():
    rng = np.random.default_rng(3)
    for name, lo, hi, d, ref in (
            ("multimodal_gaussians", -10, 10, 2, lambda x: _ref_eval(1, [0.5, 0.5], MG_MEANS, MG_COVS, None, x)),
            ("truncated_t", -2, 5, 3, lambda x: _ref_eval(2, TT_W, TT_MEANS, TT_COVS, TT_NUS, x))):
        ll = _lik(name)
        x = rng.uniform(lo, hi, (3000, d))
        lp = ll.evaluate_batch(x)
        lp = lp[0] if isinstance(lp, tuple) else lp
        _check(np.asarray(lp), ref(x))
        # the single-vector route (bcm3::Likelihood::EvaluateLogProbability) gives the same bits
        assert ll.evaluate(x[7]) == np.asarray(lp)[7]
        ll.close()


def test_dummy_through_libbcm3(tmp_path):
    ll = _lik("dummy", tmp_path, '<bcm_likelihood type="dummy"/>', prior=os.path.join(H.GOLDEN, "banana_prior.xml"))
    x = np.random.default_rng(4).uniform(-6, 20, (2048, 2))
    lp = ll.evaluate_batch(x)
    lp = np.asarray(lp[0] if isinstance(lp, tuple) else lp)
    ll.close()
    # LogPdfTnu4(values[0], 0, 1) (ProbabilityDistributions.cpp:216-224)
    want = -0.9808292530117262 - 2.5 * np.log1p(0.25 * x[:, 0] * x[:, 0]) - np.log(1.0)
    assert np.max(np.abs(lp - want) / (1 + np.abs(want))) <= 1e-14


def _run(name, chains, samples, seed, tmp_path, **kw):
    from bcm3_amd.ptmh import PTMHNative
    from scipy.io import netcdf_file
    ll = _lik(name)
    pri = os.path.join(H.GOLDEN, f"{name}_prior.xml")
    s = PTMHNative(ll, pri, chains, seed=seed, **kw)
    out = str(tmp_path / f"{name}.nc")
    s.set_output(out, samples, flush_every=256)
    s.run(samples)
    c = s.counters()
    s.close()
    with netcdf_file(out, "r", mmap=False) as f:
        x = np.array(f.variables["samples.variable_values"][:])
    return x[:, -1, :], c


def test_multimodal_gaussians_example_posterior(tmp_path):
    # examples/multimodal_gaussians/config_gmm.txt's sampler settings, 8 chains instead of 2
    x, c = _run("multimodal_gaussians", 8, 8000, 11, tmp_path, adapt_proposal_samples=2000, adapt_proposal_times=1,
                exploration_steps=1, use_every_nth=1)
    post = x[2000:]
    # two equal-weight modes around (-5,-5) and (5,5), both inside U(-10,10)^2
    hi = post[:, 0] > 0
    assert 0.3 < hi.mean() < 0.7, hi.mean()
    for sel, mu, cov in ((~hi, MG_MEANS[0], MG_COVS[0]), (hi, MG_MEANS[1], MG_COVS[1])):
        m = post[sel].mean(0)
        assert np.all(np.abs(m - mu) < 0.2), m
        assert np.all(np.abs(np.cov(post[sel].T) - cov) < 0.35), np.cov(post[sel].T)


def test_truncated_t_example_posterior(tmp_path):
    # examples/truncated_t/config_gmm_t.txt: t proposals (proposal_t_dof = 5), 2 exploration steps
    x, c = _run("truncated_t", 4, 8000, 12, tmp_path, adapt_proposal_samples=2000, adapt_proposal_times=2,
                exploration_steps=2, t_dof=5.0)
    post = x[2000:]
    assert np.all((post >= -2) & (post <= 5))
    # exact moments of the truncated mixture on U(-2, 5)^3 by grid integration of the checker's density
    g = np.linspace(-2, 5, 71)
    G = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
    lp = _ref_eval(2, TT_W, TT_MEANS, TT_COVS, TT_NUS, G)
    w = np.exp(lp - lp.max())
    w /= w.sum()
    m = (w[:, None] * G).sum(0)
    s = np.sqrt((w[:, None] * (G - m) ** 2).sum(0))
    assert np.all(np.abs(post.mean(0) - m) < 0.25), (post.mean(0), m)
    assert np.all(np.abs(post.std(0) - s) < 0.25), (post.std(0), s)
