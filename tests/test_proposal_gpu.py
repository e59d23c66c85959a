"""GPU tests of the adaptive proposal kernels (bcm3_amd/csrc/proposal_kernels.hip) against their
Python restatement (tests/proposal_reference.py), and of the device sampler with them."""
import math
import os

import numpy as np
import pytest

import helpers as H
import proposal_reference as R

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _prior(name="c3_prior.xml"):
    from bcm3_amd.sampler import DevicePrior, load_prior
    return DevicePrior(load_prior(os.path.join(H.GOLDEN, name)), "cuda")


def _prior_arrays(prior):
    return prior.kind_codes, prior.p0, prior.p1, prior.p2


def _state(P):
    return {"kind": P.struct.kind, "t_dof": P.t_dof, "target": P.target, "ncomp": P.ncomp.cpu().numpy(),
            "weights": P.weights.cpu().numpy(), "mean": P.mean.cpu().numpy(), "chol": P.chol.cpu().numpy(),
            "logc": P.logc.cpu().numpy(), "scale": P.scale.cpu().numpy().copy(), "ema": P.ema.cpu().numpy().copy(),
            "selected": P.selected.cpu().numpy().copy(), "lower": P.lower.cpu().numpy(),
            "upper": P.upper.cpu().numpy()}


def _random_mixtures(P, rng, K):
    d = P.d
    for c in range(P.C):
        w = rng.uniform(0.2, 1.0, K)
        w /= w.sum()
        mu = P.prior_mean.cpu().numpy() + rng.normal(0, 0.3, (K, d)) * np.sqrt(P.prior_var.cpu().numpy())
        cov = []
        for _ in range(K):
            A = rng.normal(0, 1, (d, d)) * np.sqrt(P.prior_var.cpu().numpy())[:, None] * 0.2
            cov.append(A @ A.T + np.diag(0.05 * P.prior_var.cpu().numpy()))
        P.set_mixture(c, w, mu, np.array(cov))


def _check_propose(kind, K, t_dof, its=(0, 7, 2**40), prior_xml="c3_prior.xml", C=48):
    from bcm3_amd import _hip
    from bcm3_amd.proposal import DeviceProposal
    from bcm3_amd.pt import temperature_ladder
    prior = _prior(prior_xml) if isinstance(prior_xml, str) else prior_xml
    kd, p0, p1, p2 = _prior_arrays(prior)
    d = prior.d
    temps = torch.tensor(temperature_ladder(C), dtype=torch.float64, device="cuda")
    P = DeviceProposal(kind, prior, temps, kmax=max(K, 1), t_dof=t_dof)
    rng = np.random.default_rng(11 + K)
    if kind == "gaussian_mixture" and K > 1:
        _random_mixtures(P, rng, K)
    # some chains have proposed before (Update runs on them), with EMAs on both sides of target
    P.selected[::2] = 0
    P.ema.copy_(torch.tensor(rng.uniform(0.1, 0.4, P.ema.shape), device="cuda"))
    if prior.simple:
        gen = torch.Generator(device="cuda")
        gen.manual_seed(3)
        values = prior.sample(C, gen)
    else:  # inside every support: the prior moments, jittered
        rng0 = np.random.default_rng(3)
        m = prior.mean.cpu().numpy()
        sd = np.sqrt(prior.var.cpu().numpy())
        lo, hi = prior.lower.cpu().numpy(), prior.upper.cpu().numpy()
        x = np.clip(m + 0.2 * sd * rng0.normal(size=(C, d)), np.where(np.isfinite(lo), lo + 1e-3, -np.inf),
                    np.where(np.isfinite(hi), hi - 1e-3, np.inf))
        values = torch.tensor(x, device="cuda")
    prop = torch.empty_like(values)
    lp = torch.empty(C, dtype=torch.float64, device="cuda")
    lmh = torch.empty(C, dtype=torch.float64, device="cuda")
    for it in its:
        ref = _state(P)
        _hip.ptmh_propose_adaptive(C, d, kd.data_ptr(), p0.data_ptr(), p1.data_ptr(), p2.data_ptr(),
                                   temps.data_ptr(), values.data_ptr(), prop.data_ptr(), lp.data_ptr(), lmh.data_ptr(),
                                   P.struct, 128, 77, it)
        torch.cuda.synchronize()
        rp, rl, rm = R.propose(ref, kd.cpu().numpy(), p0.cpu().numpy(), p1.cpu().numpy(), temps.cpu().numpy(),
                               values.cpu().numpy(), 128, 77, it, p2=p2.cpu().numpy())
        # (heavy-tailed t steps of ~1e3 prior widths fold an ulp of pow/sqrt into ~1e-12 absolute)
        np.testing.assert_allclose(prop.cpu().numpy(), rp, rtol=1e-12, atol=1e-11)
        assert np.array_equal(P.selected.cpu().numpy(), ref["selected"])
        np.testing.assert_allclose(P.scale.cpu().numpy(), ref["scale"], rtol=1e-14)
        got = lp.cpu().numpy()
        assert np.array_equal(np.isinf(got), np.isinf(rl))
        np.testing.assert_allclose(got[np.isfinite(rl)], rl[np.isfinite(rl)], rtol=1e-12)
        np.testing.assert_allclose(lmh.cpu().numpy(), rm, rtol=1e-9, atol=1e-11)
        # proposals reflect on the prior bounds: every marginal stays inside its support
        assert np.all(np.isfinite(got)) or not prior.simple
        values.copy_(prop)
    return P


def test_propose_global_covariance():
    _check_propose("global_covariance", 1, 0.0)


def test_propose_gaussian_mixture_single():
    P = _check_propose("gaussian_mixture", 1, 0.0)
    assert float(P.ema.abs().sum()) > 0


@pytest.mark.parametrize("K", [2, 3])
def test_propose_gaussian_mixture_components(K):
    _check_propose("gaussian_mixture", K, 0.0)


@pytest.mark.parametrize("t_dof", [0.5, 5.0])
def test_propose_t_distributed(t_dof):
    _check_propose("gaussian_mixture", 2, t_dof)


@pytest.mark.parametrize("kind", ["gaussian_mixture", "global_covariance"])
def test_propose_many_variables(kind):
    """d = 138 (the P = 64 PopPK variant): the thread-per-chain kernel beyond 64 variables."""
    _check_propose(kind, 2 if kind == "gaussian_mixture" else 1, 0.0, its=(0, 3), prior_xml="p64_prior.xml", C=6)


def test_accept_adaptive_matches_reference():
    from bcm3_amd import _hip
    from bcm3_amd.proposal import DeviceProposal
    from bcm3_amd.pt import temperature_ladder
    prior = _prior()
    C, d = 200, prior.d
    temps = torch.tensor(temperature_ladder(C), dtype=torch.float64, device="cuda")
    P = DeviceProposal("gaussian_mixture", prior, temps, kmax=2)
    rng = np.random.default_rng(5)
    P.selected.copy_(torch.tensor(rng.integers(0, 2, C), dtype=torch.int32, device="cuda"))
    values = torch.tensor(rng.normal(size=(C, d)), device="cuda")
    prop = torch.tensor(rng.normal(size=(C, d)), device="cuda")
    lprior = torch.tensor(rng.normal(size=C), device="cuda")
    llh = torch.tensor(rng.normal(size=C) * 10, device="cuda")
    lpp = lprior + temps * llh
    lprior_prop = torch.tensor(rng.normal(size=C), device="cuda")
    llh_prop = torch.tensor(rng.normal(size=C) * 10, device="cuda")
    llh_prop[5] = -math.inf
    lprior_prop[7] = -math.inf
    log_mh = torch.tensor(rng.normal(size=C), device="cuda")
    ref = _state(P)
    rv, rq, rl, rp = (values.cpu().numpy(), lprior.cpu().numpy(), llh.cpu().numpy(), lpp.cpu().numpy())
    racc = R.accept(ref, temps.cpu().numpy(), prop.cpu().numpy(), lprior_prop.cpu().numpy(),
                    llh_prop.cpu().numpy(), log_mh.cpu().numpy(), 0.7, rv, rq, rl, rp, 9, 21, 4)
    acc = torch.zeros(C, dtype=torch.uint8, device="cuda")
    n_acc = torch.zeros(1, dtype=torch.int64, device="cuda")
    _hip.ptmh_accept_adaptive(C, d, temps.data_ptr(), prop.data_ptr(), lprior_prop.data_ptr(), llh_prop.data_ptr(),
                              log_mh.data_ptr(), 0.7, values.data_ptr(), lprior.data_ptr(), llh.data_ptr(),
                              lpp.data_ptr(), acc.data_ptr(), n_acc.data_ptr(), P.struct, 9, 21, 4)
    torch.cuda.synchronize()
    assert np.array_equal(acc.cpu().numpy().astype(bool), racc)
    assert int(n_acc.item()) == int(racc.sum())
    np.testing.assert_array_equal(values.cpu().numpy(), rv)
    np.testing.assert_array_equal(lpp.cpu().numpy(), rp)
    np.testing.assert_allclose(P.ema.cpu().numpy(), ref["ema"], rtol=1e-15)


def test_history_ring_matches_reference():
    from bcm3_amd.proposal import SampleHistory
    rng = np.random.default_rng(9)
    C, d, Hs, sub = 6, 3, 4, 2
    temps = torch.tensor([0.0, 0.1, 0.2, 0.5, 0.8, 1.0], dtype=torch.float64, device="cuda")
    hist = SampleHistory(C, d, Hs, sub, "cuda")
    rh = np.zeros((C, Hs, d), dtype=np.float32)
    rc = np.zeros((C, 2), dtype=np.int64)
    for step in range(13):
        vals = torch.tensor(rng.normal(size=(C, d)), device="cuda")
        mask = None if step % 3 else torch.tensor([1, 0, 1, 1, 0, 1], dtype=torch.uint8, device="cuda")
        hist.add(temps, vals, mask)
        R.history_add(temps.cpu().numpy(), vals.cpu().numpy(), None if mask is None else mask.cpu().numpy(), rh, rc,
                      sub)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(hist.samples.cpu().numpy(), rh)
    np.testing.assert_array_equal(hist.counters.cpu().numpy(), rc)
    assert rc[0, 0] == 0  # T == 0 chain keeps no history


@pytest.mark.parametrize("proposal", ["gaussian_mixture", "global_covariance"])
def test_sampler_adaptive_proposals(proposal):
    """Circular ridge (config C2) with the reference's proposals: the run stays finite, the scale
    adaptation steers the acceptance of the posterior chain toward the target, and the proposal
    adapts from the sample history."""
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.pt import temperature_ladder
    from bcm3_amd.sampler import DevicePrior, PTMHDevice, load_prior
    prior = DevicePrior(load_prior(os.path.join(H.GOLDEN, "circular_prior.xml")), "cuda")
    ll = Likelihood(os.path.join(H.GOLDEN, "circular_likelihood.xml"), os.path.join(H.GOLDEN, "circular_prior.xml"),
                    device=0)
    C = 16
    s = PTMHDevice(ll, prior, temperature_ladder(C), seed=5, proposal=proposal, adapt_proposal_samples=100,
                   adapt_proposal_times=1)
    s.run(300)
    torch.cuda.synchronize()
    assert s.adaptations_done == 1
    assert torch.isfinite(s.lpp).all()
    assert torch.isfinite(s.proposal.chol).all()
    ema = s.proposal.ema.cpu().numpy()
    # the posterior chain's acceptance EMA has moved toward the d = 2 target of 0.35
    assert 0.05 < ema[-1, 0] < 0.8
    n = s.history.counters.cpu().numpy()
    assert n[0, 0] == 0 and n[1:, 0].min() > 0


ALL_KINDS_PRIOR = """<?xml version="1.0" encoding="utf-8"?>
<variableset>
  <variable name="u" distribution="uniform" lower="-1.0" upper="2.0"/>
  <variable name="n" distribution="normal" mu="0.5" sigma="2.0"/>
  <variable name="e" distribution="exponential" lambda="1.5"/>
  <variable name="g" distribution="gamma" k="2.5" theta="0.7"/>
  <variable name="g1" distribution="gamma" k="0.6" theta="2.0"/>
  <variable name="b" distribution="beta" a="2.0" b="3.0"/>
  <variable name="h" distribution="half_cauchy" scale="0.8"/>
  <variable name="bp" distribution="beta_prime" a="3.0" b="4.0" scale="1.5"/>
  <variable name="em" distribution="exponential_mix" lambda="1.0" lambda2="5.0" mix="0.3"/>
</variableset>
"""


def test_prior_all_marginal_types(tmp_path):
    """Every UnivariateMarginal type: T = 0 draws and prior log densities of the kernels vs the
    restatement (tests/proposal_reference.py), draws inside each support."""
    from bcm3_amd.sampler import DevicePrior, load_prior
    path = tmp_path / "prior.xml"
    path.write_text(ALL_KINDS_PRIOR)
    prior = DevicePrior(load_prior(str(path)), "cuda")
    assert prior.kind_codes.tolist() == [0, 1, 2, 3, 3, 4, 5, 6, 7]
    P = _check_propose("global_covariance", 1, 0.0, its=(0, 9), prior_xml=prior, C=40)
    # draws of T = 0 chains cover each marginal's support and match its moments roughly
    from bcm3_amd import _hip
    from bcm3_amd.pt import temperature_ladder
    C = 4000
    d = prior.d
    temps = torch.zeros(C, dtype=torch.float64, device="cuda")
    from bcm3_amd.proposal import DeviceProposal
    Q = DeviceProposal("global_covariance", prior, temps)
    vals = torch.zeros((C, d), dtype=torch.float64, device="cuda")
    prop = torch.empty_like(vals)
    lp = torch.empty(C, dtype=torch.float64, device="cuda")
    lmh = torch.empty(C, dtype=torch.float64, device="cuda")
    _hip.ptmh_propose_adaptive(C, d, prior.kind_codes.data_ptr(), prior.p0.data_ptr(), prior.p1.data_ptr(),
                               prior.p2.data_ptr(), temps.data_ptr(), vals.data_ptr(), prop.data_ptr(), lp.data_ptr(),
                               lmh.data_ptr(), Q.struct, 0, 5, 1)
    torch.cuda.synchronize()
    x = prop.cpu().numpy()
    assert np.all(np.isfinite(lp.cpu().numpy()))
    mean = prior.mean.cpu().numpy()
    sd = np.sqrt(prior.var.cpu().numpy())
    for i in range(d):
        if i == 6:  # half-Cauchy: no mean; check the median = scale
            assert abs(np.median(x[:, i]) - 0.8) < 0.08
            continue
        assert abs(x[:, i].mean() - mean[i]) < 5 * sd[i] / math.sqrt(C), (i, x[:, i].mean(), mean[i])


def test_device_mixture_density_pinned_to_reference_golden_values():
    """The propose kernel's mixture arithmetic (wave_responsibilities_lsum, through
    bcm3hip_gmm_eval) against the reference's own golden values: GMM LogPdf / responsibilities
    (tests/stats/GMM.cpp:4-31) and dmvnormal (tests/stats/mvn.cpp:17-44), 1e-12 relative. The
    Cholesky factors and log normalisers come from the host GMM::Set (bcm3_gmm_eval)."""
    import test_gmm as TG
    from bcm3_amd import _hip
    cases = [(TG.GMM_W, TG.GMM_MU, TG.GMM_COV, TG.GMM_X, TG.GMM_LOGPDF, TG.GMM_RESP)]
    cases += [([1.0], [mu], [sig], x, lp, [1.0]) for mu, sig, x, _, lp in TG.MVN_CASES]
    for w, mu, cov, x, want_lp, want_r in cases:
        _, _, L, lc = TG.gmm_eval(w, mu, cov, x)
        K, d = len(w), len(x)
        t = {k: torch.tensor(np.asarray(v, dtype=np.float64).ravel(), device="cuda")
             for k, v in dict(x=x, mean=mu, chol=L, logc=lc, w=w).items()}
        lp = torch.empty(1, dtype=torch.float64, device="cuda")
        r = torch.empty(K, dtype=torch.float64, device="cuda")
        _hip.gmm_eval(1, d, K, t["x"].data_ptr(), t["mean"].data_ptr(), t["chol"].data_ptr(), t["logc"].data_ptr(),
                      t["w"].data_ptr(), lp.data_ptr(), r.data_ptr())
        torch.cuda.synchronize()
        assert abs(lp.item() / want_lp - 1) < 1e-12, (lp.item(), want_lp)
        np.testing.assert_allclose(r.cpu().numpy(), want_r, rtol=1e-12)


def test_circular_ridge_adapts_to_a_mixture():
    """Config C2 (circular ridge, bimodal): after an adaptation from the device history the
    gaussian_mixture proposals of the tempered chains hold more than one component
    (ProposalGaussianMixture::InitializeImpl selecting K > 1 by AIC)."""
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.pt import temperature_ladder
    from bcm3_amd.sampler import DevicePrior, PTMHDevice, load_prior
    pri = os.path.join(H.GOLDEN, "circular_prior.xml")
    ll = Likelihood(os.path.join(H.GOLDEN, "circular_likelihood.xml"), pri, device=0)
    prior = DevicePrior(load_prior(pri), "cuda")
    loop = PTMHDevice(ll, prior, temperature_ladder(32), seed=6, device="cuda", adapt_proposal_samples=400,
                      adapt_proposal_times=1)
    loop.run(401)
    torch.cuda.synchronize()
    assert loop.adaptations_done == 1
    nc = loop.proposal.ncomp.cpu().numpy()
    assert nc.max() > 1, nc
    assert (loop.proposal.selected.cpu().numpy() >= -1).all()
    acc = int(loop.accepted_mutate.item()) / loop.attempted_mutate
    assert 0.05 < acc < 0.9


DIRICHLET_PRIOR = """<?xml version="1.0" encoding="utf-8"?>
<variableset>
  <variable name="x" distribution="uniform" lower="-1.0" upper="2.0"/>
  <variable name="w0" multivariate="true" id="1" distribution="dirichlet" alpha="2.0"/>
  <variable name="w1" multivariate="true" id="1" distribution="dirichlet" alpha="3.0"/>
  <variable name="w2" multivariate="true" id="1" distribution="dirichlet" alpha="4.5"/>
  <variable name="y" distribution="normal" mu="0.5" sigma="2.0"/>
</variableset>
"""


def _dirichlet_prior(tmp_path):
    from bcm3_amd.sampler import DevicePrior, load_prior
    path = tmp_path / "dirichlet_prior.xml"
    path.write_text(DIRICHLET_PRIOR)
    return str(path), DevicePrior(load_prior(str(path)), "cuda")


@pytest.mark.parametrize("K", [1, 2])
def test_dirichlet_prior_propose(tmp_path, K):
    """A 3-component Dirichlet prior (MultivariateMarginal, PriorIndependence.cpp:40-77): T = 0 draws
    (Gamma draws over their sum), the residual fix-up of T > 0 proposals after the MH ratio of the
    unmodified proposal (SamplerPTChain.cpp:270-278) and the group-first prior density
    (PriorIndependence.cpp:129-157) of the kernels against the restatement, over several iterations"""
    _, prior = _dirichlet_prior(tmp_path)
    assert prior.kind_codes.tolist() == [0, 8, 8, 8, 1]
    assert prior.p1.cpu().numpy()[1:4].tolist() == [1.0, 1.0, 1.0]
    _check_propose("gaussian_mixture", K, 0.0, its=(0, 9, 2**40), prior_xml=prior, C=40)


def test_dirichlet_prior_draws(tmp_path):
    from bcm3_amd import _hip
    from bcm3_amd.proposal import DeviceProposal
    _, prior = _dirichlet_prior(tmp_path)
    C, d = 4000, prior.d
    temps = torch.zeros(C, dtype=torch.float64, device="cuda")
    Q = DeviceProposal("global_covariance", prior, temps)
    vals = torch.zeros((C, d), dtype=torch.float64, device="cuda")
    prop = torch.empty_like(vals)
    lp = torch.empty(C, dtype=torch.float64, device="cuda")
    lmh = torch.empty(C, dtype=torch.float64, device="cuda")
    _hip.ptmh_propose_adaptive(C, d, prior.kind_codes.data_ptr(), prior.p0.data_ptr(), prior.p1.data_ptr(),
                               prior.p2.data_ptr(), temps.data_ptr(), vals.data_ptr(), prop.data_ptr(), lp.data_ptr(),
                               lmh.data_ptr(), Q.struct, 0, 5, 1)
    torch.cuda.synchronize()
    x = prop.cpu().numpy()
    w = x[:, 1:4]
    assert np.all((w >= 0) & (w <= 1)) and np.all(np.abs(w.sum(axis=1) - 1.0) <= 1e-15)
    assert np.all(np.isfinite(lp.cpu().numpy()))
    a = np.array([2.0, 3.0, 4.5])
    mean, var = a / a.sum(), a * (a.sum() - a) / (a.sum() ** 2 * (a.sum() + 1))
    assert np.all(np.abs(w.mean(axis=0) - mean) < 5 * np.sqrt(var / C))
    np.testing.assert_allclose(prior.mean.cpu().numpy()[1:4], mean, rtol=1e-15)
    np.testing.assert_allclose(prior.var.cpu().numpy()[1:4], var, rtol=1e-15)


def test_sampler_runs_with_dirichlet_prior(tmp_path):
    """The C++ sampler (bcm3_ptmh_*) on a banana likelihood over a prior with a Dirichlet group: every
    chain's group stays on the simplex (sum 1 within the reference's 1e-15), and each chain's log prior
    equals the restated PriorIndependence density of its values"""
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.ptmh import PTMHNative
    prior_xml, prior = _dirichlet_prior(tmp_path)
    lik = tmp_path / "banana5.xml"
    lik.write_text('<bcm_likelihood type="banana" dimension="5" sd1="2.0" sd2="1.0"></bcm_likelihood>\n')
    ll = Likelihood(str(lik), prior_xml, device=0)
    s = PTMHNative(ll, prior_xml, 16, seed=4, adapt_proposal_samples=30, adapt_proposal_times=1)
    s.iterate(80)
    s.synchronize()
    st = s.state()
    c = s.counters()
    s.close()
    assert c["accepted_mutate"] > 16 and c["adaptations_done"] == 1
    w = st["values"][:, 1:4]
    assert np.all((w >= 0) & (w <= 1)) and np.all(np.abs(w.sum(axis=1) - 1.0) <= 1e-15)
    kd, p0, p1, p2 = (t.cpu().numpy() for t in _prior_arrays(prior))
    for i in range(len(w)):
        ref = R.prior_total(kd, p0, p1, p2, [float(v) for v in st["values"][i]])
        assert abs(st["lprior"][i] - ref) <= 1e-12 * (1 + abs(ref)), (i, st["lprior"][i], ref)
    ll.close()
