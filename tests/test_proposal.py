"""CPU tests of the proposal host logic (bcm3_amd/proposal.py, bcm3_amd/sampler.py): the initial
proposal state, the adaptation from the sample history, the history geometry and the exchange
participants whose histories grow in a round."""
import math
import os

import numpy as np
import pytest

import helpers as H

torch = pytest.importorskip("torch")


def _prior(name="c3_prior.xml"):
    from bcm3_amd.sampler import DevicePrior, load_prior
    return DevicePrior(load_prior(os.path.join(H.GOLDEN, name)), "cpu")


def _reference_pairs(Ctot, start):
    """SamplerPT::DoExchangeMove's pair loop (SamplerPT.cpp:279-298)."""
    pairs = []
    ci = start
    while ci < Ctot:
        ix2 = ci + 1
        if ix2 == Ctot:
            ix2 = 0
        pairs.append((ci, ix2))
        ci += 2
    return pairs


@pytest.mark.parametrize("Ctot,world", [(8, 1), (7, 1), (5, 1), (2, 1), (16, 2), (16, 4), (8, 4)])
def test_exchange_participants_match_pair_loop(Ctot, world):
    from bcm3_amd.sampler import exchange_participants
    C = Ctot // world
    for start in (0, 1):
        want = np.zeros(Ctot, dtype=int)
        for a, b in _reference_pairs(Ctot, start):
            want[a] += 1
            want[b] += 1
        got = np.zeros(Ctot, dtype=int)
        for r in range(world):
            for m in exchange_participants(C, r * C, Ctot, world, start):
                got[r * C:(r + 1) * C] += 1 if m is None else np.array(m, dtype=int)
        assert np.array_equal(got, want), (start, got, want)


def test_history_geometry():
    from bcm3_amd.proposal import history_geometry
    # SamplerPT::Initialize with the defaults: 2000 * 1 * (1 + 1) = 4000 > 2000 -> every 2nd, 2000
    assert history_geometry(2000, 1, 1, 6, 2000) == (2000, 2)
    assert history_geometry(2000, 1, 1, 1, 2000) == (2000, 1)
    assert history_geometry(300, 2, 2, 8, 2000) == (1800, 1)
    assert history_geometry(1500, 1, 2, 8, 2000) == (1500, 3)


def test_initial_state_from_prior():
    from bcm3_amd.proposal import DeviceProposal
    prior = _prior()
    d = prior.d
    temps = torch.linspace(0, 1, 6, dtype=torch.float64)
    for kind in ("gaussian_mixture", "global_covariance"):
        P = DeviceProposal(kind, prior, temps, kmax=3 if kind == "gaussian_mixture" else 1)
        var = ((prior.b - prior.a) ** 2 / 12.0).numpy()
        L0 = P.chol[:, 0].numpy()
        for c in range(6):
            assert np.allclose(np.diag(L0[c]), np.sqrt(var), rtol=1e-15)
            assert np.count_nonzero(L0[c] - np.diag(np.diag(L0[c]))) == 0
        want_logc = -np.log(np.sqrt(var)).sum() - 0.5 * d * math.log(2 * math.pi)
        assert np.allclose(P.logc[:, 0].numpy(), want_logc, rtol=1e-14)
        assert P.target == 0.234
        if kind == "gaussian_mixture":
            assert np.allclose(P.scale.numpy(), 2.38 / math.sqrt(d))
            assert np.allclose(P.ema.numpy(), 0.234)
            assert np.allclose(P.mean[:, 0].numpy(), (0.5 * (prior.a + prior.b)).numpy())
        else:
            assert np.allclose(P.scale.numpy(), 1.0) and np.allclose(P.ema.numpy(), 0.23)
        assert (P.selected.numpy() == -1).all()
        assert (P.ncomp.numpy() == 1).all()
    assert np.isinf(P.lower.numpy()).sum() == 0  # every C3 marginal is uniform


def test_adapt_from_history():
    """DeviceProposal.adapt runs the reference's InitializeImpl on the host (bcm3_adapt_proposals,
    checked in detail by tests/test_gmm.py): stored samples of the ring only, T == 0 untouched,
    fallback to the prior's moments below two samples, fresh scales / EMAs per adaptation."""
    import gmm_oracle as G
    from bcm3_amd.proposal import DeviceProposal
    prior = _prior()
    d, C, Hs = prior.d, 4, 50
    temps = torch.tensor([0.0, 0.3, 0.7, 1.0], dtype=torch.float64)
    P = DeviceProposal("gaussian_mixture", prior, temps, kmax=13)
    P.scale.fill_(0.5)
    rng = np.random.default_rng(1)
    hist = torch.tensor(rng.normal(size=(C, Hs, d)) * 0.1 + 1.0, dtype=torch.float32)
    counters = torch.tensor([[0, 0], [Hs + 17, 0], [30, 1], [1, 0]], dtype=torch.int64)
    chol0 = P.chol.clone()
    P.adapt(hist, counters, seed=3, adaptation=0, chain0=0)
    # T == 0 chain untouched
    assert torch.equal(P.chol[0], chol0[0]) and P.scale[0, 0] == 0.5
    pm, pv = P.prior_mean.numpy(), P.prior_var.numpy()
    for c, n in ((1, Hs), (2, 30)):
        r = G.CtrRng(3, G.chain_key(c, 0))
        g, have = G.fit_gaussian_mixture(hist[c, :n].double().numpy(), r, pm, pv)
        assert int(P.ncomp[c]) == len(g.means)
        L = P.chol[c, 0].numpy()
        np.testing.assert_allclose(L @ L.T, g.covs[0], rtol=1e-9, atol=1e-14)
        np.testing.assert_allclose(P.mean[c, 0].numpy(), g.means[0], rtol=1e-12)
        assert P.scale[c, 0] == 2.38 / math.sqrt(d) and P.ema[c, 0] == P.target
    # chain 3 (one sample) restarts from the prior's moments
    assert torch.equal(P.chol[3, 0], chol0[3, 0])
    # global covariance: a fresh Proposal (adaptive scale 1, EMA 0.23) and the diagonal floored at
    # 1e-6 of the prior variance (ProposalGlobalCovariance.cpp:83-87)
    Gp = DeviceProposal("global_covariance", prior, temps)
    Gp.scale.fill_(0.7)
    flat = torch.ones((C, Hs, d), dtype=torch.float32)
    flat[:, ::2, 0] = 2.0
    Gp.adapt(flat, torch.tensor([[0, 0], [Hs, 0], [Hs, 0], [Hs, 0]], dtype=torch.int64))
    L = Gp.chol[1, 0].numpy()
    cov = L @ L.T
    var = ((prior.b - prior.a) ** 2 / 12.0).numpy()
    np.testing.assert_allclose(np.diag(cov)[1:], 1e-6 * var[1:], rtol=1e-12)
    assert Gp.scale[1, 0] == 1.0 and Gp.ema[1, 0] == 0.23 and Gp.scale[0, 0] == 0.7


def test_set_mixture_validates():
    from bcm3_amd.proposal import DeviceProposal
    prior = _prior()
    P = DeviceProposal("gaussian_mixture", prior, torch.linspace(0, 1, 3, dtype=torch.float64), kmax=2)
    d = prior.d
    P.set_mixture(1, [0.3, 0.7], np.zeros((2, d)), np.stack([np.eye(d), 2 * np.eye(d)]))
    assert P.ncomp[1] == 2 and abs(float(P.weights[1].sum()) - 1.0) < 1e-15
    np.testing.assert_allclose(P.logc[1, 1].item(), -0.5 * d * math.log(2.0) - 0.5 * d * math.log(2 * math.pi))
    with pytest.raises(ValueError):
        P.set_mixture(1, [1.0, 1.0, 1.0], np.zeros((3, d)), np.stack([np.eye(d)] * 3))
    with pytest.raises(ValueError):
        P.set_mixture(1, [1.0], np.zeros((1, d)), -np.eye(d)[None])
    with pytest.raises(ValueError):
        DeviceProposal("clustered_covariance", prior, torch.zeros(2, dtype=torch.float64))
