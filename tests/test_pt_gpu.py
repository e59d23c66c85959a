"""GPU tests of the PT-MH kernels (bcm3_amd/csrc/pt_kernels.hip) against their numpy restatement
(tests/ptmh_reference.py) and the sequential exchange oracle (oracle/pt_oracle.py)."""
import math
import os

import numpy as np
import pytest

import helpers as H
import pt_oracle
import ptmh_reference as R

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _prior():
    from bcm3_amd.sampler import DevicePrior, load_prior
    return DevicePrior(load_prior(os.path.join(H.GOLDEN, "c3_prior.xml")), "cuda")


def _prior_arrays(prior):
    kind = torch.where(prior.is_uniform, 0, 1).to(torch.int32)
    p0 = torch.where(prior.is_uniform, prior.a, prior.mu).contiguous()
    p1 = torch.where(prior.is_uniform, prior.b, prior.sigma).contiguous()
    return kind, p0, p1, prior.scale.contiguous()


def test_propose_matches_reference():
    from bcm3_amd import _hip
    from bcm3_amd.pt import temperature_ladder
    prior = _prior()
    kind, p0, p1, scale = _prior_arrays(prior)
    C, d = 64, prior.d
    temps = torch.tensor(temperature_ladder(C), dtype=torch.float64, device="cuda")
    gen = torch.Generator(device="cuda")
    gen.manual_seed(3)
    values = prior.sample(C, gen)
    prop = torch.empty_like(values)
    lp = torch.empty(C, dtype=torch.float64, device="cuda")
    for it in (0, 5, 2**40):
        _hip.ptmh_propose(C, d, kind.data_ptr(), p0.data_ptr(), p1.data_ptr(), scale.data_ptr(), temps.data_ptr(),
                          values.data_ptr(), prop.data_ptr(), lp.data_ptr(), 128, 77, it)
        torch.cuda.synchronize()
        rp, rl = R.propose(kind.cpu().numpy(), p0.cpu().numpy(), p1.cpu().numpy(), scale.cpu().numpy(),
                           temps.cpu().numpy(), values.cpu().numpy(), 128, 77, it)
        np.testing.assert_allclose(prop.cpu().numpy(), rp, rtol=1e-13, atol=1e-15)
        got = lp.cpu().numpy()
        assert np.array_equal(np.isinf(got), np.isinf(rl))
        np.testing.assert_allclose(got[np.isfinite(rl)], rl[np.isfinite(rl)], rtol=1e-13)
    # the T == 0 chain draws inside the prior bounds
    assert np.isfinite(lp.cpu().numpy()[0])


def test_accept_matches_reference():
    from bcm3_amd import _hip
    from bcm3_amd.pt import temperature_ladder
    rng = np.random.default_rng(5)
    C, d = 200, 4
    temps = np.array(temperature_ladder(C))
    prop = rng.normal(size=(C, d))
    lprior_prop = rng.normal(-3, 1, size=C)
    lprior_prop[rng.random(C) < 0.1] = -math.inf
    llh_prop = rng.normal(-50, 3, size=C)
    llh_prop[rng.random(C) < 0.1] = -math.inf
    values = rng.normal(size=(C, d))
    lprior = rng.normal(-3, 1, size=C)
    llh = rng.normal(-50, 3, size=C)
    lpp = np.where(temps == 0, lprior, lprior + temps * llh)
    ref = [a.copy() for a in (values, lprior, llh, lpp)]
    racc = R.accept(temps, prop, lprior_prop, llh_prop, 0.5, *ref, 1000, 9, 3)
    t = {k: torch.tensor(v, device="cuda") for k, v in dict(temps=temps, prop=prop, lprior_prop=lprior_prop,
                                                             llh_prop=llh_prop, values=values, lprior=lprior,
                                                             llh=llh, lpp=lpp).items()}
    acc = torch.zeros(C, dtype=torch.uint8, device="cuda")
    n = torch.zeros(1, dtype=torch.int64, device="cuda")
    _hip.ptmh_accept(C, d, t["temps"].data_ptr(), t["prop"].data_ptr(), t["lprior_prop"].data_ptr(),
                     t["llh_prop"].data_ptr(), 0.5, t["values"].data_ptr(), t["lprior"].data_ptr(), t["llh"].data_ptr(),
                     t["lpp"].data_ptr(), acc.data_ptr(), n.data_ptr(), 1000, 9, 3)
    torch.cuda.synchronize()
    assert np.array_equal(acc.cpu().numpy().astype(bool), racc)
    assert int(n.item()) == int(racc.sum())
    for k, r in zip(("values", "lprior", "llh", "lpp"), ref):
        assert np.array_equal(t[k].cpu().numpy(), r), k
    assert 0 < racc.mean() < 1


@pytest.mark.parametrize("Ctot,rounds", [(8, 6), (7, 6), (256, 4)])
def test_exchange_kernel_matches_sequential_oracle(Ctot, rounds):
    from bcm3_amd import _hip
    from bcm3_amd.pt import exchange_uniform, temperature_ladder
    rng = np.random.default_rng(Ctot)
    d = 3
    temps = temperature_ladder(Ctot)
    values = rng.normal(size=(Ctot, d))
    llh = rng.normal(-50.0, 2.0, size=Ctot)
    llh[rng.random(Ctot) < 0.1] = -math.inf
    lprior = rng.normal(-5.0, 1.0, size=Ctot)
    lpp = np.array([lprior[i] if temps[i] == 0.0 else lprior[i] + temps[i] * llh[i] for i in range(Ctot)])
    chains = [{"values": list(values[i]), "llh": float(llh[i]), "lprior": float(lprior[i]), "lpp": float(lpp[i])}
              for i in range(Ctot)]
    tv = torch.tensor(values, device="cuda")
    tl = torch.tensor(llh, device="cuda")
    tq = torch.tensor(lprior, device="cuda")
    tp = torch.tensor(lpp, device="cuda")
    tt = torch.tensor(temps, dtype=torch.float64, device="cuda")
    mask = torch.zeros(Ctot, dtype=torch.uint8, device="cuda")
    for r in range(rounds):
        log = pt_oracle.exchange_round(chains, temps, r, 11, exchange_uniform)
        start = r % 2
        wrap = (Ctot - 1 - start) % 2 == 0
        _hip.pt_exchange_local(Ctot, d, 0, start, wrap, tt.data_ptr(), tv.data_ptr(), tl.data_ptr(), tq.data_ptr(),
                               tp.data_ptr(), mask.data_ptr(), None, 11, r)
        torch.cuda.synchronize()
        m = mask.cpu().numpy()
        for ci, _, a in log:
            assert bool(m[ci]) == a, (r, ci)
    for i in range(Ctot):
        assert np.array_equal(tv[i].cpu().numpy(), np.array(chains[i]["values"]))
        assert tl[i].item() == chains[i]["llh"]
        assert tq[i].item() == chains[i]["lprior"]
        a, b = tp[i].item(), chains[i]["lpp"]
        assert a == b or (math.isnan(a) and math.isnan(b))


def test_device_sampler_runs_and_accepts():
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.pt import temperature_ladder
    from bcm3_amd.sampler import PTMHDevice
    prior = _prior()
    ll = Likelihood(os.path.join(H.GOLDEN, "c3_likelihood.xml"), os.path.join(H.GOLDEN, "c3_prior.xml"), device=0)
    loop = PTMHDevice(ll, prior, temperature_ladder(32), seed=4, device="cuda")
    lpp0 = loop.lpp.clone()
    for _ in range(20):
        loop.iteration()
    torch.cuda.synchronize()
    acc = int(loop.accepted_mutate.item()) / loop.attempted_mutate
    assert 0.05 < acc <= 1.0
    assert int(loop.accepted_exchange.item()) > 0
    # lpp bookkeeping stays consistent with lprior + T llh
    T = loop.T
    want = torch.where(T == 0, loop.lprior, loop.lprior + T * loop.llh)
    assert torch.allclose(loop.lpp, want, rtol=0, atol=1e-9, equal_nan=True)
    assert not torch.equal(lpp0, loop.lpp)


def test_exchange_pair_kernel_matches_sequential():
    """stochastic_random's single-pair exchange (bcm3hip_pt_exchange_pair) vs the sequential
    restatement of ExchangeMove, over many random pairs."""
    from bcm3_amd import _hip
    from bcm3_amd import pt
    Ctot, d, seed = 12, 4, 31
    temps = pt.temperature_ladder(Ctot)
    rng = np.random.default_rng(2)
    values = rng.normal(size=(Ctot, d))
    llh = rng.normal(-40.0, 3.0, size=Ctot)
    llh[3] = -math.inf
    lprior = rng.normal(-4.0, 1.0, size=Ctot)
    chains = []
    for i in range(Ctot):
        lpp = lprior[i] if temps[i] == 0.0 else lprior[i] + temps[i] * llh[i]
        chains.append({"values": list(values[i]), "llh": float(llh[i]), "lprior": float(lprior[i]), "lpp": lpp})
    T = torch.tensor(temps, dtype=torch.float64, device="cuda")
    v = torch.tensor(values, device="cuda")
    l = torch.tensor(llh, device="cuda")
    q = torch.tensor(lprior, device="cuda")
    p = torch.tensor([c["lpp"] for c in chains], device="cuda")
    acc = torch.zeros(1, dtype=torch.uint8, device="cuda")
    n_acc = 0
    for r in range(200):
        ci = pt.random_pair(seed, r, Ctot)
        want = pt_oracle.exchange_single(chains, temps, ci, r, seed, pt.exchange_uniform)
        _hip.pt_exchange_pair(Ctot, d, ci, ci + 1, ci, T.data_ptr(), v.data_ptr(), l.data_ptr(), q.data_ptr(),
                              p.data_ptr(), acc.data_ptr(), None, seed, r)
        torch.cuda.synchronize()
        assert bool(acc.item()) == want, r
        n_acc += want
    assert n_acc > 0
    for i in range(Ctot):
        assert np.array_equal(v[i].cpu().numpy(), np.array(chains[i]["values"]))
        a, b = p[i].item(), chains[i]["lpp"]
        assert a == b or (math.isnan(a) and math.isnan(b))


@pytest.mark.parametrize("scheme", ["stochastic_even_odd", "stochastic_random"])
def test_device_sampler_stochastic_schemes(scheme):
    from bcm3_amd import pt
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.pt import temperature_ladder
    from bcm3_amd.sampler import DevicePrior, PTMHDevice, load_prior
    prior = DevicePrior(load_prior(os.path.join(H.GOLDEN, "circular_prior.xml")), "cuda")
    ll = Likelihood(os.path.join(H.GOLDEN, "circular_likelihood.xml"), os.path.join(H.GOLDEN, "circular_prior.xml"),
                    device=0)
    s = PTMHDevice(ll, prior, temperature_ladder(16), seed=8, swapping_scheme=scheme, exchange_probability=0.3)
    s.run(200)
    torch.cuda.synchronize()
    n_ex = sum(pt.move_uniform(8, i) < 0.3 for i in range(200))
    assert s.attempted_mutate == 16 * (200 - n_ex)
    per_move = 8 if scheme == "stochastic_even_odd" else 1
    assert s.attempted_exchange == per_move * n_ex
    assert int(s.accepted_exchange.item()) > 0
    T = s.T
    want = torch.where(T == 0, s.lprior, s.lprior + T * s.llh)
    assert torch.allclose(s.lpp, want, rtol=0, atol=1e-9, equal_nan=True)


@pytest.mark.parametrize("adaptive", [False, True])
def test_accept_flags_nan_llh(adaptive):
    """Sampler::EvaluateLikelihood (Sampler.cpp:172-178): a NaN log-likelihood is fatal. The accept
    kernels leave that chain unchanged (T = 0 chains included) and raise the device flag."""
    from bcm3_amd import _hip
    from bcm3_amd.pt import temperature_ladder
    rng = np.random.default_rng(11)
    C, d = 64, 3
    temps = np.array(temperature_ladder(C))
    prop = rng.normal(size=(C, d))
    lprior_prop = rng.normal(-3, 1, size=C)
    llh_prop = rng.normal(-50, 3, size=C)
    llh_prop[[0, 9, 40]] = math.nan  # chain 0 is the T = 0 chain
    values = rng.normal(size=(C, d))
    lprior = rng.normal(-3, 1, size=C)
    llh = rng.normal(-50, 3, size=C)
    lpp = np.where(temps == 0, lprior, lprior + temps * llh)
    t = {k: torch.tensor(v, device="cuda") for k, v in dict(temps=temps, prop=prop, lprior_prop=lprior_prop,
                                                             llh_prop=llh_prop, values=values, lprior=lprior,
                                                             llh=llh, lpp=lpp).items()}
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    acc = torch.zeros(C, dtype=torch.uint8, device="cuda")
    ptr = {k: v.data_ptr() for k, v in t.items()}
    if adaptive:
        from bcm3_amd.proposal import DeviceProposal
        from bcm3_amd.sampler import DevicePrior, load_prior
        prior = DevicePrior(load_prior(os.path.join(H.GOLDEN, "banana_prior.xml"))[:1] * d, "cuda")
        P = DeviceProposal("gaussian_mixture", prior, t["temps"])
        P.selected.fill_(0)  # the propose kernel's choice of component (accept updates its EMA)
        log_mh = torch.zeros(C, dtype=torch.float64, device="cuda")
        _hip.ptmh_accept_adaptive(C, d, ptr["temps"], ptr["prop"], ptr["lprior_prop"], ptr["llh_prop"],
                                  log_mh.data_ptr(), 1.0, ptr["values"], ptr["lprior"], ptr["llh"], ptr["lpp"],
                                  acc.data_ptr(), None, P.struct, 0, 5, 2, nan_llh=flag.data_ptr())
    else:
        _hip.ptmh_accept(C, d, ptr["temps"], ptr["prop"], ptr["lprior_prop"], ptr["llh_prop"], 1.0, ptr["values"],
                         ptr["lprior"], ptr["llh"], ptr["lpp"], acc.data_ptr(), None, 0, 5, 2,
                         nan_llh=flag.data_ptr())
    torch.cuda.synchronize()
    assert int(flag.item()) == 1
    a = acc.cpu().numpy().astype(bool)
    for c in (0, 9, 40):
        assert not a[c]
        assert np.array_equal(t["values"][c].cpu().numpy(), values[c])
        assert t["llh"][c].item() == llh[c] and t["lpp"][c].item() == lpp[c]
    assert a.sum() > 0


def test_sampler_stops_on_nan_llh():
    """A NaN from the likelihood stops PTMHDevice.run, as the reference sampler stops."""
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.pt import temperature_ladder
    from bcm3_amd.sampler import DevicePrior, PTMHDevice, load_prior

    class NaNAfter:
        """The circular likelihood, with chain 5's result replaced by NaN from call `k` on."""

        def __init__(self, ll, k):
            self.ll, self.k, self.calls, self.loop = ll, k, 0, None

        def evaluate_batch_device(self, n, x, out, status, stream):
            self.ll.evaluate_batch_device(n, x, out, status, stream)
            self.calls += 1
            if self.loop is not None and self.calls >= self.k and out == self.loop.llh_prop.data_ptr():
                self.loop.llh_prop[5] = math.nan

    pri = os.path.join(H.GOLDEN, "circular_prior.xml")
    ll = NaNAfter(Likelihood(os.path.join(H.GOLDEN, "circular_likelihood.xml"), pri, device=0), 10)
    prior = DevicePrior(load_prior(pri), "cuda")
    loop = PTMHDevice(ll, prior, temperature_ladder(16), seed=3, device="cuda")
    ll.loop = loop
    loop.nan_check_every = 5
    with pytest.raises(RuntimeError, match="NaN"):
        loop.run(50)
    assert loop.samples_done <= 15
    # without the NaN the same loop runs through
    ok = PTMHDevice(ll.ll, prior, temperature_ladder(16), seed=3, device="cuda")
    ok.run(50)


def test_c5_2048_chains_on_one_gpu():
    """Config C5's ladder (2,048 chains) on one GPU through the product loop:
    the likelihoods of a proposal batch agree with the oracle within the parity envelope, and an
    exchange round over 2,048 chains is bit-identical to the sequential DoExchangeMove replay."""
    import oracle as O
    import parity
    from bcm3_amd import pt
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.sampler import PTMHDevice
    C, seed = 2048, 21
    prior = _prior()
    ll = Likelihood(os.path.join(H.GOLDEN, "c3_likelihood.xml"), os.path.join(H.GOLDEN, "c3_prior.xml"), device=0)
    temps = pt.temperature_ladder(C)
    loop = PTMHDevice(ll, prior, temps, seed=seed, device="cuda")
    for _ in range(3):
        loop.iteration()
    torch.cuda.synchronize()
    prop, got = loop.prop.cpu().numpy(), loop.llh_prop.cpu().numpy()
    r = O.Oracle("restated").popk_eval(H.c3_problem(1), prop, nthreads=8, want_traj=False)
    ref = r["logp"]
    # ok/fail may differ only where the oracle's trajectory ends within 1% of max_steps
    mism = np.isfinite(got) != np.isfinite(ref)
    assert np.all(r["stats"][mism, 0, 0] >= 1980)
    err = parity.llh_err(got[~mism], ref[~mism])
    parity.log_summary({"llh_t1": float(np.mean(err <= parity.LLH_T1)), "llh_max": float(err.max())}, n=int(err.size))
    assert np.mean(err <= parity.LLH_T1) >= parity.LLH_T1_FRAC and np.all(err <= parity.LLH_T2)
    # one exchange round of the whole ladder
    snap = [t.cpu().numpy().copy() for t in (loop.values, loop.llh, loop.lprior, loop.lpp)]
    rnd = loop.round
    loop.exchange()
    torch.cuda.synchronize()
    chains = [{"values": list(snap[0][i]), "llh": float(snap[1][i]), "lprior": float(snap[2][i]),
               "lpp": float(snap[3][i])} for i in range(C)]
    log = pt_oracle.exchange_round(chains, temps, rnd, seed, pt.exchange_uniform)
    assert len(log) == C // 2 and any(a for _, _, a in log)
    tv, tl, tq, tp = (t.cpu().numpy() for t in (loop.values, loop.llh, loop.lprior, loop.lpp))
    for i in range(C):
        assert np.array_equal(tv[i], np.array(chains[i]["values"])), i
        assert tl[i] == chains[i]["llh"] or (math.isinf(tl[i]) and math.isinf(chains[i]["llh"]))
        assert tq[i] == chains[i]["lprior"]
        assert tp[i] == chains[i]["lpp"] or (math.isnan(tp[i]) and math.isnan(chains[i]["lpp"]))
