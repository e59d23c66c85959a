"""The C++ PT-MH sampler (libbcm3.so bcm3_ptmh_*, csrc/host/SamplerPTDevice.cpp) on the GPU:
* bit for bit the chains of the Python loop bcm3_amd.sampler.PTMHDevice over the same kernels
  (values, llh, lprior, lpp, acceptance counters), for C3 and for C2 with proposal adaptations;
* a ladder sharded over 2 and 4 in-process ranks (one host thread each, host-staged transport in
  place of RCCL) gives the chains of the single-rank run bit for bit -- the counter-based random
  numbers make the result independent of the rank count, as SURVEY.md §8(e) requires."""
import os
import threading

import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _python_loop(lik, pri, C, seed, steps, **kw):
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.pt import temperature_ladder
    from bcm3_amd.sampler import DevicePrior, PTMHDevice, load_prior
    ll = Likelihood(lik, pri, device=0)
    loop = PTMHDevice(ll, DevicePrior(load_prior(pri), "cuda"), temperature_ladder(C), seed=seed, device="cuda", **kw)
    for _ in range(steps):
        loop.iteration()
    torch.cuda.synchronize()
    st = dict(values=loop.values.cpu().numpy(), llh=loop.llh.cpu().numpy(), lprior=loop.lprior.cpu().numpy(),
              lpp=loop.lpp.cpu().numpy())
    cnt = dict(accepted_mutate=int(loop.accepted_mutate.item()), attempted_mutate=loop.attempted_mutate,
               accepted_exchange=int(loop.accepted_exchange.item()), attempted_exchange=loop.attempted_exchange,
               adaptations_done=loop.adaptations_done)
    return st, cnt, (loop.proposal.ncomp.cpu().numpy() if loop.adaptive else None)


def _native(lik, pri, C, seed, steps, rank=0, world=1, group=None, **kw):
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.ptmh import TRANSPORT_LOCAL, PTMHNative
    ll = Likelihood(lik, pri, device=0)
    extra = dict(transport=TRANSPORT_LOCAL, group=group) if world > 1 else {}
    return PTMHNative(ll, pri, C, rank=rank, world=world, seed=seed, **extra, **kw)


def _same(a, b):
    return np.array_equal(a, b, equal_nan=True)


def _semantic(c):
    """the sampler's counters without the launch statistics (which speculation changes by design)"""
    return {k: v for k, v in c.items() if k not in ("likelihood_launches", "evaluated_entries")}


def _compare(st_py, st_nat):
    for k in ("values", "llh", "lprior", "lpp"):
        assert _same(st_py[k], st_nat[k]), k


C3 = (os.path.join(H.GOLDEN, "c3_likelihood.xml"), os.path.join(H.GOLDEN, "c3_prior.xml"))
C2 = (os.path.join(H.GOLDEN, "circular_likelihood.xml"), os.path.join(H.GOLDEN, "circular_prior.xml"))


def test_native_matches_python_loop_c3():
    st, cnt, _ = _python_loop(*C3, 256, 11, 50)
    s = _native(*C3, 256, 11, 50)
    s.iterate(50)
    s.synchronize()
    _compare(st, s.state())
    c = s.counters()
    for k in ("accepted_mutate", "attempted_mutate", "accepted_exchange", "attempted_exchange"):
        assert c[k] == cnt[k], k
    assert c["samples_done"] == 50 and c["rounds"] == 50
    # not only self-consistent: every chain's llh is the oracle's value of its parameter vector
    # (the reference's CVODE restated bit for bit) inside the parity envelope (tests/parity.py)
    _assert_llh_matches_oracle(s.state())


def _assert_llh_matches_oracle(st):
    import oracle as O
    import parity
    r = O.Oracle("restated").popk_eval(H.c3_problem(1), st["values"], nthreads=8, want_traj=False)
    got, ref = st["llh"], r["logp"]
    mism = np.isfinite(got) != np.isfinite(ref)
    assert np.all(r["stats"][mism, 0, 0] >= 0.99 * H.c3_problem(1).max_steps)
    err = parity.llh_err(got[~mism], ref[~mism])
    parity.log_summary({"llh_t1": float(np.mean(err <= parity.LLH_T1)), "llh_max": float(err.max())}, n=int(err.size))
    assert np.mean(err <= parity.LLH_T1) >= parity.llh_min_fraction(err.size) and np.all(err <= parity.LLH_T2)


@pytest.mark.parametrize("proposal,scheme", [("gaussian_mixture", "deterministic_even_odd"),
                                             ("global_covariance", "stochastic_even_odd"),
                                             ("gaussian_mixture_adjustedAIC", "stochastic_random"),
                                             ("random_walk", "deterministic_even_odd")])
def test_native_matches_python_loop_with_adaptation(proposal, scheme):
    kw = dict(adapt_proposal_samples=40, adapt_proposal_times=2)
    py_kw = dict(kw, proposal=proposal, swapping_scheme=scheme)
    st, cnt, nc = _python_loop(*C2, 32, 5, 130, **py_kw)
    s = _native(*C2, 32, 5, 130, proposal=proposal, swapping_scheme=scheme, **kw)
    s.iterate(130)
    s.synchronize()
    _compare(st, s.state())
    c = s.counters()
    for k in cnt:
        assert c[k] == cnt[k], k
    if proposal != "random_walk":
        assert c["adaptations_done"] == 2
        assert np.array_equal(s.components(), nc)


@pytest.mark.parametrize("world,scheme", [(2, "deterministic_even_odd"), (4, "deterministic_even_odd"),
                                          (2, "stochastic_random")])
def test_native_sharded_ladder_equals_single_rank(world, scheme):
    C, seed, steps = 32, 9, 90
    kw = dict(adapt_proposal_samples=30, adapt_proposal_times=1, swapping_scheme=scheme)
    one = _native(*C2, C, seed, steps, **kw)
    one.iterate(steps)
    one.synchronize()
    ref = one.state()
    from bcm3_amd.ptmh import LocalGroup
    group = LocalGroup(world)
    ranks = [_native(*C2, C, seed, steps, rank=r, world=world, group=group, **kw) for r in range(world)]
    errors = []

    def go(s):
        try:
            s.iterate(steps)
            s.synchronize()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=go, args=(s,)) for s in ranks]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errors, errors
    n = C // world
    for r, s in enumerate(ranks):
        st = s.state()
        for k in ("values", "llh", "lprior", "lpp"):
            assert _same(st[k], ref[k][r * n:(r + 1) * n]), (r, k)
    tot = {k: sum(s.counters()[k] for s in ranks) for k in ("accepted_mutate", "attempted_exchange",
                                                             "accepted_exchange")}
    c1 = one.counters()
    for k, v in tot.items():
        assert v == c1[k], k


def _samples(path):
    from scipy.io import netcdf_file
    with netcdf_file(path, "r", mmap=False) as f:
        return {k.partition(".")[2]: np.array(x[:]) for k, x in f.variables.items()}


def test_sample_output_file(tmp_path):
    """SampleHandlerNetCDF: every use_every_nth-th iteration all chains are stored (SamplerPT::
    EmitSample); the last stored sample equals the final chain state; the sharded ladder's ranks
    write one shared file identical to the single-rank one"""
    C, seed, nth, N = 32, 4, 3, 10
    kw = dict(adapt_proposal_samples=4, adapt_proposal_times=1, use_every_nth=nth)
    one = _native(*C2, C, seed, 0, **kw)
    p1 = str(tmp_path / "one.nc")
    one.set_output(p1, N, flush_every=4)
    one.run(N)
    st = one.state()
    one.close()
    v = _samples(p1)
    assert v["variable_values"].shape == (N, C, 2)
    assert np.array_equal(v["variable_values"][N - 1], st["values"])
    assert np.array_equal(v["log_prior"][N - 1], st["lprior"]) and np.array_equal(v["log_likelihood"][N - 1], st["llh"])
    assert np.all(v["weights"] == 1.0) and list(v["sample_ix"]) == list(range(N))
    from bcm3_amd.pt import temperature_ladder
    np.testing.assert_allclose(v["temperature"], np.asarray(temperature_ladder(C)), rtol=1e-15, atol=0)
    # the sharded ladder: 2 ranks, one file
    from bcm3_amd.ptmh import LocalGroup
    group = LocalGroup(2)
    p2 = str(tmp_path / "two.nc")
    ranks = [_native(*C2, C, seed, 0, rank=r, world=2, group=group, **kw) for r in range(2)]
    for s in ranks:
        s.set_output(p2, N, flush_every=3)
    errors = []

    def go(s):
        try:
            s.run(N)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=go, args=(s,)) for s in ranks]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errors, errors
    for s in ranks:
        s.close()
    w = _samples(p2)
    for k in v:
        assert np.array_equal(v[k], w[k]), k


def test_adaptation_output_file(tmp_path):
    """ptmhsampler.output_proposal_adaptation in the reference's layout (SamplerPTChain.cpp:88-97,
    149-166): adapt0 = the hottest chain's initial prior-moment proposal without history, then one
    group adapt<k> per fit k = 1, 2, ... with the mixture (weights, means, covariances) and the
    history it was fitted to"""
    from scipy.io import netcdf_file
    C, seed = 16, 6
    s = _native(*C2, C, seed, 0, adapt_proposal_samples=40, adapt_proposal_times=2)
    path = str(tmp_path / "sampler_adaptation.nc")
    s.set_adaptation_output(path)
    s.iterate(130)
    s.synchronize()
    nc = s.components()
    s.close()
    with netcdf_file(path, "r", mmap=False) as f:
        v = {k: np.array(x[:]) for k, x in f.variables.items()}
    for a in (0, 1, 2):
        g = f"adapt{a}.block1."
        assert list(v[g + "variable_indices"]) == [0, 1]
        w = v[g + "gmm_weights"]
        assert abs(w.sum() - 1.0) < 1e-12 and np.all(w > 0)
        for k in range(len(w)):
            S = v[g + f"cluster{k}_covariance"]
            assert S.shape == (2, 2) and np.allclose(S, S.T) and np.all(np.linalg.eigvalsh(S) > 0)
            assert v[g + f"cluster{k}_mean"].shape == (2,)
        assert list(v[g + "gmm_weights_dim"]) == list(range(1, len(w) + 1))
    # adapt0: one component at the prior's moments (C2 prior: U(-6, 6)^2 -> mean 0, variance 12)
    assert len(v["adapt0.block1.gmm_weights"]) == 1
    np.testing.assert_allclose(v["adapt0.block1.cluster0_mean"], [0.0, 0.0], atol=1e-12)
    np.testing.assert_allclose(v["adapt0.block1.cluster0_covariance"], np.diag([12.0, 12.0]), rtol=1e-12)
    assert len(v["adapt2.block1.gmm_weights"]) == nc[-1]
    assert "adapt0.block1.history" not in v
    assert v["adapt1.block1.history"].shape[1] == 2 and v["adapt2.block1.history"].shape[1] == 2
    assert "adapt3.block1.gmm_weights" not in v


def test_netcdf4_outputs_through_libnetcdf(tmp_path, monkeypatch):
    """with libnetcdf loadable (the test double tests/plugins/fake_netcdf.c here) the sampler writes
    output.nc and sampler_adaptation.nc as netCDF-4, as the reference does (NetCDFDataFile::Create,
    NC_CLOBBER | NC_NETCDF4): real groups samples and adapt<k>/block1, the same content as the
    classic files of the same run"""
    import subprocess
    from bcm3_amd.ptmh import read_data_file
    so = str(tmp_path / "libfake_netcdf.so")
    subprocess.run(["gcc", "-O1", "-shared", "-fPIC", "-o", so, os.path.join(os.path.dirname(H.GOLDEN), "plugins", "fake_netcdf.c")],
                   check=True)

    def run(tag):
        s = _native(*C2, 16, 6, 0, adapt_proposal_samples=40, adapt_proposal_times=2)
        out, ad = str(tmp_path / f"output_{tag}.nc"), str(tmp_path / f"adapt_{tag}.nc")
        try:
            s.set_output(out, 130, flush_every=16)
            s.set_adaptation_output(ad)
            s.iterate(130)
            s.synchronize()
            s.flush_output()
        finally:
            s.close()
        return out, ad

    monkeypatch.setenv("BCM3_LIBNETCDF", so)
    out4, ad4 = run("4")
    monkeypatch.setenv("BCM3_OUTPUT_FORMAT", "classic")
    out3, ad3 = run("3")
    monkeypatch.setenv("BCM3_OUTPUT_FORMAT", "auto")
    for p in (out4, ad4):
        assert open(p, "rb").read(8) == b"\x89HDF\r\n\x1a\n", p
    a4, a3 = read_data_file(out4), read_data_file(out3)
    assert a4["samples"]["variable_values"] == {k: v for k, v in a3["samples"]["variable_values"].items()}
    for k in ("log_prior", "log_likelihood", "weights", "sample_ix", "variable", "temperature"):
        assert a4["samples"][k]["data"] == a3["samples"][k]["data"], k
    b4, b3 = read_data_file(ad4), read_data_file(ad3)
    groups = sorted(g for g in b4 if g)
    assert groups == ["adapt0.block1", "adapt1.block1", "adapt2.block1"] and groups == sorted(g for g in b3 if g)
    for g in groups:
        for k, v in b4[g].items():
            assert v["dims"] == b3[g][k]["dims"] and v["data"] == b3[g][k]["data"], (g, k)


@pytest.mark.parametrize("proposal,C,t_dof", [("gaussian_mixture", 64, 0.0), ("global_covariance", 64, 0.0),
                                              ("gaussian_mixture_adjustedAIC", 63, 0.0), ("gaussian_mixture", 32, 5.0)])
def test_speculative_pairs_bit_identical(tmp_path, proposal, C, t_dof):
    """SamplerPTDevice's speculative iteration pairs (one likelihood launch per two iterations, the
    second iteration's proposal picked from the candidates after accept / exchange) against the
    one-launch-per-iteration loop: the same chains, counters, fitted mixtures and sample file bit for
    bit, with adaptations falling on either iteration of a pair (use_every_nth 1 and 3),
    an odd ladder (one chain without an exchange partner in alternate rounds) and t proposals"""
    from scipy.io import netcdf_file
    res = []
    for spec in (0, 1):
        for every in (1, 3):
            # adaptation after si = 40 (the first iteration of a pair: that pair is not formed) or after
            # si = 41 (every = 3, adaptation every 14 samples: the second iteration of a pair)
            s = _native(*C3, C, 17, 0, proposal=proposal, adapt_proposal_samples=41 if every == 1 else 14,
                        adapt_proposal_times=2, t_dof=t_dof, speculate=spec, use_every_nth=every)
            out = str(tmp_path / f"out_{spec}_{every}.nc")
            s.set_output(out, 130 // every, flush_every=7)
            s.iterate(131 if every == 1 else 130)
            s.synchronize()
            s.flush_output()
            st, c, nc = s.state(), s.counters(), s.components()
            s.close()
            with netcdf_file(out, "r", mmap=False) as f:
                vv = np.array(f.variables["samples.variable_values"][:])
            res.append((spec, every, st, c, nc, vv))
    for (s0, e0, st0, c0, nc0, v0), (s1, e1, st1, c1, nc1, v1) in zip(res[:2], res[2:]):
        assert (s0, s1, e0) == (0, 1, e1)
        _compare(st0, st1)
        assert _semantic(c0) == _semantic(c1) and c0["adaptations_done"] == 2
        assert np.array_equal(nc0, nc1)
        assert _same(v0, v1)


@pytest.mark.parametrize("C", [256, 512])
def test_speculative_pairs_bit_identical_large_batches(C):
    """the batch layouts of ptmh_spec_batch_kernel at the chip's size: 256 chains make ~1,300 entries
    (more than the 1,024 SIMDs: the shortest pair up on shared SIMDs, the longest run alone); 512
    chains make ~2,600 (more than two per SIMD: plain longest-first order). Either way every entry is
    evaluated once and the chains match the one-launch-per-iteration loop bit for bit"""
    res = []
    for spec in (0, 1):
        s = _native(*C3, C, 23, 0, speculate=spec)
        s.iterate(24)
        s.synchronize()
        res.append((s.state(), s.counters()))
        if spec:
            info = s.spec_batch_info()
            assert info is not None and len(info[0]) > C  # speculation was used
            assert len(set(info[0].tolist())) == len(info[0])  # each entry at one position
        s.close()
    _compare(res[0][0], res[1][0])
    assert _semantic(res[0][1]) == _semantic(res[1][1])
    # the launch statistics: one launch per iteration vs one per two, the speculative one evaluating
    # the proposals plus their candidates
    c0, c1 = res[0][1], res[1][1]
    assert c0["evaluated_entries"] == C * c0["likelihood_launches"]
    assert c1["likelihood_launches"] < c0["likelihood_launches"] and c1["evaluated_entries"] > c0["evaluated_entries"]


def test_spec_tail_matches_separate_launches(monkeypatch):
    """the end of a speculative pair in one launch (bcm3hip_ptmh_spec_tail: commit r, exchange r + 1,
    commit r + 1 in one workgroup) against the three launches it replaces (BCM3_NO_SPEC_TAIL): the
    same chains and counters bit for bit, 256 chains (the bench's ladder)"""
    res = []
    for off in (False, True):
        if off:
            monkeypatch.setenv("BCM3_NO_SPEC_TAIL", "1")
        s = _native(*C3, 256, 29, 0, speculate=1)
        s.iterate(24)
        s.synchronize()
        res.append((s.state(), s.counters()))
        s.close()
    _compare(res[0][0], res[1][0])
    assert _semantic(res[0][1]) == _semantic(res[1][1])


def test_speculation_is_used_for_popk():
    """the C3 sampler runs its iterations as speculative pairs: one likelihood launch per two
    iterations (the timing log counts launches)"""
    from bcm3_amd import _hip
    s = _native(*C3, 64, 3, 0)
    s.ll.set_option(_hip.OPT_TIMING_LOG, 1)
    s.iterate(20)
    s.synchronize()
    _, launches, _ = s.ll.kernel_time_log()
    s.ll.set_option(_hip.OPT_TIMING_LOG, 0)
    s.close()
    assert launches == 10


@pytest.mark.parametrize("world", [2, 4])
def test_speculative_pairs_sharded_ladder(world):
    """speculative pairs on a sharded C3 ladder (in-process ranks, host-staged transport): the boundary
    chains' candidates start from the neighbour rank's (state, proposal) rows, the cross-rank swap
    picks among them -- bit-identical to the single-rank loop without speculation"""
    C, seed, steps = 32, 13, 61
    kw = dict(adapt_proposal_samples=25, adapt_proposal_times=1)
    one = _native(*C3, C, seed, steps, speculate=0, **kw)
    one.iterate(steps)
    one.synchronize()
    ref, cref = one.state(), one.counters()
    one.close()
    from bcm3_amd.ptmh import LocalGroup
    group = LocalGroup(world)
    ranks = [_native(*C3, C, seed, steps, rank=r, world=world, group=group, speculate=1, **kw)
             for r in range(world)]
    errors = []

    def go(s):
        try:
            s.iterate(steps)
            s.synchronize()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=go, args=(s,)) for s in ranks]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    assert not errors, errors
    got = [s.state() for s in ranks]
    infos = [s.spec_batch_info() for s in ranks]
    acc = sum(s.counters()["accepted_mutate"] for s in ranks)
    for s in ranks:
        s.close()
    assert all(i is not None for i in infos), "speculation not used"
    for k in ("values", "llh", "lprior", "lpp"):
        assert _same(np.concatenate([g[k] for g in got]), ref[k]), k
    assert acc == cref["accepted_mutate"]
