"""The sharded C++ sampler across OS processes (VERDICT r03 "next" 4): two processes, one rank each,
sharing the test GPU, exchange the slice-boundary PT swap records (SamplerPT::DoExchangeMove,
src/sampler/SamplerPT.cpp:277-306; SamplerPTChain::ExchangeMove, SamplerPTChain.cpp:328-381)
over the socket transport (RCCL, the production transport between GPUs, refuses two ranks on one
device). With the counter-based random numbers the ladder is bit-identical to one rank in one
process -- including the speculative pairs, whose boundary candidates start from the neighbour
rank's (state, proposal) rows."""
import os
import subprocess
import sys

import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu

WORKER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "workers", "ptmh_rank.py")
C3 = (os.path.join(H.GOLDEN, "c3_likelihood.xml"), os.path.join(H.GOLDEN, "c3_prior.xml"))


def _single_rank(C, seed, steps):
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.ptmh import PTMHNative
    ll = Likelihood(*C3, device=0)
    s = PTMHNative(ll, C3[1], C, seed=seed, speculate=0, adapt_proposal_samples=25, adapt_proposal_times=1)
    s.iterate(steps)
    s.synchronize()
    st, cnt = s.state(), s.counters()
    s.close()
    return st, cnt


@pytest.mark.parametrize("speculate", [1, 0])
def test_two_processes_bit_identical_to_one_rank(tmp_path, speculate):
    C, seed, steps, world = 32, 17, 61, 2
    ref, cref = _single_rank(C, seed, steps)
    sock = str(tmp_path / "s")
    os.makedirs(sock)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, WORKER, str(tmp_path / f"rank{r}.npz"), sock, str(r), str(world), str(C),
                               str(seed), str(steps), str(speculate)], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=240)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), outs
    got = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    if speculate:
        assert all(bool(g["speculated"]) for g in got), "speculation not used"
    for k in ("values", "llh", "lprior", "lpp"):
        assert np.array_equal(np.concatenate([g[k] for g in got]), ref[k], equal_nan=True), k
    assert sum(int(g["accepted_mutate"]) for g in got) == cref["accepted_mutate"]


def test_two_processes_netcdf4_output_is_the_one_rank_file(tmp_path, monkeypatch):
    """a sharded ladder writes the reference's netCDF-4 output.nc
    (SampleHandlerNetCDF.cpp:24-110) -- rank 0 receives the other ranks' staged sample rows over the
    transport at each flush and writes every temperature; through the libnetcdf test double
    (tests/plugins/fake_netcdf.c) the file holds exactly what one rank writes for the same seed"""
    from test_netcdf import _fake_netcdf
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.ptmh import PTMHNative, read_data_file
    C, seed, steps, world = 16, 23, 30, 2
    monkeypatch.setenv("BCM3_LIBNETCDF", _fake_netcdf(tmp_path))
    one = str(tmp_path / "one.nc")
    ll = Likelihood(*C3, device=0)
    s = PTMHNative(ll, C3[1], C, seed=seed, speculate=0, adapt_proposal_samples=25, adapt_proposal_times=1)
    s.set_output(one, steps, flush_every=7)
    s.iterate(steps)
    s.synchronize()
    s.flush_output()
    s.close()
    sharded = str(tmp_path / "sharded.nc")
    sock = str(tmp_path / "s")
    os.makedirs(sock)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, WORKER, str(tmp_path / f"rank{r}.npz"), sock, str(r), str(world), str(C),
                               str(seed), str(steps), "0", sharded], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=240)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    assert all(p.returncode == 0 for p in procs), outs
    for f in (one, sharded):
        assert open(f, "rb").read(8) == b"\x89HDF\r\n\x1a\n", f  # netCDF-4 (the double's HDF5 signature)
    a, b = read_data_file(one)["samples"], read_data_file(sharded)["samples"]
    assert set(a) == set(b)
    for k in a:
        assert a[k]["dims"] == b[k]["dims"], k
        assert a[k]["data"] == b[k]["data"], k
    assert len(a["temperature"]["data"]) == C
