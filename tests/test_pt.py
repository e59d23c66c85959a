"""PT exchange step (bcm3_amd.pt) against the sequential restatement of
SamplerPT::DoExchangeMove / SamplerPTChain::ExchangeMove (oracle/pt_oracle.py): swap bookkeeping
must be bit-identical for 1 rank and for the sharded ladder over 2 and 4 gloo ranks."""
import copy
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import pt_oracle
from bcm3_amd import pt

ROUNDS = 40


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _initial_state(Ctot, d, seed):
    rng = np.random.default_rng(seed)
    values = rng.normal(size=(Ctot, d))
    llh = rng.normal(-50.0, 2.0, size=Ctot)
    llh[rng.random(Ctot) < 0.1] = -math.inf  # failed likelihoods, as the reference produces
    lprior = rng.normal(-5.0, 1.0, size=Ctot)
    return values, llh, lprior


def _run_oracle(temps, values, llh, lprior, seed, rounds):
    chains = []
    for i in range(len(temps)):
        lpp = lprior[i] if temps[i] == 0.0 else lprior[i] + temps[i] * llh[i]
        chains.append({"values": list(values[i]), "llh": float(llh[i]), "lprior": float(lprior[i]), "lpp": lpp})
    log = []
    for r in range(rounds):
        log.append(pt_oracle.exchange_round(chains, temps, r, seed, pt.exchange_uniform))
    return chains, log


def _run_sharded(temps, values, llh, lprior, seed, rounds, rank, world):
    ex = pt.PTExchange(temps, rank=rank, world=world, seed=seed)
    C = ex.C
    sl = slice(rank * C, (rank + 1) * C)
    v = torch.tensor(values[sl]).clone()
    l = torch.tensor(llh[sl]).clone()
    q = torch.tensor(lprior[sl]).clone()
    lpp = ex.lpowerposterior(l, q)
    acc = []
    for _ in range(rounds):
        acc.append(ex.step(v, l, q, lpp).numpy().copy())
    return v.numpy(), l.numpy(), q.numpy(), lpp.numpy(), np.array(acc)


def _compare(chains, log, res, rank, C):
    v, l, q, lpp, acc = res
    for i in range(C):
        g = rank * C + i
        assert np.array_equal(v[i], np.array(chains[g]["values"]))
        assert l[i] == chains[g]["llh"] or (math.isinf(l[i]) and math.isinf(chains[g]["llh"]))
        assert q[i] == chains[g]["lprior"]
        assert lpp[i] == chains[g]["lpp"] or (math.isnan(lpp[i]) and math.isnan(chains[g]["lpp"]))
    for r, pairs in enumerate(log):
        for ci, _, a in pairs:
            if rank * C <= ci < (rank + 1) * C:
                assert bool(acc[r][ci - rank * C]) == a, (r, ci)


def test_uniform_tensor_matches_host():
    pairs = torch.arange(0, 300, dtype=torch.int64)
    for seed, rnd in ((0, 0), (12345, 7), (2**63 + 5, 2**40)):
        u = pt.exchange_uniforms_tensor(seed, rnd, pairs)
        ref = [pt.exchange_uniform(seed, rnd, int(p)) for p in pairs]
        assert u.tolist() == ref
        assert 0.0 <= min(ref) and max(ref) < 1.0


def test_ladder_matches_reference_schedule():
    t = pt.temperature_ladder(8, power=3.0, tmax=1.0)
    assert t[0] == 0.0 and t[-1] == 1.0
    assert t[3] == 1.0 * math.pow(3 / 7.0, 3.0)
    assert all(a < b for a, b in zip(t, t[1:]))


@pytest.mark.parametrize("Ctot", [2, 7, 8, 16])
def test_single_rank_matches_sequential(Ctot):
    temps = pt.temperature_ladder(Ctot)
    values, llh, lprior = _initial_state(Ctot, 5, Ctot)
    chains, log = _run_oracle(temps, values, llh, lprior, 99, ROUNDS)
    res = _run_sharded(temps, values, llh, lprior, 99, ROUNDS, 0, 1)
    _compare(chains, log, res, 0, Ctot)
    assert any(a for pairs in log for _, _, a in pairs)


def _worker(rank, world, port, Ctot, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        temps = pt.temperature_ladder(Ctot)
        values, llh, lprior = _initial_state(Ctot, 3, 1234)
        res = _run_sharded(temps, values, llh, lprior, 7, ROUNDS, rank, world)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,Ctot", [(2, 8), (4, 16), (2, 4)])
def test_sharded_gloo_matches_sequential(world, Ctot):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, Ctot, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    temps = pt.temperature_ladder(Ctot)
    values, llh, lprior = _initial_state(Ctot, 3, 1234)
    chains, log = _run_oracle(temps, values, llh, lprior, 7, ROUNDS)
    C = Ctot // world
    for r in range(world):
        _compare(chains, log, results[r], r, C)
    # at least one cross-rank swap happened, so the P2P path was exercised
    cross = [a for pairs in log for ci, _, a in pairs if (ci + 1) % C == 0]
    assert any(cross)


# ---- stochastic_random: one pair per exchange move (SamplerPT.cpp:300-305)

def _run_oracle_single(temps, values, llh, lprior, seed, rounds):
    chains = []
    for i in range(len(temps)):
        lpp = lprior[i] if temps[i] == 0.0 else lprior[i] + temps[i] * llh[i]
        chains.append({"values": list(values[i]), "llh": float(llh[i]), "lprior": float(lprior[i]), "lpp": lpp})
    log = []
    for r in range(rounds):
        ci = pt.random_pair(seed, r, len(temps))
        log.append([(ci, ci + 1, pt_oracle.exchange_single(chains, temps, ci, r, seed, pt.exchange_uniform))])
    return chains, log


def _run_sharded_single(temps, values, llh, lprior, seed, rounds, rank, world):
    ex = pt.PTExchange(temps, rank=rank, world=world, seed=seed)
    C = ex.C
    sl = slice(rank * C, (rank + 1) * C)
    v = torch.tensor(values[sl]).clone()
    l = torch.tensor(llh[sl]).clone()
    q = torch.tensor(lprior[sl]).clone()
    lpp = ex.lpowerposterior(l, q)
    acc = []
    for r in range(rounds):
        ci = pt.random_pair(seed, r, len(temps))
        a = ex.step_single(v, l, q, lpp, ci)
        m = np.zeros(C, dtype=bool)
        if a is not None and 0 <= ci - rank * C < C:
            m[ci - rank * C] = bool(a.item())
        acc.append(m)
    return v.numpy(), l.numpy(), q.numpy(), lpp.numpy(), np.array(acc)


def test_random_pair_range():
    got = {pt.random_pair(3, r, 6) for r in range(400)}
    assert got == {0, 1, 2, 3, 4}
    assert all(0.0 <= pt.move_uniform(9, i) < 1.0 for i in range(100))


def test_single_pair_single_rank_matches_sequential():
    Ctot = 9
    temps = pt.temperature_ladder(Ctot)
    values, llh, lprior = _initial_state(Ctot, 4, 5)
    chains, log = _run_oracle_single(temps, values, llh, lprior, 17, ROUNDS)
    _compare(chains, log, _run_sharded_single(temps, values, llh, lprior, 17, ROUNDS, 0, 1), 0, Ctot)
    assert any(a for pairs in log for _, _, a in pairs)


def _worker_single(rank, world, port, Ctot, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        temps = pt.temperature_ladder(Ctot)
        values, llh, lprior = _initial_state(Ctot, 3, 4321)
        q.put((rank, _run_sharded_single(temps, values, llh, lprior, 11, 3 * ROUNDS, rank, world)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,Ctot", [(2, 8), (4, 8)])
def test_single_pair_sharded_gloo_matches_sequential(world, Ctot):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_single, args=(r, world, port, Ctot, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    temps = pt.temperature_ladder(Ctot)
    values, llh, lprior = _initial_state(Ctot, 3, 4321)
    chains, log = _run_oracle_single(temps, values, llh, lprior, 11, 3 * ROUNDS)
    C = Ctot // world
    for r in range(world):
        _compare(chains, log, results[r], r, C)
    assert any(a for pairs in log for ci, _, a in pairs if (ci + 1) % C == 0)  # a cross-rank swap happened


# ---- the device sampler's exchange driver (sampler.sharded_exchange_round + exchange_participants),
# with the pairs inside a slice on PTExchange.local_pairs in place of the HIP kernel

def _run_driver(temps, values, llh, lprior, seed, rounds, rank, world):
    from bcm3_amd.sampler import exchange_participants, sharded_exchange_round
    ex = pt.PTExchange(temps, rank=rank, world=world, seed=seed)
    C, Ctot = ex.C, ex.Ctot
    g0 = rank * C
    sl = slice(g0, g0 + C)
    v = torch.tensor(values[sl]).clone()
    l = torch.tensor(llh[sl]).clone()
    q = torch.tensor(lprior[sl]).clone()
    lpp = ex.lpowerposterior(l, q)
    accepted = torch.zeros(1, dtype=torch.int64)
    attempted = 0
    hist = []
    for r in range(rounds):
        def local(start, wrap_local, r=r):
            ex.round = r
            a = ex.local_pairs(v, l, q, lpp, start, wrap_local)
            accepted.add_(a.sum())
        attempted += sharded_exchange_round(ex, local, v, l, q, lpp, r, accepted)
        masks = exchange_participants(C, g0, Ctot, world, r % 2)
        cnt = np.zeros(C, dtype=int)
        for m in masks:
            cnt += 1 if m is None else np.array(m, dtype=int)
        hist.append(cnt)
    return (v.numpy(), l.numpy(), q.numpy(), lpp.numpy()), attempted, int(accepted.item()), np.array(hist)


def _worker_driver(rank, world, port, Ctot, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        temps = pt.temperature_ladder(Ctot)
        values, llh, lprior = _initial_state(Ctot, 3, 99)
        q.put((rank, _run_driver(temps, values, llh, lprior, 5, ROUNDS, rank, world)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,Ctot", [(1, 8), (2, 8), (4, 16)])
def test_device_exchange_driver_matches_sequential(world, Ctot):
    """PTMHDevice.exchange's driver: states bit-identical to the sequential DoExchangeMove replay,
    attempted / accepted counts per rank (each pair on the rank of its first chain), and the
    history masks add each chain exactly as often as the reference's ExchangeMove adds it
    (SamplerPTChain.cpp:374-379: both chains of every pair)."""
    temps = pt.temperature_ladder(Ctot)
    values, llh, lprior = _initial_state(Ctot, 3, 99)
    chains, log = _run_oracle(temps, values, llh, lprior, 5, ROUNDS)
    if world == 1:
        results = {0: _run_driver(temps, values, llh, lprior, 5, ROUNDS, 0, 1)}
    else:
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_worker_driver, args=(r, world, port, Ctot, q)) for r in range(world)]
        for p in procs:
            p.start()
        results = dict(q.get(timeout=120) for _ in range(world))
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    C = Ctot // world
    for r in range(world):
        state, attempted, accepted, hist = results[r]
        _compare(chains, [[]] * ROUNDS, (*state, None), r, C)
        mine = [(ci, a) for pairs in log for ci, _, a in pairs if r * C <= ci < (r + 1) * C]
        assert attempted == len(mine)
        assert accepted == sum(a for _, a in mine)
        for rnd, pairs in enumerate(log):
            want = np.zeros(C, dtype=int)
            for ci, ix2, _ in pairs:
                for g in (ci, ix2):
                    if r * C <= g < (r + 1) * C:
                        want[g - r * C] += 1
            assert np.array_equal(hist[rnd], want), (r, rnd)
