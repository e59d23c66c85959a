"""Parallel-tempering exchange step on GPU tensors, sharded over ranks.

Restates SamplerPT::DoExchangeMove (src/sampler/SamplerPT.cpp:277-306, even/odd scheme) and
SamplerPTChain::ExchangeMove (src/sampler/SamplerPTChain.cpp:328-381) for chains laid out as
contiguous ladder slices per rank: rank r owns global chains [r*C, (r+1)*C).

Per round, pairs (i, i+1) for i = start, start+2, ... with start alternating 0/1 (first round 0)
and the reference's wrap pair (C_total-1 <-> 0). Pairs inside a slice are swapped locally with
tensor ops; a pair straddling two ranks (a slice boundary, or the wrap pair) exchanges one
record {values[d], llh, lprior, lpowerposterior, T} with the neighbour over RCCL point-to-point
(torch.distributed batch_isend_irecv; backend "nccl" == RCCL on ROCm, over xGMI). Both ranks
then take the identical decision: the acceptance uniform is counter based -- splitmix64 of
(seed, round, global index of the pair's first chain) -- so 1/2/4/8-rank runs produce
bit-identical swap bookkeeping. (The reference draws it from one global ranlux48 stream in pair
order; its runs are not reproducible anyway)

Requires an even number of chains per rank when world > 1 (then no chain is in two pairs).
"""
from __future__ import annotations

import math
from typing import Optional

import torch

_M64 = (1 << 64) - 1


def _u64(x: int) -> int:
    return x & _M64


def splitmix64(x: int) -> int:
    x = _u64(x + 0x9E3779B97F4A7C15)
    z = x
    z = _u64((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9)
    z = _u64((z ^ (z >> 27)) * 0x94D049BB133111EB)
    return z ^ (z >> 31)


def exchange_uniform(seed: int, rnd: int, pair: int) -> float:
    """Counter-based uniform in [0, 1) for (seed, round, pair) -- host reference."""
    z = splitmix64(_u64(splitmix64(_u64(seed)) ^ _u64(rnd * 0x100000001B3) ^ _u64(pair * 0xC2B2AE3D27D4EB4F)))
    return (z >> 11) * (1.0 / 9007199254740992.0)


# salts of the stochastic swapping schemes' draws (SamplerPT::Run, SamplerPT.cpp:195-202, 300-305):
# the reference draws both from its global ranlux48 stream; here they are counter based too
_MOVE_SALT = 0x6D6F76655F747970
_PAIR_SALT = 0x706169725F696478


def move_uniform(seed: int, iteration: int) -> float:
    """Uniform deciding exchange (< exchange_probability) vs mutate in a stochastic scheme."""
    return exchange_uniform(seed ^ _MOVE_SALT, iteration, 0)


def random_pair(seed: int, rnd: int, Ctot: int) -> int:
    """stochastic_random: first chain ci of the pair (ci, ci + 1), uniform in [0, Ctot - 2]
    (rng.GetUnsignedInt(chains.size() - 2), SamplerPT.cpp:301)."""
    return min(int(exchange_uniform(seed ^ _PAIR_SALT, rnd, 0) * (Ctot - 1)), Ctot - 2)


def _t_splitmix64(x: torch.Tensor) -> torch.Tensor:
    # int64 tensors with two's-complement wraparound; >> emulated as a logical shift
    def lsr(v, k):
        return (v >> k) & ((1 << (64 - k)) - 1)

    x = x + torch.tensor(0x9E3779B97F4A7C15 - (1 << 64), dtype=torch.int64, device=x.device)
    z = x
    z = (z ^ lsr(z, 30)) * torch.tensor(0xBF58476D1CE4E5B9 - (1 << 64), dtype=torch.int64, device=x.device)
    z = (z ^ lsr(z, 27)) * torch.tensor(0x94D049BB133111EB - (1 << 64), dtype=torch.int64, device=x.device)
    return z ^ lsr(z, 31)


def _signed(v: int) -> int:
    v &= _M64
    return v - (1 << 64) if v >= (1 << 63) else v


def exchange_uniforms_tensor(seed: int, rnd: int, pairs: torch.Tensor) -> torch.Tensor:
    """Same as exchange_uniform, vectorised over pair indices (int64 tensor) on any device."""
    base = _signed(splitmix64(_u64(seed)) ^ _u64(rnd * 0x100000001B3))
    mul = _signed(0xC2B2AE3D27D4EB4F)
    z = _t_splitmix64(torch.tensor(base, dtype=torch.int64, device=pairs.device) ^ (pairs * mul))
    hi = (z >> 11) & ((1 << 53) - 1)
    return hi.to(torch.float64) * (1.0 / 9007199254740992.0)


def temperature_ladder(num_chains: int, power: float = 3.0, tmax: float = 1.0):
    """SamplerPT::LoadSettings ladder (SamplerPT.cpp:83-93): T0 = 0, Ti = Tmax (i/(C-1))^power."""
    t = [0.0] * num_chains
    for i in range(1, num_chains - 1):
        alpha = i / float(num_chains - 1)
        t[i] = tmax * math.pow(alpha, power)
    t[num_chains - 1] = tmax
    return t


def _proposed(t_self, llh_other, lprior_other):
    # ExchangeMove (.cpp:336-347): T == 0 -> lprior of the other chain (avoids 0 * -inf)
    return torch.where(t_self == 0.0, lprior_other, t_self * llh_other + lprior_other)


class PTExchange:
    """Even/odd exchange over a sharded temperature ladder (see module docstring)."""

    def __init__(self, temperatures, rank: int = 0, world: int = 1, seed: int = 0, device="cpu",
                 group: Optional[object] = None):
        self.Ctot = len(temperatures)
        assert self.Ctot % world == 0, "chains must divide evenly over ranks"
        self.C = self.Ctot // world
        if world > 1:
            assert self.C % 2 == 0, "distributed exchange needs an even number of chains per rank"
        self.rank, self.world, self.seed, self.device, self.group = rank, world, seed, torch.device(device), group
        self.T = torch.tensor(temperatures[rank * self.C:(rank + 1) * self.C], dtype=torch.float64,
                              device=self.device)
        self.round = 0
        self.attempted = 0
        self.accepted = torch.zeros((), dtype=torch.int64, device=self.device)

    def lpowerposterior(self, llh, lprior):
        return torch.where(self.T == 0.0, lprior, lprior + self.T * llh)

    def _accept(self, t1, t2, llh1, llh2, lp1, lp2, lpp1, lpp2, pair_idx):
        p1 = _proposed(t1, llh2, lp2)
        p2 = _proposed(t2, llh1, lp1)
        tp = torch.exp((p1 + p2) - (lpp1 + lpp2))
        tp = torch.where(tp < 1.0, tp, torch.ones_like(tp))  # std::min(1.0, tp): NaN -> 1
        u = exchange_uniforms_tensor(self.seed, self.round, pair_idx)
        return u < tp, p1, p2

    def step(self, values: torch.Tensor, llh: torch.Tensor, lprior: torch.Tensor, lpp: torch.Tensor):
        """One exchange round in place. Returns the boolean accept mask of pairs whose FIRST
        chain is local (index = local chain id), for bookkeeping tests."""
        start = self.round % 2
        C, r = self.C, self.rank
        g0 = r * C
        acc_mask = torch.zeros(C, dtype=torch.bool, device=self.device)
        # (Ctot-1, 0) both local
        wrap_local = self.world == 1 and (self.Ctot - 1 - start) % 2 == 0 and self.Ctot > 1
        self.local_pairs(values, llh, lprior, lpp, start, wrap_local, acc_mask)
        if self.world > 1 and (g0 + C - 1 - start) % 2 == 0:
            self._cross(values, llh, lprior, lpp, acc_mask)
        self.round += 1
        return acc_mask

    def local_pairs(self, values, llh, lprior, lpp, start: int, wrap_local: bool, acc_mask=None):
        """The pairs of this round inside the rank's slice, with tensor ops (the device sampler
        runs the same decisions in pt_exchange_kernel)."""
        C, g0, dev = self.C, self.rank * self.C, self.device
        if acc_mask is None:
            acc_mask = torch.zeros(C, dtype=torch.bool, device=dev)
        # local pairs: global first index i with i >= g0, i+1 < g0 + C
        loc_first = [i for i in range(C - 1) if (g0 + i - start) % 2 == 0]
        if loc_first:
            i1 = torch.tensor(loc_first, dtype=torch.int64, device=dev)
            i2 = i1 + 1
            a, p1, p2 = self._accept(self.T[i1], self.T[i2], llh[i1], llh[i2], lprior[i1], lprior[i2], lpp[i1],
                                     lpp[i2], i1 + g0)
            self._apply_local(values, llh, lprior, lpp, i1, i2, a, p1, p2)
            acc_mask[i1] = a
            self.attempted += len(loc_first)
            self.accepted = self.accepted + a.sum()
        if wrap_local:
            i1 = torch.tensor([C - 1], dtype=torch.int64, device=dev)
            i2 = torch.tensor([0], dtype=torch.int64, device=dev)
            a, p1, p2 = self._accept(self.T[i1], self.T[i2], llh[i1], llh[i2], lprior[i1], lprior[i2], lpp[i1],
                                     lpp[i2], i1 + g0)
            self._apply_local(values, llh, lprior, lpp, i1, i2, a, p1, p2)
            acc_mask[i1] = a
            self.attempted += 1
            self.accepted = self.accepted + a.sum()
        return acc_mask

    def step_single(self, values: torch.Tensor, llh: torch.Tensor, lprior: torch.Tensor, lpp: torch.Tensor, ci: int):
        """One stochastic_random exchange of the global pair (ci, ci + 1) in place (SamplerPT.cpp:300-305);
        ranks owning neither chain do nothing. Returns the accept flag (a 1-element tensor) on the
        ranks that own a chain of the pair, else None."""
        C, g0, dev = self.C, self.rank * self.C, self.device
        l1, l2 = ci - g0, ci + 1 - g0
        a = None
        gl = torch.tensor([ci], dtype=torch.int64, device=dev)
        if 0 <= l1 and l2 < C:
            i1 = torch.tensor([l1], dtype=torch.int64, device=dev)
            i2 = torch.tensor([l2], dtype=torch.int64, device=dev)
            a, p1, p2 = self._accept(self.T[i1], self.T[i2], llh[i1], llh[i2], lprior[i1], lprior[i2], lpp[i1],
                                     lpp[i2], gl)
            self._apply_local(values, llh, lprior, lpp, i1, i2, a, p1, p2)
        elif self.world > 1 and l1 == C - 1:
            o = self._exchange_record(values, llh, lprior, lpp, C - 1, (self.rank + 1) % self.world)
            d = values.shape[1]
            a, p1, _ = self._accept(self.T[C - 1:C], o[d + 3:d + 4], llh[C - 1:C], o[d:d + 1], lprior[C - 1:C],
                                    o[d + 1:d + 2], lpp[C - 1:C], o[d + 2:d + 3], gl)
            self._take(values, llh, lprior, lpp, C - 1, o, a, p1)
        elif self.world > 1 and l2 == 0:
            q = self._exchange_record(values, llh, lprior, lpp, 0, (self.rank - 1) % self.world)
            d = values.shape[1]
            a, _, p2 = self._accept(q[d + 3:d + 4], self.T[0:1], q[d:d + 1], llh[0:1], q[d + 1:d + 2], lprior[0:1],
                                    q[d + 2:d + 3], lpp[0:1], gl)
            self._take(values, llh, lprior, lpp, 0, q, a, p2)
        if a is not None and 0 <= l1:
            self.attempted += 1
            self.accepted = self.accepted + a.sum()
        self.round += 1
        return a

    def _exchange_record(self, values, llh, lprior, lpp, i, peer):
        """Send chain i's {values, llh, lprior, lpp, T} to `peer` and receive the peer's record."""
        import torch.distributed as dist
        d = values.shape[1]
        mine = torch.cat([values[i], torch.stack([llh[i], lprior[i], lpp[i], self.T[i]])])
        other = torch.empty(d + 4, dtype=torch.float64, device=self.device)
        ops = [dist.P2POp(dist.isend, mine, peer, self.group), dist.P2POp(dist.irecv, other, peer, self.group)]
        for req in dist.batch_isend_irecv(ops):
            req.wait()
        return other

    @staticmethod
    def _take(values, llh, lprior, lpp, i, rec, a, p):
        d = values.shape[1]
        values[i] = torch.where(a, rec[:d], values[i])
        llh[i:i + 1] = torch.where(a, rec[d:d + 1], llh[i:i + 1])
        lprior[i:i + 1] = torch.where(a, rec[d + 1:d + 2], lprior[i:i + 1])
        lpp[i:i + 1] = torch.where(a, p, lpp[i:i + 1])

    @staticmethod
    def _apply_local(values, llh, lprior, lpp, i1, i2, a, p1, p2):
        """Swap accepted pairs without a host sync: gather through a pair permutation."""
        C = llh.shape[0]
        perm = torch.arange(C, device=llh.device)
        perm[i1] = torch.where(a, i2, i1)
        perm[i2] = torch.where(a, i1, i2)
        new_lpp = lpp.clone()
        new_lpp[i1] = torch.where(a, p1, lpp[i1])
        new_lpp[i2] = torch.where(a, p2, lpp[i2])
        values.copy_(values[perm])
        llh.copy_(llh[perm])
        lprior.copy_(lprior[perm])
        lpp.copy_(new_lpp)

    def _cross(self, values, llh, lprior, lpp, acc_mask):
        """Slice-boundary pairs: (my last, next rank's first) and (prev rank's last, my first)."""
        import torch.distributed as dist
        C, d = self.C, values.shape[1]
        nxt, prv = (self.rank + 1) % self.world, (self.rank - 1) % self.world

        def record(i):
            return torch.cat([values[i], torch.stack([llh[i], lprior[i], lpp[i], self.T[i]])])

        send_last, send_first = record(C - 1), record(0)
        recv_next = torch.empty(d + 4, dtype=torch.float64, device=self.device)
        recv_prev = torch.empty(d + 4, dtype=torch.float64, device=self.device)
        ops = [dist.P2POp(dist.isend, send_last, nxt, self.group), dist.P2POp(dist.irecv, recv_prev, prv, self.group),
               dist.P2POp(dist.isend, send_first, prv, self.group), dist.P2POp(dist.irecv, recv_next, nxt, self.group)]
        for req in dist.batch_isend_irecv(ops):
            req.wait()
        dev = self.device
        # pair A: (my last = chain1, next rank's first = chain2); its global index is my last chain's
        o = recv_next
        gl = torch.tensor([self.rank * C + C - 1], dtype=torch.int64, device=dev)
        a, p1, _ = self._accept(self.T[C - 1:C], o[d + 3:d + 4], llh[C - 1:C], o[d:d + 1], lprior[C - 1:C],
                                o[d + 1:d + 2], lpp[C - 1:C], o[d + 2:d + 3], gl)
        # pair B: (previous rank's last = chain1, my first = chain2)
        q = recv_prev
        gp = torch.tensor([prv * C + C - 1], dtype=torch.int64, device=dev)
        b, _, r2 = self._accept(q[d + 3:d + 4], self.T[0:1], q[d:d + 1], llh[0:1], q[d + 1:d + 2], lprior[0:1],
                                q[d + 2:d + 3], lpp[0:1], gp)
        values[C - 1] = torch.where(a, o[:d], values[C - 1])
        llh[C - 1:C] = torch.where(a, o[d:d + 1], llh[C - 1:C])
        lprior[C - 1:C] = torch.where(a, o[d + 1:d + 2], lprior[C - 1:C])
        lpp[C - 1:C] = torch.where(a, p1, lpp[C - 1:C])
        values[0] = torch.where(b, q[:d], values[0])
        llh[0:1] = torch.where(b, q[d:d + 1], llh[0:1])
        lprior[0:1] = torch.where(b, q[d + 1:d + 2], lprior[0:1])
        lpp[0:1] = torch.where(b, r2, lpp[0:1])
        acc_mask[C - 1:C] = a
        self.attempted += 1
        self.accepted = self.accepted + a.sum()
