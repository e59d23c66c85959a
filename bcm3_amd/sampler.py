"""Device-resident PT-MH iteration: per-chain mutate move with one batched likelihood launch,
then the even/odd exchange (bcm3_amd.pt).

Restates, for the sampler's hot loop only (SURVEY.md §8 a):
* SamplerPT::Run's DeterministicEvenOdd iteration (src/sampler/SamplerPT.cpp:203-212):
  DoExchangeMove then num_exploration_steps DoMutateMove;
* SamplerPTChain::MutateMove (src/sampler/SamplerPTChain.cpp:217-313): T == 0 chains draw from
  the prior and always accept; T > 0 chains propose, evaluate prior + likelihood, and accept by
  TestSample (:465-481, MH ratio of a symmetric proposal = 0);
* Sampler::EvaluateLikelihood (src/sampler/Sampler.cpp:164-180): llh *= learning rate;
* PriorIndependence::EvaluateLogPDF (src/sampler/PriorIndependence.cpp:129-157) with
  UnivariateMarginal::EvaluateLogPDF uniform / normal (src/sampler/UnivariateMarginal.cpp:326-345).

* the per-block proposal of MutateMove (SamplerPTChain.cpp:241-310) with its state in HBM:
  gaussian_mixture (the reference's default proposal_type) or global_covariance, with the scale
  adaptation, MH ratio and sample history (bcm3_amd/proposal.py, csrc/proposal_kernels.hip), and the
  periodic proposal adaptation of SamplerPT::Run (SamplerPT.cpp:229-248).

The reference evaluates the C chains' likelihoods one per task-manager thread; here all C
proposals go to the GPU in one bcm3_likelihood_evaluate_batch_device launch, between the
propose / accept kernels. proposal="random_walk" keeps a fixed diagonal Gaussian random walk
(bcm3_amd/csrc/pt_kernels.hip) for comparisons.
"""
from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from dataclasses import dataclass
from typing import List, Optional

import torch

from .proposal import DeviceProposal, SampleHistory, history_geometry
from .pt import PTExchange, move_uniform, random_pair


@dataclass
class Marginal:
    kind: str  # "uniform" | "normal"
    a: float = 0.0
    b: float = 0.0
    mu: float = 0.0
    sigma: float = 1.0


def load_prior(path: str) -> List[Marginal]:
    """Univariate marginals of a prior.xml in variable order (VariableSet::LoadFromXML repeat rule)."""
    root = ET.parse(path).getroot()
    out = []
    for v in root.iter("variable"):
        dist = v.get("distribution")
        if dist == "uniform":
            m = Marginal("uniform", a=float(v.get("lower")), b=float(v.get("upper")))
            if m.b <= m.a:
                raise ValueError("Uniform distribution with upper bound less than or equal to lower bound.")
        elif dist == "normal":
            m = Marginal("normal", mu=float(v.get("mu")), sigma=float(v.get("sigma")))
        else:
            raise ValueError(f"prior distribution '{dist}' not supported by the device sampler")
        out += [m] * int(v.get("repeat", "1"))
    return out


class DevicePrior:
    def __init__(self, marginals: List[Marginal], device):
        dev = torch.device(device)
        self.d = len(marginals)
        self.is_uniform = torch.tensor([m.kind == "uniform" for m in marginals], device=dev)
        self.a = torch.tensor([m.a for m in marginals], dtype=torch.float64, device=dev)
        self.b = torch.tensor([m.b for m in marginals], dtype=torch.float64, device=dev)
        self.mu = torch.tensor([m.mu for m in marginals], dtype=torch.float64, device=dev)
        self.sigma = torch.tensor([m.sigma for m in marginals], dtype=torch.float64, device=dev)
        self.log_uniform = -torch.log(self.b - self.a)
        self.log_norm = torch.log(torch.rsqrt(2.0 * self.sigma * self.sigma * math.pi))
        self.inv2s2 = 1.0 / (2.0 * self.sigma * self.sigma)
        # proposal scale for the random walk: a fixed fraction of the marginal's spread
        self.scale = torch.where(self.is_uniform, 0.02 * (self.b - self.a), 0.1 * self.sigma)

    def log_pdf(self, x: torch.Tensor) -> torch.Tensor:
        inside = (x >= self.a) & (x <= self.b)
        lu = torch.where(inside, self.log_uniform, torch.full_like(x, -math.inf))
        dx = x - self.mu
        ln = self.log_norm - dx * dx * self.inv2s2
        return torch.where(self.is_uniform, lu, ln).sum(dim=1)

    def sample(self, n: int, gen: torch.Generator) -> torch.Tensor:
        u = torch.rand((n, self.d), dtype=torch.float64, device=self.a.device, generator=gen)
        z = torch.randn((n, self.d), dtype=torch.float64, device=self.a.device, generator=gen)
        return torch.where(self.is_uniform, self.a + u * (self.b - self.a), self.mu + self.sigma * z)


class PTMHDevice:
    """C chains of one rank, state in HBM; one iteration = exchange kernel (+ RCCL for the pairs
    that straddle ranks) -> propose kernel -> batched likelihood launch -> accept kernel, all on
    torch's current stream (include/bcm3hip.h: bcm3hip_pt_exchange_local, bcm3hip_ptmh_propose,
    bcm3hip_ptmh_accept). No host synchronisation inside an iteration."""

    INIT_ITER = (1 << 63) - 1  # RNG iteration index reserved for the initial prior draw

    def __init__(self, likelihood, prior: DevicePrior, temperatures, rank=0, world=1, seed=0, device="cuda",
                 learning_rate: float = 1.0, exploration_steps: int = 1, group=None,
                 proposal: str = "gaussian_mixture", t_dof: float = 0.0, kmax: int = 1,
                 adapt_proposal_samples: int = 2000, adapt_proposal_times: int = 2, max_history_size: int = 2000,
                 use_every_nth: int = 1, swapping_scheme: str = "deterministic_even_odd",
                 exchange_probability: float = 0.5):
        from . import _hip
        self._hip = _hip
        _hip.lib()  # fails loudly without the HIP library
        self.ll, self.prior = likelihood, prior
        self.dev = torch.device(device)
        self.ex = PTExchange(temperatures, rank=rank, world=world, seed=seed, device=self.dev, group=group)
        self.C, self.d = self.ex.C, prior.d
        self.Ctot, self.rank, self.world = self.ex.Ctot, rank, world
        self.g0 = rank * self.C
        self.T = self.ex.T
        self.lr = float(learning_rate)
        self.seed = int(seed)
        self.exploration_steps = exploration_steps
        self.iter = 0
        self.round = 0
        C, d, dev = self.C, self.d, self.dev
        self.kind = torch.where(prior.is_uniform, 0, 1).to(torch.int32)
        self.p0 = torch.where(prior.is_uniform, prior.a, prior.mu).contiguous()
        self.p1 = torch.where(prior.is_uniform, prior.b, prior.sigma).contiguous()
        self.scale = prior.scale.contiguous()
        self.values = torch.empty((C, d), dtype=torch.float64, device=dev)
        self.prop = torch.empty((C, d), dtype=torch.float64, device=dev)
        self.lprior = torch.empty(C, dtype=torch.float64, device=dev)
        self.lprior_prop = torch.empty(C, dtype=torch.float64, device=dev)
        self.llh = torch.empty(C, dtype=torch.float64, device=dev)
        self.llh_prop = torch.empty(C, dtype=torch.float64, device=dev)
        self.status = torch.empty(C, dtype=torch.int32, device=dev)
        self.lpp = torch.empty(C, dtype=torch.float64, device=dev)
        self.accepted_mutate = torch.zeros(1, dtype=torch.int64, device=dev)
        self.accepted_exchange = torch.zeros(1, dtype=torch.int64, device=dev)
        self.attempted_mutate = 0
        self.attempted_exchange = 0
        # ptmhsampler.swapping_scheme / exchange_probability (SamplerPT.cpp:63-75, 163-164)
        if swapping_scheme not in ("deterministic_even_odd", "stochastic_even_odd", "stochastic_random"):
            raise ValueError(f"Unknown swapping scheme \"{swapping_scheme}\"")
        self.scheme = swapping_scheme
        self.exchange_probability = float(exchange_probability)
        # proposals (ptmhsampler.proposal_type) and the sample history that adapts them
        self.proposal_type = proposal
        self.adaptive = proposal != "random_walk"
        self.use_every_nth = int(use_every_nth)
        self.adapt_samples, self.adapt_times = int(adapt_proposal_samples), int(adapt_proposal_times)
        self.adaptations_done = 0
        self.samples_done = 0
        if self.adaptive:
            self.proposal = DeviceProposal(proposal, prior, self.T, kmax=kmax, t_dof=t_dof)
            H, sub = history_geometry(self.adapt_samples, self.use_every_nth, exploration_steps, self.Ctot,
                                      max_history_size, deterministic=(swapping_scheme == "deterministic_even_odd"))
            self.history = SampleHistory(C, d, H, sub, dev)
            self.log_mh = torch.zeros(C, dtype=torch.float64, device=dev)
            self._masks = {start: self._exchange_masks(start) for start in (0, 1)}
        # initial state: every chain draws from the prior (the propose kernel at T = 0)
        zeros = torch.zeros(C, dtype=torch.float64, device=dev)
        _hip.ptmh_propose(C, d, self.kind.data_ptr(), self.p0.data_ptr(), self.p1.data_ptr(), self.scale.data_ptr(),
                          zeros.data_ptr(), self.values.data_ptr(), self.values.data_ptr(), self.lprior.data_ptr(),
                          self.g0, self.seed, self.INIT_ITER, self._stream())
        self._eval(self.values, self.llh)
        self.llh.mul_(self.lr)
        self.lpp.copy_(self.ex.lpowerposterior(self.llh, self.lprior))

    def _stream(self):
        return torch.cuda.current_stream(self.dev).cuda_stream

    def _eval(self, x: torch.Tensor, out: torch.Tensor):
        self.ll.evaluate_batch_device(self.C, x.data_ptr(), out.data_ptr(), self.status.data_ptr(), self._stream())

    def exchange(self):
        """DoExchangeMove round (SamplerPT.cpp:277-298): local pairs on the GPU, boundary pairs
        over RCCL point-to-point."""
        if self.Ctot < 2:
            return
        start = self.round % 2
        wrap_local = self.world == 1 and (self.Ctot - 1 - start) % 2 == 0
        self._hip.pt_exchange_local(self.C, self.d, self.g0, start, wrap_local, self.T.data_ptr(),
                                    self.values.data_ptr(), self.llh.data_ptr(), self.lprior.data_ptr(),
                                    self.lpp.data_ptr(), None, self.accepted_exchange.data_ptr(), self.seed,
                                    self.round, self._stream())
        n_local = sum(1 for i in range(self.C - 1) if (self.g0 + i - start) % 2 == 0) + int(wrap_local)
        self.attempted_exchange += n_local
        if self.world > 1 and (self.g0 + self.C - 1 - start) % 2 == 0:
            acc = torch.zeros(self.C, dtype=torch.bool, device=self.dev)
            self.ex.round = self.round
            self.ex._cross(self.values, self.llh, self.lprior, self.lpp, acc)
            self.accepted_exchange += acc[self.C - 1:].to(torch.int64)
            self.attempted_exchange += 1
        if self.adaptive:
            # ExchangeMove adds the (possibly swapped) state of both chains of a pair to their
            # histories (SamplerPTChain.cpp:374-379)
            for mask in self._masks[start]:
                self.history.add(self.T, self.values, mask, self._stream())
        self.round += 1

    def _exchange_masks(self, start: int):
        return [None if m is None else torch.tensor(m, dtype=torch.uint8, device=self.dev)
                for m in exchange_participants(self.C, self.g0, self.Ctot, self.world, start)]

    def mutate(self):
        """DoMutateMove (SamplerPT.cpp:308-319): all chains' proposals in one likelihood launch."""
        h, C, d, st = self._hip, self.C, self.d, self._stream()
        if self.adaptive:
            P = self.proposal.struct
            h.ptmh_propose_adaptive(C, d, self.kind.data_ptr(), self.p0.data_ptr(), self.p1.data_ptr(),
                                    self.T.data_ptr(), self.values.data_ptr(), self.prop.data_ptr(),
                                    self.lprior_prop.data_ptr(), self.log_mh.data_ptr(), P, self.g0, self.seed,
                                    self.iter, st)
            self._eval(self.prop, self.llh_prop)
            h.ptmh_accept_adaptive(C, d, self.T.data_ptr(), self.prop.data_ptr(), self.lprior_prop.data_ptr(),
                                   self.llh_prop.data_ptr(), self.log_mh.data_ptr(), self.lr, self.values.data_ptr(),
                                   self.lprior.data_ptr(), self.llh.data_ptr(), self.lpp.data_ptr(), None,
                                   self.accepted_mutate.data_ptr(), P, self.g0, self.seed, self.iter, st)
            self.history.add(self.T, self.values, None, st)  # SamplerPTChain.cpp:309
            self.attempted_mutate += C
            self.iter += 1
            return
        h.ptmh_propose(C, d, self.kind.data_ptr(), self.p0.data_ptr(), self.p1.data_ptr(), self.scale.data_ptr(),
                       self.T.data_ptr(), self.values.data_ptr(), self.prop.data_ptr(), self.lprior_prop.data_ptr(),
                       self.g0, self.seed, self.iter, st)
        self._eval(self.prop, self.llh_prop)
        h.ptmh_accept(C, d, self.T.data_ptr(), self.prop.data_ptr(), self.lprior_prop.data_ptr(),
                      self.llh_prop.data_ptr(), self.lr, self.values.data_ptr(), self.lprior.data_ptr(),
                      self.llh.data_ptr(), self.lpp.data_ptr(), None, self.accepted_mutate.data_ptr(), self.g0,
                      self.seed, self.iter, st)
        self.attempted_mutate += C
        self.iter += 1

    def exchange_random(self):
        """stochastic_random DoExchangeMove (SamplerPT.cpp:300-305): one pair (ci, ci + 1), ci drawn
        from a counter-based stream every rank computes alike; a pair inside this rank's slice
        runs on the GPU, a pair across a slice boundary over RCCL between its two ranks."""
        ci = random_pair(self.seed, self.round, self.Ctot)
        l1, l2 = ci - self.g0, ci + 1 - self.g0
        if 0 <= l1 and l2 < self.C:
            self._hip.pt_exchange_pair(self.C, self.d, l1, l2, ci, self.T.data_ptr(), self.values.data_ptr(),
                                       self.llh.data_ptr(), self.lprior.data_ptr(), self.lpp.data_ptr(), None,
                                       self.accepted_exchange.data_ptr(), self.seed, self.round, self._stream())
            self.attempted_exchange += 1
        elif self.world > 1 and (l1 == self.C - 1 or l2 == 0):
            self.ex.round = self.round
            a = self.ex.step_single(self.values, self.llh, self.lprior, self.lpp, ci)
            if l1 == self.C - 1:
                self.accepted_exchange += a.to(torch.int64)
                self.attempted_exchange += 1
        if self.adaptive:
            mine = [i for i in (l1, l2) if 0 <= i < self.C]
            if mine:
                mask = torch.zeros(self.C, dtype=torch.uint8, device=self.dev)
                mask[mine] = 1
                self.history.add(self.T, self.values, mask, self._stream())
        self.round += 1

    def iteration(self, last: bool = False):
        """One iteration of SamplerPT::Run (SamplerPT.cpp:191-219): deterministic_even_odd = an
        exchange round then num_exploration_steps mutate moves; the stochastic schemes make an
        exchange move with probability exchange_probability, else one mutate move; a single chain
        only mutates. Then the proposal adaptation every adapt_proposal_samples samples, at most
        adapt_proposal_times times and not after the last sample (SamplerPT.cpp:226-248)."""
        if self.Ctot < 2:
            self.mutate()
        elif self.scheme == "deterministic_even_odd":
            self.exchange()
            for _ in range(self.exploration_steps):
                self.mutate()
        elif move_uniform(self.seed, self.samples_done) < self.exchange_probability:
            if self.scheme == "stochastic_even_odd":
                self.exchange()
            else:
                self.exchange_random()
        else:
            self.mutate()
        si = self.samples_done
        self.samples_done += 1
        if self.adaptive and (si + 1) % self.use_every_nth == 0:
            sample_ix = si // self.use_every_nth
            if (self.adapt_samples > 0 and (sample_ix + 1) % self.adapt_samples == 0 and not last
                    and self.adaptations_done < self.adapt_times):
                self.adapt_proposal()

    def adapt_proposal(self):
        """SamplerPTChain::AdaptProposal for every chain of the rank (T == 0 chains excepted)."""
        self.proposal.adapt(self.history.samples, self.history.counters)
        self.adaptations_done += 1

    def run(self, num_samples: int):
        """SamplerPT::Run's loop over num_samples * use_every_nth iterations."""
        total = num_samples * self.use_every_nth
        for si in range(total):
            self.iteration(last=(si + 1 == total))

def exchange_participants(C: int, g0: int, Ctot: int, world: int, start: int):
    """Chains of the rank owning global chains [g0, g0+C) that are in a pair in an exchange round
    with this start (SamplerPT.cpp:279-298), as one list of flags per pair set; [None] when every
    chain is in exactly one pair. A chain in two pairs (the wrap pair of an odd single-rank ladder)
    appears in two lists, so its history receives both samples as in the reference."""
    if Ctot < 2:
        return []
    local = [False] * C
    for i in range(C - 1):
        if (g0 + i - start) % 2 == 0:
            local[i] = local[i + 1] = True
    extra = [False] * C
    if world == 1:
        if (Ctot - 1 - start) % 2 == 0:  # wrap pair (C-1, 0)
            extra[C - 1] = extra[0] = True
    else:
        if (g0 + C - 1 - start) % 2 == 0:  # the last chain pairs with the next rank's first
            extra[C - 1] = True
        if ((g0 - 1) % Ctot - start) % 2 == 0:  # the first chain pairs with the previous rank's last
            extra[0] = True
    if all(a != b for a, b in zip(local, extra)):
        return [None]
    return [m for m in (local, extra) if any(m)]
