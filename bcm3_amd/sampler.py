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


PRIOR_KINDS = {"uniform": 0, "normal": 1, "exponential": 2, "gamma": 3, "beta": 4, "half_cauchy": 5, "beta_prime": 6,
               "exponential_mix": 7, "dirichlet": 8}


@dataclass
class Marginal:
    """One UnivariateMarginal (src/sampler/UnivariateMarginal.cpp:25-101): kind and its
    parameters p = (p0, p1, p2) in the order of BCM3HIP_PRIOR_* (include/bcm3hip.h)."""
    kind: str
    a: float = 0.0
    b: float = 0.0
    mu: float = 0.0
    sigma: float = 1.0
    p: tuple = (0.0, 0.0, 0.0)

    def bounds(self):
        """GetLowerBound / GetUpperBound (UnivariateMarginal.cpp:627-647)."""
        lo = self.a if self.kind == "uniform" else (
            0.0 if self.kind in ("beta", "exponential", "gamma", "half_cauchy", "beta_prime", "dirichlet") else -math.inf)
        hi = self.b if self.kind == "uniform" else (1.0 if self.kind in ("beta", "dirichlet") else math.inf)
        return lo, hi

    def moments(self):
        """EvaluateMean / EvaluateVariance (UnivariateMarginal.cpp:448-540)."""
        p0, p1, p2 = self.p
        k = self.kind
        if k == "dirichlet":
            return self.mu, self.sigma  # set from the whole group by load_prior
        if k == "uniform":
            d = p1 - p0
            return 0.5 * (p1 + p0), (d * d) / 12.0
        if k == "normal":
            return p0, p1 * p1
        if k == "exponential":
            return 1.0 / p0, 1.0 / (p0 * p0)
        if k == "gamma":
            return p0 * p1, p0 * p1 * p1
        if k == "beta":
            apb = p0 + p1
            return p0 / apb, (p0 * p1) / (apb * apb * (apb + 1))
        if k == "half_cauchy":
            return p0, p0 * p0
        if k == "beta_prime":
            mean = p2 * p0 / (p1 - 1) if p1 > 1.0 else p2
            var = (p2 * p2 * p0 * (p0 + p1 - 1.0) / ((p1 - 2) * (p1 - 1) * (p1 - 1))) if p1 > 2.0 else p2 * p2
            return mean, var
        # exponential_mix
        return p2 / p0 + (1.0 - p2) / p1, p2 * p2 / (p0 * p0) + (1.0 - p2) ** 2 / (p1 * p1)


def _marginal(v) -> Marginal:
    """UnivariateMarginal::Initialize (UnivariateMarginal.cpp:25-101) for one <variable>."""
    dist = v.get("distribution")

    def f(k):
        x = v.get(k)
        if x is None:
            raise ValueError(f"Error parsing UnivariateMarginal: no attribute {k}")
        return float(x)

    if dist == "uniform":
        a, b = f("lower"), f("upper")
        if b <= a:
            raise ValueError("Uniform distribution with upper bound less than or equal to lower bound.")
        return Marginal("uniform", a=a, b=b, p=(a, b, 0.0))
    if dist == "normal":
        mu, sigma = f("mu"), f("sigma")
        if sigma <= 0.0:
            raise ValueError("Normal distribution with non-positive sigma.")
        return Marginal("normal", mu=mu, sigma=sigma, p=(mu, sigma, 0.0))
    if dist == "exponential":
        lam = f("lambda")
        if lam <= 0.0:
            raise ValueError("Exponential distribution with non-positive lambda.")
        return Marginal("exponential", p=(lam, 0.0, 0.0))
    if dist == "gamma":
        k, theta = f("k"), f("theta")
        if k <= 0.0 or theta <= 0.0:
            raise ValueError("Gamma distribution with non-positive k or theta.")
        return Marginal("gamma", p=(k, theta, 0.0))
    if dist == "beta":
        a, b = f("a"), f("b")
        if a <= 0.0 or b <= 0.0:
            raise ValueError("Beta distribution with non-positive a or b.")
        return Marginal("beta", p=(a, b, 0.0))
    if dist == "half_cauchy":
        sc = f("scale")
        if sc <= 0.0:
            raise ValueError("Half-Cauchy distribution with non-positive scale.")
        return Marginal("half_cauchy", p=(sc, 0.0, 0.0))
    if dist == "beta_prime":
        return Marginal("beta_prime", p=(f("a"), f("b"), f("scale")))
    if dist == "exponential_mix":
        return Marginal("exponential_mix", p=(f("lambda"), f("lambda2"), f("mix")))
    raise ValueError(f"Invalid distribution type \"{dist}\"")


def load_prior(path: str) -> List[Marginal]:
    """Marginals of a prior.xml in variable order (VariableSet::LoadFromXML repeat rule). Members of a
    multivariate (Dirichlet) group (PriorIndependence.cpp:20-77) become Marginal("dirichlet",
    p=(alpha_i, index of the group's first variable, log normalisation constant)), moments in
    mu / sigma (MultivariateMarginal.cpp:47-158), as csrc/host/Prior.cpp does."""
    root = ET.parse(path).getroot()
    out = []
    groups = {}
    for v in root.iter("variable"):
        if v.get("multivariate", "false").lower() in ("true", "1"):
            if int(v.get("repeat", "1")) > 1:
                raise ValueError("Multivariate prior with repeat not supported")
            gid = int(v.get("id", "0"))
            if gid <= 0:
                raise ValueError("Multivariate distribution IDs should start at 1.")
            if gid not in groups:
                if v.get("distribution") != "dirichlet":
                    raise ValueError("Multivariate distribution of unknown type (only dirichlet supported).")
                groups[gid] = (len(out), [])
            first, alphas = groups[gid]
            if len(out) != first + len(alphas):
                raise ValueError("All variables in a multivariate distribution should follow each other directly")
            alphas.append(float(v.get("alpha")))
            out.append(Marginal("dirichlet", p=(alphas[-1], float(first), 0.0)))
        else:
            out += [_marginal(v)] * int(v.get("repeat", "1"))
    for first, alphas in groups.values():
        s = 0.0
        lprod = 0.0
        for a in alphas:
            s += a
            lprod += math.lgamma(a)
        lnc = math.lgamma(s) - lprod
        for k, a in enumerate(alphas):
            out[first + k] = Marginal("dirichlet", mu=a / s, sigma=a * (s - a) / (s * s * (s + 1.0)),
                                      p=(a, float(first), lnc))
    return out


class DevicePrior:
    """PriorIndependence over the marginals of a prior.xml, as device arrays: kind codes and
    parameters for the kernels, bounds and moments for the proposals."""

    def __init__(self, marginals: List[Marginal], device):
        dev = torch.device(device)
        self.d = len(marginals)
        f64 = dict(dtype=torch.float64, device=dev)
        self.kind_codes = torch.tensor([PRIOR_KINDS[m.kind] for m in marginals], dtype=torch.int32, device=dev)
        self.p0 = torch.tensor([m.p[0] for m in marginals], **f64)
        self.p1 = torch.tensor([m.p[1] for m in marginals], **f64)
        self.p2 = torch.tensor([m.p[2] for m in marginals], **f64)
        self.lower = torch.tensor([m.bounds()[0] for m in marginals], **f64)
        self.upper = torch.tensor([m.bounds()[1] for m in marginals], **f64)
        self.mean = torch.tensor([m.moments()[0] for m in marginals], **f64)
        self.var = torch.tensor([m.moments()[1] for m in marginals], **f64)
        self.simple = all(m.kind in ("uniform", "normal") for m in marginals)
        self.is_uniform = torch.tensor([m.kind == "uniform" for m in marginals], device=dev)
        self.a = torch.tensor([m.a for m in marginals], **f64)
        self.b = torch.tensor([m.b for m in marginals], **f64)
        self.mu = torch.tensor([m.mu for m in marginals], **f64)
        self.sigma = torch.tensor([m.sigma for m in marginals], **f64)
        self.log_uniform = -torch.log(self.b - self.a)
        self.log_norm = torch.log(torch.rsqrt(2.0 * self.sigma * self.sigma * math.pi))
        self.inv2s2 = 1.0 / (2.0 * self.sigma * self.sigma)
        # proposal scale for the random walk: a fixed fraction of the marginal's spread
        self.scale = 0.05 * torch.sqrt(self.var)

    def log_pdf(self, x: torch.Tensor) -> torch.Tensor:
        """Uniform / normal marginals (a host check for tests; the kernels evaluate every type)."""
        inside = (x >= self.a) & (x <= self.b)
        lu = torch.where(inside, self.log_uniform, torch.full_like(x, -math.inf))
        dx = x - self.mu
        ln = self.log_norm - dx * dx * self.inv2s2
        return torch.where(self.is_uniform, lu, ln).sum(dim=1)

    def sample(self, n: int, gen: torch.Generator) -> torch.Tensor:
        """Uniform / normal marginals (test inputs; T = 0 chains draw on the device)."""
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
                 proposal: str = "gaussian_mixture", t_dof: float = 0.0, kmax: Optional[int] = None,
                 adapt_proposal_samples: int = 2000, adapt_proposal_times: int = 2, max_history_size: int = 2000,
                 use_every_nth: int = 1, swapping_scheme: str = "deterministic_even_odd",
                 exchange_probability: float = 0.5, initial_position_tries: int = 100,
                 adapt_proposal_max_history_samples: int = 2000):
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
        self.kind = prior.kind_codes.contiguous()
        self.p0, self.p1, self.p2 = prior.p0.contiguous(), prior.p1.contiguous(), prior.p2.contiguous()
        self.scale = prior.scale.contiguous()
        if proposal == "random_walk" and not prior.simple:
            raise ValueError("the random-walk proposal kernel supports uniform and normal priors only")
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
        # set by the accept kernels on a NaN log-likelihood (Sampler.cpp:172-178: fatal)
        self.nan_llh = torch.zeros(1, dtype=torch.int32, device=dev)
        self.nan_check_every = 100
        self.attempted_mutate = 0
        self.attempted_exchange = 0
        # ptmhsampler.swapping_scheme / exchange_probability (SamplerPT.cpp:63-75, 163-164)
        if swapping_scheme not in ("deterministic_even_odd", "stochastic_even_odd", "stochastic_random"):
            raise ValueError(f"Unknown swapping scheme \"{swapping_scheme}\"")
        self.scheme = swapping_scheme
        self.exchange_probability = float(exchange_probability)
        # proposals (ptmhsampler.proposal_type) and the sample history that adapts them
        # gaussian_mixture_adjustedAIC: the same proposal, selection by adjusted AIC
        # (SamplerPTChain.cpp:433-436)
        self.adjusted_aic = proposal == "gaussian_mixture_adjustedAIC"
        if self.adjusted_aic:
            proposal = "gaussian_mixture"
        self.proposal_type = proposal
        self.adaptive = proposal != "random_walk"
        self.max_history_samples = int(adapt_proposal_max_history_samples)
        if kmax is None:
            kmax = 13 if proposal == "gaussian_mixture" else 1  # GMM candidates 1..13 components
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
        self._initial_positions(initial_position_tries)

    def _initial_positions(self, tries: int):
        """Starting positions (SamplerPTChain::Initialize, SamplerPTChain.cpp:188-214): every chain
        draws from the prior until lprior + T llh > -inf, at most `tries` times. The draws are the
        propose kernel's T = 0 path on counter streams INIT_ITER, INIT_ITER - 1, ..."""
        C, d, dev = self.C, self.d, self.dev
        zeros = torch.zeros(C, dtype=torch.float64, device=dev)
        bad = torch.ones(C, dtype=torch.bool, device=dev)
        self.values.zero_()
        self.lprior.fill_(-math.inf)
        self.llh.fill_(-math.inf)
        for k in range(tries):
            it = self.INIT_ITER - k
            if self.adaptive:
                self._hip.ptmh_propose_adaptive(C, d, self.kind.data_ptr(), self.p0.data_ptr(), self.p1.data_ptr(),
                                                self.p2.data_ptr(), zeros.data_ptr(), self.values.data_ptr(),
                                                self.prop.data_ptr(), self.lprior_prop.data_ptr(),
                                                self.log_mh.data_ptr(), self.proposal.struct, self.g0, self.seed, it,
                                                self._stream())
            else:
                self._hip.ptmh_propose(C, d, self.kind.data_ptr(), self.p0.data_ptr(), self.p1.data_ptr(),
                                       self.scale.data_ptr(), zeros.data_ptr(), self.values.data_ptr(),
                                       self.prop.data_ptr(), self.lprior_prop.data_ptr(), self.g0, self.seed, it,
                                       self._stream())
            self._eval(self.prop, self.llh_prop)
            if bool(torch.isnan(self.llh_prop * self.lr).any()):
                # SamplerPTChain::Initialize -> EvaluatePriorLikelihood fails on NaN (Sampler.cpp:172-178)
                raise RuntimeError("Likelihood evaluation returned NaN while finding starting positions")
            self.values.copy_(torch.where(bad.view(-1, 1), self.prop, self.values))
            self.lprior.copy_(torch.where(bad, self.lprior_prop, self.lprior))
            self.llh.copy_(torch.where(bad, self.llh_prop * self.lr, self.llh))
            bad = ~(self.lprior + self.T * self.llh > -math.inf)
            if not bool(bad.any()):
                break
        if bool(bad.any()):
            raise RuntimeError(f"Could not find starting position with power posterior != inf after {tries} tries")
        self.lpp.copy_(self.ex.lpowerposterior(self.llh, self.lprior))

    def _stream(self):
        return torch.cuda.current_stream(self.dev).cuda_stream

    def _eval(self, x: torch.Tensor, out: torch.Tensor):
        self.ll.evaluate_batch_device(self.C, x.data_ptr(), out.data_ptr(), self.status.data_ptr(), self._stream())

    def exchange(self):
        """DoExchangeMove round (SamplerPT.cpp:277-298): local pairs on the GPU, boundary pairs
        over RCCL point-to-point (sharded_exchange_round)."""
        if self.Ctot < 2:
            return
        start = self.round % 2

        def local_pairs(start_, wrap_local):
            self._hip.pt_exchange_local(self.C, self.d, self.g0, start_, wrap_local, self.T.data_ptr(),
                                        self.values.data_ptr(), self.llh.data_ptr(), self.lprior.data_ptr(),
                                        self.lpp.data_ptr(), None, self.accepted_exchange.data_ptr(), self.seed,
                                        self.round, self._stream())

        self.attempted_exchange += sharded_exchange_round(self.ex, local_pairs, self.values, self.llh, self.lprior,
                                                          self.lpp, self.round, self.accepted_exchange)
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
                                    self.p2.data_ptr(), self.T.data_ptr(), self.values.data_ptr(), self.prop.data_ptr(),
                                    self.lprior_prop.data_ptr(), self.log_mh.data_ptr(), P, self.g0, self.seed,
                                    self.iter, st)
            self._eval(self.prop, self.llh_prop)
            h.ptmh_accept_adaptive(C, d, self.T.data_ptr(), self.prop.data_ptr(), self.lprior_prop.data_ptr(),
                                   self.llh_prop.data_ptr(), self.log_mh.data_ptr(), self.lr, self.values.data_ptr(),
                                   self.lprior.data_ptr(), self.llh.data_ptr(), self.lpp.data_ptr(), None,
                                   self.accepted_mutate.data_ptr(), P, self.g0, self.seed, self.iter, st,
                                   nan_llh=self.nan_llh.data_ptr())
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
                      self.seed, self.iter, st, nan_llh=self.nan_llh.data_ptr())
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

    def check_nan(self) -> bool:
        """Raise if any likelihood evaluation since the start returned NaN (the accept kernels set
        the flag; Sampler::EvaluateLikelihood stops the sampler, Sampler.cpp:172-178). One host
        synchronisation; run() calls it every nan_check_every iterations and at the end."""
        if int(self.nan_llh.item()) != 0:
            raise RuntimeError("Likelihood evaluation returned NaN (Sampler::EvaluateLikelihood, fatal)")
        return False

    def adapt_proposal(self):
        """SamplerPTChain::AdaptProposal for every chain of the rank (T == 0 chains excepted)."""
        self.check_nan()
        self.proposal.adapt(self.history.samples, self.history.counters, seed=self.seed,
                            adaptation=self.adaptations_done, chain0=self.g0,
                            max_history_samples=self.max_history_samples, adjusted_aic=self.adjusted_aic)
        # SamplerPTChain::AdaptProposal discards the history it adapted on (SampleHistory::Reset,
        # SamplerPTChain.cpp:174-177 / SampleHistory.cpp:27-31)
        self.history.counters.zero_()
        self.adaptations_done += 1

    def run(self, num_samples: int):
        """SamplerPT::Run's loop over num_samples * use_every_nth iterations."""
        total = num_samples * self.use_every_nth
        for si in range(total):
            self.iteration(last=(si + 1 == total))
            if (si + 1) % self.nan_check_every == 0:
                self.check_nan()
        self.check_nan()

def sharded_exchange_round(ex: PTExchange, local_pairs, values, llh, lprior, lpp, rnd: int,
                           accepted: torch.Tensor) -> int:
    """One even/odd exchange round of a rank's ladder slice (SamplerPT::DoExchangeMove,
    SamplerPT.cpp:277-298): local_pairs(start, wrap_local) swaps the pairs inside the slice (the
    HIP kernel in PTMHDevice), then -- on ranks whose last chain starts a pair this round, which
    with an even slice size is every rank or none -- the two slice-boundary pairs go over
    point-to-point send/recv with the neighbours (PTExchange._cross; RCCL over xGMI, gloo in the
    CPU tests). Returns the number of pairs this rank attempted (pairs counted on the rank of
    their first chain); accepted += the accepted ones of the cross pair."""
    C, Ctot, world = ex.C, ex.Ctot, ex.world
    g0 = ex.rank * C
    start = rnd % 2
    wrap_local = world == 1 and (Ctot - 1 - start) % 2 == 0
    local_pairs(start, wrap_local)
    attempted = sum(1 for i in range(C - 1) if (g0 + i - start) % 2 == 0) + int(wrap_local)
    if world > 1 and (g0 + C - 1 - start) % 2 == 0:
        acc = torch.zeros(C, dtype=torch.bool, device=values.device)
        ex.round = rnd
        ex._cross(values, llh, lprior, lpp, acc)
        accepted += acc[C - 1:].to(torch.int64)
        attempted += 1
    return attempted


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
