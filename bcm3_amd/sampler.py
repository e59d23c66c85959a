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

The reference evaluates the C chains' likelihoods one per task-manager thread; here all C
proposals go to the GPU in one bcm3_likelihood_evaluate_batch_device launch. The proposal is a
fixed diagonal Gaussian random walk (the reference's adaptive proposals, src/sampler/Proposal*.cpp,
are outside the hot-path scope; SURVEY.md §8 f).
"""
from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from dataclasses import dataclass
from typing import List, Optional

import torch

from .pt import PTExchange


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
    """C chains of one rank: state tensors in HBM, one batched likelihood launch per mutate."""

    def __init__(self, likelihood, prior: DevicePrior, temperatures, rank=0, world=1, seed=0, device="cuda",
                 learning_rate: float = 1.0, exploration_steps: int = 1):
        self.ll, self.prior = likelihood, prior
        self.dev = torch.device(device)
        self.ex = PTExchange(temperatures, rank=rank, world=world, seed=seed, device=self.dev)
        self.C, self.d = self.ex.C, prior.d
        self.T = self.ex.T
        self.lr = learning_rate
        self.exploration_steps = exploration_steps
        self.gen = torch.Generator(device=self.dev)
        self.gen.manual_seed(seed * 1000003 + rank)
        self.values = prior.sample(self.C, self.gen)
        self.lprior = prior.log_pdf(self.values)
        self.llh = self._eval(self.values)
        self.lpp = self.ex.lpowerposterior(self.llh, self.lprior)
        self.status = torch.zeros(self.C, dtype=torch.int32, device=self.dev)
        self.attempted_mutate = 0
        self.accepted_mutate = torch.zeros((), dtype=torch.int64, device=self.dev)

    def _eval(self, x: torch.Tensor) -> torch.Tensor:
        x = x.contiguous()
        out = torch.empty(x.shape[0], dtype=torch.float64, device=self.dev)
        status = torch.empty(x.shape[0], dtype=torch.int32, device=self.dev)
        stream = torch.cuda.current_stream(self.dev).cuda_stream if self.dev.type == "cuda" else None
        self.ll.evaluate_batch_device(x.shape[0], x.data_ptr(), out.data_ptr(), status.data_ptr(), stream)
        return out * self.lr if self.lr != 1.0 else out

    def mutate(self):
        C = self.C
        t0 = self.T == 0.0
        step = torch.randn((C, self.d), dtype=torch.float64, device=self.dev, generator=self.gen) * self.prior.scale
        prop = torch.where(t0[:, None], self.prior.sample(C, self.gen), self.values + step)
        new_lprior = self.prior.log_pdf(prop)
        new_llh = self._eval(prop)
        # T == 0: lpp = lprior (also when llh == -inf, .cpp:231-237); T > 0: lprior + T * llh (.cpp:284)
        new_lpp = torch.where(t0, new_lprior, new_lprior + self.T * new_llh)
        u = torch.rand(C, dtype=torch.float64, device=self.dev, generator=self.gen)
        tp = torch.clamp(torch.exp(new_lpp - self.lpp), max=1.0)
        accept = t0 | ((new_lpp > -math.inf) & (u < tp))
        self.values = torch.where(accept[:, None], prop, self.values)
        self.lprior = torch.where(accept, new_lprior, self.lprior)
        self.llh = torch.where(accept, new_llh, self.llh)
        self.lpp = torch.where(accept, new_lpp, self.lpp)
        self.attempted_mutate += C
        self.accepted_mutate += accept.sum()

    def iteration(self):
        """One DeterministicEvenOdd iteration (SamplerPT.cpp:203-212)."""
        if self.ex.Ctot > 1:
            self.ex.step(self.values, self.llh, self.lprior, self.lpp)
        for _ in range(self.exploration_steps):
            self.mutate()
