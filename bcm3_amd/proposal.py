"""Adaptive MCMC proposals with their state in HBM (one_block blocking).

Host side of bcm3_amd/csrc/proposal_kernels.hip (include/bcm3hip.h: bcm3hip_proposal). Restates
for the device sampler:

* the proposal state a chain's Proposal object holds -- ProposalGlobalCovariance
  (src/sampler/ProposalGlobalCovariance.cpp) and ProposalGaussianMixture
  (src/sampler/ProposalGaussianMixture.cpp) with the base Proposal (src/sampler/Proposal.cpp):
  Cholesky factors, log normalisers, adaptive scales and acceptance-rate EMAs per chain;
* Proposal::Initialize / InitializeImpl (Proposal.cpp:33-140, ProposalGlobalCovariance.cpp:64-104,
  ProposalGaussianMixture.cpp:125-254) -- the infrequent adaptation step, on the host in C++
  (libbcm3.so bcm3_adapt_proposals, csrc/host/GMM.cpp: history thinning, effective sample size,
  GMM fits with 1, 2, 3, 4, 5, 8, 13 components by k-means++ + EM, AIC selection), one host thread
  per core like the reference's per-chain adaptation tasks, then uploaded to HBM;
* SampleHistory (src/sampler/SampleHistory.cpp) as a per-chain float ring buffer in HBM.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import numpy as np
import torch

from . import _hip

KINDS = {"global_covariance": _hip.PROPOSAL_GLOBAL_COVARIANCE, "gaussian_mixture": _hip.PROPOSAL_GAUSSIAN_MIXTURE}


def target_acceptance_rate(d: int) -> float:
    """Proposal::Initialize (Proposal.cpp:45-53)."""
    return {1: 0.44, 2: 0.35, 3: 0.3}.get(d, 0.234)


def log_normaliser(chol: torch.Tensor) -> torch.Tensor:
    """-sum_j log L_jj - d/2 log(2 pi) over the last two dims (ProposalGlobalCovariance.cpp:96-101,
    GMM::Set), summed in j order on the host with the C library's log -- the arithmetic of the C++
    host code (csrc/host/GMM.cpp, SamplerPTDevice.cpp), so both samplers start from the same bits."""
    d = chol.shape[-1]
    diag = torch.diagonal(chol, dim1=-2, dim2=-1).detach().to("cpu").numpy().reshape(-1, d)
    c2 = 0.5 * d * math.log(2.0 * math.pi)
    cache = {}
    out = np.empty(len(diag))
    for i, row in enumerate(diag):
        key = row.tobytes()
        if key not in cache:
            det = 0.0
            for v in row.tolist():
                det += math.log(v)
            cache[key] = -det - c2
        out[i] = cache[key]
    return torch.tensor(out.reshape(chol.shape[:-2]), dtype=torch.float64, device=chol.device)


class DeviceProposal:
    """Per-chain proposal state of C chains (rank-local) for d variables."""

    def __init__(self, kind: str, prior, temps: torch.Tensor, kmax: int = 1, t_dof: float = 0.0):
        if kind not in KINDS:
            raise ValueError(f"Unknown proposal type \"{kind}\"")
        if not 1 <= kmax <= _hip.PROPOSAL_KMAX:
            raise ValueError(f"kmax must be in 1..{_hip.PROPOSAL_KMAX}")
        if kind == "global_covariance":
            kmax = 1
        dev = temps.device
        self.kind, self.kmax, self.t_dof = kind, int(kmax), float(t_dof)
        self.C, self.d = int(temps.numel()), prior.d
        self.temps = temps
        C, d, K = self.C, self.d, self.kmax
        f64 = dict(dtype=torch.float64, device=dev)
        # Prior::GetLowerBound / GetUpperBound (UnivariateMarginal.cpp:627-647)
        self.lower = prior.lower.to(**f64).contiguous()
        self.upper = prior.upper.to(**f64).contiguous()
        # EvaluateMarginalMean / Variance (UnivariateMarginal.cpp:448-540)
        self.prior_mean = prior.mean.to(**f64)
        self.prior_var = prior.var.to(**f64)
        self.target = target_acceptance_rate(d)
        self.ncomp = torch.ones(C, dtype=torch.int32, device=dev)
        self.weights = torch.zeros((C, K), **f64)
        self.mean = torch.zeros((C, K, d), **f64)
        self.chol = torch.zeros((C, K, d, d), **f64)
        self.logc = torch.zeros((C, K), **f64)
        self.scale = torch.zeros((C, K), **f64)
        self.ema = torch.zeros((C, K), **f64)
        self.selected = torch.full((C,), -1, dtype=torch.int32, device=dev)
        self.work = torch.zeros((C, 2 * K + 2 * d), **f64)
        self.reset_from_prior(torch.ones(C, dtype=torch.bool, device=dev))
        self.struct = _hip.Proposal(
            kind=KINDS[kind], kmax=K, t_dof=self.t_dof, target_acceptance=self.target,
            scaling_learning_rate=0.05, scaling_ema_period=1000.0,
            lower=self.lower.data_ptr(), upper=self.upper.data_ptr(), ncomp=self.ncomp.data_ptr(),
            weights=self.weights.data_ptr(), mean=self.mean.data_ptr(), chol=self.chol.data_ptr(),
            logc=self.logc.data_ptr(), scale=self.scale.data_ptr(), ema=self.ema.data_ptr(),
            selected=self.selected.data_ptr(), work=self.work.data_ptr())

    # ---- InitializeImpl without usable history: a single Gaussian from the prior's moments
    def reset_from_prior(self, chains: torch.Tensor):
        d = self.d
        L = torch.diag_embed(torch.sqrt(self.prior_var))  # llt of a diagonal matrix
        self._set_single(chains, self.prior_mean.expand(self.C, d), L.expand(self.C, d, d))
        self._reset_scales(chains, initial=True)

    def _set_single(self, chains, mean, L):
        m = chains.view(-1, 1)
        self.ncomp.copy_(torch.where(chains, torch.ones_like(self.ncomp), self.ncomp))
        w = torch.zeros_like(self.weights)
        w[:, 0] = 1.0
        self.weights.copy_(torch.where(m, w, self.weights))
        newmean = torch.zeros_like(self.mean)
        newmean[:, 0] = mean
        self.mean.copy_(torch.where(m.view(-1, 1, 1), newmean, self.mean))
        newchol = torch.zeros_like(self.chol)
        newchol[:, 0] = L
        # unused slots keep an identity factor so that no kernel path can divide by zero
        for k in range(1, self.kmax):
            newchol[:, k] = torch.eye(self.d, dtype=torch.float64, device=self.chol.device)
        self.chol.copy_(torch.where(m.view(-1, 1, 1, 1), newchol, self.chol))
        self.logc.copy_(torch.where(m, log_normaliser(self.chol), self.logc))

    def _reset_scales(self, chains, initial: bool):
        """A freshly constructed proposal's scale state: every adaptation builds a new Proposal
        object (SamplerPTChain::CreateProposalInstance, SamplerPTChain.cpp:428-462)."""
        m = chains.view(-1, 1)
        if self.kind == "gaussian_mixture":
            # ProposalGaussianMixture::InitializeImpl (:250-251)
            s = torch.full_like(self.scale, 2.38 / math.sqrt(self.d))
            e = torch.full_like(self.ema, self.target)
        elif initial:
            # Proposal() constructor (Proposal.cpp:26-29): adaptive_scale 1, acceptance EMA 0.23
            s = torch.ones_like(self.scale)
            e = torch.full_like(self.ema, 0.23)
        else:
            return
        self.scale.copy_(torch.where(m, s, self.scale))
        self.ema.copy_(torch.where(m, e, self.ema))
        # selected_component = -1 in the constructor (ProposalGaussianMixture.cpp:10-14)
        stale = (self.selected >= self.ncomp) if not initial else torch.ones_like(chains)
        self.selected.copy_(torch.where(chains & stale, torch.full_like(self.selected, -1), self.selected))

    def set_mixture(self, chain: int, weights, means, covariances):
        """Load a fitted mixture for one chain (ProposalGaussianMixture after GMM::Set)."""
        if self.kind != "gaussian_mixture":
            raise ValueError("set_mixture needs a gaussian_mixture proposal")
        w = torch.as_tensor(weights, dtype=torch.float64, device=self.chol.device)
        K = int(w.numel())
        if not 1 <= K <= self.kmax:
            raise ValueError(f"{K} components do not fit kmax={self.kmax}")
        mu = torch.as_tensor(means, dtype=torch.float64, device=self.chol.device).reshape(K, self.d)
        cov = torch.as_tensor(covariances, dtype=torch.float64, device=self.chol.device).reshape(K, self.d, self.d)
        L, info = torch.linalg.cholesky_ex(cov)
        if bool((info != 0).any()):
            raise ValueError("component covariance is not positive definite")
        self.ncomp[chain] = K
        self.weights[chain].zero_()
        self.weights[chain, :K] = w
        self.mean[chain].zero_()
        self.mean[chain, :K] = mu
        eye = torch.eye(self.d, dtype=torch.float64, device=self.chol.device)
        self.chol[chain] = eye
        self.chol[chain, :K] = L
        self.logc[chain] = log_normaliser(self.chol[chain])
        self.scale[chain] = 2.38 / math.sqrt(self.d)
        self.ema[chain] = self.target
        self.selected[chain] = -1

    # ---- Proposal::Initialize from the sample history (AdaptProposal, SamplerPTChain.cpp:120-200)
    def adapt(self, history: torch.Tensor, counters: torch.Tensor, seed: int = 0, adaptation: int = 0,
              chain0: int = 0, max_history_samples: int = 2000, adjusted_aic: bool = False,
              nthreads: Optional[int] = None):
        """history [C][H][d] float32 ring, counters [C][2] (bcm3hip_history_add). Chains at T == 0
        are not adapted (SamplerPTChain::AdaptProposal returns early); every other chain gets a
        freshly initialised proposal, as AdaptProposal creates a new Proposal object
        (SamplerPTChain.cpp:143-152, 428-462): fitted state, default scales and EMAs, no selected
        component. The fit runs in C++ on the host (bcm3_adapt_proposals)."""
        from .likelihood import lib as host_lib
        C, H, d = history.shape
        K = self.kmax
        hist = np.ascontiguousarray(history.detach().to("cpu").numpy(), dtype=np.float32)
        counts = np.ascontiguousarray(counters[:, 0].detach().to("cpu").numpy(), dtype=np.int64)
        active = np.ascontiguousarray((self.temps != 0.0).to("cpu").numpy(), dtype=np.uint8)
        pm = np.ascontiguousarray(self.prior_mean.to("cpu").numpy(), dtype=np.float64)
        pv = np.ascontiguousarray(self.prior_var.to("cpu").numpy(), dtype=np.float64)
        ncomp = np.zeros(C, dtype=np.int32)
        fitted = np.zeros(C, dtype=np.int32)
        w = np.zeros((C, K))
        mu = np.zeros((C, K, d))
        L = np.zeros((C, K, d, d))
        lc = np.zeros((C, K))
        if nthreads is None:
            nthreads = max(1, min(16, len(os.sched_getaffinity(0))))
        kind = 1 if self.kind == "gaussian_mixture" else 0
        rc = host_lib().bcm3_adapt_proposals(kind, int(adjusted_aic), C, H, d, K, hist.ctypes.data, counts.ctypes.data,
                                             active.ctypes.data, int(max_history_samples), pm.ctypes.data,
                                             pv.ctypes.data, int(seed) & ((1 << 64) - 1), int(adaptation),
                                             int(chain0), int(nthreads), ncomp.ctypes.data, w.ctypes.data,
                                             mu.ctypes.data, L.ctypes.data, lc.ctypes.data, fitted.ctypes.data)
        if rc != 0:
            msg = host_lib().bcm3_last_error()
            raise RuntimeError(f"proposal adaptation failed: {msg.decode() if msg else rc}")
        dev = self.chol.device
        act = torch.from_numpy(active.astype(bool)).to(dev)
        m = act.view(-1, 1)
        self.ncomp.copy_(torch.where(act, torch.from_numpy(ncomp).to(dev), self.ncomp))
        self.weights.copy_(torch.where(m, torch.from_numpy(w).to(dev), self.weights))
        self.mean.copy_(torch.where(m.view(-1, 1, 1), torch.from_numpy(mu).to(dev), self.mean))
        self.chol.copy_(torch.where(m.view(-1, 1, 1, 1), torch.from_numpy(L).to(dev), self.chol))
        self.logc.copy_(torch.where(m, torch.from_numpy(lc).to(dev), self.logc))
        self._reset_scales(act, initial=True)
        self.last_fitted = fitted

    def adapt_torch_single(self, history: torch.Tensor, counters: torch.Tensor):
        """Round-1 device-side adaptation (one Gaussian from the history's mean and covariance);
        kept for comparison only -- adapt() is the reference's algorithm."""
        C, H, d = history.shape
        n = torch.clamp(counters[:, 0], max=H)
        active = self.temps != 0.0
        fit = active & (n >= 2)
        if bool(fit.any()):
            idx = torch.arange(H, device=history.device).view(1, H, 1)
            valid = (idx < n.view(C, 1, 1)).to(torch.float64)
            x = history.to(torch.float64) * valid
            cnt = n.to(torch.float64).clamp(min=2.0).view(C, 1)
            mean = x.sum(dim=1) / cnt
            xc = (history.to(torch.float64) - mean.view(C, 1, d)) * valid
            cov = xc.transpose(1, 2) @ xc / (cnt.view(C, 1, 1) - 1.0)
            # diagonal at least 1e-6 of the prior variance (ProposalGlobalCovariance.cpp:83-87)
            diag = torch.diagonal(cov, dim1=-2, dim2=-1)
            floor = 1e-6 * self.prior_var
            cov = cov + torch.diag_embed(torch.clamp(floor - diag, min=0.0))
            L, info = torch.linalg.cholesky_ex(cov)
            ok = fit & (info == 0)
            # (global_covariance never reads the mean: its random walk is symmetric)
            self._set_single(ok, mean, torch.where(ok.view(C, 1, 1), L, self.chol[:, 0]))
            fit = ok
        # chains without a usable history (or a failed factorisation) restart from the prior
        rest = active & ~fit
        if bool(rest.any()):
            L = torch.diag_embed(torch.sqrt(self.prior_var))
            self._set_single(rest, self.prior_mean.expand(C, d), L.expand(C, d, d))
        self._reset_scales(active, initial=False)


class SampleHistory:
    """Per-chain float ring buffer in HBM (SampleHistory.cpp:14-45)."""

    def __init__(self, C: int, d: int, size: int, subsampling: int, device):
        self.C, self.d, self.H, self.sub = C, d, int(size), int(subsampling)
        self.samples = torch.zeros((C, self.H, d), dtype=torch.float32, device=device)
        self.counters = torch.zeros((C, 2), dtype=torch.int64, device=device)

    def add(self, temps: torch.Tensor, values: torch.Tensor, mask: Optional[torch.Tensor] = None, stream=None):
        _hip.history_add(self.C, self.d, self.H, self.sub, temps.data_ptr(), values.data_ptr(),
                         None if mask is None else mask.data_ptr(), self.samples.data_ptr(),
                         self.counters.data_ptr(), stream)


def history_geometry(adapt_proposal_samples: int, use_every_nth: int, exploration_steps: int, num_chains: int,
                     max_history_size: int, deterministic: bool = True):
    """History size and subsampling (SamplerPT::Initialize, SamplerPT.cpp:113-123)."""
    expected = adapt_proposal_samples * use_every_nth
    if num_chains > 1 and deterministic:
        expected *= exploration_steps + 1
    sub = 1
    size = expected
    if size > max_history_size:
        sub = (expected + max_history_size - 1) // max_history_size
        size = expected // sub
    return max(size, 1), sub
