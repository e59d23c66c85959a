"""gmm_oracle.py -- TEST INFRASTRUCTURE (the parity oracle of the proposal adaptation). Never
imported by the product.

numpy restatement of the reference's proposal adaptation, the checker for the C++ host code
(bcm3_amd/csrc/host/GMM.cpp, libbcm3.so bcm3_adapt_proposals):

* bcm3::GMM (src/stats/GMM.cpp): Set :14-45, Fit :48-158, LogPdf :160-170,
  CalculateResponsibilities :172-186, KMeanspp :188-245, CalculateMeanCovariance :247-337,
  EM_maximization :339-345, EM_expectation :347-390;
* Proposal::Initialize's history thinning (src/sampler/Proposal.cpp:92-121);
* ProposalGaussianMixture::InitializeImpl (src/sampler/ProposalGaussianMixture.cpp:125-254) with
  mean / var / acf of src/utils/SummaryStats.cpp;
* ProposalGlobalCovariance::InitializeImpl (src/sampler/ProposalGlobalCovariance.cpp:64-104) with
  cov() (SummaryStats.cpp:195-240).

Random numbers: the counter-based stream of GMM.cpp's CtrRng (splitmix64 of (seed, key, n)),
reproduced exactly, so k-means++ picks the same samples. Sums and the eigendecomposition use
numpy (closed-form weighted moments, LAPACK eigh), so the checker agrees with the C++ code to
rounding, not bit for bit. Pinned against the reference's own golden values
(tests/stats/GMM.cpp:4-31, tests/stats/mvn.cpp:17-44) by tests/test_gmm.py.
"""
from __future__ import annotations

import math

import numpy as np
from scipy.linalg import solve_triangular

M64 = (1 << 64) - 1
DBL_EPSILON = np.finfo(np.float64).eps


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & M64
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


class CtrRng:
    """GMM.cpp CtrRng."""

    def __init__(self, seed: int, key: int):
        self.base = splitmix64(splitmix64(seed & M64) ^ ((key * 0xC2B2AE3D27D4EB4F) & M64))
        self.n = 0

    def next(self) -> int:
        self.n += 1
        return splitmix64(self.base ^ ((self.n * 0x100000001B3) & M64))

    def real(self) -> float:
        return (self.next() >> 11) * (1.0 / 9007199254740992.0)

    def uint(self, mx: int) -> int:
        return min(int(self.real() * (mx + 1)), mx)

    def sample(self, probs) -> int:
        t = self.real()
        p = 0.0
        for i, q in enumerate(probs):
            p += q
            if t < p:
                return i
        return len(probs) - 1


def chain_key(chain: int, adaptation: int) -> int:
    return ((chain << 20) & M64) ^ adaptation


def logsum2(a, b):
    """MathFunctions.h:67-82, elementwise."""
    a, b = np.maximum(a, b), np.minimum(a, b)
    with np.errstate(invalid="ignore", over="ignore"):
        out = a + np.log1p(np.exp(b - a))
    out = np.where(b - a < -500, a, out)
    return np.where(a == -np.inf, a, out)


def chol(cov):
    try:
        return np.linalg.cholesky(cov)
    except np.linalg.LinAlgError:
        return None


def log_normaliser(L):
    return -np.sum(np.log(np.diag(L))) - 0.5 * L.shape[0] * math.log(2.0 * math.pi)


class GMM:
    def set(self, means, covs, weights):
        self.means = [np.asarray(m, dtype=np.float64) for m in means]
        self.covs = [np.asarray(c, dtype=np.float64) for c in covs]
        self.L = [chol(c) for c in self.covs]
        if any(L is None for L in self.L):
            return False
        self.logC = [log_normaliser(L) for L in self.L]
        self.weights = np.asarray(weights, dtype=np.float64)
        return True

    def _comp_logp(self, X, k):
        v = solve_triangular(self.L[k], (np.atleast_2d(X) - self.means[k]).T, lower=True)
        return self.logC[k] - 0.5 * np.sum(v * v, axis=0)

    def log_pdf(self, x):
        lp = -np.inf
        for k in range(len(self.means)):
            lp = logsum2(lp, self._comp_logp(x, k)[0] + math.log(self.weights[k]))
        return float(lp)

    def responsibilities(self, x):
        p = np.array([self._comp_logp(x, k)[0] + math.log(self.weights[k]) for k in range(len(self.means))])
        m = p.max()
        lsum = math.log(np.sum(np.exp(p - m))) + m
        e = np.exp(p - lsum)
        return e / e.sum()

    # GMM.cpp:247-337
    @staticmethod
    def mean_cov(X, w, ess_factor):
        D = X.shape[1]
        sel = w >= DBL_EPSILON
        ws, Xs = w[sel], X[sel]
        wsum = ws.sum()
        mean = (ws[:, None] * Xs).sum(axis=0) / wsum if wsum > 0 else np.zeros(D)
        if wsum < 2.0:
            return mean, np.eye(D)
        dx = Xs - mean
        cov = (ws[:, None] * dx).T @ dx / (wsum - 1)
        n_eff = wsum / ess_factor
        if n_eff < 2:
            return mean, np.diag(np.diag(cov))
        n_eff = max(n_eff, float(D))
        sd = np.sqrt(np.diag(cov))
        corr = cov / np.outer(sd, sd)
        ev, V = np.linalg.eigh(corr)  # ascending
        m = len(ev)
        ne = int(math.floor(n_eff))
        for i in range(m):
            if ne < m and i >= ne:
                ev[m - 1 - i] = 0.0
            else:
                ev[m - 1 - i] *= n_eff / (n_eff + D + 1 - 2.0 * i)
        corr = (V * ev) @ V.T
        cov = sd[:, None] * corr * sd[None, :]
        cov[np.diag_indices(D)] += 1e-8
        return mean, cov

    def kmeanspp(self, X, K, rng):
        n, D = X.shape
        ix = rng.uint(n - 1)
        centers = [X[ix].copy()]
        used = {ix}
        for _ in range(1, K):
            d2 = np.min([np.sum((X - c) ** 2, axis=1) for c in centers], axis=0)
            d2[list(used)] = 0.0
            p = d2 / d2.sum()
            nix = rng.sample(p)
            centers.append(X[nix].copy())
            used.add(nix)
        dist = np.stack([np.sum((X - c) ** 2, axis=1) for c in centers], axis=1)
        resp = np.zeros((n, K))
        resp[np.arange(n), np.argmin(dist, axis=1)] = 1.0
        return resp

    def e_step(self, X):
        n = X.shape[0]
        K = len(self.means)
        resp = np.zeros((n, K))
        slog = np.full(n, -np.inf)
        for k in range(K):
            L = chol(self.covs[k])
            if L is None:
                return None, None
            self.L[k] = L
            self.logC[k] = log_normaliser(L)
            p = self._comp_logp(X, k) + math.log(self.weights[k])
            resp[:, k] = np.exp(p)
            slog = logsum2(slog, p)
        tot = resp.sum(axis=1)
        resp = np.where(tot[:, None] == 0, 1.0 / K, resp / np.where(tot == 0, 1.0, tot)[:, None])
        return resp, float(slog.sum())

    def fit(self, X, K, rng, ess_factor):
        n, D = X.shape
        singular = False
        logl = -np.inf
        if K == 1:
            m, c = self.mean_cov(X, np.ones(n), ess_factor)
            if not self.set([m], [c], [1.0]):
                return False
            logl = float(np.sum(self._comp_logp(X, 0)))
        else:
            if n < 2.0 * D * K:
                return False
            for _ in range(4):
                singular = converged = False
                resp = self.kmeanspp(X, K, rng)
                mc = [self.mean_cov(X, resp[:, k], ess_factor) for k in range(K)]
                self.means = [a for a, _ in mc]
                self.covs = [b for _, b in mc]
                self.L = [None] * K
                self.logC = [0.0] * K
                self.weights = np.full(K, 1.0 / K)
                prev = -np.inf
                for _ in range(100):
                    r, ll = self.e_step(X)
                    if r is None:
                        singular = True
                        break
                    resp, logl = r, ll
                    if logl < prev:
                        converged = prev - logl < abs(logl * 1e-5 * 10)
                        break
                    elif logl - prev < abs(logl * 1e-5):
                        converged = True
                        break
                    prev = logl
                    self.weights = resp.sum(axis=0) / n
                    mc = [self.mean_cov(X, resp[:, k], ess_factor) for k in range(K)]
                    self.means = [a for a, _ in mc]
                    self.covs = [b for _, b in mc]
                if converged:
                    break
        nparam = K * (D + D * (D + 1) // 2) + K - 1
        self.logl = logl
        self.aic = 2.0 * nparam - 2.0 * logl
        return not singular


def thin_history(h, max_samples, rng):
    """Proposal.cpp:92-121."""
    rows = h.shape[0]
    if rows <= max_samples:
        return h
    sub = rows // max_samples
    use = [i * sub for i in range(rows // sub)] if sub > 1 else list(range(rows))
    while len(use) > max_samples:
        del use[rng.uint(len(use) - 1)]
    return h[use]


def _mean(x):
    mu = 0.0
    for i, v in enumerate(x):
        mu += (v - mu) / (i + 1)
    return mu


def _var(x, mu):
    s = 0.0
    for i, v in enumerate(x):
        d = v - mu
        s += (d * d - s) / (i + 1)
    n = len(x)
    return s * (n / (n - 1.0))


def _acf(x, lag, mu, s2):
    r = 0.0
    for i in range(len(x) - lag):
        r += ((x[i] - mu) * (x[i + lag] - mu) - r) / (i + 1)
    return r / s2


def fit_gaussian_mixture(h, rng, prior_mean, prior_var, adjusted=False, kmax=13):
    """ProposalGaussianMixture::InitializeImpl; returns (GMM, fitted)."""
    n, D = h.shape
    best, have = GMM(), False
    if n >= 2:
        ess = []
        for i in range(D):
            col = h[:, i]
            mu = _mean(col)
            s2 = _var(col, mu)
            lag_max = max(5, int(10 * math.log10(n)))
            rho = sum(_acf(col, lag, mu, s2) for lag in range(1, lag_max))
            ess.append(n / (1.0 + 2.0 * rho))
        min_ess = min(ess)
        adj = min_ess / n
        best_aic = math.inf
        for K in (1, 2, 3, 4, 5, 8, 13):
            if K > kmax:
                break
            if min_ess < K * (1 + min(D // 2, 10)):
                continue
            g = GMM()
            if not g.fit(h, K, rng, n / min_ess):
                continue
            nparam = 0.5 * g.aic + g.logl
            adjusted_aic = 2.0 * nparam - 2.0 * adj * g.logl
            if (adjusted_aic < best_aic) if adjusted else (g.aic < best_aic):
                best, have, best_aic = g, True, g.aic
    if not have:
        best.set([np.asarray(prior_mean, dtype=np.float64)], [np.diag(np.asarray(prior_var, dtype=np.float64))], [1.0])
    return best, have


def fit_global_covariance(h, prior_var):
    """ProposalGlobalCovariance::InitializeImpl (cov() with ddof 1, diagonal floor)."""
    n, D = h.shape
    if n < 2:
        c = np.diag(np.asarray(prior_var, dtype=np.float64))
    else:
        c = np.cov(h, rowvar=False, ddof=1).reshape(D, D)
        idx = np.diag_indices(D)
        c[idx] = np.maximum(c[idx], 1e-6 * np.asarray(prior_var))
    g = GMM()
    g.set([np.zeros(D)], [c], [1.0])
    return g, n >= 2
