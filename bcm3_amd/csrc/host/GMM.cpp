// GMM.cpp -- see GMM.h. Every function cites the reference code it restates.
#include "GMM.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <limits>
#include <set>

namespace bcm3 {

static const Real kInf = std::numeric_limits<Real>::infinity();

// ---------------------------------------------------------------------------------------------
// random numbers

static uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

CtrRng::CtrRng(uint64_t seed, uint64_t key) : base_(splitmix64(splitmix64(seed) ^ (key * 0xC2B2AE3D27D4EB4Full))), n_(0) {}

uint64_t CtrRng::Next() { return splitmix64(base_ ^ (++n_ * 0x100000001B3ull)); }

Real CtrRng::GetReal() { return (Real)(Next() >> 11) * (1.0 / 9007199254740992.0); }

unsigned CtrRng::GetUnsignedInt(unsigned max)
{
    const uint64_t span = (uint64_t)max + 1;
    return (unsigned)std::min<uint64_t>((uint64_t)(GetReal() * (Real)span), (uint64_t)max);
}

unsigned CtrRng::Sample(const std::vector<Real>& probabilities)
{
    // RNG::Sample (src/utils/RNG.cpp:41-56)
    if (probabilities.empty()) return (unsigned)-1;
    const Real t = GetReal();
    Real p = 0.0;
    for (size_t i = 0; i < probabilities.size(); i++) {
        p += probabilities[i];
        if (t < p) return (unsigned)i;
    }
    return (unsigned)probabilities.size() - 1;
}

// ---------------------------------------------------------------------------------------------
// linear algebra

bool Cholesky(const Mat& A, Mat& L)
{
    const int n = A.rows;
    L = Mat(n, n, 0.0);
    for (int j = 0; j < n; j++) {
        Real s = A(j, j);
        for (int k = 0; k < j; k++) s -= L(j, k) * L(j, k);
        if (!(s > 0.0)) return false;  // NaN or non-positive pivot: not positive definite
        const Real ljj = std::sqrt(s);
        L(j, j) = ljj;
        for (int i = j + 1; i < n; i++) {
            Real t = A(i, j);
            for (int k = 0; k < j; k++) t -= L(i, k) * L(j, k);
            L(i, j) = t / ljj;
        }
    }
    return true;
}

// L v = x in place (LLT::matrixL().solveInPlace): forward substitution
static void LowerSolve(const Mat& L, Real* v)
{
    const int n = L.rows;
    for (int i = 0; i < n; i++) {
        Real acc = 0.0;
        for (int j = 0; j < i; j++) acc += L(i, j) * v[j];
        v[i] = (v[i] - acc) / L(i, i);
    }
}

static Real Dot(const Real* a, const Real* b, int n)
{
    Real s = 0.0;
    for (int i = 0; i < n; i++) s += a[i] * b[i];
    return s;
}

// Householder reduction to tridiagonal form followed by the implicit QL iteration (the classic
// tred2 / tql2 pair); eigenvalues ascending, eigenvectors in the columns of V
void SymmetricEigen(const Mat& A, std::vector<Real>& d, Mat& V)
{
    const int n = A.rows;
    V = A;
    d.assign(n, 0.0);
    std::vector<Real> e(n, 0.0);
    if (n == 0) return;
    for (int j = 0; j < n; j++) d[j] = V(n - 1, j);
    for (int i = n - 1; i > 0; i--) {
        Real scale = 0.0, h = 0.0;
        for (int k = 0; k < i; k++) scale += std::fabs(d[k]);
        if (scale == 0.0) {
            e[i] = d[i - 1];
            for (int j = 0; j < i; j++) {
                d[j] = V(i - 1, j);
                V(i, j) = 0.0;
                V(j, i) = 0.0;
            }
        } else {
            for (int k = 0; k < i; k++) {
                d[k] /= scale;
                h += d[k] * d[k];
            }
            Real f = d[i - 1];
            Real g = std::sqrt(h);
            if (f > 0) g = -g;
            e[i] = scale * g;
            h = h - f * g;
            d[i - 1] = f - g;
            for (int j = 0; j < i; j++) e[j] = 0.0;
            for (int j = 0; j < i; j++) {
                f = d[j];
                V(j, i) = f;
                g = e[j] + V(j, j) * f;
                for (int k = j + 1; k <= i - 1; k++) {
                    g += V(k, j) * d[k];
                    e[k] += V(k, j) * f;
                }
                e[j] = g;
            }
            f = 0.0;
            for (int j = 0; j < i; j++) {
                e[j] /= h;
                f += e[j] * d[j];
            }
            const Real hh = f / (h + h);
            for (int j = 0; j < i; j++) e[j] -= hh * d[j];
            for (int j = 0; j < i; j++) {
                f = d[j];
                g = e[j];
                for (int k = j; k <= i - 1; k++) V(k, j) -= (f * e[k] + g * d[k]);
                d[j] = V(i - 1, j);
                V(i, j) = 0.0;
            }
        }
        d[i] = h;
    }
    for (int i = 0; i < n - 1; i++) {
        V(n - 1, i) = V(i, i);
        V(i, i) = 1.0;
        const Real h = d[i + 1];
        if (h != 0.0) {
            for (int k = 0; k <= i; k++) d[k] = V(k, i + 1) / h;
            for (int j = 0; j <= i; j++) {
                Real g = 0.0;
                for (int k = 0; k <= i; k++) g += V(k, i + 1) * V(k, j);
                for (int k = 0; k <= i; k++) V(k, j) -= g * d[k];
            }
        }
        for (int k = 0; k <= i; k++) V(k, i + 1) = 0.0;
    }
    for (int j = 0; j < n; j++) {
        d[j] = V(n - 1, j);
        V(n - 1, j) = 0.0;
    }
    V(n - 1, n - 1) = 1.0;
    e[0] = 0.0;

    for (int i = 1; i < n; i++) e[i - 1] = e[i];
    e[n - 1] = 0.0;
    Real f = 0.0, tst1 = 0.0;
    const Real eps = DBL_EPSILON;
    for (int l = 0; l < n; l++) {
        tst1 = std::max(tst1, std::fabs(d[l]) + std::fabs(e[l]));
        int m = l;
        while (m < n) {
            if (std::fabs(e[m]) <= eps * tst1) break;
            m++;
        }
        if (m == n) m = n - 1;
        if (m > l) {
            int iter = 0;
            do {
                iter++;
                Real g = d[l];
                Real p = (d[l + 1] - g) / (2.0 * e[l]);
                Real r = std::hypot(p, 1.0);
                if (p < 0) r = -r;
                d[l] = e[l] / (p + r);
                d[l + 1] = e[l] * (p + r);
                const Real dl1 = d[l + 1];
                Real h = g - d[l];
                for (int i = l + 2; i < n; i++) d[i] -= h;
                f += h;
                p = d[m];
                Real c = 1.0, c2 = c, c3 = c;
                const Real el1 = e[l + 1];
                Real s = 0.0, s2 = 0.0;
                for (int i = m - 1; i >= l; i--) {
                    c3 = c2;
                    c2 = c;
                    s2 = s;
                    g = c * e[i];
                    h = c * p;
                    r = std::hypot(p, e[i]);
                    e[i + 1] = s * r;
                    s = e[i] / r;
                    c = p / r;
                    p = c * d[i] - s * g;
                    d[i + 1] = h + s * (c * g + s * d[i]);
                    for (int k = 0; k < n; k++) {
                        h = V(k, i + 1);
                        V(k, i + 1) = s * V(k, i) + c * h;
                        V(k, i) = c * V(k, i) - s * h;
                    }
                }
                p = -s * s2 * c3 * el1 * e[l] / dl1;
                e[l] = s * p;
                d[l] = c * p;
            } while (std::fabs(e[l]) > eps * tst1 && iter < 200);
        }
        d[l] = d[l] + f;
        e[l] = 0.0;
    }
    for (int i = 0; i < n - 1; i++) {
        int k = i;
        Real p = d[i];
        for (int j = i + 1; j < n; j++)
            if (d[j] < p) {
                k = j;
                p = d[j];
            }
        if (k != i) {
            d[k] = d[i];
            d[i] = p;
            for (int j = 0; j < n; j++) std::swap(V(j, i), V(j, k));
        }
    }
}

Real LogSum(Real loga, Real logb)
{
    // bcm3::logsum (src/utils/MathFunctions.h:67-82)
    if (logb > loga) std::swap(loga, logb);
    if (loga == -kInf) return loga;
    const Real diff = logb - loga;
    if (diff < -500) return loga;
    return loga + std::log1p(std::exp(diff));
}

static Real LogNormaliser(const Mat& L)
{
    // -sum log L_jj - d/2 log(2 pi) (GMM.cpp:36-40)
    Real det = 0.0;
    for (int j = 0; j < L.rows; j++) det += std::log(L(j, j));
    return -det - 0.5 * L.rows * std::log(2.0 * M_PI);
}

// ---------------------------------------------------------------------------------------------
// GMM (src/stats/GMM.cpp)

bool GMM::Set(const std::vector<std::vector<Real>>& means, const std::vector<Mat>& covariances,
              const std::vector<Real>& w)
{
    // GMM.cpp:14-45
    if (means.empty() || means.size() != covariances.size() || means.size() != w.size()) return false;
    comps.assign(means.size(), Component());
    for (size_t i = 0; i < means.size(); i++) {
        comps[i].mean = means[i];
        comps[i].cov = covariances[i];
        if (!Cholesky(comps[i].cov, comps[i].L)) return false;
        comps[i].logC = LogNormaliser(comps[i].L);
    }
    weights = w;
    return true;
}

Real GMM::LogPdfMVN(const Real* x, const Component& c) const
{
    // GMM.cpp:392-398
    const int D = (int)c.mean.size();
    std::vector<Real> v(D);
    for (int i = 0; i < D; i++) v[i] = x[i] - c.mean[i];
    LowerSolve(c.L, v.data());
    return c.logC - 0.5 * Dot(v.data(), v.data(), D);
}

Real GMM::LogPdf(const Real* x) const
{
    // GMM.cpp:160-170
    Real logp = -kInf;
    for (size_t i = 0; i < comps.size(); i++) logp = LogSum(logp, LogPdfMVN(x, comps[i]) + std::log(weights[i]));
    return logp;
}

std::vector<Real> GMM::CalculateResponsibilities(const Real* x) const
{
    // GMM.cpp:172-186; logsum(VectorReal) (MathFunctions.h:84-92) = max + log(sum exp(p - max))
    const size_t K = comps.size();
    std::vector<Real> probs(K);
    for (size_t i = 0; i < K; i++) probs[i] = LogPdfMVN(x, comps[i]) + std::log(weights[i]);
    Real m = probs[0];
    for (size_t i = 0; i < K; i++) m = std::max(m, probs[i]);
    Real sum = 0.0;
    for (size_t i = 0; i < K; i++) sum += std::exp(probs[i] - m);
    const Real lsum = std::log(sum) + m;
    Real tot = 0.0;
    for (size_t i = 0; i < K; i++) {
        probs[i] = std::exp(probs[i] - lsum);
        tot += probs[i];
    }
    for (size_t i = 0; i < K; i++) probs[i] /= tot;
    return probs;
}

bool GMM::KMeanspp(const Mat& samples, size_t n, size_t K, CtrRng& rng, Mat& resp)
{
    // GMM.cpp:188-245
    if (K < 2) return false;
    const int D = samples.cols;
    comps.assign(K, Component());
    unsigned ix = rng.GetUnsignedInt((unsigned)n - 1);
    comps[0].mean.assign(samples.row(ix), samples.row(ix) + D);
    std::set<unsigned> used{ix};
    std::vector<Real> dv(D);
    for (size_t i = 1; i < K; i++) {
        std::vector<Real> mindistsq(n, 0.0);
        Real total = 0.0;
        for (size_t j = 0; j < n; j++) {
            if (used.count((unsigned)j)) continue;
            Real best = std::numeric_limits<Real>::max();
            for (size_t l = 0; l < i; l++) {
                for (int k = 0; k < D; k++) dv[k] = samples((int)j, k) - comps[l].mean[k];
                best = std::min(best, Dot(dv.data(), dv.data(), D));
            }
            mindistsq[j] = best;
            total += mindistsq[j];
        }
        for (size_t j = 0; j < n; j++) mindistsq[j] /= total;
        const unsigned nix = rng.Sample(mindistsq);
        comps[i].mean.assign(samples.row(nix), samples.row(nix) + D);
        used.insert(nix);
    }
    resp = Mat((int)n, (int)K, 0.0);
    for (size_t i = 0; i < n; i++) {
        Real mindist = std::numeric_limits<Real>::max();
        size_t which = 0;
        for (size_t j = 0; j < K; j++) {
            for (int k = 0; k < D; k++) dv[k] = samples((int)i, k) - comps[j].mean[k];
            const Real ds = Dot(dv.data(), dv.data(), D);
            if (ds < mindist) {
                mindist = ds;
                which = j;
            }
        }
        resp((int)i, (int)which) = 1.0;
    }
    return true;
}

void GMM::CalculateMeanCovariance(const Mat& samples, size_t n, const Mat& resp, int col, std::vector<Real>& mean,
                                  Mat& cov, Real ess_factor) const
{
    // GMM.cpp:247-337: weighted incremental mean / covariance, then eigenvalue shrinkage of the
    // correlation matrix with the effective sample size
    const int D = samples.cols;
    mean.assign(D, 0.0);
    cov = Mat(D, D, 0.0);
    std::vector<Real> d(D), d2(D);
    Real wsum = 0.0;
    for (size_t i = 0; i < n; i++) {
        const Real* x = samples.row((int)i);
        const Real w = resp((int)i, col);
        if (w >= DBL_EPSILON) {
            wsum += w;
            for (int k = 0; k < D; k++) d[k] = x[k] - mean[k];
            const Real f = w / wsum;
            for (int k = 0; k < D; k++) mean[k] += f * d[k];
            for (int k = 0; k < D; k++) d2[k] = x[k] - mean[k];
            for (int j = 0; j < D; j++) {
                const Real wd = w * d[j];
                for (int k = 0; k < D; k++) cov(j, k) += wd * d2[k];
            }
        }
    }
    if (wsum < 2.0) {
        cov = Mat(D, D, 0.0);
        for (int j = 0; j < D; j++) cov(j, j) = 1.0;
        return;
    }
    for (Real& v : cov.a) v /= (wsum - 1);

    Real n_eff = wsum / ess_factor;
    if (n_eff < 2) {
        for (int j = 0; j < D; j++)
            for (int k = 0; k < D; k++)
                if (j != k) cov(j, k) = 0.0;
        return;
    }
    n_eff = std::max(n_eff, (Real)D);
    std::vector<Real> sd(D);
    for (int i = 0; i < D; i++) sd[i] = std::sqrt(cov(i, i));
    Mat corr(D, D, 0.0);
    for (int i = 0; i < D; i++) {
        corr(i, i) = 1.0;
        for (int j = i; j < D; j++) {
            corr(i, j) = cov(i, j) / (sd[i] * sd[j]);
            corr(j, i) = corr(i, j);
        }
    }
    std::vector<Real> ev;
    Mat V;
    SymmetricEigen(corr, ev, V);
    const size_t n_eff_int = (size_t)std::floor(n_eff);
    const size_t m = ev.size();
    if (n_eff_int < m) {
        for (size_t i = 0; i < n_eff_int; i++) ev[(m - 1) - i] *= n_eff / (n_eff + D + 1 - 2.0 * (Real)i);
        for (size_t i = n_eff_int; i < m; i++) ev[(m - 1) - i] = 0.0;
    } else {
        for (size_t i = 0; i < m; i++) ev[(m - 1) - i] *= n_eff / (n_eff + D + 1 - 2.0 * (Real)i);
    }
    // corr = V diag(ev) V^T; cov = diag(sd) corr diag(sd); diagonal += 1e-8
    for (int i = 0; i < D; i++)
        for (int j = 0; j < D; j++) {
            Real s = 0.0;
            for (int k = 0; k < D; k++) s += V(i, k) * ev[k] * V(j, k);
            corr(i, j) = s;
        }
    for (int i = 0; i < D; i++)
        for (int j = 0; j < D; j++) cov(i, j) = sd[i] * corr(i, j) * sd[j];
    for (int i = 0; i < D; i++) cov(i, i) += 1e-8;
}

void GMM::EM_maximization(const Mat& samples, size_t n, const Mat& resp, Real ess_factor)
{
    // GMM.cpp:339-345
    for (size_t i = 0; i < comps.size(); i++) {
        Real s = 0.0;
        for (size_t j = 0; j < n; j++) s += resp((int)j, (int)i);
        weights[i] = s / (Real)n;
        CalculateMeanCovariance(samples, n, resp, (int)i, comps[i].mean, comps[i].cov, ess_factor);
    }
}

bool GMM::EM_expectation(const Mat& samples, size_t n, Mat& resp, Real& logl)
{
    // GMM.cpp:347-390
    const int D = samples.cols;
    std::vector<Real> sample_logl(n, -kInf), v(D);
    for (size_t i = 0; i < comps.size(); i++) {
        if (!Cholesky(comps[i].cov, comps[i].L)) return false;
        const Real logC = LogNormaliser(comps[i].L);
        comps[i].logC = logC;
        const Real log_weight = std::log(weights[i]);
        for (size_t j = 0; j < n; j++) {
            const Real* x = samples.row((int)j);
            for (int k = 0; k < D; k++) v[k] = x[k] - comps[i].mean[k];
            LowerSolve(comps[i].L, v.data());
            const Real p = logC - 0.5 * Dot(v.data(), v.data(), D) + log_weight;
            resp((int)j, (int)i) = std::exp(p);
            sample_logl[j] = LogSum(sample_logl[j], p);
        }
    }
    logl = 0.0;
    for (size_t j = 0; j < n; j++) logl += sample_logl[j];
    const int K = (int)comps.size();
    for (size_t j = 0; j < n; j++) {
        Real total = 0.0;
        for (int i = 0; i < K; i++) total += resp((int)j, i);
        for (int i = 0; i < K; i++) resp((int)j, i) = (total == 0) ? 1.0 / K : resp((int)j, i) / total;
    }
    return true;
}

bool GMM::Fit(const Mat& samples, size_t num_samples, size_t K, CtrRng& rng, Real ess_factor)
{
    // GMM.cpp:48-158
    const size_t maxsteps = 100, retries = 4;
    const Real logl_epsilon = 1e-5;
    const int D = samples.cols;
    Real logl = -kInf;
    bool singular = false;
    if (K == 1) {
        Mat resp((int)num_samples, 1, 1.0);
        comps.assign(1, Component());
        CalculateMeanCovariance(samples, num_samples, resp, 0, comps[0].mean, comps[0].cov, ess_factor);
        if (!Cholesky(comps[0].cov, comps[0].L)) return false;
        comps[0].logC = LogNormaliser(comps[0].L);
        logl = 0.0;
        for (size_t j = 0; j < num_samples; j++) logl += LogPdfMVN(samples.row((int)j), comps[0]);
        weights.assign(1, 1.0);
    } else {
        if ((Real)num_samples < 2.0 * D * K) return false;
        for (size_t ri = 0; ri < retries; ri++) {
            singular = false;
            bool converged = false;
            Mat resp;
            if (!KMeanspp(samples, num_samples, K, rng, resp)) return false;
            for (size_t i = 0; i < comps.size(); i++)
                CalculateMeanCovariance(samples, num_samples, resp, (int)i, comps[i].mean, comps[i].cov, ess_factor);
            weights.assign(K, 1.0 / K);
            Real prev_logl = -kInf;
            for (size_t i = 0; i < maxsteps; i++) {
                if (!EM_expectation(samples, num_samples, resp, logl)) {
                    singular = true;
                    break;
                }
                if (logl < prev_logl) {
                    // a decrease: converged if small, else retry
                    converged = prev_logl - logl < std::fabs(logl * logl_epsilon * 10);
                    break;
                } else if (logl - prev_logl < std::fabs(logl * logl_epsilon)) {
                    converged = true;
                    break;
                }
                prev_logl = logl;
                EM_maximization(samples, num_samples, resp, ess_factor);
            }
            if (converged) break;
        }
    }
    const size_t nparam = K * (D + D * (D + 1) / 2) + K - 1;
    full_logl = logl;
    aic = 2.0 * (Real)nparam - 2.0 * logl;
    return !singular;
}

// ---------------------------------------------------------------------------------------------
// proposal adaptation

Mat ThinHistory(const Mat& history, size_t max_samples, CtrRng& rng)
{
    // Proposal::Initialize (src/sampler/Proposal.cpp:92-121)
    const size_t rows = history.rows;
    if (rows <= max_samples) return history;
    std::vector<size_t> use;
    const size_t subsample = rows / max_samples;
    if (subsample > 1) {
        use.resize(rows / subsample);
        for (size_t i = 0; i < use.size(); i++) use[i] = i * subsample;
    } else {
        use.resize(rows);
        for (size_t i = 0; i < rows; i++) use[i] = i;
    }
    while (use.size() > max_samples) use.erase(use.begin() + rng.GetUnsignedInt((unsigned)use.size() - 1));
    Mat out((int)use.size(), history.cols);
    for (size_t i = 0; i < use.size(); i++)
        std::copy(history.row((int)use[i]), history.row((int)use[i]) + history.cols, &out((int)i, 0));
    return out;
}

// SummaryStats.cpp mean / var / acf (incremental forms)
static Real ColMean(const Mat& h, int c)
{
    Real mu = 0.0;
    for (int i = 0; i < h.rows; i++) mu += (h(i, c) - mu) / (Real)(i + 1);
    return mu;
}
static Real ColVar(const Mat& h, int c, Real mu)
{
    Real s = 0.0;
    for (int i = 0; i < h.rows; i++) {
        const Real d = h(i, c) - mu;
        s += (d * d - s) / (Real)(i + 1);
    }
    const Real n = (Real)h.rows;
    return s * (n / (n - 1.0));
}
static Real ColAcf(const Mat& h, int c, int lag, Real mu, Real sigmaSq)
{
    if (lag == 0) return 1.0;
    if (h.rows <= lag) return std::numeric_limits<Real>::quiet_NaN();
    Real r = 0.0;
    for (int i = 0; i < h.rows - lag; i++) {
        const Real x1 = h(i, c) - mu, x2 = h(i + lag, c) - mu;
        r += (x1 * x2 - r) / (Real)(i + 1);
    }
    return r / sigmaSq;
}

static void StoreFit(const GMM& g, int D, int kmax, ProposalFit& out)
{
    const int K = (int)g.GetNumComponents();
    out.ncomp = K;
    out.weights.assign(kmax, 0.0);
    out.means.assign((size_t)kmax * D, 0.0);
    out.chol.assign((size_t)kmax * D * D, 0.0);
    out.logc.assign(kmax, 0.0);
    Mat I(D, D, 0.0);
    for (int j = 0; j < D; j++) I(j, j) = 1.0;
    const Real logc_id = LogNormaliser(I);
    for (int k = 0; k < kmax; k++) {
        const Mat& L = (k < K) ? g.GetCholesky(k) : I;
        std::copy(L.a.begin(), L.a.end(), out.chol.begin() + (size_t)k * D * D);
        out.logc[k] = (k < K) ? g.GetLogC(k) : logc_id;
        if (k < K) {
            out.weights[k] = g.GetWeights()[k];
            std::copy(g.GetMean(k).begin(), g.GetMean(k).end(), out.means.begin() + (size_t)k * D);
        }
    }
}

bool FitGaussianMixtureProposal(const Mat& history, bool select_with_adjusted_aic, CtrRng& rng,
                                const Real* prior_mean, const Real* prior_var, int kmax, ProposalFit& out)
{
    // ProposalGaussianMixture::InitializeImpl (ProposalGaussianMixture.cpp:125-254)
    const int D = history.cols;
    const size_t n = history.rows;
    GMM best;
    bool have = false;
    if (n >= 2) {
        std::vector<Real> ess(D);
        for (int i = 0; i < D; i++) {
            Real rho_t = 0.0;
            const Real mu = ColMean(history, i);
            const Real sigmaSq = ColVar(history, i, mu);
            const int lag_max = std::max(5, (int)(10 * std::log10((Real)n)));
            for (int lag = 1; lag < lag_max; lag++) rho_t += ColAcf(history, i, lag, mu, sigmaSq);
            ess[i] = (Real)n / (1.0 + 2.0 * rho_t);
        }
        const Real min_ess = *std::min_element(ess.begin(), ess.end());
        const Real aic_adjust = min_ess / (Real)n;
        Real best_aic = kInf;
        static const size_t num_components[7] = {1, 2, 3, 4, 5, 8, 13};
        for (size_t i = 0; i < 7; i++) {
            const size_t K = num_components[i];
            if ((int)K > kmax) break;
            // min_ess < K (1 + min(D/2, 10)) -> not enough effective samples (:157-160)
            if (min_ess < (Real)(K * (1 + std::min((size_t)D / 2, (size_t)10)))) continue;
            GMM g;
            if (!g.Fit(history, n, K, rng, (Real)n / min_ess)) continue;
            const Real nparam = 0.5 * g.GetAIC() + g.GetLogLikelihood();
            const Real adjusted = 2.0 * nparam - 2.0 * aic_adjust * g.GetLogLikelihood();
            // as the reference: the adjusted AIC is compared, the unadjusted one kept (:171-176)
            if (select_with_adjusted_aic ? (adjusted < best_aic) : (g.GetAIC() < best_aic)) {
                best = g;
                have = true;
                best_aic = g.GetAIC();
            }
        }
    }
    out.fitted = have;
    if (!have) {
        // single Gaussian with the prior's moments (:211-241)
        std::vector<std::vector<Real>> means(1, std::vector<Real>(prior_mean, prior_mean + D));
        std::vector<Mat> covs(1, Mat(D, D, 0.0));
        for (int i = 0; i < D; i++) covs[0](i, i) = prior_var[i];
        if (!best.Set(means, covs, std::vector<Real>(1, 1.0))) return false;
    }
    StoreFit(best, D, kmax, out);
    return true;
}

bool FitGlobalCovarianceProposal(const Mat& history, const Real* prior_var, ProposalFit& out)
{
    // ProposalGlobalCovariance::InitializeImpl (ProposalGlobalCovariance.cpp:64-104) with cov()
    // (src/utils/SummaryStats.cpp:195-240)
    const int D = history.cols;
    Mat c(D, D, 0.0);
    if (history.rows < 2) {
        for (int j = 0; j < D; j++) c(j, j) = prior_var[j];
    } else {
        std::vector<Real> m(D, 0.0), m1(D);
        Mat acc(D, D, 0.0);
        Real en = 0.0;
        for (int si = 0; si < history.rows; si++) {
            en += 1.0;
            const Real invN = 1.0 / en;
            m1 = m;
            for (int i = 0; i < D; i++) m[i] += (history(si, i) - m[i]) * invN;
            if (en > 1) {
                const Real ratio = (en - 1) / en;
                for (int i = 0; i < D; i++) {
                    const Real dx = history(si, i) - m1[i];
                    for (int j = i; j < D; j++) acc(i, j) += dx * (history(si, j) - m1[j]) * ratio;
                }
            }
        }
        for (int i = 0; i < D; i++)
            for (int j = 0; j < D; j++) c(i, j) = ((j >= i) ? acc(i, j) : acc(j, i)) * (1.0 / (en - 1.0));
        for (int j = 0; j < D; j++) c(j, j) = std::max(c(j, j), 1e-6 * prior_var[j]);
    }
    GMM g;
    std::vector<std::vector<Real>> means(1, std::vector<Real>(D, 0.0));
    if (!g.Set(means, std::vector<Mat>(1, c), std::vector<Real>(1, 1.0))) return false;
    out.fitted = history.rows >= 2;
    StoreFit(g, D, 1, out);
    return true;
}

}  // namespace bcm3
