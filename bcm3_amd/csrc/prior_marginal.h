// prior_marginal.h -- the univariate prior marginals of PriorIndependence on the device:
// UnivariateMarginal::EvaluateLogPDF and ::Sample (src/sampler/UnivariateMarginal.cpp:215-380)
// for the eight distribution types the reference's prior.xml accepts (:25-101). Parameters per
// variable: p0, p1, p2 as listed at BCM3HIP_PRIOR_* (include/bcm3hip.h).
//
// Log densities follow the reference's expressions; where the reference takes log(pdf) of a
// Boost density (gamma, beta: ProbabilityDistributions.cpp:11-49) the log density is evaluated
// directly (lgamma form), which agrees to rounding where the pdf does not underflow. Draws use
// the counter-based streams of ctr_rng.h: normals by Box-Muller, Gamma by Marsaglia-Tsang
// (RNG::GetGamma, RNG.cpp:84-111), Beta from two Gammas (RNG.h:63-68), exponentials as
// -mu log1p(-u) (RNG.h:48-52), Cauchy as scale tan(pi (u - 1/2)).
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/bcm3hip.h"
#include "ctr_rng.h"

namespace bcm3hip {
namespace prior {

// per-variable stream for the draws of a T = 0 chain: slot base 0x100000 + (i << 10);
// normal slots base + n, uniform keys 2 (base + 0x200) + u
struct Stream {
    uint64_t seed, iter, chain, base;
    int n = 0, u = 0;
    __device__ double uniform() { return rng::u01(rng::rng_key(seed, iter, chain, 2 * (base + 0x200) + u++)); }
    __device__ double normal() { return rng::normal01(seed, iter, chain, base + n++); }
};

// RNG::GetGamma(k, theta) (RNG.cpp:84-111)
__device__ inline double gamma(double k, double theta, Stream& s)
{
    double scale_u = 1.0;
    if (k < 1.0) {
        const double u = s.uniform();
        scale_u = pow(u, 1.0 / k);
        k = 1.0 + k;
    }
    const double d = k - 0.33333333333333333333333333333333;
    const double c = 0.33333333333333333333333333333333 / sqrt(d);
    double v = 1.0;
    for (int it = 0; it < 256; it++) {  // Marsaglia-Tsang accepts > 95 % per attempt
        double x;
        int tries = 0;
        do {
            x = s.normal();
            v = 1.0 + c * x;
        } while (v <= 0.0 && ++tries < 64);
        v = v * v * v;
        const double u = s.uniform();
        if (u < 1 - 0.0331 * x * x * x * x) break;
        if (log(u) < 0.5 * x * x + d * (1 - v + log(v))) break;
    }
    return theta * d * v * scale_u;
}

__device__ inline double beta(double a, double b, Stream& s)
{
    const double x1 = gamma(a, 1.0, s);
    const double x2 = gamma(b, 1.0, s);
    return x1 / (x1 + x2);
}

__device__ inline double exponential(double mu, Stream& s)
{
    const double u = s.uniform();
    return -mu * log1p(-u);
}

// UnivariateMarginal::Sample (UnivariateMarginal.cpp:215-258)
__device__ inline double sample(int kind, double p0, double p1, double p2, uint64_t seed, uint64_t iter,
                                uint64_t chain, int i)
{
    if (kind == BCM3HIP_PRIOR_UNIFORM)
        return p0 + rng::u01(rng::rng_key(seed, iter, chain, rng::KEY_PRIOR_UNIFORM + i)) * (p1 - p0);
    if (kind == BCM3HIP_PRIOR_NORMAL) return p0 + p1 * rng::normal01(seed, iter, chain, rng::SLOT_PRIOR_NORMAL + i);
    Stream s{seed, iter, chain, 0x100000ull + ((uint64_t)i << 10)};
    switch (kind) {
    case BCM3HIP_PRIOR_EXPONENTIAL: return exponential(1.0 / p0, s);
    case BCM3HIP_PRIOR_GAMMA: return gamma(p0, p1, s);
    case BCM3HIP_PRIOR_BETA: return beta(p0, p1, s);
    case BCM3HIP_PRIOR_HALF_CAUCHY: return fabs(p0 * tan(3.141592653589793 * (s.uniform() - 0.5)));
    case BCM3HIP_PRIOR_BETA_PRIME: {
        const double x = beta(p0, p1, s);
        return p2 * ((x) / (1.0 - x));
    }
    case BCM3HIP_PRIOR_EXPONENTIAL_MIX: {
        const double p = s.uniform();
        return (p < p2) ? exponential(1.0 / p0, s) : exponential(1.0 / p1, s);
    }
    // a Dirichlet member's Gamma(alpha_i, 1) draw; the caller divides by the group's sum
    // (MultivariateMarginal::Sample, MultivariateMarginal.cpp:66-84)
    case BCM3HIP_PRIOR_DIRICHLET: return gamma(p0, 1.0, s);
    default: return NAN;
    }
}

__device__ inline double log_pdf_exponential(double x, double lambda)
{
    // LogPdfExponential (ProbabilityDistributions.cpp:121-127)
    if (x < 0.0) return -INFINITY;
    return log(lambda) - lambda * x;
}

// MathFunctions.h:67-82 (boost::math::log1p -> log1p)
__device__ inline double logsum(double loga, double logb)
{
    if (logb > loga) {
        const double t = loga;
        loga = logb;
        logb = t;
    }
    if (loga == -INFINITY) return loga;
    const double diff = logb - loga;
    if (diff < -500) return loga;
    return loga + log1p(exp(diff));
}

// UnivariateMarginal::EvaluateLogPDF (UnivariateMarginal.cpp:326-380)
__device__ inline double log_pdf(int kind, double p0, double p1, double p2, double x)
{
    switch (kind) {
    case BCM3HIP_PRIOR_UNIFORM: return (x < p0 || x > p1) ? -INFINITY : -log(p1 - p0);
    case BCM3HIP_PRIOR_NORMAL: {
        const double s = p1;
        const double dx = x - p0;
        return log(1.0 / sqrt(2.0 * s * s * 3.141592653589793)) - dx * dx * (1.0 / (2.0 * s * s));
    }
    case BCM3HIP_PRIOR_EXPONENTIAL: return log_pdf_exponential(x, p0);
    case BCM3HIP_PRIOR_GAMMA:
        // log(PdfGamma(x, k, theta)) (ProbabilityDistributions.cpp:39-49)
        if (x < 0.0 || x == INFINITY) return -INFINITY;
        if (p0 == 1.0) return log_pdf_exponential(x, 1.0 / p1);
        return (p0 - 1.0) * log(x) - x / p1 - lgamma(p0) - p0 * log(p1);
    case BCM3HIP_PRIOR_BETA:
        // log(PdfBeta(x, a, b)) (ProbabilityDistributions.cpp:11-18)
        if (x < 0.0 || x > 1.0) return -INFINITY;
        return (p0 - 1.0) * log(x) + (p1 - 1.0) * log1p(-x) - (lgamma(p0) + lgamma(p1) - lgamma(p0 + p1));
    case BCM3HIP_PRIOR_HALF_CAUCHY:
        if (x <= 0.0) return -INFINITY;
        return -0.45158270528945486472619522989488 - log(p0 + x * x / p0);
    case BCM3HIP_PRIOR_BETA_PRIME: {
        // LogPdfBetaPrime (ProbabilityDistributions.cpp:110-119)
        if (x < 0.0) return -INFINITY;
        const double lnc = -log(exp(lgamma(p0) + lgamma(p1) - lgamma(p0 + p1)) * p2);
        const double sx = x / p2;
        const double lrv = (p0 - 1.0) * log(sx) - (p0 + p1) * log(sx + 1.0);
        return lnc + lrv;
    }
    case BCM3HIP_PRIOR_EXPONENTIAL_MIX:
        return logsum(log(p2) + log_pdf_exponential(x, p0), log(1.0 - p2) + log_pdf_exponential(x, p1));
    default: return NAN;
    }
}

// Dirichlet group of variables [first, last] (BCM3HIP_PRIOR_DIRICHLET): the last member of the
// group starting at `first`
__device__ inline int dirichlet_last(int d, const int32_t* kind, const double* p1, int first)
{
    int l = first;
    while (l + 1 < d && kind[l + 1] == BCM3HIP_PRIOR_DIRICHLET && (int)p1[l + 1] == first) l++;
    return l;
}

__device__ inline bool has_dirichlet(int d, const int32_t* kind)
{
    for (int i = 0; i < d; i++)
        if (kind[i] == BCM3HIP_PRIOR_DIRICHLET) return true;
    return false;
}

// MultivariateMarginal::EvaluateLogPDF (MultivariateMarginal.cpp:86-118) of the group
// [first, last]; x(j) returns variable j's value
template <class X>
__device__ inline double dirichlet_log_pdf(int first, int last, const double* alpha, double lnc, X&& x)
{
    double sum = 0.0;
    for (int j = first; j <= last; j++) {
        const double v = x(j);
        if (v < 0.0 || v > 1.0) return -INFINITY;
        sum += v;
    }
    if (fabs(sum - 1.0) > 1e-15) return -INFINITY;
    double lp = 0.0;
    for (int j = first; j <= last; j++) lp += (alpha[j] - 1) * log(x(j));
    return lp + lnc;
}

}  // namespace prior
}  // namespace bcm3hip
