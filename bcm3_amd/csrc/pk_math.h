// pk_math.h -- scalar math shared by the PK likelihood kernels (popk_kernel.hip,
// expm_pk_kernel.hip): VariableSet::TransformVariable (src/sampler/VariableSet.cpp:97-124),
// fastpow10 (src/utils/MathFunctions.h:13), QuantileNormal (ProbabilityDistributions.cpp:359-363), LogPdfTnu4 (src/utils/ProbabilityDistributions.cpp:216-224).
#pragma once
#include <hip/hip_runtime.h>

#include "bdf_lane.h"

namespace bcm3hip {

// libm's exp / log / log1p / erf / erfc through libm_exact.h (the glibc results of the oracle);
// COLD: call them out of line (xm::lib)
template <bool COLD = false>
BDF_INL double fastpow10(double x) { return xm::lib<COLD>::exp(x * 2.3025850929940459); }

template <bool COLD = false>
BDF_INL double transform_var(int tf, double x)
{
    switch (tf) {
    case 1: return xm::lib<COLD>::exp(x);
    case 2: return fastpow10<COLD>(x);
    case 3:
        if (x > 0) {
            double z = xm::lib<COLD>::exp(-x);
            return 1.0 / (1.0 + z);
        } else {
            double z = xm::lib<COLD>::exp(x);
            return z / (1.0 + z);
        }
    default: return x;
    }
}

// (out of line and with external linkage, as the PopPK kernel was tuned with; every kernel
// translation unit is compiled to its own code object, so the definitions do not collide)
// standard normal quantile for p in (0, 0.5]: rational initial guess + Halley refinement
__device__ double ndtri_lower(double p)
{
    double x;
    if (p < 0.02425) {
        double q = sqrt(-2.0 * xm::log(p));
        x = (((((-7.784894002430293e-03 * q - 3.223964580411365e-01) * q - 2.400758277161838e+00) * q -
               2.549732539343734e+00) * q + 4.374664141464968e+00) * q + 2.938163982698783e+00) /
            ((((7.784695709041462e-03 * q + 3.224671290700398e-01) * q + 2.445134137142996e+00) * q +
              3.754408661907416e+00) * q + 1.0);
    } else {
        double q = p - 0.5, r = q * q;
        x = (((((-3.969683028665376e+01 * r + 2.209460984245205e+02) * r - 2.759285104469687e+02) * r +
               1.383577518672690e+02) * r - 3.066479806614716e+01) * r + 2.506628277459239e+00) * q /
            (((((-5.447609879822406e+01 * r + 1.615858368580409e+02) * r - 1.556989798598866e+02) * r +
               6.680131188771972e+01) * r - 1.328068155288572e+01) * r + 1.0);
    }
    const bool central = (p > 0.25);  // residual via erf near p = 0.5 (p - 0.5 exact)
    for (int it = 0; it < 3; it++) {
        double e = central ? 0.5 * xm::erf(x / 1.4142135623730951) - (p - 0.5)
                           : 0.5 * xm::erfc(-x / 1.4142135623730951) - p;
        double u = e * 2.5066282746310002 * xm::exp(0.5 * x * x);
        x = x - u / (1.0 + 0.5 * x * u);
    }
    return x;
}

// bcm3::QuantileNormal = Boost quantile(normal(mu, sigma), p) = mean - sigma*sqrt2*erfc_inv(2p)
__device__ double quantile_normal(double p, double mu, double sigma)
{
    double z;
    if (!(p > 0.0))
        z = (p == 0.0) ? -__builtin_inf() : __builtin_nan("");
    else if (!(p < 1.0))
        z = (p == 1.0) ? __builtin_inf() : __builtin_nan("");
    else if (p <= 0.5)
        z = ndtri_lower(p);
    else
        z = -ndtri_lower(1.0 - p);
    double r = z / 1.4142135623730951;  // -erfc_inv(2p)
    r *= sigma * 1.4142135623730951;
    r += mu;
    return r;
}

template <bool COLD = false>
BDF_INL double log_pdf_tnu4(double x, double mu, double sigma)
{
    double xn = (x - mu) / sigma;
    return -0.9808292530117262 - 2.5 * xm::lib<COLD>::log1p(0.25 * xn * xn) - xm::lib<COLD>::log(sigma);
}

}  // namespace bcm3hip
