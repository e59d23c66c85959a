// pk_math.h -- scalar math shared by the PK likelihood kernels (popk_kernel.hip,
// expm_pk_kernel.hip): VariableSet::TransformVariable (src/sampler/VariableSet.cpp:97-124),
// fastpow10 (src/utils/MathFunctions.h:13), LogPdfTnu4 (src/utils/ProbabilityDistributions.cpp:216-224).
#pragma once
#include <hip/hip_runtime.h>

#include "bdf_lane.h"

namespace bcm3hip {

BDF_INL double fastpow10(double x) { return exp(x * 2.3025850929940459); }

BDF_INL double transform_var(int tf, double x)
{
    switch (tf) {
    case 1: return exp(x);
    case 2: return fastpow10(x);
    case 3:
        if (x > 0) {
            double z = exp(-x);
            return 1.0 / (1.0 + z);
        } else {
            double z = exp(x);
            return z / (1.0 + z);
        }
    default: return x;
    }
}

BDF_INL double log_pdf_tnu4(double x, double mu, double sigma)
{
    double xn = (x - mu) / sigma;
    return -0.9808292530117262 - 2.5 * log1p(0.25 * xn * xn) - log(sigma);
}

}  // namespace bcm3hip
