// analytic_kernel.hip -- batched analytic test likelihoods (configs C1/C2) on MI355X.
//
//   banana   TestLikelihoodBanana::EvaluateLogProbability   (TestLikelihoodBanana.cpp:42-55)
//   circular TestLikelihoodCircular::EvaluateLogProbability (TestLikelihoodCircular.cpp:42-53)
// One lane per evaluation; values[n][d] row-major is streamed once (HBM-bound: 8*d bytes in,
// 8 bytes out per evaluation).
//
// PdfNormal in the reference uses an SSE rsqrtss estimate + two Newton steps
// (MathFunctions.h:35-48), whose bits depend on the CPU vendor; here the same two Newton steps
// start from the correctly rounded 1/sqrt, so results agree to ~1e-14 relative.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "popk_kernel.h"

namespace bcm3hip {

__device__ __forceinline__ double bcm3_rsqrt(double x)
{
    double r = (double)(1.0f / sqrtf((float)x));
    r *= ((3.0 - r * r * x) * 0.5);
    r *= ((3.0 - r * r * x) * 0.5);
    return r;
}

__device__ __forceinline__ double pdf_normal(double x, double mu, double sigma)
{
    double two_sigma_sq = 2.0 * sigma * sigma;
    double d = x - mu;
    return bcm3_rsqrt(two_sigma_sq * M_PI) * exp(-(d * d) / two_sigma_sq);
}

__device__ __forceinline__ double log_pdf_normal(double x, double mu, double sigma)
{
    double two_sigma_sq = 2.0 * sigma * sigma;
    double d = x - mu;
    return -log(sigma) - 0.91893853320467274178032973640562 - d * d / two_sigma_sq;
}

// bcm3::logsum (MathFunctions.h:67-82)
__device__ __forceinline__ double logsum(double loga, double logb)
{
    if (logb > loga) {
        double t = loga;
        loga = logb;
        logb = t;
    }
    if (loga == -INFINITY) return loga;
    double diff = logb - loga;
    if (diff < -500) return loga;
    return loga + log1p(exp(diff));
}

__global__ void __launch_bounds__(256) banana_kernel(int64_t n, int d, double sd1, double sd2,
                                                     const double* __restrict__ values, double* __restrict__ logp,
                                                     int32_t* __restrict__ status)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const double* v = values + e * d;
    double p = 1.0;
    for (int i = 0; i < d - 1; i++) p = p * pdf_normal(v[i], 0, sd1);
    double y = v[0];
    for (int i = 1; i < d - 1; i++) y += v[i];
    p *= pdf_normal(v[d - 1], y + 3 * y + (1 - y) * (1 - y), sd2);
    logp[e] = log(p);
    if (status) status[e] = 0;
}

__global__ void __launch_bounds__(256) circular_kernel(int64_t n, int d, double radius, double offset, double width,
                                                       const double* __restrict__ values,
                                                       double* __restrict__ logp, int32_t* __restrict__ status)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const double* v = values + e * d;
    double s1 = 0.0, s2 = 0.0;
    for (int i = 0; i < d; i++) {
        double m1 = (i == 0) ? -offset : 0.0;
        double m2 = (i == 0) ? offset : 0.0;
        double a = v[i] - m1, b = v[i] - m2;
        s1 += a * a;
        s2 += b * b;
    }
    logp[e] = logsum(log_pdf_normal(sqrt(s1), radius, width), log_pdf_normal(sqrt(s2), radius, width));
    if (status) status[e] = 0;
}

hipError_t launch_analytic(const AnalyticDevModel& m, int64_t n, const double* values, double* logp,
                           int32_t* status, hipStream_t stream, hipEvent_t ev_start, hipEvent_t ev_stop)
{
    if (n == 0) return hipSuccess;
    const int tb = 256;
    dim3 grid((unsigned)((n + tb - 1) / tb)), block(tb);
    if (ev_start) hipEventRecord(ev_start, stream);
    if (m.kind == BCM3HIP_ANALYTIC_BANANA)
        hipLaunchKernelGGL(banana_kernel, grid, block, 0, stream, n, m.d, m.p0, m.p1, values, logp, status);
    else if (m.kind == BCM3HIP_ANALYTIC_CIRCULAR)
        hipLaunchKernelGGL(circular_kernel, grid, block, 0, stream, n, m.d, m.p0, m.p1, m.p2, values, logp,
                           status);
    else
        return hipErrorInvalidValue;
    if (ev_stop) hipEventRecord(ev_stop, stream);
    return hipGetLastError();
}

}  // namespace bcm3hip
