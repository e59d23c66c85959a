// analytic_kernel.hip -- batched analytic test likelihoods (configs C1/C2) on MI355X.
//
//   banana   TestLikelihoodBanana::EvaluateLogProbability   (TestLikelihoodBanana.cpp:42-55)
//   circular TestLikelihoodCircular::EvaluateLogProbability (TestLikelihoodCircular.cpp:42-53)
//   dummy    LikelihoodDummy::EvaluateLogProbability        (LikelihoodDummy.cpp:18-32)
//   multimodal_gaussians / truncated_t: mixtures of dmvnormal (src/stats/mvn.cpp:9-33) / dmvt
//            (src/stats/mvt.cpp:119-157) components (TestLikelihoodMultimodalGaussians.cpp:36-42,
//            TestLikelihoodTruncatedT.cpp:81-90)
// One lane per evaluation; values[n][d] row-major is streamed once (HBM-bound: 8*d bytes in,
// 8 bytes out per evaluation).
//
// PdfNormal in the reference uses an SSE rsqrtss estimate + two Newton steps
// (MathFunctions.h:35-48), whose bits depend on the CPU vendor; here the same two Newton steps
// start from the correctly rounded 1/sqrt, so results agree to ~1e-14 relative.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/bcm3hip.h"
#include "pk_math.h"
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

__global__ void __launch_bounds__(256) dummy_kernel(int64_t n, int d, const double* __restrict__ values,
                                                    double* __restrict__ logp, int32_t* __restrict__ status)
{
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    logp[e] = log_pdf_tnu4(values[e * d], 0.0, 1.0);
    if (status) status[e] = 0;
}

// One evaluation per lane. Per component k: v = L_k^-1 (x - mu_k) by forward substitution (Eigen's
// TriangularView::solveInPlace; dot products in index order), then
//   NORMAL  logC_k - 0.5 v.v                                   (dmvnormal, logC = -sum log L_ii - p/2 log 2pi)
//   T       logC_k - 0.5 (p + nu) log1p(v.v / nu)              (dmvt, p >= 2)
//   T, p=1  LogPdfT(x, mu, sigma = cov(0,0), nu): xn = (x - mu) * sigma (the reference multiplies),
//           -inf when xn^2/nu overflows, logC - 0.5 (nu + 1) log1p(xn^2/nu); LogPdfNormal for nu > 1e10
// and logp = logsum(logp, log w_k + density_k) from logp = -inf, as TestLikelihoodTruncatedT does
// (logsum(-inf, a) = a, so the two-component MultimodalGaussians form logsum(l1, l2) is the same).
template <int TKIND>
__global__ void __launch_bounds__(256) mixture_kernel(int64_t n, int d, int K, const double* __restrict__ mean,
                                                      const double* __restrict__ chol,
                                                      const double* __restrict__ cst,
                                                      const double* __restrict__ values, double* __restrict__ logp,
                                                      int32_t* __restrict__ status)
{
    constexpr int DM = BCM3HIP_MIXTURE_DMAX;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    const double* x = values + e * d;
    double xv[DM];
#pragma unroll
    for (int i = 0; i < DM; i++) xv[i] = (i < d) ? x[i] : 0.0;
    double lp = -INFINITY;
    for (int k = 0; k < K; k++) {
        const double* mu = mean + (int64_t)k * d;
        const double* L = chol + (int64_t)k * d * d;
        const double lw = cst[3 * k], logc = cst[3 * k + 1], nu = cst[3 * k + 2];
        double comp;
        if (TKIND == BCM3HIP_MIXTURE_T && d == 1) {
            const double sigma = L[0];
            if (nu > 1e10) {
                const double two_sigma_sq = 2.0 * sigma * sigma;
                const double dd = xv[0] - mu[0];
                comp = -log(sigma) - 0.91893853320467274178032973640562 - dd * dd / two_sigma_sq;
            } else {
                const double xn = (xv[0] - mu[0]) * sigma;
                const double basem1 = xn * xn / nu;
                comp = (basem1 == INFINITY) ? -INFINITY : logc + -0.5 * (nu + 1.0) * log1p(basem1);
            }
        } else {
            double v[DM];
            double dot = 0.0;
#pragma unroll
            for (int i = 0; i < DM; i++) {
                if (i < d) {
                    double s = xv[i] - mu[i];
#pragma unroll
                    for (int j = 0; j < i; j++) s -= L[i * d + j] * v[j];
                    v[i] = s / L[i * d + i];
                    dot += v[i] * v[i];
                }
            }
            if (TKIND == BCM3HIP_MIXTURE_NORMAL)
                comp = logc - 0.5 * dot;
            else
                comp = logc - 0.5 * ((double)d + nu) * log1p(dot / nu);
        }
        lp = logsum(lp, comp + lw);
    }
    logp[e] = lp;
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
    else if (m.kind == BCM3HIP_ANALYTIC_DUMMY)
        hipLaunchKernelGGL(dummy_kernel, grid, block, 0, stream, n, m.d, values, logp, status);
    else if (m.kind == kAnalyticMixtureBase + BCM3HIP_MIXTURE_NORMAL)
        hipLaunchKernelGGL(mixture_kernel<BCM3HIP_MIXTURE_NORMAL>, grid, block, 0, stream, n, m.d, m.K, m.mean,
                           m.chol, m.cst, values, logp, status);
    else if (m.kind == kAnalyticMixtureBase + BCM3HIP_MIXTURE_T)
        hipLaunchKernelGGL(mixture_kernel<BCM3HIP_MIXTURE_T>, grid, block, 0, stream, n, m.d, m.K, m.mean, m.chol,
                           m.cst, values, logp, status);
    else
        return hipErrorInvalidValue;
    if (ev_stop) hipEventRecord(ev_stop, stream);
    return hipGetLastError();
}

}  // namespace bcm3hip
