// pt_exchange.h -- SamplerPTChain::ExchangeMove of one pair of local chains (SamplerPT.cpp:277-306,
// SamplerPTChain.cpp:328-381), shared by the exchange kernels (pt_kernels.hip) and the fused
// exchange of the speculative pairs (proposal_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ctr_rng.h"

namespace bcm3hip {

// dst[0..n) = src[0..n) with every load of a block of 16 issued before its stores: the compiler cannot
// tell that the rows do not alias, so a plain element loop waits one memory round trip per element
template <class T>
__device__ __forceinline__ void copy_row(T* dst, const double* src, int n)
{
    constexpr int R = 16;
    for (int k0 = 0; k0 < n; k0 += R) {
        double v[R];
#pragma unroll
        for (int k = 0; k < R; k++)
            if (k0 + k < n) v[k] = src[k0 + k];
#pragma unroll
        for (int k = 0; k < R; k++)
            if (k0 + k < n) dst[k0 + k] = (T)v[k];
    }
}

// rows a[0..n) and b[0..n) exchanged, both blocks loaded before any store
__device__ __forceinline__ void swap_rows(double* a, double* b, int n)
{
    constexpr int R = 16;
    for (int k0 = 0; k0 < n; k0 += R) {
        double va[R], vb[R];
#pragma unroll
        for (int k = 0; k < R; k++)
            if (k0 + k < n) {
                va[k] = a[k0 + k];
                vb[k] = b[k0 + k];
            }
#pragma unroll
        for (int k = 0; k < R; k++)
            if (k0 + k < n) {
                a[k0 + k] = vb[k];
                b[k0 + k] = va[k];
            }
    }
}

// one ExchangeMove between local chains i1 and i2 of the slice (global index of i1 = g1)
__device__ inline bool exchange_pair(int d, int i1, int i2, int64_t g1, const double* temps, double* values, double* llh,
                              double* lprior, double* lpp, uint8_t* acc_mask, unsigned long long* accepted,
                              uint64_t seed, uint64_t round)
{
    const double t1 = temps[i1], t2 = temps[i2];
    const double p1 = (t1 == 0.0) ? lprior[i2] : t1 * llh[i2] + lprior[i2];
    const double p2 = (t2 == 0.0) ? lprior[i1] : t2 * llh[i1] + lprior[i1];
    double tp = exp((p1 + p2) - (lpp[i1] + lpp[i2]));
    tp = (tp < 1.0) ? tp : 1.0;  // std::min((Real)1.0, tp): a NaN probability becomes 1
    // bcm3_amd.pt.exchange_uniform(seed, round, g1)
    const uint64_t key = rng::splitmix64(rng::splitmix64(seed) ^ (round * 0x100000001B3ull) ^ ((uint64_t)g1 * 0xC2B2AE3D27D4EB4Full));
    const bool swap = rng::u01(key) < tp;
    if (swap) {
        swap_rows(values + (int64_t)i1 * d, values + (int64_t)i2 * d, d);
        const double l = llh[i1];
        llh[i1] = llh[i2];
        llh[i2] = l;
        const double q = lprior[i1];
        lprior[i1] = lprior[i2];
        lprior[i2] = q;
        lpp[i1] = p1;
        lpp[i2] = p2;
        if (accepted) atomicAdd(accepted, 1ull);
    }
    if (acc_mask) acc_mask[i1] = swap ? 1 : 0;
    return swap;
}

}  // namespace bcm3hip
