// pt_exchange.h -- SamplerPTChain::ExchangeMove of one pair of local chains (SamplerPT.cpp:277-306,
// SamplerPTChain.cpp:328-381), shared by the exchange kernels (pt_kernels.hip) and the fused
// exchange of the speculative pairs (proposal_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "ctr_rng.h"

namespace bcm3hip {

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
        for (int k = 0; k < d; k++) {
            const double a = values[(int64_t)i1 * d + k];
            values[(int64_t)i1 * d + k] = values[(int64_t)i2 * d + k];
            values[(int64_t)i2 * d + k] = a;
        }
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
