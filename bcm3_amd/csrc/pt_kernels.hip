// pt_kernels.hip -- the sampler side of one PT-MH iteration as three small HIP kernels, so that
// an iteration is propose -> batched likelihood -> accept -> exchange with everything in HBM and
// no host round trip:
//   ptmh_propose_kernel   SamplerPTChain::MutateMove proposal + PriorIndependence::EvaluateLogPDF
//                         (src/sampler/SamplerPTChain.cpp:217-279, src/sampler/PriorIndependence.cpp:129-157,
//                          src/sampler/UnivariateMarginal.cpp:326-345)
//   ptmh_accept_kernel    TestSample + the state update (SamplerPTChain.cpp:280-313, 465-481)
//   pt_exchange_kernel    SamplerPT::DoExchangeMove / SamplerPTChain::ExchangeMove for the pairs inside
//                         one rank's slice of the temperature ladder (SamplerPT.cpp:277-298,
//                         SamplerPTChain.cpp:328-381); pairs that straddle ranks are exchanged by the
//                         host over RCCL (bcm3_amd/pt.py).
// Random numbers are counter based (ctr_rng.h), so a chain's stream does not depend on how chains
// are distributed over ranks or blocks.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/bcm3hip.h"
#include "ctr_rng.h"
#include "pt_exchange.h"

namespace bcm3hip {
namespace {

using rng::normal01;
using rng::rng_key;
using rng::splitmix64;
using rng::u01;

__global__ void ptmh_propose_kernel(int C, int d, const int32_t* __restrict__ kind, const double* __restrict__ p0,
                                    const double* __restrict__ p1, const double* __restrict__ scale,
                                    const double* __restrict__ temps, const double* __restrict__ values,
                                    double* __restrict__ prop, double* __restrict__ lprior_prop, int64_t chain0,
                                    uint64_t seed, uint64_t iter)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const uint64_t gc = (uint64_t)(chain0 + c);
    const bool t0 = temps[c] == 0.0;
    double lp = 0.0;
    for (int i = 0; i < d; i++) {
        double x;
        if (t0) {
            // PriorIndependence::Sample: uniform a + u (b - a), normal mu + sigma z
            if (kind[i] == BCM3HIP_PRIOR_UNIFORM)
                x = p0[i] + u01(rng_key(seed, iter, gc, rng::KEY_PRIOR_UNIFORM + i)) * (p1[i] - p0[i]);
            else
                x = p0[i] + p1[i] * normal01(seed, iter, gc, rng::SLOT_PRIOR_NORMAL + i);
        } else {
            x = values[(int64_t)c * d + i] + scale[i] * normal01(seed, iter, gc, i);
        }
        prop[(int64_t)c * d + i] = x;
        // UnivariateMarginal::EvaluateLogPDF
        double l;
        if (kind[i] == BCM3HIP_PRIOR_UNIFORM) {
            l = (x < p0[i] || x > p1[i]) ? -INFINITY : -log(p1[i] - p0[i]);
        } else {
            const double s = p1[i];
            const double dx = x - p0[i];
            l = log(1.0 / sqrt(2.0 * s * s * 3.141592653589793)) - dx * dx * (1.0 / (2.0 * s * s));
        }
        lp += l;
    }
    lprior_prop[c] = lp;
}

__global__ void ptmh_accept_kernel(int C, int d, const double* __restrict__ temps, const double* __restrict__ prop,
                                   const double* __restrict__ lprior_prop, const double* __restrict__ llh_prop,
                                   double learning_rate, double* __restrict__ values, double* __restrict__ lprior,
                                   double* __restrict__ llh, double* __restrict__ lpp, uint8_t* __restrict__ acc_out,
                                   unsigned long long* __restrict__ accepted, int32_t* __restrict__ nan_llh,
                                   int64_t chain0, uint64_t seed, uint64_t iter)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const double T = temps[c];
    const double nl = llh_prop[c] * learning_rate;  // Sampler::EvaluateLikelihood
    const double nq = lprior_prop[c];
    bool acc;
    double npp;
    if (isnan(nl)) {
        // Sampler::EvaluateLikelihood (Sampler.cpp:172-178): a NaN log-likelihood is fatal; the
        // chain keeps its state and the host raises at its next check of the flag
        if (nan_llh) *nan_llh = 1;
        acc = false;
        npp = 0.0;
    } else if (T == 0.0) {
        // sample from the prior, always accepted; 0 * -inf avoided (SamplerPTChain.cpp:231-237)
        acc = true;
        npp = (nl == -INFINITY) ? nq : nq + T * nl;
    } else {
        npp = nq + T * nl;
        acc = false;
        if (npp > -INFINITY) {
            double tp = exp(npp - lpp[c]);
            tp = (tp < 1.0) ? tp : 1.0;  // std::min((Real)1.0, tp): NaN -> 1
            acc = u01(rng_key(seed, iter, (uint64_t)(chain0 + c), rng::KEY_ACCEPT)) < tp;
        }
    }
    if (acc) {
        for (int i = 0; i < d; i++) values[(int64_t)c * d + i] = prop[(int64_t)c * d + i];
        lprior[c] = nq;
        llh[c] = nl;
        lpp[c] = npp;
    }
    if (acc_out) acc_out[c] = acc ? 1 : 0;
    if (accepted && acc) atomicAdd(accepted, 1ull);
}

// local pairs of one round: first chains i (local index) with (g0 + i - start) even and i + 1 < C,
// then -- single rank only -- the wrap pair (C-1, 0) after them (the reference loops in order)
__global__ void pt_exchange_kernel(int C, int d, int64_t g0, int start, int wrap_local, const double* temps,
                                   double* values, double* llh, double* lprior, double* lpp, uint8_t* acc_mask,
                                   unsigned long long* accepted, uint64_t seed, uint64_t round)
{
    const int par = (int)(((g0 - start) % 2 + 2) % 2);  // local i is a first chain iff (i + par) even
    const int first = par;                              // smallest such i
    for (int p = threadIdx.x;; p += blockDim.x) {
        const int i = first + 2 * p;
        if (i + 1 >= C) break;
        exchange_pair(d, i, i + 1, g0 + i, temps, values, llh, lprior, lpp, acc_mask, accepted, seed, round);
    }
    __syncthreads();
    if (wrap_local && threadIdx.x == 0) {
        exchange_pair(d, C - 1, 0, g0 + C - 1, temps, values, llh, lprior, lpp, acc_mask, accepted, seed, round);
    }
}

// one pair (stochastic_random swapping, SamplerPT.cpp:300-305): local chains i1, i2, uniform keyed by
// the global index g1 of the first
__global__ void pt_exchange_pair_kernel(int d, int i1, int i2, int64_t g1, const double* temps, double* values,
                                        double* llh, double* lprior, double* lpp, uint8_t* acc_out,
                                        unsigned long long* accepted, uint64_t seed, uint64_t round)
{
    if (threadIdx.x != 0) return;
    const bool a = exchange_pair(d, i1, i2, g1, temps, values, llh, lprior, lpp, nullptr, accepted, seed, round);
    if (acc_out) *acc_out = a ? 1 : 0;
}

// the record a rank sends for a slice-boundary pair: {values[d], llh, lprior, lpp, T}
__global__ void pt_pack_boundary_kernel(int C, int d, const double* temps, const double* values, const double* llh,
                                        const double* lprior, const double* lpp, double* send_last,
                                        double* send_first)
{
    const int k = threadIdx.x;
    for (int side = 0; side < 2; side++) {
        const int i = side ? 0 : C - 1;
        double* out = side ? send_first : send_last;
        if (!out) continue;
        if (k < d) out[k] = values[(int64_t)i * d + k];
        if (k == 0) {
            out[d] = llh[i];
            out[d + 1] = lprior[i];
            out[d + 2] = lpp[i];
            out[d + 3] = temps[i];
        }
    }
}

// ExchangeMove of a pair whose chains live on two ranks (SamplerPTChain.cpp:328-381): both ranks
// evaluate the same decision from the same two records (exchange_pair's arithmetic, uniform keyed
// by the global index of the pair's first chain) and keep their own side.
//   pair A (do_next): (my last chain C-1, the next rank's first chain = record nxt), first = g0+C-1
//   pair B (do_prev): (the previous rank's last chain = record prv, my first chain 0), first = gp
__global__ void pt_cross_accept_kernel(int C, int d, int64_t g0, int64_t gp, int do_next, int do_prev,
                                       const double* temps, double* values, double* llh, double* lprior, double* lpp,
                                       const double* nxt, const double* prv, uint8_t* acc_out,
                                       unsigned long long* accepted, uint64_t seed, uint64_t round)
{
    if (threadIdx.x != 0) return;
    if (do_next) {
        const int i = C - 1;
        const double t1 = temps[i], t2 = nxt[d + 3];
        const double p1 = (t1 == 0.0) ? nxt[d + 1] : t1 * nxt[d] + nxt[d + 1];
        const double p2 = (t2 == 0.0) ? lprior[i] : t2 * llh[i] + lprior[i];
        double tp = exp((p1 + p2) - (lpp[i] + nxt[d + 2]));
        tp = (tp < 1.0) ? tp : 1.0;
        const uint64_t key = splitmix64(splitmix64(seed) ^ (round * 0x100000001B3ull) ^
                                        ((uint64_t)(g0 + C - 1) * 0xC2B2AE3D27D4EB4Full));
        const bool a = u01(key) < tp;
        if (a) {
            for (int k = 0; k < d; k++) values[(int64_t)i * d + k] = nxt[k];
            llh[i] = nxt[d];
            lprior[i] = nxt[d + 1];
            lpp[i] = p1;
            if (accepted) atomicAdd(accepted, 1ull);
        }
        if (acc_out) acc_out[0] = a ? 1 : 0;
    }
    if (do_prev) {
        const double t1 = prv[d + 3], t2 = temps[0];
        const double p1 = (t1 == 0.0) ? lprior[0] : t1 * llh[0] + lprior[0];
        const double p2 = (t2 == 0.0) ? prv[d + 1] : t2 * prv[d] + prv[d + 1];
        double tp = exp((p1 + p2) - (prv[d + 2] + lpp[0]));
        tp = (tp < 1.0) ? tp : 1.0;
        const uint64_t key = splitmix64(splitmix64(seed) ^ (round * 0x100000001B3ull) ^
                                        ((uint64_t)gp * 0xC2B2AE3D27D4EB4Full));
        const bool b = u01(key) < tp;
        if (b) {
            for (int k = 0; k < d; k++) values[k] = prv[k];
            llh[0] = prv[d];
            lprior[0] = prv[d + 1];
            lpp[0] = p2;
        }
        if (acc_out) acc_out[1] = b ? 1 : 0;
    }
}

}  // namespace
}  // namespace bcm3hip

using namespace bcm3hip;

extern "C" {

int bcm3hip_ptmh_propose(int C, int d, const int32_t* prior_kind, const double* prior_p0, const double* prior_p1,
                         const double* scale, const double* temps, const double* values, double* prop,
                         double* lprior_prop, int64_t chain0, uint64_t seed, uint64_t iter, void* stream)
{
    if (C < 0 || d <= 0 || (C > 0 && (!prior_kind || !prior_p0 || !prior_p1 || !scale || !temps || !values || !prop ||
                                      !lprior_prop)))
        return BCM3HIP_ERR_ARG;
    if (C == 0) return 0;
    hipLaunchKernelGGL(ptmh_propose_kernel, dim3((C + 63) / 64), dim3(64), 0, (hipStream_t)stream, C, d, prior_kind,
                       prior_p0, prior_p1, scale, temps, values, prop, lprior_prop, chain0, seed, iter);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_ptmh_accept(int C, int d, const double* temps, const double* prop, const double* lprior_prop,
                        const double* llh_prop, double learning_rate, double* values, double* lprior, double* llh,
                        double* lpp, uint8_t* accept_out, uint64_t* accepted, int32_t* nan_llh, int64_t chain0,
                        uint64_t seed, uint64_t iter, void* stream)
{
    if (C < 0 || d <= 0 ||
        (C > 0 && (!temps || !prop || !lprior_prop || !llh_prop || !values || !lprior || !llh || !lpp)))
        return BCM3HIP_ERR_ARG;
    if (C == 0) return 0;
    hipLaunchKernelGGL(ptmh_accept_kernel, dim3((C + 63) / 64), dim3(64), 0, (hipStream_t)stream, C, d, temps, prop,
                       lprior_prop, llh_prop, learning_rate, values, lprior, llh, lpp, accept_out,
                       (unsigned long long*)accepted, nan_llh, chain0, seed, iter);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_pt_pack_boundary(int C, int d, const double* temps, const double* values, const double* llh,
                             const double* lprior, const double* lpp, double* send_last, double* send_first,
                             void* stream)
{
    if (C < 1 || d <= 0 || d > 1024 || !temps || !values || !llh || !lprior || !lpp) return BCM3HIP_ERR_ARG;
    hipLaunchKernelGGL(pt_pack_boundary_kernel, dim3(1), dim3(d < 64 ? 64 : ((d + 63) / 64) * 64), 0,
                       (hipStream_t)stream, C, d, temps, values, llh, lprior, lpp, send_last, send_first);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_pt_cross_accept(int C, int d, int64_t g0, int64_t gp, int do_next, int do_prev, const double* temps,
                            double* values, double* llh, double* lprior, double* lpp, const double* recv_next,
                            const double* recv_prev, uint8_t* acc_out, uint64_t* accepted, uint64_t seed,
                            uint64_t round, void* stream)
{
    if (C < 1 || d <= 0 || !temps || !values || !llh || !lprior || !lpp || (do_next && !recv_next) ||
        (do_prev && !recv_prev))
        return BCM3HIP_ERR_ARG;
    hipLaunchKernelGGL(pt_cross_accept_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, C, d, g0, gp, do_next,
                       do_prev, temps, values, llh, lprior, lpp, recv_next, recv_prev, acc_out,
                       (unsigned long long*)accepted, seed, round);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_pt_exchange_local(int C, int d, int64_t g0, int start, int wrap_local, const double* temps,
                              double* values, double* llh, double* lprior, double* lpp, uint8_t* acc_mask,
                              uint64_t* accepted, uint64_t seed, uint64_t round, void* stream)
{
    if (C < 0 || d <= 0 || (start != 0 && start != 1) ||
        (C > 0 && (!temps || !values || !llh || !lprior || !lpp)))
        return BCM3HIP_ERR_ARG;
    if (C < 2 && !wrap_local) return 0;
    if (C == 0) return 0;
    hipLaunchKernelGGL(pt_exchange_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, C, d, g0, start, wrap_local,
                       temps, values, llh, lprior, lpp, acc_mask, (unsigned long long*)accepted, seed, round);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_pt_exchange_pair(int C, int d, int i1, int i2, int64_t g1, const double* temps, double* values,
                             double* llh, double* lprior, double* lpp, uint8_t* acc_out, uint64_t* accepted,
                             uint64_t seed, uint64_t round, void* stream)
{
    if (C < 2 || d <= 0 || i1 < 0 || i2 < 0 || i1 >= C || i2 >= C || i1 == i2 || !temps || !values || !llh ||
        !lprior || !lpp)
        return BCM3HIP_ERR_ARG;
    hipLaunchKernelGGL(pt_exchange_pair_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, d, i1, i2, g1, temps,
                       values, llh, lprior, lpp, acc_out, (unsigned long long*)accepted, seed, round);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

}  // extern "C"
