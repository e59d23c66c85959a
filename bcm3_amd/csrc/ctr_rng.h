// ctr_rng.h -- counter-based random numbers of the sampler kernels: every draw is splitmix64 of
// (seed, iteration, global chain index, slot), so a chain's stream does not depend on how chains
// are distributed over ranks, blocks or threads (the reference's per-thread ranlux48 streams,
// src/utils/RNG.cpp:15-61, are clock seeded and not reproducible).
//
// Slot map (one iteration of one chain); normal01(slot s) consumes the keys 2s and 2s + 1:
//   proposal normals z_i             normal slots i                   keys 0x0000..0x1FFF
//   prior draws, normal marginals    normal slots 0x2000 + i          keys 0x4000..0x5FFF
//   Gamma draws (t proposals)        normal slots 0x3000 + a          keys 0x6000..0x7FFF
//   prior draws, other marginals     uniform keys 0x8000 + i
//   Gamma draws, uniforms            uniform keys 0x9000 + a, 0x9800 (k < 1)
//   Proposal::Update learn rate      uniform key 0xA000
//   component selection (RNG::Sample) uniform key 0xA001
//   TestSample                       uniform key 0xC000
// (tests/ptmh_reference.py and tests/proposal_reference.py restate the same map.)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace bcm3hip {
namespace rng {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// uniform in [0, 1) from 53 random bits
__device__ __forceinline__ double u01(uint64_t z) { return (double)(z >> 11) * (1.0 / 9007199254740992.0); }

// key for (seed, iteration, chain, slot); slot < 2^16
__device__ __forceinline__ uint64_t rng_key(uint64_t seed, uint64_t iter, uint64_t chain, uint64_t slot)
{
    return splitmix64(splitmix64(seed) ^ (iter * 0x100000001B3ull) ^ (chain * 0xC2B2AE3D27D4EB4Full) ^
                      (slot * 0x165667B19E3779F9ull));
}

__device__ __forceinline__ double uniform(uint64_t seed, uint64_t iter, uint64_t chain, uint64_t k)
{
    return u01(rng_key(seed, iter, chain, k));
}

// standard normal by Box-Muller from two counter-based uniforms
__device__ __forceinline__ double normal01(uint64_t seed, uint64_t iter, uint64_t chain, uint64_t slot)
{
    const double u1 = 1.0 - u01(rng_key(seed, iter, chain, 2 * slot));  // (0, 1]
    const double u2 = u01(rng_key(seed, iter, chain, 2 * slot + 1));
    return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

enum : uint64_t {
    SLOT_PRIOR_NORMAL = 0x2000,
    SLOT_GAMMA_NORMAL = 0x3000,
    KEY_PRIOR_UNIFORM = 0x8000,
    KEY_GAMMA_UNIFORM = 0x9000,
    KEY_GAMMA_SMALLK = 0x9800,
    KEY_UPDATE = 0xA000,
    KEY_SELECT = 0xA001,
    KEY_ACCEPT = 0xC000,
};

}  // namespace rng
}  // namespace bcm3hip
