// Single-wave latency / issue microbenchmarks on gfx950 (one wave, clock64 = s_memtime cycles).
// Guides the BDF lane kernel design: what a dependent FP64 op, a select, a cross-lane move, a
// uniform branch and an LDS / L2 round trip cost when ONE wavefront runs alone on a SIMD.
//   hipcc -O3 --offload-arch=gfx950 -o build/lat lat.hip && ./build/lat
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP 64
#define OUTER 16
#define NOPS (REP * OUTER)

__device__ __forceinline__ double opq(double x)
{
    asm volatile("" : "+v"(x));
    return x;
}

template <int TEST>
__global__ void kern(double* out, long long* cyc, const double* gin, double a, double b, int ia)
{
    __shared__ double lds[1024];
    __shared__ int ldsi[1024];
    int lane = threadIdx.x;
    for (int i = lane; i < 1024; i += 64) {
        lds[i] = 1.0 + i;
        ldsi[i] = (i * 17 + 1) & 1023;
    }
    __syncthreads();
    double x = a + lane * 1e-9, y = b + lane * 1e-9, z = a * 0.5, w = b * 0.25;
    double x4 = a * 0.3, x5 = b * 0.2, x6 = a * 0.7, x7 = b * 0.9;
    float f = (float)a;
    int k = lane & ia;
    long long t0 = clock64();
    for (int o = 0; o < OUTER; o++) {
#pragma unroll
        for (int r = 0; r < REP; r++) {
            if constexpr (TEST == 0) x = __builtin_fma(x, a, b);  // dependent fma f64
            if constexpr (TEST == 1) {                            // 2 chains
                x = __builtin_fma(x, a, b);
                y = __builtin_fma(y, a, b);
            }
            if constexpr (TEST == 2) {  // 4 chains
                x = __builtin_fma(x, a, b);
                y = __builtin_fma(y, a, b);
                z = __builtin_fma(z, a, b);
                w = __builtin_fma(w, a, b);
            }
            if constexpr (TEST == 3) {  // 8 chains
                x = __builtin_fma(x, a, b);
                y = __builtin_fma(y, a, b);
                z = __builtin_fma(z, a, b);
                w = __builtin_fma(w, a, b);
                x4 = __builtin_fma(x4, a, b);
                x5 = __builtin_fma(x5, a, b);
                x6 = __builtin_fma(x6, a, b);
                x7 = __builtin_fma(x7, a, b);
            }
            if constexpr (TEST == 4) x = x + a;                      // dependent add f64
            if constexpr (TEST == 5) f = __builtin_fmaf(f, (float)a, (float)b);  // dependent fma f32
            if constexpr (TEST == 6) x = __builtin_amdgcn_rcp(x);                 // v_rcp_f64
            if constexpr (TEST == 7) x = __builtin_sqrt(x) + a;                   // sqrt f64 (libcall?)
            if constexpr (TEST == 8) x = opq(x < a ? x * b : x + b);             // cmp + select + arith
            if constexpr (TEST == 9) x = (double)__builtin_amdgcn_readfirstlane((int)x) + a;  // VALU->SALU->VALU
            if constexpr (TEST == 10) {
                int v = __builtin_bit_cast(int, f);
                v = __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
                f = __builtin_bit_cast(float, v) + (float)a;
            }
            if constexpr (TEST == 11) {
                int v = __builtin_bit_cast(int, f);
                v = __builtin_amdgcn_ds_bpermute(((lane + 1) & 63) << 2, v);
                f = __builtin_bit_cast(float, v) + (float)a;
            }
            if constexpr (TEST == 12) k = ldsi[k];                 // LDS pointer chase
            if constexpr (TEST == 13) k = (int)gin[k & 255];      // global (L1/L2) chase
            if constexpr (TEST == 14) f = __builtin_amdgcn_exp2f(f) * (float)a;  // v_exp_f32
            if constexpr (TEST == 15) x = b / x;                   // IEEE f64 divide
            if constexpr (TEST == 16) {                            // uniform branch per op
                if (__builtin_amdgcn_readfirstlane(k) > ia) x = x * a;
                else x = x + a;
                k = k + 1;
            }
            if constexpr (TEST == 17) x = x * a;                   // dependent mul f64
            if constexpr (TEST == 18) {                            // 2-element f64 cross-lane: two dpp movs + add
                long long v = __builtin_bit_cast(long long, x);
                int lo = (int)v, hi = (int)(v >> 32);
                lo = __builtin_amdgcn_update_dpp(0, lo, 0x111, 0xf, 0xf, false);
                hi = __builtin_amdgcn_update_dpp(0, hi, 0x111, 0xf, 0xf, false);
                x = __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo) + a;
            }
            if constexpr (TEST == 19) {  // f64 from lane 0 broadcast via readlane (x2) + add
                long long v = __builtin_bit_cast(long long, x);
                int lo = __builtin_amdgcn_readlane((int)v, 1), hi = __builtin_amdgcn_readlane((int)(v >> 32), 1);
                x = __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo) + a;
            }
            if constexpr (TEST == 20) {  // LDS f64 store + load round trip
                lds[lane] = x;
                __builtin_amdgcn_s_waitcnt(0xc07f);
                x = lds[(lane + 1) & 63] + a;
            }
        }
    }
    long long t1 = clock64();
    if (lane == 0) cyc[0] = t1 - t0;
    out[lane] = x + y + z + w + x4 + x5 + x6 + x7 + f + k;
}

template <int T>
static double run(const char* name, double* out, long long* cyc, const double* gin, int ops_per)
{
    long long h = 0;
    for (int rep = 0; rep < 3; rep++) {
        kern<T><<<1, 64>>>(out, cyc, gin, 1.0000001, 1e-7, 0);
        hipDeviceSynchronize();
    }
    hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double per = (double)h / NOPS;
    printf("%-44s %8.2f cycles per iteration (%d op(s))\n", name, per, ops_per);
    return per;
}

int main()
{
    double* out;
    long long* cyc;
    double* gin;
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&cyc, sizeof(long long));
    hipMalloc(&gin, 256 * sizeof(double));
    double h[256];
    for (int i = 0; i < 256; i++) h[i] = (double)((i * 37 + 11) & 255);
    hipMemcpy(gin, h, sizeof(h), hipMemcpyHostToDevice);
    run<0>("v_fma_f64 dependent", out, cyc, gin, 1);
    run<1>("v_fma_f64 2 chains", out, cyc, gin, 2);
    run<2>("v_fma_f64 4 chains", out, cyc, gin, 4);
    run<3>("v_fma_f64 8 chains", out, cyc, gin, 8);
    run<4>("v_add_f64 dependent", out, cyc, gin, 1);
    run<17>("v_mul_f64 dependent", out, cyc, gin, 1);
    run<5>("v_fma_f32 dependent", out, cyc, gin, 1);
    run<6>("v_rcp_f64 dependent", out, cyc, gin, 1);
    run<7>("sqrt f64 + add dependent", out, cyc, gin, 2);
    run<15>("IEEE f64 divide dependent", out, cyc, gin, 1);
    run<8>("cmp f64 + 2 arith + select", out, cyc, gin, 4);
    run<9>("cvt+readfirstlane+cvt+add", out, cyc, gin, 4);
    run<10>("dpp row_shr f32 + add", out, cyc, gin, 2);
    run<18>("dpp row_shr f64 (2 movs) + add f64", out, cyc, gin, 3);
    run<19>("readlane f64 (2) + add f64", out, cyc, gin, 3);
    run<11>("ds_bpermute + add f32", out, cyc, gin, 2);
    run<12>("LDS load chase", out, cyc, gin, 1);
    run<20>("LDS f64 store+load round trip", out, cyc, gin, 2);
    run<13>("global load chase (L1/L2 hit)", out, cyc, gin, 2);
    run<14>("v_exp_f32 + mul", out, cyc, gin, 2);
    run<16>("uniform branch + op", out, cyc, gin, 3);
    hipFree(out);
    hipFree(cyc);
    hipFree(gin);
    return 0;
}
