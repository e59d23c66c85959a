// Single-wave cost of compare / branch / select idioms on gfx950 (clock64 cycles per iteration).
//   hipcc -O3 --offload-arch=gfx950 -o build/branch branch.hip && ./build/branch
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP 64
#define OUTER 16

template <int TEST>
__global__ void kern(double* out, long long* cyc, double a, double b, int ia)
{
    double x = a + threadIdx.x * 0.0;  // uniform value in VGPRs
    double y = b;
    int k = ia;
    unsigned xl = 3, xh = 5;
    long long t0 = clock64();
    for (int o = 0; o < OUTER; o++) {
#pragma unroll
        for (int r = 0; r < REP; r++) {
            if constexpr (TEST == 0) {  // v_cmp -> vcc -> s_cbranch_vccz, branch usually taken over 1 op
                asm volatile(
                    "v_cmp_gt_f64 vcc, %0, %1\n\t"
                    "s_cbranch_vccz 1f\n\t"
                    "v_mul_f64 %0, %0, %2\n\t"
                    "1:\n\t"
                    "v_add_f64 %0, %0, %2\n\t"
                    : "+v"(x)
                    : "v"(y), "v"(a)
                    : "vcc");
            }
            if constexpr (TEST == 1) {  // SALU compare + scc branch, not taken
                asm volatile(
                    "s_cmp_gt_i32 %1, 100\n\t"
                    "s_cbranch_scc1 1f\n\t"
                    "v_add_f64 %0, %0, %2\n\t"
                    "1:\n\t"
                    : "+v"(x)
                    : "s"(k), "v"(a)
                    : "scc");
            }
            if constexpr (TEST == 2) {  // SALU compare + scc branch, taken
                asm volatile(
                    "s_cmp_lt_i32 %1, 100\n\t"
                    "s_cbranch_scc1 1f\n\t"
                    "v_mul_f64 %0, %0, %2\n\t"
                    "1:\n\t"
                    "v_add_f64 %0, %0, %2\n\t"
                    : "+v"(x)
                    : "s"(k), "v"(a)
                    : "scc");
            }
            if constexpr (TEST == 3) {  // v_cmp + 2x v_cndmask select, then cvt back (dependent chain)
                asm volatile(
                    "v_cmp_gt_f64 vcc, %0, %3\n\t"
                    "v_cndmask_b32 %1, %1, %4, vcc\n\t"
                    "v_cndmask_b32 %2, %2, %4, vcc\n\t"
                    "v_cvt_f64_u32 %0, %1\n\t"
                    : "+v"(x), "+v"(xl), "+v"(xh)
                    : "v"(y), "v"(k)
                    : "vcc");
            }
            if constexpr (TEST == 4) {  // v_max_f64 + add
                asm volatile(
                    "v_max_f64 %0, %0, %1\n\t"
                    "v_add_f64 %0, %0, %2\n\t"
                    : "+v"(x)
                    : "v"(y), "v"(a));
            }
            if constexpr (TEST == 5) {  // add only (baseline)
                asm volatile("v_add_f64 %0, %0, %1\n\t" : "+v"(x) : "v"(a));
            }
            if constexpr (TEST == 6) {  // unconditional forward branch + add
                asm volatile(
                    "s_branch 1f\n\t"
                    "v_mul_f64 %0, %0, %1\n\t"
                    "1:\n\t"
                    "v_add_f64 %0, %0, %1\n\t"
                    : "+v"(x)
                    : "v"(a));
            }
            if constexpr (TEST == 7) {  // v_cmp to SGPR pair + s_cmp_lg_u64 + scc branch (ballot style)
                asm volatile(
                    "v_cmp_gt_f64 s[40:41], %0, %1\n\t"
                    "s_cmp_lg_u64 s[40:41], 0\n\t"
                    "s_cbranch_scc0 1f\n\t"
                    "v_mul_f64 %0, %0, %2\n\t"
                    "1:\n\t"
                    "v_add_f64 %0, %0, %2\n\t"
                    : "+v"(x)
                    : "v"(y), "v"(a)
                    : "s40", "s41", "scc");
            }
            if constexpr (TEST == 8) {  // v_cmp (no use) + dependent add: cost of the compare alone
                asm volatile(
                    "v_cmp_gt_f64 vcc, %0, %1\n\t"
                    "v_add_f64 %0, %0, %2\n\t"
                    : "+v"(x)
                    : "v"(y), "v"(a)
                    : "vcc");
            }
            if constexpr (TEST == 9) {  // v_readfirstlane -> SALU op -> VALU reads SGPR
                asm volatile(
                    "v_readfirstlane_b32 s40, %1\n\t"
                    "s_add_u32 s40, s40, 1\n\t"
                    "v_mov_b32 %1, s40\n\t"
                    : "+v"(x), "+v"(xl)
                    :
                    : "s40", "scc");
            }
            if constexpr (TEST == 10) {  // 2 v_cndmask (vcc ready) + cvt back
                asm volatile(
                    "v_cndmask_b32 %1, %1, %3, vcc\n\t"
                    "v_cndmask_b32 %2, %2, %3, vcc\n\t"
                    "v_cvt_f64_u32 %0, %1\n\t"
                    : "+v"(x), "+v"(xl), "+v"(xh)
                    : "v"(k)
                    : "vcc");
            }
            if constexpr (TEST == 13) {  // cvt only baseline for tests 3/10
                asm volatile("v_cvt_f64_u32 %0, %1\n\t v_cvt_u32_f64 %1, %0\n\t" : "+v"(x), "+v"(xl));
            }
            if constexpr (TEST == 11) {  // v_fma_f64 dependent
                asm volatile("v_fma_f64 %0, %0, %1, %1\n\t" : "+v"(x) : "v"(a));
            }
            if constexpr (TEST == 12) {  // v_rcp_f64 + 2 Newton steps (5 dependent ops: frcp)
                asm volatile(
                    "v_rcp_f64 %1, %0\n\t"
                    "v_fma_f64 %2, -%0, %1, 1.0\n\t"
                    "v_fma_f64 %1, %2, %1, %1\n\t"
                    "v_fma_f64 %2, -%0, %1, 1.0\n\t"
                    "v_fma_f64 %0, %2, %1, %1\n\t"
                    : "+v"(x), "+v"(y), "+v"(b));
            }
        }
    }
    long long t1 = clock64();
    if (threadIdx.x == 0) cyc[0] = t1 - t0;
    out[threadIdx.x] = x + y + k + xl + xh;
}

template <int T>
static void run(const char* name, double* out, long long* cyc)
{
    long long h = 0;
    for (int rep = 0; rep < 3; rep++) {
        kern<T><<<1, 64>>>(out, cyc, 1.0000001, 0.5, 7);
        (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    printf("%-58s %8.2f cycles/iter\n", name, (double)h / (REP * OUTER));
}

int main()
{
    double* out;
    long long* cyc;
    (void)hipMalloc(&out, 64 * sizeof(double));
    (void)hipMalloc(&cyc, sizeof(long long));
    run<5>("v_add_f64 dependent (baseline)", out, cyc);
    run<11>("v_fma_f64 dependent", out, cyc);
    run<8>("v_cmp_f64->vcc (unused) + add", out, cyc);
    run<0>("v_cmp_f64 + s_cbranch_vccz (taken) + add", out, cyc);
    run<7>("v_cmp_f64->sgpr + s_cmp_lg_u64 + cbranch_scc (taken) + add", out, cyc);
    run<1>("s_cmp + s_cbranch_scc (not taken) + add", out, cyc);
    run<2>("s_cmp + s_cbranch_scc (taken) + add", out, cyc);
    run<6>("s_branch (taken) + add", out, cyc);
    run<3>("v_cmp + 2 v_cndmask (dependent) + cvt", out, cyc);
    run<10>("2 v_cndmask (vcc ready) + cvt", out, cyc);
    run<13>("cvt f64<-u32 + cvt u32<-f64 (baseline for 3/10)", out, cyc);
    run<4>("v_max_f64 + add", out, cyc);
    run<9>("readfirstlane + s_add + v_mov (VALU->SALU->VALU)", out, cyc);
    run<12>("frcp (rcp + 2 newton, 5 dep ops)", out, cyc);
    (void)hipFree(out);
    (void)hipFree(cyc);
    return 0;
}
