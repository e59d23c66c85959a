// bdf_lane.h -- one CVODE-5.3.0-equivalent variable-order BDF integrator per GPU lane.
//
// Restates, for small dense systems (NS <= 3, everything in VGPRs), the algorithm of
//   dependencies/cvode-5.3.0/src/cvode/cvode.c      (CVode ONE_STEP, cvHin, cvStep, cvNls,
//                                                    cvDoErrorTest, cvCompleteStep,
//                                                    cvPrepareNextStep, CVodeGetDky, CVodeReInit)
//   dependencies/cvode-5.3.0/src/cvode/cvode_ls.c   (cvLsSetup/cvLsLinSys/cvLsSolve)
//   dependencies/cvode-5.3.0/src/cvode/cvode_nls.c + sunnonlinsol_newton.c (Newton, maxiters 3)
//   src/odecommon/sunlinsol_dense_eigen.cpp:111-178 (closed-form 2x2/3x3 inverse)
//   src/odecommon/nvector_serial_eigen.cpp          (vector-op formulas)
// as BCM3 configures them (user Jacobian, hmin = hmax_inv = 0, no roots/constraints).
//
// GPU design (latency-bound: one trajectory's ~10^3 BDF steps are strictly sequential):
//  * one trajectory per lane; Nordsieck array zn[0..5][NS], error weights, the explicit
//    (I - gamma J)^-1 and all step-control scalars live in VGPRs for the whole solve;
//  * every expensive operation has ONE call site (rescale, restore, residual/RHS in Newton,
//    the h-ratio root), so the hot loop is short and the instruction cache stays warm;
//  * every array index is a compile-time constant at the source level (cfor: template
//    recursion, not loops), so the first SROA pass turns the whole state into SSA values before
//    any pass can form a pointer select; loops over the runtime order q are expanded over
//    1..QMAX with per-j guards on q. No inline-asm barriers: with one trajectory per wavefront
//    (UNI launch) every value stays wave-uniform to the compiler and every solver branch is a
//    scalar branch;
//  * division / sqrt / x^(1/k) use hardware reciprocal + one Newton refinement (within ~11 ulp;
//    correctly rounded with -DBCM3_CORRECTLY_ROUNDED), a perturbation well inside the
//    reference's own FMA-contraction build differences -- see DESIGN.md "parity envelope";
//  * the model supplies a structured (I - gamma J) inverse: for constant-Jacobian models the
//    saved Jacobian of cvLsLinSys is re-derived from the parameters instead of stored.
#pragma once
#include <hip/hip_runtime.h>

#include "libm_exact.h"

namespace bcm3hip {

constexpr int QMAX = 5;

// cvode.c:145-172, cvode_nls.c:29-31, cvode_ls_impl.h:40-41
constexpr double FUZZ_FACTOR = 100.0;
constexpr double HLB_FACTOR = 100.0;
constexpr double HUB_FACTOR = 0.1;
constexpr double H_BIAS = 0.5;
constexpr int MAX_ITERS = 4;
constexpr double CORTES = 0.1;
constexpr double THRESH = 1.5;
constexpr double ETAMX1 = 10000.0;
constexpr double ETAMX2 = 10.0;
constexpr double ETAMX3 = 10.0;
constexpr double ETAMXF = 0.2;
constexpr double ETAMIN = 0.1;
constexpr double ETACF = 0.25;
constexpr double ADDON = 0.000001;
constexpr double BIAS1 = 6.0;
constexpr double BIAS2 = 6.0;
constexpr double BIAS3 = 10.0;
constexpr int SMALL_NST = 10;
constexpr int MXNCF = 10;
constexpr int MXNEF = 7;
constexpr int MXNEF1 = 3;
constexpr int SMALL_NEF = 2;
constexpr int LONG_WAIT = 10;
constexpr double DGMAX = 0.3;
constexpr int MSBP = 20;
constexpr int NLS_MAXCOR = 3;
constexpr double CRDOWN = 0.3;
constexpr double RDIV = 2.0;
constexpr int CVLS_MSBJ = 50;
constexpr double CVLS_DGMAX = 0.2;
constexpr double UROUND = 2.220446049250313e-16;  // DBL_EPSILON

enum { FIRST_CALL = 6, PREV_CONV_FAIL = 7, PREV_ERR_FAIL = 8 };
enum { CONV_NONE = 0, CONV_BAD_J = 1, CONV_OTHER = 2 };
enum { CV_SUCCESS = 0, CV_TSTOP_RETURN = 1, CV_TOO_MUCH_ACC = -2, CV_ERR_FAILURE = -3,
       CV_CONV_FAILURE = -4, CV_ILL_INPUT = -22, CV_BAD_T = -26, CV_TOO_CLOSE = -27 };

#define BDF_INL __device__ __forceinline__
// BCM3_DBL=k (cost-probe builds only, tools/dbl_probe.sh): component k of the step runs twice, the
// second time on operands laundered through an empty asm and with its results consumed by one, so
// the solve's results are unchanged and the kernel time grows by what that component costs
// (1 step-size root, 2 order-change screen, 3 exact order-change evaluation, 4 cvSet coefficients,
// 5 Newton correction, 6 linear-solver setup, 7 error weights, 8 fast-loop exit test, 9 predict)
#ifdef BCM3_DBL
#define BDF_DBL(k) (BCM3_DBL == (k))
#else
#define BDF_DBL(k) false
#endif
BDF_INL double bdf_launder(double x)
{
    asm volatile("" : "+v"(x));
    return x;
}
BDF_INL void bdf_consume(double x) { asm volatile("" ::"v"(x)); }

// branch-layout hints for the UNI solver (hot path falls through; rare work out of line)
#ifdef BCM3_NO_EXPECT
#define BDF_LIKELY(x) (x)
#define BDF_UNLIKELY(x) (x)
#else
#define BDF_LIKELY(x) __builtin_expect(!!(x), 1)
#define BDF_UNLIKELY(x) __builtin_expect(!!(x), 0)
#endif

// readfirstlane of both halves: the value is (already) the same in every lane, or only lane 0's
// value is wanted; the result is uniform to the compiler
BDF_INL double wave_uniform(double x)
{
    const long long b = __builtin_bit_cast(long long, x);
    const int lo = __builtin_amdgcn_readfirstlane((int)b);
    const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// compile-time index loops: f(IC<j>{}) for j = B..E-1 (cfor) or j = B down to E (cfor_down)
template <int V>
struct IC {
    static constexpr int value = V;
};
template <int B, int E, class F>
BDF_INL void cfor(F&& f)
{
    if constexpr (B < E) {
        f(IC<B>{});
        cfor<B + 1, E>(static_cast<F&&>(f));
    }
}
template <int B, int E, class F>
BDF_INL void cfor_down(F&& f)
{
    if constexpr (B >= E) {
        f(IC<B>{});
        cfor_down<B - 1, E>(static_cast<F&&>(f));
    }
}
#define CI(J) decltype(J)::value
#define SUNMAX(A, B) ((A) > (B) ? (A) : (B))
#define SUNMIN(A, B) ((A) < (B) ? (A) : (B))

// ---------------------------------------------------------------------------------------------
// Fast arithmetic for the divisions, reciprocals and square roots of the BDF step. By default
// v_rcp_f64 / v_rsq_f64 with ONE Newton (Goldschmidt) step: within ~11 ulp (tools/ubench/
// rcp_acc.hip, sqrt_acc.hip), 5 % faster per launch at 256 draws (1.425 vs 1.505 ms, C3) and 9 %
// at 2048 than the correctly rounded forms, which -DBCM3_CORRECTLY_ROUNDED restores (one more
// Newton step / a residual correction; identical to the CPU's IEEE results on 4M random
// operands). Either way the three solver forms share these functions and agree bit for bit
// (tools/lane_diff.py); a divisor that is a compile-time constant in the order-specialised forms
// but not in the lane form must go through fdiv_c with its folded reciprocal (tq_ra3) or a runtime
// 1.0 (BdfState::unity), since the compiler folds v_rcp_f64 of a constant to the correctly rounded
// value. The GPU-vs-CPU llh parity envelope (tests/parity.py) holds for both (512 C3 draws:
// 99.6 % within 1e-8 fast, 99.4 % correctly rounded).

// Default (round 3): the correctly rounded forms -- the reference's IEEE quotients, and the GPU's
// llh agreement with the reference CVODE then meets the reference's own FMA on/off spread (4,096
// C3 draws: 99.05 % within 1e-8 vs 98.88 % with the one-step forms; profiles/r03_parity_variants.txt).
// -DBCM3_FAST_DIV selects the one-Newton-step forms (tools/build_variant.sh).
#if !defined(BCM3_FAST_DIV) && !defined(BCM3_CORRECTLY_ROUNDED)
#define BCM3_CORRECTLY_ROUNDED
#endif

// reciprocal
BDF_INL double frcp(double b)
{
    double r = __builtin_amdgcn_rcp(b);
    double e = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(e, r, r);
#ifndef BCM3_CORRECTLY_ROUNDED
    return r;
#else
    e = __builtin_fma(-b, r, 1.0);
    return __builtin_fma(e, r, r);
#endif
}
// a / b: a times the one-step reciprocal (correctly rounded: + one residual correction of the
// quotient)
BDF_INL double fdiv(double a, double b)
{
    double r = __builtin_amdgcn_rcp(b);
    const double e0 = __builtin_fma(-b, r, 1.0);
    r = __builtin_fma(e0, r, r);
    const double q = a * r;
#ifndef BCM3_CORRECTLY_ROUNDED
    return q;
#else
    const double e = __builtin_fma(-b, q, a);
    return __builtin_fma(e, r, q);
#endif
}
// SUNRsqrt: x <= 0 -> 0; v_rsq_f64 estimate + one Goldschmidt step (correctly rounded: + one
// correction). Branch-free: the refinement runs for every x (x <= 0 gives NaN there) and x <= 0
// is zeroed with a bit mask, NaN passes through (a select here is turned back into a branch by
// the compiler).
BDF_INL double fsqrt(double x)
{
    double r = __builtin_amdgcn_rsq(x);
    double g = x * r, hh = 0.5 * r;
    double e = __builtin_fma(-g, hh, 0.5);
    g = __builtin_fma(g, e, g);
#ifdef BCM3_CORRECTLY_ROUNDED
    hh = __builtin_fma(hh, e, hh);
    const double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, hh, g);
#endif
    const long long keep = (x <= 0.0) ? 0LL : -1LL;
    return __builtin_bit_cast(double, __builtin_bit_cast(long long, g) & keep);
}
// a / b for a compile-time b with rb = 1/b correctly rounded: a * rb (correctly rounded: + the
// residual correction of fdiv)
BDF_INL double fdiv_c(double a, double b, double rb)
{
    const double q = a * rb;
#ifndef BCM3_CORRECTLY_ROUNDED
    return q;
#else
    const double e = __builtin_fma(-b, q, a);
    return __builtin_fma(e, rb, q);
#endif
}

// 1/j for j = 1..7 (the correctly rounded quotients 1.0/j)
BDF_INL double recip_int(int j)
{
    double r = 1.0;
    r = (j == 2) ? 0.5 : r;
    r = (j == 3) ? 0.33333333333333331 : r;
    r = (j == 4) ? 0.25 : r;
    r = (j == 5) ? 0.2 : r;
    r = (j == 6) ? 0.16666666666666666 : r;
    r = (j == 7) ? 0.14285714285714285 : r;
    return r;
}

// A3 of cvSetTqBDF (cvode.c:2620) depends on q alone: alpha0 + 1/q with alpha0 = -sum_{j<=q} 1/j,
// evaluated in the same order as set_bdf. The divisor of Cpinv is therefore a compile-time
// constant in the order-specialised solvers and a runtime value in the lane solver; dividing by
// it through fdiv_c with the constant reciprocal keeps the three forms bit-identical (the
// hardware reciprocal estimate differs from the compiler's folded 1.0 / A3).
constexpr double tq_a3(int q)
{
    double a = -1.0;
    for (int j = 2; j < q; j++) a -= 1.0 / j;
    a -= 1.0 / q;
    return a + 1.0 / q;
}
BDF_INL double tq_ra3(int q)
{
    double r = 1.0 / tq_a3(2);
    r = (q == 3) ? 1.0 / tq_a3(3) : r;
    r = (q == 4) ? 1.0 / tq_a3(4) : r;
    r = (q == 5) ? 1.0 / tq_a3(5) : r;
    return r;
}

// eta = 1 / (pow(bias*x, 1/k) + ADDON)  (cvode.c:2996, 3101, 3160, 3185), SUNRpowerR(x, 1/k)
// with x <= 0 -> 0 (sundials_math.c:40-52), k in 2..7.
// Division-free Newton iteration for z = x^(-1/k) (z <- z + z (1 - x z^k) / k) from a
// single-precision log2/exp2 seed; eta = z / (1 + ADDON z). Two iterations reach double
// accuracy from the ~2^-22 seed. Outside [1e-30, 1e30] (never on the solver's paths in
// practice) the library pow is used.
BDF_INL double eta_from(double bx, int k)
{
    if (!(bx > 1e-30 && bx < 1e30)) return frcp((bx > 0.0 ? pow(bx, recip_int(k)) : 0.0) + ADDON);
    const double rk = recip_int(k);
    const float lf = __builtin_amdgcn_logf((float)bx);  // log2
    double z = (double)__builtin_amdgcn_exp2f(-lf * (float)rk);
    cfor<0, 2>([&](auto) __attribute__((always_inline)) {
        double zk = z;  // z^k, k >= 2
        cfor<2, 8>([&](auto I) __attribute__((always_inline)) {
            if (CI(I) <= k) zk *= z;
        });
        const double t = __builtin_fma(-bx, zk, 1.0);
        z = __builtin_fma(z * t, rk, z);
    });
    return fdiv(z, __builtin_fma(ADDON, z, 1.0));
}

// The PopPK solvers (bdf_lane.h cvode_one_step, bdf_uni.h, bdf_vec.h) compute every quantity
// of the step with the reference's own operations: the products and sums of its C statements
// in their order (no contraction: the reference is compared against its build without FMA
// contraction, oracle/_ref/libbcm3ref_nofma.so, which the C restatement matches bit for bit),
// IEEE quotients and square roots (frcp / fdiv / fsqrt above, correctly rounded), and libm's
// pow through xm::pow_glibc (libm_exact.h). The cell-population solver keeps eta_from.

// SUNRpowerR(bx, fl(1/k)) (sundials_math.c:40-52, libm's pow)
// with the tables popk_prepare_device uploaded (xm::xm_tables: the host libm's own, so that the
// roots are glibc's results bit for bit, or computed ones of the same layout, ~1 ulp)
#ifdef BCM3_TABLES_LDS
// (variant) a workgroup copy of the tables in LDS, filled at kernel entry (popk_traj_kernel)
static __shared__ xm::GlibcPow lds_tables;
#define BDF_ROOT_TABLES lds_tables
#else
#define BDF_ROOT_TABLES xm::xm_tables
#endif
// SUNRpowerR's pow: glibc's table-driven pow (the tables popk_prepare_device uploaded). Measured
// against the alternatives on one box (profiles/r04n_variants.txt, 256 C3 draws): the correctly
// rounded Newton root alone is 6 % faster but not glibc's result on ~0.07 % of roots; checking it
// against the rounding midpoints and falling back to glibc's pow near them (BCM3_ROOT_HYBRID,
// xm::pow_inv_k_checked) is glibc's result everywhere but 4 % slower than this -- two root code
// paths inlined at every call site cost more than the table loads.
#ifdef BCM3_ROOT_CALL
__device__ __attribute__((noinline)) double pow_glibc_call(double bx, int k)
{
    return xm::pow_glibc(bx, xm::inv_k(k), BDF_ROOT_TABLES);
}
#endif
BDF_INL double pow_root(double bx, int k)
{
#ifdef BCM3_ROOT_LEAN
    // the tables are always uploaded before a launch (popk_prepare_device: the loaded libm's, else
    // computed ones of the same layout, ok = 1 either way), so every finite bx > 0 takes glibc's
    // algorithm (subnormal bx normalised as e_pow.c does); SUNRpowerR's base <= 0 -> 0 and pow's
    // inf -> inf, NaN -> NaN by selects: one straight-line copy per call site
    const bool fin = (bx > 0.0) & (bx < __builtin_inf());
    const double p = xm::pow_glibc_pos(fin ? bx : 1.0, xm::inv_k(k), BDF_ROOT_TABLES);
    return fin ? p : ((bx > 0.0) ? bx : ((bx == bx) ? 0.0 : bx + bx));
#endif
#if defined(BCM3_ROOT_HYBRID) || defined(BCM3_ROOT_CALL) || defined(BCM3_ROOT_CR)
    if (BDF_LIKELY((bx > 1e-30) & (bx < 1e30))) {
        bool safe;
        const double p = xm::pow_inv_k_checked(bx, k, safe);
#if defined(BCM3_ROOT_CALL)
        if (BDF_UNLIKELY(!safe & (BDF_ROOT_TABLES.ok != 0))) return pow_glibc_call(bx, k);
#elif defined(BCM3_ROOT_HYBRID)
        if (BDF_UNLIKELY(!safe & (BDF_ROOT_TABLES.ok != 0))) return xm::pow_glibc(bx, xm::inv_k(k), BDF_ROOT_TABLES);
#endif
        return p;
    }
#endif
    if (BDF_LIKELY(BDF_ROOT_TABLES.ok & (bx >= 0x1p-1022) & (bx < 0x1p1023)))
        return xm::pow_glibc(bx, xm::inv_k(k), BDF_ROOT_TABLES);
    if (bx > 1e-30 && bx < 1e30) return xm::pow_inv_k(bx, k);
    return (bx > 0.0) ? pow(bx, xm::inv_k(k)) : 0.0;
}

// eta = ONE / (SUNRpowerR(bx, ONE / k) + ADDON) (cvode.c:2986, 3105, 3163, 3187): the rounded
// exponent fl(1/k) as the reference passes it, libm's pow, the IEEE quotient
BDF_INL double eta_exact(double bx, int k)
{
    if constexpr (BDF_DBL(1)) bdf_consume(frcp(pow_root(bdf_launder(bx), k) + ADDON));
    return frcp(pow_root(bx, k) + ADDON);
}

// cvNlsConvTest (cvode_nls.c:262-263): dcon = del * min(1, crate) / tol, converged when dcon <= 1,
// tol = tq[4] = CORTES / tq[2]. RN(a / b) <= 1 iff a / b <= 1 + 2^-53 (the midpoint rounds to even,
// i.e. to 1) iff a <= b: for finite b > 0 no double lies in (b, b (1 + 2^-53)] (the successor of b
// is b (1 + 2^-52 / m), mantissa m < 2). a >= 0 or NaN (false).
BDF_INL bool div_le_one(double a, double b) { return a <= b; }

// SUNRpowerI for exponent 1..7 (repeated multiplication, sundials_math.c:28-38)
BDF_INL double powI(double base, int e)
{
    double prod = 1.0;
    cfor<1, QMAX + 3>([&](auto I) __attribute__((always_inline)) {
        if (CI(I) <= e) prod *= base;
    });
    return prod;
}

// Runtime-indexed read of a small register array as a chain of constant-index selects whose
// first link selects against a constant: a select between TWO loads would be folded by
// InstCombine (run on this function before it is inlined into the kernel, where the array is
// still behind a pointer) into a load through a selected pointer, and the state array could no
// longer be promoted to registers.
template <int K>
BDF_INL double sel(const double (&a)[K], int i)
{
    double r = 0.0;
    cfor<0, K>([&](auto k) __attribute__((always_inline)) { r = (i == CI(k)) ? a[CI(k)] : r; });
    return r;
}
template <int NS>
BDF_INL void sel_row(const double (&zn)[QMAX + 1][NS], int q, double (&r)[NS])
{
    cfor<0, NS>([&](auto i) __attribute__((always_inline)) {
        double v = 0.0;
        cfor<1, QMAX + 1>([&](auto j) __attribute__((always_inline)) { v = (q == CI(j)) ? zn[CI(j)][CI(i)] : v; });
        r[CI(i)] = v;
    });
}

// BCM3_PHASES (profiling build only): per-phase s_memtime cycle accumulators
#ifdef BCM3_PHASES
#define BDF_PH(k)                                  \
    do {                                           \
        __builtin_amdgcn_sched_barrier(0);         \
        const unsigned t_ = (unsigned)clock64();   \
        s.ph[k] += t_ - s.tlast;                   \
        s.tlast = t_;                              \
        __builtin_amdgcn_sched_barrier(0);         \
    } while (0)
// the fast loop's cycles of a whole step, split by kind (plain / recomputing) via selects
#define BDF_PH_STEP(t0, kp, kg, c)                     \
    do {                                               \
        __builtin_amdgcn_sched_barrier(0);             \
        const unsigned d_ = (unsigned)clock64() - (t0); \
        s.ph[kp] += (c) ? d_ : 0u;                     \
        s.ph[kg] += (c) ? 0u : d_;                     \
        __builtin_amdgcn_sched_barrier(0);             \
    } while (0)
#define BDF_PH_NOW() ((unsigned)clock64())
// cycles since t0 into ph[k] (the running phase clock tlast is left alone), and event counts
#define BDF_PH_ADD(k, t0)                               \
    do {                                                \
        __builtin_amdgcn_sched_barrier(0);              \
        s.ph[k] += (unsigned)clock64() - (t0);          \
        __builtin_amdgcn_sched_barrier(0);              \
    } while (0)
#define BDF_PH_CNT(k, c) (s.ph[k] += (c) ? 1u : 0u)
#elif defined(BCM3_MARKS)
// ISA study build: a comment per phase boundary in the -S output (tools/step_isa.py)
#define BDF_PH(k) asm volatile("; BDFMARK %0" ::"i"(k))
#endif
#ifndef BDF_PH
#define BDF_PH(k) \
    do {          \
    } while (0)
#endif
#ifndef BDF_PH_STEP
#define BDF_PH_STEP(t0, kp, kg, c) \
    do {                           \
    } while (0)
#define BDF_PH_NOW() 0u
#define BDF_PH_ADD(k, t0) \
    do {                  \
    } while (0)
#define BDF_PH_CNT(k, c) \
    do {                 \
    } while (0)
#endif
// 32-bit cycle accumulators (wrapping differences of the low word), so that the profiling build
// adds few scalar registers. 0-9: the general step (tools/phase_probe.py NAMES); 10-17: the phases
// of a plain fast-loop step (vec::fast_run, coefficients held); 18: the loop's exit test and back
// edge (every fast-loop step); 19/20: whole plain / recomputing fast-loop steps; 21/22: their
// counts; 23: the marker's own cost (16 back-to-back markers per trajectory); 24-26: the
// convergence test and completion of a recomputing fast-loop step; 28-31 (vec::complete_eta_q):
// order-change checks due, checks the screen skipped, cycles in the screen, cycles in the exact
// evaluation
constexpr int NPHASES = 32;

struct BdfCounters {
    int nst_total, nfe, nni, nsetups, nje, netf, ncfn, nreinit;
};

// Model concept (see popk_kernel.hip):
//   static constexpr int NS;
//   BDF_INL void rhs(double t, const double (&y)[NS], double (&ydot)[NS]) const;
//   typename Model::Inv                                  structured (I - gamma J)^-1 storage
//   BDF_INL void lin_setup(double gamma, Inv& inv) const;  inverse as sunlinsol_dense_eigen
//   BDF_INL void lin_solve(const Inv& inv, const double (&b)[NS], double (&x)[NS]) const;
template <int NS, class Inv>
struct BdfState {
    double rtol, atol;
    double unity;  // 1.0 the compiler cannot see (see set_bdf_q in bdf_vec.h)
    double zn[QMAX + 1][NS];
    double ewt[NS], acor[NS];
    Inv inv;
    double tau[QMAX + 2], tq[6], l[QMAX + 1];
    double tn, h, hprime, eta, hscale, hu, tretlast;
    double gamma, gammap, gamrat, crate, delp, acnrm, etamax, saved_tq5;
    double tstop;
    int tstopset;
    int q, qprime, qwait, L;
    int nst, nstlp, nstlj;
    int nls_jcur;
    int check_tolsf;  // 0: the too-much-accuracy test cannot fire (rtol >= 1e-10, atol >= 0)
    BdfCounters cnt;
#ifdef BCM3_PHASES
    unsigned ph[NPHASES];
    unsigned tlast;
    int qh[QMAX + 1];  // successful steps per order
#endif
};

template <int NS>
BDF_INL double wrms(const double (&x)[NS], const double (&w)[NS])
{
    // sum of rounded squares in component order (the lane-vector solver sums the same way)
    double s = 0.0;
    cfor<0, NS>([&](auto i) __attribute__((always_inline)) {
        const double p = x[CI(i)] * w[CI(i)];
        const double p2 = p * p;
        s = (CI(i) == 0) ? p2 : s + p2;
    });
    return fsqrt(fdiv_c(s, (double)NS, 1.0 / NS));
}

// cvEwtSetSV: w = 1/(rtol*|y| + atol)
template <int NS, class S>
BDF_INL void ewt_set(const S& s, const double (&ycur)[NS], double (&w)[NS])
{
    cfor<0, NS>([&](auto i) __attribute__((always_inline)) { w[CI(i)] = frcp(s.rtol * fabs(ycur[CI(i)]) + s.atol); });
}

// cvRescale (cvode.c:2393-2406): zn[j] *= eta^j, j = 1..q
template <int NS, class S>
BDF_INL void rescale(S& s)
{
    double c = s.eta;
    cfor<1, QMAX + 1>([&](auto j) __attribute__((always_inline)) {
        if (CI(j) <= s.q) {
            cfor<0, NS>([&](auto i) __attribute__((always_inline)) { s.zn[CI(j)][CI(i)] *= c; });
        }
        c = s.eta * c;
    });
    s.h = s.hscale * s.eta;
    s.hscale = s.h;
}

// cvPredict (BCM: N_VAdd(zn[j-1], zn[j]) -> zn[j-1] += zn[j]), tstop clamp of tn
template <int NS, class S>
BDF_INL void predict(S& s)
{
    s.tn += s.h;
    if (s.tstopset) {
        if ((s.tn - s.tstop) * s.h > 0.0) s.tn = s.tstop;
    }
    cfor<1, QMAX + 1>([&](auto k) __attribute__((always_inline)) {
        cfor_down<QMAX, CI(k)>([&](auto j) __attribute__((always_inline)) {
            if (CI(j) <= s.q) {
                cfor<0, NS>([&](auto i) __attribute__((always_inline)) { s.zn[CI(j) - 1][CI(i)] += s.zn[CI(j)][CI(i)]; });
            }
        });
    });
}

// cvRestore: zn[j-1] += (-1)*zn[j]
template <int NS, class S>
BDF_INL void restore(S& s, double saved_t)
{
    s.tn = saved_t;
    cfor<1, QMAX + 1>([&](auto k) __attribute__((always_inline)) {
        cfor_down<QMAX, CI(k)>([&](auto j) __attribute__((always_inline)) {
            if (CI(j) <= s.q) {
                cfor<0, NS>([&](auto i) __attribute__((always_inline)) { s.zn[CI(j) - 1][CI(i)] -= s.zn[CI(j)][CI(i)]; });
            }
        });
    });
}

// cvSetBDF + cvSetTqBDF + cvSet (cvode.c:2445-2690); returns rl1
template <class S>
BDF_INL double set_bdf(S& s)
{
    const int q = s.q;
    double alpha0, alpha0_hat, xi_inv, xistar_inv, hsum;
    s.l[0] = s.l[1] = xi_inv = xistar_inv = 1.0;
    cfor<2, QMAX + 1>([&](auto i) __attribute__((always_inline)) {
        if (CI(i) <= q) s.l[CI(i)] = 0.0;
    });
    alpha0 = alpha0_hat = -1.0;
    hsum = s.h;
    if (q > 1) {
        cfor<2, QMAX>([&](auto j) __attribute__((always_inline)) {
            if (CI(j) < q) {
                hsum += s.tau[CI(j) - 1];
                xi_inv = fdiv(s.h, hsum);
                alpha0 -= 1.0 / CI(j);
                cfor_down<CI(j), 1>([&](auto i) __attribute__((always_inline)) { s.l[CI(i)] = s.l[CI(i)] + s.l[CI(i) - 1] * xi_inv; });
            }
        });
        alpha0 -= recip_int(q);
        xistar_inv = -s.l[1] - alpha0;
        hsum += sel(s.tau, q - 1);
        xi_inv = fdiv(s.h, hsum);
        alpha0_hat = -s.l[1] - xi_inv;
        cfor_down<QMAX, 1>([&](auto i) __attribute__((always_inline)) {
            if (CI(i) <= q) s.l[CI(i)] = s.l[CI(i)] + s.l[CI(i) - 1] * xistar_inv;
        });
    }
    // cvSetTqBDF
    const double A1 = 1.0 - alpha0_hat + alpha0;
    const double A2 = 1.0 + (double)q * A1;
    const double lq = sel(s.l, q);
    s.tq[2] = fabs(fdiv(A1, alpha0 * A2));
    s.tq[5] = fabs(fdiv(A2 * xistar_inv, lq * xi_inv));
    if (s.qwait == 1) {
        if (q > 1) {
            const double C = fdiv(xistar_inv, lq);
            const double A3 = alpha0 + recip_int(q);
            const double A4 = alpha0_hat + xi_inv;
            const double Cpinv = fdiv_c(1.0 - A4 + A3, A3, tq_ra3(q));
            s.tq[1] = fabs(C * Cpinv);
        } else {
            s.tq[1] = 1.0;
        }
        hsum += sel(s.tau, q);
        xi_inv = fdiv(s.h, hsum);
        const double A5 = alpha0 - recip_int(q + 1);
        const double A6 = alpha0_hat - xi_inv;
        const double Cppinv = fdiv(1.0 - A6 + A5, A2);
        s.tq[3] = fabs(fdiv(Cppinv, xi_inv * (double)(q + 2) * A5));
    }
    s.tq[4] = fdiv(CORTES, s.tq[2]);
    // cvSet
    const double rl1 = frcp(s.l[1]);
    s.gamma = s.h * rl1;
    if (s.nst == 0) s.gammap = s.gamma;
    s.gamrat = (s.nst > 0) ? fdiv(s.gamma, s.gammap) : 1.0;
    return rl1;
}

// cvIncreaseBDF (cvode.c:2310-2340); indx_acor == QMAX always
template <int NS, class S>
BDF_INL void increase_bdf(S& s)
{
    double alpha0, alpha1, prod, xi, xiold, hsum, A1;
    double l[QMAX + 1];
    cfor<0, QMAX + 1>([&](auto i) __attribute__((always_inline)) { l[CI(i)] = 0.0; });
    l[2] = alpha1 = prod = xiold = 1.0;
    alpha0 = -1.0;
    hsum = s.hscale;
    // j < q <= QMAX - 1: an order increase never starts from QMAX
    cfor<1, QMAX - 1>([&](auto j) __attribute__((always_inline)) {
        if (CI(j) < s.q) {
            hsum += s.tau[CI(j) + 1];
            xi = fdiv(hsum, s.hscale);
            prod *= xi;
            alpha0 -= 1.0 / (CI(j) + 1);
            alpha1 += frcp(xi);
            cfor_down<CI(j) + 2, 2>([&](auto i) __attribute__((always_inline)) { l[CI(i)] = l[CI(i)] * xiold + l[CI(i) - 1]; });
            xiold = xi;
        }
    });
    A1 = fdiv(-alpha0 - alpha1, prod);
    // zn[L] = A1 * zn[QMAX]; zn[j] += l[j]*zn[L], j = 2..q  (L = q+1)
    double znL[NS];
    cfor<0, NS>([&](auto i) __attribute__((always_inline)) { znL[CI(i)] = A1 * s.zn[QMAX][CI(i)]; });
    cfor<2, QMAX + 1>([&](auto j) __attribute__((always_inline)) {
        if (CI(j) == s.q + 1) {
            cfor<0, NS>([&](auto i) __attribute__((always_inline)) { s.zn[CI(j)][CI(i)] = znL[CI(i)]; });
        } else if (CI(j) <= s.q) {
            cfor<0, NS>([&](auto i) __attribute__((always_inline)) { s.zn[CI(j)][CI(i)] = s.zn[CI(j)][CI(i)] + l[CI(j)] * znL[CI(i)]; });
        }
    });
    cfor<0, QMAX + 1>([&](auto i) __attribute__((always_inline)) { s.l[CI(i)] = l[CI(i)]; });
}

// cvDecreaseBDF (cvode.c:2352-2375)
template <int NS, class S>
BDF_INL void decrease_bdf(S& s)
{
    double l[QMAX + 1];
    cfor<0, QMAX + 1>([&](auto i) __attribute__((always_inline)) { l[CI(i)] = 0.0; });
    l[2] = 1.0;
    double hsum = 0.0;
    cfor<1, QMAX - 1>([&](auto j) __attribute__((always_inline)) {
        if (CI(j) <= s.q - 2) {
            hsum += s.tau[CI(j)];
            const double xi = fdiv(hsum, s.hscale);
            cfor_down<CI(j) + 2, 2>([&](auto i) __attribute__((always_inline)) { l[CI(i)] = l[CI(i)] * xi + l[CI(i) - 1]; });
        }
    });
    double znq[NS];
    sel_row<NS>(s.zn, s.q, znq);
    cfor<2, QMAX>([&](auto j) __attribute__((always_inline)) {
        if (CI(j) < s.q) {
            cfor<0, NS>([&](auto i) __attribute__((always_inline)) { s.zn[CI(j)][CI(i)] = s.zn[CI(j)][CI(i)] + (-l[CI(j)]) * znq[CI(i)]; });
        }
    });
    cfor<0, QMAX + 1>([&](auto i) __attribute__((always_inline)) { s.l[CI(i)] = l[CI(i)]; });
}

// cvAdjustOrder (cvode.c:2212-2225)
template <int NS, class S>
BDF_INL void adjust_order(S& s, int deltaq)
{
    if ((s.q == 2) && (deltaq != 1)) return;
    if (deltaq == 1)
        increase_bdf<NS>(s);
    else if (deltaq == -1)
        decrease_bdf<NS>(s);
}

// CVodeGetDky(t, k = 0) (cvode.c:1467-1533): z = sum_{j=q..0} s^j zn[j], the first term a product
// (N_VLinearCombination / N_VLinearSum of the Eigen N_Vector, nvector_serial_eigen.cpp)
template <int NS, class S>
BDF_INL int get_dky(const S& s, double t, double (&dky)[NS])
{
    double tfuzz = FUZZ_FACTOR * UROUND * (fabs(s.tn) + fabs(s.hu));
    if (s.hu < 0.0) tfuzz = -tfuzz;
    const double tp = s.tn - s.hu - tfuzz;
    const double tn1 = s.tn + tfuzz;
    if ((t - tp) * (t - tn1) > 0.0) return CV_BAD_T;
    const double sv = fdiv(t - s.tn, s.h);
    double c[QMAX + 1];
    c[0] = 1.0;
    cfor<1, QMAX + 1>([&](auto j) __attribute__((always_inline)) { c[CI(j)] = c[CI(j) - 1] * sv; });
    cfor<0, NS>([&](auto i) __attribute__((always_inline)) { dky[CI(i)] = 0.0; });
    cfor_down<QMAX, 0>([&](auto j) __attribute__((always_inline)) {
        if (CI(j) == s.q) {
            cfor<0, NS>([&](auto i) __attribute__((always_inline)) { dky[CI(i)] = c[CI(j)] * s.zn[CI(j)][CI(i)]; });
        } else if (CI(j) < s.q) {
            cfor<0, NS>([&](auto i) __attribute__((always_inline)) { dky[CI(i)] = dky[CI(i)] + c[CI(j)] * s.zn[CI(j)][CI(i)]; });
        }
    });
    return CV_SUCCESS;
}

// CVodeReInit (cvode.c:586-683): tau, saved_tq5, tstop persist.
template <int NS, class S>
BDF_INL void reinit(S& s, double t0, const double (&y0)[NS])
{
    s.tn = t0;
    s.q = 1;
    s.L = 2;
    s.qwait = 2;
    s.etamax = ETAMX1;
    s.hu = 0.0;
    cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
        constexpr int i = CI(I_);
        s.zn[0][i] = y0[i];
    });
    s.nst = 0;
    s.nstlp = 0;
    s.cnt.nreinit++;
}

// Newton iteration of cvNls (cvode.c:2701-2770) = SUNNonlinSolSolve_Newton
// (sunnonlinsol_newton.c:183-322) + cvNlsResidual + cvNlsLSetup/cvLsSetup + cvLsSolve +
// cvNlsConvTest. One residual call site. Returns true on convergence.
template <int NS, class S, class Model>
BDF_INL bool newton(S& s, const Model& mdl, double rl1, int convfail, bool callSetup)
{
    bool jbad = false;
    // 2/(1+gamrat) scaling of cvLsSolve: constant within the solve, 1 after a setup
    double cscale = (s.gamrat != 1.0) ? fdiv(2.0, 1.0 + s.gamrat) : 1.0;
    int curiter = 0;
    for (;;) {
        // residual: y = zn0 + ycor; f(tn, y); res = rl1*zn1 + ycor; res += -gamma*f
        double y[NS], f[NS], delta[NS];
        cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
            constexpr int i = CI(I_);
            y[i] = s.zn[0][i] + s.acor[i];
        });
        mdl.rhs(s.tn, y, f);
        s.cnt.nfe++;
        cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
            constexpr int i = CI(I_);
            delta[i] = rl1 * s.zn[1][i] + s.acor[i];
            delta[i] = delta[i] + (-s.gamma) * f[i];
        });
        if (callSetup) {
            // cvNlsLSetup -> cvLsSetup (cvode_ls.c:1415-1500)
            if (jbad) convfail = CONV_BAD_J;
            const double dgamma = fabs(fdiv(s.gamma, s.gammap) - 1.0);
            const bool jnew = (s.nst == 0) || (s.nst > s.nstlj + CVLS_MSBJ) ||
                              ((convfail == CONV_BAD_J) && (dgamma < CVLS_DGMAX)) || (convfail == CONV_OTHER);
            if (jnew) {
                s.cnt.nje++;
                s.nstlj = s.nst;
            }
            mdl.lin_setup(s.gamma, s.inv);  // A = I - gamma*J, closed-form inverse
            s.cnt.nsetups++;
            s.nls_jcur = jnew;
            s.gamrat = 1.0;
            cscale = 1.0;
            s.gammap = s.gamma;
            s.crate = 1.0;
            s.nstlp = s.nst;
            callSetup = false;
            curiter = 0;
        }
        s.cnt.nni++;
        // cvLsSolve: x = A^-1 (-res); scale by 2/(1+gamrat) when gamma changed
        double b[NS], x[NS];
        cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
            constexpr int i = CI(I_);
            b[i] = -delta[i];
        });
        mdl.lin_solve(s.inv, b, x);
        if (s.gamrat != 1.0) {
            const double c = cscale;
            cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
                constexpr int i = CI(I_);
                x[i] *= c;
            });
        }
        cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
            constexpr int i = CI(I_);
            s.acor[i] += x[i];
        });
        // cvNlsConvTest (cvode_nls.c:236-280)
        const double del = wrms<NS>(x, s.ewt);
        if (curiter > 0) s.crate = SUNMAX(CRDOWN * s.crate, fdiv(del, s.delp));
        // cvNlsConvTest: dcon = del min(1, crate) / tq[4] <= 1
        if (div_le_one(del * SUNMIN(1.0, s.crate), s.tq[4])) {
            s.acnrm = (curiter == 0) ? del : wrms<NS>(s.acor, s.ewt);
            s.nls_jcur = 0;
            return true;
        }
        bool fail = (curiter >= 1) && (del > RDIV * s.delp);
        if (!fail) {
            s.delp = del;
            curiter++;
            fail = (curiter >= NLS_MAXCOR);
            if (!fail) continue;
        }
        if (!s.nls_jcur) {  // retry with a fresh Jacobian (jbad)
            callSetup = true;
            jbad = true;
            cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
                constexpr int i = CI(I_);
                s.acor[i] = 0.0;
            });
            continue;
        }
        return false;
    }
}

// cvHin (cvode.c:1884-1990); the models' RHS never fails recoverably
template <int NS, class S, class Model>
BDF_INL int hin(S& s, const Model& mdl, double tout)
{
    const double tdiff = tout - s.tn;
    if (tdiff == 0.0) return CV_TOO_CLOSE;
    const int sign = (tdiff > 0.0) ? 1 : -1;
    const double tdist = fabs(tdiff);
    const double tround = UROUND * SUNMAX(fabs(s.tn), fabs(tout));
    if (tdist < 2.0 * tround) return CV_TOO_CLOSE;
    const double hlb = HLB_FACTOR * tround;
    // cvUpperBoundH0 (cvode.c:2000-2035)
    double hub_inv = 0.0;
    cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
        constexpr int i = CI(I_);
        double t1 = frcp(s.ewt[i]);  // N_VInv of the error weights
        t1 = t1 + HUB_FACTOR * fabs(s.zn[0][i]);
        const double r = fdiv(fabs(s.zn[1][i]), t1);
        hub_inv = (i == 0) ? r : ((r > hub_inv) ? r : hub_inv);  // maxCoeff
    });
    double hub = HUB_FACTOR * tdist;
    if (hub * hub_inv > 1.0) hub = frcp(hub_inv);
    double hg = fsqrt(hlb * hub);
    if (hub < hlb) {
        s.h = (sign == -1) ? -hg : hg;
        return CV_SUCCESS;
    }
    double hnew = hg;
#pragma unroll 1
    for (int count1 = 1; count1 <= MAX_ITERS; count1++) {
        // cvYddNorm (cvode.c:2046-2066)
        const double hgs = hg * sign;
        double yy[NS], tv[NS];
        cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
            constexpr int i = CI(I_);
            yy[i] = hgs * s.zn[1][i] + s.zn[0][i];
        });
        mdl.rhs(s.tn + hgs, yy, tv);
        s.cnt.nfe++;
        const double a = frcp(hgs);
        cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
            constexpr int i = CI(I_);
            tv[i] = a * (tv[i] - s.zn[1][i]);
        });
        const double yddnrm = wrms<NS>(tv, s.ewt);
        hnew = (yddnrm * hub * hub > 2.0) ? fsqrt(fdiv(2.0, yddnrm)) : fsqrt(hg * hub);
        if (count1 == MAX_ITERS) break;
        const double hrat = fdiv(hnew, hg);
        if ((hrat > 0.5) && (hrat < 2.0)) break;
        if ((count1 > 1) && (hrat > 2.0)) {
            hnew = hg;
            break;
        }
        hg = hnew;
    }
    double h0 = H_BIAS * hnew;
    if (h0 < hlb) h0 = hlb;
    if (h0 > hub) h0 = hub;
    if (sign == -1) h0 = -h0;
    s.h = h0;
    return CV_SUCCESS;
}

// CVode(..., CV_ONE_STEP) (cvode.c:1006-1443) with cvStep (cvode.c:2082-2174) inlined as an
// attempt loop with single rescale / restore / Newton call sites.
template <int NS, class S, class Model>
BDF_INL int cvode_one_step(S& s, const Model& mdl, double tout, double (&yout)[NS], double& tret)
{
    BDF_PH(0);  // driver: output interpolation, callbacks, ReInit
    if (s.nst == 0) {
        s.tretlast = tret = s.tn;
        ewt_set<NS>(s, s.zn[0], s.ewt);
        s.nstlj = 0;     // cvLsInitializeCounters
        s.nls_jcur = 0;  // SUNNonlinSolInitialize_Newton
        mdl.rhs(s.tn, s.zn[0], s.zn[1]);
        s.cnt.nfe++;
        if (s.tstopset) {
            if ((s.tstop - s.tn) * (tout - s.tn) <= 0.0) return CV_ILL_INPUT;
        }
        double tout_hin = tout;
        if (s.tstopset && (tout - s.tn) * (tout - s.tstop) > 0.0) tout_hin = s.tstop;
        const int hflag = hin<NS>(s, mdl, tout_hin);
        if (hflag != CV_SUCCESS) return hflag;
        if (s.tstopset) {
            if ((s.tn + s.h - s.tstop) * s.h > 0.0) s.h = (s.tstop - s.tn) * (1.0 - 4.0 * UROUND);
        }
        s.hscale = s.h;
        s.hprime = s.h;
        cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
            constexpr int i = CI(I_);
            s.zn[1][i] *= s.h;
        });
    } else {
        const double troundoff = FUZZ_FACTOR * UROUND * (fabs(s.tn) + fabs(s.h));
        if (fabs(s.tn - s.tretlast) > troundoff) {
            s.tretlast = tret = s.tn;
            cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
                constexpr int i = CI(I_);
                yout[i] = s.zn[0][i];
            });
            return CV_SUCCESS;
        }
        if (s.tstopset) {
            if (fabs(s.tn - s.tstop) <= troundoff) {
                if (get_dky<NS>(s, s.tstop, yout) != CV_SUCCESS) return CV_ILL_INPUT;
                s.tretlast = tret = s.tstop;
                s.tstopset = 0;
                return CV_TSTOP_RETURN;
            }
            if ((s.tn + s.hprime - s.tstop) * s.h > 0.0) {
                s.hprime = (s.tstop - s.tn) * (1.0 - 4.0 * UROUND);
                s.eta = fdiv(s.hprime, s.h);
            }
        }
        ewt_set<NS>(s, s.zn[0], s.ewt);
    }
    // too much accuracy requested (cvode.c:1318-1331): uround * wrms(zn0) > 1
    {
        double ss = 0.0;
        cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
            constexpr int i = CI(I_);
            const double p = s.zn[0][i] * s.ewt[i];
            ss = (i == 0) ? p * p : ss + p * p;
        });
        if (ss > (double)NS * (1.0 / (UROUND * UROUND))) {
            s.tretlast = tret = s.tn;
            cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
                constexpr int i = CI(I_);
                yout[i] = s.zn[0][i];
            });
            return CV_TOO_MUCH_ACC;
        }
    }

    BDF_PH(1);  // entry checks, error weights
    // ---------------- cvStep
    const double saved_t = s.tn;
    int ncf = 0, nef = 0, nflag = FIRST_CALL;
    bool do_rescale = false;
    if ((s.nst > 0) && (s.hprime != s.h)) {
        // cvAdjustParams
        if (s.qprime != s.q) {
            adjust_order<NS>(s, s.qprime - s.q);
            s.q = s.qprime;
            s.L = s.q + 1;
            s.qwait = s.L;
        }
        do_rescale = true;
    }
    double dsm = 0.0;
    for (;;) {
        if (do_rescale) rescale<NS>(s);
        do_rescale = true;
        BDF_PH(2);
        predict<NS>(s);
        BDF_PH(3);
        const double rl1 = set_bdf(s);
        BDF_PH(4);
        // cvNls
        const int convfail = ((nflag == FIRST_CALL) || (nflag == PREV_ERR_FAIL)) ? CONV_NONE : CONV_OTHER;
        const bool callSetup = (nflag == PREV_CONV_FAIL) || (nflag == PREV_ERR_FAIL) || (s.nst == 0) ||
                               (s.nst >= s.nstlp + MSBP) || (fabs(s.gamrat - 1.0) > DGMAX);
        cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
            constexpr int i = CI(I_);
            s.acor[i] = 0.0;
        });
        const bool conv = newton<NS>(s, mdl, rl1, convfail, callSetup);
        BDF_PH(5);
        if (conv) {
            // cvDoErrorTest (cvode.c:2958-3030)
            dsm = s.acnrm * s.tq[2];
            if (dsm <= 1.0) break;
        }
        restore<NS>(s, saved_t);
        s.etamax = 1.0;
        if (!conv) {
            // cvHandleNFlag (cvode.c:2905-2945), recoverable convergence failure
            s.cnt.ncfn++;
            ncf++;
            if (ncf == MXNCF) return CV_CONV_FAILURE;
            s.eta = ETACF;
            nflag = PREV_CONV_FAIL;
            continue;
        }
        nef++;
        s.cnt.netf++;
        nflag = PREV_ERR_FAIL;
        if (nef == MXNEF) return CV_ERR_FAILURE;
        if (nef <= MXNEF1) {
            double eta = eta_exact(BIAS2 * dsm, s.L);
            eta = SUNMAX(ETAMIN, eta);
            if (nef >= SMALL_NEF) eta = SUNMIN(eta, ETAMXF);
            s.eta = eta;
            continue;
        }
        s.eta = ETAMIN;
        if (s.q > 1) {
            adjust_order<NS>(s, -1);
            s.L = s.q;
            s.q--;
            s.qwait = s.L;
            continue;
        }
        // order 1 restart: reload zn[1] from scratch
        s.h *= s.eta;
        s.hscale = s.h;
        s.qwait = LONG_WAIT;
        double tv[NS];
        mdl.rhs(s.tn, s.zn[0], tv);
        s.cnt.nfe++;
        cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
            constexpr int i = CI(I_);
            s.zn[1][i] = s.h * tv[i];
        });
        do_rescale = false;
    }

    BDF_PH(6);  // error test, failure handling
    // cvCompleteStep (cvode.c:3043-3080)
    s.nst++;
    s.cnt.nst_total++;
    s.hu = s.h;
    cfor_down<QMAX, 2>([&](auto i) __attribute__((always_inline)) {
        if (CI(i) <= s.q) s.tau[CI(i)] = s.tau[CI(i) - 1];
    });
    if ((s.q == 1) && (s.nst > 1)) s.tau[2] = s.tau[1];
    s.tau[1] = s.h;
    cfor<0, QMAX + 1>([&](auto J_) __attribute__((always_inline)) {
        constexpr int j = CI(J_);
        if (j <= s.q) {
            cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
                constexpr int i = CI(I_);
                s.zn[j][i] = s.zn[j][i] + s.l[j] * s.acor[i];
            });
        }
    });
    s.qwait--;
    if ((s.qwait == 1) && (s.q != QMAX)) {
        cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
            constexpr int i = CI(I_);
            s.zn[QMAX][i] = s.acor[i];
        });
        s.saved_tq5 = s.tq[5];
    }

    BDF_PH(7);
    // cvPrepareNextStep + cvComputeEtaqm1/qp1 + cvChooseEta + cvSetEta (cvode.c:3093-3258)
    if (s.etamax == 1.0) {
        s.qwait = SUNMAX(s.qwait, 2);
        s.qprime = s.q;
        s.hprime = s.h;
        s.eta = 1.0;
    } else {
        const double etaq = eta_exact(BIAS2 * dsm, s.L);
        double eta = etaq;
        s.qprime = s.q;
        if (s.qwait == 0) {
            s.qwait = 2;
            double etaqm1 = 0.0, etaqp1 = 0.0;
            double xm = 0.0, xp = 0.0;
            if (s.q > 1) {
                double znq[NS];
                sel_row<NS>(s.zn, s.q, znq);
                xm = BIAS1 * (wrms<NS>(znq, s.ewt) * s.tq[1]);
            }
            const bool do_p = (s.q != QMAX) && (s.saved_tq5 != 0.0);
            if (do_p) {
                const double cquot = fdiv(s.tq[5], s.saved_tq5) * powI(fdiv(s.h, s.tau[2]), s.L);
                double tv[NS];
                cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
                    constexpr int i = CI(I_);
                    tv[i] = (-cquot) * s.zn[QMAX][i] + s.acor[i];
                });
                xp = BIAS3 * (wrms<NS>(tv, s.ewt) * s.tq[3]);
            }
            // the two candidate ratios share one root call site
#pragma unroll 1
            for (int c = 0; c < 2; c++) {
                const bool act = (c == 0) ? (s.q > 1) : do_p;
                if (act) {
                    const double e = eta_exact((c == 0) ? xm : xp, (c == 0) ? s.q : s.L + 1);
                    if (c == 0)
                        etaqm1 = e;
                    else
                        etaqp1 = e;
                }
            }
            // cvChooseEta
            const double etam = SUNMAX(etaqm1, SUNMAX(etaq, etaqp1));
            if (etam < THRESH) {
                eta = 1.0;
            } else if (etam == etaq) {
                eta = etaq;
            } else if (etam == etaqm1) {
                eta = etaqm1;
                s.qprime = s.q - 1;
            } else {
                eta = etaqp1;
                s.qprime = s.q + 1;
                cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
                    constexpr int i = CI(I_);
                    s.zn[QMAX][i] = s.acor[i];
                });
            }
        }
        // cvSetEta (hmax_inv = 0)
        if (eta < THRESH) {
            s.eta = 1.0;
            s.hprime = s.h;
        } else {
            s.eta = SUNMIN(eta, s.etamax);
            s.hprime = s.h * s.eta;
        }
    }
    BDF_PH(8);
    s.etamax = (s.nst <= SMALL_NST) ? ETAMX2 : ETAMX3;
    cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
        constexpr int i = CI(I_);
        s.acor[i] *= s.tq[2];
    });

    // stop tests after the step (cvode.c:1395-1437)
    if (s.tstopset) {
        const double troundoff = FUZZ_FACTOR * UROUND * (fabs(s.tn) + fabs(s.h));
        if (fabs(s.tn - s.tstop) <= troundoff) {
            get_dky<NS>(s, s.tstop, yout);
            s.tretlast = tret = s.tstop;
            s.tstopset = 0;
            return CV_TSTOP_RETURN;
        }
        if ((s.tn + s.hprime - s.tstop) * s.h > 0.0) {
            s.hprime = (s.tstop - s.tn) * (1.0 - 4.0 * UROUND);
            s.eta = fdiv(s.hprime, s.h);
        }
    }
    s.tretlast = tret = s.tn;
    cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
        constexpr int i = CI(I_);
        yout[i] = s.zn[0][i];
    });
    BDF_PH(9);
    return CV_SUCCESS;
}

}  // namespace bcm3hip
