// libm_exact.h -- the libm results the reference's CPU build gets from glibc, reproduced on the
// device, so that the GPU's arithmetic on the PopPK path is the reference's operation for
// operation (DESIGN.md §3 "bit-exact arithmetic").
//
// Where the reference calls libm (glibc 2.35 on this image):
//   exp, log      LikelihoodPopPKTrajectory.cpp:283-286 via bcm3::fastpow10 (MathFunctions.h:13),
//                 VariableSet::TransformVariable (VariableSet.cpp:97-124), LogPdfTnu4
//                 (ProbabilityDistributions.cpp:216-224), the QuantileNormal restatement
//   pow(x, 1/k)   SUNRpowerR in cvode.c:2986, 3105, 3163, 3187 (sundials_math.c:40-52)
// glibc's exp / log / pow are accurate to ~2^-63..2^-68 before their final rounding, so they
// return the correctly rounded (CR) result except on a ~2^-15 fraction of arguments. The
// functions here compute the CR result from double-double arithmetic (relative error ~2^-95
// before the final rounding) and therefore agree with glibc wherever glibc is correctly rounded
// (tests/test_libm_exact.py counts the agreement on random arguments against the host's glibc).
//
// Every function is plain IEEE double arithmetic with explicit fma -- identical on the host and
// on gfx950 (the library is built with -ffp-contract=off) -- so the host test exercises the
// device code itself. pow_inv_k takes its seed from single-precision hardware log2 / exp2 on
// the device and from libm's log2f / exp2f on the host: the result does not depend on the seed
// (the double-double correction step below fixes every bit).
#pragma once

#ifdef __HIP__
#include <hip/hip_runtime.h>
#define XM_FN __host__ __device__ __forceinline__
// exp, log, log1p, erf and erfc come in two forms: name_i always inline, and name out of line (a
// call), so that their registers do not add to the pressure of a kernel that calls them off its
// hot loop. lib<COLD> picks one at a call site: the one-trajectory-per-wavefront PopPK kernel with
// vector state calls them out of line; the other kernels inline them (a call from the scalar-state
// two-compartment transit kernel was miscompiled: every solve failed on its first step)
#ifdef BCM3_XM_INLINE
#define XM_COLD XM_FN
#else
#define XM_COLD __host__ __device__ __attribute__((noinline)) inline
#endif
#else
#include <cmath>
#define XM_FN inline
#define XM_COLD inline
#endif

namespace xm {

struct dd {
    double hi, lo;
};

XM_FN dd two_sum(double a, double b)
{
    const double s = a + b;
    const double bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
// |a| >= |b|
XM_FN dd fast_two_sum(double a, double b)
{
    const double s = a + b;
    return {s, b - (s - a)};
}
XM_FN dd two_prod(double a, double b)
{
    const double p = a * b;
    return {p, __builtin_fma(a, b, -p)};
}
XM_FN dd dd_add(dd a, dd b)
{
    dd s = two_sum(a.hi, b.hi);
    const dd t = two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = fast_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return fast_two_sum(s.hi, s.lo);
}
XM_FN dd dd_add_d(dd a, double b)
{
    dd s = two_sum(a.hi, b);
    s.lo += a.lo;
    return fast_two_sum(s.hi, s.lo);
}
XM_FN dd dd_mul(dd a, dd b)
{
    dd p = two_prod(a.hi, b.hi);
    p.lo = __builtin_fma(a.hi, b.lo, p.lo);
    p.lo = __builtin_fma(a.lo, b.hi, p.lo);
    return fast_two_sum(p.hi, p.lo);
}

XM_FN double as_double(long long b) { return __builtin_bit_cast(double, b); }
XM_FN long long as_bits(double x) { return __builtin_bit_cast(long long, x); }
// 2^k for -1022 <= k <= 1023
XM_FN double pow2i(int k) { return as_double((long long)((unsigned long long)(k + 1023) << 52)); }

// The tables of glibc's pow and exp (e_pow.c, e_exp.c since glibc 2.28; see pow_glibc below)
struct GlibcPow {
    double ln2hi, ln2lo, A[7];      // __pow_log_data: ln2 split, log1p polynomial (A[0] = -1/2)
    double logtab[128][4];          //   invc, pad, logc, logctail
    double invln2N, shift, negln2hiN, negln2loN, C[4];  // __exp_data: reduction, C2..C5
    unsigned long long exptab[256];  //   (tail, sbits) pairs of 2^(i/128)
    int ok;                          // 1: filled (a zero-initialised copy selects the fallbacks)
};

#ifdef __HIP__
// the device's copy, per translation unit (popk_prepare_device / expm_prepare_device upload it;
// never uploaded, ok = 0 selects the correctly rounded functions)
static __constant__ GlibcPow xm_tables;
#endif

// glibc's exp for 2^-54 <= |x| < 512 (the main path of e_exp.c as its FMA variant computes it):
// x = (k + i/128) ln2 + r, 2^(i/128) = scale (1 + tail) from the table, exp(r) by its polynomial
XM_FN double exp_glibc(double x, const GlibcPow& D)
{
    const double kz = __builtin_fma(x, D.invln2N, D.shift);
    const unsigned long long ki = (unsigned long long)as_bits(kz);
    const double kd = kz - D.shift;
    double r = __builtin_fma(kd, D.negln2hiN, x);
    r = __builtin_fma(kd, D.negln2loN, r);
    const int idx = 2 * (int)(ki & 127);
    const unsigned long long sbits = D.exptab[idx + 1] + (ki << 45);
    const double c23 = __builtin_fma(r, D.C[1], D.C[0]);
    const double tr = r + as_double((long long)D.exptab[idx]);
    const double r2 = r * r;
    const double c45 = __builtin_fma(r, D.C[3], D.C[2]);
    const double s1 = __builtin_fma(c23, r2, tr);
    const double t = __builtin_fma(c45, r2 * r2, s1);
    const double scale = as_double((long long)sbits);
    return __builtin_fma(scale, t, scale);
}

// ln 2 = LN2_1 + LN2_2 + LN2_3, LN2_1 and LN2_2 with 42 significant bits (k * LN2_i exact for
// |k| < 2^11)
constexpr double LN2_1 = 0.6931471805598903;
constexpr double LN2_2 = 5.49792301870721e-14;
constexpr double LN2_3 = 1.1612227229362532e-26;
constexpr double INV_LN2 = 1.4426950408889634;
constexpr double SIXTH_HI = 0.16666666666666666, SIXTH_LO = 9.25185853854297e-18;

// exp(x) as a double-double, x finite with -745 < x < 709.8 (2^k scaling applied to both parts;
// for results below the normal range the low part is meaningless). Reduction x = k ln2 + r,
// |r| <= ln2/2, r = 2^8 s, expm1(s) by its Taylor series (dd up to s^3), then eight steps of
// expm1(2s) = expm1(s) (expm1(s) + 2), which keep the relative error of expm1 from doubling.
XM_FN dd exp_dd(double x)
{
    const double k = __builtin_rint(x * INV_LN2);
    const double r1 = x - k * LN2_1;  // exact (Sterbenz; k * LN2_1 exact)
    dd r = two_sum(r1, -(k * LN2_2));  // k * LN2_2 exact
    r.lo = __builtin_fma(-k, LN2_3, r.lo);
    r = fast_two_sum(r.hi, r.lo);
    const dd s = {r.hi * 0x1p-8, r.lo * 0x1p-8};
    const dd s2 = dd_mul(s, s);
    const dd s3 = dd_mul(s2, s);
    // s^4 (1/24 + s/120 + s^2/720 + s^3/5040 + s^4/40320): ~2^-75 of expm1(s), double suffices
    const double sh = s.hi;
    double v = 2.48015873015873e-05;
    v = __builtin_fma(v, sh, 0.0001984126984126984);
    v = __builtin_fma(v, sh, 0.001388888888888889);
    v = __builtin_fma(v, sh, 0.008333333333333333);
    v = __builtin_fma(v, sh, 0.041666666666666664);
    const double t4 = (s2.hi * s2.hi) * v;
    dd e = dd_mul(s3, dd{SIXTH_HI, SIXTH_LO});
    e = dd_add_d(e, t4);
    e = dd_add(e, dd{s2.hi * 0.5, s2.lo * 0.5});
    e = dd_add(e, s);
    for (int i = 0; i < 8; i++) e = dd_mul(e, dd_add_d(e, 2.0));
    dd y = fast_two_sum(1.0, e.hi);  // 1 + expm1(r), expm1(r) in [-0.293, 0.415]
    y.lo += e.lo;
    y = fast_two_sum(y.hi, y.lo);
    const int ki = (int)k;
    if (ki > 1000 || ki < -1000) {
        const double a = pow2i(ki / 2), b = pow2i(ki - ki / 2);
        return {(y.hi * a) * b, (y.lo * a) * b};
    }
    const double sc = pow2i(ki);
    return {y.hi * sc, y.lo * sc};
}

// exp, correctly rounded
XM_FN double exp_cr(double x)
{
    if (!(x == x)) return x + x;
    if (x > 709.782712893384) return __builtin_inf();
    if (x < -745.1332191019412) return 0.0;
    const dd y = exp_dd(x);  // (below ~-708 the result is subnormal and not CR; off the path)
    return y.hi + y.lo;
}

// glibc's exp: on the device with the uploaded tables (its own results, in the range its main
// path covers), else the correctly rounded exp (glibc agrees with it on all but ~0.03 %)
XM_FN double exp_i(double x)
{
#if defined(__HIP__) && defined(__HIP_DEVICE_COMPILE__)
    const double ax = __builtin_fabs(x);
    if (xm_tables.ok & (ax >= 0x1p-54) & (ax < 512.0)) return exp_glibc(x, xm_tables);
#endif
    return exp_cr(x);
}

// glibc log (correctly rounded result): one Newton step y0 + log1p(x e^-y0 - 1) from the
// library estimate y0, with e^-y0 in double-double
XM_FN double log_i(double x)
{
    if (!(x > 0.0) || x == __builtin_inf()) {
        if (x == 0.0) return -__builtin_inf();
        return (x < 0.0) ? __builtin_nan("") : x + x;
    }
    double xs = x, off = 0.0;
    if (x < 0x1p-1000) {  // subnormal arguments: scale
        xs = x * 0x1p200;
        off = -200.0;
    }
    const double y0 = ::log(xs) + off * (LN2_1 + LN2_2);
    if (y0 == 0.0) return 0.0;  // x == 1 exactly (log is exact there)
    const dd E = exp_dd(-y0);
    // x E - 1 with x = xs 2^off
    const double xe = (off != 0.0) ? x * 0x1p200 : x;
    const dd p = two_prod(xe, E.hi);
    const double d = p.hi - 1.0;  // exact: p.hi in [0.5, 2]
    const double t = d + __builtin_fma(xe, E.lo, p.lo);
    return y0 + __builtin_fma(-0.5 * t, t, t);
}

// f = fl(1/k) - 1/k times ln 2, k = 2..7 (the exponents ONE/L of cvode.c are rounded)
XM_FN double inv_k_err_ln2(int k)
{
    double r = 0.0;
    r = (k == 3) ? -1.2825799321861034e-17 : r;
    r = (k == 5) ? 7.69547959311662e-18 : r;
    r = (k == 6) ? -6.412899660930517e-18 : r;
    r = (k == 7) ? -5.496771137940443e-18 : r;
    return r;
}
XM_FN double inv_k(int k)
{
    double r = 0.5;
    r = (k == 3) ? 0.3333333333333333 : r;
    r = (k == 4) ? 0.25 : r;
    r = (k == 5) ? 0.2 : r;
    r = (k == 6) ? 0.16666666666666666 : r;
    r = (k == 7) ? 0.14285714285714285 : r;
    return r;
}

#ifdef __HIP_DEVICE_COMPILE__
XM_FN float seed_log2f(float x) { return __builtin_amdgcn_logf(x); }
XM_FN float seed_exp2f(float x) { return __builtin_amdgcn_exp2f(x); }
#else
XM_FN float seed_log2f(float x) { return ::log2f(x); }
XM_FN float seed_exp2f(float x) { return ::exp2f(x); }
#endif

// glibc pow(x, fl(1/k)) for 1e-30 < x < 1e30, k = 2..7 (correctly rounded result).
//   z ~ x^(-1/k): single-precision seed + two Newton steps z <- z + z (1 - x z^k) / k;
//   p0 = x z^(k-1) ~ x^(1/k) within a few ulp;
//   the exact root is p0 + (x - p0^k) / (k p0^(k-1)), with p0^k in double-double;
//   x^fl(1/k) = x^(1/k) (1 + (fl(1/k) - 1/k) ln x + ...), ln x from the single-precision log2.
// zk_out (optional): z^k ~ 1/x, reused by callers.
XM_FN double pow_inv_k(double x, int k)
{
    const double rk = inv_k(k);
    const float lf = seed_log2f((float)x);
    double z = (double)seed_exp2f(-lf * (float)rk);
    double zk = z;
    for (int it = 0; it < 2; it++) {
        zk = z;
        for (int i = 2; i <= 7; i++)
            if (i <= k) zk *= z;
        const double t = __builtin_fma(-x, zk, 1.0);
        z = __builtin_fma(z * t, rk, z);
    }
    double zk1 = 1.0;  // z^(k-1)
    for (int i = 1; i <= 6; i++)
        if (i < k) zk1 *= z;
    const double p0 = x * zk1;
    // p0^k in double-double
    dd P = {p0, 0.0};
    for (int i = 2; i <= 7; i++) {
        if (i <= k) {
            const double h = P.hi * p0;
            const double e = __builtin_fma(P.hi, p0, -h);
            P.lo = __builtin_fma(P.lo, p0, e);
            P.hi = h;
        }
    }
    const double d = (x - P.hi) - P.lo;  // x - P.hi exact (Sterbenz)
    // (x - p0^k) / (k p0^(k-1)) = d p0 / (k x) ~ d p0 z^k / k
    const double delta = d * (p0 * (zk1 * z)) * rk;
    const double c = __builtin_fma(p0 * (double)lf, inv_k_err_ln2(k), delta);
    return p0 + c;
}

// pow_inv_k, and whether its result is certainly glibc's too: glibc's pow is within 0.52 ulp of
// the exact value (e_pow.c), so it can round differently only when the exact root lies within
// 0.02 ulp of a rounding midpoint. p0 + c carries the root to ~2^-100 relative; `safe` when the
// rounding residual of p0 + c is below 0.44 ulp (0.06 ulp from a midpoint, three times the bound)
XM_FN double pow_inv_k_checked(double x, int k, bool& safe)
{
    const double rk = inv_k(k);
    const float lf = seed_log2f((float)x);
    double z = (double)seed_exp2f(-lf * (float)rk);
    double zk = z;
    for (int it = 0; it < 2; it++) {
        zk = z;
        for (int i = 2; i <= 7; i++)
            if (i <= k) zk *= z;
        const double t = __builtin_fma(-x, zk, 1.0);
        z = __builtin_fma(z * t, rk, z);
    }
    double zk1 = 1.0;
    for (int i = 1; i <= 6; i++)
        if (i < k) zk1 *= z;
    const double p0 = x * zk1;
    dd P = {p0, 0.0};
    for (int i = 2; i <= 7; i++) {
        if (i <= k) {
            const double h = P.hi * p0;
            const double e = __builtin_fma(P.hi, p0, -h);
            P.lo = __builtin_fma(P.lo, p0, e);
            P.hi = h;
        }
    }
    const double d = (x - P.hi) - P.lo;
    const double delta = d * (p0 * (zk1 * z)) * rk;
    const double c = __builtin_fma(p0 * (double)lf, inv_k_err_ln2(k), delta);
    const double r = p0 + c;
    const double res = c - (r - p0);  // p0 + c - r, exact (|c| << |p0|)
    const double ulp = as_double(as_bits(r) & 0x7ff0000000000000LL) * 0x1p-52;
    safe = __builtin_fabs(res) < 0.44 * ulp;
    return r;
}

// ---------------------------------------------------------------------------------------------
// glibc's pow itself (sysdeps/ieee754/dbl-64/e_pow.c, glibc >= 2.28: a table-driven log in
// double-double and a table-driven exp), as the x86-64 libm runs it on FMA/AVX2 hosts (its
// __pow_fma variant, selected by the ifunc): the operations of that build in its order and with
// its fused multiply-adds. glibc's pow is not correctly rounded (it differs from pow_inv_k on
// ~0.08 % of the step-size roots, which alone decided whether 11 % of C3 trajectories came out
// bit-identical to the reference), so the solvers run this algorithm on the host libm's own tables
// -- located in the loaded libm at run time (libm_tables.cpp), never shipped -- or, without them,
// on tables of the same layout computed on the host (about 1 ulp).

// pow(x, y) for a positive normal x and 2^-65 <= |y| < 2^63 with |y log x| < 512 (the main path
// of e_pow.c; the step-size roots: x in (1e-30, 1e30), y = fl(1/k))
XM_FN double pow_glibc_ix(unsigned long long ix, double y, const GlibcPow& D);
XM_FN double pow_glibc(double x, double y, const GlibcPow& D) { return pow_glibc_ix((unsigned long long)as_bits(x), y, D); }

// pow(x, y) for every finite x > 0 (e_pow.c: a subnormal x is normalised first, its exponent field
// going negative: asuint64(x 2^52) - 52 << 52), without a branch
XM_FN double pow_glibc_pos(double x, double y, const GlibcPow& D)
{
    const unsigned long long ix = (unsigned long long)as_bits(x);
    const unsigned long long ixs = (unsigned long long)as_bits(x * 0x1p52) - (52ull << 52);
    return pow_glibc_ix((ix < 0x0010000000000000ull) ? ixs : ix, y, D);
}

// x given as its bit pattern ix (see pow_glibc_pos for subnormal x)
XM_FN double pow_glibc_ix(unsigned long long ix, double y, const GlibcPow& D)
{
    // log_inline: x = 2^k z, z/c - 1 = r exact, log x = k ln2 + log c + log1p(r) in double-double
    const unsigned long long tmp = ix + 0xC0196AAB00000000ull;  // ix - 0x3fe6955500000000
    const int i = (int)((tmp >> 45) & 127);
    const double kd = (double)(int)((long long)tmp >> 52);
    const double z = as_double((long long)(ix - (tmp & 0xfff0000000000000ull)));
    const double invc = D.logtab[i][0], logc = D.logtab[i][2], logctail = D.logtab[i][3];
    const double t1 = __builtin_fma(kd, D.ln2hi, logc);
    const double r = __builtin_fma(z, invc, -1.0);
    const double ar = r * D.A[0];
    const double lo1 = __builtin_fma(kd, D.ln2lo, logctail);
    const double p12 = __builtin_fma(r, D.A[2], D.A[1]);
    const double p34 = __builtin_fma(r, D.A[4], D.A[3]);
    const double t2 = r + t1;
    const double ar2 = r * ar;
    const double ar3 = r * ar2;
    const double lo3 = __builtin_fma(ar, r, -ar2);
    const double lo2 = (t1 - t2) + r;
    const double p56 = __builtin_fma(r, D.A[6], D.A[5]);
    const double hi = t2 + ar2;
    const double lo4 = (t2 - hi) + ar2;
    const double q = __builtin_fma(ar2, __builtin_fma(p56, ar2, p34), p12);
    double lo = ((lo1 + lo2) + lo3) + lo4;
    lo = __builtin_fma(ar3, q, lo);
    const double ly = hi + lo;
    const double ltail = (hi - ly) + lo;
    // y log x = ehi + elo
    const double ehi = y * ly;
    const double elo = __builtin_fma(y, ltail, __builtin_fma(ly, y, -ehi));
    const int abstop = (int)((as_bits(ehi) >> 52) & 0x7ff);
#ifndef BCM3_ROOT_LEAN
    if (abstop < 0x3c9) return 1.0 + ehi;  // |y log x| < 2^-54
#endif
    // exp_inline: ehi = (k + i/128) ln2 + r, 2^(i/128) from the table, exp(r) by its polynomial
    const double kz = __builtin_fma(ehi, D.invln2N, D.shift);
    const unsigned long long ki = (unsigned long long)as_bits(kz);
    const double kk = kz - D.shift;
    double rr = __builtin_fma(kk, D.negln2hiN, ehi);
    rr = __builtin_fma(kk, D.negln2loN, rr);
    const int idx = 2 * (int)(ki & 127);
    const double tail = as_double((long long)D.exptab[idx]);
    const unsigned long long sbits = D.exptab[idx + 1] + (ki << 45);
    rr = elo + rr;
    const double c23 = __builtin_fma(rr, D.C[1], D.C[0]);
    const double tr = rr + tail;
    const double r2 = rr * rr;
    const double c45 = __builtin_fma(rr, D.C[3], D.C[2]);
    const double s1 = __builtin_fma(c23, r2, tr);
    const double t = __builtin_fma(c45, r2 * r2, s1);
    const double scale = as_double((long long)sbits);
#ifdef BCM3_ROOT_LEAN
    // (the tiny case as a select: the exp path's operands are finite there too)
    return (abstop < 0x3c9) ? 1.0 + ehi : __builtin_fma(t, scale, scale);  // |y log x| < 2^-54
#else
    return __builtin_fma(t, scale, scale);
#endif
}

// ---------------------------------------------------------------------------------------------
// glibc's log1p, erf and erfc are the fdlibm algorithms (not correctly rounded), so they are
// restated operation for operation, with glibc's evaluation order of the polynomials
// (second-order Horner / Estrin splits) and its constants; exp inside erf / erfc is the CR exp
// above. Checked bit for bit against the host's glibc (tests/test_libm_exact.py).

XM_FN int hi_word(double x) { return (int)(as_bits(x) >> 32); }
XM_FN double with_hi_word(double x, int h)
{
    return as_double((long long)(((unsigned long long)as_bits(x) & 0xffffffffULL) | ((unsigned long long)(unsigned)h << 32)));
}
XM_FN double with_lo_zero(double x) { return as_double(as_bits(x) & ~0xffffffffLL); }

XM_FN double log1p_i(double x)
{
    constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    constexpr double Lp1 = 6.666666666666735130e-01, Lp2 = 3.999999999940941908e-01,
                     Lp3 = 2.857142874366239149e-01, Lp4 = 2.222219843214978396e-01,
                     Lp5 = 1.818357216161805012e-01, Lp6 = 1.531383769920937332e-01,
                     Lp7 = 1.479819860511658591e-01;
    double hfsq, f = 0.0, c = 0.0, s, z, R, u;
    const int hx = hi_word(x);
    const int ax = hx & 0x7fffffff;
    int k = 1, hu = 0;
    if (hx < 0x3FDA827A) {  // x < 0.41422
        if (ax >= 0x3ff00000) return (x == -1.0) ? -__builtin_inf() : __builtin_nan("");
        if (ax < 0x3e200000) {  // |x| < 2^-29
            if (ax < 0x3c900000) return x;
            return x - x * x * 0.5;
        }
        if (hx > 0 || hx <= (int)0xbfd2bec3) {  // -0.2929 < x < 0.41422
            k = 0;
            f = x;
            hu = 1;
        }
    }
    if (hx >= 0x7ff00000) return x + x;
    if (k != 0) {
        if (hx < 0x43400000) {
            u = 1.0 + x;
            hu = hi_word(u);
            k = (hu >> 20) - 1023;
            c = (k > 0) ? 1.0 - (u - x) : x - (u - 1.0);  // correction term
            c /= u;
        } else {
            u = x;
            hu = hi_word(u);
            k = (hu >> 20) - 1023;
            c = 0.0;
        }
        hu &= 0x000fffff;
        if (hu < 0x6a09e) {
            u = with_hi_word(u, hu | 0x3ff00000);  // normalise u
        } else {
            k += 1;
            u = with_hi_word(u, hu | 0x3fe00000);  // normalise u / 2
            hu = (0x00100000 - hu) >> 2;
        }
        f = u - 1.0;
    }
    hfsq = 0.5 * f * f;
    if (hu == 0) {  // |f| < 2^-20
        if (f == 0.0) {
            if (k == 0) return 0.0;
            c += k * ln2_lo;
            return k * ln2_hi + c;
        }
        R = hfsq * (1.0 - 0.66666666666666666 * f);
        if (k == 0) return f - R;
        return k * ln2_hi - ((R - (k * ln2_lo + c)) - f);
    }
    s = f / (2.0 + f);
    z = s * s;
    const double R1 = z * Lp1, z2 = z * z, R2 = Lp2 + z * Lp3, z4 = z2 * z2, R3 = Lp4 + z * Lp5, z6 = z4 * z2,
                 R4 = Lp6 + z * Lp7;
    R = R1 + z2 * R2 + z4 * R3 + z6 * R4;
    if (k == 0) return f - (hfsq - s * (hfsq + R));
    return k * ln2_hi - ((hfsq - (s * (hfsq + R) + (k * ln2_lo + c))) - f);
}

// erf / erfc coefficients (fdlibm s_erf.c)
struct ErfC {
    static constexpr double erx = 8.45062911510467529297e-01, efx = 1.28379167095512586316e-01;
    static constexpr double pp0 = 1.28379167095512558561e-01, pp1 = -3.25042107247001499370e-01,
                            pp2 = -2.84817495755985104766e-02, pp3 = -5.77027029648944159157e-03,
                            pp4 = -2.37630166566501626084e-05, qq1 = 3.97917223959155352819e-01,
                            qq2 = 6.50222499887672944485e-02, qq3 = 5.08130628187576562776e-03,
                            qq4 = 1.32494738004321644526e-04, qq5 = -3.96022827877536812320e-06;
    static constexpr double pa0 = -2.36211856075265944077e-03, pa1 = 4.14856118683748331666e-01,
                            pa2 = -3.72207876035701323847e-01, pa3 = 3.18346619901161753674e-01,
                            pa4 = -1.10894694282396677476e-01, pa5 = 3.54783043256182359371e-02,
                            pa6 = -2.16637559486879084300e-03, qa1 = 1.06420880400844228286e-01,
                            qa2 = 5.40397917702171048937e-01, qa3 = 7.18286544141962662868e-02,
                            qa4 = 1.26171219808761642112e-01, qa5 = 1.36370839120290507362e-02,
                            qa6 = 1.19844998467991074170e-02;
    static constexpr double ra0 = -9.86494403484714822705e-03, ra1 = -6.93858572707181764372e-01,
                            ra2 = -1.05586262253232909814e+01, ra3 = -6.23753324503260060396e+01,
                            ra4 = -1.62396669462573470355e+02, ra5 = -1.84605092906711035994e+02,
                            ra6 = -8.12874355063065934246e+01, ra7 = -9.81432934416914548592e+00,
                            sa1 = 1.96512716674392571292e+01, sa2 = 1.37657754143519042600e+02,
                            sa3 = 4.34565877475229228821e+02, sa4 = 6.45387271733267880336e+02,
                            sa5 = 4.29008140027567833386e+02, sa6 = 1.08635005541779435134e+02,
                            sa7 = 6.57024977031928170135e+00, sa8 = -6.04244152148580987438e-02;
    static constexpr double rb0 = -9.86494292470009928597e-03, rb1 = -7.99283237680523006574e-01,
                            rb2 = -1.77579549177547519889e+01, rb3 = -1.60636384855821916062e+02,
                            rb4 = -6.37566443368389627722e+02, rb5 = -1.02509513161107724954e+03,
                            rb6 = -4.83519191608651397019e+02, sb1 = 3.03380607434824582924e+01,
                            sb2 = 3.25792512996573918826e+02, sb3 = 1.53672958608443695994e+03,
                            sb4 = 3.19985821950859553908e+03, sb5 = 2.55305040643316442583e+03,
                            sb6 = 4.74528541206955367215e+02, sb7 = -2.24409524465858183362e+01;
};

// |x| < 0.84375: y with erf(x) = x + x y
XM_FN double erf_small_y(double x)
{
    using C = ErfC;
    const double z = x * x;
    const double r1 = C::pp0 + z * C::pp1, z2 = z * z;
    const double r2 = C::pp2 + z * C::pp3, z4 = z2 * z2;
    const double s1 = 1.0 + z * C::qq1;
    const double s2 = C::qq2 + z * C::qq3;
    const double s3 = C::qq4 + z * C::qq5;
    const double r = r1 + z2 * r2 + z4 * C::pp4;
    const double s = s1 + z2 * s2 + z4 * s3;
    return r / s;
}
// 0.84375 <= |x| < 1.25: P / Q
XM_FN void erf_mid_pq(double ax, double& P, double& Q)
{
    using C = ErfC;
    const double s = ax - 1.0;
    const double P1 = C::pa0 + s * C::pa1, s2 = s * s;
    const double Q1 = 1.0 + s * C::qa1, s4 = s2 * s2;
    const double P2 = C::pa2 + s * C::pa3, s6 = s4 * s2;
    const double Q2 = C::qa2 + s * C::qa3;
    const double P3 = C::pa4 + s * C::pa5;
    const double Q3 = C::qa4 + s * C::qa5;
    P = P1 + s2 * P2 + s4 * P3 + s6 * C::pa6;
    Q = Q1 + s2 * Q2 + s4 * Q3 + s6 * C::qa6;
}
// |x| >= 1.25: exp(-z^2 - 0.5625) exp((z - x)(z + x) + R / S), ax = |x|; `lo` selects the
// 1.25 <= |x| < 1/0.35 coefficients
XM_FN double erf_tail_r(double ax, bool lo)
{
    using C = ErfC;
    const double s = 1.0 / (ax * ax);
    double R, S;
    if (lo) {
        const double R1 = C::ra0 + s * C::ra1, s2 = s * s;
        const double S1 = 1.0 + s * C::sa1, s4 = s2 * s2;
        const double R2 = C::ra2 + s * C::ra3, s6 = s4 * s2;
        const double S2 = C::sa2 + s * C::sa3, s8 = s4 * s4;
        const double R3 = C::ra4 + s * C::ra5;
        const double S3 = C::sa4 + s * C::sa5;
        const double R4 = C::ra6 + s * C::ra7;
        const double S4 = C::sa6 + s * C::sa7;
        R = R1 + s2 * R2 + s4 * R3 + s6 * R4;
        S = S1 + s2 * S2 + s4 * S3 + s6 * S4 + s8 * C::sa8;
    } else {
        const double R1 = C::rb0 + s * C::rb1, s2 = s * s;
        const double S1 = 1.0 + s * C::sb1, s4 = s2 * s2;
        const double R2 = C::rb2 + s * C::rb3, s6 = s4 * s2;
        const double S2 = C::sb2 + s * C::sb3;
        const double R3 = C::rb4 + s * C::rb5;
        const double S3 = C::sb4 + s * C::sb5;
        const double S4 = C::sb6 + s * C::sb7;
        R = R1 + s2 * R2 + s4 * R3 + s6 * C::rb6;
        S = S1 + s2 * S2 + s4 * S3 + s6 * S4;
    }
    const double z = with_lo_zero(ax);
    return exp_i(-z * z - 0.5625) * exp_i((z - ax) * (z + ax) + R / S);
}

XM_FN double erf_i(double x)
{
    const int hx = hi_word(x);
    const int ix = hx & 0x7fffffff;
    if (ix >= 0x7ff00000) return (x != x) ? x + x : ((hx < 0) ? -1.0 : 1.0);
    if (ix < 0x3feb0000) {  // |x| < 0.84375
        if (ix < 0x3e300000) return x + ErfC::efx * x;
        return x + x * erf_small_y(x);
    }
    if (ix < 0x3ff40000) {  // 0.84375 <= |x| < 1.25
        double P, Q;
        erf_mid_pq(fabs(x), P, Q);
        return (hx >= 0) ? ErfC::erx + P / Q : -ErfC::erx - P / Q;
    }
    if (ix >= 0x40180000) return (hx >= 0) ? 1.0 : -1.0;  // |x| >= 6: 1 - tiny rounds to 1
    const double ax = fabs(x);
    const double r = erf_tail_r(ax, ix < 0x4006DB6E);
    return (hx >= 0) ? 1.0 - r / ax : r / ax - 1.0;
}

XM_FN double erfc_i(double x)
{
    const int hx = hi_word(x);
    const int ix = hx & 0x7fffffff;
    if (ix >= 0x7ff00000) return (x != x) ? x + x : ((hx < 0) ? 2.0 : 0.0);
    if (ix < 0x3feb0000) {  // |x| < 0.84375
        if (ix < 0x3c700000) return 1.0 - x;
        const double y = erf_small_y(x);
        if (hx < 0x3fd00000) return 1.0 - (x + x * y);  // x < 1/4
        double r = x * y;
        r += (x - 0.5);
        return 0.5 - r;
    }
    if (ix < 0x3ff40000) {  // 0.84375 <= |x| < 1.25
        double P, Q;
        erf_mid_pq(fabs(x), P, Q);
        if (hx >= 0) {
            const double z = 1.0 - ErfC::erx;
            return z - P / Q;
        }
        const double z = ErfC::erx + P / Q;
        return 1.0 + z;
    }
    if (ix < 0x403c0000) {  // |x| < 28
        if (hx < 0 && ix >= 0x40180000) return 2.0;  // x < -6: 2 - tiny rounds to 2
        const double ax = fabs(x);
        const double r = erf_tail_r(ax, ix < 0x4006DB6D);
        return (hx > 0) ? r / ax : 2.0 - r / ax;
    }
    return (hx > 0) ? 0.0 : 2.0;
}

XM_COLD double exp(double x) { return exp_i(x); }
XM_COLD double log(double x) { return log_i(x); }
XM_COLD double log1p(double x) { return log1p_i(x); }
XM_COLD double erf(double x) { return erf_i(x); }
XM_COLD double erfc(double x) { return erfc_i(x); }

template <bool COLD>
struct lib {
    static XM_FN double exp(double x)
    {
        if constexpr (COLD) return xm::exp(x);
        else return exp_i(x);
    }
    static XM_FN double log(double x)
    {
        if constexpr (COLD) return xm::log(x);
        else return log_i(x);
    }
    static XM_FN double log1p(double x)
    {
        if constexpr (COLD) return xm::log1p(x);
        else return log1p_i(x);
    }
    static XM_FN double erf(double x)
    {
        if constexpr (COLD) return xm::erf(x);
        else return erf_i(x);
    }
    static XM_FN double erfc(double x)
    {
        if constexpr (COLD) return xm::erfc(x);
        else return erfc_i(x);
    }
};

}  // namespace xm
