// cellpop_solver.h -- the cell-population ODE solve kernel, compiled at run time (hipRTC) per
// model together with the model's generated right-hand side (cellpop_rt.cpp prepends the
// definitions CP_NS / CP_NC / CP_NP and `generated_derivative`, the text of the reference's
// SBMLModel::GenerateCode, src/sbml/SBMLModel.cpp:291-367, as a device template).
//
// One workgroup = one wavefront = one cell. The reference integrates each cell with CVODE 5.3.0
// BDF (ODESolverCVODE::Solve, src/odecommon/ODESolverCVODE.cpp:322-463; Cell::Simulate,
// src/cellpop/Cell.cpp:193-273): Newton with a difference-quotient Jacobian
// (ODESolverCVODE::DifferenceQuotientJacobian, :496-537) and a dense partial-pivoting LU
// (PartialPivLUExtended::compute_optimized, src/utils/EigenPartialPivLUSomewhatSparse.h) --
// N = tens of species, so unlike the PopPK kernels nothing is closed-form:
//   * lane i holds component i of every solver vector (Nordsieck zn[0..5], ewt, acor): every
//     component-wise operation of the BDF step is one instruction, as in bdf_vec.h;
//   * the saved Jacobian and the LU factors live in LDS (column-major N x N per wave); the
//     factorisation runs lanes = rows, the row swaps lanes = columns; solves are
//     column-oriented substitutions with one broadcast per column;
//   * the generated right-hand side runs wave-uniform (every lane evaluates the model's rate
//     laws on the broadcast state) and lane i keeps component i; the N perturbed evaluations of
//     the difference-quotient Jacobian run in ONE pass, lane j evaluating f(y + inc_j e_j), so a
//     Jacobian costs one RHS evaluation instead of N;
//   * weighted norms sum the rounded squares in component order (nvector_serial's N_VWrmsNorm).
// The step control is the reference's cvode.c (the runtime-order form of bdf_lane.h, with the
// hmin rules cellpop sets: CVodeSetMinStep, cvode.c:1123-1124, 2893-2903, 2977-3007); the cell
// driver restates Cell::integration_step_cb (Cell.cpp:463-538) in the non-stored mode.
#pragma once
#include "bdf_lane.h"
#include "cellpop_args.h"
#if defined(CP_QUEUE) && CP_QUEUE
#include "cellpop_init.h"
#endif

namespace cpk {
using namespace bcm3hip;

#ifndef CP_NTREAT
#define CP_NTREAT 0
#endif
#ifndef CP_QUEUE
#define CP_QUEUE 0
#endif
constexpr int WAVE = 64;
// A cell's state lives in one ROW of lanes (component i in lane i of the row). With NS <= 16 four
// cells share a wavefront -- the 16-lane DPP rows -- so every vector instruction advances four
// cells; with more species one cell takes the whole wavefront. Control flow that depends on a
// cell's state (step size, order, Newton iterations, failures) diverges between the rows of a
// wavefront and runs under the execution mask.
constexpr int ROW = (CP_NS <= 16) ? 16 : 64;
constexpr int CPW = WAVE / ROW;

BDF_INL int lane() { return (int)threadIdx.x & (ROW - 1); }  // component index within the row
BDF_INL int row() { return (int)threadIdx.x / ROW; }

BDF_INL double bcast(double v, int k)
{
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)b, k);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

BDF_INL void wave_sync() { __syncthreads(); }

// value of lane k (runtime) of this lane's row (ds_bpermute; the whole row must be active)
BDF_INL double rowget(double v, int k)
{
    const int addr = ((int)(threadIdx.x & ~(unsigned)(ROW - 1)) + k) << 2;
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_ds_bpermute(addr, (int)b);
    const int hi = __builtin_amdgcn_ds_bpermute(addr, (int)(b >> 32));
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

struct LdsSpecies {
    const double* y;
    BDF_INL double operator[](int k) const { return y[k]; }
};
// the row's state in registers: component k broadcast from lane k of the row (row_newbcast, NS <= 16)
template <int NS>
struct RegSpecies {
    double v[NS];
    BDF_INL double operator[](int k) const { return v[k]; }
};
// lane j: the state with component j perturbed (DifferenceQuotientJacobian's y_copy)
struct PertSpecies {
    const double* y;
    double yp;
    int me;
    BDF_INL double operator[](int k) const { return (me == k) ? yp : y[k]; }
};

template <int NS, int NP, int NC, int M>
struct Shared {
    double outl[M];      // the cell's values at the output entries
    double sy[ROW];      // state broadcast
    double sf[ROW];      // f(y) broadcast (Jacobian)
    double red[ROW];     // reductions
    double J[NS * NS];   // saved Jacobian, column-major
    double A[NS * NS];   // I - gamma J -> LU factors, column-major
    int perm[NS];        // (P b)[i] = b[perm[i]]
    double dinv[NS];     // 1 / u(i, i), correctly rounded (lin_solve's quotients)
    int dinv_ok;         // every 1 / u(i, i) finite: the quotients through dinv
    double prm[NP > 0 ? NP : 1];
    double cs[NC > 0 ? NC : 1];
#if CP_NTREAT > 0
    const double* treat_times;     // the pulse start times (a.treat_times)
    int treat_off[CP_NTREAT + 1];
    double creation;               // the cell's creation time (treatment times are experiment times)
#endif
#ifdef CP_PHASES
    long long ph[8];
#endif
};

// CP_PHASES (BCM3_CP_PHASES=1, diagnostic build): clock64 cycles per part of the solve, summed per
// cell into sh.ph and returned in end_y[0..5] (tools/cellpop_phases.py)
#ifdef CP_PHASES
#define CP_PH_BEGIN() const long long ph_t0_ = clock64()
#define CP_PH_END(sh, k) \
    if (lane() == 0) (sh).ph[k] += clock64() - ph_t0_
#else
#define CP_PH_BEGIN() \
    do {              \
    } while (0)
#define CP_PH_END(sh, k) \
    do {                 \
    } while (0)
#endif

template <int NS>
struct GenState {
    double rtol, atol, hmin;
    double zn[QMAX + 1];  // lane i: component i
    double ewt, acor;
    double tau[QMAX + 2], tq[6], l[QMAX + 1];
    double tn, h, hprime, eta, hscale, hu, tretlast;
    double gamma, gammap, gamrat, crate, delp, acnrm, etamax, saved_tq5;
    int q, qprime, qwait, L;
    int nst, nstlp, nstlj;
    int nls_jcur;
    double tstop;  // CVodeSetStopTime (treatment discontinuities)
    int tstopset;
};

// value of lane J of this lane's 16-lane row, in every lane (v_mov_b64_dpp row_newbcast:J; no
// LDS round trip and no SGPR hop)
template <int J>
BDF_INL double rbc(double v)
{
    return __builtin_amdgcn_mov_dpp(v, 0x150 + J, 0xf, 0xf, false);
}
// value of lane (l - D) of the row in lane l; `old` where l - D leaves the row (row_shr:D)
template <int D>
BDF_INL int shr_i(int v, int old)
{
    return __builtin_amdgcn_update_dpp(old, v, 0x110 + D, 0xf, 0xf, false);
}
template <int D>
BDF_INL double shr_d(double v, double old)
{
    const long long b = __builtin_bit_cast(long long, v), o = __builtin_bit_cast(long long, old);
    const int lo = shr_i<D>((int)b, (int)o), hi = shr_i<D>((int)(b >> 32), (int)(o >> 32));
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// sum over the components in component order of a lane value (uniform result): ((p0 + p1) + p2)
// ..., the order of nvector_serial's loops
template <int NS, class SH>
BDF_INL double lane_sum(SH& sh, double p)
{
    if constexpr (NS <= 16) {
        double s = rbc<0>(p);
        cfor<1, NS>([&](auto i) __attribute__((always_inline)) { s = s + rbc<CI(i)>(p); });
        return s;
    } else {
        wave_sync();
        sh.red[lane()] = p;
        wave_sync();
        double s = sh.red[0];
#pragma unroll
        for (int i = 1; i < NS; i++) s += sh.red[i];
        return s;
    }
}

// N_VWrmsNorm
template <int NS, class SH>
BDF_INL double wrms(SH& sh, double x, double w)
{
    const double p = x * w;
    return fsqrt(fdiv_c(lane_sum<NS>(sh, p * p), (double)NS, 1.0 / NS));
}

// ---- treatment trajectories (TreatmentTrajectoryPulses.cpp) --------------------------------------
// pulses starting at times tp[0..n) (sorted): 0 until start + 2, linear up to 1 over 2, 1 until
// start + 10, linear down over 4 (GetConcentration, :22-41)
BDF_INL double pulse_concentration(const double* tp, int n, double time, double creation)
{
    const double global_time = time + creation;
    for (int i = 0; i < n; i++) {
        const double t_in_pulse = global_time - tp[i] - 2.0;
        if (t_in_pulse >= 14.0) continue;
        if (t_in_pulse <= 0.0) return 0.0;
        if (t_in_pulse < 2.0) return t_in_pulse * 0.5;
        if (t_in_pulse < 10.0) return 1.0;
        return 1 - (t_in_pulse - 10.0) * 0.25;
    }
    return 0.0;
}
// FirstDiscontinuity (:44-51): NaN without pulses
BDF_INL double pulse_first(const double* tp, int n, double creation)
{
    return (n > 0) ? tp[0] - creation + 2.0 : __builtin_nan("");
}
// NextDiscontinuity (:53-71): the corner after `time` (exact corner times), NaN past the last
BDF_INL double pulse_next(const double* tp, int n, double time, double creation)
{
    for (int i = 0; i < n; i++) {
        if (time == tp[i] - creation + 2.0) return tp[i] - creation + 4.0;
        if (time == tp[i] - creation + 4.0) return tp[i] - creation + 10.0;
        if (time == tp[i] - creation + 10.0) return tp[i] - creation + 14.0;
        if (time == tp[i] - creation + 14.0) return (i < n - 1) ? tp[i + 1] - creation + 2.0 : __builtin_nan("");
    }
    return __builtin_nan("");
}

#if CP_NTREAT > 0
// the constant species with the treatment species at their concentration at time t
// (Cell::SetTreatmentConcentration before every right-hand side, Cell.cpp:414-430); the generated
// code indexes with literals, so the selects fold at compile time
struct TreatedConstants {
    const double* cs;
    double v[CP_NTREAT];
    BDF_INL double operator[](int k) const
    {
        double r = cs[k];
#pragma unroll
        for (int i = 0; i < CP_NTREAT; i++) r = (k == kTreatSpecies[i]) ? v[i] : r;
        return r;
    }
};
template <class SH>
BDF_INL TreatedConstants treated(const SH& sh, double t)
{
    TreatedConstants c{sh.cs, {}};
#pragma unroll
    for (int i = 0; i < CP_NTREAT; i++)
        c.v[i] = pulse_concentration(sh.treat_times + sh.treat_off[i], sh.treat_off[i + 1] - sh.treat_off[i], t,
                                     sh.creation);
    return c;
}
#define CP_CONSTANTS(sh, t) treated(sh, t)
#else
#define CP_CONSTANTS(sh, t) (sh).cs
#endif

// ---- the model ---------------------------------------------------------------------------------
template <int NS, int NP, int NC, class SH>
BDF_INL double rhs_v(SH& sh, double y, double t)
{
    (void)t;
    double o[NS];
    if constexpr (NS <= 16) {
        // the state reaches every lane of the row by DPP broadcasts: no LDS round trip
        RegSpecies<NS> sp;
        cfor<0, NS>([&](auto k) __attribute__((always_inline)) { sp.v[CI(k)] = rbc<CI(k)>(y); });
        generated_derivative(o, sp, CP_CONSTANTS(sh, t), sh.prm, (const double*)nullptr);
    } else {
        wave_sync();
        if (lane() < NS) sh.sy[lane()] = y;
        wave_sync();
        generated_derivative(o, LdsSpecies{sh.sy}, CP_CONSTANTS(sh, t), sh.prm, (const double*)nullptr);
    }
    double r = o[NS - 1];
#pragma unroll
    for (int k = NS - 2; k >= 0; k--) r = (lane() == k) ? o[k] : r;
    return r;
}

// DifferenceQuotientJacobian (ODESolverCVODE.cpp:496-537) into sh.J: lane j evaluates the
// perturbed state of column j
template <int NS, int NP, int NC, class SH, class S>
BDF_INL void dq_jacobian(SH& sh, const S& s, double y, double fy, double t)
{
    (void)t;
    const double p = fy * s.ewt;
    const double fnorm = sqrt(lane_sum<NS>(sh, p * p) / NS);
    const double srur = 1.4901161193847656e-08;  // SUNRsqrt(DBL_EPSILON)
    const double minInc = (fnorm != 0.0) ? (1000.0 * fabs(s.h) * UROUND * NS * fnorm) : 1.0;
    const double inc = fmax(srur * fabs(y), minInc / s.ewt);
    wave_sync();
    if (lane() < NS) {
        sh.sy[lane()] = y;
        sh.sf[lane()] = fy;
    }
    wave_sync();
    double o[NS];
    generated_derivative(o, PertSpecies{sh.sy, y + inc, lane()}, CP_CONSTANTS(sh, t), sh.prm, (const double*)nullptr);
    const double inc_inv = 1.0 / inc;
    if (lane() < NS) {
#pragma unroll
        for (int i = 0; i < NS; i++) sh.J[lane() * NS + i] = inc_inv * (o[i] - sh.sf[i]);
    }
    wave_sync();
}

// A = I - gamma J (SUNMatCopy + SUNMatScaleAddI), then PartialPivLUExtended::compute_optimized:
// per column k the first largest |a(i, k)|, i >= k, as pivot (a DPP max-scan over the 16 lanes of
// row 0), the row swap (lanes = columns), the scaling of column k, and the Schur update of the
// trailing block element-parallel (lane = (row, column group)), skipping the columns whose pivot-row
// entry a(k, j) is zero as the reference does. Every element sees the same operations in the same
// order as the sequential form.
template <int NS, class SH>
BDF_INL void lin_setup(SH& sh, double gamma)
{
    const int ln = lane();
    wave_sync();
    if constexpr (ROW == 16) {
        // all loads of the saved Jacobian first, then the stores (one LDS latency, not one per element)
        constexpr int NE = (NS * NS + ROW - 1) / ROW;
        double jv[NE];
        cfor<0, NE>([&](auto kk) __attribute__((always_inline)) {
            const int e = ln + CI(kk) * ROW;
            jv[CI(kk)] = (e < NS * NS) ? sh.J[e] : 0.0;
        });
        cfor<0, NE>([&](auto kk) __attribute__((always_inline)) {
            const int e = ln + CI(kk) * ROW;
            const int j = e / NS, i = e - j * NS;
            double a = (-gamma) * jv[CI(kk)];
            if (i == j) a += 1.0;
            if (e < NS * NS) sh.A[e] = a;
        });
    } else {
        for (int e = ln; e < NS * NS; e += ROW) {
            const int j = e / NS, i = e - j * NS;
            double a = (-gamma) * sh.J[e];
            if (i == j) a += 1.0;
            sh.A[e] = a;
        }
    }
    if (ln < NS) sh.perm[ln] = ln;
    wave_sync();
    for (int k = 0; k < NS; k++) {
        int p;
        double biggest, pivot = 0.0;
        if constexpr (NS <= 16) {
            // inclusive max-scan, the lower lane winning ties (maxCoeff's first index); the signed
            // pivot rides along, so the reciprocal needs no read after the row swap
            const double akk = (ln >= k && ln < NS) ? sh.A[k * NS + ln] : 0.0;
            double v = (ln >= k && ln < NS) ? fabs(akk) : -1.0, sv = akk;
            int ix = ln;
            cfor<0, 4>([&](auto r) __attribute__((always_inline)) {
                constexpr int D = 1 << CI(r);
                const double ov = shr_d<D>(v, -2.0);
                const double osv = shr_d<D>(sv, 0.0);
                const int oi = shr_i<D>(ix, ix);
                const bool take = ov >= v;
                v = take ? ov : v;
                sv = take ? osv : sv;
                ix = take ? oi : ix;
            });
            p = __builtin_amdgcn_mov_dpp(ix, 0x15F, 0xf, 0xf, false);  // lane 15 of the row
            biggest = rbc<15>(v);
            pivot = rbc<15>(sv);
        } else {
            biggest = -1.0;
            p = k;
            for (int i = k; i < NS; i++) {
                const double v = fabs(sh.A[k * NS + i]);
                if (v > biggest) {
                    biggest = v;
                    p = i;
                }
            }
            p = __builtin_amdgcn_readfirstlane(p);
            biggest = wave_uniform(biggest);
        }
        if (biggest != 0.0) {
            if (p != k) {
                if (ln < NS) {
                    const double a = sh.A[ln * NS + k];
                    const double b = sh.A[ln * NS + p];
                    sh.A[ln * NS + k] = b;
                    sh.A[ln * NS + p] = a;
                }
                if (ln == 0) {
                    const int t = sh.perm[k];
                    sh.perm[k] = sh.perm[p];
                    sh.perm[p] = t;
                }
                wave_sync();
            }
            if constexpr (ROW != 16) {
                const double inv = 1.0 / sh.A[k * NS + k];
                if (ln > k && ln < NS) sh.A[k * NS + ln] *= inv;
                wave_sync();
            }
        }
        if constexpr (ROW == 16) {
            // lane i of the row: row i of the trailing block. It scales its own column-k entry
            // (l(i, k) = a(i, k) / u(k, k) through the reciprocal, as above), then loads the row and
            // the pivot row in one batch, updates, and stores: one LDS latency per column instead of
            // one per element
            const int i = k + 1 + ln;
            if (i < NS) {
                double lik = sh.A[k * NS + i];
                if (biggest != 0.0) {
                    lik *= 1.0 / pivot;
                    sh.A[k * NS + i] = lik;
                }
                double akj[NS], aij[NS];
                cfor<0, NS>([&](auto jj) __attribute__((always_inline)) {
                    constexpr int j = CI(jj);
                    akj[j] = sh.A[j * NS + k];
                    aij[j] = sh.A[j * NS + i];
                });
                cfor<0, NS>([&](auto jj) __attribute__((always_inline)) {
                    constexpr int j = CI(jj);
                    if (j > k && akj[j] != 0.0) aij[j] -= akj[j] * lik;
                });
                cfor<0, NS>([&](auto jj) __attribute__((always_inline)) {
                    constexpr int j = CI(jj);
                    if (j > k) sh.A[j * NS + i] = aij[j];
                });
            }
        } else {
            for (int i = k + 1 + (ln & 15); i < NS; i += 16) {
                const double lik = sh.A[k * NS + i];
                for (int j = k + 1 + (ln >> 4); j < NS; j += 4) {
                    const double akj = sh.A[j * NS + k];
                    if (akj != 0.0) sh.A[j * NS + i] -= akj * lik;
                }
            }
        }
        wave_sync();
    }
    double r = 1.0;
    if (ln < NS) {
        r = 1.0 / sh.A[ln * NS + ln];
        sh.dinv[ln] = r;
    }
    // singular or subnormal pivots keep the IEEE division (x / 0 = inf, not NaN)
    if (ln == 0) sh.dinv_ok = 1;
    wave_sync();
    if (!(fabs(r) <= 1.7976931348623157e308)) sh.dinv_ok = 0;
}

// The same factorisation for 16-lane rows (NS <= 16) with the matrix in registers: lane i of the row
// holds row i, the row swap exchanges two lanes' rows by ds_bpermute, the pivot row reaches the other
// rows by row broadcasts (the column loop unrolled, so column k is a register and lane k a DPP
// operand); no LDS round trip or barrier per column. The factors and the permutation go to LDS at the
// end in the layout lin_solve reads. Same operations per element in the same order as lin_setup
// (which serves NS > 16): the C4 batch 27.9 -> 25.1 ms with bit-identical logp
// (profiles/r05ag_cellpop_lu_registers.txt).
BDF_INL int rowget_i(int v, int k)
{
    const int addr = ((int)(threadIdx.x & ~(unsigned)(ROW - 1)) + k) << 2;
    return __builtin_amdgcn_ds_bpermute(addr, v);
}
template <int NS, class SH>
BDF_INL void lin_setup_reg(SH& sh, double gamma)
{
    static_assert(NS <= 16, "register LU: one 16-lane row per cell");
    const int ln = lane();
    const bool act = ln < NS;
    const int li = act ? ln : 0;
    wave_sync();
    double a[NS];
    cfor<0, NS>([&](auto J) __attribute__((always_inline)) { a[CI(J)] = sh.J[CI(J) * NS + li]; });
    cfor<0, NS>([&](auto J) __attribute__((always_inline)) {
        double v = (-gamma) * a[CI(J)];
        if (ln == CI(J)) v += 1.0;
        a[CI(J)] = v;
    });
    int perm = ln;
    cfor<0, NS>([&](auto K) __attribute__((always_inline)) {
        constexpr int k = CI(K);
        const double akk = (ln >= k && act) ? a[k] : 0.0;
        double v = (ln >= k && act) ? fabs(akk) : -1.0, sv = akk;
        int ix = ln;
        cfor<0, 4>([&](auto r) __attribute__((always_inline)) {
            constexpr int D = 1 << CI(r);
            const double ov = shr_d<D>(v, -2.0);
            const double osv = shr_d<D>(sv, 0.0);
            const int oi = shr_i<D>(ix, ix);
            const bool take = ov >= v;
            v = take ? ov : v;
            sv = take ? osv : sv;
            ix = take ? oi : ix;
        });
        const int p = __builtin_amdgcn_mov_dpp(ix, 0x15F, 0xf, 0xf, false);
        const double biggest = rbc<15>(v);
        const double pivot = rbc<15>(sv);
        if (biggest != 0.0 && p != k) {
            const int src = (ln == k) ? p : (ln == p) ? k : ln;
            cfor<0, NS>([&](auto J) __attribute__((always_inline)) { a[CI(J)] = rowget(a[CI(J)], src); });
            perm = rowget_i(perm, src);
        }
        const bool below = act && ln > k;
        double lik = a[k];
        if (biggest != 0.0) lik *= 1.0 / pivot;
        if (below) a[k] = lik;
        cfor<k + 1, NS>([&](auto J) __attribute__((always_inline)) {
            const double ukj = rbc<CI(K)>(a[CI(J)]);
            if (below && ukj != 0.0) a[CI(J)] -= ukj * lik;
        });
    });
    if (act) {
        cfor<0, NS>([&](auto J) __attribute__((always_inline)) { sh.A[CI(J) * NS + ln] = a[CI(J)]; });
        sh.perm[ln] = perm;
    }
    double diag = 1.0;
    cfor<0, NS>([&](auto J) __attribute__((always_inline)) { diag = (ln == CI(J)) ? a[CI(J)] : diag; });
    double r = 1.0;
    if (act) {
        r = 1.0 / diag;
        sh.dinv[ln] = r;
    }
    if (ln == 0) sh.dinv_ok = 1;
    wave_sync();
    if (!(fabs(r) <= 1.7976931348623157e308)) sh.dinv_ok = 0;
}

// x / d from r = RN(1 / d): q = RN(x r), then one residual correction RN(q + (x - d q) r) -- the
// correctly rounded quotient (Markstein) in three dependent operations instead of the IEEE
// division sequence, which sits on the critical path of the back substitution
BDF_INL double div_by(double x, double d, double r)
{
    const double q = x * r;
    const double e = __builtin_fma(-d, q, x);
    return __builtin_fma(e, r, q);
}

// x = A^-1 b: P b, unit-lower forward and upper backward substitution (PartialPivLU::solve); the
// solution component of column j reaches the other lanes by a row broadcast
template <int NS, class SH>
BDF_INL double lin_solve(SH& sh, double b)
{
    const int ln = lane();
    double x;
    if constexpr (NS <= 16) {
        // P b by one ds_bpermute within the row (the permutation is read independently of b)
        const int pl = sh.perm[(ln < NS) ? ln : 0];
        x = rowget(b, pl);
        x = (ln < NS) ? x : 0.0;
    } else {
        wave_sync();
        if (ln < NS) sh.red[ln] = b;
        wave_sync();
        x = (ln < NS) ? sh.red[sh.perm[ln]] : 0.0;
    }
    if (BDF_UNLIKELY(!sh.dinv_ok)) {
        for (int j = 0; j < NS - 1; j++) {
            const double xj = rowget(x, j);
            if (ln > j && ln < NS) x = x - sh.A[j * NS + ln] * xj;
        }
        for (int j = NS - 1; j >= 0; j--) {
            if (ln == j) x = x / sh.A[j * NS + j];
            const double xj = rowget(x, j);
            if (ln < j) x = x - sh.A[j * NS + ln] * xj;
        }
    } else if constexpr (NS <= 16) {
        // lane i holds row i of the factors in registers (one batch of LDS loads); the
        // substitutions are then branch-free: every lane computes, selects keep the lanes a
        // column does not update
        double a[NS];
        const int li = (ln < NS) ? ln : 0;
        cfor<0, NS>([&](auto J) __attribute__((always_inline)) { a[CI(J)] = sh.A[CI(J) * NS + li]; });
        const double rinv = sh.dinv[li];
        cfor<0, NS - 1>([&](auto J) __attribute__((always_inline)) {
            constexpr int j = CI(J);
            const double xj = rbc<j>(x);
            const double t = x - a[j] * xj;
            x = (ln > j && ln < NS) ? t : x;
        });
        cfor_down<NS - 1, 0>([&](auto J) __attribute__((always_inline)) {
            constexpr int j = CI(J);
            const double qd = div_by(x, a[j], rinv);
            x = (ln == j) ? qd : x;
            const double xj = rbc<j>(x);
            const double t = x - a[j] * xj;
            x = (ln < j) ? t : x;
        });
    } else {
        for (int j = 0; j < NS - 1; j++) {
            const double xj = bcast(x, j);
            if (ln > j && ln < NS) x = x - sh.A[j * NS + ln] * xj;
        }
        for (int j = NS - 1; j >= 0; j--) {
            if (ln == j) x = div_by(x, sh.A[j * NS + j], sh.dinv[j]);
            const double xj = bcast(x, j);
            if (ln < j) x = x - sh.A[j * NS + ln] * xj;
        }
    }
    return x;
}

// ---- BDF (runtime order; bdf_lane.h with the state across lanes) --------------------------------
template <class S>
BDF_INL void ewt_set(S& s)
{
    s.ewt = frcp(__builtin_fma(s.rtol, fabs(s.zn[0]), s.atol));
}

// q: the order (s.q), or a compile-time order on the path where every cell of the wavefront is at
// the same order, where the order selects fold away (same operations on the same elements)

// f(QMAX) when every active lane is at the maximum order (72 % of cell steps are, per the reference
// solver's own step records), else f(s.q): a wave-uniform branch. Paths for every order measured
// slower than this one (code size; profiles/r05am_cellpop_order_paths.txt)
template <class F>
BDF_INL void with_order(int q, F&& f)
{
#ifndef CP_NO_ORDER_PATHS
    if (__all(q == QMAX)) {
        f(QMAX);
        return;
    }
#endif
    f(q);
}
template <class S>
BDF_INL void rescale(S& s, const int q)
{
    double c = s.eta;
    cfor<1, QMAX + 1>([&](auto j) __attribute__((always_inline)) {
        if (CI(j) <= q) s.zn[CI(j)] *= c;
        c = s.eta * c;
    });
    s.h = s.hscale * s.eta;
    s.hscale = s.h;
}

template <class S>
BDF_INL void predict(S& s, const int q)
{
    s.tn += s.h;
    cfor<1, QMAX + 1>([&](auto k) __attribute__((always_inline)) {
        cfor_down<QMAX, CI(k)>([&](auto j) __attribute__((always_inline)) {
            if (CI(j) <= q) s.zn[CI(j) - 1] += s.zn[CI(j)];
        });
    });
}

template <class S>
BDF_INL void restore(S& s, double saved_t, const int q)
{
    s.tn = saved_t;
    cfor<1, QMAX + 1>([&](auto k) __attribute__((always_inline)) {
        cfor_down<QMAX, CI(k)>([&](auto j) __attribute__((always_inline)) {
            if (CI(j) <= q) s.zn[CI(j) - 1] -= s.zn[CI(j)];
        });
    });
}

template <class S>
BDF_INL double znq_of(const S& s, int q)
{
    double v = 0.0;
    cfor<1, QMAX + 1>([&](auto j) __attribute__((always_inline)) { v = (q == CI(j)) ? s.zn[CI(j)] : v; });
    return v;
}

template <class S>
BDF_INL void increase_bdf(S& s)
{
    double alpha0, alpha1, prod, xi, xiold, hsum, A1;
    double l[QMAX + 1];
    cfor<0, QMAX + 1>([&](auto i) __attribute__((always_inline)) { l[CI(i)] = 0.0; });
    l[2] = alpha1 = prod = xiold = 1.0;
    alpha0 = -1.0;
    hsum = s.hscale;
    cfor<1, QMAX - 1>([&](auto j) __attribute__((always_inline)) {
        if (CI(j) < s.q) {
            hsum += s.tau[CI(j) + 1];
            xi = fdiv(hsum, s.hscale);
            prod *= xi;
            alpha0 -= 1.0 / (CI(j) + 1);
            alpha1 += frcp(xi);
            cfor_down<CI(j) + 2, 2>([&](auto i) __attribute__((always_inline)) { l[CI(i)] = __builtin_fma(l[CI(i)], xiold, l[CI(i) - 1]); });
            xiold = xi;
        }
    });
    A1 = fdiv(-alpha0 - alpha1, prod);
    const double znL = A1 * s.zn[QMAX];
    cfor<2, QMAX + 1>([&](auto j) __attribute__((always_inline)) {
        if (CI(j) == s.q + 1)
            s.zn[CI(j)] = znL;
        else if (CI(j) <= s.q)
            s.zn[CI(j)] = __builtin_fma(l[CI(j)], znL, s.zn[CI(j)]);
    });
    cfor<0, QMAX + 1>([&](auto i) __attribute__((always_inline)) { s.l[CI(i)] = l[CI(i)]; });
}

template <class S>
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
            cfor_down<CI(j) + 2, 2>([&](auto i) __attribute__((always_inline)) { l[CI(i)] = __builtin_fma(l[CI(i)], xi, l[CI(i) - 1]); });
        }
    });
    const double znq = znq_of(s, s.q);
    cfor<2, QMAX>([&](auto j) __attribute__((always_inline)) {
        if (CI(j) < s.q) s.zn[CI(j)] = __builtin_fma(-l[CI(j)], znq, s.zn[CI(j)]);
    });
    cfor<0, QMAX + 1>([&](auto i) __attribute__((always_inline)) { s.l[CI(i)] = l[CI(i)]; });
}

template <class S>
BDF_INL void adjust_order(S& s, int deltaq)
{
    if ((s.q == 2) && (deltaq != 1)) return;
    if (deltaq == 1)
        increase_bdf(s);
    else if (deltaq == -1)
        decrease_bdf(s);
}

template <class S>
BDF_INL int get_dky(const S& s, double t, double& dky)
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
    dky = 0.0;
    cfor_down<QMAX, 0>([&](auto j) __attribute__((always_inline)) {
        if (CI(j) <= s.q) dky = __builtin_fma(c[CI(j)], s.zn[CI(j)], dky);
    });
    return CV_SUCCESS;
}

template <class S>
BDF_INL double set_bdf(S& s, const int q)
{
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
                cfor_down<CI(j), 1>([&](auto i) __attribute__((always_inline)) { s.l[CI(i)] = __builtin_fma(s.l[CI(i) - 1], xi_inv, s.l[CI(i)]); });
            }
        });
        alpha0 -= recip_int(q);
        xistar_inv = -s.l[1] - alpha0;
        hsum += sel(s.tau, q - 1);
        xi_inv = fdiv(s.h, hsum);
        alpha0_hat = -s.l[1] - xi_inv;
        cfor_down<QMAX, 1>([&](auto i) __attribute__((always_inline)) {
            if (CI(i) <= q) s.l[CI(i)] = __builtin_fma(s.l[CI(i) - 1], xistar_inv, s.l[CI(i)]);
        });
    }
    const double A1 = 1.0 - alpha0_hat + alpha0;
    const double A2 = __builtin_fma((double)q, A1, 1.0);
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
    const double rl1 = frcp(s.l[1]);
    s.gamma = s.h * rl1;
    if (s.nst == 0) s.gammap = s.gamma;
    s.gamrat = (s.nst > 0) ? fdiv(s.gamma, s.gammap) : 1.0;
    return rl1;
}

// Newton iteration of cvNls (sunnonlinsol_newton.c:183-322, cvode_nls.c, cvode_ls.c:1415-1663)
template <int NS, int NP, int NC, class SH, class S>
BDF_INL bool newton(SH& sh, S& s, double rl1, int convfail, bool callSetup)
{
    bool jbad = false;
    double cscale = (s.gamrat != 1.0) ? fdiv(2.0, 1.0 + s.gamrat) : 1.0;
    int curiter = 0;
    for (;;) {
        const double y = s.zn[0] + s.acor;
        double f;
        {
            CP_PH_BEGIN();
            f = rhs_v<NS, NP, NC>(sh, y, s.tn);
            CP_PH_END(sh, 0);
        }
        double delta = __builtin_fma(rl1, s.zn[1], s.acor);
        delta = __builtin_fma(-s.gamma, f, delta);
        if (callSetup) {
            if (jbad) convfail = CONV_BAD_J;
            const double dgamma = fabs(fdiv(s.gamma, s.gammap) - 1.0);
            const bool jnew = (s.nst == 0) || (s.nst > s.nstlj + CVLS_MSBJ) ||
                              ((convfail == CONV_BAD_J) && (dgamma < CVLS_DGMAX)) || (convfail == CONV_OTHER);
            if (jnew) {
                s.nstlj = s.nst;
                CP_PH_BEGIN();
                dq_jacobian<NS, NP, NC>(sh, s, y, f, s.tn);
                CP_PH_END(sh, 1);
            }
            {
                CP_PH_BEGIN();
                if constexpr (ROW == 16)
                    lin_setup_reg<NS>(sh, s.gamma);
                else
                    lin_setup<NS>(sh, s.gamma);
                CP_PH_END(sh, 2);
            }
            s.nls_jcur = jnew;
            s.gamrat = 1.0;
            cscale = 1.0;
            s.gammap = s.gamma;
            s.crate = 1.0;
            s.nstlp = s.nst;
            callSetup = false;
            curiter = 0;
        }
        double x;
        {
            CP_PH_BEGIN();
            x = lin_solve<NS>(sh, -delta);
            CP_PH_END(sh, 3);
        }
        if (s.gamrat != 1.0) x *= cscale;
        s.acor += x;
        const double del = wrms<NS>(sh, x, s.ewt);
        if (curiter > 0) s.crate = SUNMAX(CRDOWN * s.crate, fdiv(del, s.delp));
        if (del * SUNMIN(1.0, s.crate) * s.tq[2] <= CORTES) {
            s.acnrm = (curiter == 0) ? del : wrms<NS>(sh, s.acor, s.ewt);
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
        if (!s.nls_jcur) {
            callSetup = true;
            jbad = true;
            s.acor = 0.0;
            continue;
        }
        return false;
    }
}

// cvHin (cvode.c:1884-1990)
template <int NS, int NP, int NC, class SH, class S>
BDF_INL int hin(SH& sh, S& s, double tout)
{
    const double tdiff = tout - s.tn;
    if (tdiff == 0.0) return CV_TOO_CLOSE;
    const int sign = (tdiff > 0.0) ? 1 : -1;
    const double tdist = fabs(tdiff);
    const double tround = UROUND * SUNMAX(fabs(s.tn), fabs(tout));
    if (tdist < 2.0 * tround) return CV_TOO_CLOSE;
    const double hlb = HLB_FACTOR * tround;
    double t1 = frcp(s.ewt);
    t1 = __builtin_fma(HUB_FACTOR, fabs(s.zn[0]), t1);
    const double r = fdiv(fabs(s.zn[1]), t1);
    wave_sync();
    sh.red[lane()] = r;
    wave_sync();
    double hub_inv = sh.red[0];
    for (int i = 1; i < NS; i++) {
        const double ri = sh.red[i];
        hub_inv = (ri > hub_inv) ? ri : hub_inv;
    }
    double hub = HUB_FACTOR * tdist;
    if (hub * hub_inv > 1.0) hub = frcp(hub_inv);
    double hg = fsqrt(hlb * hub);
    if (hub < hlb) {
        s.h = (sign == -1) ? -hg : hg;
        return CV_SUCCESS;
    }
    double hnew = hg;
    for (int count1 = 1; count1 <= MAX_ITERS; count1++) {
        const double hgs = hg * sign;
        const double yy = __builtin_fma(hgs, s.zn[1], s.zn[0]);
        double tv = rhs_v<NS, NP, NC>(sh, yy, s.tn + hgs);
        const double a = frcp(hgs);
        tv = a * (tv - s.zn[1]);
        const double yddnrm = wrms<NS>(sh, tv, s.ewt);
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

constexpr double ONEPSM = 1.000001;

// CVode(..., CV_ONE_STEP) (cvode.c:1016-1440); tstop only with treatment trajectories (CVodeSetStopTime
// of ODESolverCVODE::Solve); returns tret and the output vector's component in yout
template <int NS, int NP, int NC, class SH, class S>
BDF_INL int cvode_one_step(SH& sh, S& s, double tout, double& tret, double& yout)
{
    if (s.nst == 0) {
        s.tretlast = tret = s.tn;
        ewt_set(s);
        s.nstlj = 0;
        s.nls_jcur = 0;
        s.zn[1] = rhs_v<NS, NP, NC>(sh, s.zn[0], s.tn);
        double tout_hin = tout;
        if constexpr (CP_NTREAT > 0) {
            if (s.tstopset && ((s.tstop - s.tn) * (tout - s.tn) <= 0.0)) return CV_ILL_INPUT;
            if (s.tstopset && ((tout - s.tn) * (tout - s.tstop) > 0.0)) tout_hin = s.tstop;
        }
        const int hflag = hin<NS, NP, NC>(sh, s, tout_hin);
        if (hflag != CV_SUCCESS) return hflag;
        // hmax_inv = 0 (no clamp); |h| < hmin -> hmin (cvode.c:1121-1124)
        if (fabs(s.h) < s.hmin) s.h *= s.hmin / fabs(s.h);
        if constexpr (CP_NTREAT > 0)
            if (s.tstopset && ((s.tn + s.h - s.tstop) * s.h > 0.0)) s.h = (s.tstop - s.tn) * (1.0 - 4.0 * UROUND);
        s.hscale = s.h;
        s.hprime = s.h;
        s.zn[1] *= s.h;
    } else {
        const double troundoff = FUZZ_FACTOR * UROUND * (fabs(s.tn) + fabs(s.h));
        if (fabs(s.tn - s.tretlast) > troundoff) {
            s.tretlast = tret = s.tn;
            yout = s.zn[0];
            return CV_SUCCESS;
        }
        if (CP_NTREAT > 0 && s.tstopset) {
            if (fabs(s.tn - s.tstop) <= troundoff) {
                if (get_dky(s, s.tstop, yout) != CV_SUCCESS) return CV_ILL_INPUT;
                s.tretlast = tret = s.tstop;
                s.tstopset = 0;
                return CV_TSTOP_RETURN;
            }
            if ((s.tn + s.hprime - s.tstop) * s.h > 0.0) {
                s.hprime = (s.tstop - s.tn) * (1.0 - 4.0 * UROUND);
                s.eta = fdiv(s.hprime, s.h);
            }
        }
        ewt_set(s);
    }
    {
        const double p = s.zn[0] * s.ewt;
        constexpr double thr = (double)NS * (1.0 / (UROUND * UROUND));
        bool too_much;
        if constexpr (NS <= 16) {
            // NS * max p^2 bounds the sum: far below the threshold (every step in practice) the
            // component-order sum is not needed to decide; near or above it, it decides
            double m = (lane() < NS) ? p * p : 0.0;
            cfor<0, 4>([&](auto r) __attribute__((always_inline)) { m = fmax(m, shr_d<(1 << CI(r))>(m, 0.0)); });
            m = rbc<15>(m);
            too_much = !((double)NS * m <= 0.5 * thr) && (lane_sum<NS>(sh, p * p) > thr);
        } else {
            too_much = lane_sum<NS>(sh, p * p) > thr;
        }
        if (too_much) {
            s.tretlast = tret = s.tn;
            yout = s.zn[0];
            return CV_TOO_MUCH_ACC;
        }
    }
    const double saved_t = s.tn;
    int ncf = 0, nef = 0, nflag = FIRST_CALL;
    bool do_rescale = false;
    if ((s.nst > 0) && (s.hprime != s.h)) {
        if (s.qprime != s.q) {
            adjust_order(s, s.qprime - s.q);
            s.q = s.qprime;
            s.L = s.q + 1;
            s.qwait = s.L;
        }
        do_rescale = true;
    }
    double dsm = 0.0;
    for (;;) {
        double rl1 = 0.0;
        with_order(s.q, [&](const int q) __attribute__((always_inline)) {
            if (do_rescale) rescale(s, q);
            predict(s, q);
            rl1 = set_bdf(s, q);
        });
        do_rescale = true;
        const int convfail = ((nflag == FIRST_CALL) || (nflag == PREV_ERR_FAIL)) ? CONV_NONE : CONV_OTHER;
        const bool callSetup = (nflag == PREV_CONV_FAIL) || (nflag == PREV_ERR_FAIL) || (s.nst == 0) ||
                               (s.nst >= s.nstlp + MSBP) || (fabs(s.gamrat - 1.0) > DGMAX);
        s.acor = 0.0;
        bool conv;
        {
            CP_PH_BEGIN();
            conv = newton<NS, NP, NC>(sh, s, rl1, convfail, callSetup);
            CP_PH_END(sh, 6);
        }
        if (conv) {
            dsm = s.acnrm * s.tq[2];
            if (dsm <= 1.0) break;
        }
        restore(s, saved_t, s.q);
        if (!conv) {
            // cvHandleNFlag (cvode.c:2886-2910)
            ncf++;
            s.etamax = 1.0;
            if ((fabs(s.h) <= s.hmin * ONEPSM) || (ncf == MXNCF)) return CV_CONV_FAILURE;
            s.eta = SUNMAX(ETACF, (s.hmin / fabs(s.h)));
            nflag = PREV_CONV_FAIL;
            continue;
        }
        // cvDoErrorTest (cvode.c:2958-3030)
        nef++;
        nflag = PREV_ERR_FAIL;
        if ((fabs(s.h) <= s.hmin * ONEPSM) || (nef == MXNEF)) return CV_ERR_FAILURE;
        s.etamax = 1.0;
        if (nef <= MXNEF1) {
            double eta = eta_from(BIAS2 * dsm, s.L);
            eta = SUNMAX(ETAMIN, SUNMAX(eta, (s.hmin / fabs(s.h))));
            if (nef >= SMALL_NEF) eta = SUNMIN(eta, ETAMXF);
            s.eta = eta;
            continue;
        }
        if (s.q > 1) {
            s.eta = SUNMAX(ETAMIN, (s.hmin / fabs(s.h)));
            adjust_order(s, -1);
            s.L = s.q;
            s.q--;
            s.qwait = s.L;
            continue;
        }
        s.eta = SUNMAX(ETAMIN, (s.hmin / fabs(s.h)));
        s.h *= s.eta;
        s.hscale = s.h;
        s.qwait = LONG_WAIT;
        const double tv = rhs_v<NS, NP, NC>(sh, s.zn[0], s.tn);
        s.zn[1] = s.h * tv;
        do_rescale = false;
    }
    // cvCompleteStep
    s.nst++;
    s.hu = s.h;
    auto complete = [&](const int q) __attribute__((always_inline)) {
        cfor_down<QMAX, 2>([&](auto i) __attribute__((always_inline)) {
            if (CI(i) <= q) s.tau[CI(i)] = s.tau[CI(i) - 1];
        });
        if ((q == 1) && (s.nst > 1)) s.tau[2] = s.tau[1];
        s.tau[1] = s.h;
        cfor<0, QMAX + 1>([&](auto j) __attribute__((always_inline)) {
            if (CI(j) <= q) s.zn[CI(j)] = __builtin_fma(s.l[CI(j)], s.acor, s.zn[CI(j)]);
        });
    };
    with_order(s.q, complete);
    s.qwait--;
    if ((s.qwait == 1) && (s.q != QMAX)) {
        s.zn[QMAX] = s.acor;
        s.saved_tq5 = s.tq[5];
    }
    // cvPrepareNextStep (L = q + 1 throughout: every order change sets both)
    CP_PH_BEGIN();
    if (s.etamax == 1.0) {
        s.qwait = SUNMAX(s.qwait, 2);
        s.qprime = s.q;
        s.hprime = s.h;
        s.eta = 1.0;
    } else {
        with_order(s.q, [&](const int q) __attribute__((always_inline)) {
            const int L = q + 1;
            const double etaq = eta_from(BIAS2 * dsm, L);
            double eta = etaq;
            s.qprime = q;
            if (s.qwait == 0) {
                s.qwait = 2;
                double etaqm1 = 0.0, etaqp1 = 0.0;
                if (q > 1) etaqm1 = eta_from(BIAS1 * wrms<NS>(sh, znq_of(s, q), s.ewt) * s.tq[1], q);
                if ((q != QMAX) && (s.saved_tq5 != 0.0)) {
                    const double cquot = fdiv(s.tq[5], s.saved_tq5) * powI(fdiv(s.h, s.tau[2]), L);
                    const double tv = __builtin_fma(-cquot, s.zn[QMAX], s.acor);
                    etaqp1 = eta_from(BIAS3 * wrms<NS>(sh, tv, s.ewt) * s.tq[3], L + 1);
                }
                const double etam = SUNMAX(etaqm1, SUNMAX(etaq, etaqp1));
                if (etam < THRESH) {
                    eta = 1.0;
                } else if (etam == etaq) {
                    eta = etaq;
                } else if (etam == etaqm1) {
                    eta = etaqm1;
                    s.qprime = q - 1;
                } else {
                    eta = etaqp1;
                    s.qprime = q + 1;
                    s.zn[QMAX] = s.acor;
                }
            }
            if (eta < THRESH) {
                s.eta = 1.0;
                s.hprime = s.h;
            } else {
                s.eta = SUNMIN(eta, s.etamax);
                s.hprime = s.h * s.eta;
            }
        });
    }
    CP_PH_END(sh, 7);
    s.etamax = (s.nst <= SMALL_NST) ? ETAMX2 : ETAMX3;
    s.acor *= s.tq[2];
    // tn at or near tstop (cvode.c:1410-1426)
    if (CP_NTREAT > 0 && s.tstopset) {
        const double troundoff = FUZZ_FACTOR * UROUND * (fabs(s.tn) + fabs(s.h));
        if (fabs(s.tn - s.tstop) <= troundoff) {
            get_dky(s, s.tstop, yout);
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
    yout = s.zn[0];
    return CV_SUCCESS;
}

// get_threshold_crossing_time in the non-stored mode (see oracle/cellpop_ref.cpp): the
// interpolant of the unused buffer is 0, so the bisection only walks to one end
// component J of the row's state in every lane of the row (the event species' value)
template <int J>
BDF_INL double ev_value(double y)
{
    if constexpr (ROW == 16)
        return rbc<J>(y);
    else
        return rowget(y, J);
}

BDF_INL double crossing_time(double t, double prev, double threshold, bool above)
{
    double dt = (t - prev) * 0.5;
    double time = prev + dt;
    for (int it = 0; it < 10; it++) {
        const double x = 0.0;
        dt *= 0.5;
        const bool down = above ? (x > threshold) : (x < threshold);
        time = down ? time - dt : time + dt;
    }
    return time;
}

// ---- stored integration points (synchronised data; Cell.cpp:152, 232-233) -----------------------
#ifndef CP_STORED
#define CP_STORED 0
#endif
#ifndef CP_NSTORE
#define CP_NSTORE 0
#endif
// one CVodeTimepoint record (ODESolverCVODE.cpp:375-401): cvode_time, tn, h, hu, q, then zn[j] of
// the stored species m at 5 + j * CP_NSTORE + m (the species the data read, kStoreIx)
constexpr int CP_REC = cpk::cp_record_doubles(QMAX, CP_NSTORE);
static_assert(QMAX == cpk::CP_STORE_QMAX, "cellpop_args.h's record layout (the host's store size) assumes QMAX");

// the step's interpolating polynomial at `time` in every lane: sum over j = q..0 of s^j zn[j], s =
// (time - tn) / h, s^j by repeated products (GetInterpolatedY / get_threshold_crossing_time's
// loop, ODESolverCVODE.cpp:232-240, 292-301)
template <class S>
BDF_INL double interp_lane(const S& s, double time)
{
    const double sv = (time - s.tn) / s.h;
    double pw[QMAX + 1];
    pw[0] = 1.0;
    cfor<1, QMAX + 1>([&](auto j) __attribute__((always_inline)) { pw[CI(j)] = pw[CI(j) - 1] * sv; });
    double y = 0.0;
    cfor_down<QMAX, 0>([&](auto j) __attribute__((always_inline)) {
        if (CI(j) <= s.q) y = __builtin_fma(pw[CI(j)], s.zn[CI(j)], y);
    });
    return y;
}

// get_threshold_crossing_time with stored integration points (ODESolverCVODE.cpp:264-320): ten
// bisection steps between the previous step's time and t on the polynomial of the step just
// taken (its record is the solver's current state), species J
template <int J, class S>
BDF_INL double crossing_time_stored(const S& s, double t, double prev, double threshold, bool above)
{
    double dt = (t - prev) * 0.5;
    double time = prev + dt;
    for (int it = 0; it < 10; it++) {
        const double x = ev_value<J>(interp_lane(s, time));
        dt *= 0.5;
        const bool down = above ? (x > threshold) : (x < threshold);
        time = down ? time - dt : time + dt;
    }
    return time;
}

// ---- solver_type="DP5" (ODESolverDP5, src/odecommon/ODESolverDP5.cpp) ------------------------------
#ifndef CP_DP5
#define CP_DP5 0
#endif
static_assert(!(CP_DP5 && CP_STORED), "the DP5 solver has no stored integration points");
// the largest of the components' values, NaN ignored (std::max(maxdiff, diff) from -inf in component
// order keeps the first of equal values and skips NaN: the maximum of the non-NaN values, exact in
// any order), uniform over the row
BDF_INL double row_max_nonnan(double v)
{
    double m = (lane() < CP_NS && v == v) ? v : -__builtin_inf();
    if constexpr (ROW == 16) {
        cfor<0, 4>([&](auto r) __attribute__((always_inline)) {
            const double o = shr_d<(1 << CI(r))>(m, -__builtin_inf());
            m = (m < o) ? o : m;
        });
        return rbc<15>(m);
    } else {
        for (int k = 0; k < CP_NS; k++) {
            const double o = bcast(m, k);
            m = (m < o) ? o : m;
        }
        return m;
    }
}

// pow(maxdiff, -0.2) of Hairer's step-size factor (ODESolverDP5.cpp:158, 174): glibc's pow on the
// loaded libm's tables (xm::pow_glibc_pos: e_pow.c's main path, which every finite x > 0 takes for
// y = -0.2), so the step sequence is the reference's; 0, inf and NaN through the device's pow (the
// IEEE special values, the same in both)
BDF_INL double dp5_pow_m02(double x, const void* tables)
{
    const xm::GlibcPow* T = static_cast<const xm::GlibcPow*>(tables);
    if (T && T->ok && x > 0.0 && x < __builtin_inf()) return xm::pow_glibc_pos(x, -0.2, *T);
    return pow(x, -0.2);
}

// ODESolverDP5::ApplyRK (ODESolverDP5.cpp:327-412): the stages k1..k6, the 5th-order solution ytmp,
// FSAL k6, and the error ratio max_i |err_i| / (atol + rtol |ytmp_i + k6_i dt|); lane i = component i
struct Dp5 {
    double yn, ytmp, k0, k1, k2, k3, k4, k5, k6;
};
template <int NS, int NP, int NC, class SH>
BDF_INL double dp5_apply_rk(SH& sh, Dp5& s, double t, double dt, double rtol, double atol)
{
    s.ytmp = s.yn + dt * 0.2 * s.k0;
    s.k1 = rhs_v<NS, NP, NC>(sh, s.ytmp, t + 0.2 * dt);
    s.ytmp = s.yn + dt * (+0.075 * s.k0 + 0.225 * s.k1);
    s.k2 = rhs_v<NS, NP, NC>(sh, s.ytmp, t + 0.3 * dt);
    s.ytmp = s.yn + dt * (+0.97777777777777777777777777777778 * s.k0 - 3.7333333333333333333333333333333 * s.k1 +
                          3.5555555555555555555555555555556 * s.k2);
    s.k3 = rhs_v<NS, NP, NC>(sh, s.ytmp, t + 0.8 * dt);
    s.ytmp = s.yn + dt * (+2.9525986892242036274958085657674 * s.k0 - 11.595793324188385916780978509374 * s.k1 +
                          9.8228928516994360615759792714525 * s.k2 - 0.29080932784636488340192043895748 * s.k3);
    s.k4 = rhs_v<NS, NP, NC>(sh, s.ytmp, t + 0.88888888888888888888888888888889 * dt);
    s.ytmp = s.yn + dt * (+2.8462752525252525252525252525253 * s.k0 - 10.757575757575757575757575757576 * s.k1 +
                          8.9064227177434724604535925290642 * s.k2 + 0.27840909090909090909090909090909 * s.k3 -
                          0.27353130360205831903945111492281 * s.k4);
    s.k5 = rhs_v<NS, NP, NC>(sh, s.ytmp, t + dt);
    s.ytmp = s.yn + dt * (+0.09114583333333333333333333333333 * s.k0 + 0.44923629829290206648697214734951 * s.k2 +
                          0.65104166666666666666666666666667 * s.k3 - 0.32237617924528301886792452830189 * s.k4 +
                          0.13095238095238095238095238095238 * s.k5);
    s.k6 = rhs_v<NS, NP, NC>(sh, s.ytmp, t + dt);
    double error = dt * (+0.00123263888888888888888888888889 * s.k0 - 0.00425277029050613956274333632824 * s.k2 +
                         0.03697916666666666666666666666667 * s.k3 - 0.05086379716981132075471698113208 * s.k4 +
                         0.04190476190476190476190476190476 * s.k5 - 0.025 * s.k6);
    error = fabs(error);
    const double D = atol + rtol * fabs(s.ytmp + s.k6 * dt);
    return row_max_nonnan(error / D);
}

// Hairer's dense output of the step (ODESolverDP5.cpp:205-221; Hairer I, II.5 p179)
BDF_INL double dp5_dense(const Dp5& s, double theta, double dt)
{
    const double thetaSq = theta * theta;
    const double b1 = theta * (1.0 + theta * (-2.7854166666666669 + theta * (2.8861111111111111 + theta * (-1.0095486111111112))));
    const double b3 = 33.33333333333333 * thetaSq * (0.11363881401617251 + theta * (-0.1682659478885894 + theta * 0.068104222821203958));
    const double b4 = -2.5 * thetaSq * (0.675 + theta * (-1.8 + theta * (0.8645833333333333)));
    const double b5 = 21.491745283018869 * thetaSq * (-0.012 + theta * (0.058666666666666666 + theta * (-0.06166666666666666)));
    const double b6 = -3.1428571428571428 * thetaSq * (-0.3 + theta * (0.9666666666666666 + theta * (-0.7083333333333333)));
    return s.yn + dt * (b1 * s.k0 + b3 * s.k2 + b4 * s.k3 + b5 * s.k4 + b6 * s.k5);
}

// GetInterpolatedY's time check on a record (tn, hu): false = "Time error for interpolation" (NaN)
BDF_INL bool interp_time_ok(double t, double tn, double hu)
{
    double tfuzz = 100.0 * UROUND * (fabs(tn) + fabs(hu));
    if (hu < 0.0) tfuzz = -tfuzz;
    const double tp = tn - hu - tfuzz;
    const double tn1 = tn + tfuzz;
    return !((t - tp) * (t - tn1) > 0.0);
}

}  // namespace cpk

// One cell per workgroup (64 lanes): Cell::Simulate -> ODESolver::SolveReturnSolution ->
// ODESolverCVODE::Solve with the integration-step callback, then the values the experiment's
// data likelihoods read (GetInterpolatedSpeciesValue) at every output entry.
#ifndef CP_WAVES_PER_EU
// occupancy target: four-cell wavefronts hold 4 cells' LDS (~18 KB, so at most 2 per SIMD) and
// get the full 256 VGPRs; one-cell wavefronts run 3 per SIMD at 168 VGPRs (measured best for
// NS = 15 in that layout: 2 waves 62 ms, 3 waves 51 ms, 4 waves 61 ms per C4 batch)
#define CP_WAVES_PER_EU ((CP_NS <= 16) ? 2 : 3)
#endif
// CP_CELLS_PER_WAVE cells per workgroup (one wavefront): cell blockIdx.x * CPW + row
namespace cpk {
using CellShared = Shared<CP_NS, CP_NP, CP_NC, CP_M>;

// the work queue's per-row cell inputs in LDS (cp_queue_kernel's init writes them, and sh.prm)
struct CellIn {
    double y0[CP_NS];
    double creation;
};
// a cell's end state: read by its daughters' initialisation, which the work queue runs on any wavefront
// of the launch -- stored device-coherent there (no cache write-back of the whole L2 to publish it)
__device__ __forceinline__ void st_end(double* p, double v)
{
#if CP_QUEUE
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    *p = v;
#endif
}

// One cell on this lane's row: Cell::Simulate (Cell.cpp:193-273) from params / y0 / creation[slot] (or,
// in the work queue, sh.prm and `in`) to the cell's outputs at [slot]; wi = the row's index in the launch
// (the stored mode's records)
__device__ __forceinline__ void cp_solve_cell(const CpSolveArgs& a, CellShared& sh, const int slot, const int wi,
                                              const CellIn* in = nullptr)
{
    constexpr int NS = CP_NS, NP = CP_NP, NC = CP_NC;
    constexpr int MM = CP_M;
    const int ln = lane();
    if (!in)
        for (int k = ln; k < NP; k += ROW) sh.prm[k] = a.params[(size_t)slot * NP + k];
    for (int k = ln; k < NC; k += ROW) sh.cs[k] = a.constant_species[k];
    const double creation = in ? in->creation : a.creation[slot];
#if CP_NTREAT > 0
    sh.treat_times = a.treat_times;
    for (int k = ln; k <= CP_NTREAT; k += ROW) sh.treat_off[k] = a.treat_offset[k];
    sh.creation = creation;
#endif
    const double y0 = (ln < NS) ? (in ? in->y0[ln] : a.y0[(size_t)slot * NS + ln]) : 0.0;
#if CP_STORED
    // the stored-species slot of this lane's component (-1: not read by the data)
    int my_store = -1;
    cfor<0, NS>([&](auto k) __attribute__((always_inline)) {
        if (ln == CI(k)) my_store = kStoreIx[CI(k)];
    });
    // the records of this work item (the store is reused by every launch: a cell's records are read
    // back by its own evaluation passes before the solve ends)
    double* const rec0 = a.store + (size_t)wi * a.store_cap * CP_REC;
    int nrec = 0;
    bool overflow = false;
#endif
    double ylast = y0, tlast = 0.0;  // stored mode: the last step's output and time
    const int M = MM;
    double* outv = sh.outl;
    for (int k = ln; k < M; k += ROW) outv[k] = __builtin_nan("");
#ifdef CP_PHASES
    if (ln < 8) sh.ph[ln] = 0;
    const long long ph_kernel0 = clock64();
#endif
    wave_sync();

    // Cell::Simulate (Cell.cpp:193-210)
    double previous_step_time = 0.0;
    double sim_end = a.end_time - creation;
    if (M > 0) sim_end = fmax(sim_end, a.output_times[M - 1] - creation);
    double ev[5];
    for (int k = 0; k < 5; k++) ev[k] = __builtin_nan("");
    bool divided = false, died = false, ok = true;
    int nst = 0;
    // SolveReturnSolution: output times before the cell's t = 0 + DBL_EPSILON get y0
    int ti = 0;
    bool solve;
    if constexpr (CP_STORED) {
        // SolveStoreIntegrationPoints (ODESolver.cpp:136-150): the whole simulation time, no outputs
        solve = sim_end > 2.220446049250313e-16;
        if (!solve) ok = false;
    } else {
        while (ti < M && a.output_times[ti] - creation < 2.220446049250313e-16) {
            const int sp = a.output_species[ti];
            if (sp >= 0 && ln == sp) outv[ti] = y0;
            ti++;
        }
        solve = ti < M;
    }
    double yend = y0;
#if CP_DP5
    if (solve) {
        // ODESolverDP5::Solve (ODESolverDP5.cpp:100-285) under SolveReturnSolution: the Solve resets
        // every output, those before the cell's t = 0 + DBL_EPSILON included, to NaN (:103-105)
        for (int k = ln; k < ti; k += ROW) outv[k] = __builtin_nan("");
        double end_time = a.output_times[M - 1] - creation;
        double t = 0.0, dt = (1.0 < a.hmax) ? 1.0 : a.hmax;  // std::min(max_dt, 1.0)
        Dp5 r;
        r.yn = y0;
        r.k0 = rhs_v<NS, NP, NC>(sh, r.yn, 0.0);
        r.k1 = r.k2 = r.k3 = r.k4 = r.k5 = r.k6 = r.ytmp = 0.0;
        int tpi = ti;
        double next_out = a.output_times[tpi] - creation;
        double ylast_out = __builtin_nan("");  // solver_output's last column (every component)
        for (;;) {
            double cur_dt = dt, next_dt = dt;
            bool succeeded = false;
            for (int att = 0; att < 10; att++) {
                double maxdiff = dp5_apply_rk<NS, NP, NC>(sh, r, t, cur_dt, a.rtol, a.atol);
                if (maxdiff != maxdiff || maxdiff == -__builtin_inf()) {
                    ok = false;
                    break;
                }
                // Hairer I, II.4 p167 (:152-184)
                if (maxdiff > 1.1) {
                    if (cur_dt == a.hmin) break;
                    double scale = 0.9 * dp5_pow_m02(maxdiff, a.pow_tables);
                    scale = (0.2 < scale) ? scale : 0.2;
                    cur_dt *= scale;
                    if (cur_dt < a.hmin) cur_dt = a.hmin;
                } else if (maxdiff < 0.5) {
                    maxdiff = (maxdiff < 1e-5) ? 1e-5 : maxdiff;
                    double scale = 0.9 * dp5_pow_m02(maxdiff, a.pow_tables);
                    scale = (5.0 < scale) ? 5.0 : scale;
                    next_dt = cur_dt * scale;
                    if (next_dt > a.hmax) next_dt = a.hmax;
                    succeeded = true;
                    break;
                } else {
                    next_dt = cur_dt;
                    succeeded = true;
                    break;
                }
            }
            if (!ok) break;
            if (!succeeded) {  // "Time step adaptation did not converge"
                ok = false;
                break;
            }
            // the outputs the step passed (:203-236): all done -> the step is not finished
            const double target_t = t + cur_dt;
            bool done = false;
            while (target_t >= next_out) {
                const double theta = (next_out - t) / cur_dt;
                const double v = (theta >= 1.0) ? r.ytmp : dp5_dense(r, theta, cur_dt);
                const int sp = a.output_species[tpi];
                if (sp >= 0 && ln == sp) outv[tpi] = v;
                if (tpi == M - 1) ylast_out = v;
                tpi++;
                if (tpi == M) {
                    done = true;
                    break;
                }
                next_out = a.output_times[tpi] - creation;
            }
            if (done) break;
            r.k0 = r.k6;
            r.yn = r.ytmp;
            t += cur_dt;
            nst++;
            // Cell::integration_step_cb (Cell.cpp:463-538), its result ignored by the DP5 solver: DP5
            // has no threshold crossings (get_threshold_crossing_time returns NaN, :322-327), so the
            // event times stay NaN, max(simulation end, NaN + past) keeps the simulation end, and a
            // division or death only moves the simulation end to the current step
            if constexpr (CP_EV4 >= 0)
                if (ev_value<CP_EV4>(r.yn) > 1e-3) end_time = sim_end;
            if constexpr (CP_EV5 >= 0) {
                if (a.divide_cells && ev_value<CP_EV5>(r.yn) > 1.0) {
                    sim_end = t;
                    yend = r.yn;
                    divided = true;
                }
            }
            if constexpr (CP_EV6 >= 0) {
                if (ev_value<CP_EV6>(r.yn) > 1.0) {
                    sim_end = t;
                    yend = r.yn;
                    died = true;
                }
            }
            if (t >= end_time) break;
            if (nst == a.max_steps) {
                ok = false;
                break;
            }
            dt = next_dt;
        }
        if (ok && !divided && !died) yend = ylast_out;
    }
#else
    if (solve) {
        GenState<NS> s;
        s.rtol = a.rtol;
        s.atol = a.atol;
        s.hmin = a.hmin;
        cfor<0, QMAX + 1>([&](auto j) __attribute__((always_inline)) { s.zn[CI(j)] = 0.0; });
        cfor<0, QMAX + 2>([&](auto j) __attribute__((always_inline)) { s.tau[CI(j)] = 0.0; });
        cfor<0, 6>([&](auto j) __attribute__((always_inline)) { s.tq[CI(j)] = 0.0; });
        cfor<0, QMAX + 1>([&](auto j) __attribute__((always_inline)) { s.l[CI(j)] = 0.0; });
        s.h = s.hprime = s.eta = s.hscale = s.tretlast = 0.0;
        s.gamma = s.gammap = s.gamrat = s.crate = s.delp = s.acnrm = s.saved_tq5 = 0.0;
        s.crate = 1.0;
        s.qprime = 1;
        s.nstlj = 0;
        s.nls_jcur = 0;
        s.ewt = 0.0;
        s.acor = 0.0;
        // CVodeReInit(0, y0)
        s.tn = 0.0;
        s.q = 1;
        s.L = 2;
        s.qwait = 2;
        s.etamax = ETAMX1;
        s.hu = 0.0;
        s.zn[0] = y0;
        s.nst = 0;
        s.nstlp = 0;
        s.tstop = 0.0;
        s.tstopset = 0;
        // Cell::Simulate: the first treatment discontinuity (Cell.cpp:212-229) becomes the solver's
        // stop time (ODESolver::SetDiscontinuity ignores times <= 0; ODESolverCVODE::Solve :337-339)
        double next_disc = __builtin_nan("");
#if CP_NTREAT > 0
        {
            double first = __builtin_nan("");
            for (int i = 0; i < CP_NTREAT; i++) {
                const double* tp = a.treat_times + sh.treat_off[i];
                const int nt = sh.treat_off[i + 1] - sh.treat_off[i];
                double dd = pulse_first(tp, nt, creation);
                if (dd == dd)
                    while (dd < 0.0) dd = pulse_next(tp, nt, dd, creation);
                if (!(first < dd)) first = dd;
            }
            if (first == first && first > 0.0) next_disc = first;
        }
        if (next_disc == next_disc) {
            s.tstop = next_disc;
            s.tstopset = 1;
        }
#endif
        double end_time = CP_STORED ? sim_end : a.output_times[M - 1] - creation;
        double t = 0.0;
        int tpi = ti;
        // the next output time in a register: no global load on every step's critical path
        double next_out = a.output_times[(tpi < M) ? tpi : M - 1] - creation;
        for (;;) {
            double tret, y;
            int r;
            {
                CP_PH_BEGIN();
                r = cvode_one_step<NS, NP, NC>(sh, s, end_time, tret, y);
                CP_PH_END(sh, 4);
            }
            if (r < 0) {
                ok = false;
                break;
            }
            t = tret;
            nst++;
#if CP_STORED
            // ODESolverCVODE::Solve (:375-401): the step's record; the buffer holds store_cap records
            // (fewer than max_steps: the host grows the store and runs the generation again)
            if (nrec >= a.store_cap) {
                overflow = true;
                ok = false;
                break;
            }
            {
                double* rec = rec0 + (size_t)nrec * CP_REC;
                if (ln == 0) {
                    rec[0] = t;
                    rec[1] = s.tn;
                    rec[2] = s.h;
                    rec[3] = s.hu;
                    rec[4] = (double)s.q;
                }
                if (my_store >= 0)
                    cfor<0, QMAX + 1>([&](auto j) __attribute__((always_inline)) {
                        if (CI(j) <= s.q) rec[5 + CI(j) * CP_NSTORE + my_store] = s.zn[CI(j)];
                    });
                nrec++;
            }
            ylast = y;
            tlast = t;
#endif
            while (!CP_STORED && tpi < M && tret >= next_out) {
                double dky;
                if (get_dky(s, next_out, dky) != CV_SUCCESS) {
                    ok = false;
                    break;
                }
                const int sp = a.output_species[tpi];
                if (sp >= 0 && ln == sp) outv[tpi] = dky;
                tpi++;
                if (tpi < M) next_out = a.output_times[tpi] - creation;
            }
            if (!ok) break;
            // Cell::integration_step_cb (Cell.cpp:463-538) on CVode's output vector
            bool cont = true;
            if constexpr (CP_EV0 >= 0)
                if (ev[0] != ev[0] && ev_value<CP_EV0>(y) > 1e-4) ev[0] = CP_STORED ? crossing_time_stored<CP_EV0>(s, t, previous_step_time, 1e-4, true) : crossing_time(t, previous_step_time, 1e-4, true);
            if constexpr (CP_EV1 >= 0)
                if (ev[1] != ev[1] && ev_value<CP_EV1>(y) > 1.95) ev[1] = CP_STORED ? crossing_time_stored<CP_EV1>(s, t, previous_step_time, 1.95, true) : crossing_time(t, previous_step_time, 1.95, true);
            if constexpr (CP_EV2 >= 0)
                if (ev[2] != ev[2] && ev_value<CP_EV2>(y) > 0.5) ev[2] = CP_STORED ? crossing_time_stored<CP_EV2>(s, t, previous_step_time, 0.5, true) : crossing_time(t, previous_step_time, 0.5, true);
            if constexpr (CP_EV3 >= 0)
                if (ev[3] != ev[3] && ev_value<CP_EV3>(y) < 0.5) ev[3] = CP_STORED ? crossing_time_stored<CP_EV3>(s, t, previous_step_time, 0.5, false) : crossing_time(t, previous_step_time, 0.5, false);
            if constexpr (CP_EV4 >= 0) {
                if (ev[4] != ev[4] && ev_value<CP_EV4>(y) > 1e-3) {
                    ev[4] = CP_STORED ? crossing_time_stored<CP_EV4>(s, t, previous_step_time, 1e-3, true)
                                      : crossing_time(t, previous_step_time, 1e-3, true);
                    sim_end = fmax(sim_end, ev[4] + a.past_cs);
                    end_time = sim_end;
                }
            }
            if constexpr (CP_EV5 >= 0) {
                if (a.divide_cells && ev_value<CP_EV5>(y) > 1.0) {
                    if constexpr (CP_STORED) {
                        // the division time on the step's interpolant and GetInterpolatedY there: the
                        // solve's iterator finds the last record (the bisection stays inside
                        // (previous step, t)), NaN when its time check fails (Cell.cpp:502-505)
                        const double td = crossing_time_stored<CP_EV5>(s, t, previous_step_time, 1.0, true);
                        sim_end = td;
                        yend = interp_time_ok(td, s.tn, s.hu) ? interp_lane(s, td) : __builtin_nan("");
                    } else {
                        sim_end = t;
                        yend = y;
                    }
                    divided = true;
                    cont = false;
                }
            }
            if constexpr (CP_EV6 >= 0) {
                if (ev_value<CP_EV6>(y) > 1.0) {
                    if constexpr (CP_STORED) {
                        const double td = crossing_time_stored<CP_EV6>(s, t, previous_step_time, 1.0, true);
                        sim_end = td;
                        yend = interp_time_ok(td, s.tn, s.hu) ? interp_lane(s, td) : __builtin_nan("");
                    } else {
                        sim_end = t;
                        yend = y;
                    }
                    died = true;
                    cont = false;
                }
            }
            previous_step_time = t;
            if (!cont) break;
            if (t >= end_time) break;
            if (nst == a.max_steps) {
                ok = false;
                break;
            }
#if CP_NTREAT > 0
            // a treatment discontinuity: Cell::discontinuity_cb gives the next one, then CVodeReInit at
            // (t, y) and the new stop time (ODESolverCVODE::Solve :449-460; Cell.cpp:447-461)
            if (next_disc == next_disc && (r == CV_TSTOP_RETURN || next_disc == t)) {
                double dn = __builtin_inf();
                for (int i = 0; i < CP_NTREAT; i++) {
                    const double dd = pulse_next(a.treat_times + sh.treat_off[i], sh.treat_off[i + 1] - sh.treat_off[i], t,
                                                 creation);
                    if (dd < dn) dn = dd;
                }
                next_disc = (dn == __builtin_inf()) ? __builtin_nan("") : dn;
                // CVodeReInit(t, y) (cvode.c:706-760)
                s.tn = t;
                s.q = 1;
                s.L = 2;
                s.qwait = 2;
                s.etamax = ETAMX1;
                s.hu = 0.0;
                s.zn[0] = y;
                s.nst = 0;
                s.nstlp = 0;
                if (next_disc == next_disc && next_disc < __builtin_inf()) {
                    s.tstop = next_disc;
                    s.tstopset = 1;
                }
            }
#endif
        }
        if (ok && !divided && !died) {
            if constexpr (CP_STORED) {
                // simulation_end_y = the solver's current y (Cell.cpp:247-249)
                yend = ylast;
            } else {
                // simulation_end_y = the solution at the last output time
                double dky = 0.0;
                get_dky(s, a.output_times[M - 1] - creation, dky);
                yend = dky;
            }
        }
    }
#endif
#if CP_STORED
    // Experiment::EvaluateLogProbability's passes (Experiment.cpp:277-292): per synchronisation
    // point in enum order, the interpolation iterator restarted, the entries of that pass in
    // time order; Cell::GetInterpolatedSpeciesValue (Cell.cpp:280-327) -> GetInterpolatedY: the
    // first record whose time is past the request, its polynomial, the cached vector while the
    // time repeats. The records are this row's own stores (visible after the barrier).
    wave_sync();
    if (ok) {
        const double toff = a.sync_offset[slot];
        for (int p = 0; p <= 4; p++) {
            const double evp = (p == 0) ? ev[0] : (p == 1) ? ev[2] : (p == 2) ? ev[3] : ev[4];
            int iter = 0;
            double itime = __builtin_nan("");
            bool inan = false;
            for (int k = 0; k < M; k++) {
                const int sp = a.output_species[k];
                if (a.output_sync[k] != p || sp < 0) continue;
                const double time = a.output_times[k] + toff;
                const double ct = (p == 4) ? time - creation : time + ((evp != evp) ? sim_end : evp);
                double x = __builtin_nan("");
                if (!(ct < 0.0 || ct > sim_end)) {
                    if (!(ct == itime)) {
                        while (iter < nrec && rec0[(size_t)iter * CP_REC] <= ct) iter++;
                        if (iter == nrec) {
                            itime = __builtin_nan("");
                            inan = true;
                        } else {
                            itime = ct;
                            const double* r = rec0 + (size_t)iter * CP_REC;
                            inan = !interp_time_ok(ct, r[1], r[3]);
                        }
                    }
                    if (!inan) {
                        const double* r = rec0 + (size_t)iter * CP_REC;
                        const int q = (int)r[4];
                        const int m = kStoreIx[sp];
                        const double sv = (ct - r[1]) / r[2];
                        double pw[QMAX + 1];
                        pw[0] = 1.0;
                        cfor<1, QMAX + 1>([&](auto j) __attribute__((always_inline)) { pw[CI(j)] = pw[CI(j) - 1] * sv; });
                        x = 0.0;
                        cfor_down<QMAX, 0>([&](auto j) __attribute__((always_inline)) {
                            if (CI(j) <= q) x = __builtin_fma(pw[CI(j)], r[5 + CI(j) * CP_NSTORE + m], x);
                        });
                    }
                }
                if (ln == 0) outv[k] = x;
            }
        }
    }
#endif
    // GetInterpolatedSpeciesValue: NaN outside [0, simulation_end_time] of the cell
    wave_sync();
    for (int k = ln; k < M; k += ROW) {
        const double ct = a.output_times[k] - creation;
        a.out_values[(size_t)slot * M + k] = (!CP_STORED && (ct < 0.0 || ct > sim_end)) ? __builtin_nan("") : outv[k];
    }
    if (ln < NS) st_end(a.end_y + (size_t)slot * NS + ln, yend);
#ifdef CP_PHASES
    if (ln == 0) sh.ph[5] = clock64() - ph_kernel0;
    wave_sync();
    if (ln < 8 && ln < NS) a.end_y[(size_t)slot * NS + ln] = (double)sh.ph[ln];
#endif
    if (ln == 0) {
#if CP_STORED
        // the stored mode ends at the last step taken (Cell.cpp:247-249)
        const double achieved_cell_time = (divided || died) ? sim_end : tlast;
#else
        const double achieved_cell_time = (divided || died) ? sim_end : (a.output_times[M - 1] - creation);
#endif
        a.sim_end[slot] = sim_end;
        st_end(a.achieved + slot, achieved_cell_time + creation);
        // bit4: SimulateCell adds two daughters (divide_cells && divide && achieved_time < target)
        const bool spawn = ok && divided && (achieved_cell_time + creation < a.end_time);
        int fl = (ok ? 1 : 0) | (divided ? 2 : 0) | (died ? 4 : 0) | ((ev[3] == ev[3]) ? 8 : 0) | (spawn ? 16 : 0);
#if CP_STORED
        if (overflow) fl |= 32;  // more steps than the store holds (cellpop_launch reports it)
#endif
        a.flags[slot] = fl;
        for (int k = 0; k < 5; k++) a.event_times[(size_t)slot * 5 + k] = ev[k];
        a.nsteps[slot] = nst;
    }
}
}  // namespace cpk

#if !CP_QUEUE
// the cells of one generation launch, four per wavefront (one per 16-lane row)
extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(CP_WAVES_PER_EU))) void cp_solve_kernel(cpk::CpSolveArgs a)
{
    __shared__ cpk::CellShared shs[cpk::CPW];
    const int wi = (int)blockIdx.x * cpk::CPW + cpk::row();
    if (wi >= a.n_work) return;  // the whole row: rows are cells
    cpk::cp_solve_cell(a, shs[cpk::row()], a.work[wi], wi);
}
#endif


#if CP_QUEUE
namespace cpk {
// the queue's counters, flags, items and the end states crossing wavefronts: device-scope relaxed atomics
// (coherent loads and stores across the XCDs' L2s); the order a publication needs is the completion of
// the earlier stores (q_drain) before the flag, and the flag's value before the later loads
template <class T> __device__ __forceinline__ T q_load(const T* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <class T> __device__ __forceinline__ void q_store(T* p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ int q_add(int32_t* p, int v) { return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ bool q_cas(int32_t* p, int expected, int desired)
{
    return __hip_atomic_compare_exchange_strong(p, &expected, desired, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
}
// every memory operation the wavefront issued has completed (and the compiler moves none across)
__device__ __forceinline__ void q_drain()
{
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
}
// a bounded wait: a wavefront that finds nothing ready for q.idle_limit ticks of the constant-rate wall
// clock (60 s: far beyond any cell's solve, which other wavefronts may still be running) gives up with
// the error counter set (a lost item would otherwise keep the persistent grid alive); its polls back
// off from ~0.2 to ~3 us between reads of the shared counters
enum { Q_HEAD = 0, Q_TAIL = 1, Q_OUTSTANDING = 2, Q_ERROR = 3, Q_ROUNDS = 4, Q_ROWS = 5 };
// the kernel arguments re-read where the queue's bookkeeping uses them: without this the compiler keeps
// their fields in SGPRs across the whole persistent loop, and the cell solve's own scalars then spill
// into VGPR lanes inside its Newton loop
template <class T> __device__ __forceinline__ const T& opaque(const T& x)
{
    const T* p = &x;
    asm volatile("" : "+s"(p));
    return *p;
}
}  // namespace cpk

// One persistent launch for all cells of a batch. Queue positions are handed out as tickets (one
// fetch-and-add per wavefront and round, no compare-and-swap retries): each row of a wavefront holds a
// ticket, and a round solves the rows whose ticket's item is ready -- initialised (cp_init_cell: the
// parent's end state, the variabilities), solved, and the daughters of the cells that divide enqueued
// under the failure rules of the generation launches (cellpop_rt.cpp): a failed cell, a daughter
// beyond max_cells or past the Sobol points fails the evaluation, whose cells then enqueue nothing. A
// row whose ticket is not filled yet waits while its sisters' cells run; a ticket past the queue's
// capacity, or one unfilled once no cell is outstanding, ends the row; the wavefront ends with its four
// rows. (No deadlock: a ticket is unfilled only when every reserved item has been handed out, and a row
// holding a filled ticket always runs in its wavefront's next round.) Outputs are indexed by queue
// position; cp_number_kernel and cp_permute_kernel (cellpop_kernels.hip) restore the reference's cell
// numbering.
extern "C" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(CP_WAVES_PER_EU))) void cp_queue_kernel(
    cpk::CpSolveArgs a_, cpk::CpQueueArgs q_, bcm3hip::CpStatic m_)
{
    using namespace cpk;
    enum { NEED = -1, DONE = -2 };
    __shared__ CellShared shs[CPW];
    __shared__ CellIn qin[CPW];
    __shared__ double qpe[CPW][CP_NS];  // the mother's end state and end time
    __shared__ double qach[CPW];
    __shared__ int ticket[CPW];  // the row's queue position, NEED or DONE
    __shared__ int run[CPW];     // the row's item is ready: it runs this round
    __shared__ int ndau[CPW], deval[CPW], dsob[CPW][2];  // the daughters a row's cell enqueues
    __shared__ int isob[CPW];    // the row's cell's Sobol index (nothing of the item stays live in registers
                                 // across the solve)
    __shared__ long idle;        // polls without a ready ticket
    __shared__ unsigned long long idle_t0;  // wall clock at the first of them
    const int r = row(), ln = lane();
    if (threadIdx.x < CPW) ticket[threadIdx.x] = NEED;
    if (threadIdx.x == 0) idle = 0;
    __syncthreads();
    for (;;) {
        if (threadIdx.x == 0) {
            const CpQueueArgs& q = opaque(q_);
            // tickets for the rows that need one, in row order
            int need = 0;
            for (int k = 0; k < CPW; k++) need += ticket[k] == NEED;
            if (need > 0) {
                int t = q_add(q.counters + Q_HEAD, need);
                for (int k = 0; k < CPW; k++)
                    if (ticket[k] == NEED) ticket[k] = (t < q.cap) ? t++ : DONE;
            }
            bool any = false, live = false;
            for (int k = 0; k < CPW; k++) {
                run[k] = ticket[k] >= 0 && q_load(q.ready + ticket[k]) == 1;
                any |= run[k] != 0;
                live |= ticket[k] >= 0;
            }
            if (!any && live) {
                // nothing ready: tickets still unfilled once no cell is outstanding never fill
                if (q_load(q.counters + Q_OUTSTANDING) == 0) {
                    for (int k = 0; k < CPW; k++)
                        if (ticket[k] >= 0 && q_load(q.ready + ticket[k]) != 1) ticket[k] = DONE;
                    for (int k = 0; k < CPW; k++) run[k] = ticket[k] >= 0;  // (filled meanwhile)
                } else {
                    const unsigned long long now = wall_clock64();
                    if (idle++ == 0) idle_t0 = now;
                    if (now - idle_t0 > (unsigned long long)q.idle_limit) {
                        q_add(q.counters + Q_ERROR, 1);
                        for (int k = 0; k < CPW; k++) ticket[k] = DONE;
                    } else if (idle < 64) {
                        __builtin_amdgcn_s_sleep(8);
                    } else {
                        __builtin_amdgcn_s_sleep(127);
                    }
                }
            }
            if (any) {
                idle = 0;
                // statistics: rounds that solve, cells solved (BCM3_CP_QUEUE_VERBOSE prints them)
                int rows = 0;
                for (int k = 0; k < CPW; k++) rows += run[k] != 0;
                q_add(q.counters + Q_ROUNDS, 1);
                q_add(q.counters + Q_ROWS, rows);
            }
        }
        __syncthreads();
        bool all_done = true;
        for (int k = 0; k < CPW; k++) all_done &= ticket[k] == DONE;
        if (all_done) return;
        const bool mine = run[r] != 0;
        const int qi = ticket[r];
        __syncthreads();
        if (mine && ln == 0) {
            CpQueueItem it{};
            const CpQueueArgs& q = opaque(q_);
            const CpSolveArgs& a = opaque(a_);
            const bcm3hip::CpStatic& m = opaque(m_);
            __atomic_signal_fence(__ATOMIC_SEQ_CST);  // the item after its flag
            CpQueueItem* src = q.items + qi;
            it.eval = q_load(&src->eval);
            it.parent = q_load(&src->parent);
            it.sobol_ix = q_load(&src->sobol_ix);
            it.is_initial = q_load(&src->is_initial);
            if (it.parent >= 0) {
                for (int i = 0; i < CP_NS; i++) qpe[r][i] = q_load(a.end_y + (size_t)it.parent * CP_NS + i);
                qach[r] = q_load(a.achieved + it.parent);
            }
            // the cell's inputs into this row's LDS (parameters: the solve's own sh.prm)
            const bcm3hip::CpInitItem ii{0, it.eval, it.parent >= 0 ? 0 : -1, it.sobol_ix, it.is_initial};
            bcm3hip::cp_init_cell(m, ii, q.values, shs[r].prm, qin[r].y0, &qin[r].creation, qpe[r], qach + r, nullptr);
            q.creation[qi] = qin[r].creation;  // (the numbering's copy, after the launch)
            deval[r] = it.eval;
            isob[r] = it.sobol_ix;
        }
        __syncthreads();
        if (mine) cp_solve_cell(a_, shs[r], qi, 0, qin + r);
        // the cells' end states (the daughters' inputs, every lane's stores) before their items are published
        q_drain();
        if (run[r] && ln == 0) {  // (re-read from LDS: nothing of the round stays live across the solve)
            const CpQueueArgs& q = opaque(q_);
            const CpSolveArgs& a = opaque(a_);
            const int e = deval[r];
            const int f = a.flags[ticket[r]];
            int nd = 0;
            if (q_load(q.failed_eval + e) == 0) {
                if (!(f & 1)) {
                    q_store(q.failed_eval + e, 1);
                } else if (f & 16) {
                    for (int child = 0; child < 2; child++) {
                        const int sidx = q.n0 + isob[r] * 2 + child;
                        if (q.sobol_dims > 0 && sidx >= q.sobol_points) {
                            q_store(q.failed_eval + e, 1);
                            break;
                        }
                        if (q_add(q.ncells_eval + e, 1) >= q.max_cells) {
                            q_store(q.failed_eval + e, 1);
                            break;
                        }
                        dsob[r][nd++] = sidx;
                    }
                }
            }
            ndau[r] = nd;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            const CpQueueArgs& q = opaque(q_);
            // the wavefront's daughters enqueued together, in row order (sisters side by side, the
            // daughters of neighbouring cells next to each other, as the generation launches order them)
            int total = 0, ran = 0;
            for (int k = 0; k < CPW; k++)
                if (run[k]) {
                    total += ndau[k];
                    ran++;
                }
            if (total > 0) {
                // outstanding first: the launch cannot drain while these cells (still outstanding) add
                q_add(q.counters + Q_OUTSTANDING, total);
                int t = q_add(q.counters + Q_TAIL, total);
                const int t0 = t;
                for (int k = 0; k < CPW; k++) {
                    if (!run[k]) continue;
                    for (int j = 0; j < ndau[k]; j++, t++) {
                        CpQueueItem* dst = q.items + t;
                        q_store(&dst->slot, t);
                        q_store(&dst->eval, deval[k]);
                        q_store(&dst->parent, ticket[k]);
                        q_store(&dst->sobol_ix, dsob[k][j]);
                        q_store(&dst->is_initial, 0);
                        q.child_qi[2 * ticket[k] + j] = t;
                    }
                }
                q_drain();  // the items before their flags
                for (int k = t0; k < t; k++) q_store(q.ready + k, 1);
            }
            if (ran > 0) {
                q_drain();
                q_add(q.counters + Q_OUTSTANDING, -ran);
            }
            for (int k = 0; k < CPW; k++)
                if (run[k]) ticket[k] = NEED;
        }
        __syncthreads();
    }
}
#endif
