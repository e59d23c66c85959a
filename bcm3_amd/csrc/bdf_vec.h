// bdf_vec.h -- the one-trajectory-per-wavefront BDF step (bdf_uni.h) with the solver's state
// VECTORS spread across lanes: lane i holds component i of zn[0..5], ewt, acor (lanes >= NS
// carry don't-care values). Every component-wise operation of the step -- predict, rescale,
// the Nordsieck update, the Newton residual / update, the error weights -- is then ONE VALU
// instruction instead of NS; the scalars of the step (tn, h, l, tq, gamma, eta, counters) stay
// wave-uniform exactly as in bdf_uni.h and share its code (set_bdf_q, eta_candidate).
//
// Cross-lane work is the right-hand side and the solve of the linear PK systems and the norms:
//   * the right-hand side is the model's (PKLane::rhs_v: each lane evaluates its component's
//     own expression of the reference, the operands moved in by DPP); the solve A^-1 b has
//     column j of the inverse in the lanes (lane i: inv(i, j)) and b_j broadcast to every lane
//     with one DPP row_newbcast move, summed as Eigen's p0 + (p1 + p2) (solvevec): the same
//     products and order as the scalar model (PKLane::rhs / lin_solve), so the bits agree;
//   * weighted RMS norms: squares in lanes, the sum ((p0^2 + p1^2) + p2^2) from broadcasts in
//     component order, made wave-uniform with readfirstlane (wrms of bdf_lane.h sums the same
//     rounded squares in the same order).
// Results are bit-identical to bdf_uni.h and bdf_lane.h (tests/test_popk_gpu.py runs all three).
#pragma once
#include "bdf_uni.h"

namespace bcm3hip {
namespace vec {

BDF_INL int lane_id() { return (int)(threadIdx.x & 63); }

// value of lane J of this 16-lane row in every lane (v_mov_b64_dpp row_newbcast:J). Every lane
// is written (full row and bank masks), so the mov form needs no tied "old" operand -- no copy
// of the source before each broadcast
template <int J>
BDF_INL double bc(double v)
{
    return __builtin_amdgcn_mov_dpp(v, 0x150 + J, 0xf, 0xf, false);
}

// component k (lane k) as a uniform value
BDF_INL double comp(double v, int k)
{
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = __builtin_amdgcn_readlane((int)b, k);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// lane vector from NS uniform values (lane i <- a[i]; lanes >= NS get a[NS-1])
template <int NS>
BDF_INL double from_array(const double (&a)[NS])
{
    const int ln = lane_id();
    double r = a[NS - 1];
    cfor_down<NS - 2, 0>([&](auto i) __attribute__((always_inline)) { r = (ln == CI(i)) ? a[CI(i)] : r; });
    return r;
}
template <int NS>
BDF_INL void to_array(double v, double (&a)[NS])
{
    cfor<0, NS>([&](auto i) __attribute__((always_inline)) { a[CI(i)] = comp(v, CI(i)); });
}

// sum over the components in component order ((c0 + c1) + c2), in every lane of row 0
template <int NS>
BDF_INL double lane_sum_v(double p)
{
    double s = bc<0>(p) + bc<1>(p);
    if constexpr (NS == 3) s = s + bc<2>(p);
    return s;
}
// ... made uniform
template <int NS>
BDF_INL double lane_sum(double p)
{
    return wave_uniform(lane_sum_v<NS>(p));
}

// N_VWrmsNorm (wrms of bdf_lane.h); the quotient and square root run on the lane value and only
// the norm is made uniform (a uniform operand pair would need a copy back into VGPRs first)
template <int NS>
BDF_INL double wrms(double x, double w)
{
    const double p = x * w;
    return wave_uniform(fsqrt(fdiv_c(vec::lane_sum_v<NS>(p * p), (double)NS, 1.0 / NS)));
}

// x = A^-1 b for the inverse held as lane columns, in PKLane::lin_solve's order: c0 b0 + c1 b1
// (N = 2, sunlinsol_dense_eigen.cpp:157-167) and c0 b0 + (c1 b1 + c2 b2) (N = 3, Eigen's unrolled
// p0 + (p1 + p2), :169-176)
template <int NS>
BDF_INL double solvevec(const double (&col)[NS], double x)
{
    if constexpr (NS == 3)
        return col[0] * bc<0>(x) + (col[1] * bc<1>(x) + col[2] * bc<2>(x));
    else
        return col[0] * bc<0>(x) + col[1] * bc<1>(x);
}

// cost-probe builds (BCM3_DBL, bdf_lane.h): launder the operands of a component's second run
template <class S>
BDF_INL void dbl_launder_state(S& s)
{
    cfor<0, QMAX + 1>([&](auto j) __attribute__((always_inline)) { s.zn[CI(j)] = bdf_launder(s.zn[CI(j)]); });
    cfor<0, QMAX + 2>([&](auto j) __attribute__((always_inline)) { s.tau[CI(j)] = bdf_launder(s.tau[CI(j)]); });
    cfor<0, 6>([&](auto j) __attribute__((always_inline)) { s.tq[CI(j)] = bdf_launder(s.tq[CI(j)]); });
    s.ewt = bdf_launder(s.ewt);
    s.acor = bdf_launder(s.acor);
    s.h = bdf_launder(s.h);
    s.tn = bdf_launder(s.tn);
    s.gamma = bdf_launder(s.gamma);
    s.gammap = bdf_launder(s.gammap);
    s.saved_tq5 = bdf_launder(s.saved_tq5);
    s.unity = bdf_launder(s.unity);
}

// per-trajectory solver statistics only when the caller asked for them: without, the counters
// compile to nothing (they would hold 8 SGPRs and a scalar add per event on the hot path)
struct NoCount {
    BDF_INL NoCount operator++(int) { return *this; }
    BDF_INL NoCount& operator+=(int) { return *this; }
    BDF_INL operator int() const { return 0; }
};
struct NoCounters {
    NoCount nst_total, nfe, nni, nsetups, nje, netf, ncfn, nreinit;
};

template <int NS, bool STATS = true>
struct VecState {
    double rtol, atol;
    double unity;  // 1.0 the compiler cannot see (see set_bdf_q)
    double zn[QMAX + 1];  // lane i: component i
    double ewt, acor;
    double acol[4];   // per-lane coefficients of the right-hand side (PKLane::rhs_columns;
                      // constant between ReInits)
    double icol[NS];  // columns of (I - gamma J)^-1 (lin_setup)
    double tau[QMAX + 2], tq[6], l[QMAX + 1];
    double tn, h, hprime, eta, hscale, hu, tretlast;
    double gamma, gammap, gamrat, crate, delp, acnrm, etamax, saved_tq5;
    double tstop;
    int tstopset;
    int q, qprime, qwait, L;
    int nst, nstlp, nstlj;
    int nls_jcur;
    int check_tolsf;
    std::conditional_t<STATS, BdfCounters, NoCounters> cnt;
#ifdef BCM3_PHASES
    unsigned ph[NPHASES];
    unsigned tlast;
    int qh[QMAX + 1];
#endif
};

template <class S>
BDF_INL void ewt_set(S& s)
{
    if constexpr (BDF_DBL(7)) bdf_consume(frcp(s.rtol * fabs(bdf_launder(s.zn[0])) + s.atol));
    s.ewt = frcp(s.rtol * fabs(s.zn[0]) + s.atol);
}

template <int Q, class S>
BDF_INL void rescale_q(S& s, double eta)
{
    double c = eta;
    cfor<1, Q + 1>([&](auto j) __attribute__((always_inline)) {
        s.zn[CI(j)] *= c;
        c = eta * c;
    });
    s.h = s.hscale * eta;
    s.hscale = s.h;
}

template <int Q, class S>
BDF_INL void predict_q(S& s)
{
    s.tn += s.h;
    const double tc = s.tstop;
    s.tn = ((s.tstopset != 0) & ((s.tn - tc) * s.h > 0.0)) ? tc : s.tn;
    cfor<1, Q + 1>([&](auto k) __attribute__((always_inline)) {
        cfor_down<Q, CI(k)>([&](auto j) __attribute__((always_inline)) { s.zn[CI(j) - 1] += s.zn[CI(j)]; });
    });
}

template <int Q, class S>
BDF_INL void restore_q(S& s, double saved_t)
{
    s.tn = saved_t;
    cfor<1, Q + 1>([&](auto k) __attribute__((always_inline)) {
        cfor_down<Q, CI(k)>([&](auto j) __attribute__((always_inline)) { s.zn[CI(j) - 1] -= s.zn[CI(j)]; });
    });
}

// cvIncreaseBDF / cvDecreaseBDF / cvAdjustOrder (bdf_lane.h increase_bdf, decrease_bdf)
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
            cfor_down<CI(j) + 2, 2>([&](auto i) __attribute__((always_inline)) { l[CI(i)] = l[CI(i)] * xiold + l[CI(i) - 1]; });
            xiold = xi;
        }
    });
    A1 = fdiv(-alpha0 - alpha1, prod);
    const double znL = A1 * s.zn[QMAX];
    cfor<2, QMAX + 1>([&](auto j) __attribute__((always_inline)) {
        if (CI(j) == s.q + 1)
            s.zn[CI(j)] = znL;
        else if (CI(j) <= s.q)
            s.zn[CI(j)] = s.zn[CI(j)] + l[CI(j)] * znL;
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
            cfor_down<CI(j) + 2, 2>([&](auto i) __attribute__((always_inline)) { l[CI(i)] = l[CI(i)] * xi + l[CI(i) - 1]; });
        }
    });
    // zn[q] by a select chain starting from a constant (see sel in bdf_lane.h)
    double znq = 0.0;
    cfor<1, QMAX + 1>([&](auto j) __attribute__((always_inline)) { znq = (s.q == CI(j)) ? s.zn[CI(j)] : znq; });
    cfor<2, QMAX>([&](auto j) __attribute__((always_inline)) {
        if (CI(j) < s.q) s.zn[CI(j)] = s.zn[CI(j)] + (-l[CI(j)]) * znq;
    });
    cfor<0, QMAX + 1>([&](auto i) __attribute__((always_inline)) { s.l[CI(i)] = l[CI(i)]; });
}

template <class S>
BDF_INL void adjust_order(S& s, int deltaq)
{
    if ((s.q == 2) && (deltaq != 1)) return;
    if (deltaq == 1)
        vec::increase_bdf(s);
    else if (deltaq == -1)
        vec::decrease_bdf(s);
}

// CVodeGetDky(t, 0) into a lane vector
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
        if (CI(j) == s.q)
            dky = c[CI(j)] * s.zn[CI(j)];
        else if (CI(j) < s.q)
            dky = dky + c[CI(j)] * s.zn[CI(j)];
    });
    return CV_SUCCESS;
}
template <int NS, class S>
BDF_INL int get_dky_array(const S& s, double t, double (&dky)[NS])
{
    double v;
    const int r = vec::get_dky(s, t, v);
    if (r == CV_SUCCESS) vec::to_array<NS>(v, dky);
    return r;
}

// CVodeReInit; also refreshes the RHS matrix columns (the dosing callbacks that precede a ReInit
// may switch the absorption rate)
template <int NS, class S, class Model>
BDF_INL void reinit(S& s, const Model& mdl, double t0, const double (&y0)[NS])
{
    s.tn = t0;
    s.q = 1;
    s.L = 2;
    s.qwait = 2;
    s.etamax = ETAMX1;
    s.hu = 0.0;
    s.zn[0] = vec::from_array<NS>(y0);
    mdl.rhs_columns(s.acol);
    s.nst = 0;
    s.nstlp = 0;
    s.cnt.nreinit++;
}

// cvHin (bdf_lane.h hin)
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
    // cvUpperBoundH0: max over components in component order
    double t1 = frcp(s.ewt);
    t1 = t1 + HUB_FACTOR * fabs(s.zn[0]);
    const double r = fdiv(fabs(s.zn[1]), t1);
    double hub_inv = bc<0>(r);
    cfor<1, NS>([&](auto i) __attribute__((always_inline)) {
        const double ri = bc<CI(i)>(r);
        hub_inv = (ri > hub_inv) ? ri : hub_inv;
    });
    hub_inv = wave_uniform(hub_inv);
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
        const double hgs = hg * sign;
        const double yy = hgs * s.zn[1] + s.zn[0];
        double tv = mdl.rhs_v(s.tn + hgs, yy, s.acol);
        s.cnt.nfe++;
        const double a = frcp(hgs);
        tv = a * (tv - s.zn[1]);
        const double yddnrm = vec::wrms<NS>(tv, s.ewt);
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

// cvSetBDF + cvSetTqBDF + cvSet for order Q (uni::set_bdf_q) without the qwait == 1 block of
// cvSetTqBDF: tq[1] and tq[3] are read only by the order-change candidates, which run in the
// completion of the same step exactly when qwait was 1 here, so tq_13 computes them there from
// the intermediates kept in TqCtx (no per-step branch on qwait in the attempt)
struct TqCtx {
    double alpha0, alpha0_hat, xi_inv, xistar_inv, hsum2, lq, A2;  // hsum2: before complete shifts tau
};

template <int Q, bool NSTPOS = false, class S>
BDF_INL double set_bdf_q(S& s, TqCtx& c)
{
    constexpr int q = Q;
    double alpha0, alpha0_hat, xi_inv, xistar_inv, hsum;
    s.l[0] = s.l[1] = xi_inv = xistar_inv = 1.0;
    cfor<2, Q + 1>([&](auto i) __attribute__((always_inline)) { s.l[CI(i)] = 0.0; });
    alpha0 = alpha0_hat = -1.0;
    hsum = s.h;
    if constexpr (q > 1) {
        cfor<2, Q>([&](auto j) __attribute__((always_inline)) {
            hsum += s.tau[CI(j) - 1];
            xi_inv = fdiv(s.h, hsum);
            alpha0 -= 1.0 / CI(j);
            cfor_down<CI(j), 1>([&](auto i) __attribute__((always_inline)) { s.l[CI(i)] = s.l[CI(i)] + s.l[CI(i) - 1] * xi_inv; });
        });
        alpha0 -= 1.0 / q;
        xistar_inv = -s.l[1] - alpha0;
        hsum += s.tau[q - 1];
        xi_inv = fdiv(s.h, hsum);
        alpha0_hat = -s.l[1] - xi_inv;
        cfor_down<Q, 1>([&](auto i) __attribute__((always_inline)) { s.l[CI(i)] = s.l[CI(i)] + s.l[CI(i) - 1] * xistar_inv; });
    }
    const double A1 = 1.0 - alpha0_hat + alpha0;
    const double A2 = 1.0 + (double)q * A1;
    const double lq = s.l[q];
    s.tq[2] = fabs(fdiv(A1, alpha0 * A2));
    s.tq[5] = fabs(fdiv(A2 * xistar_inv, lq * xi_inv));
    s.tq[4] = fdiv(CORTES, s.tq[2]);
    c.alpha0 = alpha0;
    c.alpha0_hat = alpha0_hat;
    c.xi_inv = xi_inv;
    c.xistar_inv = xistar_inv;
    c.hsum2 = hsum + s.tau[q];
    c.lq = lq;
    c.A2 = A2;
    // at q = 2, l[1] = 1.5 is a compile-time constant here but not in the lane solver (runtime q):
    // the compiler would fold v_rcp_f64(1.5) to the correctly rounded value while the hardware
    // estimate (one Newton step, frcp) differs, so the operand is passed through a runtime 1.0
    const double rl1 = frcp((q == 2) ? s.l[1] * s.unity : s.l[1]);
    s.gamma = s.h * rl1;
    if constexpr (NSTPOS) {
        // fast_run: nst > 0 by its precondition
        s.gamrat = fdiv(s.gamma, s.gammap);
    } else {
        s.gammap = (s.nst == 0) ? s.gamma : s.gammap;
        const double gr = fdiv(s.gamma, s.gammap);
        s.gamrat = (s.nst > 0) ? gr : 1.0;
    }
    return rl1;
}

// the qwait == 1 block of cvSetTqBDF (uni::set_bdf_q), from the same operands
template <int Q, class S>
BDF_INL void tq_13(S& s, const TqCtx& c)
{
    constexpr int q = Q;
    double tq1 = 1.0;
    if constexpr (q > 1) {
        const double C = fdiv(c.xistar_inv, c.lq);
        const double A3 = c.alpha0 + 1.0 / q;
        const double A4 = c.alpha0_hat + c.xi_inv;
        const double Cpinv = fdiv_c(1.0 - A4 + A3, A3, 1.0 / tq_a3(q));
        tq1 = fabs(C * Cpinv);
    }
    const double xi_inv2 = fdiv(s.h, c.hsum2);
    const double A5 = c.alpha0 - 1.0 / (q + 1);
    const double A6 = c.alpha0_hat - xi_inv2;
    const double Cppinv = fdiv(1.0 - A6 + A5, c.A2);
    const double tq3 = fabs(fdiv(Cppinv, xi_inv2 * (double)(q + 2) * A5));
    s.tq[1] = tq1;
    s.tq[3] = tq3;
}

// a / b within 2^-48 relative (v_rcp_f64 and one Newton step): the order-change screen below
BDF_INL double qdiv(double a, double b)
{
    double r = __builtin_amdgcn_rcp(b);
    r = __builtin_fma(__builtin_fma(-b, r, 1.0), r, r);
    return a * r;
}

// Order-change screen (qwait == 0, every other step): an order-change candidate only matters when
// it reaches THRESH, i.e. when its bx is at most eta_cut (which already carries a 1e-9 relative
// margin); below that it acts exactly like eta_candidate's 0 in cvChooseEta. The candidates'
// bx = BIAS (wrms tq) are bounded here from approximate quotients (qdiv, 2^-48) and without the
// square roots (bx^2 from the sum of squares): when both exceed their cut by 1e-10 relative, the
// exact evaluation below would return eta_candidate's 0 for both, and it is skipped (tq[1] and
// tq[3], read only by it, are not needed). The quotients whose operands can cancel keep their
// exact forms (xi_inv2 and 1 - A6 + A5 are computed as tq_13 computes them).
template <int Q, int NS, class S>
BDF_INL bool order_change_skippable(const S& s, const TqCtx& c)
{
    constexpr int q = Q;
    constexpr double margin = 1.0 + 1e-10;
    bool small = true;
    if constexpr (q > 1) {
        const double A3 = c.alpha0 + 1.0 / q;
        const double A4 = c.alpha0_hat + c.xi_inv;
        const double tq1 = fabs(qdiv(c.xistar_inv, c.lq) * ((1.0 - A4 + A3) * (1.0 / tq_a3(q))));
        const double p = s.zn[q] * s.ewt;
        const double b1 = BIAS1 * tq1;
        const double bx2 = wave_uniform(lane_sum_v<NS>(p * p) * (1.0 / NS) * (b1 * b1));
        constexpr double cut = uni::eta_cut(q) * margin;
        small = bx2 > cut * cut;
    }
    if constexpr (q != QMAX) {
        if (small & (s.saved_tq5 != 0.0)) {
            const double cquot = qdiv(s.tq[5], s.saved_tq5) * powI(qdiv(s.h, s.tau[2]), q + 1);
            const double tv = (-cquot) * s.zn[QMAX] + s.acor;
            const double xi_inv2 = fdiv(s.h, c.hsum2);
            const double A5 = c.alpha0 - 1.0 / (q + 1);
            const double A6 = c.alpha0_hat - xi_inv2;
            const double tq3 = fabs(qdiv(qdiv(1.0 - A6 + A5, c.A2), xi_inv2 * (double)(q + 2) * A5));
            const double p = tv * s.ewt;
            const double b3 = BIAS3 * tq3;
            const double bx2 = wave_uniform(lane_sum_v<NS>(p * p) * (1.0 / NS) * (b3 * b3));
            constexpr double cut = uni::eta_cut(q + 2) * margin;
            small = bx2 > cut * cut;
        }
    }
    return small;
}

// The same screen without the quotients of tq[1] and tq[3] (BCM3_SCREEN_DF): bx^2 > cut^2 is decided
// in cross-multiplied form, tq[1]^2 = (xistar_inv (1 - A4 + A3) / A3)^2 / lq^2 and tq[3]^2 =
// (1 - A6 + A5)^2 / (A2 xi_inv2 (q + 2) A5)^2 with both denominators moved to the right-hand side;
// the two candidates' sums of squares are formed side by side and the decision is one branch. Every
// operand is a product of a few rounded factors (relative error << the 1e-10 margin); a NaN or an
// overflow to inf on the right-hand side answers "not skippable", which is always safe (the exact
// evaluation runs). cquot keeps its two approximate quotients (a product of powers could underflow).
template <int Q, int NS, class S>
BDF_INL bool order_change_skippable_df(const S& s, const TqCtx& c)
{
    constexpr int q = Q;
    constexpr double margin = 1.0 + 1e-10;
    bool small1 = true, small3 = true;
    double lhs1 = 0.0, rhs1 = 0.0, lhs3 = 0.0, rhs3 = 0.0;
    if constexpr (q > 1) {
        const double A3 = c.alpha0 + 1.0 / q;
        const double A4 = c.alpha0_hat + c.xi_inv;
        const double n1 = c.xistar_inv * (1.0 - A4 + A3);
        const double p = s.zn[q] * s.ewt;
        constexpr double cut = uni::eta_cut(q) * margin;
        constexpr double k1 = BIAS1 * BIAS1 / (NS * tq_a3(q) * tq_a3(q));
        lhs1 = lane_sum_v<NS>(p * p) * (k1 * (n1 * n1));
        rhs1 = (cut * cut) * (c.lq * c.lq);
    }
    if constexpr (q != QMAX) {
        const double cquot = qdiv(s.tq[5], s.saved_tq5) * powI(qdiv(s.h, s.tau[2]), q + 1);
        const double tv = (-cquot) * s.zn[QMAX] + s.acor;
        const double xi_inv2 = fdiv(s.h, c.hsum2);
        const double A5 = c.alpha0 - 1.0 / (q + 1);
        const double A6 = c.alpha0_hat - xi_inv2;
        const double n3 = 1.0 - A6 + A5;
        const double d3 = c.A2 * xi_inv2 * ((double)(q + 2) * A5);
        const double p = tv * s.ewt;
        constexpr double cut = uni::eta_cut(q + 2) * margin;
        constexpr double k3 = BIAS3 * BIAS3 / NS;
        lhs3 = lane_sum_v<NS>(p * p) * (k3 * (n3 * n3));
        rhs3 = (cut * cut) * (d3 * d3);
    }
    // one uniform decision over both candidates (lanes of row 0 hold the sums)
    if constexpr (q > 1) small1 = lhs1 > rhs1;
    if constexpr (q != QMAX) small3 = (s.saved_tq5 == 0.0) | (lhs3 > rhs3);
    return __builtin_amdgcn_readfirstlane((int)(small1 & small3)) != 0;
}

// one Newton correction (uni::newton_correction)
// (PHB >= 0: the phases build marks the right-hand side, the solve and the norm as PHB, PHB + 1, PHB + 2)
template <int NS, int PHB = -1, class S, class Model>
BDF_INL double newton_correction(S& s, const Model& mdl, double rl1, double& cscale, bool setup, bool jbad,
                                 int convfail)
{
    const double y = s.zn[0] + s.acor;
    const double f = mdl.rhs_v(s.tn, y, s.acol);
    if constexpr (PHB >= 0) BDF_PH(PHB);
    s.cnt.nfe++;
    double delta = rl1 * s.zn[1] + s.acor;
    delta = delta + (-s.gamma) * f;
    if (BDF_UNLIKELY(setup)) {
        if (jbad) convfail = CONV_BAD_J;
        const double dgamma = fabs(fdiv(s.gamma, s.gammap) - 1.0);
        const bool jnew = (s.nst == 0) | (s.nst > s.nstlj + CVLS_MSBJ) |
                          ((convfail == CONV_BAD_J) & (dgamma < CVLS_DGMAX)) | (convfail == CONV_OTHER);
        s.cnt.nje += jnew ? 1 : 0;
        s.nstlj = jnew ? s.nst : s.nstlj;
        if constexpr (BDF_DBL(6)) {
            double ic2[NS];
            mdl.lin_setup_v(bdf_launder(s.gamma), ic2);
            cfor<0, NS>([&](auto k) __attribute__((always_inline)) { bdf_consume(ic2[CI(k)]); });
        }
        mdl.lin_setup_v(s.gamma, s.icol);
        s.cnt.nsetups++;
        s.nls_jcur = jnew;
        s.gamrat = 1.0;
        cscale = 1.0;
        s.gammap = s.gamma;
        s.crate = 1.0;
        s.nstlp = s.nst;
    }
    s.cnt.nni++;
    double x = vec::solvevec<NS>(s.icol, -delta);
    x *= cscale;
    s.acor += x;
    if constexpr (PHB >= 0) BDF_PH(PHB + 1);
    const double del = vec::wrms<NS>(x, s.ewt);
    if constexpr (PHB >= 0) BDF_PH(PHB + 2);
    return del;
}

// Newton iteration (uni::newton_u) after its first correction del (made by attempt_q)
template <int NS, class S, class Model>
BDF_INL bool newton_rest(S& s, const Model& mdl, double rl1, int convfail, bool callSetup, double cscale, double del)
{
    bool jbad = false;
    for (bool first = true;; first = false) {
        if (!first) del = vec::newton_correction<NS>(s, mdl, rl1, cscale, callSetup, jbad, convfail);
        if (div_le_one(del * SUNMIN(1.0, s.crate), s.tq[4])) {
            s.acnrm = del;
            s.nls_jcur = 0;
            return true;
        }
        s.delp = del;
        for (int it = 1; it < NLS_MAXCOR; it++) {
            del = vec::newton_correction<NS>(s, mdl, rl1, cscale, false, false, convfail);
            s.crate = SUNMAX(CRDOWN * s.crate, fdiv(del, s.delp));
            if (div_le_one(del * SUNMIN(1.0, s.crate), s.tq[4])) {
                s.acnrm = vec::wrms<NS>(s.acor, s.ewt);
                s.nls_jcur = 0;
                return true;
            }
            if (del > RDIV * s.delp) break;
            s.delp = del;
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

// One attempt at order Q (uni::attempt_q). The usual outcome -- Newton converges on its first
// correction and the error test passes -- is decided by ONE branch on both tests (the local
// error dsm = acnrm tq[2] of a first-iteration convergence is del tq[2]); anything else goes on
// through newton_rest, which repeats the convergence test on the same del.
template <int Q, int NS, bool NSTPOS = false, class S, class Model>
BDF_INL int attempt_q(S& s, const Model& mdl, double eta_eff, double saved_t, int nflag, double& dsm, TqCtx& tc)
{
    if (BDF_UNLIKELY(eta_eff != 1.0)) vec::rescale_q<Q>(s, eta_eff);
    BDF_PH(2);
    vec::predict_q<Q>(s);
    BDF_PH(3);
    const double rl1 = vec::set_bdf_q<Q, NSTPOS>(s, tc);
    BDF_PH(4);
    const int convfail = ((nflag == FIRST_CALL) | (nflag == PREV_ERR_FAIL)) ? CONV_NONE : CONV_OTHER;
    const bool callSetup = (nflag == PREV_CONV_FAIL) | (nflag == PREV_ERR_FAIL) | (s.nst == 0) |
                           (s.nst >= s.nstlp + MSBP) | (fabs(s.gamrat - 1.0) > DGMAX);
    s.acor = 0.0;
    double cscale = (s.gamrat != 1.0) ? fdiv(2.0, 1.0 + s.gamrat) : 1.0;
    const double del = vec::newton_correction<NS>(s, mdl, rl1, cscale, callSetup, false, convfail);
    const double dsm1 = del * s.tq[2];
    if (BDF_LIKELY(div_le_one(del * SUNMIN(1.0, s.crate), s.tq[4]) & (dsm1 <= 1.0))) {
        s.acnrm = del;
        s.nls_jcur = 0;
        dsm = dsm1;
        BDF_PH(5);
        return uni::ATTEMPT_OK;
    }
    const bool conv = vec::newton_rest<NS>(s, mdl, rl1, convfail, callSetup, cscale, del);
    BDF_PH(5);
    dsm = s.acnrm * s.tq[2];
    if (BDF_LIKELY(conv & (dsm <= 1.0))) return uni::ATTEMPT_OK;
    vec::restore_q<Q>(s, saved_t);
    return conv ? uni::ATTEMPT_ERR_FAIL : uni::ATTEMPT_CONV_FAIL;
}

// cvSet's coefficients (l, tq[2], tq[5], the tq[1]/tq[3] intermediates, gamma, gamrat) depend on
// h, tau[1..Q] and gammap only. After Q completed steps at an unchanged h, tau[1..Q] all equal h, so
// every later step at that h with no linear-solver setup in between recomputes exactly the values
// it already holds (52 % of the steps on C3 prior draws, measured in the oracle): fast_run keeps
// them instead -- the same bits as computing them again (see fast_run).

// FAST: called from fast_run, where the step's first attempt passed, so etamax is the value the
// previous completion set (ETAMX2 / ETAMX3) or ReInit's ETAMX1 -- never 1
// cvCompleteStep (complete_head_q) + cvPrepareNextStep (complete_eta_q)
// HELD: fast_run's plain step, where tau[1..Q] all equal h (the coefficients are held), so the
// shift of tau[1..Q] would store the values they have
template <int Q, int PH = 7, bool HELD = false, class S>
BDF_INL void complete_head_q(S& s)
{
    constexpr int q = Q;
    s.nst++;
    s.cnt.nst_total++;
    s.hu = s.h;
    if constexpr (!HELD) {
        cfor_down<Q, 2>([&](auto i) __attribute__((always_inline)) { s.tau[CI(i)] = s.tau[CI(i) - 1]; });
        if constexpr (q == 1) s.tau[2] = (s.nst > 1) ? s.tau[1] : s.tau[2];
        s.tau[1] = s.h;
    }
    cfor<0, Q + 1>([&](auto j) __attribute__((always_inline)) { s.zn[CI(j)] = s.zn[CI(j)] + s.l[CI(j)] * s.acor; });
    s.qwait--;
    if constexpr (q != QMAX) {
        // qwait is a scalar counter: a scalar branch instead of four VALU selects every step
        if (s.qwait == 1) {
            s.zn[QMAX] = s.acor;
            s.saved_tq5 = s.tq[5];
        }
    }
    BDF_PH(PH);
}

// complete_head_q with the plain-step flag at run time (BCM3_ONE_TAIL: one tail per order)
template <int Q, class S>
BDF_INL void complete_head_q_rt(S& s, bool held)
{
    constexpr int q = Q;
    s.nst++;
    s.cnt.nst_total++;
    s.hu = s.h;
    if (!held) {
        cfor_down<Q, 2>([&](auto i) __attribute__((always_inline)) { s.tau[CI(i)] = s.tau[CI(i) - 1]; });
        if constexpr (q == 1) s.tau[2] = (s.nst > 1) ? s.tau[1] : s.tau[2];
        s.tau[1] = s.h;
    }
    cfor<0, Q + 1>([&](auto j) __attribute__((always_inline)) { s.zn[CI(j)] = s.zn[CI(j)] + s.l[CI(j)] * s.acor; });
    s.qwait--;
    if constexpr (q != QMAX) {
        if (s.qwait == 1) {
            s.zn[QMAX] = s.acor;
            s.saved_tq5 = s.tq[5];
        }
    }
}

template <int Q, int NS, bool FAST, int PH = 8, class S>
BDF_INL void complete_eta_q(S& s, double dsm, const TqCtx& tc)
{
    constexpr int q = Q;
    const double bx = BIAS2 * dsm;
    if (BDF_LIKELY(FAST && (s.qwait != 0) & (bx > uni::eta_cut(q + 1)))) {
        // the usual outcome: no order-change check due and etaq below THRESH (eta_candidate's 0):
        // cvSetEta keeps h (eta = 1)
        s.qprime = q;
        s.eta = 1.0;
        s.hprime = s.h;
    } else if (BDF_UNLIKELY(!FAST && (s.etamax == 1.0))) {
        s.qwait = SUNMAX(s.qwait, 2);
        s.qprime = q;
        s.hprime = s.h;
        s.eta = 1.0;
    } else {
        const double etaq = uni::eta_candidate<q + 1>(bx);
        BDF_PH_CNT(27, !(bx > uni::eta_cut(q + 1)));
        double eta = etaq;
        s.qprime = q;
        const unsigned ph_s0 = BDF_PH_NOW();
#ifdef BCM3_SCREEN_DF
        const bool skip = (s.qwait == 0) && vec::order_change_skippable_df<q, NS>(s, tc);
#else
        const bool skip = (s.qwait == 0) && vec::order_change_skippable<q, NS>(s, tc);
#endif
        if constexpr (BDF_DBL(2)) {
            if (s.qwait == 0) {
                S s2 = s;
                vec::dbl_launder_state(s2);
                TqCtx tc2 = tc;
                tc2.alpha0 = bdf_launder(tc2.alpha0);
                tc2.alpha0_hat = bdf_launder(tc2.alpha0_hat);
                tc2.xi_inv = bdf_launder(tc2.xi_inv);
                tc2.xistar_inv = bdf_launder(tc2.xistar_inv);
                tc2.hsum2 = bdf_launder(tc2.hsum2);
                tc2.lq = bdf_launder(tc2.lq);
                tc2.A2 = bdf_launder(tc2.A2);
                bdf_consume(vec::order_change_skippable<q, NS>(s2, tc2) ? 1.0 : 0.0);
            }
        }
        if (s.qwait == 0) {
            BDF_PH_ADD(30, ph_s0);
            BDF_PH_CNT(28, true);
            BDF_PH_CNT(29, skip);
        }
        const unsigned ph_e0 = BDF_PH_NOW();
        if ((s.qwait == 0) && !skip) {
            if constexpr (BDF_DBL(3)) {
                S s2 = s;
                vec::dbl_launder_state(s2);
                vec::tq_13<q>(s2, tc);
                double e1 = 0.0, e3 = 0.0;
                if constexpr (q > 1) e1 = uni::eta_candidate<q>(BIAS1 * (vec::wrms<NS>(s2.zn[q], s2.ewt) * s2.tq[1]));
                if constexpr (q != QMAX) {
                    if (s2.saved_tq5 != 0.0) {
                        const double cq = fdiv(s2.tq[5], s2.saved_tq5) * powI(fdiv(s2.h, s2.tau[2]), q + 1);
                        const double tv = (-cq) * s2.zn[QMAX] + s2.acor;
                        e3 = uni::eta_candidate<q + 2>(BIAS3 * (vec::wrms<NS>(tv, s2.ewt) * s2.tq[3]));
                    }
                }
                bdf_consume(e1);
                bdf_consume(e3);
            }
            s.qwait = 2;
            vec::tq_13<q>(s, tc);  // qwait was 1 in this step's set_bdf_q
            double etaqm1 = 0.0, etaqp1 = 0.0;
            if constexpr (q > 1) etaqm1 = uni::eta_candidate<q>(BIAS1 * (vec::wrms<NS>(s.zn[q], s.ewt) * s.tq[1]));
            if constexpr (q != QMAX) {
                if (s.saved_tq5 != 0.0) {
                    const double cquot = fdiv(s.tq[5], s.saved_tq5) * powI(fdiv(s.h, s.tau[2]), q + 1);
                    const double tv = (-cquot) * s.zn[QMAX] + s.acor;
                    etaqp1 = uni::eta_candidate<q + 2>(BIAS3 * (vec::wrms<NS>(tv, s.ewt) * s.tq[3]));
                }
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
            BDF_PH_ADD(31, ph_e0);
        } else if (s.qwait == 0) {
            // both order-change candidates screened below THRESH: cvChooseEta keeps q, eta = etaq
            s.qwait = 2;
        }
        const bool small = (eta < THRESH);
        s.eta = small ? 1.0 : SUNMIN(eta, s.etamax);
        s.hprime = small ? s.h : s.h * s.eta;
    }
    BDF_PH(PH);
    s.etamax = (s.nst <= SMALL_NST) ? ETAMX2 : ETAMX3;
    s.acor *= s.tq[2];
}

template <int Q, int NS, bool FAST, int PH0 = 7, bool HELD = false, class S>
BDF_INL void complete_q(S& s, double dsm, const TqCtx& tc)
{
    vec::complete_head_q<Q, PH0, HELD>(s);
    vec::complete_eta_q<Q, NS, FAST, PH0 + 1>(s, dsm, tc);
}

template <int Q, int NS, bool FAST = false, class S, class Model>
BDF_INL int step_q(S& s, const Model& mdl, double eta_eff, double saved_t, int nflag, double& dsm)
{
    TqCtx tc;
    const int r = vec::attempt_q<Q, NS>(s, mdl, eta_eff, saved_t, nflag, dsm, tc);
    if (BDF_LIKELY(r == uni::ATTEMPT_OK)) vec::complete_q<Q, NS, FAST>(s, dsm, tc);
#ifdef BCM3_PHASES
    if (r == uni::ATTEMPT_OK) s.qh[Q]++;
#endif
    return r;
}

// The attempt loop of cvStep (cvode.c:2082-2174) from a given first attempt result onward:
// r == PENDING runs the attempt at the current order, otherwise r / dsm are the outcome of the
// first attempt (made by fast_run). Then the end of CVode's ONE_STEP return (tstop handling).
constexpr int ATTEMPT_PENDING = -1;

// end of CVode after a successful step (cvode.c:1249-1270): tstop reached / clamp the next h
template <int NS, class S>
BDF_INL int finish_step(S& s, double (&yout)[NS], double& tret)
{
    const double troundoff = FUZZ_FACTOR * UROUND * (fabs(s.tn) + fabs(s.h));
    const bool reached = fabs(s.tn - s.tstop) <= troundoff;
    if (BDF_UNLIKELY((s.tstopset != 0) & (reached | ((s.tn + s.hprime - s.tstop) * s.h > 0.0)))) {
        if (reached) {
            double v;
            vec::get_dky(s, s.tstop, v);
            vec::to_array<NS>(v, yout);
            s.tretlast = tret = s.tstop;
            s.tstopset = 0;
            BDF_PH(9);
            return CV_TSTOP_RETURN;
        }
        s.hprime = (s.tstop - s.tn) * (1.0 - 4.0 * UROUND);
        s.eta = fdiv(s.hprime, s.h);
    }
    s.tretlast = tret = s.tn;
    BDF_PH(9);
    return CV_SUCCESS;
}

template <int NS, class S, class Model>
BDF_INL int attempt_loop(S& s, const Model& mdl, double (&yout)[NS], double& tret, double saved_t, double eta_eff,
                         int r, double dsm)
{
    int ncf = 0, nef = 0, nflag = FIRST_CALL;
    for (;;) {
        if (r == ATTEMPT_PENDING) {
            switch (s.q) {
            case 1: r = vec::step_q<1, NS>(s, mdl, eta_eff, saved_t, nflag, dsm); break;
            case 2: r = vec::step_q<2, NS>(s, mdl, eta_eff, saved_t, nflag, dsm); break;
            case 3: r = vec::step_q<3, NS>(s, mdl, eta_eff, saved_t, nflag, dsm); break;
            case 4: r = vec::step_q<4, NS>(s, mdl, eta_eff, saved_t, nflag, dsm); break;
            default: r = vec::step_q<5, NS>(s, mdl, eta_eff, saved_t, nflag, dsm); break;
            }
        }
        BDF_PH(6);
        if (BDF_LIKELY(r == uni::ATTEMPT_OK)) break;
        const int failed = r;
        r = ATTEMPT_PENDING;
        eta_eff = 1.0;
        s.etamax = 1.0;
        if (failed == uni::ATTEMPT_CONV_FAIL) {
            s.cnt.ncfn++;
            ncf++;
            if (ncf == MXNCF) return CV_CONV_FAILURE;
            s.eta = ETACF;
            nflag = PREV_CONV_FAIL;
            eta_eff = s.eta;
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
            eta_eff = s.eta;
            continue;
        }
        s.eta = ETAMIN;
        if (s.q > 1) {
            vec::adjust_order(s, -1);
            s.L = s.q;
            s.q--;
            s.qwait = s.L;
            eta_eff = s.eta;
            continue;
        }
        s.h *= s.eta;
        s.hscale = s.h;
        s.qwait = LONG_WAIT;
        const double tv = mdl.rhs_v(s.tn, s.zn[0], s.acol);
        s.cnt.nfe++;
        s.zn[1] = s.h * tv;
        eta_eff = 1.0;
    }
    return vec::finish_step<NS>(s, yout, tret);
}

// The step is split so that the attempt loop (5 order-specialised steps) is instantiated once in
// the driver: cvode_entry and fast_run either finish the CVode call themselves or return
// NEED_ATTEMPTS with the arguments of attempt_loop in a Pending record.
constexpr int NEED_ATTEMPTS = 1000;
struct Pending {
    double saved_t, eta_eff, dsm;
    int r;
};

// CVode(..., CV_ONE_STEP) up to the attempt loop, same contract as uni::cvode_one_step_u
// (yout: uniform components); cvode_entry + attempt_loop == one CVode call
template <int NS, class S, class Model>
BDF_INL int cvode_entry(S& s, const Model& mdl, double tout, double (&yout)[NS], double& tret, bool hot, Pending& pd)
{
    BDF_PH(0);
    {
        bool rare_entry = false, first = false, ret_prev = false, at_stop = false;
        if (BDF_UNLIKELY(!hot)) {
            const double troundoff = FUZZ_FACTOR * UROUND * (fabs(s.tn) + fabs(s.h));
            first = (s.nst == 0);
            ret_prev = fabs(s.tn - s.tretlast) > troundoff;
            at_stop = (s.tstopset != 0) & (fabs(s.tn - s.tstop) <= troundoff);
            const bool clamp = (s.tstopset != 0) & ((s.tn + s.hprime - s.tstop) * s.h > 0.0);
            rare_entry = first | ret_prev | at_stop | clamp;
        }
        if (BDF_UNLIKELY(rare_entry)) {
            if (first) {
                s.tretlast = tret = s.tn;
                vec::ewt_set(s);
                s.nstlj = 0;
                s.nls_jcur = 0;
                s.zn[1] = mdl.rhs_v(s.tn, s.zn[0], s.acol);
                s.cnt.nfe++;
                if (s.tstopset) {
                    if ((s.tstop - s.tn) * (tout - s.tn) <= 0.0) return CV_ILL_INPUT;
                }
                double tout_hin = tout;
                if (s.tstopset && (tout - s.tn) * (tout - s.tstop) > 0.0) tout_hin = s.tstop;
                const int hflag = vec::hin<NS>(s, mdl, tout_hin);
                if (hflag != CV_SUCCESS) return hflag;
                if (s.tstopset) {
                    if ((s.tn + s.h - s.tstop) * s.h > 0.0) s.h = (s.tstop - s.tn) * (1.0 - 4.0 * UROUND);
                }
                s.hscale = s.h;
                s.hprime = s.h;
                s.zn[1] *= s.h;
            } else {
                if (ret_prev) {
                    s.tretlast = tret = s.tn;
                    vec::to_array<NS>(s.zn[0], yout);
                    return CV_SUCCESS;
                }
                if (at_stop) {
                    double v;
                    if (vec::get_dky(s, s.tstop, v) != CV_SUCCESS) return CV_ILL_INPUT;
                    vec::to_array<NS>(v, yout);
                    s.tretlast = tret = s.tstop;
                    s.tstopset = 0;
                    return CV_TSTOP_RETURN;
                }
                s.hprime = (s.tstop - s.tn) * (1.0 - 4.0 * UROUND);
                s.eta = fdiv(s.hprime, s.h);
                vec::ewt_set(s);
            }
        } else {
            vec::ewt_set(s);
        }
    }
    if (BDF_UNLIKELY(s.check_tolsf)) {
        const double p = s.zn[0] * s.ewt;
        const double ss = vec::lane_sum<NS>(p * p);
        if (ss > (double)NS * (1.0 / (UROUND * UROUND))) {
            s.tretlast = tret = s.tn;
            vec::to_array<NS>(s.zn[0], yout);
            return CV_TOO_MUCH_ACC;
        }
    }
    BDF_PH(1);

    pd.saved_t = s.tn;
    const bool adj = (s.nst > 0) & (s.hprime != s.h);
    pd.eta_eff = adj ? s.eta : 1.0;
    if (BDF_UNLIKELY(adj & (s.qprime != s.q))) {
        vec::adjust_order(s, s.qprime - s.q);
        s.q = s.qprime;
        s.L = s.q + 1;
        s.qwait = s.L;
    }
    pd.r = ATTEMPT_PENDING;
    pd.dsm = 0.0;
    return NEED_ATTEMPTS;
}

// Consecutive plain steps at order Q, as the driver would run them one cvode_one_step(hot) call
// at a time, with the per-step bookkeeping of the general path folded into ONE exit test:
// a step stays in the loop only when the general path would have (1) found no tstop event in
// finish_step (tstop neither reached nor within the next step), (2) handed the driver a
// CV_SUCCESS that triggers nothing there (no output time or end time passed, step budget not
// exhausted, no discontinuity at t), and (3) next entered cvode_one_step hot with no order change
// pending. Preconditions (checked by the caller): the last step was such a hot CV_SUCCESS, q == Q,
// qprime == Q, nst > 0, check_tolsf == 0, tstopset and tstop == next_disc. tlim = min(next
// output time, end time). Returns the result of the last step exactly as cvode_one_step would;
// the driver counts that step, the loop counts the others in current_step.
template <int Q, int NS, class S, class Model>
BDF_INL int fast_run(S& s, const Model& mdl, double (&yout)[NS], double& tret, double tlim, int& current_step,
                     int max_steps, Pending& pd)
{
    // run: completed steps of this loop since h last changed (tau[1..run] == h); have: the
    // coefficients held in s / tc / rl1 were computed with tau[1..Q] == h at the current h and no
    // setup has changed gammap since. cscale_h is the Newton scale 2 / (1 + gamrat) computed from
    // gamrat_h, the gamrat it was computed with.
    int run = 0;
    bool have = false;
    TqCtx tc;
    double rl1 = 0.0, cscale_h = 1.0, gamrat_h = 0.0;
    for (;;) {
#ifdef BCM3_MARKS
        asm volatile("; BDFMARK fast_top Q=%0" ::"i"(Q));
#endif
        BDF_PH(18);  // the loop's exit test and back edge
        const unsigned ph_t0 = BDF_PH_NOW();
        vec::ewt_set(s);
        const double saved_t = s.tn;
        const double eta_eff = (s.hprime != s.h) ? s.eta : 1.0;
        if (eta_eff != 1.0) {
            run = 0;
            have = false;
        }
        const bool reuse = have;
        // A plain step: the coefficients are held (so h is unchanged: no rescale), gamrat is the
        // one the held Newton scale was computed with, and no linear-solver setup is due -- the
        // callSetup test of the attempt (nst >= nstlp + MSBP | |gamrat - 1| > DGMAX) is false
        // because its gamrat part was false when the coefficients were computed (a setup then
        // clears `have`) and gamrat has not changed. One branch instead of the rescale, cvSet,
        // setup and scale tests.
        const bool plain = reuse & (s.nst < s.nstlp + MSBP) & (s.gamrat == gamrat_h);
        // the step's tail, instantiated in each branch: the usual outcome -- Newton converges on its
        // first correction and the error test passes (a first-iteration convergence has local error
        // dsm = acnrm tq[2] = del tq[2]) -- is ONE branch; anything else goes on through newton_rest,
        // which repeats the convergence test. false: the first attempt failed, the attempt loop takes
        // over. HELD (the plain step): tau[1..Q] all equal h, the completion skips their shift.
#ifdef BCM3_ONE_TAIL
        auto tail = [&](bool held, double del, bool setup, double cscale) __attribute__((always_inline)) {
#else
        auto tail = [&](auto held, double del, bool setup, double cscale) __attribute__((always_inline)) {
#endif
            double dsm = del * s.tq[2];
            if (BDF_LIKELY(div_le_one(del * SUNMIN(1.0, s.crate), s.tq[4]) & (dsm <= 1.0))) {
                s.acnrm = del;
                s.nls_jcur = 0;
#ifndef BCM3_ONE_TAIL
                if constexpr (decltype(held)::value)
                    BDF_PH(15);
                else
                    BDF_PH(24);
#endif
            } else {
                const bool conv = vec::newton_rest<NS>(s, mdl, rl1, CONV_NONE, setup, cscale, del);
                BDF_PH(5);
                dsm = s.acnrm * s.tq[2];
                if (BDF_UNLIKELY(!(conv & (dsm <= 1.0)))) {
                    vec::restore_q<Q>(s, saved_t);
                    s.tretlast = saved_t;
                    pd.saved_t = saved_t;
                    pd.eta_eff = eta_eff;
                    pd.r = conv ? uni::ATTEMPT_ERR_FAIL : uni::ATTEMPT_CONV_FAIL;
                    pd.dsm = dsm;
                    return false;
                }
            }
#ifdef BCM3_ONE_TAIL
            vec::complete_head_q_rt<Q>(s, held);
            vec::complete_eta_q<Q, NS, true, 25>(s, dsm, tc);
#else
            vec::complete_q<Q, NS, true, decltype(held)::value ? 16 : 25, decltype(held)::value>(s, dsm, tc);
#endif
            return true;
        };
#ifdef BCM3_ONE_TAIL
        // one instance of the tail (convergence / error test, Newton iterations, completion with its
        // order-change evaluation) for both branches: the plain flag decides the tau shift at run time
        double del_t, cscale_t;
        bool setup_t;
#endif
        if (BDF_LIKELY(plain)) {
            BDF_PH(10);
            vec::predict_q<Q>(s);
            BDF_PH(11);
            s.acor = 0.0;
            double cscale = cscale_h;
            if constexpr (BDF_DBL(9)) {
                S s2 = s;
                vec::dbl_launder_state(s2);
                vec::predict_q<Q>(s2);
                cfor<0, Q + 1>([&](auto k) __attribute__((always_inline)) { bdf_consume(s2.zn[CI(k)]); });
                bdf_consume(s2.tn);
            }
            if constexpr (BDF_DBL(5)) {
                S s2 = s;
                vec::dbl_launder_state(s2);
                double cs2 = bdf_launder(cscale);
                bdf_consume(vec::newton_correction<NS>(s2, mdl, bdf_launder(rl1), cs2, false, false, CONV_NONE));
                bdf_consume(s2.acor);
            }
            const double del = vec::newton_correction<NS, 12>(s, mdl, rl1, cscale, false, false, CONV_NONE);
            run++;  // have stays set (reuse, no setup)
#ifdef BCM3_ONE_TAIL
            del_t = del;
            cscale_t = cscale;
            setup_t = false;
#else
            if (!tail(std::true_type{}, del, false, cscale)) return NEED_ATTEMPTS;
#endif
        } else {
            BDF_PH(2);
            // cvStep's attempt at order Q (attempt_q with nflag == FIRST_CALL, nst > 0)
#ifdef BCM3_MARKS
            asm volatile("; BDFMARK general");
#endif
            if (eta_eff != 1.0) vec::rescale_q<Q>(s, eta_eff);
            vec::predict_q<Q>(s);
            BDF_PH(3);
            if (!reuse) {
                if constexpr (BDF_DBL(4)) {
                    S s2 = s;
                    vec::dbl_launder_state(s2);
                    TqCtx tc2;
                    bdf_consume(vec::set_bdf_q<Q, true>(s2, tc2));
                    cfor<0, Q + 1>([&](auto k) __attribute__((always_inline)) { bdf_consume(s2.l[CI(k)]); });
                    bdf_consume(s2.tq[2]);
                    bdf_consume(s2.tq[4]);
                    bdf_consume(s2.tq[5]);
                    bdf_consume(s2.gamma);
                    bdf_consume(s2.gamrat);
                    bdf_consume(tc2.alpha0_hat);
                    bdf_consume(tc2.xi_inv);
                    bdf_consume(tc2.xistar_inv);
                    bdf_consume(tc2.hsum2);
                    bdf_consume(tc2.lq);
                    bdf_consume(tc2.A2);
                }
                rl1 = vec::set_bdf_q<Q, true>(s, tc);
            }
            BDF_PH(4);
            const bool setup = (s.nst >= s.nstlp + MSBP) | (fabs(s.gamrat - 1.0) > DGMAX);
            double cscale = (s.gamrat != 1.0) ? fdiv(2.0, 1.0 + s.gamrat) : 1.0;
            gamrat_h = s.gamrat;
            cscale_h = cscale;
            s.acor = 0.0;
            const double del = vec::newton_correction<NS>(s, mdl, rl1, cscale, setup, false, CONV_NONE);
#ifdef BCM3_KEEP_ON_SETUP
            // a linear-solver setup leaves l, tq and gamma as they are (they depend on h and tau only)
            // and sets gammap = gamma, gamrat = 1: cvSet would recompute gamrat = gamma / gammap = 1
            // exactly (a correctly rounded x / x), so the held coefficients stay valid with gamrat 1
            // and Newton scale 1 -- the next step is plain instead of recomputing cvSet
            have = reuse | (run >= Q);
            if (setup) {
                gamrat_h = 1.0;
                cscale_h = 1.0;
            }
#else
            have = (reuse | (run >= Q)) & !setup;
#endif
            run++;
#ifdef BCM3_ONE_TAIL
            del_t = del;
            cscale_t = cscale;
            setup_t = setup;
#else
            if (!tail(std::false_type{}, del, setup, cscale)) return NEED_ATTEMPTS;
#endif
        }
#ifdef BCM3_ONE_TAIL
        if (!tail(plain, del_t, setup_t, cscale_t)) return NEED_ATTEMPTS;
#endif
        const double troundoff = FUZZ_FACTOR * UROUND * (fabs(s.tn) + fabs(s.h));
        const bool quiet = (fabs(s.tn - s.tstop) > troundoff) & !((s.tn + s.hprime - s.tstop) * s.h > 0.0) &
                           (s.tn < tlim) & (s.qprime == Q) & (current_step + 1 != max_steps);
        if constexpr (BDF_DBL(8)) {
            const double tn2 = bdf_launder(s.tn);
            const double tr2 = FUZZ_FACTOR * UROUND * (fabs(tn2) + fabs(s.h));
            const bool q2 = (fabs(tn2 - s.tstop) > tr2) & !((tn2 + s.hprime - s.tstop) * s.h > 0.0) & (tn2 < tlim) &
                            (s.qprime == Q) & (current_step + 1 != max_steps);
            bdf_consume(q2 ? 1.0 : 0.0);
        }
        BDF_PH_STEP(ph_t0, 19, 20, plain);
#ifdef BCM3_PHASES
        s.ph[21] += plain ? 1 : 0;
        s.ph[22] += plain ? 0 : 1;
#endif
        if (BDF_UNLIKELY(!quiet)) return vec::finish_step<NS>(s, yout, tret);
        current_step++;
    }
}

}  // namespace vec
}  // namespace bcm3hip
