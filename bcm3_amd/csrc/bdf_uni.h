// bdf_uni.h -- the CVODE BDF step of bdf_lane.h specialised for ONE trajectory per wavefront
// (UNI launch: every value is wave-uniform).
//
// Same algorithm and the same floating-point operations as cvode_one_step in bdf_lane.h (the
// two paths agree bit for bit, tests/test_popk_gpu.py); what changes is the control flow. One
// wavefront alone on a SIMD is issue bound: every VALU instruction costs ~4 cycles whether or
// not it depends on the previous one, a branch ~20-40 cycles taken or not, a select ~4 per
// 32-bit half (tools/ubench, profiles/r01_ubench.txt). So the instruction count is the cost:
//  * the step is instantiated per BDF order Q = 1..5 (one dispatch per attempt): no guards on
//    the runtime order inside predict / rescale / set / complete;
//  * work of a few instructions is done unconditionally and selected (rescaling by eta = 1
//    replaces the "h changed?" branch, x * 1.0 == x); work of tens of instructions that is
//    needed only every q+1 steps or rarely (tq[1]/tq[3], the order-change candidates, the
//    tstop clamp, the multi-iteration norm) sits behind one scalar branch;
//  * rare events (first step after ReInit, tstop reached, failures, order changes) stay behind
//    one branch each and reuse the generic routines of bdf_lane.h.
#pragma once
#include "bdf_lane.h"

namespace bcm3hip {
namespace uni {

// cvRescale with eta_eff (1.0 when the step size is unchanged: exact no-op)
template <int Q, int NS, class S>
BDF_INL void rescale_q(S& s, double eta)
{
    double c = eta;
    cfor<1, Q + 1>([&](auto j) __attribute__((always_inline)) {
        cfor<0, NS>([&](auto i) __attribute__((always_inline)) { s.zn[CI(j)][CI(i)] *= c; });
        c = eta * c;
    });
    s.h = s.hscale * eta;
    s.hscale = s.h;
}

template <int Q, int NS, class S>
BDF_INL void predict_q(S& s)
{
    s.tn += s.h;
    const double tc = s.tstop;
    s.tn = ((s.tstopset != 0) & ((s.tn - tc) * s.h > 0.0)) ? tc : s.tn;
    cfor<1, Q + 1>([&](auto k) __attribute__((always_inline)) {
        cfor_down<Q, CI(k)>([&](auto j) __attribute__((always_inline)) {
            cfor<0, NS>([&](auto i) __attribute__((always_inline)) {
                s.zn[CI(j) - 1][CI(i)] += s.zn[CI(j)][CI(i)];
            });
        });
    });
}

template <int Q, int NS, class S>
BDF_INL void restore_q(S& s, double saved_t)
{
    s.tn = saved_t;
    cfor<1, Q + 1>([&](auto k) __attribute__((always_inline)) {
        cfor_down<Q, CI(k)>([&](auto j) __attribute__((always_inline)) {
            cfor<0, NS>([&](auto i) __attribute__((always_inline)) {
                s.zn[CI(j) - 1][CI(i)] -= s.zn[CI(j)][CI(i)];
            });
        });
    });
}

// cvSetBDF + cvSetTqBDF + cvSet for order Q.
template <int Q, class S>
BDF_INL double set_bdf_q(S& s)
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
    // tq[5] unconditionally as cvSetTqBDF does (qwait <= 2, when it is read, holds in almost every
    // step, so a branch around it costs more than it saves); tq[1], tq[3] only at qwait == 1
    s.tq[5] = fabs(fdiv(A2 * xistar_inv, lq * xi_inv));
    {
        if (s.qwait == 1) {
            // qwait == 1 block of cvSetTqBDF
            double tq1 = 1.0;
            if constexpr (q > 1) {
                const double C = fdiv(xistar_inv, lq);
                const double A3 = alpha0 + 1.0 / q;
                const double A4 = alpha0_hat + xi_inv;
                const double Cpinv = fdiv_c(1.0 - A4 + A3, A3, 1.0 / tq_a3(q));
                tq1 = fabs(C * Cpinv);
            }
            const double hsum2 = hsum + s.tau[q];
            const double xi_inv2 = fdiv(s.h, hsum2);
            const double A5 = alpha0 - 1.0 / (q + 1);
            const double A6 = alpha0_hat - xi_inv2;
            const double Cppinv = fdiv(1.0 - A6 + A5, A2);
            const double tq3 = fabs(fdiv(Cppinv, xi_inv2 * (double)(q + 2) * A5));
            s.tq[1] = tq1;
            s.tq[3] = tq3;
        }
    }
    s.tq[4] = fdiv(CORTES, s.tq[2]);
    // at q = 2, l[1] = 1.5 is a compile-time constant here but not in the lane solver (runtime q):
    // the compiler would fold v_rcp_f64(1.5) to the correctly rounded value while the hardware
    // estimate (one Newton step, frcp) differs, so the operand is passed through a runtime 1.0
    const double rl1 = frcp((q == 2) ? s.l[1] * s.unity : s.l[1]);
    s.gamma = s.h * rl1;
    s.gammap = (s.nst == 0) ? s.gamma : s.gammap;
    const double gr = fdiv(s.gamma, s.gammap);
    s.gamrat = (s.nst > 0) ? gr : 1.0;
    return rl1;
}

// eta_exact of bdf_lane.h
BDF_INL double eta_from_u(double bx, int k) { return eta_exact(bx, k); }

// Step-size ratios below THRESH are discarded (cvSetEta: eta = 1), so an eta candidate only has
// to be computed exactly when it can reach THRESH. eta = 1 / (bx^(1/k) + ADDON) >= THRESH needs
// bx <= (1/THRESH - ADDON)^k; above that bound (with a 1e-9 relative margin, far wider than the
// few-ulp error of the seed) the candidate is replaced by 0, which every later use (the
// THRESH test, the max over candidates and the equality tests of cvChooseEta) treats exactly
// like the true value < THRESH.
constexpr double eta_cut(int k)
{
    double c = 1.0;
    for (int i = 0; i < k; i++) c *= (1.0 / THRESH - ADDON);
    return c * (1.0 + 1e-9);
}
template <int K>
BDF_INL double eta_candidate(double bx)
{
    constexpr double cut = eta_cut(K);
    if (BDF_LIKELY(bx > cut)) return 0.0;
    return eta_from_u(bx, K);
}

// One Newton correction (residual, optional setup, solve, update): the body shared by the
// first and the later iterations of newton_u.
template <int NS, class S, class Model>
BDF_INL double newton_correction(S& s, const Model& mdl, double rl1, double& cscale, bool setup, bool jbad,
                                 int convfail)
{
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
    if (BDF_UNLIKELY(setup)) {
        // cvNlsLSetup -> cvLsSetup (cvode_ls.c:1415-1500)
        if (jbad) convfail = CONV_BAD_J;
        const double dgamma = fabs(fdiv(s.gamma, s.gammap) - 1.0);
        const bool jnew = (s.nst == 0) | (s.nst > s.nstlj + CVLS_MSBJ) |
                          ((convfail == CONV_BAD_J) & (dgamma < CVLS_DGMAX)) | (convfail == CONV_OTHER);
        s.cnt.nje += jnew ? 1 : 0;
        s.nstlj = jnew ? s.nst : s.nstlj;
        mdl.lin_setup(s.gamma, s.inv);
        s.cnt.nsetups++;
        s.nls_jcur = jnew;
        s.gamrat = 1.0;
        cscale = 1.0;
        s.gammap = s.gamma;
        s.crate = 1.0;
        s.nstlp = s.nst;
    }
    s.cnt.nni++;
    double b[NS], x[NS];
    cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
        constexpr int i = CI(I_);
        b[i] = -delta[i];
    });
    mdl.lin_solve(s.inv, b, x);
    cfor<0, NS>([&](auto I_) __attribute__((always_inline)) {
        constexpr int i = CI(I_);
        x[i] *= cscale;
        s.acor[i] += x[i];
    });
    return wrms<NS>(x, s.ewt);
}

// Newton iteration of cvNls (bdf_lane.h newton; sunnonlinsol_newton.c:183-322, cvNlsConvTest
// cvode_nls.c:236-280) with the first iteration peeled: ~70 % of the steps converge there, and
// it needs neither the convergence-rate update nor the divergence test.
template <int NS, class S, class Model>
BDF_INL bool newton_u(S& s, const Model& mdl, double rl1, int convfail, bool callSetup)
{
    bool jbad = false;
    // 2/(1+gamrat) scaling of cvLsSolve: constant within the solve, 1 after a setup
    double cscale = (s.gamrat != 1.0) ? fdiv(2.0, 1.0 + s.gamrat) : 1.0;
    for (;;) {
        // iteration 0 (crate as left by the previous step)
        double del = newton_correction<NS>(s, mdl, rl1, cscale, callSetup, jbad, convfail);
        // cvNlsConvTest: dcon = del min(1, crate) / tq[4] <= 1
        if (BDF_LIKELY(div_le_one(del * SUNMIN(1.0, s.crate), s.tq[4]))) {
            s.acnrm = del;
            s.nls_jcur = 0;
            return true;
        }
        s.delp = del;
        // iterations 1 .. NLS_MAXCOR-1
        for (int it = 1; it < NLS_MAXCOR; it++) {
            del = newton_correction<NS>(s, mdl, rl1, cscale, false, false, convfail);
            s.crate = SUNMAX(CRDOWN * s.crate, fdiv(del, s.delp));
            if (div_le_one(del * SUNMIN(1.0, s.crate), s.tq[4])) {
                s.acnrm = wrms<NS>(s.acor, s.ewt);
                s.nls_jcur = 0;
                return true;
            }
            if (del > RDIV * s.delp) break;  // diverging
            s.delp = del;
        }
        if (!s.nls_jcur) {  // retry once with a fresh Jacobian (jbad)
            callSetup = true;
            jbad = true;
            cfor<0, NS>([&](auto I_) __attribute__((always_inline)) { s.acor[CI(I_)] = 0.0; });
            continue;
        }
        return false;
    }
}

enum { ATTEMPT_OK = 0, ATTEMPT_CONV_FAIL = 1, ATTEMPT_ERR_FAIL = 2 };

// One attempt of cvStep at order Q: rescale (eta_eff), predict, set, Newton, error test;
// on failure the prediction is undone (cvRestore) before returning.
template <int Q, int NS, class S, class Model>
BDF_INL int attempt_q(S& s, const Model& mdl, double eta_eff, double saved_t, int nflag, double& dsm)
{
    // h == hscale holds between steps, so eta_eff == 1 leaves zn, h and hscale as they are
    if (BDF_UNLIKELY(eta_eff != 1.0)) rescale_q<Q, NS>(s, eta_eff);
    BDF_PH(2);
    predict_q<Q, NS>(s);
    BDF_PH(3);
    const double rl1 = set_bdf_q<Q>(s);
    BDF_PH(4);
    const int convfail = ((nflag == FIRST_CALL) | (nflag == PREV_ERR_FAIL)) ? CONV_NONE : CONV_OTHER;
    const bool callSetup = (nflag == PREV_CONV_FAIL) | (nflag == PREV_ERR_FAIL) | (s.nst == 0) |
                           (s.nst >= s.nstlp + MSBP) | (fabs(s.gamrat - 1.0) > DGMAX);
    cfor<0, NS>([&](auto I_) __attribute__((always_inline)) { s.acor[CI(I_)] = 0.0; });
    const bool conv = newton_u<NS>(s, mdl, rl1, convfail, callSetup);
    BDF_PH(5);
    dsm = s.acnrm * s.tq[2];
    if (BDF_LIKELY(conv & (dsm <= 1.0))) return ATTEMPT_OK;
    restore_q<Q, NS>(s, saved_t);
    return conv ? ATTEMPT_ERR_FAIL : ATTEMPT_CONV_FAIL;
}

// cvCompleteStep + cvPrepareNextStep (+ cvComputeEtaqm1/qp1, cvChooseEta, cvSetEta) at order Q.
template <int Q, int NS, class S>
BDF_INL void complete_q(S& s, double dsm)
{
    constexpr int q = Q;
    s.nst++;
    s.cnt.nst_total++;
    s.hu = s.h;
    cfor_down<Q, 2>([&](auto i) __attribute__((always_inline)) { s.tau[CI(i)] = s.tau[CI(i) - 1]; });
    if constexpr (q == 1) s.tau[2] = (s.nst > 1) ? s.tau[1] : s.tau[2];
    s.tau[1] = s.h;
    cfor<0, Q + 1>([&](auto j) __attribute__((always_inline)) {
        cfor<0, NS>([&](auto i) __attribute__((always_inline)) { s.zn[CI(j)][CI(i)] = s.zn[CI(j)][CI(i)] + s.l[CI(j)] * s.acor[CI(i)]; });
    });
    s.qwait--;
    if constexpr (q != QMAX) {
        const bool save = (s.qwait == 1);
        cfor<0, NS>([&](auto i) __attribute__((always_inline)) {
            s.zn[QMAX][CI(i)] = save ? s.acor[CI(i)] : s.zn[QMAX][CI(i)];
        });
        s.saved_tq5 = save ? s.tq[5] : s.saved_tq5;
    }
    BDF_PH(7);

    if (BDF_UNLIKELY(s.etamax == 1.0)) {
        s.qwait = SUNMAX(s.qwait, 2);
        s.qprime = q;
        s.hprime = s.h;
        s.eta = 1.0;
    } else {
        const double etaq = eta_candidate<q + 1>(BIAS2 * dsm);
        double eta = etaq;
        s.qprime = q;
        if (s.qwait == 0) {
            // cvComputeEtaqm1 / cvComputeEtaqp1 / cvChooseEta, every q+1 steps
            s.qwait = 2;
            double etaqm1 = 0.0, etaqp1 = 0.0;
            if constexpr (q > 1) etaqm1 = eta_candidate<q>(BIAS1 * (wrms<NS>(s.zn[q], s.ewt) * s.tq[1]));
            if constexpr (q != QMAX) {
                if (s.saved_tq5 != 0.0) {
                    const double cquot = fdiv(s.tq[5], s.saved_tq5) * powI(fdiv(s.h, s.tau[2]), q + 1);
                    double tv[NS];
                    cfor<0, NS>([&](auto i) __attribute__((always_inline)) {
                        tv[CI(i)] = (-cquot) * s.zn[QMAX][CI(i)] + s.acor[CI(i)];
                    });
                    etaqp1 = eta_candidate<q + 2>(BIAS3 * (wrms<NS>(tv, s.ewt) * s.tq[3]));
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
                cfor<0, NS>([&](auto i) __attribute__((always_inline)) { s.zn[QMAX][CI(i)] = s.acor[CI(i)]; });
            }
        }
        // cvSetEta (hmax_inv = 0)
        const bool small = (eta < THRESH);
        s.eta = small ? 1.0 : SUNMIN(eta, s.etamax);
        s.hprime = small ? s.h : s.h * s.eta;
    }
    BDF_PH(8);
    s.etamax = (s.nst <= SMALL_NST) ? ETAMX2 : ETAMX3;
    cfor<0, NS>([&](auto i) __attribute__((always_inline)) { s.acor[CI(i)] *= s.tq[2]; });
}

// attempt at order Q and, when it passes, the completion at the same order (one dispatch on q)
template <int Q, int NS, class S, class Model>
BDF_INL int step_q(S& s, const Model& mdl, double eta_eff, double saved_t, int nflag, double& dsm)
{
    const int r = attempt_q<Q, NS>(s, mdl, eta_eff, saved_t, nflag, dsm);
    if (BDF_LIKELY(r == ATTEMPT_OK)) complete_q<Q, NS>(s, dsm);
#ifdef BCM3_PHASES
    if (r == ATTEMPT_OK) s.qh[Q]++;
#endif
    return r;
}

// CVode(..., CV_ONE_STEP) for the UNI launch: same contract as bcm3hip::cvode_one_step, except
// that a successful step does not copy zn[0] to yout (the caller reads s.zn[0]).
// hot: the previous call returned CV_SUCCESS and nothing changed the solver since. The entry
// tests are then known: nst > 0, tretlast == tn, the tstop tests of the step's end (same
// expressions, same values) found tstop neither reached nor inside the next step, or already
// applied the clamp (hprime, eta) that the entry test would recompute identically.
template <int NS, class S, class Model>
BDF_INL int cvode_one_step_u(S& s, const Model& mdl, double tout, double (&yout)[NS], double& tret, bool hot)
{
    BDF_PH(0);
    {
        // one scalar branch for the common entry (cvode.c:1251-1310): not the first step after
        // (Re)Init, tn was not returned before, tstop is neither reached nor within the next step
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
                ewt_set<NS>(s, s.zn[0], s.ewt);
                s.nstlj = 0;
                s.nls_jcur = 0;
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
                cfor<0, NS>([&](auto i) __attribute__((always_inline)) { s.zn[1][CI(i)] *= s.h; });
            } else {
                if (ret_prev) {
                    s.tretlast = tret = s.tn;
                    cfor<0, NS>([&](auto i) __attribute__((always_inline)) { yout[CI(i)] = s.zn[0][CI(i)]; });
                    return CV_SUCCESS;
                }
                if (at_stop) {
                    if (get_dky<NS>(s, s.tstop, yout) != CV_SUCCESS) return CV_ILL_INPUT;
                    s.tretlast = tret = s.tstop;
                    s.tstopset = 0;
                    return CV_TSTOP_RETURN;
                }
                s.hprime = (s.tstop - s.tn) * (1.0 - 4.0 * UROUND);
                s.eta = fdiv(s.hprime, s.h);
                ewt_set<NS>(s, s.zn[0], s.ewt);
            }
        } else {
            ewt_set<NS>(s, s.zn[0], s.ewt);
        }
    }
    if (BDF_UNLIKELY(s.check_tolsf)) {
        double ss = 0.0;
        cfor<0, NS>([&](auto i) __attribute__((always_inline)) {
            const double p = s.zn[0][CI(i)] * s.ewt[CI(i)];
            ss = (CI(i) == 0) ? p * p : ss + p * p;
        });
        if (ss > (double)NS * (1.0 / (UROUND * UROUND))) {
            s.tretlast = tret = s.tn;
            cfor<0, NS>([&](auto i) __attribute__((always_inline)) { yout[CI(i)] = s.zn[0][CI(i)]; });
            return CV_TOO_MUCH_ACC;
        }
    }
    BDF_PH(1);

    // ---------------- cvStep
    const double saved_t = s.tn;
    int ncf = 0, nef = 0, nflag = FIRST_CALL;
    // cvAdjustParams when the step size changed; rescaling by eta_eff = 1 is a no-op
    const bool adj = (s.nst > 0) & (s.hprime != s.h);
    double eta_eff = adj ? s.eta : 1.0;
    if (BDF_UNLIKELY(adj & (s.qprime != s.q))) {
        adjust_order<NS>(s, s.qprime - s.q);
        s.q = s.qprime;
        s.L = s.q + 1;
        s.qwait = s.L;
    }
    double dsm = 0.0;
    for (;;) {
        int r;
        switch (s.q) {
        case 1: r = step_q<1, NS>(s, mdl, eta_eff, saved_t, nflag, dsm); break;
        case 2: r = step_q<2, NS>(s, mdl, eta_eff, saved_t, nflag, dsm); break;
        case 3: r = step_q<3, NS>(s, mdl, eta_eff, saved_t, nflag, dsm); break;
        case 4: r = step_q<4, NS>(s, mdl, eta_eff, saved_t, nflag, dsm); break;
        default: r = step_q<5, NS>(s, mdl, eta_eff, saved_t, nflag, dsm); break;
        }
        BDF_PH(6);
        if (BDF_LIKELY(r == ATTEMPT_OK)) break;
        // failure handling (cvHandleNFlag / cvDoErrorTest), rare
        eta_eff = 1.0;
        s.etamax = 1.0;
        if (r == ATTEMPT_CONV_FAIL) {
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
            adjust_order<NS>(s, -1);
            s.L = s.q;
            s.q--;
            s.qwait = s.L;
            eta_eff = s.eta;
            continue;
        }
        s.h *= s.eta;
        s.hscale = s.h;
        s.qwait = LONG_WAIT;
        double tv[NS];
        mdl.rhs(s.tn, s.zn[0], tv);
        s.cnt.nfe++;
        cfor<0, NS>([&](auto i) __attribute__((always_inline)) { s.zn[1][CI(i)] = s.h * tv[CI(i)]; });
        eta_eff = 1.0;
    }

    // stop tests after the step (cvode.c:1395-1437)
    const double troundoff = FUZZ_FACTOR * UROUND * (fabs(s.tn) + fabs(s.h));
    const bool reached = fabs(s.tn - s.tstop) <= troundoff;
    if (BDF_UNLIKELY((s.tstopset != 0) & (reached | ((s.tn + s.hprime - s.tstop) * s.h > 0.0)))) {
        if (reached) {
            get_dky<NS>(s, s.tstop, yout);
            s.tretlast = tret = s.tstop;
            s.tstopset = 0;
            BDF_PH(9);
            return CV_TSTOP_RETURN;
        }
        s.hprime = (s.tstop - s.tn) * (1.0 - 4.0 * UROUND);
        s.eta = fdiv(s.hprime, s.h);
    }
    // yout = zn[0] on CV_SUCCESS is left to the caller (needed only on its rare path)
    s.tretlast = tret = s.tn;
    BDF_PH(9);
    return CV_SUCCESS;
}

}  // namespace uni
}  // namespace bcm3hip
