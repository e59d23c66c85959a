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
// GPU design: one trajectory per lane; the Nordsieck array zn[0..5][NS], error weights,
// saved Jacobian and the explicit (I - gamma J)^-1 stay in registers for the whole solve.
// Loops whose trip count depends on the runtime order q are fully unrolled over 1..QMAX with
// lane predicates so every register array is indexed with compile-time indices (a runtime
// index would spill the array to scratch). Lanes of a wavefront diverge freely; the
// reconvergence point is one CVode(ONE_STEP) call per iteration of the caller's loop.
#pragma once
#include <hip/hip_runtime.h>

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

enum { DO_ERROR_TEST = 2, PREDICT_AGAIN = 3, TRY_AGAIN = 5, FIRST_CALL = 6, PREV_CONV_FAIL = 7,
       PREV_ERR_FAIL = 8 };
enum { NLS_SUCCESS = 0, NLS_CONTINUE = 901, NLS_CONV_RECVR = 902 };
enum { CONV_NONE = 0, CONV_BAD_J = 1, CONV_OTHER = 2 };
enum { CV_SUCCESS = 0, CV_TSTOP_RETURN = 1, CV_TOO_MUCH_ACC = -2, CV_ERR_FAILURE = -3,
       CV_CONV_FAILURE = -4, CV_UNREC = -8, CV_ILL_INPUT = -22, CV_BAD_T = -26, CV_TOO_CLOSE = -27 };

#define BDF_INL __device__ __forceinline__
#define SUNMAX(A, B) ((A) > (B) ? (A) : (B))
#define SUNMIN(A, B) ((A) < (B) ? (A) : (B))

// 1/j for j = 0..7, exactly the correctly rounded quotients (1.0 / j at run time).
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

// Opaque register copy. Runtime-indexed selections are written as value selects over opaque
// copies so the optimizer cannot turn them into a switch with a pointer phi (which keeps the
// whole register state in scratch memory: SROA cannot promote through pointer phis).
BDF_INL double opq(double v)
{
    asm("" : "+v"(v));
    return v;
}

// runtime-indexed read of a small register array without scratch
template <int K>
BDF_INL double sel(const double (&a)[K], int i)
{
    double r = opq(a[0]);
#pragma unroll
    for (int k = 1; k < K; k++) r = (i == k) ? opq(a[k]) : r;
    return r;
}

// r = zn[q] for q in 1..QMAX (value select, see opq)
template <int NS>
BDF_INL void sel_row(const double (&zn)[QMAX + 1][NS], int q, double (&r)[NS])
{
#pragma unroll
    for (int i = 0; i < NS; i++) {
        double v = opq(zn[1][i]);
#pragma unroll
        for (int j = 2; j <= QMAX; j++) v = (q == j) ? opq(zn[j][i]) : v;
        r[i] = v;
    }
}

// SUNRpowerR (sundials_math.c:40-52)
BDF_INL double powR(double base, double e) { return (base <= 0.0) ? 0.0 : pow(base, e); }
// SUNRpowerI for a non-negative exponent 1..6 (repeated multiplication, sundials_math.c:28-38)
BDF_INL double powI(double base, int e)
{
    double prod = 1.0;
#pragma unroll
    for (int i = 1; i <= QMAX + 1; i++)
        if (i <= e) prod *= base;
    return prod;
}
BDF_INL double sun_sqrt(double x) { return (x <= 0.0) ? 0.0 : sqrt(x); }

struct BdfCounters {
    int nst_total, nfe, nni, nsetups, nje, netf, ncfn, nreinit;
};

// Model concept:  BDF_INL void rhs(double t, const double (&y)[NS], double (&ydot)[NS]);
//                 BDF_INL void jac(double t, double (&J)[NS][NS]);   // J pre-zeroed
template <int NS>
struct BdfState {
    double rtol, atol;
    double zn[QMAX + 1][NS];
    double ewt[NS], acor[NS], y[NS], ftemp[NS];
    double savedJ[NS][NS], inv[NS][NS];
    double tau[QMAX + 2], tq[6], l[QMAX + 1];
    double tn, h, hprime, eta, hscale, hu, tretlast;
    double rl1, gamma, gammap, gamrat, crate, delp, acnrm, etamax, saved_tq5;
    double etaq, etaqm1, etaqp1;
    double tstop;
    int tstopset;
    int q, qprime, qwait, L;
    int nst, nstlp, nstlj;
    int nls_jcur, cv_jcur, convfail;
    BdfCounters cnt;
};

template <int NS>
BDF_INL double wrms(const double (&x)[NS], const double (&w)[NS])
{
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NS; i++) {
        double p = x[i] * w[i];
        s += p * p;
    }
    return sun_sqrt(s / (double)NS);
}

// cvEwtSetSV: w = 1/(rtol*|y| + atol)
template <int NS>
BDF_INL void ewt_set(const BdfState<NS>& s, const double (&ycur)[NS], double (&w)[NS])
{
#pragma unroll
    for (int i = 0; i < NS; i++) w[i] = 1.0 / (s.rtol * fabs(ycur[i]) + s.atol);
}

// closed-form inverse (sunlinsol_dense_eigen.cpp:111-145 / Eigen compute_inverse<3>)
template <int NS>
BDF_INL void inverse(const double (&a)[NS][NS], double (&r)[NS][NS])
{
    if constexpr (NS == 2) {
        double invdet = 1.0 / (a[0][0] * a[1][1] - a[0][1] * a[1][0]);
        r[0][0] = a[1][1] * invdet;
        r[0][1] = -a[0][1] * invdet;
        r[1][0] = -a[1][0] * invdet;
        r[1][1] = a[0][0] * invdet;
    } else {
        auto cof = [&](int i, int j) {
            int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
            return a[i1][j1] * a[i2][j2] - a[i1][j2] * a[i2][j1];
        };
        double c0 = cof(0, 0), c1 = cof(1, 0), c2 = cof(2, 0);
        double det = c0 * a[0][0] + c1 * a[1][0] + c2 * a[2][0];
        double invdet = 1.0 / det;
        r[0][0] = c0 * invdet;
        r[0][1] = c1 * invdet;
        r[0][2] = c2 * invdet;
        r[1][0] = cof(0, 1) * invdet;
        r[1][1] = cof(1, 1) * invdet;
        r[1][2] = cof(2, 1) * invdet;
        r[2][0] = cof(0, 2) * invdet;
        r[2][1] = cof(1, 2) * invdet;
        r[2][2] = cof(2, 2) * invdet;
    }
}

// cvLsSetup + cvLsLinSys + SUNLinSolSetup (cvode_ls.c:1201-1282, 1415-1500)
template <int NS, class Model>
BDF_INL void ls_setup(BdfState<NS>& s, Model& mdl, int convfail)
{
    double dgamma = fabs((s.gamma / s.gammap) - 1.0);
    bool jbad = (s.nst == 0) || (s.nst > s.nstlj + CVLS_MSBJ) ||
                ((convfail == CONV_BAD_J) && (dgamma < CVLS_DGMAX)) || (convfail == CONV_OTHER);
    if (jbad) {
        double J[NS][NS];
#pragma unroll
        for (int r = 0; r < NS; r++)
#pragma unroll
            for (int c = 0; c < NS; c++) J[r][c] = 0.0;
        mdl.jac(s.tn, J);
#pragma unroll
        for (int r = 0; r < NS; r++)
#pragma unroll
            for (int c = 0; c < NS; c++) s.savedJ[r][c] = J[r][c];
        s.cv_jcur = 1;
        s.cnt.nje++;
        s.nstlj = s.nst;
    } else {
        s.cv_jcur = 0;
    }
    double A[NS][NS];
#pragma unroll
    for (int r = 0; r < NS; r++)
#pragma unroll
        for (int c = 0; c < NS; c++) A[r][c] = s.savedJ[r][c] * (-s.gamma);
#pragma unroll
    for (int i = 0; i < NS; i++) A[i][i] += 1.0;
    inverse<NS>(A, s.inv);
}

// cvNlsLSetup (cvode_nls.c)
template <int NS, class Model>
BDF_INL void nls_lsetup(BdfState<NS>& s, Model& mdl, bool jbad)
{
    if (jbad) s.convfail = CONV_BAD_J;
    ls_setup<NS>(s, mdl, s.convfail);
    s.cnt.nsetups++;
    s.nls_jcur = s.cv_jcur;
    s.gamrat = 1.0;
    s.gammap = s.gamma;
    s.crate = 1.0;
    s.nstlp = s.nst;
}

// cvNlsResidual: y = zn0 + ycor; ftemp = f(tn,y); res = rl1*zn1 + ycor; res += -gamma*ftemp
template <int NS, class Model>
BDF_INL void nls_residual(BdfState<NS>& s, Model& mdl, double (&res)[NS])
{
#pragma unroll
    for (int i = 0; i < NS; i++) s.y[i] = s.zn[0][i] + s.acor[i];
    mdl.rhs(s.tn, s.y, s.ftemp);
    s.cnt.nfe++;
#pragma unroll
    for (int i = 0; i < NS; i++) res[i] = s.rl1 * s.zn[1][i] + s.acor[i];
#pragma unroll
    for (int i = 0; i < NS; i++) res[i] += (-s.gamma) * s.ftemp[i];
}

// SUNNonlinSolSolve_Newton (sunnonlinsol_newton.c:183-322) with cvLsSolve and cvNlsConvTest
template <int NS, class Model>
BDF_INL int newton_solve(BdfState<NS>& s, Model& mdl, double tol, bool callLSetup)
{
    bool jbad = false;
    double delta[NS];
    int retval = NLS_SUCCESS;
    for (;;) {
        nls_residual<NS>(s, mdl, delta);
        if (callLSetup) nls_lsetup<NS>(s, mdl, jbad);
        int curiter = 0;
        for (;;) {
            s.cnt.nni++;
            // delta = -delta; solve; scale (cvLsSolve, cvode_ls.c:1597-1604)
            double b[NS], x[NS];
#pragma unroll
            for (int i = 0; i < NS; i++) b[i] = -delta[i];
#pragma unroll
            for (int i = 0; i < NS; i++) {
                double acc = s.inv[i][0] * b[0];
#pragma unroll
                for (int j = 1; j < NS; j++) acc = acc + s.inv[i][j] * b[j];
                x[i] = acc;
            }
            if (s.gamrat != 1.0) {
                double c = 2.0 / (1.0 + s.gamrat);
#pragma unroll
                for (int i = 0; i < NS; i++) x[i] *= c;
            }
#pragma unroll
            for (int i = 0; i < NS; i++) {
                delta[i] = x[i];
                s.acor[i] += delta[i];
            }
            // cvNlsConvTest (cvode_nls.c:236-280)
            double del = wrms<NS>(delta, s.ewt);
            if (curiter > 0) s.crate = SUNMAX(CRDOWN * s.crate, del / s.delp);
            double dcon = del * SUNMIN(1.0, s.crate) / tol;
            if (dcon <= 1.0) {
                s.acnrm = (curiter == 0) ? del : wrms<NS>(s.acor, s.ewt);
                s.nls_jcur = 0;
                return NLS_SUCCESS;
            }
            if ((curiter >= 1) && (del > RDIV * s.delp)) {
                retval = NLS_CONV_RECVR;
                break;
            }
            s.delp = del;
            curiter++;
            if (curiter >= NLS_MAXCOR) {
                retval = NLS_CONV_RECVR;
                break;
            }
            nls_residual<NS>(s, mdl, delta);
        }
        if (!s.nls_jcur) {
            callLSetup = true;
            jbad = true;
#pragma unroll
            for (int i = 0; i < NS; i++) s.acor[i] = 0.0;
            continue;
        }
        break;
    }
    return retval;
}

// cvRescale (cvode.c:2393-2406)
template <int NS>
BDF_INL void rescale(BdfState<NS>& s)
{
    double c = s.eta;
#pragma unroll
    for (int j = 1; j <= QMAX; j++) {
        const bool on = (j <= s.q);
#pragma unroll
        for (int i = 0; i < NS; i++) s.zn[j][i] = on ? s.zn[j][i] * c : s.zn[j][i];
        c = s.eta * c;
    }
    s.h = s.hscale * s.eta;
    s.hscale = s.h;
}

// cvPredict (BCM: N_VAdd(zn[j-1], zn[j]) -> zn[j-1] += zn[j])
template <int NS>
BDF_INL void predict(BdfState<NS>& s)
{
    s.tn += s.h;
    if (s.tstopset) {
        if ((s.tn - s.tstop) * s.h > 0.0) s.tn = s.tstop;
    }
#pragma unroll
    for (int k = 1; k <= QMAX; k++)
#pragma unroll
        for (int j = QMAX; j >= k; j--) {
            const bool on = (j <= s.q);
#pragma unroll
            for (int i = 0; i < NS; i++) s.zn[j - 1][i] = on ? s.zn[j - 1][i] + s.zn[j][i] : s.zn[j - 1][i];
        }
}

// cvRestore: zn[j-1] += (-1)*zn[j]
template <int NS>
BDF_INL void restore(BdfState<NS>& s, double saved_t)
{
    s.tn = saved_t;
#pragma unroll
    for (int k = 1; k <= QMAX; k++)
#pragma unroll
        for (int j = QMAX; j >= k; j--) {
            const bool on = (j <= s.q);
#pragma unroll
            for (int i = 0; i < NS; i++) s.zn[j - 1][i] = on ? s.zn[j - 1][i] - s.zn[j][i] : s.zn[j - 1][i];
        }
}

// cvSetBDF + cvSetTqBDF + cvSet (cvode.c:2445-2690)
template <int NS>
BDF_INL void set_bdf(BdfState<NS>& s)
{
    const int q = s.q;
    double alpha0, alpha0_hat, xi_inv, xistar_inv, hsum;
    s.l[0] = s.l[1] = xi_inv = xistar_inv = 1.0;
#pragma unroll
    for (int i = 2; i <= QMAX; i++)
        if (i <= q) s.l[i] = 0.0;
    alpha0 = alpha0_hat = -1.0;
    hsum = s.h;
    if (q > 1) {
#pragma unroll
        for (int j = 2; j < QMAX; j++) {
            if (j < q) {
                hsum += s.tau[j - 1];
                xi_inv = s.h / hsum;
                alpha0 -= 1.0 / j;
#pragma unroll
                for (int i = j; i >= 1; i--) s.l[i] += s.l[i - 1] * xi_inv;
            }
        }
        alpha0 -= recip_int(q);
        xistar_inv = -s.l[1] - alpha0;
        hsum += sel(s.tau, q - 1);
        xi_inv = s.h / hsum;
        alpha0_hat = -s.l[1] - xi_inv;
#pragma unroll
        for (int i = QMAX; i >= 1; i--)
            if (i <= q) s.l[i] += s.l[i - 1] * xistar_inv;
    }
    // cvSetTqBDF
    double A1 = 1.0 - alpha0_hat + alpha0;
    double A2 = 1.0 + (double)q * A1;
    double lq = sel(s.l, q);
    s.tq[2] = fabs(A1 / (alpha0 * A2));
    s.tq[5] = fabs(A2 * xistar_inv / (lq * xi_inv));
    if (s.qwait == 1) {
        if (q > 1) {
            double C = xistar_inv / lq;
            double A3 = alpha0 + recip_int(q);
            double A4 = alpha0_hat + xi_inv;
            double Cpinv = (1.0 - A4 + A3) / A3;
            s.tq[1] = fabs(C * Cpinv);
        } else {
            s.tq[1] = 1.0;
        }
        hsum += sel(s.tau, q);
        xi_inv = s.h / hsum;
        double A5 = alpha0 - recip_int(q + 1);
        double A6 = alpha0_hat - xi_inv;
        double Cppinv = (1.0 - A6 + A5) / A2;
        s.tq[3] = fabs(Cppinv / (xi_inv * (double)(q + 2) * A5));
    }
    s.tq[4] = CORTES / s.tq[2];
    // cvSet
    s.rl1 = 1.0 / s.l[1];
    s.gamma = s.h * s.rl1;
    if (s.nst == 0) s.gammap = s.gamma;
    s.gamrat = (s.nst > 0) ? s.gamma / s.gammap : 1.0;
}

// cvIncreaseBDF (cvode.c:2310-2340); indx_acor == QMAX always
template <int NS>
BDF_INL void increase_bdf(BdfState<NS>& s)
{
    double alpha0, alpha1, prod, xi, xiold, hsum, A1;
    double l[QMAX + 1];
#pragma unroll
    for (int i = 0; i <= QMAX; i++) l[i] = 0.0;
    l[2] = alpha1 = prod = xiold = 1.0;
    alpha0 = -1.0;
    hsum = s.hscale;
#pragma unroll
    for (int j = 1; j < QMAX; j++) {
        if (j < s.q) {
            hsum += s.tau[j + 1];
            xi = hsum / s.hscale;
            prod *= xi;
            alpha0 -= 1.0 / (j + 1);
            alpha1 += 1.0 / xi;
#pragma unroll
            for (int i = j + 2; i >= 2; i--) l[i] = l[i] * xiold + l[i - 1];
            xiold = xi;
        }
    }
    A1 = (-alpha0 - alpha1) / prod;
    // zn[L] = A1 * zn[QMAX]; zn[j] += l[j]*zn[L], j = 2..q  (L = q+1)
    double znL[NS];
#pragma unroll
    for (int i = 0; i < NS; i++) znL[i] = A1 * s.zn[QMAX][i];
#pragma unroll
    for (int j = 2; j <= QMAX; j++) {
        const bool isL = (j == s.q + 1), on = (j <= s.q);
#pragma unroll
        for (int i = 0; i < NS; i++) {
            double z = opq(s.zn[j][i]);
            z = isL ? znL[i] : z;
            s.zn[j][i] = on ? z + l[j] * znL[i] : z;
        }
    }
#pragma unroll
    for (int i = 0; i <= QMAX; i++) s.l[i] = l[i];
}

// cvDecreaseBDF (cvode.c:2352-2375)
template <int NS>
BDF_INL void decrease_bdf(BdfState<NS>& s)
{
    double l[QMAX + 1];
#pragma unroll
    for (int i = 0; i <= QMAX; i++) l[i] = 0.0;
    l[2] = 1.0;
    double hsum = 0.0;
#pragma unroll
    for (int j = 1; j <= QMAX - 2; j++) {
        if (j <= s.q - 2) {
            hsum += s.tau[j];
            double xi = hsum / s.hscale;
#pragma unroll
            for (int i = j + 2; i >= 2; i--) l[i] = l[i] * xi + l[i - 1];
        }
    }
    double znq[NS];
    sel_row<NS>(s.zn, s.q, znq);
#pragma unroll
    for (int j = 2; j < QMAX; j++) {
        const bool on = (j < s.q);
#pragma unroll
        for (int i = 0; i < NS; i++) s.zn[j][i] = on ? s.zn[j][i] + (-l[j]) * znq[i] : s.zn[j][i];
    }
#pragma unroll
    for (int i = 0; i <= QMAX; i++) s.l[i] = l[i];
}

template <int NS>
BDF_INL void adjust_order(BdfState<NS>& s, int deltaq)
{
    if ((s.q == 2) && (deltaq != 1)) return;
    if (deltaq == 1)
        increase_bdf<NS>(s);
    else if (deltaq == -1)
        decrease_bdf<NS>(s);
}

// cvCompleteStep (cvode.c:3043-3080)
template <int NS>
BDF_INL void complete_step(BdfState<NS>& s)
{
    s.nst++;
    s.cnt.nst_total++;
    s.hu = s.h;
#pragma unroll
    for (int i = QMAX; i >= 2; i--) s.tau[i] = (i <= s.q) ? s.tau[i - 1] : s.tau[i];
    if ((s.q == 1) && (s.nst > 1)) s.tau[2] = s.tau[1];
    s.tau[1] = s.h;
#pragma unroll
    for (int j = 0; j <= QMAX; j++) {
        const bool on = (j <= s.q);
#pragma unroll
        for (int i = 0; i < NS; i++) s.zn[j][i] = on ? s.zn[j][i] + s.l[j] * s.acor[i] : s.zn[j][i];
    }
    s.qwait--;
    if ((s.qwait == 1) && (s.q != QMAX)) {
#pragma unroll
        for (int i = 0; i < NS; i++) s.zn[QMAX][i] = s.acor[i];
        s.saved_tq5 = s.tq[5];
    }
}

// cvSetEta (hmax_inv = 0)
template <int NS>
BDF_INL void set_eta(BdfState<NS>& s)
{
    if (s.eta < THRESH) {
        s.eta = 1.0;
        s.hprime = s.h;
    } else {
        s.eta = SUNMIN(s.eta, s.etamax);
        s.hprime = s.h * s.eta;
    }
}

// cvPrepareNextStep + cvComputeEtaqm1/qp1 + cvChooseEta (cvode.c:3093-3258)
template <int NS>
BDF_INL void prepare_next_step(BdfState<NS>& s, double dsm)
{
    if (s.etamax == 1.0) {
        s.qwait = SUNMAX(s.qwait, 2);
        s.qprime = s.q;
        s.hprime = s.h;
        s.eta = 1.0;
        return;
    }
    s.etaq = 1.0 / (powR(BIAS2 * dsm, recip_int(s.L)) + ADDON);
    if (s.qwait != 0) {
        s.eta = s.etaq;
        s.qprime = s.q;
        set_eta<NS>(s);
        return;
    }
    s.qwait = 2;
    // etaqm1
    s.etaqm1 = 0.0;
    if (s.q > 1) {
        double znq[NS];
#pragma unroll
        for (int i = 0; i < NS; i++) znq[i] = 0.0;
        sel_row<NS>(s.zn, s.q, znq);
        double ddn = wrms<NS>(znq, s.ewt) * s.tq[1];
        s.etaqm1 = 1.0 / (powR(BIAS1 * ddn, recip_int(s.q)) + ADDON);
    }
    // etaqp1
    s.etaqp1 = 0.0;
    if (s.q != QMAX && s.saved_tq5 != 0.0) {
        double cquot = (s.tq[5] / s.saved_tq5) * powI(s.h / s.tau[2], s.L);
        double tv[NS];
#pragma unroll
        for (int i = 0; i < NS; i++) tv[i] = (-cquot) * s.zn[QMAX][i] + s.acor[i];
        double dup = wrms<NS>(tv, s.ewt) * s.tq[3];
        s.etaqp1 = 1.0 / (powR(BIAS3 * dup, recip_int(s.L + 1)) + ADDON);
    }
    // cvChooseEta
    double etam = SUNMAX(s.etaqm1, SUNMAX(s.etaq, s.etaqp1));
    if (etam < THRESH) {
        s.eta = 1.0;
        s.qprime = s.q;
    } else if (etam == s.etaq) {
        s.eta = s.etaq;
        s.qprime = s.q;
    } else if (etam == s.etaqm1) {
        s.eta = s.etaqm1;
        s.qprime = s.q - 1;
    } else {
        s.eta = s.etaqp1;
        s.qprime = s.q + 1;
#pragma unroll
        for (int i = 0; i < NS; i++) s.zn[QMAX][i] = s.acor[i];
    }
    set_eta<NS>(s);
}

// cvStep (cvode.c:2082-2174)
template <int NS, class Model>
BDF_INL int cv_step(BdfState<NS>& s, Model& mdl)
{
    double saved_t = s.tn, dsm = 0.0;
    int ncf = 0, nef = 0, nflag = FIRST_CALL;
    if ((s.nst > 0) && (s.hprime != s.h)) {
        // cvAdjustParams
        if (s.qprime != s.q) {
            adjust_order<NS>(s, s.qprime - s.q);
            s.q = s.qprime;
            s.L = s.q + 1;
            s.qwait = s.L;
        }
        rescale<NS>(s);
    }
    for (;;) {
        predict<NS>(s);
        set_bdf<NS>(s);
        // cvNls (cvode.c:2701-2770)
        s.convfail = ((nflag == FIRST_CALL) || (nflag == PREV_ERR_FAIL)) ? CONV_NONE : CONV_OTHER;
        bool callSetup = (nflag == PREV_CONV_FAIL) || (nflag == PREV_ERR_FAIL) || (s.nst == 0) ||
                         (s.nst >= s.nstlp + MSBP) || (fabs(s.gamrat - 1.0) > DGMAX);
#pragma unroll
        for (int i = 0; i < NS; i++) s.acor[i] = 0.0;
        nflag = newton_solve<NS>(s, mdl, s.tq[4], callSetup);
        if (nflag == NLS_SUCCESS) {
#pragma unroll
            for (int i = 0; i < NS; i++) s.y[i] = s.zn[0][i] + s.acor[i];
            s.cv_jcur = 0;
        } else {
            // cvHandleNFlag (cvode.c:2905-2945), recoverable convergence failure
            s.cnt.ncfn++;
            restore<NS>(s, saved_t);
            ncf++;
            s.etamax = 1.0;
            if ((fabs(s.h) <= 0.0) || (ncf == MXNCF)) return CV_CONV_FAILURE;
            s.eta = SUNMAX(ETACF, 0.0 / fabs(s.h));
            nflag = PREV_CONV_FAIL;
            rescale<NS>(s);
            continue;
        }
        // cvDoErrorTest (cvode.c:2958-3030)
        dsm = s.acnrm * s.tq[2];
        if (dsm <= 1.0) break;
        nef++;
        s.cnt.netf++;
        nflag = PREV_ERR_FAIL;
        restore<NS>(s, saved_t);
        if ((fabs(s.h) <= 0.0) || (nef == MXNEF)) return CV_ERR_FAILURE;
        s.etamax = 1.0;
        if (nef <= MXNEF1) {
            s.eta = 1.0 / (powR(BIAS2 * dsm, recip_int(s.L)) + ADDON);
            s.eta = SUNMAX(ETAMIN, SUNMAX(s.eta, 0.0 / fabs(s.h)));
            if (nef >= SMALL_NEF) s.eta = SUNMIN(s.eta, ETAMXF);
            rescale<NS>(s);
            continue;
        }
        if (s.q > 1) {
            s.eta = SUNMAX(ETAMIN, 0.0 / fabs(s.h));
            adjust_order<NS>(s, -1);
            s.L = s.q;
            s.q--;
            s.qwait = s.L;
            rescale<NS>(s);
            continue;
        }
        s.eta = SUNMAX(ETAMIN, 0.0 / fabs(s.h));
        s.h *= s.eta;
        s.hscale = s.h;
        s.qwait = LONG_WAIT;
        double tv[NS];
        mdl.rhs(s.tn, s.zn[0], tv);
        s.cnt.nfe++;
#pragma unroll
        for (int i = 0; i < NS; i++) s.zn[1][i] = s.h * tv[i];
    }
    complete_step<NS>(s);
    prepare_next_step<NS>(s, dsm);
    s.etamax = (s.nst <= SMALL_NST) ? ETAMX2 : ETAMX3;
#pragma unroll
    for (int i = 0; i < NS; i++) s.acor[i] *= s.tq[2];
    return CV_SUCCESS;
}

// CVodeGetDky(t, k = 0) (cvode.c:1467-1533)
template <int NS>
BDF_INL int get_dky(const BdfState<NS>& s, double t, double (&dky)[NS])
{
    double tfuzz = FUZZ_FACTOR * UROUND * (fabs(s.tn) + fabs(s.hu));
    if (s.hu < 0.0) tfuzz = -tfuzz;
    double tp = s.tn - s.hu - tfuzz;
    double tn1 = s.tn + tfuzz;
    if ((t - tp) * (t - tn1) > 0.0) return CV_BAD_T;
    double sv = (t - s.tn) / s.h;
    if (s.q == 1) {
#pragma unroll
        for (int i = 0; i < NS; i++) dky[i] = sv * s.zn[1][i] + s.zn[0][i];
        return CV_SUCCESS;
    }
    // c_j = s^j by repeated multiplication; z = c_q zn[q] + c_{q-1} zn[q-1] + ... + zn[0]
    double c[QMAX + 1];
    c[0] = 1.0;
#pragma unroll
    for (int j = 1; j <= QMAX; j++) c[j] = c[j - 1] * sv;
#pragma unroll
    for (int i = 0; i < NS; i++) dky[i] = 0.0;
#pragma unroll
    for (int j = QMAX; j >= 0; j--) {
        const bool on = (j <= s.q);
#pragma unroll
        for (int i = 0; i < NS; i++) dky[i] = on ? dky[i] + c[j] * s.zn[j][i] : dky[i];
    }
    return CV_SUCCESS;
}

// cvUpperBoundH0 (cvode.c:2000-2035)
template <int NS>
BDF_INL double upper_bound_h0(const BdfState<NS>& s, double tdist)
{
    double hub_inv = 0.0;
#pragma unroll
    for (int i = 0; i < NS; i++) {
        double w = 1.0 / (s.rtol * fabs(s.zn[0][i]) + s.atol);  // efun into temp1
        double t1 = 1.0 / w;                                  // N_VInv
        t1 += HUB_FACTOR * fabs(s.zn[0][i]);
        double r = fabs(s.zn[1][i]) / t1;
        hub_inv = (i == 0) ? r : ((r > hub_inv) ? r : hub_inv);  // maxCoeff
    }
    double hub = HUB_FACTOR * tdist;
    if (hub * hub_inv > 1.0) hub = 1.0 / hub_inv;
    return hub;
}

// cvHin (cvode.c:1884-1990); the PopPK RHS never fails recoverably
template <int NS, class Model>
BDF_INL int hin(BdfState<NS>& s, Model& mdl, double tout)
{
    double tdiff = tout - s.tn;
    if (tdiff == 0.0) return CV_TOO_CLOSE;
    int sign = (tdiff > 0.0) ? 1 : -1;
    double tdist = fabs(tdiff);
    double tround = UROUND * SUNMAX(fabs(s.tn), fabs(tout));
    if (tdist < 2.0 * tround) return CV_TOO_CLOSE;
    double hlb = HLB_FACTOR * tround;
    double hub = upper_bound_h0<NS>(s, tdist);
    double hg = sun_sqrt(hlb * hub);
    if (hub < hlb) {
        s.h = (sign == -1) ? -hg : hg;
        return CV_SUCCESS;
    }
    double hnew = hg;
    for (int count1 = 1; count1 <= MAX_ITERS; count1++) {
        // cvYddNorm
        double hgs = hg * sign;
        double yy[NS], tv[NS];
#pragma unroll
        for (int i = 0; i < NS; i++) yy[i] = hgs * s.zn[1][i] + s.zn[0][i];
        mdl.rhs(s.tn + hgs, yy, tv);
        s.cnt.nfe++;
        double a = 1.0 / hgs;
#pragma unroll
        for (int i = 0; i < NS; i++) tv[i] = a * (tv[i] - s.zn[1][i]);
        double yddnrm = wrms<NS>(tv, s.ewt);

        hnew = (yddnrm * hub * hub > 2.0) ? sun_sqrt(2.0 / yddnrm) : sun_sqrt(hg * hub);
        if (count1 == MAX_ITERS) break;
        double hrat = hnew / hg;
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

// CVodeReInit (cvode.c:586-683): tau, saved_tq5, tstop persist.
template <int NS>
BDF_INL void reinit(BdfState<NS>& s, double t0, const double (&y0)[NS])
{
    s.tn = t0;
    s.q = 1;
    s.L = 2;
    s.qwait = 2;
    s.etamax = ETAMX1;
    s.hu = 0.0;
#pragma unroll
    for (int i = 0; i < NS; i++) s.zn[0][i] = y0[i];
    s.nst = 0;
    s.nstlp = 0;
    s.cnt.nreinit++;
}

// CVode(..., CV_ONE_STEP) (cvode.c:1006-1443)
template <int NS, class Model>
BDF_INL int cvode_one_step(BdfState<NS>& s, Model& mdl, double tout, double (&yout)[NS], double& tret)
{
    if (s.nst == 0) {
        s.tretlast = tret = s.tn;
        ewt_set<NS>(s, s.zn[0], s.ewt);
        s.nstlj = 0;      // cvLsInitializeCounters
        s.nls_jcur = 0;   // SUNNonlinSolInitialize_Newton
        mdl.rhs(s.tn, s.zn[0], s.zn[1]);
        s.cnt.nfe++;
        if (s.tstopset) {
            if ((s.tstop - s.tn) * (tout - s.tn) <= 0.0) return CV_ILL_INPUT;
        }
        double tout_hin = tout;
        if (s.tstopset && (tout - s.tn) * (tout - s.tstop) > 0.0) tout_hin = s.tstop;
        int hflag = hin<NS>(s, mdl, tout_hin);
        if (hflag != CV_SUCCESS) return hflag;
        if (s.tstopset) {
            if ((s.tn + s.h - s.tstop) * s.h > 0.0) s.h = (s.tstop - s.tn) * (1.0 - 4.0 * UROUND);
        }
        s.hscale = s.h;
        s.hprime = s.h;
#pragma unroll
        for (int i = 0; i < NS; i++) s.zn[1][i] *= s.h;
    } else {
        double troundoff = FUZZ_FACTOR * UROUND * (fabs(s.tn) + fabs(s.h));
        if (fabs(s.tn - s.tretlast) > troundoff) {
            s.tretlast = tret = s.tn;
#pragma unroll
            for (int i = 0; i < NS; i++) yout[i] = s.zn[0][i];
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
                s.eta = s.hprime / s.h;
            }
        }
        ewt_set<NS>(s, s.zn[0], s.ewt);
    }
    // too much accuracy requested (cvode.c:1318-1331)
    double nrm = wrms<NS>(s.zn[0], s.ewt);
    if (UROUND * nrm > 1.0) {
        s.tretlast = tret = s.tn;
#pragma unroll
        for (int i = 0; i < NS; i++) yout[i] = s.zn[0][i];
        return CV_TOO_MUCH_ACC;
    }
    int kflag = cv_step<NS>(s, mdl);
    if (kflag != CV_SUCCESS) {
        s.tretlast = tret = s.tn;
#pragma unroll
        for (int i = 0; i < NS; i++) yout[i] = s.zn[0][i];
        return kflag;
    }
    if (s.tstopset) {
        double troundoff = FUZZ_FACTOR * UROUND * (fabs(s.tn) + fabs(s.h));
        if (fabs(s.tn - s.tstop) <= troundoff) {
            get_dky<NS>(s, s.tstop, yout);
            s.tretlast = tret = s.tstop;
            s.tstopset = 0;
            return CV_TSTOP_RETURN;
        }
        if ((s.tn + s.hprime - s.tstop) * s.h > 0.0) {
            s.hprime = (s.tstop - s.tn) * (1.0 - 4.0 * UROUND);
            s.eta = s.hprime / s.h;
        }
    }
    s.tretlast = tret = s.tn;
#pragma unroll
    for (int i = 0; i < NS; i++) yout[i] = s.zn[0][i];
    return CV_SUCCESS;
}

}  // namespace bcm3hip
