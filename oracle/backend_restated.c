/*
 * backend_restated.c -- TEST INFRASTRUCTURE (oracle). Never linked into the product.
 *
 * Plain-C restatement of the SUNDIALS CVODE 5.3.0 variable-order BDF integrator as
 * BCM3 configures it (dense Eigen N_Vector/SUNMatrix, closed-form 2x2/3x3 inverse
 * linear solver, Newton with maxiters 3, user Jacobian, no root finding, no
 * constraints, no projection, hmin = hmax_inv = 0), restricted to N <= 3.
 * Every function cites the reference code it restates. Paths are relative to
 * /root/reference/dependencies/cvode-5.3.0/src unless stated otherwise.
 *
 * Vector operations follow the dispatch of N_VLinearSum_Eigen
 * (src/odecommon/nvector_serial_eigen.cpp:301-331) at each call site so the
 * rounding of every operation matches the reference's formula.
 */
#include "ode_backend.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* cvode.c:145-172 */
#define FUZZ_FACTOR 100.0
#define HLB_FACTOR 100.0
#define HUB_FACTOR 0.1
#define H_BIAS 0.5
#define MAX_ITERS 4
#define CORTES 0.1
#define THRESH 1.5
#define ETAMX1 10000.0
#define ETAMX2 10.0
#define ETAMX3 10.0
#define ETAMXF 0.2
#define ETAMIN 0.1
#define ETACF 0.25
#define ADDON 0.000001
#define BIAS1 6.0
#define BIAS2 6.0
#define BIAS3 10.0
#define ONEPSM 1.000001
#define SMALL_NST 10
#define MXNCF 10
#define MXNEF 7
#define MXNEF1 3
#define SMALL_NEF 2
#define LONG_WAIT 10
#define DGMAX 0.3
#define MSBP 20
/* cvode_nls.c:29-31 */
#define NLS_MAXCOR 3
#define CRDOWN 0.3
#define RDIV 2.0
/* cvode_ls_impl.h:40-41 */
#define CVLS_MSBJ 50
#define CVLS_DGMAX 0.2

#define QMAX 5 /* BDF_Q_MAX */
#define SUNMAX(A, B) ((A) > (B) ? (A) : (B))
#define SUNMIN(A, B) ((A) < (B) ? (A) : (B))

/* internal flags (cvode_impl.h) */
enum { DO_ERROR_TEST = 2, PREDICT_AGAIN = 3, TRY_AGAIN = 5, FIRST_CALL = 6, PREV_CONV_FAIL = 7,
       PREV_ERR_FAIL = 8 };
enum { NLS_SUCCESS = 0, NLS_CONTINUE = 901, NLS_CONV_RECVR = 902 };
enum { CV_NO_FAILURES = 0, CV_FAIL_BAD_J = 1, CV_FAIL_OTHER = 2 };
enum { CV_TOO_MUCH_ACC = -2, CV_ERR_FAILURE = -3, CV_CONV_FAILURE = -4, CV_ILL_INPUT = -22,
       CV_TOO_CLOSE = -27, CV_BAD_T = -26 };

typedef struct {
    int N;
    orc_rhs_fn f;
    orc_jac_fn jac;
    void* user;
    double rtol, atol[ORC_NMAX];
    double uround;

    double zn[QMAX + 1][ORC_NMAX];
    double ewt[ORC_NMAX], y[ORC_NMAX], acor[ORC_NMAX], tempv[ORC_NMAX], ftemp[ORC_NMAX];
    double delta[ORC_NMAX];

    double savedJ[9], A[9], inv[9];
    long nje, nstlj;
    int cv_jcur;  /* cv_mem->cv_jcur */
    int nls_jcur; /* NEWTON_CONTENT(NLS)->jcur */
    int convfail;

    int q, qprime, next_q, qwait, L, qu, indx_acor;
    double h, hprime, next_h, eta, hscale, tn, tretlast, hu, h0u;
    double tau[QMAX + 2], tq[6], l[QMAX + 1];
    double rl1, gamma, gammap, gamrat, crate, delp, acnrm;
    double etaqm1, etaq, etaqp1, etamax, saved_tq5, tolsf;
    long nst, nfe, ncfn, netf, nni, nsetups, nstlp, nscon, nhnil;
    double tstop;
    int tstopset;

    long acc[ORC_ST_COUNT];
} rmem;

/* ---- small vector helpers (N_Vector ops of nvector_serial_eigen.cpp) ---- */

/* N_VWrmsNorm_Eigen: SUNRsqrt(sum((x*w)^2)/N)  (nvector_serial_eigen.cpp:386-396) */
static double wrms(const rmem* m, const double* x, const double* w)
{
    double s = 0.0;
    for (int i = 0; i < m->N; i++) {
        double p = x[i] * w[i];
        s += p * p;
    }
    s = s / m->N;
    return (s <= 0.0) ? 0.0 : sqrt(s); /* SUNRsqrt, sundials_math.c */
}

/* cvEwtSetSV (cvode.c): tempv = |y|; tempv = rtol*tempv + atol (VLin1); w = 1/tempv */
static int ewt_set(rmem* m, const double* ycur, double* weight)
{
    double t[ORC_NMAX];
    for (int i = 0; i < m->N; i++) t[i] = m->rtol * fabs(ycur[i]) + m->atol[i];
    /* atolmin0 is false for atol > 0 (CVodeSVtolerances) so no N_VMin check */
    for (int i = 0; i < m->N; i++) weight[i] = 1.0 / t[i];
    return 0;
}

/* ---- linear solver: sunlinsol_dense_eigen.cpp:111-178 (closed form inverse) ---- */
static void ls_inverse(rmem* m)
{
    const double* a = m->A;
    double* r = m->inv;
    if (m->N == 2) {
        /* SUNLinSolSetup_Dense_Eigen2x2 (:111-128) */
        double invdet = 1.0 / (a[0] * a[3] - a[1] * a[2]);
        r[0] = a[3] * invdet;
        r[1] = -a[1] * invdet;
        r[2] = -a[2] * invdet;
        r[3] = a[0] * invdet;
    } else {
        /* Eigen::internal::compute_inverse<.,.,3> (eigen-3.4-rc1 Eigen/src/LU/InverseImpl.h):
         * cofactor(i,j) = m(i1,j1)*m(i2,j2) - m(i1,j2)*m(i2,j1), i1=(i+1)%3 ...;
         * det = sum_i cof(i,0)*m(i,0); result(r,c) = cof(c,r)/det. */
#define M3(i, j) a[(i) * 3 + (j)]
#define COF(i, j) (M3(((i) + 1) % 3, ((j) + 1) % 3) * M3(((i) + 2) % 3, ((j) + 2) % 3) - \
                   M3(((i) + 1) % 3, ((j) + 2) % 3) * M3(((i) + 2) % 3, ((j) + 1) % 3))
        double c0 = COF(0, 0), c1 = COF(1, 0), c2 = COF(2, 0);
        double det = c0 * M3(0, 0) + c1 * M3(1, 0) + c2 * M3(2, 0);
        double invdet = 1.0 / det;
        r[0] = c0 * invdet;
        r[1] = c1 * invdet;
        r[2] = c2 * invdet;
        r[3] = COF(0, 1) * invdet;
        r[4] = COF(1, 1) * invdet;
        r[5] = COF(2, 1) * invdet;
        r[6] = COF(0, 2) * invdet;
        r[7] = COF(1, 2) * invdet;
        r[8] = COF(2, 2) * invdet;
#undef COF
#undef M3
    }
}

/* cvLsSetup (cvode_ls.c:1415-1500) + cvLsLinSys (:1201-1282) + SUNLinSolSetup. */
static int ls_setup(rmem* m, int convfail)
{
    int N = m->N;
    double dgamma = fabs((m->gamma / m->gammap) - 1.0);
    int jbad = (m->nst == 0) || (m->nst > m->nstlj + CVLS_MSBJ) ||
               ((convfail == CV_FAIL_BAD_J) && (dgamma < CVLS_DGMAX)) || (convfail == CV_FAIL_OTHER);
    if (!jbad) {
        m->cv_jcur = 0;
        memcpy(m->A, m->savedJ, sizeof(m->A));
    } else {
        m->cv_jcur = 1;
        memset(m->A, 0, sizeof(m->A));
        double J[9] = {0};
        if (m->jac(m->tn, m->y, m->ftemp, J, m->user) != 0) return -1;
        for (int r = 0; r < N; r++)
            for (int c = 0; c < N; c++) m->A[r * N + c] = J[r * 3 + c];
        memcpy(m->savedJ, m->A, sizeof(m->A));
    }
    /* SUNMatScaleAddI_DenseEigen: A *= c; diag += 1 (sunmatrix_dense_eigen.cpp:128-133) */
    for (int i = 0; i < N * N; i++) m->A[i] *= -m->gamma;
    for (int i = 0; i < N; i++) m->A[i * N + i] += 1.0;
    if (m->cv_jcur) {
        m->nje++;
        m->nstlj = m->nst;
    }
    ls_inverse(m);
    return 0;
}

/* cvLsSolve (cvode_ls.c:1509-1663) with SUNLinSolSolve_Dense_Eigen{2x2,3x3}: the 2x2 form is the
 * reference's own two-term sum (sunlinsol_dense_eigen.cpp:157-167); the 3x3 form is Eigen's
 * Matrix3d * VectorXd product (:169-176), whose coefficient-based row sum is Eigen's unrolled
 * reduction p0 + (p1 + p2) (redux_novec_unroller halves the range) -- checked bit for bit against
 * the vendored Eigen in _ref/libbcm3ref_nofma.so (oracle/eigen_ls.cpp, tests/test_oracle.py) */
static int ls_solve(rmem* m, double* b)
{
    int N = m->N;
    double x[ORC_NMAX];
    for (int i = 0; i < N; i++) {
        double s = 0.0;
        if (N == 3) {
            s = m->inv[i * N] * b[0] + (m->inv[i * N + 1] * b[1] + m->inv[i * N + 2] * b[2]);
        } else {
            for (int j = 0; j < N; j++) {
                if (j == 0)
                    s = m->inv[i * N + j] * b[j];
                else
                    s = s + m->inv[i * N + j] * b[j];
            }
        }
        x[i] = s;
    }
    for (int i = 0; i < N; i++) b[i] = x[i];
    if (m->gamrat != 1.0) {
        double c = 2.0 / (1.0 + m->gamrat);
        for (int i = 0; i < N; i++) b[i] *= c;
    }
    return 0;
}

/* cvNlsLSetup (cvode_nls.c) */
static int nls_lsetup(rmem* m, int jbad)
{
    if (jbad) m->convfail = CV_FAIL_BAD_J;
    int retval = ls_setup(m, m->convfail);
    m->nsetups++;
    m->nls_jcur = m->cv_jcur;
    m->gamrat = 1.0;
    m->gammap = m->gamma;
    m->crate = 1.0;
    m->nstlp = m->nst;
    if (retval < 0) return -1;
    return NLS_SUCCESS;
}

/* cvNlsResidual (cvode_nls.c): y = zn0 + ycor; ftemp = f(tn,y);
 * res = rl1*zn1 + ycor (VLin1); res += -gamma*ftemp (axpy) */
static int nls_residual(rmem* m, const double* ycor, double* res)
{
    int N = m->N;
    for (int i = 0; i < N; i++) m->y[i] = m->zn[0][i] + ycor[i];
    int r = m->f(m->tn, m->y, m->ftemp, m->user);
    m->nfe++;
    if (r != 0) return -1;
    for (int i = 0; i < N; i++) res[i] = m->rl1 * m->zn[1][i] + ycor[i];
    for (int i = 0; i < N; i++) res[i] += (-m->gamma) * m->ftemp[i];
    return 0;
}

/* cvNlsConvTest (cvode_nls.c:236-280) */
static int nls_conv_test(rmem* m, int curiter, const double* ycor, const double* del_v, double tol)
{
    double del = wrms(m, del_v, m->ewt);
    if (curiter > 0) m->crate = SUNMAX(CRDOWN * m->crate, del / m->delp);
    double dcon = del * SUNMIN(1.0, m->crate) / tol;
    if (dcon <= 1.0) {
        m->acnrm = (curiter == 0) ? del : wrms(m, ycor, m->ewt);
        return NLS_SUCCESS;
    }
    if ((curiter >= 1) && (del > RDIV * m->delp)) return NLS_CONV_RECVR;
    m->delp = del;
    return NLS_CONTINUE;
}

/* SUNNonlinSolSolve_Newton (sunnonlinsol/newton/sunnonlinsol_newton.c:183-322) */
static int newton_solve(rmem* m, double tol, int callLSetup)
{
    int N = m->N;
    int jbad = 0, retval;
    double* ycor = m->acor;
    double* delta = m->delta;
    for (;;) {
        retval = nls_residual(m, ycor, delta);
        if (retval != 0) break;
        if (callLSetup) {
            retval = nls_lsetup(m, jbad);
            if (retval != NLS_SUCCESS) break;
        }
        int curiter = 0;
        for (;;) {
            m->nni++;
            for (int i = 0; i < N; i++) delta[i] = -delta[i];
            retval = ls_solve(m, delta);
            if (retval != 0) break;
            for (int i = 0; i < N; i++) ycor[i] += delta[i];
            retval = nls_conv_test(m, curiter, ycor, delta, tol);
            if (retval == NLS_SUCCESS) {
                m->nls_jcur = 0;
                return NLS_SUCCESS;
            }
            if (retval != NLS_CONTINUE) break;
            curiter++;
            if (curiter >= NLS_MAXCOR) {
                retval = NLS_CONV_RECVR;
                break;
            }
            retval = nls_residual(m, ycor, delta);
            if (retval != 0) break;
        }
        if ((retval > 0) && !m->nls_jcur) {
            callLSetup = 1;
            jbad = 1;
            for (int i = 0; i < N; i++) ycor[i] = 0.0;
            continue;
        }
        break;
    }
    return retval;
}

/* cvNls (cvode.c:2701-2770) */
static int cv_nls(rmem* m, int nflag)
{
    m->convfail = ((nflag == FIRST_CALL) || (nflag == PREV_ERR_FAIL)) ? CV_NO_FAILURES : CV_FAIL_OTHER;
    int callSetup = (nflag == PREV_CONV_FAIL) || (nflag == PREV_ERR_FAIL) || (m->nst == 0) ||
                    (m->nst >= m->nstlp + MSBP) || (fabs(m->gamrat - 1.0) > DGMAX);
    for (int i = 0; i < m->N; i++) m->acor[i] = 0.0;
    int flag = newton_solve(m, m->tq[4], callSetup);
    if (flag != NLS_SUCCESS) return flag;
    for (int i = 0; i < m->N; i++) m->y[i] = m->zn[0][i] + m->acor[i];
    /* acnrmcur is TRUE after the first converged Newton solve (cvode_nls.c:266) */
    m->cv_jcur = 0;
    return 0;
}

/* cvRescale (cvode.c:2393-2406) */
static void cv_rescale(rmem* m)
{
    double c = m->eta;
    for (int j = 1; j <= m->q; j++) {
        for (int i = 0; i < m->N; i++) m->zn[j][i] *= c;
        c = m->eta * c;
    }
    m->h = m->hscale * m->eta;
    m->next_h = m->h;
    m->hscale = m->h;
    m->nscon = 0;
}

/* cvPredict (cvode.c:2412-2424), BCM variant with N_VAdd: zn[j-1] += zn[j] */
static void cv_predict(rmem* m)
{
    m->tn += m->h;
    if (m->tstopset) {
        if ((m->tn - m->tstop) * m->h > 0.0) m->tn = m->tstop;
    }
    for (int k = 1; k <= m->q; k++)
        for (int j = m->q; j >= k; j--)
            for (int i = 0; i < m->N; i++) m->zn[j - 1][i] += m->zn[j][i];
}

/* cvRestore (cvode.c): zn[j-1] += (-1)*zn[j] */
static void cv_restore(rmem* m, double saved_t)
{
    m->tn = saved_t;
    for (int k = 1; k <= m->q; k++)
        for (int j = m->q; j >= k; j--)
            for (int i = 0; i < m->N; i++) m->zn[j - 1][i] += (-1.0) * m->zn[j][i];
}

/* cvSetTqBDF (cvode.c:2660-2690) */
static void cv_set_tq_bdf(rmem* m, double hsum, double alpha0, double alpha0_hat, double xi_inv,
                          double xistar_inv)
{
    int q = m->q;
    double A1 = 1.0 - alpha0_hat + alpha0;
    double A2 = 1.0 + q * A1;
    m->tq[2] = fabs(A1 / (alpha0 * A2));
    m->tq[5] = fabs(A2 * xistar_inv / (m->l[q] * xi_inv));
    if (m->qwait == 1) {
        if (q > 1) {
            double C = xistar_inv / m->l[q];
            double A3 = alpha0 + 1.0 / q;
            double A4 = alpha0_hat + xi_inv;
            double Cpinv = (1.0 - A4 + A3) / A3;
            m->tq[1] = fabs(C * Cpinv);
        } else {
            m->tq[1] = 1.0;
        }
        hsum += m->tau[q];
        xi_inv = m->h / hsum;
        double A5 = alpha0 - (1.0 / (q + 1));
        double A6 = alpha0_hat - xi_inv;
        double Cppinv = (1.0 - A6 + A5) / A2;
        m->tq[3] = fabs(Cppinv / (xi_inv * (q + 2) * A5));
    }
    m->tq[4] = CORTES / m->tq[2];
}

/* cvSetBDF (cvode.c:2611-2650) + cvSet (cvode.c:2445-2460) */
static void cv_set(rmem* m)
{
    int q = m->q;
    double alpha0, alpha0_hat, xi_inv, xistar_inv, hsum;
    m->l[0] = m->l[1] = xi_inv = xistar_inv = 1.0;
    for (int i = 2; i <= q; i++) m->l[i] = 0.0;
    alpha0 = alpha0_hat = -1.0;
    hsum = m->h;
    if (q > 1) {
        for (int j = 2; j < q; j++) {
            hsum += m->tau[j - 1];
            xi_inv = m->h / hsum;
            alpha0 -= 1.0 / j;
            for (int i = j; i >= 1; i--) m->l[i] += m->l[i - 1] * xi_inv;
        }
        alpha0 -= 1.0 / q;
        xistar_inv = -m->l[1] - alpha0;
        hsum += m->tau[q - 1];
        xi_inv = m->h / hsum;
        alpha0_hat = -m->l[1] - xi_inv;
        for (int i = q; i >= 1; i--) m->l[i] += m->l[i - 1] * xistar_inv;
    }
    cv_set_tq_bdf(m, hsum, alpha0, alpha0_hat, xi_inv, xistar_inv);

    m->rl1 = 1.0 / m->l[1];
    m->gamma = m->h * m->rl1;
    if (m->nst == 0) m->gammap = m->gamma;
    m->gamrat = (m->nst > 0) ? m->gamma / m->gammap : 1.0;
}

/* cvIncreaseBDF (cvode.c:2310-2340) */
static void cv_increase_bdf(rmem* m)
{
    double alpha0, alpha1, prod, xi, xiold, hsum, A1;
    for (int i = 0; i <= QMAX; i++) m->l[i] = 0.0;
    m->l[2] = alpha1 = prod = xiold = 1.0;
    alpha0 = -1.0;
    hsum = m->hscale;
    if (m->q > 1) {
        for (int j = 1; j < m->q; j++) {
            hsum += m->tau[j + 1];
            xi = hsum / m->hscale;
            prod *= xi;
            alpha0 -= 1.0 / (j + 1);
            alpha1 += 1.0 / xi;
            for (int i = j + 2; i >= 2; i--) m->l[i] = m->l[i] * xiold + m->l[i - 1];
            xiold = xi;
        }
    }
    A1 = (-alpha0 - alpha1) / prod;
    /* N_VScale(A1, zn[indx_acor], zn[L]) */
    for (int i = 0; i < m->N; i++) m->zn[m->L][i] = A1 * m->zn[m->indx_acor][i];
    if (m->q > 1)
        for (int j = 2; j <= m->q; j++)
            for (int i = 0; i < m->N; i++) m->zn[j][i] += m->l[j] * m->zn[m->L][i];
}

/* cvDecreaseBDF (cvode.c:2352-2375) */
static void cv_decrease_bdf(rmem* m)
{
    double hsum, xi;
    for (int i = 0; i <= QMAX; i++) m->l[i] = 0.0;
    m->l[2] = 1.0;
    hsum = 0.0;
    for (int j = 1; j <= m->q - 2; j++) {
        hsum += m->tau[j];
        xi = hsum / m->hscale;
        for (int i = j + 2; i >= 2; i--) m->l[i] = m->l[i] * xi + m->l[i - 1];
    }
    if (m->q > 2)
        for (int j = 2; j < m->q; j++)
            for (int i = 0; i < m->N; i++) m->zn[j][i] += (-m->l[j]) * m->zn[m->q][i];
}

/* cvAdjustOrder (cvode.c:2212-2225) */
static void cv_adjust_order(rmem* m, int deltaq)
{
    if ((m->q == 2) && (deltaq != 1)) return;
    if (deltaq == 1)
        cv_increase_bdf(m);
    else if (deltaq == -1)
        cv_decrease_bdf(m);
}

/* cvAdjustParams (cvode.c:2189-2198) */
static void cv_adjust_params(rmem* m)
{
    if (m->qprime != m->q) {
        cv_adjust_order(m, m->qprime - m->q);
        m->q = m->qprime;
        m->L = m->q + 1;
        m->qwait = m->L;
    }
    cv_rescale(m);
}

/* cvHandleNFlag (cvode.c:2905-2945) */
static int cv_handle_nflag(rmem* m, int* nflagPtr, double saved_t, int* ncfPtr)
{
    int nflag = *nflagPtr;
    if (nflag == NLS_SUCCESS) return DO_ERROR_TEST;
    m->ncfn++;
    cv_restore(m, saved_t);
    if (nflag < 0) return -6; /* unrecoverable (RHS / setup failure) */
    (*ncfPtr)++;
    m->etamax = 1.0;
    if ((fabs(m->h) <= 0.0 * ONEPSM) || (*ncfPtr == MXNCF)) return CV_CONV_FAILURE;
    m->eta = SUNMAX(ETACF, 0.0 / fabs(m->h)); /* hmin = 0 */
    *nflagPtr = PREV_CONV_FAIL;
    cv_rescale(m);
    return PREDICT_AGAIN;
}

/* SUNRpowerR (sundials_math.c:40-52) */
static double powR(double base, double e) { return (base <= 0.0) ? 0.0 : pow(base, e); }
/* SUNRpowerI (sundials_math.c:28-38) */
static double powI(double base, int e)
{
    double prod = 1.0;
    int ex = abs(e);
    for (int i = 1; i <= ex; i++) prod *= base;
    if (e < 0) prod = 1.0 / prod;
    return prod;
}

/* cvDoErrorTest (cvode.c:2958-3030) */
static int cv_do_error_test(rmem* m, int* nflagPtr, double saved_t, int* nefPtr, double* dsmPtr)
{
    double dsm = m->acnrm * m->tq[2];
    *dsmPtr = dsm;
    if (dsm <= 1.0) return 0;
    (*nefPtr)++;
    m->netf++;
    *nflagPtr = PREV_ERR_FAIL;
    cv_restore(m, saved_t);
    if ((fabs(m->h) <= 0.0 * ONEPSM) || (*nefPtr == MXNEF)) return CV_ERR_FAILURE;
    m->etamax = 1.0;
    if (*nefPtr <= MXNEF1) {
        m->eta = 1.0 / (powR(BIAS2 * dsm, 1.0 / m->L) + ADDON);
        m->eta = SUNMAX(ETAMIN, SUNMAX(m->eta, 0.0 / fabs(m->h)));
        if (*nefPtr >= SMALL_NEF) m->eta = SUNMIN(m->eta, ETAMXF);
        cv_rescale(m);
        return TRY_AGAIN;
    }
    if (m->q > 1) {
        m->eta = SUNMAX(ETAMIN, 0.0 / fabs(m->h));
        cv_adjust_order(m, -1);
        m->L = m->q;
        m->q--;
        m->qwait = m->L;
        cv_rescale(m);
        return TRY_AGAIN;
    }
    m->eta = SUNMAX(ETAMIN, 0.0 / fabs(m->h));
    m->h *= m->eta;
    m->next_h = m->h;
    m->hscale = m->h;
    m->qwait = LONG_WAIT;
    m->nscon = 0;
    if (m->f(m->tn, m->zn[0], m->tempv, m->user) != 0) return -8;
    m->nfe++;
    for (int i = 0; i < m->N; i++) m->zn[1][i] = m->h * m->tempv[i];
    return TRY_AGAIN;
}

/* cvCompleteStep (cvode.c:3043-3080) */
static void cv_complete_step(rmem* m)
{
    m->nst++;
    m->nscon++;
    m->hu = m->h;
    m->qu = m->q;
    for (int i = m->q; i >= 2; i--) m->tau[i] = m->tau[i - 1];
    if ((m->q == 1) && (m->nst > 1)) m->tau[2] = m->tau[1];
    m->tau[1] = m->h;
    for (int j = 0; j <= m->q; j++)
        for (int i = 0; i < m->N; i++) m->zn[j][i] += m->l[j] * m->acor[i];
    m->qwait--;
    if ((m->qwait == 1) && (m->q != QMAX)) {
        for (int i = 0; i < m->N; i++) m->zn[QMAX][i] = m->acor[i];
        m->saved_tq5 = m->tq[5];
        m->indx_acor = QMAX;
    }
}

/* cvSetEta (cvode.c:3125-3142); hmax_inv = 0 so the hmax division is by 1 */
static void cv_set_eta(rmem* m)
{
    if (m->eta < THRESH) {
        m->eta = 1.0;
        m->hprime = m->h;
    } else {
        m->eta = SUNMIN(m->eta, m->etamax);
        m->eta /= SUNMAX(1.0, fabs(m->h) * 0.0 * m->eta);
        m->hprime = m->h * m->eta;
        if (m->qprime < m->q) m->nscon = 0;
    }
}

/* cvComputeEtaqm1 / cvComputeEtaqp1 / cvChooseEta (cvode.c:3150-3258) */
static double cv_compute_etaqm1(rmem* m)
{
    m->etaqm1 = 0.0;
    if (m->q > 1) {
        double ddn = wrms(m, m->zn[m->q], m->ewt) * m->tq[1];
        m->etaqm1 = 1.0 / (powR(BIAS1 * ddn, 1.0 / m->q) + ADDON);
    }
    return m->etaqm1;
}

static double cv_compute_etaqp1(rmem* m)
{
    m->etaqp1 = 0.0;
    if (m->q != QMAX) {
        if (m->saved_tq5 == 0.0) return m->etaqp1;
        double cquot = (m->tq[5] / m->saved_tq5) * powI(m->h / m->tau[2], m->L);
        for (int i = 0; i < m->N; i++) m->tempv[i] = (-cquot) * m->zn[QMAX][i] + m->acor[i];
        double dup = wrms(m, m->tempv, m->ewt) * m->tq[3];
        m->etaqp1 = 1.0 / (powR(BIAS3 * dup, 1.0 / (m->L + 1)) + ADDON);
    }
    return m->etaqp1;
}

static void cv_choose_eta(rmem* m)
{
    double etam = SUNMAX(m->etaqm1, SUNMAX(m->etaq, m->etaqp1));
    if (etam < THRESH) {
        m->eta = 1.0;
        m->qprime = m->q;
        return;
    }
    if (etam == m->etaq) {
        m->eta = m->etaq;
        m->qprime = m->q;
    } else if (etam == m->etaqm1) {
        m->eta = m->etaqm1;
        m->qprime = m->q - 1;
    } else {
        m->eta = m->etaqp1;
        m->qprime = m->q + 1;
        for (int i = 0; i < m->N; i++) m->zn[QMAX][i] = m->acor[i];
    }
}

/* cvPrepareNextStep (cvode.c:3093-3120) */
static void cv_prepare_next_step(rmem* m, double dsm)
{
    if (m->etamax == 1.0) {
        m->qwait = SUNMAX(m->qwait, 2);
        m->qprime = m->q;
        m->hprime = m->h;
        m->eta = 1.0;
        return;
    }
    m->etaq = 1.0 / (powR(BIAS2 * dsm, 1.0 / m->L) + ADDON);
    if (m->qwait != 0) {
        m->eta = m->etaq;
        m->qprime = m->q;
        cv_set_eta(m);
        return;
    }
    m->qwait = 2;
    m->etaqm1 = cv_compute_etaqm1(m);
    m->etaqp1 = cv_compute_etaqp1(m);
    cv_choose_eta(m);
    cv_set_eta(m);
}

/* cvStep (cvode.c:2082-2174) */
static int cv_step(rmem* m)
{
    double saved_t = m->tn, dsm = 0.0;
    int ncf = 0, nef = 0, nflag = FIRST_CALL, kflag, eflag;
    if ((m->nst > 0) && (m->hprime != m->h)) cv_adjust_params(m);
    for (;;) {
        cv_predict(m);
        cv_set(m);
        nflag = cv_nls(m, nflag);
        kflag = cv_handle_nflag(m, &nflag, saved_t, &ncf);
        if (kflag == PREDICT_AGAIN) continue;
        if (kflag != DO_ERROR_TEST) return kflag;
        eflag = cv_do_error_test(m, &nflag, saved_t, &nef, &dsm);
        if (eflag == TRY_AGAIN) continue;
        if (eflag != 0) return eflag;
        break;
    }
    cv_complete_step(m);
    cv_prepare_next_step(m, dsm);
    m->etamax = (m->nst <= SMALL_NST) ? ETAMX2 : ETAMX3;
    for (int i = 0; i < m->N; i++) m->acor[i] *= m->tq[2];
    return 0;
}

/* cvYddNorm (cvode.c:2046-2066) */
static int cv_ydd_norm(rmem* m, double hg, double* yddnrm)
{
    for (int i = 0; i < m->N; i++) m->y[i] = hg * m->zn[1][i] + m->zn[0][i];
    if (m->f(m->tn + hg, m->y, m->tempv, m->user) != 0) return -1;
    m->nfe++;
    /* N_VLinearSum(1/hg, tempv, -1/hg, zn1, tempv): a == -b -> VScaleDiff: z = a*(x - y) */
    double a = 1.0 / hg;
    for (int i = 0; i < m->N; i++) m->tempv[i] = a * (m->tempv[i] - m->zn[1][i]);
    *yddnrm = wrms(m, m->tempv, m->ewt);
    return 0;
}

/* cvUpperBoundH0 (cvode.c:2000-2035) */
static double cv_upper_bound_h0(rmem* m, double tdist)
{
    double temp1[ORC_NMAX], temp2[ORC_NMAX];
    for (int i = 0; i < m->N; i++) temp2[i] = fabs(m->zn[0][i]);
    ewt_set(m, m->zn[0], temp1);
    for (int i = 0; i < m->N; i++) temp1[i] = 1.0 / temp1[i];
    for (int i = 0; i < m->N; i++) temp1[i] += HUB_FACTOR * temp2[i];
    for (int i = 0; i < m->N; i++) temp2[i] = fabs(m->zn[1][i]);
    for (int i = 0; i < m->N; i++) temp1[i] = temp2[i] / temp1[i];
    double hub_inv = temp1[0]; /* N_VMaxNorm_Eigen = maxCoeff (nvector_serial_eigen.cpp:381-384) */
    for (int i = 1; i < m->N; i++)
        if (temp1[i] > hub_inv) hub_inv = temp1[i];
    double hub = HUB_FACTOR * tdist;
    if (hub * hub_inv > 1.0) hub = 1.0 / hub_inv;
    return hub;
}

/* cvHin (cvode.c:1884-1990) */
static int cv_hin(rmem* m, double tout)
{
    double tdiff = tout - m->tn;
    if (tdiff == 0.0) return CV_TOO_CLOSE;
    int sign = (tdiff > 0.0) ? 1 : -1;
    double tdist = fabs(tdiff);
    double tround = m->uround * SUNMAX(fabs(m->tn), fabs(tout));
    if (tdist < 2.0 * tround) return CV_TOO_CLOSE;
    double hlb = HLB_FACTOR * tround;
    double hub = cv_upper_bound_h0(m, tdist);
    double hg = (hlb * hub <= 0.0) ? 0.0 : sqrt(hlb * hub);
    if (hub < hlb) {
        m->h = (sign == -1) ? -hg : hg;
        return 0;
    }
    double hs = hg, hnew = hg, yddnrm = 0.0;
    for (int count1 = 1; count1 <= MAX_ITERS; count1++) {
        int hgOK = 0;
        for (int count2 = 1; count2 <= MAX_ITERS; count2++) {
            double hgs = hg * sign;
            if (cv_ydd_norm(m, hgs, &yddnrm) != 0) return -8;
            hgOK = 1;
            break;
        }
        if (!hgOK) {
            if (count1 <= 2) return -10;
            hnew = hs;
            break;
        }
        hs = hg;
        if (yddnrm * hub * hub > 2.0) {
            double v = 2.0 / yddnrm;
            hnew = (v <= 0.0) ? 0.0 : sqrt(v);
        } else {
            double v = hg * hub;
            hnew = (v <= 0.0) ? 0.0 : sqrt(v);
        }
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
    m->h = h0;
    return 0;
}

/* ---------------- public backend API ---------------- */

void* be_create(int N, orc_rhs_fn f, orc_jac_fn jac, void* user)
{
    rmem* m = (rmem*)calloc(1, sizeof(rmem));
    m->N = N;
    m->f = f;
    m->jac = jac;
    m->user = user;
    m->uround = DBL_EPSILON; /* UNIT_ROUNDOFF */
    m->etamax = ETAMX1;
    return m;
}

void be_destroy(void* be) { free(be); }

int be_sv_tolerances(void* be, double rtol, const double* atol)
{
    rmem* m = (rmem*)be;
    m->rtol = rtol;
    for (int i = 0; i < m->N; i++) m->atol[i] = atol[i];
    return 0;
}

static void acc_flush(rmem* m)
{
    m->acc[ORC_ST_NST] += m->nst;
    m->acc[ORC_ST_NFE] += m->nfe;
    m->acc[ORC_ST_NNI] += m->nni;
    m->acc[ORC_ST_NSETUPS] += m->nsetups;
    m->acc[ORC_ST_NJE] += m->nje;
    m->acc[ORC_ST_NETF] += m->netf;
    m->acc[ORC_ST_NCFN] += m->ncfn;
}

/* CVodeReInit (cvode.c:586-683). tau, saved_tq5, indx_acor, tstop persist. */
int be_reinit(void* be, double t0, const double* y0)
{
    rmem* m = (rmem*)be;
    acc_flush(m);
    m->acc[ORC_ST_NREINIT]++;
    m->tn = t0;
    m->q = 1;
    m->L = 2;
    m->qwait = m->L;
    m->etamax = ETAMX1;
    m->qu = 0;
    m->hu = 0.0;
    m->tolsf = 1.0;
    for (int i = 0; i < m->N; i++) m->zn[0][i] = y0[i];
    m->nst = m->nfe = m->ncfn = m->netf = m->nni = m->nsetups = m->nhnil = m->nstlp = m->nscon = 0;
    m->nje = 0; /* flushed above; cvLsInitializeCounters resets it at the next nst==0 step */
    m->h0u = 0.0;
    m->next_h = 0.0;
    m->next_q = 0;
    return 0;
}

int be_set_stop_time(void* be, double tstop)
{
    rmem* m = (rmem*)be;
    if (m->nst > 0 && (tstop - m->tn) * m->h < 0.0) return CV_ILL_INPUT;
    m->tstop = tstop;
    m->tstopset = 1;
    return 0;
}

/* CVodeGetDky(t, k=0) (cvode.c:1467-1533) */
int be_get_dky(void* be, double t, double* dky)
{
    rmem* m = (rmem*)be;
    double tfuzz = FUZZ_FACTOR * m->uround * (fabs(m->tn) + fabs(m->hu));
    if (m->hu < 0.0) tfuzz = -tfuzz;
    double tp = m->tn - m->hu - tfuzz;
    double tn1 = m->tn + tfuzz;
    if ((t - tp) * (t - tn1) > 0.0) return CV_BAD_T;
    double s = (t - m->tn) / m->h;
    int q = m->q;
    /* cvals[nvec] = s^j (repeated multiplication), vectors zn[q], zn[q-1], ..., zn[0] */
    if (q == 1) {
        /* nvec == 2 -> N_VLinearSum(s, zn1, 1, zn0, dky) -> VLin1: s*zn1 + zn0 */
        for (int i = 0; i < m->N; i++) dky[i] = s * m->zn[1][i] + m->zn[0][i];
        return 0;
    }
    double c = 1.0;
    for (int i = 0; i < q; i++) c *= s;
    for (int i = 0; i < m->N; i++) dky[i] = c * m->zn[q][i];
    for (int j = q - 1; j >= 0; j--) {
        c = 1.0;
        for (int i = 0; i < j; i++) c *= s;
        for (int i = 0; i < m->N; i++) dky[i] += c * m->zn[j][i];
    }
    return 0;
}

/* CVode(..., CV_ONE_STEP) (cvode.c:1006-1443) */
int be_step(void* be, double tout, double* yout, double* tret)
{
    rmem* m = (rmem*)be;
    int N = m->N;
    if (m->nst == 0) {
        m->tretlast = *tret = m->tn;
        /* cvInitialSetup: ewt, linit (cvLsInitializeCounters), NLS init (jcur = FALSE) */
        ewt_set(m, m->zn[0], m->ewt);
        m->nje = 0;
        m->nstlj = 0;
        m->nls_jcur = 0;
        if (m->f(m->tn, m->zn[0], m->zn[1], m->user) != 0) return -8;
        m->nfe++;
        if (m->tstopset) {
            if ((m->tstop - m->tn) * (tout - m->tn) <= 0.0) return CV_ILL_INPUT;
        }
        m->h = 0.0; /* hin */
        double tout_hin = tout;
        if (m->tstopset && (tout - m->tn) * (tout - m->tstop) > 0.0) tout_hin = m->tstop;
        int hflag = cv_hin(m, tout_hin);
        if (hflag != 0) return hflag;
        /* hmax_inv = 0, hmin = 0: no clamping */
        if (m->tstopset) {
            if ((m->tn + m->h - m->tstop) * m->h > 0.0) m->h = (m->tstop - m->tn) * (1.0 - 4.0 * m->uround);
        }
        m->hscale = m->h;
        m->h0u = m->h;
        m->hprime = m->h;
        for (int i = 0; i < N; i++) m->zn[1][i] *= m->h;
    }
    if (m->nst > 0) {
        double troundoff = FUZZ_FACTOR * m->uround * (fabs(m->tn) + fabs(m->h));
        if (fabs(m->tn - m->tretlast) > troundoff) {
            m->tretlast = *tret = m->tn;
            for (int i = 0; i < N; i++) yout[i] = m->zn[0][i];
            return 0;
        }
        if (m->tstopset) {
            if (fabs(m->tn - m->tstop) <= troundoff) {
                if (be_get_dky(m, m->tstop, yout) != 0) return CV_ILL_INPUT;
                m->tretlast = *tret = m->tstop;
                m->tstopset = 0;
                return ORC_TSTOP_RETURN;
            }
            if ((m->tn + m->hprime - m->tstop) * m->h > 0.0) {
                m->hprime = (m->tstop - m->tn) * (1.0 - 4.0 * m->uround);
                m->eta = m->hprime / m->h;
            }
        }
    }
    /* one pass of the internal step loop */
    m->next_h = m->h;
    m->next_q = m->q;
    if (m->nst > 0) ewt_set(m, m->zn[0], m->ewt);
    double nrm = wrms(m, m->zn[0], m->ewt);
    m->tolsf = m->uround * nrm;
    if (m->tolsf > 1.0) {
        m->tretlast = *tret = m->tn;
        for (int i = 0; i < N; i++) yout[i] = m->zn[0][i];
        m->tolsf *= 2.0;
        return CV_TOO_MUCH_ACC;
    }
    m->tolsf = 1.0;
    if (m->tn + m->h == m->tn) m->nhnil++;
    int kflag = cv_step(m);
    if (kflag != 0) {
        m->tretlast = *tret = m->tn;
        for (int i = 0; i < N; i++) yout[i] = m->zn[0][i];
        return kflag;
    }
    if (m->tstopset) {
        double troundoff = FUZZ_FACTOR * m->uround * (fabs(m->tn) + fabs(m->h));
        if (fabs(m->tn - m->tstop) <= troundoff) {
            be_get_dky(m, m->tstop, yout);
            m->tretlast = *tret = m->tstop;
            m->tstopset = 0;
            return ORC_TSTOP_RETURN;
        }
        if ((m->tn + m->hprime - m->tstop) * m->h > 0.0) {
            m->hprime = (m->tstop - m->tn) * (1.0 - 4.0 * m->uround);
            m->eta = m->hprime / m->h;
        }
    }
    m->tretlast = *tret = m->tn;
    for (int i = 0; i < N; i++) yout[i] = m->zn[0][i];
    m->next_q = m->qprime;
    m->next_h = m->hprime;
    return 0;
}

void be_stats_reset(void* be)
{
    rmem* m = (rmem*)be;
    memset(m->acc, 0, sizeof(m->acc));
    m->nst = m->nfe = m->ncfn = m->netf = m->nni = m->nsetups = m->nje = 0;
}

void be_stats(void* be, long* out)
{
    rmem* m = (rmem*)be;
    for (int i = 0; i < ORC_ST_COUNT; i++) out[i] = m->acc[i];
    out[ORC_ST_NST] += m->nst;
    out[ORC_ST_NFE] += m->nfe;
    out[ORC_ST_NNI] += m->nni;
    out[ORC_ST_NSETUPS] += m->nsetups;
    out[ORC_ST_NJE] += m->nje;
    out[ORC_ST_NETF] += m->netf;
    out[ORC_ST_NCFN] += m->ncfn;
}
