/*
 * backend_ref.c -- TEST INFRASTRUCTURE (oracle). Never linked into the product.
 *
 * ode_backend on top of the *vendored* SUNDIALS CVODE 5.3.0 (BCM-modified, with N_VAdd in
 * cvPredict) compiled directly from /root/reference/dependencies/cvode-5.3.0 by
 * oracle/Makefile into oracle/_ref/. Mirrors the setup of ODESolverCVODE::Initialize
 * (src/odecommon/ODESolverCVODE.cpp:81-135): BDF, Newton NLS, user Jacobian, dense matrix.
 *
 * BCM's Eigen N_Vector / SUNMatrix adapters (src/odecommon/*_eigen.cpp) cannot be built
 * here (they include src/utils/Utils.h -> Boost, absent). Substitutes:
 *   - N_Vector: vendored nvector_serial (BCM-patched, has nvadd) with fused ops enabled, which
 *     implements the same elementwise formulas as nvector_serial_eigen.cpp;
 *   - SUNMatrix: vendored sunmatrix_dense;
 *   - SUNLinearSolver: a custom SUNLinearSolver with sunlinsol_dense_eigen.cpp:111-178's
 *     closed-form 2x2 inverse (the reference's own five statements) and, for N = 3, Eigen's
 *     compute_inverse<MatrixXd, Matrix3d, 3> and Matrix3d * VectorXd product evaluated by the
 *     vendored Eigen itself (oracle/eigen_ls.cpp, when built with ORACLE_EIGEN_LS -- the _ref
 *     builds are); the cofactor restatement below otherwise.
 */
#include <cvode/cvode.h>
#include <nvector/nvector_serial.h>
#include <sundials/sundials_linearsolver.h>
#include <sundials/sundials_math.h>
#include <sunmatrix/sunmatrix_dense.h>
#include <sunnonlinsol/sunnonlinsol_newton.h>

#include <stdlib.h>
#include <string.h>

#include "ode_backend.h"

/* ---------------- closed-form inverse linear solver ---------------- */
typedef struct {
    int N;
    double inv[9];
} inv_content;

static SUNLinearSolver_Type ls_gettype(SUNLinearSolver S) { (void)S; return SUNLINEARSOLVER_DIRECT; }
static SUNLinearSolver_ID ls_getid(SUNLinearSolver S) { (void)S; return SUNLINEARSOLVER_CUSTOM; }
static int ls_initialize(SUNLinearSolver S) { (void)S; return SUNLS_SUCCESS; }

#ifdef ORACLE_EIGEN_LS
void eigenref_inverse3(const double* a, double* inv);
void eigenref_solve3(const double* inv, const double* b, double* x);
#endif

static int ls_setup(SUNLinearSolver S, SUNMatrix A)
{
    inv_content* c = (inv_content*)S->content;
    double* r = c->inv;
#ifdef ORACLE_EIGEN_LS
    if (c->N == 3) {
        eigenref_inverse3(SM_DATA_D(A), r);
        return SUNLS_SUCCESS;
    }
#endif
#define AE(i, j) SM_ELEMENT_D(A, i, j)
    if (c->N == 2) {
        double invdet = 1.0 / (AE(0, 0) * AE(1, 1) - AE(0, 1) * AE(1, 0));
        r[0] = AE(1, 1) * invdet;
        r[1] = -AE(0, 1) * invdet;
        r[2] = -AE(1, 0) * invdet;
        r[3] = AE(0, 0) * invdet;
    } else {
#define COF(i, j) (AE(((i) + 1) % 3, ((j) + 1) % 3) * AE(((i) + 2) % 3, ((j) + 2) % 3) - \
                   AE(((i) + 1) % 3, ((j) + 2) % 3) * AE(((i) + 2) % 3, ((j) + 1) % 3))
        double c0 = COF(0, 0), c1 = COF(1, 0), c2 = COF(2, 0);
        double det = c0 * AE(0, 0) + c1 * AE(1, 0) + c2 * AE(2, 0);
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
    }
#undef AE
    return SUNLS_SUCCESS;
}

static int ls_solve(SUNLinearSolver S, SUNMatrix A, N_Vector x, N_Vector b, realtype tol)
{
    (void)A;
    (void)tol;
    inv_content* c = (inv_content*)S->content;
    int N = c->N;
    double* bd = NV_DATA_S(b);
    double* xd = NV_DATA_S(x);
#ifdef ORACLE_EIGEN_LS
    if (N == 3) {
        eigenref_solve3(c->inv, bd, xd);
        return SUNLS_SUCCESS;
    }
#endif
    for (int i = 0; i < N; i++) {
        double s = c->inv[i * N] * bd[0];
        for (int j = 1; j < N; j++) s = s + c->inv[i * N + j] * bd[j];
        xd[i] = s;
    }
    return SUNLS_SUCCESS;
}

static sunindextype ls_lastflag(SUNLinearSolver S) { (void)S; return SUNLS_SUCCESS; }
static int ls_free(SUNLinearSolver S)
{
    if (!S) return SUNLS_SUCCESS;
    free(S->content);
    S->content = NULL;
    SUNLinSolFreeEmpty(S);
    return SUNLS_SUCCESS;
}

static SUNLinearSolver make_inverse_ls(int N)
{
    SUNLinearSolver S = SUNLinSolNewEmpty();
    S->ops->gettype = ls_gettype;
    S->ops->getid = ls_getid;
    S->ops->initialize = ls_initialize;
    S->ops->setup = ls_setup;
    S->ops->solve = ls_solve;
    S->ops->lastflag = ls_lastflag;
    S->ops->free = ls_free;
    inv_content* c = (inv_content*)calloc(1, sizeof(inv_content));
    c->N = N;
    S->content = c;
    return S;
}

/* ---------------- backend ---------------- */
typedef struct {
    int N;
    orc_rhs_fn f;
    orc_jac_fn jac;
    void* user;
    void* cvode_mem;
    N_Vector y, tmp;
    SUNMatrix J;
    SUNLinearSolver LS;
    SUNNonlinearSolver NLS;
    long acc[ORC_ST_COUNT];
    int skip_flush;
} refmem;

static int rhs_tramp(realtype t, N_Vector y, N_Vector ydot, void* ud)
{
    refmem* m = (refmem*)ud;
    return m->f(t, NV_DATA_S(y), NV_DATA_S(ydot), m->user);
}

static int jac_tramp(realtype t, N_Vector y, N_Vector fy, SUNMatrix Jm, void* ud, N_Vector t1, N_Vector t2,
                     N_Vector t3)
{
    (void)t1;
    (void)t2;
    (void)t3;
    refmem* m = (refmem*)ud;
    double J[9] = {0};
    int r = m->jac(t, NV_DATA_S(y), NV_DATA_S(fy), J, m->user);
    for (int i = 0; i < m->N; i++)
        for (int j = 0; j < m->N; j++)
            if (J[i * 3 + j] != 0.0) SM_ELEMENT_D(Jm, i, j) = J[i * 3 + j];
    return r;
}

static void silent_err(int error_code, const char* module, const char* function, char* msg, void* ud)
{
    (void)error_code;
    (void)module;
    (void)function;
    (void)msg;
    (void)ud;
}

void* be_create(int N, orc_rhs_fn f, orc_jac_fn jac, void* user)
{
    refmem* m = (refmem*)calloc(1, sizeof(refmem));
    m->N = N;
    m->f = f;
    m->jac = jac;
    m->user = user;
    m->y = N_VNew_Serial(N);
    m->tmp = N_VNew_Serial(N);
    N_VEnableFusedOps_Serial(m->y, SUNTRUE);
    N_VEnableFusedOps_Serial(m->tmp, SUNTRUE);
    for (int i = 0; i < N; i++) NV_Ith_S(m->y, i) = 0.0;
    m->cvode_mem = CVodeCreate(CV_BDF);
    m->J = SUNDenseMatrix(N, N);
    m->LS = make_inverse_ls(N);
    m->NLS = SUNNonlinSol_Newton(m->y);
    CVodeInit(m->cvode_mem, rhs_tramp, 0.0, m->y);
    CVodeSetUserData(m->cvode_mem, m);
    CVodeSetLinearSolver(m->cvode_mem, m->LS, m->J);
    CVodeSetNonlinearSolver(m->cvode_mem, m->NLS);
    CVodeSetJacFn(m->cvode_mem, jac_tramp);
    CVodeSetErrHandlerFn(m->cvode_mem, silent_err, NULL);
    return m;
}

void be_destroy(void* be)
{
    refmem* m = (refmem*)be;
    if (!m) return;
    CVodeFree(&m->cvode_mem);
    SUNNonlinSolFree(m->NLS);
    SUNLinSolFree(m->LS);
    SUNMatDestroy(m->J);
    N_VDestroy(m->y);
    N_VDestroy(m->tmp);
    free(m);
}

int be_sv_tolerances(void* be, double rtol, const double* atol)
{
    refmem* m = (refmem*)be;
    for (int i = 0; i < m->N; i++) NV_Ith_S(m->tmp, i) = atol[i];
    return CVodeSVtolerances(m->cvode_mem, rtol, m->tmp);
}

static void acc_flush(refmem* m)
{
    long v;
    CVodeGetNumSteps(m->cvode_mem, &v);
    m->acc[ORC_ST_NST] += v;
    CVodeGetNumRhsEvals(m->cvode_mem, &v);
    m->acc[ORC_ST_NFE] += v;
    CVodeGetNumNonlinSolvIters(m->cvode_mem, &v);
    m->acc[ORC_ST_NNI] += v;
    CVodeGetNumLinSolvSetups(m->cvode_mem, &v);
    m->acc[ORC_ST_NSETUPS] += v;
    CVodeGetNumJacEvals(m->cvode_mem, &v);
    m->acc[ORC_ST_NJE] += v;
    CVodeGetNumErrTestFails(m->cvode_mem, &v);
    m->acc[ORC_ST_NETF] += v;
    CVodeGetNumNonlinSolvConvFails(m->cvode_mem, &v);
    m->acc[ORC_ST_NCFN] += v;
}

static long nst_now(refmem* m)
{
    long v = 0;
    CVodeGetNumSteps(m->cvode_mem, &v);
    return v;
}

int be_reinit(void* be, double t0, const double* y0)
{
    refmem* m = (refmem*)be;
    /* the vendored CVodeGetNum* read counters that CVodeReInit zeroes; njes/nni are reset only at
       the next first step, so flush only when a step happened since the last re-init */
    if (!m->skip_flush && nst_now(m) > 0) acc_flush(m);
    m->skip_flush = 0;
    m->acc[ORC_ST_NREINIT]++;
    N_Vector v = N_VNew_Serial(m->N);
    for (int i = 0; i < m->N; i++) NV_Ith_S(v, i) = y0[i];
    int r = CVodeReInit(m->cvode_mem, t0, v);
    N_VDestroy(v);
    return r;
}

int be_set_stop_time(void* be, double tstop) { return CVodeSetStopTime(((refmem*)be)->cvode_mem, tstop); }

int be_step(void* be, double tout, double* yout, double* tret)
{
    refmem* m = (refmem*)be;
    for (int i = 0; i < m->N; i++) NV_Ith_S(m->y, i) = yout[i];
    int r = CVode(m->cvode_mem, tout, m->y, tret, CV_ONE_STEP);
    for (int i = 0; i < m->N; i++) yout[i] = NV_Ith_S(m->y, i);
    return r;
}

int be_get_dky(void* be, double t, double* dky)
{
    refmem* m = (refmem*)be;
    int r = CVodeGetDky(m->cvode_mem, t, 0, m->tmp);
    for (int i = 0; i < m->N; i++) dky[i] = NV_Ith_S(m->tmp, i);
    return r;
}

void be_stats_reset(void* be)
{
    refmem* m = (refmem*)be;
    memset(m->acc, 0, sizeof(m->acc));
    m->skip_flush = 1;
}

void be_stats(void* be, long* out)
{
    refmem* m = (refmem*)be;
    for (int i = 0; i < ORC_ST_COUNT; i++) out[i] = m->acc[i];
    if (nst_now(m) > 0) {
        long save[ORC_ST_COUNT];
        memcpy(save, m->acc, sizeof(save));
        acc_flush(m);
        for (int i = 0; i < ORC_ST_COUNT; i++) out[i] = m->acc[i];
        memcpy(m->acc, save, sizeof(save));
    }
}
