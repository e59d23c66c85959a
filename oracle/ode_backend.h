/*
 * ode_backend.h -- TEST INFRASTRUCTURE (oracle). Never linked into the product.
 *
 * A minimal CVODE-shaped interface used by the oracle's ODE driver
 * (oracle/ode_driver.c, which restates src/odecommon/ODESolverCVODE.cpp) so the
 * same driver + PopPK glue can run on two backends:
 *   - backend_restated.c : plain-C restatement of SUNDIALS CVODE 5.3.0 BDF
 *                          (dependencies/cvode-5.3.0/src/cvode/cvode.c etc.)
 *   - backend_ref.c      : the vendored CVODE 5.3.0 compiled from
 *                          /root/reference sources (oracle/_ref, via Makefile)
 * Only dense systems with N <= 3 (the PopPK models) are supported.
 */
#ifndef BCM3_ORACLE_ODE_BACKEND_H
#define BCM3_ORACLE_ODE_BACKEND_H

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_NMAX 3

/* Return codes mirror CVODE's (cvode.h): CV_SUCCESS 0, CV_TSTOP_RETURN 1,
 * negative = failure. */
#define ORC_SUCCESS 0
#define ORC_TSTOP_RETURN 1

/* Right-hand side f(t, y) -> ydot. Return 0 on success (CVRhsFn). */
typedef int (*orc_rhs_fn)(double t, const double* y, double* ydot, void* user);
/* Jacobian; J is zeroed by the caller, row-major J[r*3 + c] (CVLsJacFn
 * semantics, cvode_ls.c:1237 SUNMatZero before the call). */
typedef int (*orc_jac_fn)(double t, const double* y, const double* fy, double* J, void* user);

/* Solver statistics accumulated over all CVodeReInit segments of one solve.
 * Index order of orc_stats[]: */
enum { ORC_ST_NST = 0, ORC_ST_NFE, ORC_ST_NNI, ORC_ST_NSETUPS, ORC_ST_NJE, ORC_ST_NETF,
       ORC_ST_NCFN, ORC_ST_NREINIT, ORC_ST_COUNT };

void* be_create(int N, orc_rhs_fn f, orc_jac_fn jac, void* user);
void  be_destroy(void* be);
int   be_sv_tolerances(void* be, double rtol, const double* atol);
int   be_reinit(void* be, double t0, const double* y0);
int   be_set_stop_time(void* be, double tstop);
int   be_step(void* be, double tout, double* yout, double* tret);      /* CVode(..., CV_ONE_STEP) */
int   be_get_dky(void* be, double t, double* dky);                      /* CVodeGetDky(t, k=0) */
void  be_stats_reset(void* be);
void  be_stats(void* be, long* out /* [ORC_ST_COUNT] */);

#ifdef __cplusplus
}
#endif
#endif
