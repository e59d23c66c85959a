/* ode_driver.h -- TEST INFRASTRUCTURE (oracle). See ode_driver.c. */
#ifndef BCM3_ORACLE_ODE_DRIVER_H
#define BCM3_ORACLE_ODE_DRIVER_H
#include "ode_backend.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct ode_solver ode_solver;
/* ODESolver::TDiscontinuityCallback: returns the next discontinuity time. */
typedef double (*ode_disc_cb)(double t, void* user);

ode_solver* ode_create(int N, orc_rhs_fn f, orc_jac_fn jac, void* user);
void ode_destroy(ode_solver* s);
void ode_set_tolerance(ode_solver* s, double rtol, double atol);
void ode_set_max_steps(ode_solver* s, int max_steps);
void ode_set_discontinuity(ode_solver* s, double time, ode_disc_cb cb, void* user);
double ode_get_current_y(ode_solver* s, int i);
void ode_set_current_y(ode_solver* s, int i, double v);
/* returns 1 on success, 0 on failure (ODESolver::SolveReturnSolution semantics) */
int ode_solve_return_solution(ode_solver* s, const double* y0, const double* times, int ntimes, double* out);
long ode_last_steps(ode_solver* s);
void ode_stats(ode_solver* s, long* out);

#ifdef __cplusplus
}
#endif
#endif
