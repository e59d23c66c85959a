/*
 * ode_driver.c -- TEST INFRASTRUCTURE (oracle). Never linked into the product.
 *
 * Restates ODESolver::SolveReturnSolution (src/odecommon/ODESolver.cpp:93-134) and the
 * ONE_STEP loop of ODESolverCVODE::Solve (src/odecommon/ODESolverCVODE.cpp:322-463),
 * including the discontinuity (dosing) callback protocol of ODESolver::SetDiscontinuity
 * (ODESolver.cpp:62-72), on top of an ode_backend (restated or real CVODE).
 */
#include "ode_driver.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>

struct ode_solver {
    int N;
    void* be;
    double rtol, atol;
    int max_steps;
    double next_discontinuity_time;
    ode_disc_cb disc_cb;
    void* disc_user;
    double y[ORC_NMAX];
    long last_steps;
};

ode_solver* ode_create(int N, orc_rhs_fn f, orc_jac_fn jac, void* user)
{
    ode_solver* s = (ode_solver*)calloc(1, sizeof(ode_solver));
    s->N = N;
    s->be = be_create(N, f, jac, user);
    s->max_steps = 2000; /* ODESolverCVODE ctor, ODESolverCVODE.cpp:45 */
    s->next_discontinuity_time = NAN;
    return s;
}

void ode_destroy(ode_solver* s)
{
    if (!s) return;
    be_destroy(s->be);
    free(s);
}

void ode_set_tolerance(ode_solver* s, double rtol, double atol)
{
    s->rtol = rtol;
    s->atol = atol;
}

void ode_set_max_steps(ode_solver* s, int max_steps) { s->max_steps = max_steps; }

/* ODESolver::SetDiscontinuity (ODESolver.cpp:62-72) */
void ode_set_discontinuity(ode_solver* s, double time, ode_disc_cb cb, void* user)
{
    if (time <= 0.0) return; /* "ignoring" warning in the reference */
    s->next_discontinuity_time = time;
    s->disc_cb = cb;
    s->disc_user = user;
}

double ode_get_current_y(ode_solver* s, int i) { return s->y[i]; }
void ode_set_current_y(ode_solver* s, int i, double v) { s->y[i] = v; }
long ode_last_steps(ode_solver* s) { return s->last_steps; }
void ode_stats(ode_solver* s, long* out) { be_stats(s->be, out); }

int ode_solve_return_solution(ode_solver* s, const double* y0, const double* times, int ntimes,
                              double* out /* [N][ntimes] */)
{
    int N = s->N;
    be_stats_reset(s->be);
    s->last_steps = 0;
    if (ntimes <= 0) return 0;
    int ti = 0;
    while (times[ti] < DBL_EPSILON) {
        for (int i = 0; i < N; i++) out[i * ntimes + ti] = y0[i];
        ti++;
        if (ti == ntimes) return 1;
    }
    double end_time = times[ntimes - 1];

    /* ODESolverCVODE::Solve */
    double atol[ORC_NMAX];
    for (int i = 0; i < N; i++) {
        s->y[i] = y0[i];
        atol[i] = s->atol;
    }
    be_sv_tolerances(s->be, s->rtol, atol);
    be_reinit(s->be, 0.0, s->y);
    if (!isnan(s->next_discontinuity_time)) be_set_stop_time(s->be, s->next_discontinuity_time);

    long current_step = 0;
    double t = 0.0;
    int tpi = ti;
    double tmp[ORC_NMAX];
    for (;;) {
        double tret = 0.0;
        int result = be_step(s->be, end_time, s->y, &tret);
        if (result < 0) {
            if (tpi < ntimes)
                for (int i = 0; i < N; i++) out[i * ntimes + tpi] = NAN;
            s->last_steps = current_step;
            return 0;
        }
        t = tret;
        current_step++;
        /* passed output times: interpolate back (ODESolverCVODE.cpp:406-427) */
        while (tpi < ntimes && tret >= times[tpi]) {
            if (be_get_dky(s->be, times[tpi], tmp) != 0) {
                s->last_steps = current_step;
                return 0;
            }
            for (int i = 0; i < N; i++) out[i * ntimes + tpi] = tmp[i];
            tpi++;
        }
        if (t >= end_time) break;
        if (current_step == s->max_steps) {
            s->last_steps = current_step;
            return 0;
        }
        if (!isnan(s->next_discontinuity_time) &&
            (result == ORC_TSTOP_RETURN || s->next_discontinuity_time == t)) {
            s->next_discontinuity_time = s->disc_cb(t, s->disc_user);
            if (!isnan(s->next_discontinuity_time) && s->next_discontinuity_time < INFINITY) {
                be_reinit(s->be, t, s->y);
                be_set_stop_time(s->be, s->next_discontinuity_time);
            } else {
                be_reinit(s->be, t, s->y);
            }
        }
    }
    s->last_steps = current_step;
    return 1;
}
