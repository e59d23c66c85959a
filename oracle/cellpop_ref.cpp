/*
 * cellpop_ref.cpp -- TEST INFRASTRUCTURE (oracle). Never linked into the product.
 *
 * One cell of the reference's cell-population likelihood on the reference's own integrator and
 * linear algebra, built by oracle/Makefile into oracle/_ref/libcellpopref.so from the sources
 * where they lie under /root/reference:
 *   - vendored SUNDIALS CVODE 5.3.0 (dependencies/cvode-5.3.0; BDF, Newton, dense matrix);
 *   - the reference's PartialPivLUExtended::compute_optimized (src/utils/
 *     EigenPartialPivLUSomewhatSparse.h) + Eigen 3.4-rc1's PartialPivLU::solve
 *     (dependencies/eigen-3.4-rc1) as the SUNLinearSolver, as src/odecommon/
 *     sunlinsol_dense_eigen.cpp:95-108, 146-156 uses them for N >= 4.
 * Restated here (their files need Boost): the difference-quotient Jacobian
 * (ODESolverCVODE::DifferenceQuotientJacobian, src/odecommon/ODESolverCVODE.cpp:496-537; cells
 * register no analytic Jacobian, Cell.cpp:57-76), the ONE_STEP driver of ODESolverCVODE::Solve
 * (:322-463) with SolveReturnSolution (ODESolver.cpp:93-134), Cell::Simulate (Cell.cpp:193-273)
 * and Cell::integration_step_cb (:463-538) with get_threshold_crossing_time (ODESolverCVODE.cpp:
 * 264-320) in the non-stored mode a cell population without synchronisation runs in, and the stored
 * mode of synchronised data (ODESolver::SolveStoreIntegrationPoints, ODESolver.cpp:136-150; the
 * CVodeTimepoint records of ODESolverCVODE::Solve, :375-401; GetInterpolatedY's iterator, :176-242;
 * the division / death interpolation of Cell.cpp:499-529 and the evaluation passes of
 * Experiment.cpp:265-292 with Cell::GetInterpolatedSpeciesValue, Cell.cpp:280-327).
 * solver_type="DP5": ODESolverDP5 (src/odecommon/ODESolverDP5.cpp, the reference's own explicit
 * Dormand-Prince 5(4) with Hairer's dense output; its source needs Boost through Utils.h, so it is
 * restated here statement for statement: ApplyRK :327-412, Solve :100-285).
 * N_Vector: the vendored nvector_serial stands in for nvector_serial_eigen.cpp (same formulas).
 * The cell right-hand side is the generated derivative (oracle/sbml_codegen.py) compiled for the
 * host and passed in as a function pointer.
 */
#include <cvode/cvode.h>
#include <cvode/cvode_ls.h>
#include <nvector/nvector_serial.h>
#include <sundials/sundials_linearsolver.h>
#include <sundials/sundials_math.h>
#include <sunmatrix/sunmatrix_dense.h>
#include <sunnonlinsol/sunnonlinsol_newton.h>

#include <Eigen/Dense>

#include "EigenPartialPivLUSomewhatSparse.h"

#include <cfloat>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "cvode_impl.h"

typedef void (*derivative_fn)(double* out, const double* species, const double* constant_species,
                              const double* parameters, const double* non_sampled_parameters);

extern "C" {
// one cell: inputs
typedef struct {
    int N;
    derivative_fn rhs;
    const double* constant_species;
    const double* parameters;
    const double* non_sampled_parameters;
    const double* y0;             // [N]
    double creation_time;
    double end_time;              // Experiment target time (experiment time)
    int M;                        // output times (sorted experiment times)
    const double* output_times;   // [M]
    const int* output_species;    // [M] species index whose value is reported (-1 = none)
    double rtol, atol, hmin, hmax;
    int max_steps;
    int divide_cells;
    double simulate_past_chromatid_separation_time;
    // event species: SIMULATED-species indices used on the ODE state (Cell.cpp:44-50); -1 = absent
    int ev_replicating, ev_replicated, ev_pcna, ev_nuclear_envelope, ev_chromatid_separation, ev_cytokinesis,
        ev_apoptosis;
    // treatment trajectories of type pulses (TreatmentTrajectoryPulses.cpp): constant species
    // treat_cs[i] follows the pulses treat_times[treat_off[i] .. treat_off[i+1]) (sorted)
    int n_constant;  // constant species (constant_species[n_constant])
    int n_treat;
    const int* treat_cs;
    const int* treat_off;
    const double* treat_times;
    // synchronised data: store the integration points (Cell::Initialize's calculate_synchronization_points)
    int stored;
    const int* output_sync;  // [M] ESynchronizeCellTrajectory of each output (4 = None)
    double sync_offset;      // Experiment's time_offset
    int solver;              // 0 CVODE, 1 DP5 (ODESolverDP5, restated below; no treatments, no stored mode)
} cp_cell_in;

typedef struct {
    int ok;              // Cell::Simulate result
    int divided, died;
    double sim_end;      // simulation_end_time (cell time)
    double achieved_time;
    double event_times[5];  // replication start, replication finish, PCNA increase, NEBD, anaphase onset
    long nsteps;
    long nsetups, nje, nni, netf, nfe;  // CVODE counters (CVodeGetNum*)
} cp_cell_out;
}

namespace {

struct LU {
    int N;
    PartialPivLUExtended<Eigen::MatrixXd> lu;
    Eigen::MatrixXd A;
};

SUNLinearSolver_Type ls_gettype(SUNLinearSolver) { return SUNLINEARSOLVER_DIRECT; }
SUNLinearSolver_ID ls_getid(SUNLinearSolver) { return SUNLINEARSOLVER_CUSTOM; }
int ls_initialize(SUNLinearSolver) { return SUNLS_SUCCESS; }
int ls_setup(SUNLinearSolver S, SUNMatrix A)
{
    LU* c = (LU*)S->content;
    c->A = Eigen::Map<Eigen::MatrixXd>(SM_DATA_D(A), c->N, c->N);
    c->lu.compute_optimized(c->A);
    return SUNLS_SUCCESS;
}
int ls_solve(SUNLinearSolver S, SUNMatrix, N_Vector x, N_Vector b, realtype)
{
    LU* c = (LU*)S->content;
    Eigen::Map<Eigen::VectorXd> xv(NV_DATA_S(x), c->N);
    Eigen::VectorXd bv = Eigen::Map<Eigen::VectorXd>(NV_DATA_S(b), c->N);
    xv.noalias() = c->lu.solve(bv);
    return SUNLS_SUCCESS;
}
sunindextype ls_lastflag(SUNLinearSolver) { return 0; }
int ls_free(SUNLinearSolver S)
{
    if (!S) return SUNLS_SUCCESS;
    delete (LU*)S->content;
    if (S->ops) free(S->ops);
    free(S);
    return SUNLS_SUCCESS;
}

SUNLinearSolver make_ls(int N)
{
    SUNLinearSolver S = SUNLinSolNewEmpty();
    S->ops->gettype = ls_gettype;
    S->ops->getid = ls_getid;
    S->ops->initialize = ls_initialize;
    S->ops->setup = ls_setup;
    S->ops->solve = ls_solve;
    S->ops->lastflag = ls_lastflag;
    S->ops->free = ls_free;
    LU* c = new LU;
    c->N = N;
    S->content = c;
    return S;
}

// one CVodeTimepoint (ODESolverCVODE.h): the step's return time, tn, h, hu, q and zn[0..q]
struct Record {
    double time, tn, h, hu;
    int q;
    std::vector<double> zn;  // [(q + 1) * N], zn[j * N + i]
};

// the interpolation iterator of ODESolverCVODE (RestartInterpolationIteration / GetInterpolatedY)
struct Interp {
    size_t iter = 0;
    double itime = std::numeric_limits<double>::quiet_NaN();
    std::vector<double> y;
    void restart(int N)
    {
        y.assign(N, 0.0);
        iter = 0;
        itime = std::numeric_limits<double>::quiet_NaN();
    }
    const std::vector<double>& get(const std::vector<Record>& recs, int N, double t)
    {
        if (t == itime) return y;
        while (iter < recs.size()) {
            if (recs[iter].time > t) break;
            iter++;
        }
        if (iter == recs.size()) {
            itime = std::numeric_limits<double>::quiet_NaN();
            y.assign(N, std::numeric_limits<double>::quiet_NaN());
            return y;
        }
        itime = t;
        const Record& r = recs[iter];
        double tfuzz = 100.0 * DBL_EPSILON * (fabs(r.tn) + fabs(r.hu));
        if (r.hu < 0.0) tfuzz = -tfuzz;
        const double tp = r.tn - r.hu - tfuzz;
        const double tn1 = r.tn + tfuzz;
        if ((t - tp) * (t - tn1) > 0.0) {
            y.assign(N, std::numeric_limits<double>::quiet_NaN());
            return y;
        }
        const double s = (t - r.tn) / r.h;
        y.assign(N, 0.0);
        for (int j = r.q; j >= 0; j--) {
            double cval = 1.0;
            for (int i = 0; i < j; i++) cval *= s;
            for (int i = 0; i < N; i++) y[i] += cval * r.zn[(size_t)j * N + i];
        }
        return y;
    }
};

struct Cell {
    const cp_cell_in* in;
    int N;
    void* mem;
    std::vector<Record> recs;  // stored mode
    Interp interp;
    std::vector<double> end_y;  // stored mode: simulation_end_y at a division / death
    std::vector<double> y_copy, work;
    std::vector<double> cs;  // constant_species_y with the treatment concentrations
    // Cell / ODESolver state
    double t;
    double previous_integration_step_time;
    double simulation_end_time;
    bool divided, died;
    double ev[5];
};

void silent_err(int, const char*, const char*, char*, void*) {}

// TreatmentTrajectoryPulses::GetConcentration / FirstDiscontinuity / NextDiscontinuity (:22-71)
double pulse_concentration(const double* tp, int n, double time, double creation_time)
{
    const double global_time = time + creation_time;
    for (int i = 0; i < n; i++) {
        const double t_in_pulse = global_time - tp[i] - 2.0;
        if (t_in_pulse >= 14.0) {
            continue;
        } else if (t_in_pulse <= 0.0) {
            return 0.0;
        } else if (t_in_pulse < 2.0) {
            return t_in_pulse * 0.5;
        } else if (t_in_pulse < 10.0) {
            return 1.0;
        } else {
            return 1 - (t_in_pulse - 10.0) * 0.25;
        }
    }
    return 0.0;
}
double pulse_first(const double* tp, int n, double creation_time)
{
    return n > 0 ? tp[0] - creation_time + 2.0 : std::numeric_limits<double>::quiet_NaN();
}
double pulse_next(const double* tp, int n, double time, double creation_time)
{
    for (int i = 0; i < n; i++) {
        if (time == tp[i] - creation_time + 2.0) {
            return tp[i] - creation_time + 4.0;
        } else if (time == tp[i] - creation_time + 4.0) {
            return tp[i] - creation_time + 10.0;
        } else if (time == tp[i] - creation_time + 10.0) {
            return tp[i] - creation_time + 14.0;
        } else if (time == tp[i] - creation_time + 14.0) {
            if (i < n - 1) return tp[i + 1] - creation_time + 2.0;
            return std::numeric_limits<double>::quiet_NaN();
        }
    }
    return std::numeric_limits<double>::quiet_NaN();
}

// Cell::SetTreatmentConcentration (Cell.cpp:414-420)
const double* constants_at(Cell* c, double t)
{
    const cp_cell_in* in = c->in;
    for (int i = 0; i < in->n_treat; i++)
        c->cs[in->treat_cs[i]] = pulse_concentration(in->treat_times + in->treat_off[i], in->treat_off[i + 1] - in->treat_off[i],
                                                     t, in->creation_time);
    return c->cs.data();
}

// Cell::solver_rhs_fn (Cell.cpp:422-432)
int rhs_fn(realtype t, N_Vector y, N_Vector ydot, void* user)
{
    Cell* c = (Cell*)user;
    c->in->rhs(NV_DATA_S(ydot), NV_DATA_S(y), constants_at(c, t), c->in->parameters, c->in->non_sampled_parameters);
    return 0;
}

// ODESolverCVODE::DifferenceQuotientJacobian (ODESolverCVODE.cpp:496-537)
int jac_fn(realtype t, N_Vector y, N_Vector fy, SUNMatrix J, void* user, N_Vector, N_Vector, N_Vector)
{
    Cell* c = (Cell*)user;
    CVodeMem cv_mem = (CVodeMem)c->mem;
    const int N = c->N;
    const double MIN_INC_MULT = 1000.0;
    double* yd = NV_DATA_S(y);
    double* fd = NV_DATA_S(fy);
    double* ewt = NV_DATA_S(cv_mem->cv_ewt);
    for (int i = 0; i < N; i++) c->y_copy[i] = yd[i];
    const double srur = SUNRsqrt(cv_mem->cv_uround);
    Eigen::Map<Eigen::VectorXd> ydot(fd, N), ewtv(ewt, N);
    const double fnorm = sqrt((ydot.array() * ewtv.array()).square().sum() / N);
    double minInc;
    if (fnorm != 0.0)
        minInc = (MIN_INC_MULT * fabs(cv_mem->cv_h) * cv_mem->cv_uround * N * fnorm);
    else
        minInc = 1.0;
    for (int j = 0; j < N; j++) {
        const double inc = std::max(srur * fabs(yd[j]), minInc / ewt[j]);
        c->y_copy[j] += inc;
        c->in->rhs(c->work.data(), c->y_copy.data(), constants_at(c, t), c->in->parameters,
                   c->in->non_sampled_parameters);
        c->y_copy[j] = yd[j];
        const double inc_inv = 1.0 / inc;
        double* col = SM_COLUMN_D(J, j);
        for (int i = 0; i < N; i++) col[i] = inc_inv * (c->work[i] - fd[i]);
    }
    return 0;
}

// get_threshold_crossing_time without stored integration points: the reference reads the
// default-constructed timepoint record (cv_q = 0, NaN times) and a zero-filled Nordsieck buffer,
// so the interpolant is 0 and the bisection only walks towards one end (ODESolverCVODE.cpp:264-320)
double threshold_crossing_time(const Cell* c, double threshold, bool above, double prev_time)
{
    double dt = (c->t - prev_time) * 0.5;
    double time = prev_time + dt;
    for (int iter = 0; iter < 10; iter++) {
        const double x = 0.0;
        dt *= 0.5;
        if (above) {
            if (x > threshold) time -= dt; else time += dt;
        } else {
            if (x < threshold) time -= dt; else time += dt;
        }
    }
    return time;
}

// get_threshold_crossing_time with stored integration points (ODESolverCVODE.cpp:264-320): ten
// bisection steps on the polynomial of the step just taken (the last record)
double threshold_crossing_time_stored(const Cell* c, int species, double threshold, bool above, double prev_time)
{
    const Record& r = c->recs.back();
    double dt = (c->t - prev_time) * 0.5;
    double time = prev_time + dt;
    for (int iter = 0; iter < 10; iter++) {
        const double s = (time - r.tn) / r.h;
        double x = 0.0;
        for (int j = r.q; j >= 0; j--) {
            double cval = 1.0;
            for (int i = 0; i < j; i++) cval *= s;
            x += cval * r.zn[(size_t)j * c->N + species];
        }
        dt *= 0.5;
        if (above) {
            if (x > threshold) time -= dt; else time += dt;
        } else {
            if (x < threshold) time -= dt; else time += dt;
        }
    }
    return time;
}

double crossing(Cell* c, int species, double threshold, bool above)
{
    if (c->in->solver == 1) return std::numeric_limits<double>::quiet_NaN();  // ODESolverDP5.cpp:322-327
    return c->in->stored ? threshold_crossing_time_stored(c, species, threshold, above, c->previous_integration_step_time)
                         : threshold_crossing_time(c, threshold, above, c->previous_integration_step_time);
}

// Cell::integration_step_cb (Cell.cpp:463-538)
bool step_cb(Cell* c, double t, const double* y, double& end_time)
{
    const cp_cell_in* in = c->in;
    bool cont = true;
    if (in->ev_replicating >= 0 && c->ev[0] != c->ev[0]) {
        if (y[in->ev_replicating] > 1e-4) c->ev[0] = crossing(c, in->ev_replicating, 1e-4, true);
    }
    if (in->ev_replicated >= 0 && c->ev[1] != c->ev[1]) {
        if (y[in->ev_replicated] > 1.95) c->ev[1] = crossing(c, in->ev_replicated, 1.95, true);
    }
    if (in->ev_pcna >= 0 && c->ev[2] != c->ev[2]) {
        if (y[in->ev_pcna] > 0.5) c->ev[2] = crossing(c, in->ev_pcna, 0.5, true);
    }
    if (in->ev_nuclear_envelope >= 0 && c->ev[3] != c->ev[3]) {
        if (y[in->ev_nuclear_envelope] < 0.5) c->ev[3] = crossing(c, in->ev_nuclear_envelope, 0.5, false);
    }
    if (in->ev_chromatid_separation >= 0 && c->ev[4] != c->ev[4]) {
        if (y[in->ev_chromatid_separation] > 1e-3) {
            c->ev[4] = crossing(c, in->ev_chromatid_separation, 1e-3, true);
            c->simulation_end_time = std::max(c->simulation_end_time, c->ev[4] + in->simulate_past_chromatid_separation_time);
            end_time = c->simulation_end_time;
        }
    }
    if (in->divide_cells && in->ev_cytokinesis >= 0) {
        if (y[in->ev_cytokinesis] > 1.0) {
            if (in->stored) {
                const double division_time = crossing(c, in->ev_cytokinesis, 1.0, true);
                c->simulation_end_time = division_time;
                c->end_y = c->interp.get(c->recs, c->N, division_time);
            } else {
                c->simulation_end_time = t;
                c->end_y.assign(y, y + c->N);  // the "temporary hack" branch's simulation_end_y
            }
            c->divided = true;
            cont = false;
        }
    }
    if (in->ev_apoptosis >= 0) {
        if (y[in->ev_apoptosis] > 1.0) {
            if (in->stored) {
                const double death_time = crossing(c, in->ev_apoptosis, 1.0, true);
                c->simulation_end_time = death_time;
                c->end_y = c->interp.get(c->recs, c->N, death_time);
            } else {
                c->simulation_end_time = t;
                c->end_y.assign(y, y + c->N);
            }
            c->died = true;
            cont = false;
        }
    }
    c->previous_integration_step_time = t;
    return cont;
}

// ODESolverDP5::ApplyRK (ODESolverDP5.cpp:327-412)
struct Dp5State {
    int N;
    std::vector<double> yn, ytmp, k[7];
};

double dp5_apply_rk(Cell* c, Dp5State& d, double t, double cur_dt)
{
    const int N = d.N;
    const cp_cell_in* in = c->in;
    auto f = [&](double tt, const std::vector<double>& y, std::vector<double>& out) {
        in->rhs(out.data(), y.data(), constants_at(c, tt), in->parameters, in->non_sampled_parameters);
    };
    std::vector<double>&yn = d.yn, &ytmp = d.ytmp;
    std::vector<double>* k = d.k;
    for (int i = 0; i < N; i++) ytmp[i] = yn[i] + cur_dt * 0.2 * k[0][i];
    f(t + 0.2 * cur_dt, ytmp, k[1]);
    for (int i = 0; i < N; i++) ytmp[i] = yn[i] + cur_dt * (+0.075 * k[0][i] + 0.225 * k[1][i]);
    f(t + 0.3 * cur_dt, ytmp, k[2]);
    for (int i = 0; i < N; i++)
        ytmp[i] = yn[i] + cur_dt * (+0.97777777777777777777777777777778 * k[0][i] - 3.7333333333333333333333333333333 * k[1][i] +
                                    3.5555555555555555555555555555556 * k[2][i]);
    f(t + 0.8 * cur_dt, ytmp, k[3]);
    for (int i = 0; i < N; i++)
        ytmp[i] = yn[i] + cur_dt * (+2.9525986892242036274958085657674 * k[0][i] - 11.595793324188385916780978509374 * k[1][i] +
                                    9.8228928516994360615759792714525 * k[2][i] - 0.29080932784636488340192043895748 * k[3][i]);
    f(t + 0.88888888888888888888888888888889 * cur_dt, ytmp, k[4]);
    for (int i = 0; i < N; i++)
        ytmp[i] = yn[i] + cur_dt * (+2.8462752525252525252525252525253 * k[0][i] - 10.757575757575757575757575757576 * k[1][i] +
                                    8.9064227177434724604535925290642 * k[2][i] + 0.27840909090909090909090909090909 * k[3][i] -
                                    0.27353130360205831903945111492281 * k[4][i]);
    f(t + cur_dt, ytmp, k[5]);
    for (int i = 0; i < N; i++)
        ytmp[i] = yn[i] + cur_dt * (+0.09114583333333333333333333333333 * k[0][i] + 0.44923629829290206648697214734951 * k[2][i] +
                                    0.65104166666666666666666666666667 * k[3][i] - 0.32237617924528301886792452830189 * k[4][i] +
                                    0.13095238095238095238095238095238 * k[5][i]);
    f(t + cur_dt, ytmp, k[6]);
    double maxdiff = -std::numeric_limits<double>::infinity();
    for (int i = 0; i < N; i++) {
        double error = cur_dt * (+0.00123263888888888888888888888889 * k[0][i] - 0.00425277029050613956274333632824 * k[2][i] +
                                 0.03697916666666666666666666666667 * k[3][i] - 0.05086379716981132075471698113208 * k[4][i] +
                                 0.04190476190476190476190476190476 * k[5][i] - 0.025 * k[6][i]);
        error = fabs(error);
        const double D = in->atol + in->rtol * fabs(ytmp[i] + k[6][i] * cur_dt);
        const double diff = error / D;
        maxdiff = (std::max)(maxdiff, diff);
    }
    return maxdiff;
}

// ODESolverDP5::Solve with do_interpolation (SolveReturnSolution, ODESolver.cpp:93-134) and
// Cell::integration_step_cb, whose result DP5 ignores; sol[(ti) * N + i] the interpolated outputs
bool dp5_solve(Cell* c, const std::vector<double>& tp, int ti0, std::vector<double>& sol, long& steps_out)
{
    const cp_cell_in* in = c->in;
    const int N = c->N, M = (int)tp.size();
    for (auto& v : sol) v = std::numeric_limits<double>::quiet_NaN();  // interpolated_output->setConstant(NaN)
    double end_time = tp[M - 1];
    Dp5State d;
    d.N = N;
    d.yn.assign(in->y0, in->y0 + N);
    d.ytmp.assign(N, 0.0);
    for (auto& k : d.k) k.assign(N, 0.0);
    double t = 0.0;
    double dt = std::min(in->hmax, 1.0);
    in->rhs(d.k[0].data(), d.yn.data(), constants_at(c, t), in->parameters, in->non_sampled_parameters);
    unsigned int steps = 0;
    size_t ti = ti0;
    const double min_dt = in->hmin, max_dt = in->hmax;
    while (1) {
        double cur_dt = dt, next_dt = dt;
        bool succeeded = false;
        for (int i = 0; i < 10; i++) {
            double maxdiff = dp5_apply_rk(c, d, t, cur_dt);
            if (std::isnan(maxdiff) || maxdiff == -std::numeric_limits<double>::infinity()) {
                steps_out = steps;
                return false;
            }
            if (maxdiff > 1.1) {
                if (cur_dt == min_dt) {
                    break;
                } else {
                    double scale = 0.9 * pow(maxdiff, -0.2);
                    scale = std::max(0.2, scale);
                    cur_dt *= scale;
                    if (cur_dt < min_dt) cur_dt = min_dt;
                }
            } else if (maxdiff < 0.5) {
                maxdiff = std::max(maxdiff, 1e-5);
                double scale = 0.9 * pow(maxdiff, -0.2);
                scale = std::min(5.0, scale);
                next_dt = cur_dt * scale;
                if (next_dt > max_dt) next_dt = max_dt;
                succeeded = true;
                break;
            } else {
                next_dt = cur_dt;
                succeeded = true;
                break;
            }
        }
        if (!succeeded) {
            steps_out = steps;
            return false;
        }
        const double target_t = t + cur_dt;
        while (target_t >= tp[ti]) {
            const double theta = (tp[ti] - t) / cur_dt;
            if (theta >= 1.0) {
                for (int i = 0; i < N; i++) sol[ti * N + i] = d.ytmp[i];
            } else {
                const double thetaSq = theta * theta;
                const double b1 = theta * (1.0 + theta * (-2.7854166666666669 + theta * (2.8861111111111111 + theta * (-1.0095486111111112))));
                const double b3 = 33.33333333333333 * thetaSq * (0.11363881401617251 + theta * (-0.1682659478885894 + theta * 0.068104222821203958));
                const double b4 = -2.5 * thetaSq * (0.675 + theta * (-1.8 + theta * (0.8645833333333333)));
                const double b5 = 21.491745283018869 * thetaSq * (-0.012 + theta * (0.058666666666666666 + theta * (-0.06166666666666666)));
                const double b6 = -3.1428571428571428 * thetaSq * (-0.3 + theta * (0.9666666666666666 + theta * (-0.7083333333333333)));
                for (int i = 0; i < N; i++)
                    sol[ti * N + i] = d.yn[i] + cur_dt * (b1 * d.k[0][i] + b3 * d.k[2][i] + b4 * d.k[3][i] + b5 * d.k[4][i] + b6 * d.k[5][i]);
            }
            ti++;
            if (ti == (size_t)M) break;
        }
        if (ti == (size_t)M) break;
        d.k[0] = d.k[6];
        d.yn = d.ytmp;
        t += cur_dt;
        steps++;
        c->t = t;
        step_cb(c, t, d.yn.data(), end_time);  // result ignored (ODESolverDP5.cpp:259-261)
        if (t >= end_time) break;
        if ((int)steps == in->max_steps) {
            steps_out = steps;
            return false;
        }
        dt = next_dt;
    }
    steps_out = steps;
    return true;
}

}  // namespace

extern "C" {

// Cell::Simulate with SolveReturnSolution; out_values[M] = the solution at each output time for
// output_species (NaN where the reference leaves it unset or GetInterpolatedSpeciesValue returns
// NaN: before creation, after the cell's simulation end); end_y[N] = simulation_end_y.
int cp_simulate_cell(const cp_cell_in* in, cp_cell_out* out, double* out_values, double* end_y)
{
    const int N = in->N, M = in->M;
    Cell c;
    c.in = in;
    c.N = N;
    c.y_copy.assign(N, 0.0);
    c.work.assign(N, 0.0);
    c.cs.assign(in->constant_species, in->constant_species + in->n_constant);
    c.divided = c.died = false;
    for (int k = 0; k < 5; k++) c.ev[k] = std::numeric_limits<double>::quiet_NaN();
    out->nsteps = 0;
    out->nsetups = out->nje = out->nni = out->netf = out->nfe = 0;
    for (int k = 0; k < M; k++) out_values[k] = std::numeric_limits<double>::quiet_NaN();

    // Cell::Simulate (Cell.cpp:193-210)
    c.previous_integration_step_time = 0;
    c.simulation_end_time = in->end_time - in->creation_time;
    std::vector<double> tp(M);
    for (int i = 0; i < M; i++) tp[i] = in->output_times[i] - in->creation_time;
    if (M > 0) c.simulation_end_time = std::max(c.simulation_end_time, tp[M - 1]);

    std::vector<double> sol((size_t)N * M, std::numeric_limits<double>::quiet_NaN());
    bool result = true;
    // SolveReturnSolution (ODESolver.cpp:93-134)
    int ti = 0;
    bool solve = true;
    if (in->stored) {
        // SolveStoreIntegrationPoints (ODESolver.cpp:136-141)
        if (c.simulation_end_time <= std::numeric_limits<double>::epsilon()) {
            solve = false;
            result = false;
        }
    } else {
        while (ti < M && tp[ti] < std::numeric_limits<double>::epsilon()) {
            for (int i = 0; i < N; i++) sol[(size_t)ti * N + i] = in->y0[i];
            ti++;
        }
        if (ti == M) solve = false;
    }
    long nst = 0;
    if (solve && in->solver == 1) {
        result = dp5_solve(&c, tp, ti, sol, nst);
        for (int i = 0; i < N; i++) end_y[i] = (c.divided || c.died) ? c.end_y[i] : sol[(size_t)(M - 1) * N + i];
    } else if (solve) {
        double end_time = in->stored ? c.simulation_end_time : tp[M - 1];
        c.interp.restart(N);
        N_Vector y = N_VNew_Serial(N), atol = N_VNew_Serial(N), tmp = N_VNew_Serial(N);
        for (int i = 0; i < N; i++) {
            NV_Ith_S(y, i) = in->y0[i];
            NV_Ith_S(atol, i) = in->atol;
        }
        void* mem = CVodeCreate(CV_BDF);
        c.mem = mem;
        SUNMatrix J = SUNDenseMatrix(N, N);
        SUNLinearSolver LS = make_ls(N);
        SUNNonlinearSolver NLS = SUNNonlinSol_Newton(y);
        CVodeInit(mem, rhs_fn, 0.0, y);
        CVodeSetUserData(mem, &c);
        CVodeSetLinearSolver(mem, LS, J);
        CVodeSetNonlinearSolver(mem, NLS);
        CVodeSetJacFn(mem, jac_fn);
        CVodeSetMinStep(mem, in->hmin);
        CVodeSetMaxStep(mem, in->hmax);
        CVodeSetErrHandlerFn(mem, silent_err, nullptr);
        CVodeSVtolerances(mem, in->rtol, atol);
        // Cell::Simulate: the first discontinuity of the treatment trajectories (Cell.cpp:212-229);
        // ODESolver::SetDiscontinuity ignores times <= 0 (a fresh solver: NaN)
        double next_disc = std::numeric_limits<double>::quiet_NaN();
        {
            double first = std::numeric_limits<double>::quiet_NaN();
            for (int i = 0; i < in->n_treat; i++) {
                const double* tpp = in->treat_times + in->treat_off[i];
                const int nt = in->treat_off[i + 1] - in->treat_off[i];
                double d = pulse_first(tpp, nt, in->creation_time);
                if (!std::isnan(d)) {
                    while (d < 0.0) d = pulse_next(tpp, nt, d, in->creation_time);
                }
                if (!(first < d)) first = d;  // Cell.cpp:222: a NaN replaces
            }
            if (!std::isnan(first) && first > 0.0) next_disc = first;
        }
        CVodeReInit(mem, 0.0, y);
        if (!std::isnan(next_disc)) CVodeSetStopTime(mem, next_disc);
        // ODESolverCVODE::Solve (:322-463)
        long current_step = 0;
        c.t = 0.0;
        int tpi = ti;
        while (1) {
            double tret;
            int r = CVode(mem, end_time, y, &tret, CV_ONE_STEP);
            if (r < 0) {
                result = false;
                break;
            }
            c.t = tret;
            if (in->stored) {
                if (current_step >= in->max_steps) {  // "CVODE integration timepoint storage buffer too small"
                    result = false;
                    break;
                }
                CVodeMem cvm = (CVodeMem)mem;
                Record r;
                r.time = c.t;
                r.tn = cvm->cv_tn;
                r.h = cvm->cv_h;
                r.hu = cvm->cv_hu;
                r.q = cvm->cv_q;
                r.zn.assign((size_t)(r.q + 1) * N, 0.0);
                for (int j = r.q; j >= 0; j--)
                    for (int i = 0; i < N; i++) r.zn[(size_t)j * N + i] = NV_Ith_S(cvm->cv_zn[j], i);
                c.recs.push_back(r);
            }
            current_step++;
            // the reference reads past the output vector once all outputs are done; stop there
            while (!in->stored && tpi < M && tret >= tp[tpi]) {
                if (CVodeGetDky(mem, tp[tpi], 0, tmp) != CV_SUCCESS) {
                    result = false;
                    break;
                }
                for (int i = 0; i < N; i++) sol[(size_t)tpi * N + i] = NV_Ith_S(tmp, i);
                tpi++;
            }
            if (!result) break;
            if (!step_cb(&c, c.t, NV_DATA_S(y), end_time)) break;
            if (c.t >= end_time) break;
            if (current_step == in->max_steps) {
                result = false;
                break;
            }
            // ODESolverCVODE::Solve :449-460 with Cell::discontinuity_cb (Cell.cpp:447-461)
            if (!std::isnan(next_disc) && (r == CV_TSTOP_RETURN || next_disc == c.t)) {
                double disc = std::numeric_limits<double>::infinity();
                for (int i = 0; i < in->n_treat; i++) {
                    const double d = pulse_next(in->treat_times + in->treat_off[i], in->treat_off[i + 1] - in->treat_off[i],
                                                c.t, in->creation_time);
                    if (d < disc) disc = d;
                }
                next_disc = (disc == std::numeric_limits<double>::infinity()) ? std::numeric_limits<double>::quiet_NaN()
                                                                               : disc;
                if (!std::isnan(next_disc) && next_disc < std::numeric_limits<double>::infinity()) {
                    CVodeReInit(mem, c.t, y);
                    CVodeSetStopTime(mem, next_disc);
                } else {
                    CVodeReInit(mem, c.t, y);
                }
            }
        }
        nst = current_step;
        CVodeGetNumLinSolvSetups(mem, &out->nsetups);
        CVodeGetNumJacEvals(mem, &out->nje);
        CVodeGetNumNonlinSolvIters(mem, &out->nni);
        CVodeGetNumErrTestFails(mem, &out->netf);
        CVodeGetNumRhsEvals(mem, &out->nfe);
        if (in->stored) {
            // simulation_end_y: the interpolated division / death state, else the solver's y
            for (int i = 0; i < N; i++) end_y[i] = (c.divided || c.died) ? c.end_y[i] : NV_Ith_S(y, i);
        } else {
            if (!c.divided && !c.died && result)
                for (int i = 0; i < N; i++) end_y[i] = sol[(size_t)(M - 1) * N + i];
            if (c.divided || c.died)
                for (int i = 0; i < N; i++) end_y[i] = NV_Ith_S(y, i);
        }
        CVodeFree(&mem);
        SUNNonlinSolFree(NLS);
        SUNLinSolFree(LS);
        SUNMatDestroy(J);
        N_VDestroy(y);
        N_VDestroy(atol);
        N_VDestroy(tmp);
    } else {
        for (int i = 0; i < N; i++) end_y[i] = sol[(size_t)(M - 1) * N + i];
    }
    out->nsteps = nst;
    out->ok = result ? 1 : 0;
    out->divided = c.divided;
    out->died = c.died;
    double achieved_cell_time;
    if (c.divided || c.died)
        achieved_cell_time = c.simulation_end_time;
    else
        achieved_cell_time = in->stored ? c.previous_integration_step_time : tp[M - 1];
    out->sim_end = c.simulation_end_time;
    out->achieved_time = achieved_cell_time + in->creation_time;
    for (int k = 0; k < 5; k++) out->event_times[k] = c.ev[k];
    if (in->stored) {
        // the evaluation passes (Experiment.cpp:277-292): per synchronisation point in enum order the
        // iterator restarted, the entries of that pass in time order, GetInterpolatedSpeciesValue
        // (Cell.cpp:280-327) through the stored records
        if (!result) return 1;
        for (int p = 0; p <= 4; p++) {
            c.interp.restart(N);
            const double evp = p == 0 ? c.ev[0] : p == 1 ? c.ev[2] : p == 2 ? c.ev[3] : c.ev[4];
            for (int k = 0; k < M; k++) {
                const int s = in->output_species[k];
                if (in->output_sync[k] != p || s < 0 || s >= N) continue;
                const double time = in->output_times[k] + in->sync_offset;
                double cell_time;
                if (p == 4)
                    cell_time = time - in->creation_time;
                else
                    cell_time = std::isnan(evp) ? time + c.simulation_end_time : time + evp;
                if (cell_time < 0.0 || cell_time > c.simulation_end_time) continue;
                out_values[k] = c.interp.get(c.recs, N, cell_time)[s];
            }
        }
        return 0;
    }
    // GetInterpolatedSpeciesValue (Cell.cpp:280-360), species without synchronisation
    for (int k = 0; k < M; k++) {
        const int s = in->output_species[k];
        if (s < 0 || s >= N) continue;
        const double cell_time = in->output_times[k] - in->creation_time;
        if (cell_time < 0.0 || cell_time > c.simulation_end_time) continue;
        // exact-time lookup: the first stored output with this time
        for (int i = 0; i < M; i++) {
            if (tp[i] == cell_time) {
                out_values[k] = sol[(size_t)i * N + s];
                break;
            }
        }
    }
    return result ? 0 : 1;
}

}  // extern "C"
