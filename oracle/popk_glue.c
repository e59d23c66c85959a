/*
 * popk_glue.c -- TEST INFRASTRUCTURE (oracle). Never linked into the product.
 *
 * CPU restatement of BCM3's likelihood code on the hot path:
 *   - LikelihoodPopPKTrajectory::EvaluateLogProbability, RHS/Jacobians, dosing callbacks
 *     (src/likelihoods/LikelihoodPopPKTrajectory.cpp:259-718)
 *   - bcm3::LogPdfTnu4, QuantileNormal, LogPdfNormal, PdfNormal
 *     (src/utils/ProbabilityDistributions.cpp:51-56,129-138,216-224,359-363)
 *   - bcm3::fastpow10, rsqrt, logsum (src/utils/MathFunctions.h:13,35-48,67-82)
 *   - VariableSet::TransformVariable (src/sampler/VariableSet.cpp:97-124)
 *   - TestLikelihoodBanana / TestLikelihoodCircular EvaluateLogProbability
 * Linked against either ODE backend (restated CVODE or vendored CVODE).
 *
 * Third-party arithmetic not present in /root/reference: Boost.Math (unpinned version,
 * CMakeLists.txt:14) supplies quantile(normal) = mu - sigma*sqrt(2)*erfc_inv(2p) and log1p.
 * erfc_inv is restated here as the exact normal quantile (rational initial guess refined by
 * Halley steps on libm erfc), which agrees with Boost's rational approximations to a few ulp;
 * the unit test pins it against scipy.special.ndtri. log1p comes from libm.
 */
#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#ifdef __x86_64__
#include <xmmintrin.h>
#endif

#include "ode_driver.h"
#include "oracle_api.h"

/* ---------------- math (ProbabilityDistributions.cpp, MathFunctions.h) ---------------- */

static double ndtri_lower(double p) /* p in (0, 0.5] */
{
    static const double a[6] = {-3.969683028665376e+01, 2.209460984245205e+02, -2.759285104469687e+02,
                                1.383577518672690e+02,  -3.066479806614716e+01, 2.506628277459239e+00};
    static const double b[5] = {-5.447609879822406e+01, 1.615858368580409e+02, -1.556989798598866e+02,
                                6.680131188771972e+01,  -1.328068155288572e+01};
    static const double c[6] = {-7.784894002430293e-03, -3.223964580411365e-01, -2.400758277161838e+00,
                                -2.549732539343734e+00, 4.374664141464968e+00,  2.938163982698783e+00};
    static const double d[4] = {7.784695709041462e-03, 3.224671290700398e-01, 2.445134137142996e+00,
                                3.754408661907416e+00};
    double x;
    if (p < 0.02425) {
        double q = sqrt(-2.0 * log(p));
        x = (((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5]) /
            ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1.0);
    } else {
        double q = p - 0.5, r = q * q;
        x = (((((a[0] * r + a[1]) * r + a[2]) * r + a[3]) * r + a[4]) * r + a[5]) * q /
            (((((b[0] * r + b[1]) * r + b[2]) * r + b[3]) * r + b[4]) * r + 1.0);
    }
    /* Halley refinement on Phi(x) = 0.5*erfc(-x/sqrt2); in the central region the residual is
       formed as 0.5*erf(x/sqrt2) - (p - 0.5) (p - 0.5 exact) for relative accuracy near 0 */
    const int central = (p > 0.25);
    for (int it = 0; it < 3; it++) {
        double e = central ? 0.5 * erf(x / 1.4142135623730951) - (p - 0.5)
                           : 0.5 * erfc(-x / 1.4142135623730951) - p;
        double u = e * 2.5066282746310002 * exp(0.5 * x * x);
        x = x - u / (1.0 + 0.5 * x * u);
    }
    return x;
}

/* standard normal quantile */
static double ndtri(double p)
{
    if (!(p > 0.0)) return (p == 0.0) ? -INFINITY : NAN;
    if (!(p < 1.0)) return (p == 1.0) ? INFINITY : NAN;
    if (p <= 0.5) return ndtri_lower(p);
    return -ndtri_lower(1.0 - p); /* 1-p exact for p >= 0.5 */
}

/* bcm3::QuantileNormal (ProbabilityDistributions.cpp:359-363) via Boost:
 * result = -erfc_inv(2p); result *= sd*root_two; result += mean. */
double orc_quantile_normal(double p, double mu, double sigma)
{
    double erfcinv_2p = -ndtri(p) / 1.4142135623730951;
    double r = -erfcinv_2p;
    r *= sigma * 1.4142135623730951;
    r += mu;
    return r;
}

/* bcm3::LogPdfTnu4 (ProbabilityDistributions.cpp:216-224) */
double orc_log_pdf_tnu4(double x, double mu, double sigma)
{
    double xn = (x - mu) / sigma;
    return -0.9808292530117262 - 2.5 * log1p(0.25 * xn * xn) - log(sigma);
}

static double fastpow10(double x) { return exp(x * 2.3025850929940459); }

/* VariableSet::TransformVariable (VariableSet.cpp:97-124) */
double orc_transform(int32_t tf, double x)
{
    switch (tf) {
    case ORC_TF_NONE: return x;
    case ORC_TF_LOG: return exp(x);
    case ORC_TF_LOG10: return fastpow10(x);
    case ORC_TF_LOGIT:
        if (x > 0) {
            double z = exp(-x);
            return 1.0 / (1.0 + z);
        } else {
            double z = exp(x);
            return z / (1.0 + z);
        }
    default: return x;
    }
}

/* ---------------- PopPK model (LikelihoodPopPKTrajectory.cpp) ---------------- */

typedef struct {
    const orc_popk_model* m;
    ode_solver* solver;
    int patient;
    double dose, dosing_interval, dose_after_dose_change, dose_change_time;
    int intermittent;
    const uint8_t* skipped_days;
    double ka, ke, kel, vod, kf, kb, ktr, ntr, tsw, ka2;
    int biphasic_switch;
    double last_treatment;
    double current_dose_time;
} pdata;

static int is_two(int t) { return t == ORC_PK_TWO || t == ORC_PK_TWO_BIPHASIC || t == ORC_PK_TWO_TRANSIT; }
static int is_transit(int t) { return t == ORC_PK_ONE_TRANSIT || t == ORC_PK_TWO_TRANSIT; }
static int is_biphasic(int t) { return t == ORC_PK_ONE_BIPHASIC || t == ORC_PK_TWO_BIPHASIC; }

/* CalculateDerivative_* (.cpp:446-627) */
static int popk_rhs(double t, const double* y, double* dydt, void* user)
{
    pdata* pd = (pdata*)user;
    int type = pd->m->pk_type;
    double ka = pd->ka;
    if (is_biphasic(type)) ka = pd->biphasic_switch ? pd->ka : pd->ka2;
    double input = 0.0;
    if (is_transit(type)) {
        double dose = pd->dose;
        if (t >= pd->dose_change_time) dose = pd->dose_after_dose_change;
        double tst = t - pd->last_treatment;
        double n = pd->ntr;
        double lnf = 0.9189385332046727 + (n + 0.5) * log(n) - n + log(1 + 1 / (12.0 * n));
        double transit = exp((n * log(pd->ktr * tst) - pd->ktr * tst) - lnf);
        transit = pd->ktr * transit * dose;
        input = transit;
    }
    if (is_transit(type))
        dydt[0] = input - (ka + pd->ke) * y[0];
    else
        dydt[0] = -(ka + pd->ke) * y[0];
    if (is_two(type)) {
        dydt[1] = ka * y[0] - pd->kel * y[1] - pd->kf * y[1] + pd->kb * y[2];
        dydt[2] = pd->kf * y[1] - pd->kb * y[2];
    } else {
        dydt[1] = ka * y[0] - pd->kel * y[1];
    }
    return 0;
}

/* CalculateJacobian_* (.cpp:457-642); J row-major 3x3, pre-zeroed */
static int popk_jac(double t, const double* y, const double* fy, double* J, void* user)
{
    pdata* pd = (pdata*)user;
    int type = pd->m->pk_type;
    double ka = pd->ka;
    if (is_biphasic(type)) ka = pd->biphasic_switch ? pd->ka : pd->ka2;
    J[0 * 3 + 0] = -(ka + pd->ke);
    J[1 * 3 + 0] = ka;
    if (is_two(type)) {
        J[1 * 3 + 1] = -(pd->kel + pd->kf);
        J[1 * 3 + 2] = pd->kb;
        J[2 * 3 + 1] = pd->kf;
        J[2 * 3 + 2] = -pd->kb;
    } else {
        J[1 * 3 + 1] = -pd->kel;
    }
    return 0;
}

/* CheckGiveTreatment (.cpp:644-671) */
static int check_give_treatment(double t, const pdata* pd)
{
    int give = 1;
    int day = (int)floor(t / 24.0);
    if (day >= 0 && day < 29 && pd->skipped_days[day]) give = 0;
    if (pd->intermittent == 1) {
        double tiw = t - 7.0 * 24.0 * floor(t / (7.0 * 24.0));
        if (tiw >= 5.0 * 24.0) give = 0;
    } else if (pd->intermittent == 2) {
        double tic = t - 28.0 * 24.0 * floor(t / (28.0 * 24.0));
        if (tic >= 21.0 * 24.0) give = 0;
    } else if (pd->intermittent == 3) {
        double tiw = t - 7.0 * 24.0 * floor(t / (7.0 * 24.0));
        if (tiw >= 4.0 * 24.0) give = 0;
    }
    return give;
}

static void apply_dose(double t, pdata* pd)
{
    double dose = pd->dose;
    if (t >= pd->dose_change_time) dose = pd->dose_after_dose_change;
    if (is_transit(pd->m->pk_type))
        pd->last_treatment = t;
    else
        ode_set_current_y(pd->solver, 0, ode_get_current_y(pd->solver, 0) + dose);
}

/* TreatmentCallback (.cpp:673-690) */
static double treatment_cb(double t, void* user)
{
    pdata* pd = (pdata*)user;
    pd->current_dose_time += pd->dosing_interval;
    if (check_give_treatment(t, pd)) apply_dose(t, pd);
    return pd->current_dose_time;
}

/* TreatmentCallbackBiphasic (.cpp:692-718) */
static double treatment_cb_biphasic(double t, void* user)
{
    pdata* pd = (pdata*)user;
    if (pd->biphasic_switch) {
        pd->biphasic_switch = 0;
        pd->current_dose_time += pd->dosing_interval;
        return pd->current_dose_time;
    }
    if (check_give_treatment(t, pd)) {
        apply_dose(t, pd);
        pd->biphasic_switch = 1;
        return pd->current_dose_time + pd->tsw;
    }
    pd->current_dose_time += pd->dosing_interval;
    return pd->current_dose_time;
}

typedef struct {
    const orc_popk_model* m;
    int64_t begin, end;
    const double* values;
    double* logp;
    double* patient_llh;
    double* traj;
    int64_t* stats;
    int32_t* ok;
    int full;
} job;

static void eval_range(job* jb)
{
    const orc_popk_model* m = jb->m;
    int N = m->N, P = m->P, T = m->T, d = m->d;
    int npk = m->num_pk_params, npop = m->num_pk_pop_params;
    pdata pd;
    memset(&pd, 0, sizeof(pd));
    pd.m = m;
    ode_solver* solver = ode_create(N, popk_rhs, popk_jac, &pd);
    pd.solver = solver;
    ode_set_tolerance(solver, m->rtol, m->atol);
    ode_set_max_steps(solver, m->max_steps);
    double* sim = (double*)malloc(sizeof(double) * N * (T > 0 ? T : 1));

    for (int64_t e = jb->begin; e < jb->end; e++) {
        const double* v = jb->values + e * d;
        double logp = 0.0;
        int sdix = m->sd_ix;
        double sd = orc_transform(m->transforms[sdix], v[sdix]);
        double sd2 = orc_transform(m->transforms[sdix + 1], v[sdix + 1]);
        int broke = 0;
        for (int j = 0; j < P; j++) {
            int64_t tj = e * P + j;
            if (jb->patient_llh) jb->patient_llh[tj] = NAN;
            if (jb->ok) jb->ok[tj] = -1;
            if (jb->traj)
                for (int k = 0; k < N * T; k++) jb->traj[tj * N * T + k] = NAN;
            if (broke && !jb->full) continue;

            pd.patient = j;
            pd.dose = m->dose[j];
            pd.dosing_interval = m->dosing_interval[j];
            pd.dose_after_dose_change = m->dose_after_dose_change[j];
            pd.dose_change_time = m->dose_change_time[j];
            pd.intermittent = m->intermittent[j];
            pd.skipped_days = m->skipped_days + 29 * j;
            /* parameter map: population (LikelihoodPopPKTrajectory.cpp:283-310) or single patient
             * (LikelihoodPharmacokineticTrajectory.cpp:226-259) */
            const int single = (m->param_map == 1);
            pd.vod = isnan(m->fixed_vod) ? orc_transform(m->transforms[3], v[3]) : m->fixed_vod;
            if (single) {
                pd.ka = orc_transform(m->transforms[0], v[0]);
                pd.ke = orc_transform(m->transforms[1], v[1]);
                pd.kel = orc_transform(m->transforms[2], v[2]) / pd.vod;
            } else {
                pd.ka = fastpow10(orc_quantile_normal(v[npk + npop * (j + 1) + 0], v[0], v[npk + 0]));
                pd.ke = orc_transform(m->transforms[1], v[1]);
                pd.kel = fastpow10(orc_quantile_normal(v[npk + npop * (j + 1) + 1], v[2], v[npk + 1])) / pd.vod;
            }
            if (is_two(m->pk_type)) {
                if (isnan(m->fixed_kf)) {
                    pd.kf = orc_transform(m->transforms[4], v[4]);
                    pd.kb = orc_transform(m->transforms[5], v[5]);
                } else {
                    pd.kf = m->fixed_kf;
                    pd.kb = m->fixed_kb;
                }
            }
            if (is_transit(m->pk_type)) {
                pd.ntr = orc_transform(m->transforms[m->n_transit_ix], v[m->n_transit_ix]);
                pd.ktr = (pd.ntr + 1) / orc_transform(m->transforms[m->transit_time_ix], v[m->transit_time_ix]);
            }
            if (is_biphasic(m->pk_type)) {
                pd.tsw = orc_transform(m->transforms[m->biphasic_time_ix], v[m->biphasic_time_ix]);
                double lim = pd.dosing_interval - 1e-2;
                /* std::min(a,b) = (b < a) ? b : a; the single-patient likelihood does not clamp
                 * (LikelihoodPharmacokineticTrajectory.cpp:253) */
                if (!single) pd.tsw = (lim < pd.tsw) ? lim : pd.tsw;
                pd.ka2 = orc_transform(m->transforms[m->absorption2_ix], v[m->absorption2_ix]);
            }
            pd.last_treatment = 0.0;
            /* (exact-match result cache .cpp:313-353 is semantically transparent: skipped) */
            if (is_biphasic(m->pk_type)) {
                pd.biphasic_switch = 1;
                pd.current_dose_time = 0;
                ode_set_discontinuity(solver, pd.tsw, treatment_cb_biphasic, &pd);
            } else {
                pd.current_dose_time = pd.dosing_interval;
                ode_set_discontinuity(solver, pd.dosing_interval, treatment_cb, &pd);
            }
            double y0[3];
            y0[0] = is_transit(m->pk_type) ? 0.0 : pd.dose;
            y0[1] = 0.0;
            y0[2] = 0.0;
            double conversion = (1e6 / m->MW) / pd.vod;
            int nsim = m->simulate_until[j];
            double pllh = 0.0;
            int okflag = 1;
            if (nsim > 0) {
                int r = ode_solve_return_solution(solver, y0, m->time, nsim, sim);
                if (jb->stats) {
                    long st[ORC_ST_COUNT];
                    ode_stats(solver, st);
                    st[ORC_ST_NST] = ode_last_steps(solver);
                    for (int k = 0; k < ORC_ST_COUNT; k++) jb->stats[tj * ORC_ST_COUNT + k] = st[k];
                }
                if (!r) {
                    pllh = -INFINITY;
                    okflag = 0;
                } else {
                    if (jb->traj)
                        for (int s = 0; s < N; s++)
                            for (int i = 0; i < nsim; i++) jb->traj[tj * N * T + s * T + i] = sim[s * nsim + i];
                    for (int i = 0; i < nsim; i++) {
                        double x = conversion * sim[1 * nsim + i];
                        double y = m->observed[j * T + i];
                        if (!isnan(y)) {
                            double xm = (x < 0.0) ? 0.0 : x; /* std::max(x, 0.0) = (x < 0) ? 0 : x */
                            pllh += orc_log_pdf_tnu4(x, y, sd + sd2 * xm);
                        }
                        if (isnan(x) && !single) { /* (.cpp:418-421; no such rule in the single-patient one) */
                            pllh = -INFINITY;
                            break;
                        }
                    }
                }
            } else if (jb->stats) {
                for (int k = 0; k < ORC_ST_COUNT; k++) jb->stats[tj * ORC_ST_COUNT + k] = 0;
            }
            if (jb->patient_llh) jb->patient_llh[tj] = pllh;
            if (jb->ok) jb->ok[tj] = okflag;
            if (!broke) {
                logp += pllh;
                if (logp == -INFINITY) broke = 1;
            }
        }
        jb->logp[e] = logp;
    }
    free(sim);
    ode_destroy(solver);
}

static void* eval_thread(void* arg)
{
    eval_range((job*)arg);
    return NULL;
}

int orc_popk_eval(const orc_popk_model* m, int64_t n, const double* values, double* logp, double* patient_llh,
                  double* traj, int64_t* stats, int32_t* ok, int32_t full_patients, int32_t nthreads)
{
    if (!m || !values || !logp || m->N < 2 || m->N > 3) return -1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > n) nthreads = (int32_t)(n > 0 ? n : 1);
    job* jobs = (job*)calloc(nthreads, sizeof(job));
    pthread_t* th = (pthread_t*)calloc(nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; t++) {
        jobs[t].m = m;
        jobs[t].begin = n * t / nthreads;
        jobs[t].end = n * (t + 1) / nthreads;
        jobs[t].values = values;
        jobs[t].logp = logp;
        jobs[t].patient_llh = patient_llh;
        jobs[t].traj = traj;
        jobs[t].stats = stats;
        jobs[t].ok = ok;
        jobs[t].full = full_patients;
    }
    if (nthreads == 1) {
        eval_range(&jobs[0]);
    } else {
        for (int t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, eval_thread, &jobs[t]);
        for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    }
    free(jobs);
    free(th);
    return 0;
}

/* ---------------- analytic likelihoods ---------------- */

/* bcm3::rsqrt(double) (MathFunctions.h:35-48): SSE rsqrtss + two Newton steps */
static double bcm3_rsqrt(double x)
{
#ifdef __x86_64__
    __m128 f = _mm_set_ss((float)x);
    f = _mm_rsqrt_ss(f);
    double r = (double)_mm_cvtss_f32(f);
#else
    double r = 1.0 / sqrt(x);
#endif
    r *= ((3.0 - r * r * x) * 0.5);
    r *= ((3.0 - r * r * x) * 0.5);
    return r;
}

/* PdfNormal (ProbabilityDistributions.cpp:51-56) */
static double pdf_normal(double x, double mu, double sigma)
{
    double two_sigma_sq = 2.0 * sigma * sigma;
    double d = x - mu;
    return bcm3_rsqrt(two_sigma_sq * M_PI) * exp(-(d * d) / two_sigma_sq);
}

/* LogPdfNormal (ProbabilityDistributions.cpp:129-138) */
static double log_pdf_normal(double x, double mu, double sigma)
{
    double two_sigma_sq = 2.0 * sigma * sigma;
    double d = x - mu;
    return -log(sigma) - 0.91893853320467274178032973640562 - d * d / two_sigma_sq;
}

/* bcm3::logsum (MathFunctions.h:67-82) */
static double logsum(double loga, double logb)
{
    if (logb > loga) {
        double t = loga;
        loga = logb;
        logb = t;
    }
    if (loga == -INFINITY) return loga;
    double diff = logb - loga;
    if (diff < -500) return loga;
    return loga + log1p(exp(diff));
}

/* TestLikelihoodBanana::EvaluateLogProbability (TestLikelihoodBanana.cpp:42-55) */
int orc_banana_eval(int64_t n, int32_t d, double sd1, double sd2, const double* values, double* logp)
{
    for (int64_t e = 0; e < n; e++) {
        const double* v = values + e * d;
        double p = 1.0;
        for (int i = 0; i < d - 1; i++) p = p * pdf_normal(v[i], 0, sd1);
        double y = v[0];
        for (int i = 1; i < d - 1; i++) y += v[i];
        p *= pdf_normal(v[d - 1], y + 3 * y + (1 - y) * (1 - y), sd2);
        logp[e] = log(p);
    }
    return 0;
}

/* TestLikelihoodCircular::EvaluateLogProbability (TestLikelihoodCircular.cpp:42-53) */
int orc_circular_eval(int64_t n, int32_t d, double radius, double offset, double width, const double* values,
                      double* logp)
{
    for (int64_t e = 0; e < n; e++) {
        const double* v = values + e * d;
        double s1 = 0.0, s2 = 0.0;
        for (int i = 0; i < d; i++) {
            double m1 = (i == 0) ? -offset : 0.0;
            double m2 = (i == 0) ? offset : 0.0;
            double a = v[i] - m1, b = v[i] - m2;
            s1 += a * a;
            s2 += b * b;
        }
        double x1 = sqrt(s1), x2 = sqrt(s2);
        logp[e] = logsum(log_pdf_normal(x1, radius, width), log_pdf_normal(x2, radius, width));
    }
    return 0;
}
