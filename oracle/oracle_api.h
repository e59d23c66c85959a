/*
 * oracle_api.h -- TEST INFRASTRUCTURE (oracle). Never linked into the product.
 *
 * C entry points of the oracle libraries (loaded from Python tests via ctypes):
 *   oracle/liboracle.so        : popk glue + restated CVODE backend
 *   oracle/_ref/libbcm3ref.so  : popk glue + vendored CVODE 5.3.0 built from /root/reference
 * Both export the same symbols.
 */
#ifndef BCM3_ORACLE_API_H
#define BCM3_ORACLE_API_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* LikelihoodPopPKTrajectory::PKModelType (src/likelihoods/LikelihoodPopPKTrajectory.h:28-36),
 * AFTER the reference's string mapping (note "one_biphasic_uptake" -> TWO_BIPHASIC,
 * LikelihoodPopPKTrajectory.cpp:73-74). */
enum { ORC_PK_ONE = 0, ORC_PK_TWO, ORC_PK_ONE_BIPHASIC, ORC_PK_TWO_BIPHASIC, ORC_PK_ONE_TRANSIT,
       ORC_PK_TWO_TRANSIT };

/* VariableSet transforms (src/sampler/VariableSet.cpp:97-124) */
enum { ORC_TF_NONE = 0, ORC_TF_LOG = 1, ORC_TF_LOG10 = 2, ORC_TF_LOGIT = 3 };

typedef struct {
    int32_t pk_type;
    int32_t N;
    int32_t num_pk_params;
    int32_t num_pk_pop_params;
    int32_t d;
    int32_t P;
    int32_t T;
    int32_t sd_ix;
    int32_t n_transit_ix;
    int32_t transit_time_ix;
    int32_t biphasic_time_ix;
    int32_t absorption2_ix;
    int32_t max_steps;
    int32_t param_map; /* 0 population (LikelihoodPopPKTrajectory), 1 single patient
                          (LikelihoodPharmacokineticTrajectory) */
    double rtol;
    double atol;
    double MW;
    double fixed_vod;
    double fixed_kf;
    double fixed_kb;
    const int32_t* transforms;     /* [d] */
    const double* time;            /* [T] */
    const double* observed;        /* [P*T], NaN = unobserved */
    const double* dose;            /* [P] */
    const double* dosing_interval; /* [P] */
    const double* dose_after_dose_change; /* [P] */
    const double* dose_change_time;       /* [P] */
    const int32_t* intermittent;   /* [P] */
    const uint8_t* skipped_days;   /* [P*29] */
    const int32_t* simulate_until; /* [P] */
} orc_popk_model;

/* Evaluate n parameter vectors values[n*d]. Outputs (any may be NULL except logp):
 *   logp[n]                  EvaluateLogProbability result
 *   patient_llh[n*P]         per-patient log-likelihood (NaN if not evaluated due to early break)
 *   traj[n*P*N*T]            simulated states at output times (NaN where not simulated)
 *   stats[n*P*ORC_ST_COUNT]  solver counters per trajectory
 *   ok[n*P]                  1 = solve succeeded, 0 = failed (-inf), -1 = not evaluated
 * The per-patient break at -inf follows LikelihoodPopPKTrajectory.cpp:438-440 for logp;
 * with full_patients=1 every patient is simulated anyway (for parity data). */
int orc_popk_eval(const orc_popk_model* m, int64_t n, const double* values, double* logp,
                  double* patient_llh, double* traj, int64_t* stats, int32_t* ok, int32_t full_patients,
                  int32_t nthreads);

/* Analytic likelihoods (src/likelihoods/TestLikelihoodBanana.cpp:42-55,
 * TestLikelihoodCircular.cpp:42-53). */
int orc_banana_eval(int64_t n, int32_t d, double sd1, double sd2, const double* values, double* logp);
int orc_circular_eval(int64_t n, int32_t d, double radius, double offset, double width, const double* values,
                      double* logp);

/* math helpers exposed for unit tests */
double orc_quantile_normal(double p, double mu, double sigma);
double orc_log_pdf_tnu4(double x, double mu, double sigma);
double orc_transform(int32_t tf, double x);

#ifdef __cplusplus
}
#endif
#endif
