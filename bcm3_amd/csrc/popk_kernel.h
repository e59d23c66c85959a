// popk_kernel.h -- device-side model descriptor and launchers (internal to libbcm3hip.so).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/bcm3hip.h"

namespace bcm3hip {

// Same fields as bcm3hip_popk_model, with device pointers.
struct PopPKDevModel {
    int32_t pk_type, N, num_pk_params, num_pk_pop_params, d, P, T, sd_ix;
    int32_t n_transit_ix, transit_time_ix, biphasic_time_ix, absorption2_ix, max_steps, param_map;
    double rtol, atol, MW, fixed_vod, fixed_kf, fixed_kb;
    double unity;  // 1.0 (a runtime value: see set_bdf_q in bdf_vec.h)
    const int32_t* transforms;
    const double* time;
    const double* observed;
    const double* dose;
    const double* dosing_interval;
    const double* dose_after_dose_change;
    const double* dose_change_time;
    const int32_t* intermittent;
    const uint8_t* skipped_days;
    const int32_t* simulate_until;
};

// the current device's copy of the host libm's pow tables (bdf_lane.h g_glibc_pow), once per
// device; *glibc: 1 when the solvers use glibc's pow, 0 for the correctly rounded fallback
hipError_t popk_prepare_device(int* glibc);
hipError_t launch_popk(const PopPKDevModel& m, int64_t n, const double* values, double* logp, int32_t* status,
                       double* patient_llh_scratch, int32_t* traj_status_scratch, double* traj_out,
                       bcm3hip_traj_stats* stats_out, int lanes_per_wave, int block_waves, int uni_solver,
                       hipStream_t stream, hipEvent_t ev_start, hipEvent_t ev_stop, int block_lds = 0,
                       const int32_t* n_dev = nullptr, int32_t* steps_out = nullptr, uint64_t* place_out = nullptr);

struct AnalyticDevModel {
    int32_t kind, d;
    double p0, p1, p2;
    // mixtures (kind = 16 + BCM3HIP_MIXTURE_*): K components; mean [K][d], chol [K][d][d] (lower
    // factor, row-major), cst [K][3] = (log weight, log normalising constant, nu)
    int32_t K;
    const double* mean;
    const double* chol;
    const double* cst;
};
constexpr int32_t kAnalyticMixtureBase = 16;

hipError_t launch_analytic(const AnalyticDevModel& m, int64_t n, const double* values, double* logp,
                           int32_t* status, hipStream_t stream, hipEvent_t ev_start, hipEvent_t ev_stop);

// Same fields as bcm3hip_expm_pk_model, with device pointers.
struct ExpmPKDevModel {
    int32_t d, n, n_transit, peripheral, biphasic, metabolite;
    int32_t additive_sd_ix, proportional_sd_ix, absorption_ix, clearance_ix, vod_ix, excretion_ix;
    int32_t pf_ix, pb_ix, mtt_ix, direct_ix, metab_conv_ix, n_treat, n_obs;
    double MW;
    const int32_t* transforms;
    const double* treat_times;
    const double* treat_doses;
    const double* obs_times;
    const double* obs_conc;
    int32_t param_map, P;
    int32_t sigma_ix[5];
    const int32_t* patient_ix;  // [6][P]
    const int32_t* treat_offset;  // [P+1]
    const int32_t* obs_offset;    // [P+1]
    // the distinct step lengths of every patient's Solve loop (built by bcm3hip_open_expm_pk)
    int32_t n_jobs;
    const double* job_dt;          // [n_jobs]
    const int32_t* job_patient;    // [n_jobs]
    const int32_t* interval_job;   // [n_treat]: job of the step that ends dose interval tti
    const int32_t* obs_job;        // [n_obs]: job of the offset from the interval start to observation oti
};

// exps: [n][n_jobs][n*n] scratch
hipError_t expm_prepare_device();  // expm_pk_kernel.hip: its copy of the libm tables
hipError_t launch_expm_pk(const ExpmPKDevModel& m, int64_t n, const double* values, double* logp, int32_t* status,
                          double* exps, hipStream_t stream, hipEvent_t ev_start, hipEvent_t ev_stop);

}  // namespace bcm3hip
