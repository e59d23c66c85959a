// cellpop_static.h -- the model-independent cell-population kernels (cellpop_kernels.hip) and
// their host launcher (cellpop_rt.cpp): one definition of the shared structures.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

// (the run-time compiled cell kernel's work queue includes this header too: hipRTC finds it by name)
#if defined(__HIPCC_RTC__)
#include "bcm3hip.h"
#else
#include "../../include/bcm3hip.h"
#endif

namespace bcm3hip {

struct CpStatic {
    int32_t NS, NC, d, M, n0, max_cells;
    const int32_t* transforms;
    const double* y_init;
    int32_t n_reset;
    const int32_t* reset_index;
    const double* reset_value;
    bcm3hip_value_ref entry_time;
    int32_t sobol_dims;
    const double* sobol;
    const bcm3hip_value_ref* scales;
    int32_t n_actions;
    const bcm3hip_variability_action* actions;
    int32_t n_full;
    const int32_t* full_groups;          // [n_full][2] first dimension, D
    const bcm3hip_value_ref* covariance;  // D(D-1)/2 per full group
    const double* output_times;
    int32_t n_data;
    const bcm3hip_cellpop_data* data;  // device copy; observed / entry point to device arrays
    bcm3hip_value_ref sync_offset;     // synchronization_time_offset (cp_init_kernel -> sync_off[slot])
};

// one work item = one new cell: slot, eval, parent slot (-1 = initial cell), sobol index, flags
struct CpInitItem {
    int32_t slot, eval, parent, sobol_ix, is_initial;
};

// the per-cell outputs a batch leaves (cellpop_cells, the data likelihoods)
struct CpCellArrays {
    double *out_values, *end_y, *creation, *sim_end, *achieved, *event_times;
    int32_t *flags, *nsteps;
};

// the host launchers (cellpop_kernels.hip), not for the run-time compiled program
#if !defined(__HIPCC_RTC__)
hipError_t launch_cp_init(const CpStatic& m, int32_t n_items, const CpInitItem* items, const double* values,
                          double* params, double* y0, double* creation, const double* end_y, const double* achieved,
                          double* sync_off, hipStream_t s);
hipError_t launch_cp_popavg(const CpStatic& m, int32_t n, const double* values, const int32_t* ncells,
                            const int32_t* failed, const double* out_values, const double* creation,
                            const double* sim_end, double* avg, const double* tc_logp, const int32_t* tc_ok,
                            double* logp, int32_t* status, hipStream_t s);
// the time-course data likelihoods: per (evaluation, data likelihood) logp and Evaluate's result;
// ws_global = nullptr: the matching workspace of max_R cells in LDS (cp_assign_lds_fits)
// sim_child[slot]: the cell index of the slot's first daughter, -1 = none (observed lineages)
hipError_t launch_cp_timecourse(const CpStatic& m, int32_t n, int32_t max_R, const double* values,
                                const int32_t* ncells, const int32_t* failed, const double* out_values,
                                const int32_t* sim_child, unsigned char* ws_global, size_t ws_stride,
                                double* tc_logp, int32_t* tc_ok, hipStream_t s);
// the time-points data likelihoods, same outputs and workspace as the time courses
hipError_t launch_cp_timepoints(const CpStatic& m, int32_t n, int32_t max_R, const double* values,
                                const int32_t* ncells, const int32_t* failed, const double* out_values,
                                unsigned char* ws_global, size_t ws_stride, double* tc_logp, int32_t* tc_ok,
                                hipStream_t s);
// the matching alone (bcm3hip_assign_cells)
hipError_t launch_cp_assign(int32_t n_problems, int32_t R, int32_t nsim, const double* lik, unsigned char* ws_global,
                            size_t ws_stride, int32_t* match, double* sum, int32_t* ok, hipStream_t s);
size_t cp_assign_ws_bytes(int n);  // the matching workspace of n x n cells
// the dynamic workspace plus the larger kernel's static LDS (cp_timepoints_kernel, ~8.4 KB) stay within
// 64 KB, the workgroup limit of parts smaller than gfx950's 160 KB
inline bool cp_assign_lds_fits(int n) { return cp_assign_ws_bytes(n) <= 52 * 1024; }
// the work queue of the cell kernel (cellpop_solver.h cp_queue_kernel) indexes cells by queue position;
// cp_number_kernel numbers them as the generation launches do (the reference's FIFO: the initial
// cells, then per generation the two daughters of each dividing cell in cell order): perm[e][slot] =
// queue position, ncells / failed per evaluation, sim_child[e][slot] = the slot's first daughter's
// cell index (-1); first_pos[i] = the queue position of initial cell i within its evaluation's n0
hipError_t launch_cp_number(int32_t n, int32_t max_cells, int32_t n0, const int32_t* first_pos, const int32_t* child_qi,
                            const int32_t* failed_eval, int32_t* perm, int32_t* ncells, int32_t* failed,
                            int32_t* sim_child, hipStream_t s);
// dst[slot] = src[perm[slot]] for the slots of every evaluation's cells
hipError_t launch_cp_permute(int32_t n, int32_t max_cells, int32_t M, int32_t NS, const int32_t* perm,
                             const int32_t* ncells, CpCellArrays src, CpCellArrays dst, hipStream_t s);
// out[w] = flags[work[w]]
hipError_t launch_cp_gather(const int32_t* work, int32_t n, const int32_t* flags, int32_t* out, hipStream_t s);
// the next experiment's (x, xstatus) into the running sum (logp, status) of
// CellPopulationLikelihood::EvaluateLogProbability (CellPopulationLikelihood.cpp:90-98)
hipError_t launch_cp_accumulate(int32_t n, double* logp, int32_t* status, const double* x, const int32_t* xstatus,
                                hipStream_t s);

#endif

}  // namespace bcm3hip
