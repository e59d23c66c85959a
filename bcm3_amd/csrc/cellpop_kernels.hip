// cellpop_kernels.hip -- the model-independent kernels of the cell-population likelihood
// (the per-cell ODE solve is compiled per model at run time, cellpop_solver.h):
//   cp_init_kernel    one thread per new cell: Cell::Initialize (Cell.cpp:150-191) with
//                     CellPopulation::AddNewCell's initial conditions (CellPopulation.cpp:36-104):
//                     the model's initial amounts or the parent's end state with the daughter
//                     resets (Cell::SetInitialConditionsFromOtherCell, Cell.cpp:119-148), then the
//                     variabilities (VariabilityDescription::GetPseudorandomVector, diagonal
//                     gaussian: QuantileNormal(sobol) * exp(scale); ApplyVariability*);
//   cp_popavg_kernel  one wavefront per evaluation: CountCellsAtTime + NotifySimulatedValue in cell
//                     order (Experiment.cpp:298-311, DataLikelihoodTimeCoursePopulationAverage.cpp)
//                     and DataLikelihoodTimeCoursePopulationAverage::Evaluate.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/bcm3hip.h"
#include "cellpop_static.h"
#include "pk_math.h"

namespace bcm3hip {



__device__ double cp_transform(int32_t tf, double x)
{
    // VariableSet::TransformVariable (src/sampler/VariableSet.cpp:97-124)
    switch (tf) {
    case BCM3HIP_TF_LOG: return exp(x);
    case BCM3HIP_TF_LOG10: return exp(x * 2.3025850929940459);  // bcm3::fastpow10
    case BCM3HIP_TF_LOGIT:
        if (x > 0) {
            const double z = exp(-x);
            return 1.0 / (1.0 + z);
        } else {
            const double z = exp(x);
            return z / (1.0 + z);
        }
    default: return x;
    }
}

__device__ double cp_ref(const bcm3hip_value_ref& r, const double* values, const int32_t* transforms, double none)
{
    if (r.kind == BCM3HIP_REF_VARIABLE) return cp_transform(transforms[r.index], values[r.index]);
    if (r.kind == BCM3HIP_REF_FIXED) return r.value;
    return none;
}

__device__ double cp_apply(int32_t kind, double x, double v)
{
    switch (kind) {
    case BCM3HIP_APPLY_ADDITIVE: return x + v;
    case BCM3HIP_APPLY_ADDITIVE_LOG: return x + exp(v);
    case BCM3HIP_APPLY_ADDITIVE_LOG2: return x + pow(2.0, v);
    case BCM3HIP_APPLY_MULTIPLICATIVE: return x * v;
    case BCM3HIP_APPLY_MULTIPLICATIVE_LOG: return x * exp(v);
    case BCM3HIP_APPLY_MULTIPLICATIVE_LOG2: return x * pow(2.0, v);
    default: return v;  // replace
    }
}



__global__ void cp_init_kernel(CpStatic m, int32_t n_items, const CpInitItem* items, const double* values,
                               double* params, double* y0, double* creation, const double* end_y, const double* achieved)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= n_items) return;
    const CpInitItem it = items[w];
    const double* v = values + (size_t)it.eval * m.d;
    double* prm = params + (size_t)it.slot * m.d;
    double* y = y0 + (size_t)it.slot * m.NS;
    for (int i = 0; i < m.d; i++) prm[i] = cp_transform(m.transforms[i], v[i]);
    if (it.parent < 0) {
        for (int i = 0; i < m.NS; i++) y[i] = m.y_init[i];
        creation[it.slot] = cp_ref(m.entry_time, v, m.transforms, 0.0);
    } else {
        const double* pe = end_y + (size_t)it.parent * m.NS;
        for (int i = 0; i < m.NS; i++) y[i] = pe[i];
        for (int r = 0; r < m.n_reset; r++) y[m.reset_index[r]] = m.reset_value[r];
        creation[it.slot] = achieved[it.parent];
    }
    if (m.sobol_dims == 0) return;
    // pseudorandom vector, diagonal gaussian (VariabilityDescription.cpp:60-67)
    constexpr int DMAX = 32;
    double pr[DMAX];
    const double* sob = m.sobol + (size_t)it.sobol_ix * m.sobol_dims;
    for (int k = 0; k < m.sobol_dims && k < DMAX; k++)
        pr[k] = quantile_normal(sob[k], 0.0, 1.0) * exp(cp_ref(m.scales[k], v, m.transforms, 0.0));
    for (int a = 0; a < m.n_actions; a++) {
        const bcm3hip_variability_action act = m.actions[a];
        if (act.only_initial_cells && !it.is_initial) continue;
        const double r = act.negate ? -pr[act.dim] : pr[act.dim];
        if (act.target_kind == 0)
            prm[act.target_index] = cp_apply(act.apply, prm[act.target_index], r);
        else
            y[act.target_index] = cp_apply(act.apply, y[act.target_index], r);
    }
}

// one wavefront per evaluation; lanes over output entries
__global__ __launch_bounds__(64) void cp_popavg_kernel(CpStatic m, int32_t n, const double* values,
                                                       const int32_t* ncells, const int32_t* failed,
                                                       const double* out_values, const double* creation,
                                                       const double* sim_end, double* avg /*[n][M]*/,
                                                       double* logp, int32_t* status)
{
    const int e = blockIdx.x;
    if (e >= n) return;
    const int ln = threadIdx.x;
    const int nc = ncells[e];
    const double* v = values + (size_t)e * m.d;
    const size_t base = (size_t)e * m.max_cells;
    // entry_time < -7 days fails the experiment (Experiment.cpp:673-676)
    const bool fail = failed[e] || (cp_ref(m.entry_time, v, m.transforms, 0.0) < -7.0 * 24.0 * 60.0 * 60.0);
    for (int k = ln; k < m.M; k += 64) {
        const double t = m.output_times[k];
        int pop = 0;
        for (int c = 0; c < nc; c++) {
            const double ct = t - creation[base + c];
            pop += (ct >= 0.0 && ct <= sim_end[base + c]) ? 1 : 0;
        }
        double s = 0.0;
        for (int c = 0; c < nc; c++) {
            const double x = out_values[(base + c) * m.M + k];
            if (x == x) s += x / (double)pop;
        }
        avg[(size_t)e * m.M + k] = s;
    }
    __syncthreads();
    if (ln != 0) return;
    if (fail) {
        logp[e] = -INFINITY;
        if (status) status[e] = BCM3HIP_STATUS_SOLVER_FAIL;
        return;
    }
    double total = 0.0;
    for (int di = 0; di < m.n_data; di++) {
        const bcm3hip_cellpop_data dl = m.data[di];
        const double stdev = cp_ref(dl.stdev, v, m.transforms, 1.0);
        const double offset = cp_ref(dl.offset, v, m.transforms, 0.0);
        const double scale = cp_ref(dl.scale, v, m.transforms, 1.0);
        const double pstdev = cp_ref(dl.proportional_stdev, v, m.transforms, 0.0);
        const double minus_log_sigma = -log(stdev);
        const double inv2 = 1.0 / (2.0 * stdev * stdev);
        // relative_to_time_average (DataLikelihoodTimeCoursePopulationAverage.cpp:106-113): add
        // the offset, divide by the mean over the time points, take the log, then scale
        double tmean = 0.0;
        if (dl.relative_to_time_average) {
            for (int i = 0; i < dl.T; i++) tmean += avg[(size_t)e * m.M + dl.entry[i]] + offset;
            tmean /= (double)dl.T;
        }
        double lp = 0.0;
        for (int i = 0; i < dl.T; i++) {
            double x = avg[(size_t)e * m.M + dl.entry[i]];
            if (dl.relative_to_time_average) {
                x = log((x + offset) / tmean);
                x *= scale;
            } else {
                x *= scale;
                x += offset;
            }
            for (int j = 0; j < dl.R; j++) {
                const double o = dl.observed[(size_t)j * dl.T + i];
                if (o == o) {
                    // DataLikelihoodTimeCourseBase::EvaluateValue(simulated, observed) called as
                    // EvaluateValue(data, x) by the population average (.cpp:150): the data value
                    // takes the "simulated" role, so the proportional terms scale with it
                    if (dl.error_model == BCM3HIP_CP_ERR_NORMAL) {
                        const double dd = x - o;
                        lp += minus_log_sigma - 0.91893853320467274178032973640562 - dd * dd * inv2;
                    } else if (dl.error_model == BCM3HIP_CP_ERR_T4) {
                        lp += log_pdf_tnu4(o, x, stdev);
                    } else {
                        const double sp = pstdev * fmax(o, 0.0);
                        const double sigma = (dl.error_model == BCM3HIP_CP_ERR_PROPORTIONAL) ? sp : stdev + sp;
                        // bcm3::LogPdfNormal(x, o, sigma) (ProbabilityDistributions.cpp:129-138)
                        const double two_sigma_sq = 2.0 * sigma * sigma;
                        const double dd = x - o;
                        lp += -log(sigma) - 0.91893853320467274178032973640562 - dd * dd / two_sigma_sq;
                    }
                }
            }
        }
        total += lp * dl.weight;
    }
    logp[e] = 0.0 + total;
    if (status) status[e] = BCM3HIP_STATUS_OK;
}

hipError_t launch_cp_init(const CpStatic& m, int32_t n_items, const CpInitItem* items, const double* values,
                          double* params, double* y0, double* creation, const double* end_y, const double* achieved,
                          hipStream_t s)
{
    if (n_items <= 0) return hipSuccess;
    hipLaunchKernelGGL(cp_init_kernel, dim3((n_items + 127) / 128), dim3(128), 0, s, m, n_items, items, values, params,
                       y0, creation, end_y, achieved);
    return hipGetLastError();
}

hipError_t launch_cp_popavg(const CpStatic& m, int32_t n, const double* values, const int32_t* ncells,
                            const int32_t* failed, const double* out_values, const double* creation,
                            const double* sim_end, double* avg, double* logp, int32_t* status, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(cp_popavg_kernel, dim3(n), dim3(64), 0, s, m, n, values, ncells, failed, out_values, creation,
                       sim_end, avg, logp, status);
    return hipGetLastError();
}

__global__ void cp_gather_kernel(const int32_t* work, int32_t n, const int32_t* flags, int32_t* out)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w < n) out[w] = flags[work[w]];
}

hipError_t launch_cp_gather(const int32_t* work, int32_t n, const int32_t* flags, int32_t* out, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(cp_gather_kernel, dim3((n + 255) / 256), dim3(256), 0, s, work, n, flags, out);
    return hipGetLastError();
}

// logp += the next experiment's; the reference stops at the first experiment that fails (logp =
// -inf, later experiments not evaluated), so a failed sum stays as it is
__global__ void cp_accumulate_kernel(int32_t n, double* logp, int32_t* status, const double* x, const int32_t* xstatus)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || status[i] != BCM3HIP_STATUS_OK) return;
    if (xstatus[i] != BCM3HIP_STATUS_OK) {
        logp[i] = -__builtin_inf();
        status[i] = xstatus[i];
    } else {
        logp[i] = logp[i] + x[i];
    }
}

hipError_t launch_cp_accumulate(int32_t n, double* logp, int32_t* status, const double* x, const int32_t* xstatus,
                                hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(cp_accumulate_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, logp, status, x, xstatus);
    return hipGetLastError();
}

}  // namespace bcm3hip
