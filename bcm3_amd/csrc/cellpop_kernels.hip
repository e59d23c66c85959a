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
//                     and DataLikelihoodTimeCoursePopulationAverage::Evaluate, then the sum over
//                     the data likelihoods (time courses from cp_timecourse_kernel);
//   cp_timecourse_kernel  one workgroup per (evaluation, time-course data likelihood): the cell
//                     likelihood matrix and the observed-to-simulated matching
//                     (DataLikelihoodTimeCourse::Evaluate);
//   cp_timepoints_kernel  one workgroup per (evaluation, time-points data likelihood): per data
//                     time point the cells alive, their likelihood matrix and the matching
//                     (DataLikelihoodTimePoints::Evaluate).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/bcm3hip.h"
#include "cellpop_init.h"
#include "cellpop_static.h"
#include "pk_math.h"

namespace bcm3hip {



__global__ void cp_init_kernel(CpStatic m, int32_t n_items, const CpInitItem* items, const double* values,
                               double* params, double* y0, double* creation, const double* end_y, const double* achieved,
                               double* sync_off)
{
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= n_items) return;
    cp_init_cell(m, items[w], values, params, y0, creation, end_y, achieved, sync_off);
}

// one wavefront per evaluation; lanes over output entries
__global__ __launch_bounds__(64) void cp_popavg_kernel(CpStatic m, int32_t n, const double* values,
                                                       const int32_t* ncells, const int32_t* failed,
                                                       const double* out_values, const double* creation,
                                                       const double* sim_end, double* avg /*[n][M]*/,
                                                       const double* tc_logp, const int32_t* tc_ok,
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
    // lane k: entry k. The cells are staged through LDS 64 at a time with coalesced loads (every lane
    // loads), so the per-entry loops in cell order read LDS instead of waiting on one global load per
    // cell; the sum keeps the cell order and the same quotients (0.95 -> 0.63 ms per C4 batch)
    __shared__ double cr_s[64], se_s[64], pop_s[64];
    __shared__ double tile[64][65];
    // a NaN payload no arithmetic produces: "this cell's value is NaN, skip it"
    constexpr long long kPopSkip = 0x7ff8dead5eed0001ll;
    // CountCellsAtTime(st.time + time_offset, None) (Experiment.cpp:285, 301): the population is
    // counted at the data time plus the experiment's synchronization_time_offset, the time its values
    // were read at (the stored mode's evaluation passes; without synchronised data the loader refuses
    // a sampled offset, so it is 0 there)
    const double toff = cp_ref(m.sync_offset, v, m.transforms, 0.0);
    for (int k0 = 0; k0 < m.M; k0 += 64) {
        const int k = k0 + ln;
        const bool kv = k < m.M;
        const int kw = (m.M - k0 < 64) ? m.M - k0 : 64;
        const double t = kv ? m.output_times[k] + toff : 0.0;
        // each chunk's global loads are issued before the previous chunk's LDS work (software
        // pipelining: a chunk's latency hides behind the other's compares and sums)
        int pop = 0;
        double ncr = 0.0, nse = 0.0;
        if (ln < nc) {
            ncr = creation[base + ln];
            nse = sim_end[base + ln];
        }
        for (int c0 = 0; c0 < nc; c0 += 64) {
            const int cn = (nc - c0 < 64) ? nc - c0 : 64;
            __syncthreads();
            if (ln < cn) {
                cr_s[ln] = ncr;
                se_s[ln] = nse;
            }
            if (c0 + 64 + ln < nc) {
                ncr = creation[base + c0 + 64 + ln];
                nse = sim_end[base + c0 + 64 + ln];
            }
            __syncthreads();
            // (unrolled: the LDS reads of eight cells issue together, then the dependent updates)
#pragma unroll 8
            for (int j = 0; j < cn; j++) {
                const double ct = t - cr_s[j];
                const double se = se_s[j];
                pop += (int)(ct >= 0.0) & (int)(ct <= se);  // (no short circuit: both reads issue together)
            }
        }
        // the quotients x / pop are formed in parallel (lane = cell of the chunk) and only the sum runs in
        // cell order (a division's dependent chain per cell was the serial loop's cost); a cell whose value
        // is NaN is skipped as in the reference (the test is on the value, so a 0 / 0 still adds its NaN)
        pop_s[ln] = (double)pop;
        double s = 0.0;
        constexpr int PF = 32;  // values per lane of a chunk held for the next one (kw <= PF)
        double nx[PF];
        auto fetch = [&](int c0) {
            const int n_el = ((nc - c0 < 64) ? nc - c0 : 64) * kw;
#pragma unroll
            for (int r = 0; r < PF; r++) {
                const int idx = ln + 64 * r;
                if (idx < n_el) {
                    const int j = idx / kw, kk = idx - j * kw;
                    nx[r] = out_values[(base + c0 + j) * m.M + k0 + kk];
                }
            }
        };
        if (kw <= PF && nc > 0) fetch(0);
        for (int c0 = 0; c0 < nc; c0 += 64) {
            const int cn = (nc - c0 < 64) ? nc - c0 : 64;
            __syncthreads();
            if (kw <= PF) {
#pragma unroll
                for (int r = 0; r < PF; r++) {
                    const int idx = ln + 64 * r;
                    if (idx < cn * kw) {
                        const int j = idx / kw, kk = idx - j * kw;
                        const double x = nx[r];
                        tile[j][kk] = (x == x) ? x / pop_s[kk] : __longlong_as_double(kPopSkip);
                    }
                }
                if (c0 + 64 < nc) fetch(c0 + 64);
            } else {
                for (int idx = ln; idx < cn * kw; idx += 64) {
                    const int j = idx / kw, kk = idx - j * kw;
                    const double x = out_values[(base + c0 + j) * m.M + k0 + kk];
                    tile[j][kk] = (x == x) ? x / pop_s[kk] : __longlong_as_double(kPopSkip);
                }
            }
            __syncthreads();
            if (kv)
#pragma unroll 8
                for (int j = 0; j < cn; j++) {
                    const double q = tile[j][ln];
                    if (__double_as_longlong(q) != kPopSkip) s += q;
                }
        }
        if (kv) avg[(size_t)e * m.M + k] = s;
    }
    __syncthreads();
    if (ln != 0) return;
    if (fail) {
        logp[e] = -INFINITY;
        if (status) status[e] = BCM3HIP_STATUS_SOLVER_FAIL;
        return;
    }
    // Experiment::EvaluateLogProbability (Experiment.cpp:346-355): the data likelihoods in order; one
    // whose Evaluate fails (a time course with a NaN cell likelihood) ends the sum, which is kept
    double total = 0.0;
    for (int di = 0; di < m.n_data; di++) {
        const bcm3hip_cellpop_data dl = m.data[di];
        if (dl.kind == BCM3HIP_CP_DATA_TIME_COURSE || dl.kind == BCM3HIP_CP_DATA_TIME_POINTS) {
            if (!tc_ok[(size_t)e * m.n_data + di]) break;
            total += tc_logp[(size_t)e * m.n_data + di];
            continue;
        }
        const double offset = cp_ref(dl.offset, v, m.transforms, 0.0);
        const double scale = cp_ref(dl.scale, v, m.transforms, 1.0);
        double stdev = cp_ref(dl.stdev, v, m.transforms, 1.0);
        if (dl.stdev_relative_to_scale) stdev *= scale;  // GetCurrentSTDev (DataLikelihoodBase.cpp:151-153)
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

// ---------------------------------------------------------------------------------------------
// Time-course data likelihood (DataLikelihoodTimeCourse, src/cellpop/DataLikelihoodTimeCourse.cpp):
// the likelihood of every observed cell against every simulated cell, then the assignment of
// observed to simulated cells by the reference's vendored matching routine (dependencies/
// hungarian2/hungarian.cpp, hungarianMinimumWeightPerfectMatching). One workgroup per
// (evaluation, data likelihood): its threads fill the cost matrix, one lane runs the matching over
// a workspace in LDS (global memory when the matrix is too large for 64 KB).

// the matching workspace of one problem with n left and n right nodes
struct HgWs {
    double* cost;        // [n*n] -cell likelihood, row = observed cell, column = simulated cell
    uint16_t* adj;       // [n*n] each left node's edge list (right node per position)
    double *lpot, *rpot, *slack;
    int32_t *ntight, *slack_from, *slack_edge, *lmatch, *rmatch, *back, *queue;
    uint8_t* seen;
};

__host__ __device__ inline size_t hg_ws_bytes(int n)
{
    const size_t nn = (size_t)n * n;
    return nn * 8 + ((nn * 2 + 7) / 8) * 8 + (size_t)n * 3 * 8 + (size_t)n * 7 * 4 + (size_t)n;
}

__device__ inline HgWs hg_carve(unsigned char* p, int n)
{
    const size_t nn = (size_t)n * n;
    HgWs w;
    w.cost = (double*)p;
    p += nn * 8;
    w.adj = (uint16_t*)p;
    p += ((nn * 2 + 7) / 8) * 8;
    w.lpot = (double*)p;
    w.rpot = w.lpot + n;
    w.slack = w.rpot + n;
    p += (size_t)n * 3 * 8;
    w.ntight = (int32_t*)p;
    w.slack_from = w.ntight + n;
    w.slack_edge = w.slack_from + n;
    w.lmatch = w.slack_edge + n;
    w.rmatch = w.lmatch + n;
    w.back = w.rmatch + n;
    w.queue = w.back + n;
    p += (size_t)n * 7 * 4;
    w.seen = (uint8_t*)p;
    return w;
}

// (int)r < 1e-12 as compiled for x86-64 (hungarian.cpp:167-169): r stored in an int truncates
// toward zero, so every reduced cost below 1 is "tight"; NaN and out-of-range values convert to
// INT_MIN, tight as well
__device__ inline bool hg_tight0(double r)
{
    if (!(r > -2147483649.0 && r < 2147483648.0)) return true;
    return (double)(int)r < 1e-12;
}

// hungarianMinimumWeightPerfectMatching(n, n, edges) over the complete bipartite graph of the
// cost matrix, edges given row by row (the order DataLikelihoodTimeCourse::Evaluate builds them,
// .cpp:289-315), so every left node's sorted edge list starts as 0..n-1. Statement for statement
// the vendored routine (see oracle/hungarian.py for the behaviours this keeps); sequential, one
// lane. Returns false when it finds no perfect matching.
__device__ bool hg_match(int n, const HgWs& w)
{
    constexpr double OO = 1.7976931348623157e308;
    const double* C = w.cost;
    for (int i = 0; i < n; i++) {  // left potentials: the smallest incident cost (:122-134)
        double m = C[(size_t)i * n];
        for (int j = 1; j < n; j++)
            if (C[(size_t)i * n + j] < m) m = C[(size_t)i * n + j];
        w.lpot[i] = m;
    }
    for (int j = 0; j < n; j++) w.rpot[j] = OO;
    for (int i = 0; i < n; i++)  // right potentials over the edges in order (:141-148)
        for (int j = 0; j < n; j++) {
            const double red = C[(size_t)i * n + j] - w.lpot[i];
            if (w.rpot[j] > red) w.rpot[j] = red;
        }
    for (int i = 0; i < n; i++) {  // tight prefixes (:162-177)
        uint16_t* a = w.adj + (size_t)i * n;
        for (int k = 0; k < n; k++) a[k] = (uint16_t)k;
        int t = 0;
        for (int k = 0; k < n; k++) {
            const int r = a[k];
            if (hg_tight0(C[(size_t)i * n + r] - w.lpot[i] - w.rpot[r])) {
                if (k != t) {
                    const uint16_t x = a[t];
                    a[t] = a[k];
                    a[k] = x;
                }
                t++;
            }
        }
        w.ntight[i] = t;
    }
    int card = 0;
    for (int i = 0; i < n; i++) {
        w.lmatch[i] = -1;
        w.rmatch[i] = -1;
    }
    for (int i = 0; i < n; i++) {  // greedy start (:192-203)
        const uint16_t* a = w.adj + (size_t)i * n;
        for (int k = 0; k < w.ntight[i]; k++) {
            const int j = a[k];
            if (w.rmatch[j] == -1) {
                card++;
                w.rmatch[j] = i;
                w.lmatch[i] = j;
                break;
            }
        }
    }
    while (card < n) {
        for (int j = 0; j < n; j++) {
            w.slack[j] = OO;
            w.slack_from[j] = -1;
            w.back[j] = -1;
            w.seen[j] = 0;
        }
        int start = -1;
        double fewest = OO;
        for (int i = 0; i < n; i++)
            if (w.lmatch[i] == -1 && (double)w.ntight[i] < fewest) {
                fewest = (double)w.ntight[i];
                start = i;
            }
        int qh = 0, qt = 0;
        w.queue[qt++] = start;
        w.seen[start] = 1;
        int end = -1;
        while (end == -1) {
            while (end == -1 && qh < qt) {  // breadth-first over tight edges (:292-329)
                const int i = w.queue[qh++];
                uint16_t* a = w.adj + (size_t)i * n;
                for (int k = 0; k < w.ntight[i];) {
                    const int j = a[k];
                    if (C[(size_t)i * n + j] > w.lpot[i] + w.rpot[j]) {  // loose now
                        const int last = --w.ntight[i];
                        const uint16_t x = a[k];
                        a[k] = a[last];
                        a[last] = x;
                        continue;
                    }
                    if (w.back[j] == -1) {
                        w.back[j] = i;
                        const int m = w.rmatch[j];
                        if (m == -1) {
                            end = j;  // the scan goes on: the last unmatched node wins
                        } else if (!w.seen[m]) {
                            w.seen[m] = 1;
                            w.queue[qt++] = m;
                        }
                    }
                    k++;
                }
                if (end == -1) {  // slack caches (:336-357)
                    const double p = w.lpot[i];
                    for (int k = w.ntight[i]; k < n; k++) {
                        const int j = a[k];
                        const int m = w.rmatch[j];
                        if (m == -1 || !w.seen[m]) {
                            const double red = C[(size_t)i * n + j] - p - w.rpot[j];
                            if (red < w.slack[j]) {
                                w.slack[j] = red;
                                w.slack_from[j] = i;
                                w.slack_edge[j] = k;
                            }
                        }
                    }
                }
            }
            if (end == -1) {
                int jmin = -1;
                double smin = OO;
                for (int j = 0; j < n; j++) {  // (:372-381)
                    const int m = w.rmatch[j];
                    if ((m == -1 || !w.seen[m]) && w.slack[j] < smin) {
                        smin = w.slack[j];
                        jmin = j;
                    }
                }
                if (jmin == -1 || w.slack_from[jmin] == -1) return false;
                for (int i = 0; i < n; i++)  // (:396-403)
                    if (w.seen[i]) {
                        w.lpot[i] += smin;
                        if (w.lmatch[i] != -1) w.rpot[w.lmatch[i]] -= smin;
                    }
                for (int j = 0; j < n; j++) {  // (:406-444)
                    const int m0 = w.rmatch[j];
                    if (m0 == -1 || !w.seen[m0]) {
                        w.slack[j] -= smin;
                        if (w.slack[j] == 0) {
                            const int i = w.slack_from[j];
                            const int k = w.slack_edge[j];
                            uint16_t* a = w.adj + (size_t)i * n;
                            if (k != w.ntight[i]) {
                                const uint16_t x = a[k];
                                a[k] = a[w.ntight[i]];
                                a[w.ntight[i]] = x;
                            }
                            w.ntight[i]++;
                            if (end == -1) {
                                w.back[j] = i;
                                const int m = w.rmatch[j];
                                if (m == -1) {
                                    end = j;
                                } else if (!w.seen[m]) {
                                    w.seen[m] = 1;
                                    w.queue[qt++] = m;
                                }
                            }
                        }
                    }
                }
            }
        }
        card++;
        for (int j = end; j != -1;) {  // flip the augmenting path (:457-468)
            const int i = w.back[j];
            const int nxt = w.lmatch[i];
            w.rmatch[j] = i;
            w.lmatch[i] = j;
            j = nxt;
        }
    }
    return true;
}

__device__ inline double cp_log_pdf_normal(double x, double mu, double sigma)
{
    // bcm3::LogPdfNormal (src/utils/ProbabilityDistributions.cpp:129-138)
    const double two_sigma_sq = 2.0 * sigma * sigma;
    const double dd = x - mu;
    return -log(sigma) - 0.91893853320467274178032973640562 - dd * dd / two_sigma_sq;
}

// the likelihood of observed cell i against simulated cell j: CalculateCellLikelihood for one
// species and no observed lineage (DataLikelihoodTimeCourse.cpp:451-497), the simulated values
// scaled and shifted first (:236-241), a missing simulated value penalised by the distance to the
// cell's first / last simulated time point (CalculateMissingValueLikelihood, :566-588)
__device__ double cp_cell_likelihood(const bcm3hip_cellpop_data& dl, const double* times, const double* obs,
                                     const double* xv, double scale, double offset, double stdev, double pstd,
                                     double msd)
{
    const int T = dl.T;
    const double mls = -log(stdev);
    const double inv2 = 1.0 / (2.0 * stdev * stdev);
    double lp = 0.0;
    for (int k = 0; k < T; k++) {
        const double y = obs[k];
        if (y != y) continue;
        double x = xv[dl.entry[k]] * scale;
        x += offset;
        if (x != x) {
            double first = times[dl.entry[T - 1]], last = times[dl.entry[0]];
            for (int m = 0; m < T; m++) {
                double z = xv[dl.entry[m]] * scale;
                z += offset;
                if (z == z) {
                    first = times[dl.entry[m]];
                    break;
                }
            }
            for (int m = T - 1; m >= 0; m--) {
                double z = xv[dl.entry[m]] * scale;
                z += offset;
                if (z == z) {
                    last = times[dl.entry[m]];
                    break;
                }
            }
            const double tk = times[dl.entry[k]];
            const double off = fmin(fabs(tk - first), fabs(tk - last));
            lp += (dl.error_model == BCM3HIP_CP_ERR_T4) ? log_pdf_tnu4(off, 0.0, msd) : cp_log_pdf_normal(off, 0.0, msd);
        } else if (dl.error_model == BCM3HIP_CP_ERR_NORMAL) {
            const double dd = y - x;
            lp += mls - 0.91893853320467274178032973640562 - dd * dd * inv2;
        } else if (dl.error_model == BCM3HIP_CP_ERR_T4) {
            lp += log_pdf_tnu4(y, x, stdev);
        } else {
            // (:274-285, 475-483): sigma from the scaled value, -log(sigma), 1 / (2 sigma^2)
            double sigma = pstd * fmax(x, 0.0);
            if (dl.error_model == BCM3HIP_CP_ERR_ADDITIVE_PROPORTIONAL) sigma += stdev;
            const double dd = y - x;
            lp += -log(sigma) - 0.91893853320467274178032973640562 - dd * dd * (1.0 / (2.0 * (sigma * sigma)));
        }
    }
    return lp;
}

// CalculateCellLikelihood with an observed lineage (DataLikelihoodTimeCourse.cpp:431-563): observed
// cell o against simulated cell s (cell index, -1 = "the simulated cell did not divide"), recursing
// into o's observed children (ascending) and s's two simulated daughters, with the reference's
// rules: without a simulated cell every observed point of the subtree takes the missing-value
// penalty at its own time point; a -inf cell stops there; with daughters, either daughter with no
// finite child likelihood gives -inf, one observed child takes the better daughter and two or more
// add nothing (the #if TODO block); without daughters each child's penalty REPLACES the sum (the
// reference assigns instead of adding). Unrolled to 8 generations (the host refuses deeper ones).
struct CpLineage {
    const bcm3hip_cellpop_data* dl;
    const double* times;       // experiment output times (entries)
    const double* xcells;      // this evaluation's cells' entry values [cell][M]
    const int32_t* sim_child;  // this evaluation's cells' first daughters
    int M;
    double scale, offset, stdev, pstd, msd;
};

__device__ inline double cp_missing_at(const CpLineage& c, double t)
{
    // EvaluateMissingValue (DataLikelihoodTimeCourseBase.cpp:301-315)
    return (c.dl->error_model == BCM3HIP_CP_ERR_T4) ? log_pdf_tnu4(t, 0.0, c.msd) : cp_log_pdf_normal(t, 0.0, c.msd);
}

template <int D>
__device__ __attribute__((noinline)) double cp_lineage_likelihood(const CpLineage& c, int o, int s)
{
    if constexpr (D == 0) {
        return __builtin_nan("");
    } else {
        const bcm3hip_cellpop_data& dl = *c.dl;
        const double* obs = dl.observed + (size_t)o * dl.T;
        const int c0 = dl.child_off[o], c1 = dl.child_off[o + 1];
        double lp = 0.0;
        if (s < 0) {
            for (int k = 0; k < dl.T; k++)
                if (obs[k] == obs[k]) lp += cp_missing_at(c, c.times[dl.entry[k]]);
            for (int q = c0; q < c1; q++) lp += cp_lineage_likelihood<D - 1>(c, dl.child_ix[q], -1);
            return lp;
        }
        lp = cp_cell_likelihood(dl, c.times, obs, c.xcells + (size_t)s * c.M, c.scale, c.offset, c.stdev, c.pstd, c.msd);
        if (lp == -__builtin_inf()) return lp;
        if (c1 > c0) {
            const int d0 = c.sim_child[s];
            if (d0 >= 0) {
                int f1 = 0, f2 = 0;
                double a0 = 0.0, b0 = 0.0;
                for (int q = c0; q < c1; q++) {
                    const double a = cp_lineage_likelihood<D - 1>(c, dl.child_ix[q], d0);
                    const double b = cp_lineage_likelihood<D - 1>(c, dl.child_ix[q], d0 + 1);
                    if (a > -__builtin_inf()) f1++;
                    if (b > -__builtin_inf()) f2++;
                    if (q == c0) {
                        a0 = a;
                        b0 = b;
                    }
                }
                if (f1 == 0 || f2 == 0) return -__builtin_inf();
                if (c1 - c0 == 1) lp += (a0 > b0) ? a0 : b0;
            } else {
                for (int q = c0; q < c1; q++) lp = cp_lineage_likelihood<D - 1>(c, dl.child_ix[q], -1);
            }
        }
        return lp;
    }
}

// the cost matrix rows' checks and the matching, on the workspace; lane 0 of the block. Returns
// Evaluate's result (false: a NaN cell likelihood, .cpp:299-302) and the data likelihood's logp
__device__ bool cp_tc_assign(int R, int nsim, const HgWs& w, const uint8_t* row_nan, const int32_t* row_finite,
                             double weight, double* logp, int32_t* match_out)
{
    for (int i = 0; i < R; i++) {  // rows in order: NaN -> failure, then too few finite entries
        if (row_nan[i]) {
            *logp = -__builtin_inf();
            return false;
        }
        if (row_finite[i] < R) {
            *logp = -__builtin_inf();
            return true;
        }
    }
    // n = max(R, nsim); a node without edges (R != nsim) ends the routine (hungarian.cpp:66-71)
    if (R != nsim || !hg_match(R, w)) {
        *logp = -__builtin_inf();
        return true;
    }
    double lp = 0.0;
    for (int i = 0; i < R; i++) {
        lp += -w.cost[(size_t)i * R + w.lmatch[i]];
        if (match_out) match_out[i] = w.lmatch[i];
    }
    *logp = lp * weight;
    return true;
}

// grid (evaluation, data likelihood); blocks of non-time-course data likelihoods return at once
__global__ __launch_bounds__(256) void cp_timecourse_kernel(CpStatic m, int32_t n, const double* values,
                                                             const int32_t* ncells, const int32_t* failed,
                                                             const double* out_values, const int32_t* sim_child,
                                                             unsigned char* ws_global, size_t ws_stride,
                                                             double* tc_logp, int32_t* tc_ok)
{
    extern __shared__ __align__(16) unsigned char cp_lds[];
    const int e = blockIdx.x, di = blockIdx.y;
    const bcm3hip_cellpop_data dl = m.data[di];
    if (dl.kind != BCM3HIP_CP_DATA_TIME_COURSE || e >= n || failed[e]) return;
    // the matched rows: the observed cells without a parent (all of them without a lineage)
    const int R = (dl.n_roots > 0) ? dl.n_roots : dl.R, nsim = ncells[e];
    const int nw = R > nsim ? R : nsim;
    unsigned char* base = ws_global ? ws_global + ((size_t)e * m.n_data + di) * ws_stride : cp_lds;
    const HgWs w = hg_carve(base, nw);
    __shared__ int32_t row_finite[1024];
    __shared__ uint8_t row_nan[1024];
    const double* v = values + (size_t)e * m.d;
    const double offset = cp_ref(dl.offset, v, m.transforms, 0.0);
    const double scale = cp_ref(dl.scale, v, m.transforms, 1.0);
    double stdev = cp_ref(dl.stdev, v, m.transforms, 1.0);
    if (dl.stdev_relative_to_scale) stdev *= scale;
    const double pstd = cp_ref(dl.proportional_stdev, v, m.transforms, 0.0);
    const double msd = cp_ref(dl.missing_stdev, v, m.transforms, 300.0);
    const size_t cbase = (size_t)e * m.max_cells;
    const CpLineage lin{&dl, m.output_times, out_values + cbase * m.M, sim_child + cbase, m.M, scale, offset, stdev, pstd, msd};
    for (int p = threadIdx.x; p < R * nsim; p += blockDim.x) {
        const int i = p / nsim, j = p % nsim;
        // simulated cells with a parent are not matched (.cpp:307-309): the initial cells are the
        // first n0 slots
        double L = -__builtin_inf();
        if (j < m.n0)
            L = (dl.n_roots > 0) ? cp_lineage_likelihood<8>(lin, dl.roots[i], j)
                                 : cp_cell_likelihood(dl, m.output_times, dl.observed + (size_t)i * dl.T,
                                                      out_values + (cbase + j) * m.M, scale, offset, stdev, pstd, msd);
        w.cost[(size_t)i * nw + j] = -L;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < R; i += blockDim.x) {
        int fin = 0;
        uint8_t nan = 0;
        for (int j = 0; j < nsim; j++) {
            const double c = w.cost[(size_t)i * nw + j];
            if (j < m.n0 && c != c) nan = 1;
            fin += (c < __builtin_inf()) ? 1 : 0;
        }
        row_finite[i] = fin;
        row_nan[i] = nan;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    double lp;
    const bool ok = cp_tc_assign(R, nsim, w, row_nan, row_finite, dl.weight, &lp, nullptr);
    tc_logp[(size_t)e * m.n_data + di] = lp;
    tc_ok[(size_t)e * m.n_data + di] = ok ? 1 : 0;
}

hipError_t launch_cp_timecourse(const CpStatic& m, int32_t n, int32_t max_R, const double* values,
                                const int32_t* ncells, const int32_t* failed, const double* out_values,
                                const int32_t* sim_child, unsigned char* ws_global, size_t ws_stride,
                                double* tc_logp, int32_t* tc_ok, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    const size_t lds = ws_global ? 0 : hg_ws_bytes(max_R);
    hipLaunchKernelGGL(cp_timecourse_kernel, dim3(n, m.n_data), dim3(256), lds, s, m, n, values, ncells, failed,
                       out_values, sim_child, ws_global, ws_stride, tc_logp, tc_ok);
    return hipGetLastError();
}

size_t cp_assign_ws_bytes(int n) { return hg_ws_bytes(n); }

// ---------------------------------------------------------------------------------------------
// Time-points data likelihood (DataLikelihoodTimePoints, src/cellpop/DataLikelihoodTimePoints.cpp):
// at every data time point, the observed cells with a finite marker are matched to the simulated
// cells alive then by the same vendored routine; logp = the matched cell likelihoods summed over
// the time points in order, times the weight.

// cell_trajectories[j](ti, l) (NotifySimulatedValue, .cpp:345-370): the column's species values
// summed in notification order, NaN when none was notified (a value is notified when it is not NaN)
__device__ inline double cp_tp_value(const bcm3hip_cellpop_data& dl, const double* xv, int ti, int l)
{
    double v = __builtin_nan("");
    for (int k = dl.term_offset[l]; k < dl.term_offset[l + 1]; k++) {
        const double x = xv[dl.term_entry[(size_t)k * dl.T + ti]];
        if (x == x) v = (v != v) ? x : v + x;
    }
    return v;
}

// the simulated cell j takes part at ti (.cpp:234-239, 351-353)
__device__ inline bool cp_tp_sim(const CpStatic& m, const bcm3hip_cellpop_data& dl, const double* xv, int j, int ti)
{
    if (dl.only_nondivided && j >= m.n0) return false;  // is_newborn: i >= initial_number_of_cells
    if (cp_tp_value(dl, xv, ti, 0) != cp_tp_value(dl, xv, ti, 0)) return false;
    return dl.relative_ix < 0 || cp_tp_value(dl, xv, dl.relative_ix, 0) == cp_tp_value(dl, xv, dl.relative_ix, 0);
}

// observed cell i has a finite marker at ti (observed_data[ti].row(i).isFinite().any())
__device__ inline bool cp_tp_data(const bcm3hip_cellpop_data& dl, int i, int ti)
{
    const double* o = dl.observed + ((size_t)i * dl.T + ti) * dl.MK;
    for (int k = 0; k < dl.MK; k++)
        if (fabs(o[k]) < __builtin_inf()) return true;
    return false;
}

// wavefront 0 lists, in order, the indices i < count with pred(i), at most cap of them; returns how
// many satisfy pred (all of them, also beyond cap)
template <typename F>
__device__ inline int cp_compact(int count, int cap, F pred, int32_t* out)
{
    const int lane = threadIdx.x & 63;
    int total = 0;
    for (int b = 0; b < count; b += 64) {
        const int i = b + lane;
        const bool c = i < count && pred(i);
        const unsigned long long mask = __ballot(c);
        const int pos = total + __popcll(mask & ((1ull << lane) - 1ull));
        if (c && pos < cap) out[pos] = i;
        total += __popcll(mask);
    }
    return total;
}

__global__ __launch_bounds__(256) void cp_timepoints_kernel(CpStatic m, int32_t n, const double* values,
                                                             const int32_t* ncells, const int32_t* failed,
                                                             const double* out_values, unsigned char* ws_global,
                                                             size_t ws_stride, double* tc_logp, int32_t* tc_ok)
{
    extern __shared__ __align__(16) unsigned char cp_lds[];
    const int e = blockIdx.x, di = blockIdx.y;
    const bcm3hip_cellpop_data dl = m.data[di];
    if (dl.kind != BCM3HIP_CP_DATA_TIME_POINTS || e >= n || failed[e]) return;
    __shared__ int32_t rows[1024], sims[1024];
    __shared__ double stdevs[8], offsets[8], scales[8];
    __shared__ int32_t counts[2];
    __shared__ int32_t stop;
    const int nc = ncells[e];
    const double* v = values + (size_t)e * m.d;
    const double* xcells = out_values + (size_t)e * m.max_cells * m.M;
    unsigned char* base = ws_global ? ws_global + ((size_t)e * m.n_data + di) * ws_stride : cp_lds;
    if (threadIdx.x < dl.L) {  // GetCurrentSTDev / DataOffset / DataScale per column (.cpp:212-219)
        const int l = threadIdx.x;
        const double sc = cp_ref(dl.col_ref[3 * l + 2], v, m.transforms, 1.0);
        double sd = cp_ref(dl.col_ref[3 * l], v, m.transforms, 0.0);
        if (dl.stdev_relative_to_scale) sd *= sc;
        stdevs[l] = sd;
        offsets[l] = cp_ref(dl.col_ref[3 * l + 1], v, m.transforms, 0.0);
        scales[l] = sc;
    }
    if (threadIdx.x == 0) stop = 0;
    double lp = 0.0;     // thread 0's running sum
    bool early = false;  // thread 0: Evaluate returned -inf before the weight
    for (int ti = 0; ti < dl.T; ti++) {
        __syncthreads();
        if (threadIdx.x < 64) {
            const int fd = cp_compact(dl.R, dl.R, [&](int i) { return cp_tp_data(dl, i, ti); }, rows);
            const int fs = cp_compact(nc, fd, [&](int j) { return cp_tp_sim(m, dl, xcells + (size_t)j * m.M, j, ti); }, sims);
            if (threadIdx.x == 0) {
                counts[0] = fd;
                counts[1] = fs;
            }
        }
        __syncthreads();
        const int fd = counts[0], fs = counts[1];
        if (fd == 0) continue;
        if (fs < fd) {  // too few simulated cells at this time point: -inf, no weight (.cpp:241-245)
            early = true;
            break;
        }
        // the routine keeps the edges to right nodes < fd only (hungarian.cpp:52-84): the first fd
        // simulated cells of the list
        const HgWs w = hg_carve(base, fd);
        for (int p = threadIdx.x; p < fd * fd; p += blockDim.x) {
            const int i = p / fd, j = p % fd;
            const double* o = dl.observed + ((size_t)rows[i] * dl.T + ti) * dl.MK;
            const double* xv = xcells + (size_t)sims[j] * m.M;
            double cl = 0.0;
            for (int l = 0; l < dl.L; l++) {
                double x = cp_tp_value(dl, xv, ti, l);
                if (dl.relative_ix >= 0) {
                    x += offsets[l];
                    x /= cp_tp_value(dl, xv, dl.relative_ix, l);
                    x *= scales[l];
                } else {
                    x *= scales[l];
                    x += offsets[l];
                }
                const double y = o[l];
                if (y != y) continue;
                cl += (dl.error_model == BCM3HIP_CP_ERR_T4) ? log_pdf_tnu4(y, x, stdevs[l]) : cp_log_pdf_normal(y, x, stdevs[l]);
            }
            w.cost[(size_t)i * fd + j] = -cl;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            if (!hg_match(fd, w)) {  // no perfect matching (.cpp:308-311)
                early = true;
                stop = 1;
            } else {
                for (int i = 0; i < fd; i++) lp += -w.cost[(size_t)i * fd + w.lmatch[i]];
            }
        }
        __syncthreads();
        if (stop) break;
    }
    if (threadIdx.x != 0) return;
    // Evaluate returns true in every case; the weight applies when the loop ran through
    tc_logp[(size_t)e * m.n_data + di] = early ? -__builtin_inf() : lp * dl.weight;
    tc_ok[(size_t)e * m.n_data + di] = 1;
}

hipError_t launch_cp_timepoints(const CpStatic& m, int32_t n, int32_t max_R, const double* values,
                                const int32_t* ncells, const int32_t* failed, const double* out_values,
                                unsigned char* ws_global, size_t ws_stride, double* tc_logp, int32_t* tc_ok,
                                hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    const size_t lds = ws_global ? 0 : hg_ws_bytes(max_R);
    hipLaunchKernelGGL(cp_timepoints_kernel, dim3(n, m.n_data), dim3(256), lds, s, m, n, values, ncells, failed,
                       out_values, ws_global, ws_stride, tc_logp, tc_ok);
    return hipGetLastError();
}

// the matching alone on given cell likelihoods (bcm3hip_assign_cells): one block per problem
__global__ __launch_bounds__(64) void cp_assign_kernel(int32_t R, int32_t nsim, const double* lik,
                                                       unsigned char* ws_global, size_t ws_stride, int32_t* match,
                                                       double* sum, int32_t* ok)
{
    extern __shared__ __align__(16) unsigned char cp_lds[];
    const int p = blockIdx.x;
    const int nw = R > nsim ? R : nsim;
    unsigned char* base = ws_global ? ws_global + (size_t)p * ws_stride : cp_lds;
    const HgWs w = hg_carve(base, nw);
    __shared__ int32_t row_finite[1024];
    __shared__ uint8_t row_nan[1024];
    const double* L = lik + (size_t)p * R * nsim;
    for (int q = threadIdx.x; q < R * nsim; q += blockDim.x) w.cost[(size_t)(q / nsim) * nw + q % nsim] = -L[q];
    __syncthreads();
    for (int i = threadIdx.x; i < R; i += blockDim.x) {
        int fin = 0;
        uint8_t nan = 0;
        for (int j = 0; j < nsim; j++) {
            const double c = w.cost[(size_t)i * nw + j];
            nan |= (c != c) ? 1 : 0;
            fin += (c < __builtin_inf()) ? 1 : 0;
        }
        row_finite[i] = fin;
        row_nan[i] = nan;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int i = 0; i < R; i++) match[(size_t)p * R + i] = -1;
    double lp;
    ok[p] = cp_tc_assign(R, nsim, w, row_nan, row_finite, 1.0, &lp, match + (size_t)p * R) ? 1 : 0;
    sum[p] = lp;
}

hipError_t launch_cp_assign(int32_t n_problems, int32_t R, int32_t nsim, const double* lik, unsigned char* ws_global,
                            size_t ws_stride, int32_t* match, double* sum, int32_t* ok, hipStream_t s)
{
    if (n_problems <= 0) return hipSuccess;
    const int nw = R > nsim ? R : nsim;
    const size_t lds = ws_global ? 0 : hg_ws_bytes(nw);
    hipLaunchKernelGGL(cp_assign_kernel, dim3(n_problems), dim3(64), lds, s, R, nsim, lik, ws_global, ws_stride, match,
                       sum, ok);
    return hipGetLastError();
}

hipError_t launch_cp_init(const CpStatic& m, int32_t n_items, const CpInitItem* items, const double* values,
                          double* params, double* y0, double* creation, const double* end_y, const double* achieved,
                          double* sync_off, hipStream_t s)
{
    if (n_items <= 0) return hipSuccess;
    hipLaunchKernelGGL(cp_init_kernel, dim3((n_items + 127) / 128), dim3(128), 0, s, m, n_items, items, values, params,
                       y0, creation, end_y, achieved, sync_off);
    return hipGetLastError();
}

hipError_t launch_cp_popavg(const CpStatic& m, int32_t n, const double* values, const int32_t* ncells,
                            const int32_t* failed, const double* out_values, const double* creation,
                            const double* sim_end, double* avg, const double* tc_logp, const int32_t* tc_ok,
                            double* logp, int32_t* status, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(cp_popavg_kernel, dim3(n), dim3(64), 0, s, m, n, values, ncells, failed, out_values, creation,
                       sim_end, avg, tc_logp, tc_ok, logp, status);
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

// one workgroup per evaluation: the FIFO numbering level by level -- a generation's cells in cell order,
// each dividing cell's daughters (child_qi, in enqueue order: first, second) appended by a prefix sum
__global__ __launch_bounds__(256) void cp_number_kernel(int32_t max_cells, int32_t n0, const int32_t* first_pos,
                                                        const int32_t* child_qi, const int32_t* failed_eval,
                                                        int32_t* perm, int32_t* ncells, int32_t* failed,
                                                        int32_t* sim_child)
{
    __shared__ int32_t scan[256];
    const int e = blockIdx.x, t = threadIdx.x;
    int32_t* pe = perm + (size_t)e * max_cells;
    int32_t* sc = sim_child + (size_t)e * max_cells;
    for (int i = t; i < n0; i += 256) pe[i] = e * n0 + first_pos[i];
    __syncthreads();
    int lo = 0, hi = n0;
    while (lo < hi) {
        int next = hi;  // the next generation's first slot
        for (int c0 = lo; c0 < hi; c0 += 256) {
            const int j = c0 + t;
            int a = -1, b = -1;
            if (j < hi) {
                const int q = pe[j];
                a = child_qi[2 * q];
                b = child_qi[2 * q + 1];
            }
            const int k = (a >= 0) + (b >= 0);
            scan[t] = k;
            __syncthreads();
            for (int o = 1; o < 256; o <<= 1) {
                const int v = (t >= o) ? scan[t - o] : 0;
                __syncthreads();
                scan[t] += v;
                __syncthreads();
            }
            const int at = next + scan[t] - k;
            if (j < hi) {
                sc[j] = (a >= 0 && at < max_cells) ? at : -1;
                if (a >= 0 && at < max_cells) pe[at] = a;
                if (b >= 0 && at + 1 < max_cells) pe[at + 1] = b;
            }
            next += scan[255];
            __syncthreads();
        }
        lo = hi;
        hi = next < max_cells ? next : max_cells;
    }
    for (int j = hi + t; j < max_cells; j += 256) sc[j] = -1;
    if (t == 0) {
        ncells[e] = hi;
        failed[e] = failed_eval[e];
    }
}

hipError_t launch_cp_number(int32_t n, int32_t max_cells, int32_t n0, const int32_t* first_pos, const int32_t* child_qi,
                            const int32_t* failed_eval, int32_t* perm, int32_t* ncells, int32_t* failed,
                            int32_t* sim_child, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(cp_number_kernel, dim3(n), dim3(256), 0, s, max_cells, n0, first_pos, child_qi, failed_eval, perm,
                       ncells, failed, sim_child);
    return hipGetLastError();
}

// one wavefront per slot, lanes over the cell's entries (coalesced rows)
__global__ __launch_bounds__(256) void cp_permute_kernel(int32_t max_cells, int32_t M, int32_t NS, const int32_t* perm,
                                                         const int32_t* ncells, CpCellArrays src, CpCellArrays dst)
{
    const int e = blockIdx.y;
    const int j = blockIdx.x * 4 + (int)threadIdx.x / 64, ln = (int)threadIdx.x & 63;
    if (j >= ncells[e]) return;
    const size_t d = (size_t)e * max_cells + j, q = (size_t)perm[d];
    for (int k = ln; k < M; k += 64) dst.out_values[d * M + k] = src.out_values[q * M + k];
    for (int k = ln; k < NS; k += 64) dst.end_y[d * NS + k] = src.end_y[q * NS + k];
    if (ln < 5) dst.event_times[d * 5 + ln] = src.event_times[q * 5 + ln];
    if (ln == 0) {
        dst.creation[d] = src.creation[q];
        dst.sim_end[d] = src.sim_end[q];
        dst.achieved[d] = src.achieved[q];
        dst.flags[d] = src.flags[q];
        dst.nsteps[d] = src.nsteps[q];
    }
}

hipError_t launch_cp_permute(int32_t n, int32_t max_cells, int32_t M, int32_t NS, const int32_t* perm,
                             const int32_t* ncells, CpCellArrays src, CpCellArrays dst, hipStream_t s)
{
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(cp_permute_kernel, dim3((max_cells + 3) / 4, n), dim3(256), 0, s, max_cells, M, NS, perm, ncells,
                       src, dst);
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
