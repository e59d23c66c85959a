// expm_pk_kernel.hip -- batched pharmaco_single likelihood on MI355X (gfx950).
//
// Two phases: all matrix exponentials of a launch in parallel (one wavefront per evaluation x
// distinct step length), then one wavefront per evaluation for the state chain. The linear compartment model
// dy/dt = A y is advanced from dose to dose with matrix exponentials exactly as
// PharmacokineticModel::Solve does (src/pharmaco/PharmacokineticModel.cpp:111-177), each
// exp(A t) by Eigen's algorithm (unsupported/Eigen/src/MatrixFunctions/MatrixExponential.h):
// Pade degree 3/5/7/9 chosen by the 1-norm, degree 13 with scaling by 2^-s beyond, the rational
// form solved by an LU with partial pivoting (PartialPivLU's unblocked_lu + its two triangular
// solves), then s squarings.
//
// Layout: the n x n matrices (n <= 16) live in the wavefront's LDS, column-major with a padded
// column stride. Products, linear combinations, scalings and the LU's Schur updates are
// element-parallel (lane L computes entries L, L + 64, ...: all 64 lanes busy for n = 8, each
// entry one dot product of length n); column sums, pivot swaps and the triangular solves of the
// right-hand side stay column-per-lane (lane j owns column j). Every entry is formed by the same
// operations in the same order either way. The exponential of the dose interval is kept and reused
// while the interval repeats (the same bits as recomputing it). HBM traffic per evaluation: the
// parameter vector in, logp / status out; the patient's treatment and observation arrays are
// shared by every wavefront (L2 resident).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <mutex>

#include "pk_math.h"
#include "popk_kernel.h"

const xm::GlibcPow* bcm3_pow_tables(int* from_libm);  // libm_tables.cpp

namespace bcm3hip {
namespace {

constexpr int NM = BCM3HIP_EXPM_NMAX;
constexpr int NP = NM + 1;  // padded column stride (doubles)
using Mat = double[NM][NP];  // [column][row]

struct ExpmShared {
    Mat A, S, A2, A4, A6, U, V, W, E, Eo;
    double y[NM];
    double colsum[NM];
    int perm[NM];
    int fail;
};

__device__ __forceinline__ void wsync() { __syncthreads(); }

// element-parallel sweep: lane L visits the entries L, L + 64, ... of an n x n matrix in
// column-major order, f(column, row); every entry is computed by exactly the arithmetic the
// column-per-lane form used, so results do not depend on which lane computes them
template <class F>
__device__ __forceinline__ void for_elems(int n, int L, F f)
{
    const int nn = n * n;
    for (int e = L; e < nn; e += 64) {
        const int c = e / n;
        f(c, e - c * n);
    }
}

// C = X Y (C distinct from X and Y): C(i,j) = X(i,0) Y(0,j) + ... in ascending k, the order of
// Eigen's coefficient-based product for these sizes
__device__ void matmul(Mat& C, const Mat& X, const Mat& Y, int n, int L)
{
    for_elems(n, L, [&](int j, int i) {
        double acc = X[0][i] * Y[j][0];
        for (int k = 1; k < n; k++) acc = __builtin_fma(X[k][i], Y[j][k], acc);
        C[j][i] = acc;
    });
    wsync();
}

// R = c2 X2 + c1 X1 + c0 X0 + ci I  (left to right, as Eigen evaluates the sum expression);
// X0 may be null (term absent)
__device__ void lincomb(Mat& R, double c2, const Mat& X2, double c1, const Mat& X1, double c0, const Mat* X0,
                        double ci, int n, int L)
{
    for_elems(n, L, [&](int j, int i) {
        double r = c2 * X2[j][i] + c1 * X1[j][i];
        if (X0) r = r + c0 * (*X0)[j][i];
        r = r + ci * (i == j ? 1.0 : 0.0);
        R[j][i] = r;
    });
    wsync();
}

// R += (c2 X2 + c1 X1 + c0 X0 + ci I)
__device__ void lincomb_add(Mat& R, double c2, const Mat& X2, double c1, const Mat& X1, double c0, const Mat& X0,
                            double ci, int n, int L)
{
    for_elems(n, L, [&](int j, int i) {
        double r = c2 * X2[j][i] + c1 * X1[j][i];
        r = r + c0 * X0[j][i];
        r = r + ci * (i == j ? 1.0 : 0.0);
        R[j][i] = R[j][i] + r;
    });
    wsync();
}

// exp(M) into out (M = sh.S is overwritten by the scaling); matrix_exp_compute / computeUV<double>
__device__ void expm(ExpmShared& sh, Mat& out, int n, int j)
{
    // l1norm = max over columns of the column sums of |M|
    if (j < n) {
        double s = 0.0;
        for (int i = 0; i < n; i++) s += fabs(sh.S[j][i]);
        sh.colsum[j] = s;
    }
    wsync();
    double l1 = sh.colsum[0];
    for (int k = 1; k < n; k++) l1 = (sh.colsum[k] > l1) ? sh.colsum[k] : l1;
    int squarings = 0;
    Mat& M = sh.S;
    if (l1 < 1.495585217958292e-002) {
        // pade3: b = {120, 60, 12, 1}
        matmul(sh.A2, M, M, n, j);
        lincomb(sh.W, 1.0, sh.A2, 0.0, sh.A2, 0.0, nullptr, 60.0, n, j);  // b3 A2 + b1 I
        matmul(sh.U, M, sh.W, n, j);
        lincomb(sh.V, 12.0, sh.A2, 0.0, sh.A2, 0.0, nullptr, 120.0, n, j);
    } else if (l1 < 2.539398330063230e-001) {
        // pade5: b = {30240, 15120, 3360, 420, 30, 1}
        matmul(sh.A2, M, M, n, j);
        matmul(sh.A4, sh.A2, sh.A2, n, j);
        lincomb(sh.W, 1.0, sh.A4, 420.0, sh.A2, 0.0, nullptr, 15120.0, n, j);
        matmul(sh.U, M, sh.W, n, j);
        lincomb(sh.V, 30.0, sh.A4, 3360.0, sh.A2, 0.0, nullptr, 30240.0, n, j);
    } else if (l1 < 9.504178996162932e-001) {
        // pade7: b = {17297280, 8648640, 1995840, 277200, 25200, 1512, 56, 1}
        matmul(sh.A2, M, M, n, j);
        matmul(sh.A4, sh.A2, sh.A2, n, j);
        matmul(sh.A6, sh.A4, sh.A2, n, j);
        lincomb(sh.W, 1.0, sh.A6, 1512.0, sh.A4, 277200.0, &sh.A2, 8648640.0, n, j);
        matmul(sh.U, M, sh.W, n, j);
        lincomb(sh.V, 56.0, sh.A6, 25200.0, sh.A4, 1995840.0, &sh.A2, 17297280.0, n, j);
    } else if (l1 < 2.097847961257068e+000) {
        // pade9: b = {17643225600, 8821612800, 2075673600, 302702400, 30270240, 2162160, 110880,
        //             3960, 90, 1}; tmp = b9 A8 + b7 A6 + b5 A4 + b3 A2 + b1 I (A8 in E as scratch)
        matmul(sh.A2, M, M, n, j);
        matmul(sh.A4, sh.A2, sh.A2, n, j);
        matmul(sh.A6, sh.A4, sh.A2, n, j);
        matmul(sh.Eo, sh.A6, sh.A2, n, j);  // A8 (Eo is free until the result is written)
        for_elems(n, j, [&](int j, int i) {
            {
                const double I = (i == j) ? 1.0 : 0.0;
                double t = 1.0 * sh.Eo[j][i] + 3960.0 * sh.A6[j][i];
                t = t + 2162160.0 * sh.A4[j][i];
                t = t + 302702400.0 * sh.A2[j][i];
                t = t + 8821612800.0 * I;
                sh.W[j][i] = t;
                double v = 90.0 * sh.Eo[j][i] + 110880.0 * sh.A6[j][i];
                v = v + 30270240.0 * sh.A4[j][i];
                v = v + 2075673600.0 * sh.A2[j][i];
                v = v + 17643225600.0 * I;
                sh.V[j][i] = v;
            }
        });
        wsync();
        matmul(sh.U, M, sh.W, n, j);
    } else {
        // pade13 on M / 2^s
        int e;
        frexp(l1 / 5.371920351148152, &e);
        squarings = e < 0 ? 0 : e;
        for_elems(n, j, [&](int j, int i) { M[j][i] = ldexp(M[j][i], -squarings); });
        wsync();
        matmul(sh.A2, M, M, n, j);
        matmul(sh.A4, sh.A2, sh.A2, n, j);
        matmul(sh.A6, sh.A4, sh.A2, n, j);
        lincomb(sh.V, 1.0, sh.A6, 16380.0, sh.A4, 40840800.0, &sh.A2, 0.0, n, j);
        matmul(sh.W, sh.A6, sh.V, n, j);
        lincomb_add(sh.W, 33522128640.0, sh.A6, 10559470521600.0, sh.A4, 1187353796428800.0, sh.A2,
                    32382376266240000.0, n, j);
        matmul(sh.U, M, sh.W, n, j);
        lincomb(sh.W, 182.0, sh.A6, 960960.0, sh.A4, 1323241920.0, &sh.A2, 0.0, n, j);
        matmul(sh.V, sh.A6, sh.W, n, j);
        lincomb_add(sh.V, 670442572800.0, sh.A6, 129060195264000.0, sh.A4, 7771770303897600.0, sh.A2,
                    64764752532480000.0, n, j);
    }
    // numer = U + V (into out), denom = -U + V (into W)
    for_elems(n, j, [&](int j, int i) {
        out[j][i] = sh.U[j][i] + sh.V[j][i];
        sh.W[j][i] = -sh.U[j][i] + sh.V[j][i];
    });
    wsync();
    // PartialPivLU (unblocked_lu) of W: pivot = first row of the largest |value| in column k
    Mat& D = sh.W;
    for (int k = 0; k < n; k++) {
        wsync();
        double big = fabs(D[k][k]);
        int row = k;
        for (int i = k + 1; i < n; i++) {
            const double a = fabs(D[k][i]);
            if (a > big) {
                big = a;
                row = i;
            }
        }
        if (j == 0) sh.perm[k] = row;
        if (big != 0.0) {
            if (row != k && j < n) {
                const double t = D[j][k];
                D[j][k] = D[j][row];
                D[j][row] = t;
            }
            wsync();
            const double piv = D[k][k];
            // column k below the pivot /= pivot (l_i), then the Schur update of the columns j > k:
            // every lane forms the same quotients; column k is written after all reads of it
            // (element-parallel over the trailing (n-k-1)^2 block; row k and column k are only read)
            const int m = n - k - 1;
            for_elems(m, j, [&](int c, int r) {
                const int jj = k + 1 + c, i = k + 1 + r;
                D[jj][i] = D[jj][i] - (D[k][i] / piv) * D[jj][k];
            });
            wsync();
            if (j == k)
                for (int i = k + 1; i < n; i++) D[k][i] = D[k][i] / piv;
        }
        wsync();
    }
    // solve: permute the right-hand side rows, unit-lower forward substitution, then upper
    // backward substitution with multiplication by 1/U_ii (TriangularSolverMatrix's column kernel)
    if (j < n) {
        for (int k = 0; k < n; k++) {
            const int r = sh.perm[k];
            if (r != k) {
                const double t = out[j][k];
                out[j][k] = out[j][r];
                out[j][r] = t;
            }
        }
        for (int k = 0; k < n; k++) {
            const double b = out[j][k];
            for (int i = k + 1; i < n; i++) out[j][i] = out[j][i] - b * D[k][i];
        }
        for (int k = n - 1; k >= 0; k--) {
            const double b = out[j][k] * (1.0 / D[k][k]);
            out[j][k] = b;
            for (int i = 0; i < k; i++) out[j][i] = out[j][i] - b * D[k][i];
        }
    }
    wsync();
    // undo the scaling: result *= result
    for (int s = 0; s < squarings; s++) {
        matmul(sh.U, out, out, n, j);
        for_elems(n, j, [&](int j, int i) { out[j][i] = sh.U[j][i]; });
        wsync();
    }
}

// the rates of PharmacoLikelihoodSingle::EvaluateLogProbability (.cpp:153-197), or of patient j in
// PharmacoLikelihoodPopulation::SetupSimulation (PharmacoLikelihoodPopulation.cpp:271-340), into A
// (PharmacokineticModel::ConstructMatrix, .cpp:189-247, in its order of += / -=)
__device__ void construct_matrix(const ExpmPKDevModel& m, const double* v, int j, Mat& A, double& conv,
                                 double& add_sd, double& prop_sd, double& bioavailability)
{
    auto tv = [&](int ix) { return transform_var(m.transforms[ix], v[ix]); };
    add_sd = m.additive_sd_ix >= 0 ? tv(m.additive_sd_ix) : 0.0;
    prop_sd = m.proportional_sd_ix >= 0 ? tv(m.proportional_sd_ix) : 0.0;
    double absorption, clearance, vod, excretion, transit_time = 0.0;
    bioavailability = 1.0;
    if (m.param_map == BCM3HIP_PARAM_MAP_SINGLE) {
        absorption = tv(m.absorption_ix);
        clearance = tv(m.clearance_ix);
        vod = tv(m.vod_ix);
        excretion = m.excretion_ix >= 0 ? tv(m.excretion_ix) : 0.0;
        if (m.n_transit > 0) transit_time = tv(m.mtt_ix);
    } else {
        // mean only: fastpow10(mean); with a random effect: fastpow10(QuantileNormal(p_j, mean, sigma))
        auto pop = [&](int which, int mean_ix) {
            const int s = m.sigma_ix[which];
            if (s < 0) return fastpow10(v[mean_ix]);
            return fastpow10(quantile_normal(v[m.patient_ix[which * m.P + j]], v[mean_ix], v[s]));
        };
        absorption = pop(0, m.absorption_ix);
        excretion = m.excretion_ix >= 0 ? pop(1, m.excretion_ix) : 0.0;
        clearance = pop(2, m.clearance_ix);
        vod = pop(3, m.vod_ix);
        if (m.n_transit > 0) transit_time = (m.sigma_ix[4] < 0) ? tv(m.mtt_ix) : pop(4, m.mtt_ix);
        const int bi = m.patient_ix[5 * m.P + j];
        if (bi >= 0) bioavailability = v[bi];
    }
    const double elimination = clearance / vod;
    conv = (1e6 / m.MW) / vod;
    int nc = 2, mi = -1, ft = 0;
    if (m.peripheral) nc++;
    if (m.metabolite) mi = nc++;
    if (m.n_transit > 0) {
        ft = nc;
        nc += m.n_transit;
    }
    for (int c = 0; c < nc; c++)
        for (int r = 0; r < nc; r++) A[c][r] = 0.0;
    A[0][0] -= excretion;
    A[0][0] -= absorption;
    if (m.n_transit > 0) {
        const int nt = m.n_transit;
        const double tr = (nt + 1.0) / transit_time;
        A[0][ft] += absorption;
        if (nt > 2) {
            for (int i = 0; i < nt - 1; i++) {
                A[ft + i][ft + i] -= tr;
                A[ft + i][ft + i + 1] += tr;
            }
        }
        A[ft + nt - 1][ft + nt - 1] = -tr;
        A[ft + nt - 1][1] += tr;
    } else {
        A[0][1] += absorption;
    }
    if (m.peripheral) {
        const double pf = tv(m.pf_ix), pb = tv(m.pb_ix);
        A[1][1] -= pf;
        A[1][2] += pf;
        A[2][1] += pb;
        A[2][2] -= pb;
    }
    if (m.biphasic) {
        const double da = tv(m.direct_ix);
        A[0][0] -= da;
        A[0][1] += da;
    }
    if (m.metabolite) {
        const double mc = tv(m.metab_conv_ix);
        A[1][1] -= mc;
        A[1][mi] += mc;
        A[mi][mi] -= 1.0;  // SetMetaboliteElimination(1.0) (PharmacoLikelihoodSingle.cpp:140)
    }
    A[1][1] -= elimination;
}

// Phase 1: every matrix exponential of a launch at once. The exponentials of a solve depend on
// the parameters and the schedule only, never on the state, so the host enumerates per patient
// the distinct step lengths the Solve loop will use (job_dt: dose intervals and observation
// offsets, computed with the loop's own subtractions) and one wavefront per (evaluation, job)
// forms exp(A dt) -- n_eval x n_jobs independent waves instead of one sequential chain per
// evaluation. Identical dt values share a job; exp is deterministic, so this is bit-identical to
// recomputing them in the loop. Output: exps[e][job] column-major n x n.
__global__ void __launch_bounds__(64) expm_pk_exp_kernel(ExpmPKDevModel m, int64_t nev,
                                                         const double* __restrict__ values,
                                                         double* __restrict__ exps)
{
    __shared__ ExpmShared sh;
    const int64_t b = blockIdx.x;
    const int64_t e = b / m.n_jobs;
    const int job = (int)(b - e * m.n_jobs);
    if (e >= nev) return;  // uniform per block
    const int L = threadIdx.x;
    const int n = m.n;
    if (L == 0) {
        double c, a, p, ba;
        construct_matrix(m, values + e * m.d, m.job_patient[job], sh.A, c, a, p, ba);
    }
    wsync();
    const double dt = m.job_dt[job];
    for_elems(n, L, [&](int j, int i) { sh.S[j][i] = sh.A[j][i] * dt; });
    wsync();
    expm(sh, sh.E, n, L);
    double* out = exps + b * (int64_t)(n * n);
    for_elems(n, L, [&](int j, int i) { out[j * n + i] = sh.E[j][i]; });
}

// Phase 2: one wavefront per evaluation walks its patients in order: PharmacokineticModel::Solve
// (.cpp:127-174) with the exponentials of phase 1 (lane j = state component j), the observation
// model of PharmacoLikelihoodSingle::EvaluateLogProbability (.cpp:199-215) /
// PharmacoLikelihoodPopulation (.cpp:217-247) folded in, log-likelihoods summed in patient order.
__global__ void __launch_bounds__(64) expm_pk_chain_kernel(ExpmPKDevModel m, int64_t nev,
                                                           const double* __restrict__ values,
                                                           const double* __restrict__ exps,
                                                           double* __restrict__ logp, int32_t* __restrict__ status)
{
    __shared__ Mat A;
    __shared__ double y[NM];
    __shared__ double scal[4];
    __shared__ int fail;
    const int64_t e = blockIdx.x;
    if (e >= nev) return;
    const int j = threadIdx.x;
    const int n = m.n;
    const int nn = n * n;
    const double* v = values + e * m.d;
    const double* ex = exps + e * (int64_t)m.n_jobs * nn;
    double total = 0.0;
    bool any_fail = false;
    for (int pj = 0; pj < m.P; pj++) {
        if (j == 0) {
            double c, a, p, ba;
            construct_matrix(m, v, pj, A, c, a, p, ba);
            scal[0] = c;
            scal[1] = a;
            scal[2] = p;
            scal[3] = ba;
            fail = 0;
        }
        if (j < n) y[j] = 0.0;
        wsync();
        const double conv = scal[0], add_sd = scal[1], prop_sd = scal[2], bioavailability = scal[3];
        const int t0 = m.treat_offset[pj], n_treat = m.treat_offset[pj + 1] - t0;
        const int o0 = m.obs_offset[pj], n_obs = m.obs_offset[pj + 1] - o0;
        const double* treat_times = m.treat_times + t0;
        const double* treat_doses = m.treat_doses + t0;
        const double* obs_times = m.obs_times + o0;
        const double* obs_conc = m.obs_conc + o0;
        const double simulate_until = obs_times[n_obs - 1];
        double llh = 0.0;
        bool llh_done = false;
        int tti = 0, oti = 0;
        double current_t = 0.0;
        while (tti < n_treat && current_t < simulate_until) {
            const double target_t = (tti < n_treat - 1) ? treat_times[tti + 1] : simulate_until;
            if (j == 0) y[0] += treat_doses[tti] * bioavailability;
            wsync();
            while (oti < n_obs && obs_times[oti] <= target_t) {
                const double* Eo = ex + (int64_t)m.obs_job[o0 + oti] * nn;  // [col][row]
                double c = Eo[1] * y[0];
                for (int k = 1; k < n; k++) c = __builtin_fma(Eo[k * n + 1], y[k], c);
                if (!llh_done) {
                    const double x = conv * c;
                    if (isnan(x) || isinf(x)) {
                        llh = -INFINITY;
                        llh_done = true;
                    } else {
                        const double yobs = obs_conc[oti];
                        if (!isnan(yobs)) llh += log_pdf_tnu4(x, yobs, add_sd + prop_sd * fmax(x, 0.0));
                    }
                }
                oti++;
            }
            const double* E = ex + (int64_t)m.interval_job[t0 + tti] * nn;
            double ynew = 0.0;
            if (j < n) {
                ynew = E[j] * y[0];
                for (int k = 1; k < n; k++) ynew = __builtin_fma(E[k * n + j], y[k], ynew);
            }
            wsync();
            if (j < n) {
                y[j] = ynew;
                if (isnan(ynew)) fail = 1;
            }
            wsync();
            if (fail) break;
            current_t = target_t;
            tti++;
        }
        const bool f = fail != 0;
        total += f ? -INFINITY : llh;
        any_fail = any_fail || f;
        wsync();
    }
    if (j == 0) {
        logp[e] = total;
        if (status) status[e] = any_fail ? BCM3HIP_STATUS_SOLVER_FAIL : BCM3HIP_STATUS_OK;
    }
}

}  // namespace

// this translation unit's copy of the libm tables (libm_exact.h xm_tables: glibc's exp in the
// parameter maps), once per device
hipError_t expm_prepare_device()
{
    static std::mutex mu;
    static bool done[64] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(mu);
    if (dev >= 0 && dev < 64 && done[dev]) return hipSuccess;
    e = hipMemcpyToSymbol(HIP_SYMBOL(xm::xm_tables), bcm3_pow_tables(nullptr), sizeof(xm::GlibcPow));
    if (e == hipSuccess && dev >= 0 && dev < 64) done[dev] = true;
    return e;
}

hipError_t launch_expm_pk(const ExpmPKDevModel& m, int64_t n, const double* values, double* logp, int32_t* status,
                          double* exps, hipStream_t stream, hipEvent_t ev_start, hipEvent_t ev_stop)
{
    if (n == 0) return hipSuccess;
    if (ev_start) hipEventRecord(ev_start, stream);
    if (m.n_jobs > 0)  // (none when every observation is at t = 0: the Solve loop never runs)
        hipLaunchKernelGGL(expm_pk_exp_kernel, dim3((unsigned)(n * m.n_jobs)), dim3(64), 0, stream, m, n, values,
                           exps);
    hipLaunchKernelGGL(expm_pk_chain_kernel, dim3((unsigned)n), dim3(64), 0, stream, m, n, values, exps, logp, status);
    const hipError_t e = hipGetLastError();
    if (ev_stop) hipEventRecord(ev_stop, stream);
    return e;
}

}  // namespace bcm3hip
