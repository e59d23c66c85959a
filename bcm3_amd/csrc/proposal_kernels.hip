// proposal_kernels.hip -- the adaptive proposals of SamplerPTChain::MutateMove (one_block blocking,
// src/sampler/SamplerPTChain.cpp:241-310) as HIP kernels over all chains of a rank, with the
// proposal state resident in HBM (bcm3hip_proposal, include/bcm3hip.h):
//
//   ptmh_propose_adaptive_kernel  Proposal::Update, GetNewSample (+ ReflectOnBounds), the prior of
//                                 the new point and CalculateMHRatio, for
//       global_covariance  ProposalGlobalCovariance (ProposalGlobalCovariance.cpp:20-47) with the
//                          base Proposal::Update (Proposal.cpp:197-208);
//       gaussian_mixture   ProposalGaussianMixture (ProposalGaussianMixture.cpp:20-99): component
//                          chosen by the responsibilities of the current point (GMM.cpp:172-186),
//                          per-component scale adaptation, MH ratio of the mixture densities;
//     T == 0 chains draw from the prior (SamplerPTChain.cpp:221-240);
//   ptmh_accept_adaptive_kernel   TestSample with the MH ratio (SamplerPTChain.cpp:465-481), the
//                                 state update and Proposal::NotifyAccepted (Proposal.cpp:210-220,
//                                 ProposalGaussianMixture.cpp:91-103);
//   history_add_kernel            SampleHistory::AddSample (SampleHistory.cpp:32-45) after a mutate
//                                 move (SamplerPTChain.cpp:309) or an exchange move (:374-379).
//
// One thread per chain: the per-chain work is O(K d^2) sequential triangular algebra on small
// matrices (d = 12 for the PopPK configs), a few microseconds against the millisecond likelihood
// launch between propose and accept. Arithmetic follows the reference's expressions in order
// (sequential sums, no contraction: the library is built with -ffp-contract=off), so
// tests/proposal_reference.py restates it operation for operation.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "../../include/bcm3hip.h"
#include "ctr_rng.h"
#include "prior_marginal.h"
#include "pt_exchange.h"

namespace bcm3hip {
namespace {

using rng::normal01;
using rng::rng_key;
using rng::u01;

// MathFunctions.h:67-82 (boost::math::log1p -> log1p)
__device__ double logsum2(double loga, double logb)
{
    if (logb > loga) {
        const double t = loga;
        loga = logb;
        logb = t;
    }
    if (loga == -INFINITY) return loga;
    const double diff = logb - loga;
    if (diff < -500) return loga;
    return loga + log1p(exp(diff));
}

// Proposal::ReflectOnBounds (Proposal.cpp:384-397); bounded to 4096 reflections (a proposal that
// far outside is then folded in one step -- never reached by proposals within ~10^3 ranges)
__device__ double reflect(double x, double lb, double ub)
{
    for (int it = 0; it < 4096; it++) {
        if (x < lb)
            x = lb + (lb - x);
        else if (x > ub)
            x = ub - (x - ub);
        else
            return x;
    }
    const double w = ub - lb;
    double r = fmod(x - lb, 2.0 * w);
    if (r < 0.0) r += 2.0 * w;
    return (r <= w) ? lb + r : ub - (r - w);
}

// L s = v in place (Eigen matrixL().solveInPlace): forward substitution, sequential sums
__device__ __forceinline__ void lower_solve(int d, const double* L, double* v)
{
    for (int i = 0; i < d; i++)
    {
        double acc = 0.0;
        for (int j = 0; j < i; j++) acc += L[i * d + j] * v[j];
        v[i] = (v[i] - acc) / L[i * d + i];
    }
}

__device__ __forceinline__ double dot(int d, const double* a)
{
    double s = 0.0;
    for (int i = 0; i < d; i++) s += a[i] * a[i];
    return s;
}

// GMM::CalculateResponsibilities (GMM.cpp:172-186) with GMM::LogPdfMVN (:392-398) and
// logsum(VectorReal) (MathFunctions.h:84-92)
__device__ __forceinline__ void responsibilities(int K, int d, const double* x, const double* mean,
                                                 const double* chol, const double* logc, const double* w, double* r,
                                                 double* tmp)
{
    for (int k = 0; k < K; k++)
    {
        for (int i = 0; i < d; i++) tmp[i] = x[i] - mean[k * d + i];
        lower_solve(d, chol + (int64_t)k * d * d, tmp);
        r[k] = (logc[k] - 0.5 * dot(d, tmp)) + log(w[k]);
    }
    double m = r[0];
    for (int k = 0; k < K; k++) m = (r[k] > m) ? r[k] : m;
    double sum = 0.0;
    for (int k = 0; k < K; k++) sum += exp(r[k] - m);
    const double lsum = log(sum) + m;
    double tot = 0.0;
    for (int k = 0; k < K; k++)
    {
        r[k] = exp(r[k] - lsum);
        tot += r[k];
    }
    for (int k = 0; k < K; k++) r[k] = r[k] / tot;
}

// RNG::GetGamma(k, theta) (RNG.cpp:84-111), Marsaglia-Tsang, normals by Box-Muller
__device__ double gamma_draw(double k, double theta, uint64_t seed, uint64_t iter, uint64_t gc)
{
    double scale_u = 1.0;
    if (k < 1.0) {
        const double u = u01(rng_key(seed, iter, gc, rng::KEY_GAMMA_SMALLK));
        scale_u = pow(u, 1.0 / k);
        k = 1.0 + k;
    }
    const double dd = k - 0.33333333333333333333333333333333;
    const double c = 0.33333333333333333333333333333333 / sqrt(dd);
    int ni = 0, ui = 0;
    double v = 1.0;
    while (ni < 0x800 && ui < 0x800) {
        double x;
        do {
            x = normal01(seed, iter, gc, rng::SLOT_GAMMA_NORMAL + ni);
            ni++;
            v = 1.0 + c * x;
        } while (v <= 0.0 && ni < 0x800);
        v = v * v * v;
        const double u = u01(rng_key(seed, iter, gc, rng::KEY_GAMMA_UNIFORM + ui));
        ui++;
        if (u < 1 - 0.0331 * x * x * x * x) break;
        if (log(u) < 0.5 * x * x + dd * (1 - v + log(v))) break;
    }
    return theta * dd * v * scale_u;
}


// one chain of ptmh_propose_adaptive (see the file header); v, t: [d], rf, rr: [K] scratch
__device__ __forceinline__ void propose_chain(int c, int d, const int32_t* __restrict__ kind,
                                              const double* __restrict__ p0, const double* __restrict__ p1,
                                              const double* __restrict__ p2, const double* __restrict__ temps, const double* __restrict__ values,
                                              double* __restrict__ prop, double* __restrict__ lprior_prop,
                                              double* __restrict__ log_mh, const bcm3hip_proposal& P, uint64_t gc,
                                              uint64_t seed, uint64_t iter, double* v, double* t, double* rf,
                                              double* rr)
{
    const double* cur = values + (int64_t)c * d;
    double* nxt = prop + (int64_t)c * d;
    double lmh = 0.0;
    const bool dir = prior::has_dirichlet(d, kind);
    if (temps[c] == 0.0) {
        // PriorIndependence::Sample (PriorIndependence.cpp:158-178)
        for (int i = 0; i < d; i++) nxt[i] = prior::sample(kind[i], p0[i], p1[i], p2[i], seed, iter, gc, i);
        if (dir) {
            for (int f = 0; f < d; f++) {
                if (kind[f] != BCM3HIP_PRIOR_DIRICHLET || (int)p1[f] != f) continue;
                const int l = prior::dirichlet_last(d, kind, p1, f);
                double sum = 0.0;
                for (int j = f; j <= l; j++) sum += nxt[j];
                const double inv = 1.0 / sum;
                for (int j = f; j <= l; j++) nxt[j] *= inv;
            }
        }
    } else {
        const int Km = P.kmax;
        int K = (P.kind == BCM3HIP_PROPOSAL_GAUSSIAN_MIXTURE) ? P.ncomp[c] : 1;
        K = (K < 1) ? 1 : ((K > Km) ? Km : K);
        double* scale = P.scale + (int64_t)c * Km;
        double* ema = P.ema + (int64_t)c * Km;
        const double* mean = P.mean + (int64_t)c * Km * d;
        const double* chol = P.chol + (int64_t)c * Km * d * d;
        const double* logc = P.logc + (int64_t)c * Km;
        const double* w = P.weights + (int64_t)c * Km;
        const double slr = P.scaling_learning_rate;
        const double target = P.target_acceptance;
        int sel;
        if (P.kind == BCM3HIP_PROPOSAL_GAUSSIAN_MIXTURE) {
            // ProposalGaussianMixture::Update: only the component used last
            const int last = P.selected[c];
            if (last != -1) {
                const double lrate = 1.0 + u01(rng_key(seed, iter, gc, rng::KEY_UPDATE)) * slr * K;
                if (ema[last] < target / (1.0 - slr)) {
                    scale[last] /= lrate;
                    scale[last] = (scale[last] > 1e-4) ? scale[last] : 1e-4;
                } else if (ema[last] > (1 + slr) * target) {
                    scale[last] *= lrate;
                    scale[last] = (scale[last] < 10.0) ? scale[last] : 10.0;
                }
            }
            // the current point's values in v (read once)
            for (int i = 0; i < d; i++) v[i] = cur[i];
            responsibilities(K, d, v, mean, chol, logc, w, rf, t);
            // RNG::Sample (RNG.cpp:41-56)
            const double u = u01(rng_key(seed, iter, gc, rng::KEY_SELECT));
            double acc = 0.0;
            sel = K - 1;
            bool found = false;
            for (int k = 0; k < K; k++)
            {
                acc += rf[k];
                if (!found && u < acc) {
                    sel = k;
                    found = true;
                }
            }
        } else {
            // Proposal::Update (base class)
            const double lrate = 1.0 + u01(rng_key(seed, iter, gc, rng::KEY_UPDATE)) * slr;
            if (ema[0] < 0.952381 * target) {
                scale[0] /= lrate;
                scale[0] = (scale[0] > 1e-4) ? scale[0] : 1e-4;
            } else if (ema[0] > 1.05 * target) {
                scale[0] *= lrate;
                scale[0] = (scale[0] < 10.0) ? scale[0] : 10.0;
            }
            sel = 0;
        }
        double t_scale = 1.0;
        if (P.t_dof > 0.0) {
            const double wg = gamma_draw(0.5 * P.t_dof, 0.5 * P.t_dof, seed, iter, gc);
            t_scale = 1.0 / sqrt(wg);  // bcm3::rsqrt (MathFunctions.h:35-48) to full precision
        }
        // x = L z, x *= t_scale * scale, new = x + current, reflected on the prior bounds
        const double* Ls = chol + (int64_t)sel * d * d;
        for (int i = 0; i < d; i++) t[i] = normal01(seed, iter, gc, i);
        const double f = t_scale * scale[sel];
        for (int i = 0; i < d; i++)
        {
            double x = 0.0;
            for (int j = 0; j < i + 1; j++) x += Ls[i * d + j] * t[j];
            v[i] = reflect(x * f + cur[i], P.lower[i], P.upper[i]);
        }
        if (P.kind == BCM3HIP_PROPOSAL_GAUSSIAN_MIXTURE) {
            // ProposalGaussianMixture::CalculateMHRatio; v holds the new point, t is scratch
            responsibilities(K, d, v, mean, chol, logc, w, rr, t);
            double fwd = -INFINITY, rev = -INFINITY;
            for (int k = 0; k < K; k++)
            {
                const double* Lk = chol + (int64_t)k * d * d;
                const double sk = scale[k];
                // forward: L s = (new - cur) / s_k; reverse: L s = -(new - cur) / s_k = -s
                for (int i = 0; i < d; i++) t[i] = (v[i] - cur[i]) / sk;
                lower_solve(d, Lk, t);
                const double base = -log(sk * sk) + logc[k];
                const double q = 0.5 * dot(d, t);  // the reverse solution is -t: same square sum
                fwd = logsum2(fwd, (base - q) + log(rf[k]));
                rev = logsum2(rev, (base - q) + log(rr[k]));
            }
            lmh = rev - fwd;
        }
        for (int i = 0; i < d; i++) nxt[i] = v[i];
        // Dirichlet residual: the group's last member := 1 - sum(others) after the MH ratio of the
        // unmodified proposal (SamplerPTChain.cpp:270-278, 295)
        if (dir) {
            for (int f = 0; f < d; f++) {
                if (kind[f] != BCM3HIP_PRIOR_DIRICHLET || (int)p1[f] != f) continue;
                const int l = prior::dirichlet_last(d, kind, p1, f);
                double sum = 0.0;
                for (int j = f; j < l; j++) sum += nxt[j];
                nxt[l] = 1.0 - sum;
            }
        }
        P.selected[c] = sel;
    }
    // PriorIndependence::EvaluateLogPDF (PriorIndependence.cpp:129-157): multivariate groups first,
    // then the univariate marginals in variable order
    double lp = 0.0;
    if (dir) {
        for (int f = 0; f < d; f++)
            if (kind[f] == BCM3HIP_PRIOR_DIRICHLET && (int)p1[f] == f)
                lp += prior::dirichlet_log_pdf(f, prior::dirichlet_last(d, kind, p1, f), p0, p2[f],
                                               [&](int j) { return nxt[j]; });
    }
    for (int i = 0; i < d; i++)
        if (kind[i] != BCM3HIP_PRIOR_DIRICHLET) lp += prior::log_pdf(kind[i], p0[i], p1[i], p2[i], nxt[i]);
    lprior_prop[c] = lp;
    log_mh[c] = lmh;
}

// ---- one wavefront per chain, lane i = variable i (d <= 64) ----
// The same arithmetic as propose_chain, element for element: the triangular solve runs in its
// column form (after s_j is known, every row i > j adds L_ij s_j), which accumulates each row's
// sum in the same j order as the row form; sums over variables / components run sequentially
// over lanes (readlane chains), so the results are those of the thread-per-chain kernel.

__device__ __forceinline__ double lane_bcast(double x, int j)  // x of lane j (j wave-uniform)
{
    const long long b = __builtin_bit_cast(long long, x);
    const int lo = __builtin_amdgcn_readlane((int)b, j);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), j);
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// generic form, any d <= 64
__device__ __forceinline__ double wave_lower_solve_any(int d, const double* Lrow, double v, int lane)
{
    double acc = 0.0, s = 0.0;
    for (int j = 0; j < d; j++) {
        if (lane == j) s = (v - acc) / Lrow[j];
        const double sj = lane_bcast(s, j);
        if (lane > j && lane < d) acc += Lrow[j] * sj;
    }
    return s;
}

// d <= MD: the lane's row is loaded into registers first (every row pointer is valid -- lanes >= d
// read row 0 -- and indices are clamped, so the loads are unconditional and issue back to back),
// so the dependent division -> broadcast chain waits on memory once, not once per column. The same
// arithmetic, in the same order, as wave_lower_solve_any.
template <int MD>
__device__ __forceinline__ double wave_lower_solve_reg(int d, const double* Lrow, double v, int lane)
{
    double L[MD];
#pragma unroll
    for (int j = 0; j < MD; j++) L[j] = Lrow[(j < d) ? j : d - 1];
    double acc = 0.0, s = 0.0;
#pragma unroll
    for (int j = 0; j < MD; j++) {
        if (j >= d) break;
        if (lane == j) s = (v - acc) / L[j];
        const double sj = lane_bcast(s, j);
        if (lane > j && lane < d) acc += L[j] * sj;
    }
    return s;
}

// two right-hand sides with the same L (the proposal's reverse-responsibility and MH solves of
// one component): two independent division -> broadcast chains in one pass over the columns,
// each with exactly the arithmetic of wave_lower_solve
template <int MD>
__device__ __forceinline__ void wave_lower_solve2_reg(int d, const double* Lrow, double va, double vb, int lane,
                                                      double& sa_out, double& sb_out)
{
    double L[MD];
#pragma unroll
    for (int j = 0; j < MD; j++) L[j] = Lrow[(j < d) ? j : d - 1];
    double acca = 0.0, accb = 0.0, sa = 0.0, sb = 0.0;
#pragma unroll
    for (int j = 0; j < MD; j++) {
        if (j >= d) break;
        if (lane == j) {
            sa = (va - acca) / L[j];
            sb = (vb - accb) / L[j];
        }
        const double saj = lane_bcast(sa, j);
        const double sbj = lane_bcast(sb, j);
        if (lane > j && lane < d) {
            acca += L[j] * saj;
            accb += L[j] * sbj;
        }
    }
    sa_out = sa;
    sb_out = sb;
}

// lane i (< d) holds v_i and row i of L (Lrow); returns s_i of L s = v
__device__ __forceinline__ double wave_lower_solve(int d, const double* Lrow, double v, int lane)
{
    if (d <= 16) return wave_lower_solve_reg<16>(d, Lrow, v, lane);
    return wave_lower_solve_any(d, Lrow, v, lane);
}

// sum_{i<n} x_i in lane order (uniform result)
__device__ __forceinline__ double wave_seq_sum(int n, double x)
{
    double s = 0.0;
    for (int i = 0; i < n; i++) s += lane_bcast(x, i);
    return s;
}

// lane k holds log(w_k N_k(x)); returns the responsibility r_k in lane k and the mixture's
// log-density in lsum_out (GMM::CalculateResponsibilities' log-sum-exp, components in order)
__device__ __forceinline__ double wave_normalize_resp(int K, double r, double& lsum_out)
{
    double m = lane_bcast(r, 0);
    for (int k = 1; k < K; k++) {
        const double rk = lane_bcast(r, k);
        m = (rk > m) ? rk : m;
    }
    double sum = 0.0;
    for (int k = 0; k < K; k++) sum += exp(lane_bcast(r, k) - m);
    const double lsum = log(sum) + m;
    const double e = exp(r - lsum);
    const double tot = wave_seq_sum(K, e);
    lsum_out = lsum;
    return e / tot;
}

// responsibilities of the point x (lane i = x_i); lane k of the result = r_k; lsum = the mixture's
// log-density log sum_k w_k N(x; mean_k, L_k L_k^T) (logsum of GMM::CalculateResponsibilities)
__device__ __forceinline__ double wave_responsibilities_lsum(int K, int d, double x, const double* mean,
                                                             const double* chol, const double* logc,
                                                             const double* w, int lane, double& lsum_out)
{
    double r = 0.0;
    for (int k = 0; k < K; k++) {
        const double t0 = (lane < d) ? x - mean[k * d + lane] : 0.0;
        const double t = wave_lower_solve(d, chol + (int64_t)k * d * d + (int64_t)((lane < d) ? lane : 0) * d, t0,
                                          lane);
        const double rk = (logc[k] - 0.5 * wave_seq_sum(d, (lane < d) ? t * t : 0.0)) + log(w[k]);
        r = (lane == k) ? rk : r;
    }
    return wave_normalize_resp(K, r, lsum_out);
}

__device__ __forceinline__ double wave_responsibilities(int K, int d, double x, const double* mean,
                                                        const double* chol, const double* logc, const double* w,
                                                        int lane)
{
    double lsum;
    return wave_responsibilities_lsum(K, d, x, mean, chol, logc, w, lane, lsum);
}

// bcm3hip_gmm_eval: the propose kernel's mixture arithmetic (wave_responsibilities_lsum) at n
// points, one wavefront per point -- the hook that pins the device proposal density to the
// reference's GMM / dmvnormal golden values (tests/stats/GMM.cpp, tests/stats/mvn.cpp)
__global__ void __launch_bounds__(64) gmm_eval_wave_kernel(int n, int d, int K, const double* __restrict__ X,
                                                           const double* __restrict__ mean,
                                                           const double* __restrict__ chol,
                                                           const double* __restrict__ logc,
                                                           const double* __restrict__ w, double* __restrict__ logpdf,
                                                           double* __restrict__ resp)
{
    const int lane = threadIdx.x & 63;
    const int p = __builtin_amdgcn_readfirstlane((int)blockIdx.x);
    if (p >= n) return;
    const double x = (lane < d) ? X[(int64_t)p * d + lane] : 0.0;
    double lsum;
    const double r = wave_responsibilities_lsum(K, d, x, mean, chol, logc, w, lane, lsum);
    if (resp && lane < K) resp[(int64_t)p * K + lane] = r;
    if (logpdf && lane == 0) logpdf[p] = lsum;
}

// One chain's proposal (see ptmh_propose_wave_kernel). cur_row: the point proposed from. SPEC = false:
// the proposal state is updated in place (Proposal::Update's scale, the selected component), the
// results go to out_row / *lprior_out / *log_mh_out. SPEC = true (speculative candidates for the next
// iteration, ptmh_spec_candidates_kernel): the acceptance EMA of the component Update reads is
// ema_last (the value the accept step leaves for an assumed outcome), and instead of writing the
// proposal state the kernel reports what the sequential propose would write: *sel_out (selected
// component), *upd_out / *sc_out (the scale Update's component, -1 for none, and its new value).
template <bool SPEC>
__device__ __forceinline__ void propose_wave_one(int c, int d, const int32_t* __restrict__ kind,
                                                 const double* __restrict__ p0, const double* __restrict__ p1,
                                                 const double* __restrict__ p2, const double* __restrict__ temps,
                                                 const double* __restrict__ cur_row, double ema_last,
                                                 double* __restrict__ out_row, double* __restrict__ lprior_out,
                                                 double* __restrict__ log_mh_out, const bcm3hip_proposal& P,
                                                 uint64_t gc, uint64_t seed, uint64_t iter, int32_t* sel_out,
                                                 int32_t* upd_out, double* sc_out)
{
    const int lane = threadIdx.x & 63;
    const bool on = lane < d;
    const int li = on ? lane : 0;
    const double cur = cur_row[li];
    double nxt;
    double lmh = 0.0;
    const bool dir = prior::has_dirichlet(d, kind);
    if (temps[c] == 0.0) {
        nxt = prior::sample(kind[li], p0[li], p1[li], p2[li], seed, iter, gc, li);
        if (dir) {
            // MultivariateMarginal::Sample: each member's Gamma draw over the group's sum
            for (int f = 0; f < d; f++) {
                if (kind[f] != BCM3HIP_PRIOR_DIRICHLET || (int)p1[f] != f) continue;
                const int l = prior::dirichlet_last(d, kind, p1, f);
                double sum = 0.0;
                for (int j = f; j <= l; j++) sum += lane_bcast(nxt, j);
                const double inv = 1.0 / sum;
                if (lane >= f && lane <= l) nxt *= inv;
            }
        }
    } else {
        const int Km = P.kmax;
        int K = (P.kind == BCM3HIP_PROPOSAL_GAUSSIAN_MIXTURE) ? P.ncomp[c] : 1;
        K = (K < 1) ? 1 : ((K > Km) ? Km : K);
        double* scale = P.scale + (int64_t)c * Km;
        double* ema = P.ema + (int64_t)c * Km;
        const double* mean = P.mean + (int64_t)c * Km * d;
        const double* chol = P.chol + (int64_t)c * Km * d * d;
        const double* logc = P.logc + (int64_t)c * Km;
        const double* w = P.weights + (int64_t)c * Km;
        const double slr = P.scaling_learning_rate;
        const double target = P.target_acceptance;
        int sel;
        double rf = 0.0;
        // the scale Update changes (component upd, new value sc): kept in registers, since other
        // lanes read it after lane 0's store
        int upd = -1;
        double sc = 0.0;
        if (P.kind == BCM3HIP_PROPOSAL_GAUSSIAN_MIXTURE) {
            const int last = P.selected[c];
            if (last != -1) {
                const double lrate = 1.0 + u01(rng_key(seed, iter, gc, rng::KEY_UPDATE)) * slr * K;
                sc = scale[last];
                const double e = SPEC ? ema_last : ema[last];
                if (e < target / (1.0 - slr)) {
                    sc /= lrate;
                    sc = (sc > 1e-4) ? sc : 1e-4;
                } else if (e > (1 + slr) * target) {
                    sc *= lrate;
                    sc = (sc < 10.0) ? sc : 10.0;
                }
                if (!SPEC && lane == 0) scale[last] = sc;
                upd = last;
            }
            rf = wave_responsibilities(K, d, cur, mean, chol, logc, w, lane);
            const double u = u01(rng_key(seed, iter, gc, rng::KEY_SELECT));
            double acc = 0.0;
            sel = K - 1;
            for (int k = 0; k < K; k++) {
                acc += lane_bcast(rf, k);
                if (u < acc) {
                    sel = k;
                    break;
                }
            }
        } else {
            const double lrate = 1.0 + u01(rng_key(seed, iter, gc, rng::KEY_UPDATE)) * slr;
            sc = scale[0];
            const double e = SPEC ? ema_last : ema[0];
            if (e < 0.952381 * target) {
                sc /= lrate;
                sc = (sc > 1e-4) ? sc : 1e-4;
            } else if (e > 1.05 * target) {
                sc *= lrate;
                sc = (sc < 10.0) ? sc : 10.0;
            }
            if (!SPEC && lane == 0) scale[0] = sc;
            upd = 0;
            sel = 0;
        }
        double t_scale = 1.0;
        if (P.t_dof > 0.0) {
            const double wg = gamma_draw(0.5 * P.t_dof, 0.5 * P.t_dof, seed, iter, gc);
            t_scale = 1.0 / sqrt(wg);
        }
        const double* Ls = chol + (int64_t)sel * d * d + (int64_t)li * d;
        const double z = normal01(seed, iter, gc, li);
        const double f = t_scale * ((sel == upd) ? sc : scale[sel]);
        double x = 0.0;
        for (int j = 0; j < d; j++) {
            const double zj = lane_bcast(z, j);
            const double a = x + Ls[j] * zj;  // Ls: this lane's row (row 0 for lanes >= d)
            x = (j <= lane) ? a : x;
        }
        nxt = reflect(x * f + cur, P.lower[li], P.upper[li]);
        if (P.kind == BCM3HIP_PROPOSAL_GAUSSIAN_MIXTURE && d <= 16) {
            // the reverse responsibilities at nxt and the MH solve of component k use the same
            // L_k: one pass solves both (values as in the branch below, bit for bit)
            double r = 0.0, qv = 0.0;
            for (int k = 0; k < K; k++) {
                const double sk = (k == upd) ? sc : scale[k];
                const double ta0 = on ? nxt - mean[k * d + lane] : 0.0;
                const double tb0 = on ? (nxt - cur) / sk : 0.0;
                double ta, tb;
                wave_lower_solve2_reg<16>(d, chol + (int64_t)k * d * d + (int64_t)li * d, ta0, tb0, lane, ta, tb);
                const double rk = (logc[k] - 0.5 * wave_seq_sum(d, on ? ta * ta : 0.0)) + log(w[k]);
                r = (lane == k) ? rk : r;
                const double q = 0.5 * wave_seq_sum(d, on ? tb * tb : 0.0);
                qv = (lane == k) ? q : qv;
            }
            double lsum;
            const double rr = wave_normalize_resp(K, r, lsum);
            double fwd = -INFINITY, rev = -INFINITY;
            for (int k = 0; k < K; k++) {
                const double sk = (k == upd) ? sc : scale[k];
                const double base = -log(sk * sk) + logc[k];
                const double q = lane_bcast(qv, k);
                fwd = logsum2(fwd, (base - q) + log(lane_bcast(rf, k)));
                rev = logsum2(rev, (base - q) + log(lane_bcast(rr, k)));
            }
            lmh = rev - fwd;
        } else if (P.kind == BCM3HIP_PROPOSAL_GAUSSIAN_MIXTURE) {
            const double rr = wave_responsibilities(K, d, nxt, mean, chol, logc, w, lane);
            double fwd = -INFINITY, rev = -INFINITY;
            for (int k = 0; k < K; k++) {
                const double sk = (k == upd) ? sc : scale[k];
                const double t0 = on ? (nxt - cur) / sk : 0.0;
                const double t = wave_lower_solve(d, chol + (int64_t)k * d * d + (int64_t)li * d, t0, lane);
                const double base = -log(sk * sk) + logc[k];
                const double q = 0.5 * wave_seq_sum(d, on ? t * t : 0.0);
                fwd = logsum2(fwd, (base - q) + log(lane_bcast(rf, k)));
                rev = logsum2(rev, (base - q) + log(lane_bcast(rr, k)));
            }
            lmh = rev - fwd;
        }
        if (dir) {
            // Dirichlet residual after the MH ratio of the unmodified proposal (SamplerPTChain.cpp:270-278)
            for (int f = 0; f < d; f++) {
                if (kind[f] != BCM3HIP_PRIOR_DIRICHLET || (int)p1[f] != f) continue;
                const int l = prior::dirichlet_last(d, kind, p1, f);
                double sum = 0.0;
                for (int j = f; j < l; j++) sum += lane_bcast(nxt, j);
                if (lane == l) nxt = 1.0 - sum;
            }
        }
        if (SPEC) {
            if (lane == 0) {
                *sel_out = sel;
                *upd_out = upd;
                *sc_out = sc;
            }
        } else if (lane == 0) {
            P.selected[c] = sel;
        }
    }
    if (on) out_row[lane] = nxt;
    double lp;
    if (!dir) {
        lp = wave_seq_sum(d, on ? prior::log_pdf(kind[li], p0[li], p1[li], p2[li], nxt) : 0.0);
    } else {
        // PriorIndependence::EvaluateLogPDF: multivariate groups first, then the univariate
        // marginals in variable order
        const double ul = (on && kind[li] != BCM3HIP_PRIOR_DIRICHLET) ? prior::log_pdf(kind[li], p0[li], p1[li], p2[li], nxt)
                                                                        : 0.0;
        lp = 0.0;
        for (int f = 0; f < d; f++)
            if (kind[f] == BCM3HIP_PRIOR_DIRICHLET && (int)p1[f] == f)
                lp += prior::dirichlet_log_pdf(f, prior::dirichlet_last(d, kind, p1, f), p0, p2[f],
                                               [&](int j) { return lane_bcast(nxt, j); });
        for (int i = 0; i < d; i++)
            if (kind[i] != BCM3HIP_PRIOR_DIRICHLET) lp += lane_bcast(ul, i);
    }
    if (lane == 0) {
        *lprior_out = lp;
        *log_mh_out = lmh;
    }
}

__global__ void __launch_bounds__(64) ptmh_propose_wave_kernel(
    int C, int d, const int32_t* __restrict__ kind, const double* __restrict__ p0, const double* __restrict__ p1,
    const double* __restrict__ p2, const double* __restrict__ temps, const double* __restrict__ values, double* __restrict__ prop,
    double* __restrict__ lprior_prop, double* __restrict__ log_mh, bcm3hip_proposal P, int64_t chain0,
    uint64_t seed, uint64_t iter)
{
    const int c = __builtin_amdgcn_readfirstlane((int)blockIdx.x);
    if (c >= C) return;
    propose_wave_one<false>(c, d, kind, p0, p1, p2, temps, values + (int64_t)c * d, 0.0, prop + (int64_t)c * d,
                            lprior_prop + c, log_mh + c, P, (uint64_t)(chain0 + c), seed, iter, nullptr, nullptr,
                            nullptr);
}

// generic path (d > 64): one thread per chain, its vectors in the global work buffer
__global__ void __launch_bounds__(64) ptmh_propose_adaptive_kernel(
    int C, int d, const int32_t* __restrict__ kind, const double* __restrict__ p0, const double* __restrict__ p1,
    const double* __restrict__ p2, const double* __restrict__ temps, const double* __restrict__ values, double* __restrict__ prop,
    double* __restrict__ lprior_prop, double* __restrict__ log_mh, bcm3hip_proposal P, int64_t chain0,
    uint64_t seed, uint64_t iter)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const int Km = P.kmax;
    double* work = P.work + (int64_t)c * (2 * Km + 2 * d);
    propose_chain(c, d, kind, p0, p1, p2, temps, values, prop, lprior_prop, log_mh, P, (uint64_t)(chain0 + c), seed,
                  iter, work + 2 * Km, work + 2 * Km + d, work, work + Km);
}

// Sampler::TestSample / MutateMove's accept of chain c (one thread per chain); returns the flag
__device__ __forceinline__ bool accept_one(int c, int d, const double* __restrict__ temps, const double* __restrict__ prop,
                           const double* __restrict__ lprior_prop, const double* __restrict__ llh_prop,
                           const double* __restrict__ log_mh, double learning_rate, double* __restrict__ values,
                           double* __restrict__ lprior, double* __restrict__ llh, double* __restrict__ lpp,
                           uint8_t* __restrict__ acc_out, unsigned long long* __restrict__ accepted,
                           int32_t* __restrict__ nan_llh, const bcm3hip_proposal& P, int64_t chain0, uint64_t seed,
                           uint64_t iter)
{
    const double T = temps[c];
    const double nl = llh_prop[c] * learning_rate;  // Sampler::EvaluateLikelihood
    const double nq = lprior_prop[c];
    bool acc;
    double npp;
    if (isnan(nl)) {
        // Sampler::EvaluateLikelihood (Sampler.cpp:172-178): a NaN log-likelihood is fatal; the
        // chain keeps its state (no EMA update) and the host raises at its next check of the flag
        if (nan_llh) *nan_llh = 1;
        acc = false;
        npp = 0.0;
    } else if (T == 0.0) {
        acc = true;
        npp = (nl == -INFINITY) ? nq : nq + T * nl;
    } else {
        npp = nq + T * nl;
        acc = false;
        if (npp > -INFINITY) {
            double tp = npp - lpp[c];
            tp = exp(tp + log_mh[c]);
            tp = (tp < 1.0) ? tp : 1.0;  // std::min((Real)1.0, tp): NaN -> 1
            acc = u01(rng_key(seed, iter, (uint64_t)(chain0 + c), rng::KEY_ACCEPT)) < tp;
        }
        // NotifyAccepted (EMA of the acceptance of the component that proposed)
        const int sel = P.selected[c];
        double* ema = P.ema + (int64_t)c * P.kmax + sel;
        const double alpha = 2.0 / (P.scaling_ema_period + 1);
        *ema += ((acc ? 1.0 : 0.0) - *ema) * alpha;
    }
    if (acc) {
        copy_row(values + (int64_t)c * d, prop + (int64_t)c * d, d);
        lprior[c] = nq;
        llh[c] = nl;
        lpp[c] = npp;
    }
    if (acc_out) acc_out[c] = acc ? 1 : 0;
    if (accepted && acc) atomicAdd(accepted, 1ull);
    return acc;
}

__global__ void ptmh_accept_adaptive_kernel(int C, int d, const double* __restrict__ temps,
                                            const double* __restrict__ prop, const double* __restrict__ lprior_prop,
                                            const double* __restrict__ llh_prop, const double* __restrict__ log_mh,
                                            double learning_rate, double* __restrict__ values,
                                            double* __restrict__ lprior, double* __restrict__ llh,
                                            double* __restrict__ lpp, uint8_t* __restrict__ acc_out,
                                            unsigned long long* __restrict__ accepted,
                                            int32_t* __restrict__ nan_llh, bcm3hip_proposal P, int64_t chain0,
                                            uint64_t seed, uint64_t iter)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    accept_one(c, d, temps, prop, lprior_prop, llh_prop, log_mh, learning_rate, values, lprior, llh, lpp, acc_out,
               accepted, nan_llh, P, chain0, seed, iter);
}

// SampleHistory::AddSample for the chains with T != 0 (and mask[c] != 0 when a mask is given):
// every `subsampling`-th call stores the values as float in slot n % H of the chain's ring
__device__ __forceinline__ void history_one(int c, int d, int H, int subsampling, const double* __restrict__ temps,
                            const double* __restrict__ values, const uint8_t* __restrict__ mask,
                            float* __restrict__ hist, int64_t* __restrict__ counters)
{
    if (temps[c] == 0.0 || (mask && !mask[c])) return;
    int64_t* n = counters + 2 * (int64_t)c;
    const int64_t n0 = n[0], n1 = n[1] + 1;  // both counters in one memory round trip
    if (n1 == subsampling) {
        copy_row(hist + ((int64_t)c * H + n0 % H) * d, values + (int64_t)c * d, d);
        n[0] = n0 + 1;
        n[1] = 0;
    } else {
        n[1] = n1;
    }
}

__global__ void history_add_kernel(int C, int d, int H, int subsampling, const double* __restrict__ temps,
                                   const double* __restrict__ values, const uint8_t* __restrict__ mask,
                                   float* __restrict__ hist, int64_t* __restrict__ counters)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    history_one(c, d, H, subsampling, temps, values, mask, hist, counters);
}

// ---- speculative iteration pairs (include/bcm3hip.h "speculative iteration pairs") ----

// Proposal::Update's branch for an acceptance EMA e: 0 shrink, 1 keep, 2 grow (the comparisons of
// propose_wave_one, in the same form)
__device__ __forceinline__ int update_branch(const bcm3hip_proposal& P, double e)
{
    const double slr = P.scaling_learning_rate, target = P.target_acceptance;
    if (P.kind == BCM3HIP_PROPOSAL_GAUSSIAN_MIXTURE) {
        if (e < target / (1.0 - slr)) return 0;
        if (e > (1 + slr) * target) return 2;
        return 1;
    }
    if (e < 0.952381 * target) return 0;
    if (e > 1.05 * target) return 2;
    return 1;
}

// one wavefront per (chain c, slot k): candidate k of c for iteration `iter` (= r + 1)
__global__ void __launch_bounds__(64) ptmh_spec_candidates_kernel(
    int C, int d, const int32_t* __restrict__ kind, const double* __restrict__ p0, const double* __restrict__ p1,
    const double* __restrict__ p2, const double* __restrict__ temps, const double* __restrict__ values,
    const double* __restrict__ prop, const int32_t* __restrict__ partner, const double* __restrict__ remote,
    bcm3hip_proposal P, bcm3hip_spec S, int64_t chain0, uint64_t seed, uint64_t iter)
{
    const int w = __builtin_amdgcn_readfirstlane((int)blockIdx.x);
    const int c = w / BCM3HIP_SPEC_SLOTS, k = w - c * BCM3HIP_SPEC_SLOTS;
    if (c >= C) return;
    const int lane = threadIdx.x & 63;
    const int pc = partner[c];
    const double* row = values + (int64_t)c * d;
    // the partner's (state, proposal) rows: local chains, or the neighbour rank's boundary chain
    // (BCM3HIP_SPEC_REMOTE_NEXT / _PREV: remote[0..2d) / remote[2d..4d), state then proposal)
    const bool has_p = pc >= 0 || pc == BCM3HIP_SPEC_REMOTE_NEXT || pc == BCM3HIP_SPEC_REMOTE_PREV;
    const double* p_old = (pc >= 0) ? values + (int64_t)pc * d
                          : (pc == BCM3HIP_SPEC_REMOTE_NEXT) ? remote : (pc == BCM3HIP_SPEC_REMOTE_PREV) ? remote + 2 * d : row;
    const double* p_new = (pc >= 0) ? prop + (int64_t)pc * d : (pc < -1) ? p_old + d : row;
    double ema_last = 0.0;
    bool active;
    if (temps[c] == 0.0) {
        active = (k == 0);  // a prior draw: the state does not matter
    } else {
        // the EMA NotifyAccepted leaves for component selected[c] (ptmh_accept_adaptive_kernel's
        // arithmetic) after a reject (e0) or an accept (e1) of iteration r
        const int sel = P.selected[c];
        const double e = P.ema[(int64_t)c * P.kmax + (sel < 0 ? 0 : sel)];
        const double alpha = 2.0 / (P.scaling_ema_period + 1);
        const double e0 = e + (0.0 - e) * alpha;
        const double e1 = e + (1.0 - e) * alpha;
        const bool two = update_branch(P, e0) != update_branch(P, e1);
        int a = 0;
        switch (k) {
        case 0: active = true; a = 0; break;
        case 1: active = true; row = prop + (int64_t)c * d; a = 1; break;
        case 2: active = has_p; row = p_old; a = 0; break;
        case 3: active = has_p; row = p_new; a = 0; break;
        case 4: active = has_p && two; row = p_old; a = 1; break;
        default: active = has_p && two; row = p_new; a = 1; break;
        }
        ema_last = a ? e1 : e0;
    }
    if (lane == 0) {
        S.cand_active[w] = active ? 1 : 0;
        S.cand_sel[w] = -1;
        S.cand_upd[w] = -1;
        S.cand_sc[w] = 0.0;
    }
    if (!active) return;
    propose_wave_one<true>(c, d, kind, p0, p1, p2, temps, row, ema_last, S.cand_x + (int64_t)w * d, S.cand_lp + w,
                           S.cand_lmh + w, P, (uint64_t)(chain0 + c), seed, iter, S.cand_sel + w, S.cand_upd + w,
                           S.cand_sc + w);
}

// The solve length of an entry, predicted from the previous launch's entries (batch_x / batch_steps
// before this pair's batch overwrites them): the mean steps of its 4 nearest neighbours in parameter
// space, coordinates scaled by 1 / (prior sd). On C3 prior draws this ranks solve lengths with a
// Spearman correlation of 0.93 (the state's own last solve: 0.58). One workgroup of 4 wavefronts
// per entry, each scanning a quarter of the previous entries; entries with nothing to compare
// against (first pair) keep the steps_hint of their source.
constexpr int kKnn = 4;
constexpr int kKnnWaves = 4;
__global__ void __launch_bounds__(64 * kKnnWaves) ptmh_spec_predict_kernel(int C, int d, const double* __restrict__ prop,
                                                                           const int32_t* __restrict__ partner,
                                                                           const double* __restrict__ inv_scale,
                                                                           bcm3hip_spec S)
{
    __shared__ double wd[kKnnWaves * kKnn];
    __shared__ int ws[kKnnWaves * kKnn];
    const int e = __builtin_amdgcn_readfirstlane((int)blockIdx.x);
    const int n_all = C * (1 + BCM3HIP_SPEC_SLOTS);
    if (e >= n_all) return;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const double* x;
    int src;
    if (e < C) {
        x = prop + (int64_t)e * d;
        src = e;
    } else {
        const int sl = e - C, c = sl / BCM3HIP_SPEC_SLOTS, k = sl - c * BCM3HIP_SPEC_SLOTS;
        if (!S.cand_active[sl]) return;
        x = S.cand_x + (int64_t)sl * d;
        src = (k <= 1 || partner[c] < 0) ? c : partner[c];
    }
    const int mem_n = S.batch_n[0];
    if (mem_n <= 0) {
        if (tid == 0) S.pred_steps[e] = S.steps_hint[src];
        return;
    }
    double bd[kKnn];
    int bs[kKnn];
    for (int q = 0; q < kKnn; q++) {
        bd[q] = INFINITY;
        bs[q] = 0;
    }
    if (S.batch_xs) {
        // (round 6) the previous entries as single-precision coordinates pre-scaled by 1 / prior sd,
        // written by the batch kernel: half the L2 traffic of the double rows, which bounded this
        // kernel; the distances only order the launch
        __shared__ float qs[64];
        if (tid < d) qs[tid] = (float)(x[tid] * inv_scale[tid]);
        __syncthreads();
        for (int m = tid; m < mem_n; m += 64 * kKnnWaves) {
            const float* y = S.batch_xs + (int64_t)m * d;
            float dist = 0.0f;
            for (int j = 0; j < d; j++) {
                const float t = qs[j] - y[j];
                dist = __builtin_fmaf(t, t, dist);
            }
            if (dist < bd[kKnn - 1]) {
                int q = kKnn - 1;
                const int st = S.batch_steps[m];
                while (q > 0 && bd[q - 1] > dist) {
                    bd[q] = bd[q - 1];
                    bs[q] = bs[q - 1];
                    q--;
                }
                bd[q] = dist;
                bs[q] = st;
            }
        }
    } else
    for (int m = tid; m < mem_n; m += 64 * kKnnWaves) {
        const double* y = S.batch_x + (int64_t)m * d;
        double dist = 0.0;
        for (int j = 0; j < d; j++) {
            const double t = (x[j] - y[j]) * inv_scale[j];
            dist = __builtin_fma(t, t, dist);
        }
        if (dist < bd[kKnn - 1]) {
            int q = kKnn - 1;
            const int st = S.batch_steps[m];
            while (q > 0 && bd[q - 1] > dist) {
                bd[q] = bd[q - 1];
                bs[q] = bs[q - 1];
                q--;
            }
            bd[q] = dist;
            bs[q] = st;
        }
    }
    // the kKnn smallest of each wavefront: repeatedly take the minimum head
    for (int r = 0; r < kKnn; r++) {
        double mn = bd[0];
        for (int off = 32; off >= 1; off >>= 1) {
            const double o = __shfl_xor(mn, off);
            mn = (o < mn) ? o : mn;
        }
        int st = 0;
        if (mn != INFINITY) {
            // the lowest lane holding the minimum pops it
            const unsigned long long who = __ballot(bd[0] == mn);
            const int owner = __builtin_ctzll(who);
            st = __shfl(bs[0], owner);
            if (lane == owner) {
                for (int q = 0; q < kKnn - 1; q++) {
                    bd[q] = bd[q + 1];
                    bs[q] = bs[q + 1];
                }
                bd[kKnn - 1] = INFINITY;
            }
        }
        if (lane == 0) {
            wd[wv * kKnn + r] = mn;
            ws[wv * kKnn + r] = st;
        }
    }
    __syncthreads();
    if (tid == 0) {
        // the kKnn smallest of the wavefronts' lists
        int sum = 0, got = 0;
        for (int r = 0; r < kKnn; r++) {
            int best = -1;
            for (int i = 0; i < kKnnWaves * kKnn; i++)
                if (wd[i] != INFINITY && (best < 0 || wd[i] < wd[best])) best = i;
            if (best < 0) break;
            sum += ws[best];
            got++;
            wd[best] = INFINITY;
        }
        S.pred_steps[e] = got ? sum / got : S.steps_hint[src];
    }
}

// one workgroup: the batch of iteration r's proposals and the active candidates, ordered by the
// predicted solve length (ptmh_spec_predict_kernel), longest first. A counting sort over buckets of
// 2 steps (atomic ranks inside a bucket: the order of equal keys is arbitrary, which changes timing
// only -- every entry's result is its own). Layout for a batch of M > R wavefronts, R = the
// wavefronts the device runs at once one per SIMD (first_round): the hardware gives batch
// positions p and p + R the same SIMD (measured, tools/placement.py), so the M - R shortest go to
// positions R.., the next M - R shortest to positions 0.. (they share SIMDs with each other), and
// the 2R - M longest run alone at positions M - R .. R - 1 (R < M <= 2R); otherwise, or with
// first_round = 0, plain longest first.
constexpr int kSpecSortMax = 4096;
constexpr int kSpecBuckets = 2048;
__global__ void __launch_bounds__(1024) ptmh_spec_batch_kernel(int C, int d, const double* __restrict__ prop,
                                                               const int32_t* __restrict__ partner, int first_round,
                                                               const double* __restrict__ inv_scale, bcm3hip_spec S)
{
    __shared__ int cnt[kSpecBuckets];
    __shared__ int wsum[16];
    __shared__ int pos_of[kSpecSortMax];  // entry id -> batch position (-1 inactive)
    const int tid = threadIdx.x;
    const int n_all = C * (1 + BCM3HIP_SPEC_SLOTS);
    for (int b = tid; b < kSpecBuckets; b += blockDim.x) cnt[b] = 0;
    __syncthreads();
    constexpr int kPer = kSpecSortMax / 1024;
    int bk[kPer], rk[kPer];
    for (int q = 0; q < kPer; q++) {
        const int i = tid + q * 1024;
        bk[q] = -1;
        const bool on = (i < C) || (i < n_all && S.cand_active[i - C]);
        if (on) {
            int h = S.pred_steps[i];
            h = h < 0 ? 0 : (h >> 1);
            h = h > kSpecBuckets - 1 ? kSpecBuckets - 1 : h;
            bk[q] = kSpecBuckets - 1 - h;  // longest first
            rk[q] = atomicAdd(&cnt[bk[q]], 1);
        }
    }
    __syncthreads();
    // exclusive prefix sum of the bucket counts: two buckets per thread, then a scan over the
    // 16 wavefronts' totals
    const int lane = tid & 63, wv = tid >> 6;
    const int c0 = cnt[2 * tid], c1 = cnt[2 * tid + 1];
    int incl = c0 + c1;
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int before = 0;
    for (int w = 0; w < wv; w++) before += wsum[w];
    int M = 0;
    for (int w = 0; w < 16; w++) M += wsum[w];
    const int ex = before + incl - c0 - c1;
    __syncthreads();
    cnt[2 * tid] = ex;
    cnt[2 * tid + 1] = ex + c0;
    for (int i = tid; i < kSpecSortMax; i += blockDim.x) pos_of[i] = -1;
    __syncthreads();
    const int R = first_round;
    // entries of the second round; beyond 2R entries every SIMD takes two and more wait for a free
    // one, so the layout is plain longest first there
    const int S2 = (R > 0 && M > R && M <= 2 * R) ? M - R : 0;
    const int L = M - 2 * S2;  // entries that run alone (L >= 0)
    for (int q = 0; q < kPer; q++) {
        if (bk[q] < 0) continue;
        const int r = cnt[bk[q]] + rk[q];
        int p = r;
        if (S2 > 0) p = (r < L) ? S2 + r : (r < L + S2) ? r - L : R + (r - L - S2);
        pos_of[tid + q * 1024] = p;
    }
    if (tid == 0) {
        S.batch_n[0] = M;
        if (S.batch_total) S.batch_total[0] += M;
    }
    __syncthreads();
    for (int i = tid; i < n_all; i += blockDim.x) {
        if (pos_of[i] >= 0) S.batch_src[pos_of[i]] = i;
        if (S.batch_pos) S.batch_pos[i] = pos_of[i];
    }
    for (int t = tid; t < n_all * d; t += blockDim.x) {
        const int id = t / d, j = t - id * d;
        const int p = pos_of[id];
        if (p < 0) continue;
        const double* src = (id < C) ? prop + (int64_t)id * d : S.cand_x + (int64_t)(id - C) * d;
        const double v = src[j];
        S.batch_x[(int64_t)p * d + j] = v;
        if (S.batch_xs) S.batch_xs[(int64_t)p * d + j] = (float)(v * inv_scale[j]);
    }
}

__global__ void ptmh_spec_scatter_kernel(int C, bcm3hip_spec S, double* __restrict__ llh_prop)
{
    const int pos = blockIdx.x * blockDim.x + threadIdx.x;
    if (pos >= S.batch_n[0]) return;
    const int id = S.batch_src[pos];
    if (id < C) {
        llh_prop[id] = S.batch_llh[pos];
        S.steps_prop[id] = S.batch_steps[pos];
    } else {
        S.cand_llh[id - C] = S.batch_llh[pos];
        S.cand_steps[id - C] = S.batch_steps[pos];
    }
}

// one thread per chain: the candidate that the accept of r and the exchange of r + 1 made real
__device__ __forceinline__ void select_one(int c, int d, const double* __restrict__ temps, const int32_t* __restrict__ partner,
                           const int32_t* __restrict__ pair_first, const uint8_t* __restrict__ acc_mut,
                           const uint8_t* __restrict__ acc_exc, const uint8_t* __restrict__ cross_acc,
                           const double* __restrict__ remote, const double* __restrict__ values, const bcm3hip_spec& S,
                           double* __restrict__ prop, double* __restrict__ lprior_prop, double* __restrict__ log_mh,
                           double* __restrict__ llh_prop, const bcm3hip_proposal& P, int32_t* __restrict__ error)
{
    int k = 0;
    const bool hot = temps[c] != 0.0;
    if (hot) {
        const int pc = partner[c];
        const bool own = acc_mut[c] != 0;
        bool swapped = false, partner_acc = false;
        if (pc >= 0) {
            swapped = acc_exc[pair_first[c]] != 0;
            partner_acc = acc_mut[pc] != 0;
        } else if (pc == BCM3HIP_SPEC_REMOTE_NEXT || pc == BCM3HIP_SPEC_REMOTE_PREV) {
            // cross-rank pair (pt_cross_accept: flag 0 for my last chain, 1 for my first); the
            // partner's accept is read off the state it sent: its proposal row or not (if the two
            // rows are equal the two candidates are the same proposal)
            swapped = cross_acc[pc == BCM3HIP_SPEC_REMOTE_NEXT ? 0 : 1] != 0;
            const double* pn = remote + (pc == BCM3HIP_SPEC_REMOTE_NEXT ? 0 : 2 * d) + d;
            bool same = true;
            for (int i = 0; i < d; i++) same &= (__builtin_bit_cast(unsigned long long, values[(int64_t)c * d + i]) ==
                                                 __builtin_bit_cast(unsigned long long, pn[i]));
            partner_acc = same;
        }
        if (!swapped) {
            k = own ? 1 : 0;
        } else {
            k = partner_acc ? 3 : 2;
            if (own && S.cand_active[c * BCM3HIP_SPEC_SLOTS + k + 2]) k += 2;
        }
    }
    const int sl = c * BCM3HIP_SPEC_SLOTS + k;
    if (!S.cand_active[sl]) {
        // internal error: poison the row, so the accept step's fatal-NaN path stops the sampler at
        // its next check instead of letting this chain reuse iteration r's proposal
        if (error) *error = 1;
        llh_prop[c] = __builtin_nan("");
        return;
    }
    copy_row(prop + (int64_t)c * d, S.cand_x + (int64_t)sl * d, d);
    lprior_prop[c] = S.cand_lp[sl];
    log_mh[c] = S.cand_lmh[sl];
    llh_prop[c] = S.cand_llh[sl];
    S.steps_prop[c] = S.cand_steps[sl];
    if (hot) {
        const int upd = S.cand_upd[sl];
        if (upd >= 0) P.scale[(int64_t)c * P.kmax + upd] = S.cand_sc[sl];
        P.selected[c] = S.cand_sel[sl];
    }
}

__global__ void ptmh_spec_select_kernel(int C, int d, const double* __restrict__ temps,
                                        const int32_t* __restrict__ partner, const int32_t* __restrict__ pair_first,
                                        const uint8_t* __restrict__ acc_mut, const uint8_t* __restrict__ acc_exc,
                                        const uint8_t* __restrict__ cross_acc, const double* __restrict__ remote,
                                        const double* __restrict__ values, bcm3hip_spec S, double* __restrict__ prop,
                                        double* __restrict__ lprior_prop, double* __restrict__ log_mh,
                                        double* __restrict__ llh_prop, bcm3hip_proposal P, int32_t* __restrict__ error)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    select_one(c, d, temps, partner, pair_first, acc_mut, acc_exc, cross_acc, remote, values, S, prop, lprior_prop,
               log_mh, llh_prop, P, error);
}

// The end of one iteration of a speculative pair in ONE launch, one thread per chain: [select
// (iteration r + 1)], accept, the dispatch-order tracking of the accept, SampleHistory::AddSample --
// per chain the operations of ptmh_spec_select / ptmh_accept_adaptive / ptmh_spec_track_accept /
// history_add in that order. Every write is to the thread's own chain; the one cross-chain read, the
// partner's accept flag of iteration r in select, comes from acc_prev, never from acc_out.
__device__ __forceinline__ void commit_one(int c, int C, int d, int select, const double* __restrict__ temps,
                           const int32_t* __restrict__ partner, const int32_t* __restrict__ pair_first,
                           const uint8_t* __restrict__ acc_prev, const uint8_t* __restrict__ acc_exc,
                           const uint8_t* __restrict__ cross_acc, const double* __restrict__ remote,
                           const bcm3hip_spec& S, double* __restrict__ prop, double* __restrict__ lprior_prop,
                           double* __restrict__ log_mh, double* __restrict__ llh_prop, double learning_rate,
                           double* __restrict__ values, double* __restrict__ lprior, double* __restrict__ llh,
                           double* __restrict__ lpp, uint8_t* __restrict__ acc_out,
                           unsigned long long* __restrict__ accepted, int32_t* __restrict__ nan_llh,
                           const bcm3hip_proposal& P, int64_t chain0, uint64_t seed, uint64_t iter, int H,
                           int subsampling, float* __restrict__ hist, int64_t* __restrict__ counters,
                           int32_t* __restrict__ error)
{
    if (!select && S.batch_pos) {
        // the batch's results of this chain's entries -- its proposal and its candidates -- through
        // the inverse permutation (ptmh_spec_scatter_kernel's writes for chain c, in this launch)
        const int p = S.batch_pos[c];
        if (p >= 0) {
            llh_prop[c] = S.batch_llh[p];
            S.steps_prop[c] = S.batch_steps[p];
        }
        for (int k = 0; k < BCM3HIP_SPEC_SLOTS; k++) {
            const int sl = c * BCM3HIP_SPEC_SLOTS + k;
            const int q = S.batch_pos[C + sl];
            if (q >= 0) {
                S.cand_llh[sl] = S.batch_llh[q];
                S.cand_steps[sl] = S.batch_steps[q];
            }
        }
    }
    if (select)
        select_one(c, d, temps, partner, pair_first, acc_prev, acc_exc, cross_acc, remote, values, S, prop, lprior_prop,
                   log_mh, llh_prop, P, error);
    const bool acc = accept_one(c, d, temps, prop, lprior_prop, llh_prop, log_mh, learning_rate, values, lprior, llh,
                                lpp, acc_out, accepted, nan_llh, P, chain0, seed, iter);
    if (acc) S.steps_hint[c] = S.steps_prop[c];
    if (hist) history_one(c, d, H, subsampling, temps, values, nullptr, hist, counters);
}

__global__ void ptmh_spec_commit_kernel(int C, int d, int select, const double* __restrict__ temps,
                                        const int32_t* __restrict__ partner, const int32_t* __restrict__ pair_first,
                                        const uint8_t* __restrict__ acc_prev, const uint8_t* __restrict__ acc_exc,
                                        const uint8_t* __restrict__ cross_acc, const double* __restrict__ remote,
                                        bcm3hip_spec S, double* __restrict__ prop, double* __restrict__ lprior_prop,
                                        double* __restrict__ log_mh, double* __restrict__ llh_prop,
                                        double learning_rate, double* __restrict__ values, double* __restrict__ lprior,
                                        double* __restrict__ llh, double* __restrict__ lpp, uint8_t* __restrict__ acc_out,
                                        unsigned long long* __restrict__ accepted, int32_t* __restrict__ nan_llh,
                                        bcm3hip_proposal P, int64_t chain0, uint64_t seed, uint64_t iter, int H,
                                        int subsampling, float* __restrict__ hist, int64_t* __restrict__ counters,
                                        int32_t* __restrict__ error)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    commit_one(c, C, d, select, temps, partner, pair_first, acc_prev, acc_exc, cross_acc, remote, S, prop, lprior_prop,
               log_mh, llh_prop, learning_rate, values, lprior, llh, lpp, acc_out, accepted, nan_llh, P, chain0, seed,
               iter, H, subsampling, hist, counters, error);
}

// dispatch-order bookkeeping of the pairs: steps_hint[c] = BDF steps of the solve of the state now in
// slot c; after an accept (acc[c]: the proposal, whose steps are steps_prop[c], became the state) ...
__global__ void ptmh_spec_track_accept_kernel(int C, const uint8_t* __restrict__ acc, bcm3hip_spec S)
{
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    if (acc[c]) S.steps_hint[c] = S.steps_prop[c];
}
// ... and after an exchange round (acc_exc[pair_first[c]]: c took its partner's state); one
// workgroup, the old values read before any is written
__global__ void __launch_bounds__(1024) ptmh_spec_track_exchange_kernel(int C, const int32_t* __restrict__ partner,
                                                                        const int32_t* __restrict__ pair_first,
                                                                        const uint8_t* __restrict__ acc_exc,
                                                                        bcm3hip_spec S)
{
    int v[4];
    int n = 0;
    for (int c = threadIdx.x; c < C && n < 4; c += blockDim.x, n++) {
        const int p = partner[c];
        v[n] = (p >= 0 && acc_exc[pair_first[c]]) ? S.steps_hint[p] : S.steps_hint[c];
    }
    __syncthreads();
    n = 0;
    for (int c = threadIdx.x; c < C && n < 4; c += blockDim.x, n++) S.steps_hint[c] = v[n];
}

// One exchange round of a single-rank ladder whose pairs cover every chain exactly once, with what
// follows it in a speculative pair, in ONE workgroup: the local pairs (pt_exchange_kernel), the wrap
// pair after them, the dispatch-order tracking of the round (ptmh_spec_track_exchange_kernel) and
// SampleHistory::AddSample of every chain (ExchangeMove adds both chains of each pair,
// SamplerPTChain.cpp:374-379; history_add_kernel) -- the same per-chain operations in the same order.
__device__ __forceinline__ void exchange_round(int C, int d, int64_t g0, int start, int wrap_local, const double* temps, double* values,
                               double* llh, double* lprior, double* lpp, uint8_t* acc_mask,
                               unsigned long long* accepted, uint64_t seed, uint64_t round,
                               const int32_t* __restrict__ partner, const int32_t* __restrict__ pair_first,
                               const bcm3hip_spec& S, int H, int subsampling, float* __restrict__ hist,
                               int64_t* __restrict__ counters)
{
    const int par = (int)(((g0 - start) % 2 + 2) % 2);
    for (int p = threadIdx.x;; p += blockDim.x) {
        const int i = par + 2 * p;
        if (i + 1 >= C) break;
        exchange_pair(d, i, i + 1, g0 + i, temps, values, llh, lprior, lpp, acc_mask, accepted, seed, round);
    }
    __syncthreads();
    if (wrap_local && threadIdx.x == 0)
        exchange_pair(d, C - 1, 0, g0 + C - 1, temps, values, llh, lprior, lpp, acc_mask, accepted, seed, round);
    __syncthreads();
    int v[4];
    int n = 0;
    for (int c = threadIdx.x; c < C && n < 4; c += blockDim.x, n++) {
        const int p = partner[c];
        v[n] = (p >= 0 && acc_mask[pair_first[c]]) ? S.steps_hint[p] : S.steps_hint[c];
    }
    __syncthreads();
    n = 0;
    for (int c = threadIdx.x; c < C && n < 4; c += blockDim.x, n++) {
        S.steps_hint[c] = v[n];
        if (hist) history_one(c, d, H, subsampling, temps, values, nullptr, hist, counters);
    }
}

__global__ void __launch_bounds__(1024) ptmh_spec_exchange_kernel(
    int C, int d, int64_t g0, int start, int wrap_local, const double* temps, double* values, double* llh,
    double* lprior, double* lpp, uint8_t* acc_mask, unsigned long long* accepted, uint64_t seed, uint64_t round,
    const int32_t* __restrict__ partner, const int32_t* __restrict__ pair_first, bcm3hip_spec S, int H,
    int subsampling, float* __restrict__ hist, int64_t* __restrict__ counters)
{
    exchange_round(C, d, g0, start, wrap_local, temps, values, llh, lprior, lpp, acc_mask, accepted, seed, round, partner,
                   pair_first, S, H, subsampling, hist, counters);
}

// The end of a speculative pair of a single-rank ladder in ONE workgroup (round 6): the commit of
// iteration r (ptmh_spec_commit_kernel, select = 0), the exchange round of r + 1
// (ptmh_spec_exchange_kernel) and the commit of r + 1 (select = 1) -- the three launches' per-chain
// operations in their order, a workgroup barrier where a kernel boundary was (each phase reads what the
// previous ones wrote: partners' accept flags, the exchanged states). Saves two launches and their
// memory round trips per pair.
__global__ void __launch_bounds__(1024) ptmh_spec_tail_kernel(
    int C, int d, int64_t g0, int start, int wrap_local, const double* __restrict__ temps,
    const int32_t* __restrict__ partner, const int32_t* __restrict__ pair_first, uint8_t* __restrict__ acc_mut,
    uint8_t* __restrict__ acc_mut2, uint8_t* __restrict__ acc_exc, const uint8_t* __restrict__ cross_acc,
    const double* __restrict__ remote, unsigned long long* __restrict__ acc_mutate,
    unsigned long long* __restrict__ acc_exchange, bcm3hip_spec S, double* __restrict__ prop,
    double* __restrict__ lprior_prop, double* __restrict__ log_mh, double* __restrict__ llh_prop, double learning_rate,
    double* __restrict__ values, double* __restrict__ lprior, double* __restrict__ llh, double* __restrict__ lpp,
    int32_t* __restrict__ nan_llh, bcm3hip_proposal P, uint64_t seed, uint64_t iter, uint64_t round, int H,
    int subsampling, float* __restrict__ hist, int64_t* __restrict__ counters, int32_t* __restrict__ error)
{
    for (int c = threadIdx.x; c < C; c += blockDim.x)
        commit_one(c, C, d, 0, temps, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, S, prop, lprior_prop, log_mh,
                   llh_prop, learning_rate, values, lprior, llh, lpp, acc_mut, acc_mutate, nan_llh, P, g0, seed, iter, H,
                   subsampling, hist, counters, error);
    __syncthreads();
    exchange_round(C, d, g0, start, wrap_local, temps, values, llh, lprior, lpp, acc_exc, acc_exchange, seed, round,
                   partner, pair_first, S, H, subsampling, hist, counters);
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += blockDim.x)
        commit_one(c, C, d, 1, temps, partner, pair_first, acc_mut, acc_exc, cross_acc, remote, S, prop, lprior_prop,
                   log_mh, llh_prop, learning_rate, values, lprior, llh, lpp, acc_mut2, acc_mutate, nan_llh, P, g0, seed,
                   iter + 1, H, subsampling, hist, counters, error);
}

bool proposal_ok(const bcm3hip_proposal* P, int C, int d)
{
    if (!P || P->kmax < 1 || P->kmax > BCM3HIP_PROPOSAL_KMAX) return false;
    if (P->kind != BCM3HIP_PROPOSAL_GLOBAL_COVARIANCE && P->kind != BCM3HIP_PROPOSAL_GAUSSIAN_MIXTURE) return false;
    if (!(P->scaling_ema_period > 0.0) || !(P->t_dof >= 0.0)) return false;
    if (C > 0 && (!P->lower || !P->upper || !P->ncomp || !P->weights || !P->mean || !P->chol || !P->logc ||
                  !P->scale || !P->ema || !P->selected || !P->work))
        return false;
    return true;
}

}  // namespace
}  // namespace bcm3hip

using namespace bcm3hip;

extern "C" {

int bcm3hip_ptmh_propose_adaptive(int C, int d, const int32_t* prior_kind, const double* prior_p0,
                                  const double* prior_p1, const double* prior_p2, const double* temps,
                                  const double* values, double* prop, double* lprior_prop, double* log_mh,
                                  const bcm3hip_proposal* proposal, int64_t chain0, uint64_t seed, uint64_t iter,
                                  void* stream)
{
    if (C < 0 || d <= 0 || !proposal_ok(proposal, C, d) ||
        (C > 0 && (!prior_kind || !prior_p0 || !prior_p1 || !prior_p2 || !temps || !values || !prop ||
                   !lprior_prop || !log_mh)))
        return BCM3HIP_ERR_ARG;
    if (C == 0) return 0;
    // one wavefront per chain (lanes over variables) up to 64 variables, beyond one thread per chain
    if (d <= 64)
        hipLaunchKernelGGL(ptmh_propose_wave_kernel, dim3(C), dim3(64), 0, (hipStream_t)stream, C, d, prior_kind,
                           prior_p0, prior_p1, prior_p2, temps, values, prop, lprior_prop, log_mh, *proposal, chain0,
                           seed, iter);
    else
        hipLaunchKernelGGL(ptmh_propose_adaptive_kernel, dim3((C + 63) / 64), dim3(64), 0, (hipStream_t)stream, C,
                           d, prior_kind, prior_p0, prior_p1, prior_p2, temps, values, prop, lprior_prop, log_mh,
                           *proposal, chain0, seed, iter);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_ptmh_accept_adaptive(int C, int d, const double* temps, const double* prop, const double* lprior_prop,
                                 const double* llh_prop, const double* log_mh, double learning_rate, double* values,
                                 double* lprior, double* llh, double* lpp, uint8_t* accept_out, uint64_t* accepted,
                                 int32_t* nan_llh, const bcm3hip_proposal* proposal, int64_t chain0, uint64_t seed,
                                 uint64_t iter, void* stream)
{
    if (C < 0 || d <= 0 || !proposal_ok(proposal, C, d) ||
        (C > 0 && (!temps || !prop || !lprior_prop || !llh_prop || !log_mh || !values || !lprior || !llh || !lpp)))
        return BCM3HIP_ERR_ARG;
    if (C == 0) return 0;
    hipLaunchKernelGGL(ptmh_accept_adaptive_kernel, dim3((C + 63) / 64), dim3(64), 0, (hipStream_t)stream, C, d,
                       temps, prop, lprior_prop, llh_prop, log_mh, learning_rate, values, lprior, llh, lpp, accept_out,
                       (unsigned long long*)accepted, nan_llh, *proposal, chain0, seed, iter);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

static bool spec_ok(const bcm3hip_spec* S)
{
    return S && S->cand_x && S->cand_lp && S->cand_lmh && S->cand_llh && S->cand_sel && S->cand_upd && S->cand_sc &&
           S->cand_active && S->cand_steps && S->steps_hint && S->steps_prop && S->batch_x && S->batch_llh &&
           S->batch_status && S->batch_steps && S->batch_src && S->batch_n;
}

int bcm3hip_ptmh_spec_candidates(int C, int d, const int32_t* prior_kind, const double* prior_p0,
                                 const double* prior_p1, const double* prior_p2, const double* temps,
                                 const double* values, const double* prop, const int32_t* partner,
                                 const double* remote, const bcm3hip_proposal* proposal, const bcm3hip_spec* spec,
                                 int64_t chain0, uint64_t seed, uint64_t iter_next, void* stream)
{
    if (C < 0 || d <= 0 || d > 64 || !proposal_ok(proposal, C, d) || !spec_ok(spec) ||
        (C > 0 && (!prior_kind || !prior_p0 || !prior_p1 || !prior_p2 || !temps || !values || !prop || !partner)))
        return BCM3HIP_ERR_ARG;
    if (C == 0) return 0;
    hipLaunchKernelGGL(ptmh_spec_candidates_kernel, dim3(C * BCM3HIP_SPEC_SLOTS), dim3(64), 0, (hipStream_t)stream, C,
                       d, prior_kind, prior_p0, prior_p1, prior_p2, temps, values, prop, partner, remote, *proposal,
                       *spec, chain0, seed, iter_next);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_ptmh_spec_batch(int C, int d, const double* prop, const int32_t* partner, const double* inv_scale,
                            int first_round, const bcm3hip_spec* spec, void* stream)
{
    if (C <= 0 || d <= 0 || C * (1 + BCM3HIP_SPEC_SLOTS) > kSpecSortMax || !prop || !partner || !inv_scale ||
        first_round < 0 || !spec_ok(spec) || !spec->pred_steps)
        return BCM3HIP_ERR_ARG;
    hipLaunchKernelGGL(ptmh_spec_predict_kernel, dim3(C * (1 + BCM3HIP_SPEC_SLOTS)), dim3(64 * kKnnWaves), 0,
                       (hipStream_t)stream,
                       C, d, prop, partner, inv_scale, *spec);
    hipLaunchKernelGGL(ptmh_spec_batch_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, C, d, prop, partner,
                       first_round, inv_scale, *spec);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_ptmh_spec_scatter(int C, const bcm3hip_spec* spec, double* llh_prop, void* stream)
{
    if (C <= 0 || !spec_ok(spec) || !llh_prop) return BCM3HIP_ERR_ARG;
    const int n = C * (1 + BCM3HIP_SPEC_SLOTS);
    hipLaunchKernelGGL(ptmh_spec_scatter_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, C, *spec,
                       llh_prop);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_ptmh_spec_select(int C, int d, const double* temps, const int32_t* partner, const int32_t* pair_first,
                             const uint8_t* acc_mutate, const uint8_t* acc_exchange, const uint8_t* cross_acc,
                             const double* remote, const double* values, const bcm3hip_spec* spec, double* prop,
                             double* lprior_prop, double* log_mh, double* llh_prop, const bcm3hip_proposal* proposal,
                             int32_t* error, void* stream)
{
    if (C <= 0 || d <= 0 || !temps || !partner || !pair_first || !acc_mutate || !acc_exchange || !spec_ok(spec) ||
        !values || !prop || !lprior_prop || !log_mh || !llh_prop || !proposal_ok(proposal, C, d))
        return BCM3HIP_ERR_ARG;
    hipLaunchKernelGGL(ptmh_spec_select_kernel, dim3((C + 63) / 64), dim3(64), 0, (hipStream_t)stream, C, d, temps,
                       partner, pair_first, acc_mutate, acc_exchange, cross_acc, remote, values, *spec, prop,
                       lprior_prop, log_mh, llh_prop, *proposal, error);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_ptmh_spec_commit(int C, int d, int select, const double* temps, const int32_t* partner,
                             const int32_t* pair_first, const uint8_t* acc_prev, const uint8_t* acc_exchange,
                             const uint8_t* cross_acc, const double* remote, const bcm3hip_spec* spec, double* prop,
                             double* lprior_prop, double* log_mh, double* llh_prop, double learning_rate, double* values,
                             double* lprior, double* llh, double* lpp, uint8_t* accept_out, uint64_t* accepted,
                             int32_t* nan_llh, const bcm3hip_proposal* proposal, int64_t chain0, uint64_t seed,
                             uint64_t iter, int H, int subsampling, float* history, int64_t* counters, int32_t* error,
                             void* stream)
{
    if (C <= 0 || d <= 0 || !spec_ok(spec) || !proposal_ok(proposal, C, d) || !temps || !prop || !lprior_prop ||
        !log_mh || !llh_prop || !values || !lprior || !llh || !lpp || !accept_out ||
        (select && (!partner || !pair_first || !acc_prev || !acc_exchange || acc_prev == accept_out)) ||
        (history && (H <= 0 || subsampling <= 0 || !counters)))
        return BCM3HIP_ERR_ARG;
    hipLaunchKernelGGL(ptmh_spec_commit_kernel, dim3((C + 63) / 64), dim3(64), 0, (hipStream_t)stream, C, d, select,
                       temps, partner, pair_first, acc_prev, acc_exchange, cross_acc, remote, *spec, prop, lprior_prop,
                       log_mh, llh_prop, learning_rate, values, lprior, llh, lpp, accept_out,
                       (unsigned long long*)accepted, nan_llh, *proposal, chain0, seed, iter, H, subsampling, history,
                       counters, error);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_ptmh_spec_exchange(int C, int d, int64_t g0, int start, int wrap_local, const double* temps,
                               double* values, double* llh, double* lprior, double* lpp, uint8_t* acc_exchange,
                               uint64_t* accepted, uint64_t seed, uint64_t round, const int32_t* partner,
                               const int32_t* pair_first, const bcm3hip_spec* spec, int H, int subsampling,
                               float* history, int64_t* counters, void* stream)
{
    if (C < 2 || C > 4096 || d <= 0 || !temps || !values || !llh || !lprior || !lpp || !acc_exchange || !partner ||
        !pair_first || !spec_ok(spec) || (history && (H <= 0 || subsampling <= 0 || !counters)))
        return BCM3HIP_ERR_ARG;
    hipLaunchKernelGGL(ptmh_spec_exchange_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, C, d, g0, start,
                       wrap_local, temps, values, llh, lprior, lpp, acc_exchange, (unsigned long long*)accepted, seed,
                       round, partner, pair_first, *spec, H, subsampling, history, counters);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_ptmh_spec_tail(int C, int d, int64_t g0, int start, int wrap_local, const double* temps,
                           const int32_t* partner, const int32_t* pair_first, uint8_t* acc_mut, uint8_t* acc_mut2,
                           uint8_t* acc_exc, const uint8_t* cross_acc, const double* remote, uint64_t* accepted_mutate,
                           uint64_t* accepted_exchange, const bcm3hip_spec* spec, double* prop, double* lprior_prop,
                           double* log_mh, double* llh_prop, double learning_rate, double* values, double* lprior,
                           double* llh, double* lpp, int32_t* nan_llh, const bcm3hip_proposal* proposal, uint64_t seed,
                           uint64_t iter, uint64_t round, int H, int subsampling, float* history, int64_t* counters,
                           int32_t* error, void* stream)
{
    if (C < 2 || C > 4096 || d <= 0 || !spec_ok(spec) || !spec->batch_pos || !proposal_ok(proposal, C, d) || !temps ||
        !partner || !pair_first || !acc_mut || !acc_mut2 || acc_mut == acc_mut2 || !acc_exc || !prop || !lprior_prop ||
        !log_mh || !llh_prop || !values || !lprior || !llh || !lpp || (history && (H <= 0 || subsampling <= 0 || !counters)))
        return BCM3HIP_ERR_ARG;
    hipLaunchKernelGGL(ptmh_spec_tail_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, C, d, g0, start, wrap_local,
                       temps, partner, pair_first, acc_mut, acc_mut2, acc_exc, cross_acc, remote,
                       (unsigned long long*)accepted_mutate, (unsigned long long*)accepted_exchange, *spec, prop,
                       lprior_prop, log_mh, llh_prop, learning_rate, values, lprior, llh, lpp, nan_llh, *proposal, seed,
                       iter, round, H, subsampling, history, counters, error);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_ptmh_spec_track(int C, const uint8_t* acc_mutate, const int32_t* partner, const int32_t* pair_first,
                            const uint8_t* acc_exchange, const bcm3hip_spec* spec, void* stream)
{
    if (C <= 0 || C > 4096 || !spec_ok(spec) || (!acc_mutate && !acc_exchange) ||
        (acc_exchange && (!partner || !pair_first)))
        return BCM3HIP_ERR_ARG;
    if (acc_mutate)
        hipLaunchKernelGGL(ptmh_spec_track_accept_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)stream, C,
                           acc_mutate, *spec);
    else
        hipLaunchKernelGGL(ptmh_spec_track_exchange_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, C, partner,
                           pair_first, acc_exchange, *spec);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_gmm_eval(int n, int d, int K, const double* x, const double* mean, const double* chol, const double* logc,
                     const double* weights, double* logpdf, double* resp, void* stream)
{
    if (n < 0 || d <= 0 || d > 64 || K <= 0 || K > 64 || (n > 0 && (!x || !mean || !chol || !logc || !weights)))
        return BCM3HIP_ERR_ARG;
    if (n == 0) return 0;
    hipLaunchKernelGGL(gmm_eval_wave_kernel, dim3(n), dim3(64), 0, (hipStream_t)stream, n, d, K, x, mean, chol, logc,
                       weights, logpdf, resp);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

int bcm3hip_history_add(int C, int d, int H, int subsampling, const double* temps, const double* values,
                        const uint8_t* mask, float* history, int64_t* counters, void* stream)
{
    if (C < 0 || d <= 0 || H <= 0 || subsampling <= 0 || (C > 0 && (!temps || !values || !history || !counters)))
        return BCM3HIP_ERR_ARG;
    if (C == 0) return 0;
    hipLaunchKernelGGL(history_add_kernel, dim3((C + 63) / 64), dim3(64), 0, (hipStream_t)stream, C, d, H,
                       subsampling, temps, values, mask, history, counters);
    return hipGetLastError() == hipSuccess ? 0 : BCM3HIP_ERR_HIP;
}

}  // extern "C"
