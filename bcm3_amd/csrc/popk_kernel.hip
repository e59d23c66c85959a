// popk_kernel.hip -- batched PopPK likelihood on MI355X (gfx950).
//
// One lane = one (chain-eval, patient) trajectory. Per lane:
//   parameter map        LikelihoodPopPKTrajectory.cpp:283-310 (QuantileNormal, fastpow10,
//                        VariableSet::TransformVariable)
//   CVODE solve          ODESolver::SolveReturnSolution + ODESolverCVODE::Solve
//                        (ODESolver.cpp:93-134, ODESolverCVODE.cpp:322-463) on bdf_lane.h
//   dosing callbacks     TreatmentCallback / TreatmentCallbackBiphasic / CheckGiveTreatment
//                        (.cpp:644-718)
//   observation model    Student-t(nu=4), streamed as each output time is interpolated
//                        (.cpp:410-424)
// A second tiny kernel sums the per-patient terms of one evaluation in patient order with the
// reference's break at -inf (.cpp:427-440) when P > 1.
//
// HBM layout: values[n][d] row-major (the sampler's layout); per-patient data arrays [P] / [P][T]
// are read a handful of times per trajectory (L2/L1 resident). No other global traffic: the
// whole integrator state lives in VGPRs.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

#include <cmath>
#include <cstdint>
#include <type_traits>

#include "bdf_lane.h"
#include "bdf_uni.h"
#include "bdf_vec.h"
#include "pk_math.h"
#include "popk_kernel.h"

namespace bcm3hip {

// ---------------------------------------------------------------------------------------------
// math on the path (ProbabilityDistributions.cpp, MathFunctions.h, VariableSet.cpp)

// ---------------------------------------------------------------------------------------------
// PK models (LikelihoodPopPKTrajectory.cpp:446-642)

template <int PKT>
struct PKTraits {
    static constexpr bool two = (PKT == BCM3HIP_PK_TWO || PKT == BCM3HIP_PK_TWO_BIPHASIC ||
                                 PKT == BCM3HIP_PK_TWO_TRANSIT);
    static constexpr bool transit = (PKT == BCM3HIP_PK_ONE_TRANSIT || PKT == BCM3HIP_PK_TWO_TRANSIT);
    static constexpr bool biphasic = (PKT == BCM3HIP_PK_ONE_BIPHASIC || PKT == BCM3HIP_PK_TWO_BIPHASIC);
    static constexpr int NS = two ? 3 : 2;
};

// COLD: the library functions of the parameter map, the transit input and the observation model
// are called out of line (libm_exact.h xm::lib) -- the vector-state kernel only
template <int PKT, bool COLD = false>
struct PKLane {
    using TR = PKTraits<PKT>;
    static constexpr int NS = TR::NS;
    double ka, ke, kel, kf, kb, ktr, ntr, lnf, ka2;
    double dose, dose_after, dose_change_time, last_treatment;
    bool biphasic_switch;

    BDF_INL double cur_ka() const
    {
        if constexpr (TR::biphasic) return biphasic_switch ? ka : ka2;
        return ka;
    }

    // CalculateDerivative_* (.cpp:446-627): every component in the reference's own expression,
    //   dydt0 = [transit -] (ka + ke) y0
    //   dydt1 = ka y0 - kel y1 [- kf y1 + kb y2]
    //   dydt2 = kf y1 - kb y2
    // (left to right, no contraction), so the one-trajectory-per-wavefront solver, which forms the
    // same expressions lane by lane, and the reference produce identical bits.
    BDF_INL double a00() const { return -(cur_ka() + ke); }

    // transit absorption input (.cpp:568-592), 0 for the other models; libm's exp / log
    BDF_INL double input(double t) const
    {
        if constexpr (TR::transit) {
            double d = dose;
            if (t >= dose_change_time) d = dose_after;
            const double tst = t - last_treatment;
            const double transit = xm::lib<COLD>::exp((ntr * xm::lib<COLD>::log(ktr * tst) - ktr * tst) - lnf);
            return ktr * transit * d;
        }
        return 0.0;
    }

    BDF_INL void rhs(double t, const double (&y)[NS], double (&dydt)[NS]) const
    {
        const double k = cur_ka();
        const double m0 = a00() * y[0];  // = -((ka + ke) y0), exactly
        if constexpr (TR::transit)
            dydt[0] = input(t) + m0;
        else
            dydt[0] = m0;
        if constexpr (TR::two) {
            dydt[1] = k * y[0] - kel * y[1] - kf * y[1] + kb * y[2];
            dydt[2] = kf * y[1] - kb * y[2];
        } else {
            dydt[1] = k * y[0] - kel * y[1];
        }
    }

    // Jacobian (CalculateJacobian_*, .cpp:457-642) is constant within a dosing segment, so the
    // saved Jacobian of cvLsLinSys is re-derived here: A = J (-gamma), then 1 added to the diagonal
    // (SUNMatScaleAddI, sunmatrix_dense_eigen.cpp:128-133). Structural zeros of J make every
    // cofactor term with a zero factor an exact (signed) zero in the closed-form inverse of
    // sunlinsol_dense_eigen.cpp:111-178 / Eigen compute_inverse<3>, so only the other terms are
    // formed; the remaining products and differences are the reference's.
    struct Inv {
        double i00, i10, i11, i12, i20, i21, i22;
    };

    BDF_INL void lin_setup(double gamma, Inv& r) const
    {
        const double a = cur_ka();
        const double ng = -gamma;
        const double a00 = (-(a + ke)) * ng + 1.0;
        const double a10 = a * ng;
        if constexpr (TR::two) {
            const double a11 = (-(kel + kf)) * ng + 1.0;
            const double a12 = kb * ng;
            const double a21 = kf * ng;
            const double a22 = (-kb) * ng + 1.0;
            const double c0 = a11 * a22 - a12 * a21;  // cofactor(0,0)
            const double invdet = frcp(c0 * a00);     // det = c0*a00 + (+-0) + (+-0)
            r.i00 = c0 * invdet;
            r.i10 = (-(a10 * a22)) * invdet;
            r.i11 = (a22 * a00) * invdet;
            r.i12 = (-(a00 * a12)) * invdet;
            r.i20 = (a10 * a21) * invdet;
            r.i21 = (-(a21 * a00)) * invdet;
            r.i22 = (a00 * a11) * invdet;
        } else {
            const double a11 = (-kel) * ng + 1.0;
            const double invdet = frcp(a00 * a11);  // a00*a11 - a01*a10, a01 = -0
            r.i00 = a11 * invdet;
            r.i10 = -a10 * invdet;
            r.i11 = a00 * invdet;
            r.i12 = r.i20 = r.i21 = r.i22 = 0.0;
        }
    }

    // x = A^-1 b with the full row sums (structural zeros included, see rhs)
    BDF_INL static double inv_at(const Inv& r, int i, int j)
    {
        const double m[3][3] = {{r.i00, 0.0, 0.0}, {r.i10, r.i11, r.i12}, {r.i20, r.i21, r.i22}};
        return m[i][j];
    }
    // SUNLinSolSolve_Dense_Eigen2x2 (sunlinsol_dense_eigen.cpp:157-167): inv(i,0) b0 + inv(i,1) b1;
    // _Eigen3x3 (:169-176): Eigen's Matrix3d * VectorXd, whose row sum is its unrolled reduction
    // p0 + (p1 + p2) (checked against the vendored Eigen, oracle/eigen_ls.cpp)
    BDF_INL void lin_solve(const Inv& r, const double (&b)[NS], double (&x)[NS]) const
    {
        cfor<0, NS>([&](auto I) __attribute__((always_inline)) {
            constexpr int i = CI(I);
            if constexpr (NS == 3)
                x[i] = inv_at(r, i, 0) * b[0] + (inv_at(r, i, 1) * b[1] + inv_at(r, i, 2) * b[2]);
            else
                x[i] = inv_at(r, i, 0) * b[0] + inv_at(r, i, 1) * b[1];
        });
    }

    // ---- lane-vector forms for bdf_vec.h (lane i = component i; same expressions)
    // Lane i evaluates ((c0 u - c1 y) - c2 y) + c3 y2 and keeps the prefix its component's
    // expression has: lane 0 c0 u = a00 y0; lane 1 the whole chain with (ka, kel, kf, kb), u = y0;
    // lane 2 c0 u - c1 y = kf y1 - kb y2, u = y1. u comes from one DPP quad permutation
    // (lanes 0, 1 <- lane 0, lane 2 <- lane 1), y2 from a row broadcast.
    BDF_INL void rhs_columns(double (&c)[4]) const
    {
        const double k = cur_ka();
        if constexpr (TR::two) {
            const double p[3] = {a00(), k, kf}, qv[3] = {0.0, kel, kb}, rv[3] = {0.0, kf, 0.0}, sv[3] = {0.0, kb, 0.0};
            c[0] = vec::from_array<3>(p);
            c[1] = vec::from_array<3>(qv);
            c[2] = vec::from_array<3>(rv);
            c[3] = vec::from_array<3>(sv);
        } else {
            const double p[2] = {a00(), k}, qv[2] = {0.0, kel};
            c[0] = vec::from_array<2>(p);
            c[1] = vec::from_array<2>(qv);
            c[2] = c[3] = 0.0;
        }
    }
    BDF_INL double rhs_v(double t, double y, const double (&c)[4]) const
    {
        const int ln = vec::lane_id();
        // quad_perm [0, 0, 1, 3]
        const double u = __builtin_amdgcn_mov_dpp(y, 0xD0, 0xf, 0xf, false);
        const double t1 = c[0] * u;
        const double t2 = t1 - c[1] * y;
        double f;
        if constexpr (TR::two) {
            const double t3 = t2 - c[2] * y;
            const double t4 = t3 + c[3] * vec::bc<2>(y);
            f = (ln == 1) ? t4 : t2;
        } else {
            f = t2;
        }
        if constexpr (TR::transit) {
            const double uin = input(t);
            f = (ln == 0) ? uin + t1 : f;
        } else {
            f = (ln == 0) ? t1 : f;
        }
        return f;
    }
    BDF_INL void lin_setup_v(double gamma, double (&icol)[NS]) const
    {
        Inv r;
        lin_setup(gamma, r);
        cfor<0, NS>([&](auto J) __attribute__((always_inline)) {
            constexpr int j = CI(J);
            double col[NS];
            cfor<0, NS>([&](auto I) __attribute__((always_inline)) { col[CI(I)] = inv_at(r, CI(I), j); });
            icol[j] = vec::from_array<NS>(col);
        });
    }
};

// CheckGiveTreatment (.cpp:644-671)
BDF_INL bool check_give_treatment(double t, const uint8_t* skipped, int intermittent)
{
    bool give = true;
    int day = (int)floor(t / 24.0);
    if (day >= 0 && day < 29 && skipped[day]) give = false;
    if (intermittent == 1) {
        double tiw = t - 7.0 * 24.0 * floor(t / (7.0 * 24.0));
        if (tiw >= 5.0 * 24.0) give = false;
    } else if (intermittent == 2) {
        double tic = t - 28.0 * 24.0 * floor(t / (28.0 * 24.0));
        if (tic >= 21.0 * 24.0) give = false;
    } else if (intermittent == 3) {
        double tiw = t - 7.0 * 24.0 * floor(t / (7.0 * 24.0));
        if (tiw >= 4.0 * 24.0) give = false;
    }
    return give;
}

// ---------------------------------------------------------------------------------------------

// UNI (lanes_per_wave == 1): the wavefront integrates ONE trajectory and its index is made
// wave-uniform (readfirstlane), so every value derived from it is uniform to the compiler: the
// model data come in through scalar loads and every solver branch is a uniform (scalar) branch
// instead of exec-mask manipulation. All 64 lanes compute and store the same numbers (a
// same-address same-value store from every lane is one well-defined store).
// MODE: POPK_LANES (lanes_per_wave trajectories per wavefront, bdf_lane.h), POPK_UNI (one
// trajectory per wavefront, scalar state: bdf_uni.h), POPK_VEC (one trajectory per wavefront,
// state vectors across lanes: bdf_vec.h). All three give the same bits.
enum { POPK_LANES = 0, POPK_UNI = 1, POPK_VEC = 2 };

// the kernel's argument list as a struct: the byte offsets of its members are those of the kernarg
// segment (the code object's .args metadata: logp_direct at 216 ... place_out at 272)
struct PopkArgsLayout {
    PopPKDevModel m;
    int64_t ntraj;
    int lpw;
    const double* values;
    double* logp_direct;
    double* patient_llh;
    int32_t* traj_status;
    double* traj_out;
    bcm3hip_traj_stats* stats_out;
    const int32_t* n_dev;
    int32_t* steps_out;
    uint64_t* place_out;
};
static_assert(offsetof(PopkArgsLayout, logp_direct) == 216 && offsetof(PopkArgsLayout, place_out) == 272,
              "popk_traj_kernel's kernarg layout changed: re-check the code object's .args offsets");

template <int PKT, int MODE, bool STATS>
__global__ void __launch_bounds__(256) popk_traj_kernel(PopPKDevModel m, int64_t ntraj, int lpw,
                                                        const double* __restrict__ values,
                                                        double* __restrict__ logp_direct,
                                                        double* __restrict__ patient_llh,
                                                        int32_t* __restrict__ traj_status,
                                                        double* __restrict__ traj_out,
                                                        bcm3hip_traj_stats* __restrict__ stats_out,
                                                        const int32_t* __restrict__ n_dev,
                                                        int32_t* __restrict__ steps_out,
                                                        uint64_t* __restrict__ place_out)
{
    using TR = PKTraits<PKT>;
    constexpr int NS = TR::NS;
    constexpr bool UNI = (MODE != POPK_LANES);
    constexpr bool VEC = (MODE == POPK_VEC);
    // library functions out of line (libm_exact.h xm::lib) in both one-trajectory-per-wavefront
    // kernels. Round 6 closed the round-4 question: the scalar-state kernel built this way under the
    // product's flags is bit-identical to the inlining build on all 6 PK models x 7 dosing rules x 3
    // solver forms (tools/flag_diff.py, profiles/r06e_flag_diff.txt), so the inline workaround is
    // dropped; BCM3_UNI_INLINE restores it for diagnostics
#ifdef BCM3_UNI_INLINE
    constexpr bool COLD = VEC;
#else
    constexpr bool COLD = UNI;
#endif
    const int lane = threadIdx.x & 63;
#ifdef BCM3_TABLES_LDS
    {
        const unsigned long long* src = reinterpret_cast<const unsigned long long*>(&xm::xm_tables);
        unsigned long long* dst = reinterpret_cast<unsigned long long*>(&lds_tables);
        for (int i = threadIdx.x; i < (int)(sizeof(xm::GlibcPow) / 8); i += blockDim.x) dst[i] = src[i];
        __syncthreads();
    }
#endif
    // n_dev: the number of evaluations is a device value (the speculative batches of the sampler
    // size themselves on the device); the grid covers the maximum and the rest return here
    if (n_dev) ntraj = (int64_t)__builtin_amdgcn_readfirstlane(*n_dev) * m.P;
    int64_t g;
    if constexpr (UNI) {
        g = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
        if (g >= ntraj) return;
    } else {
        if (lane >= lpw) return;
        const int64_t gwave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        g = gwave * lpw + lane;
        if (g >= ntraj) return;
    }
    // placement diagnostics (BCM3HIP_OPT_PLACEMENT_LOG): where (HW_ID, XCC_ID) and when (100 MHz
    // wall clock) this trajectory ran; read from hardware registers, written by lane 0
    const uint64_t place_t0 = place_out ? wall_clock64() : 0;
    const uint64_t place_c0 = place_out ? __builtin_amdgcn_s_memtime() : 0;  // shader clock
    const int P = m.P;
    const int64_t e = g / P;
    const int j = (int)(g - e * P);
    const int T = m.T;
    const double* v = values + e * m.d;
    const int npk = m.num_pk_params, npop = m.num_pk_pop_params;

    // ---- parameter map (.cpp:263-310)
    const int sdix = m.sd_ix;
    const double sd = transform_var<COLD>(m.transforms[sdix], v[sdix]);
    const double sd2 = transform_var<COLD>(m.transforms[sdix + 1], v[sdix + 1]);
    PKLane<PKT, COLD> mdl;
    // single-patient likelihood (LikelihoodPharmacokineticTrajectory.cpp:226-259): the rates are the
    // transformed variables; the population likelihood draws ka and CL per patient (.cpp:283-286)
    const bool single = (m.param_map == BCM3HIP_PARAM_MAP_SINGLE);
    const double vod = isnan(m.fixed_vod) ? transform_var<COLD>(m.transforms[3], v[3]) : m.fixed_vod;
    if (single) {
        mdl.ka = transform_var<COLD>(m.transforms[0], v[0]);
        mdl.ke = transform_var<COLD>(m.transforms[1], v[1]);
        mdl.kel = transform_var<COLD>(m.transforms[2], v[2]) / vod;
    } else {
        mdl.ka = fastpow10<COLD>(quantile_normal(v[npk + npop * (j + 1) + 0], v[0], v[npk + 0]));
        mdl.ke = transform_var<COLD>(m.transforms[1], v[1]);
        mdl.kel = fastpow10<COLD>(quantile_normal(v[npk + npop * (j + 1) + 1], v[2], v[npk + 1])) / vod;
    }
    mdl.kf = mdl.kb = 0.0;
    if constexpr (TR::two) {
        if (isnan(m.fixed_kf)) {
            mdl.kf = transform_var<COLD>(m.transforms[4], v[4]);
            mdl.kb = transform_var<COLD>(m.transforms[5], v[5]);
        } else {
            mdl.kf = m.fixed_kf;
            mdl.kb = m.fixed_kb;
        }
    }
    mdl.ktr = mdl.ntr = mdl.lnf = 0.0;
    if constexpr (TR::transit) {
        const int ni = m.n_transit_ix, ti = m.transit_time_ix;
        mdl.ntr = transform_var<COLD>(m.transforms[ni], v[ni]);
        mdl.ktr = (mdl.ntr + 1) / transform_var<COLD>(m.transforms[ti], v[ti]);
        const double n = mdl.ntr;
        mdl.lnf = 0.9189385332046727 + (n + 0.5) * xm::lib<COLD>::log(n) - n + xm::lib<COLD>::log(1 + 1 / (12.0 * n));
    }
    const double interval = m.dosing_interval[j];
    double tsw = 0.0;
    mdl.ka2 = 0.0;
    if constexpr (TR::biphasic) {
        const int bi = m.biphasic_time_ix, ai = m.absorption2_ix;
        tsw = transform_var<COLD>(m.transforms[bi], v[bi]);
        const double lim = interval - 1e-2;
        // (the population likelihood keeps the switch inside the dosing interval, .cpp:303-305;
        //  the single-patient one does not, LikelihoodPharmacokineticTrajectory.cpp:253)
        tsw = (!single && lim < tsw) ? lim : tsw;
        mdl.ka2 = transform_var<COLD>(m.transforms[ai], v[ai]);
    }
    if constexpr (UNI && !VEC) {
        // values returned by out-of-line calls (ndtri_lower) count as divergent to the compiler;
        // re-assert uniformity once so the whole solve stays on scalar control flow (the VEC
        // solver keeps them in VGPRs: its control flow depends on them only through norms made
        // uniform by lane_sum, and 20 fewer live SGPRs cut its SGPR spilling)
        mdl.ka = wave_uniform(mdl.ka);
        mdl.ke = wave_uniform(mdl.ke);
        mdl.kel = wave_uniform(mdl.kel);
        mdl.kf = wave_uniform(mdl.kf);
        mdl.kb = wave_uniform(mdl.kb);
        mdl.ktr = wave_uniform(mdl.ktr);
        mdl.ntr = wave_uniform(mdl.ntr);
        mdl.lnf = wave_uniform(mdl.lnf);
        mdl.ka2 = wave_uniform(mdl.ka2);
        tsw = wave_uniform(tsw);
    }
    mdl.dose = m.dose[j];
    mdl.dose_after = m.dose_after_dose_change[j];
    mdl.dose_change_time = m.dose_change_time[j];
    mdl.last_treatment = 0.0;
    mdl.biphasic_switch = true;
    const int intermittent = m.intermittent[j];
    const uint8_t* skipped = m.skipped_days + 29 * j;

    // SetDiscontinuity (.cpp:357-364)
    double current_dose_time;
    double next_disc;
    if constexpr (TR::biphasic) {
        current_dose_time = 0.0;
        next_disc = tsw;
    } else {
        current_dose_time = interval;
        next_disc = interval;
    }
    // (a non-positive discontinuity time is ignored by ODESolver::SetDiscontinuity; the
    //  host rejects such models, so next_disc > 0 here)

    const double conversion = UNI ? wave_uniform((1e6 / m.MW) / vod) : (1e6 / m.MW) / vod;
    const double sd_u = UNI ? wave_uniform(sd) : sd, sd2_u = UNI ? wave_uniform(sd2) : sd2;
    const int nsim = m.simulate_until[j];
    const double* obs = m.observed + (int64_t)j * T;
    double* tro = traj_out ? traj_out + g * (int64_t)NS * T : nullptr;

    double llh = 0.0;
    int nsteps = 0;         // BDF steps of the solve (steps_out: the sampler's dispatch-order hint)
    bool llh_done = false;  // NaN concentration seen: llh = -inf, stop accumulating
    int status = BCM3HIP_STATUS_OK;

    std::conditional_t<VEC, vec::VecState<NS, STATS>, BdfState<NS, typename PKLane<PKT, COLD>::Inv>> s;
    s.cnt = {};
    s.nst = 0;
#ifdef BCM3_PHASES
    cfor<0, NPHASES>([&](auto k) __attribute__((always_inline)) { s.ph[CI(k)] = 0; });
    cfor<0, QMAX + 1>([&](auto k) __attribute__((always_inline)) { s.qh[CI(k)] = 0; });
    s.tlast = (unsigned)clock64();
    for (int k = 0; k < 16; k++) BDF_PH(23);  // the marker's own cost
    s.tlast = (unsigned)clock64();
#endif

    // observation term for output index i with state yi (.cpp:412-423)
    auto observe = [&](int i, const double (&yi)[NS]) __attribute__((always_inline)) {
        if (tro) {
            cfor<0, NS>([&](auto k) __attribute__((always_inline)) { tro[CI(k) * T + i] = yi[CI(k)]; });
        }
        if (llh_done) return;
        const double x = conversion * yi[1];
        const double yo = obs[i];
        if (!isnan(yo)) {
            const double xm = (x < 0.0) ? 0.0 : x;
            llh += log_pdf_tnu4<COLD>(x, yo, sd_u + sd2_u * xm);
        }
        // population likelihood: a NaN concentration ends the patient at -inf (.cpp:418-421); the
        // single-patient likelihood has no such rule, NaN reaches the caller as in the reference
        if (isnan(x) && !single) {
            llh = -INFINITY;
            llh_done = true;
        }
    };

    if (tro) {
        for (int k = 0; k < NS * T; k++) tro[k] = NAN;
    }

    if (nsim > 0) {
        double y0[NS];
        y0[0] = TR::transit ? 0.0 : mdl.dose;
        cfor<1, NS>([&](auto k) __attribute__((always_inline)) { y0[CI(k)] = 0.0; });

        // ODESolver::SolveReturnSolution: rows with t < DBL_EPSILON take y0
        int tpi = 0;
        bool done = false;
        while (m.time[tpi] < 2.220446049250313e-16) {
            observe(tpi, y0);
            tpi++;
            if (tpi == nsim) {
                done = true;
                break;
            }
        }
        if (!done) {
            const double end_time = m.time[nsim - 1];
            double next_out = m.time[tpi];
            // ODESolverCVODE::Solve
            s.rtol = m.rtol;
            s.atol = m.atol;
            s.unity = m.unity;
            // |y| ewt <= 1/rtol (1 + few ulp), so the sum of squares stays far below NS/UROUND^2
            s.check_tolsf = !((m.rtol >= 1e-10) && (m.atol >= 0.0));
            cfor<0, QMAX + 2>([&](auto k) __attribute__((always_inline)) { s.tau[CI(k)] = 0.0; });
            s.saved_tq5 = 0.0;
            s.hprime = s.h = s.eta = 0.0;
            s.tstopset = 0;
            double y[NS];
            cfor<0, NS>([&](auto k) __attribute__((always_inline)) { y[CI(k)] = y0[CI(k)]; });
            if constexpr (VEC)
                vec::reinit<NS>(s, mdl, 0.0, y);
            else
                reinit<NS>(s, 0.0, y);
            s.tstop = next_disc;
            s.tstopset = 1;
            int current_step = 0;
            bool hot = false;  // previous step was a plain CV_SUCCESS (uni::cvode_one_step_u)
#ifdef BCM3_PRIO_STEPS
            int prio_level = 0;
#endif
            for (;;) {
                double tret = 0.0;
                int result;
#ifdef BCM3_PRIO_STEPS
                // (variant) a trajectory that has run long gets the higher issue priority on a shared
                // SIMD (s_setprio; the launch waits for its longest trajectory): checked once per
                // return to this loop
                if (BDF_UNLIKELY(current_step >= BCM3_PRIO_STEPS * (prio_level + 1) && prio_level < 3)) {
                    prio_level++;
                    if (prio_level == 1) __builtin_amdgcn_s_setprio(1);
                    else if (prio_level == 2) __builtin_amdgcn_s_setprio(2);
                    else __builtin_amdgcn_s_setprio(3);
                }
#endif
                if constexpr (VEC) {
                    // after a plain step: run the following plain steps in vec::fast_run (same
                    // results, one exit test per step); an order change the last step decided is
                    // made here first, as cvode_entry would (it always comes with hprime != h)
                    const bool fast = hot & ((s.qprime == s.q) | (s.hprime != s.h)) & (s.check_tolsf == 0) &
                                      (s.tstopset != 0) & (s.tstop == next_disc);
                    vec::Pending pd;
                    if (BDF_LIKELY(fast)) {
                        if (BDF_UNLIKELY(s.qprime != s.q)) {
                            vec::adjust_order(s, s.qprime - s.q);
                            s.q = s.qprime;
                            s.L = s.q + 1;
                            s.qwait = s.L;
                        }
                        const double tlim = (next_out < end_time) ? next_out : end_time;
                        const int ms = m.max_steps;
                        switch (s.q) {
                        case 1: result = vec::fast_run<1, NS>(s, mdl, y, tret, tlim, current_step, ms, pd); break;
                        case 2: result = vec::fast_run<2, NS>(s, mdl, y, tret, tlim, current_step, ms, pd); break;
                        case 3: result = vec::fast_run<3, NS>(s, mdl, y, tret, tlim, current_step, ms, pd); break;
                        case 4: result = vec::fast_run<4, NS>(s, mdl, y, tret, tlim, current_step, ms, pd); break;
                        default: result = vec::fast_run<5, NS>(s, mdl, y, tret, tlim, current_step, ms, pd); break;
                        }
                    } else {
                        result = vec::cvode_entry<NS>(s, mdl, end_time, y, tret, hot, pd);
                    }
                    if (result == vec::NEED_ATTEMPTS)
                        result = vec::attempt_loop<NS>(s, mdl, y, tret, pd.saved_t, pd.eta_eff, pd.r, pd.dsm);
                } else if constexpr (UNI)
                    result = uni::cvode_one_step_u<NS>(s, mdl, end_time, y, tret, hot);
                else
                    result = cvode_one_step<NS>(s, mdl, end_time, y, tret);
                if (result < 0) {
                    status = BCM3HIP_STATUS_SOLVER_FAIL;
                    break;
                }
                const double t = tret;
                current_step++;
                // one scalar branch for the common step: nothing to output, no discontinuity,
                // not at the end (the checks below in the reference's order otherwise)
                const bool rare = (result != CV_SUCCESS) | (tret >= next_out) | (t >= end_time) |
                                  (current_step == m.max_steps) | (next_disc == t);
                hot = !rare;
                if (BDF_LIKELY(!rare)) continue;
                if (result == CV_SUCCESS) {
                    if constexpr (VEC)
                        vec::to_array<NS>(s.zn[0], y);
                    else
                        cfor<0, NS>([&](auto k) __attribute__((always_inline)) { y[CI(k)] = s.zn[0][CI(k)]; });
                }
                while (tret >= next_out) {
                    double dky[NS];
                    int dr;
                    if constexpr (VEC)
                        dr = vec::get_dky_array<NS>(s, m.time[tpi], dky);
                    else
                        dr = get_dky<NS>(s, m.time[tpi], dky);
                    if (dr != CV_SUCCESS) {
                        status = BCM3HIP_STATUS_SOLVER_FAIL;
                        break;
                    }
                    observe(tpi, dky);
                    tpi++;
                    if (tpi >= nsim) {
                        next_out = INFINITY;
                        break;
                    }
                    next_out = m.time[tpi];
                }
                if (status != BCM3HIP_STATUS_OK) break;
                if (t >= end_time) break;
                if (current_step == m.max_steps) {
                    status = BCM3HIP_STATUS_SOLVER_FAIL;
                    break;
                }
                if (result == CV_TSTOP_RETURN || next_disc == t) {
                    // discontinuity callback
                    if constexpr (TR::biphasic) {
                        if (mdl.biphasic_switch) {
                            mdl.biphasic_switch = false;
                            current_dose_time += interval;
                            next_disc = current_dose_time;
                        } else if (check_give_treatment(t, skipped, intermittent)) {
                            double d = mdl.dose;
                            if (t >= mdl.dose_change_time) d = mdl.dose_after;
                            y[0] = y[0] + d;
                            mdl.biphasic_switch = true;
                            next_disc = current_dose_time + tsw;
                        } else {
                            current_dose_time += interval;
                            next_disc = current_dose_time;
                        }
                    } else {
                        current_dose_time += interval;
                        if (check_give_treatment(t, skipped, intermittent)) {
                            double d = mdl.dose;
                            if (t >= mdl.dose_change_time) d = mdl.dose_after;
                            if constexpr (TR::transit)
                                mdl.last_treatment = t;
                            else
                                y[0] = y[0] + d;
                        }
                        next_disc = current_dose_time;
                    }
                    if constexpr (VEC)
                        vec::reinit<NS>(s, mdl, t, y);
                    else
                        reinit<NS>(s, t, y);
                    s.tstop = next_disc;
                    s.tstopset = 1;
                }
            }
            nsteps = current_step;
        }
    }
    if (status != BCM3HIP_STATUS_OK) llh = -INFINITY;

#ifdef BCM3_PHASES
    if (tro) cfor<0, NPHASES>([&](auto k) __attribute__((always_inline)) { tro[CI(k)] = (double)s.ph[CI(k)]; });
    if (tro) cfor<1, QMAX + 1>([&](auto k) __attribute__((always_inline)) { tro[NPHASES + CI(k) - 1] = (double)s.qh[CI(k)]; });
#endif
#ifdef BCM3_LATE_ARGS
    {
        // (variant) the output pointers read from the kernarg segment only now, through a laundered
        // segment pointer, so that none of them holds scalar registers through the solve
        const char* ka = (const char*)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(ka));
        const PopkArgsLayout* A = reinterpret_cast<const PopkArgsLayout*>(ka);
        logp_direct = A->logp_direct;
        patient_llh = A->patient_llh;
        traj_status = A->traj_status;
        stats_out = A->stats_out;
        steps_out = A->steps_out;
        place_out = A->place_out;
    }
#endif
    // one lane stores a wave-uniform trajectory's results (UNI / VEC: every lane holds the same
    // values; 64 same-address stores were 375 B of write traffic per trajectory)
    const bool writer = !UNI || lane == 0;
    if (logp_direct && writer) logp_direct[e] = 0.0 + llh;  // P == 1: logp = 0 + patient term
    if (patient_llh && writer) patient_llh[g] = llh;
    if (traj_status && writer) traj_status[g] = status;
    if (steps_out && m.P == 1 && writer) steps_out[g] = nsteps;
    if (UNI && place_out && lane == 0) {
        // HW_ID (hwreg 4, all 32 bits) and XCC_ID (hwreg 20, bits 0..3)
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
        const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
        // upper half: the shader-clock cycles the trajectory took (s_memtime), so the in-kernel
        // clock is that / (wall-clock end - start) x 100 MHz
        const uint64_t cyc = __builtin_amdgcn_s_memtime() - place_c0;
        place_out[4 * g + 0] = (uint64_t)hw | (cyc << 32);
        place_out[4 * g + 1] = xcc;
        place_out[4 * g + 2] = place_t0;
        place_out[4 * g + 3] = wall_clock64();
    }
    if (STATS && stats_out && writer) {
        bcm3hip_traj_stats st;
        st.nst = s.cnt.nst_total;
        st.nfe = s.cnt.nfe;
        st.nni = s.cnt.nni;
        st.nsetups = s.cnt.nsetups;
        st.nje = s.cnt.nje;
        st.netf = s.cnt.netf;
        st.ncfn = s.cnt.ncfn;
        st.nreinit = s.cnt.nreinit;
        stats_out[g] = st;
    }
}

// Sequential per-evaluation sum over patients with the reference's break at -inf
// (LikelihoodPopPKTrajectory.cpp:427-440); status = max over patients.
__global__ void __launch_bounds__(256) popk_reduce_kernel(int64_t n, int P, const double* __restrict__ patient_llh,
                                                          const int32_t* __restrict__ traj_status,
                                                          double* __restrict__ logp, int32_t* __restrict__ status,
                                                          const int32_t* __restrict__ n_dev)
{
    if (n_dev) n = *n_dev;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n) return;
    double acc = 0.0;
    int32_t st = 0;
    for (int j = 0; j < P; j++) {
        acc += patient_llh[e * P + j];
        int32_t sj = traj_status[e * P + j];
        st = sj > st ? sj : st;
        if (acc == -INFINITY) break;
    }
    logp[e] = acc;
    if (status) status[e] = st;
}

}  // namespace bcm3hip

const xm::GlibcPow* bcm3_pow_tables(int* from_libm);  // libm_tables.cpp

namespace bcm3hip {

hipError_t popk_prepare_device(int* glibc)
{
    static std::mutex mu;
    static int state[64] = {};  // per device: 0 not uploaded, 1 libm's tables, 2 computed ones
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(mu);
    if (dev >= 0 && dev < 64 && state[dev]) {
        if (glibc) *glibc = state[dev] == 1;
        return hipSuccess;
    }
    int found = 0;
    const xm::GlibcPow* t = bcm3_pow_tables(&found);
    e = hipMemcpyToSymbol(HIP_SYMBOL(xm::xm_tables), t, sizeof(*t));
    if (e != hipSuccess) return e;
    if (dev >= 0 && dev < 64) state[dev] = found ? 1 : 2;
    if (glibc) *glibc = found;
    return hipSuccess;
}

hipError_t launch_popk(const PopPKDevModel& m, int64_t n, const double* values, double* logp, int32_t* status,
                       double* patient_llh_scratch, int32_t* traj_status_scratch, double* traj_out,
                       bcm3hip_traj_stats* stats_out, int lanes_per_wave, int block_waves, int uni_solver,
                       hipStream_t stream, hipEvent_t ev_start, hipEvent_t ev_stop, int block_lds,
                       const int32_t* n_dev, int32_t* steps_out, uint64_t* place_out)
{
    const int64_t ntraj = n * (int64_t)m.P;
    if (ntraj == 0) return hipSuccess;
    const int lpw = lanes_per_wave < 1 ? 1 : (lanes_per_wave > 64 ? 64 : lanes_per_wave);
    const int bw = block_waves < 1 ? 1 : (block_waves > 4 ? 4 : block_waves);
    const int64_t nwaves = (ntraj + lpw - 1) / lpw;
    const int64_t nblocks = (nwaves + bw - 1) / bw;
    dim3 grid((unsigned)nblocks), block(64 * bw);
    const bool direct = (m.P == 1);
    const bool uni = (lpw == 1) && ntraj < (int64_t)1 << 30;
    const bool vec_state = uni && (uni_solver == 0);
    double* logp_direct = direct ? logp : nullptr;
    // one patient: the trajectory status is the evaluation status, written in place (no copy kernel)
    int32_t* tstat = (direct && status) ? status : traj_status_scratch;
    if (ev_start) hipEventRecord(ev_start, stream);
#ifdef BCM3_VEC_STATS_ALWAYS
    constexpr bool vec_nostats = false;  // (variant) the counting kernel for every vector-state launch
#else
    constexpr bool vec_nostats = true;
#endif
#define LAUNCH(PKT)                                                                                           \
    if (vec_state && !stats_out && vec_nostats)                                                               \
        hipLaunchKernelGGL((popk_traj_kernel<PKT, POPK_VEC, false>), grid, block, block_lds, stream, m, ntraj, lpw,     \
                           values, logp_direct, patient_llh_scratch, tstat, traj_out, nullptr, n_dev, steps_out, place_out); \
    else if (vec_state)                                                                                       \
        hipLaunchKernelGGL((popk_traj_kernel<PKT, POPK_VEC, true>), grid, block, block_lds, stream, m, ntraj, lpw,      \
                           values, logp_direct, patient_llh_scratch, tstat, traj_out, stats_out, n_dev, steps_out, place_out); \
    else if (uni)                                                                                             \
        hipLaunchKernelGGL((popk_traj_kernel<PKT, POPK_UNI, true>), grid, block, block_lds, stream, m, ntraj, lpw, values, \
                           logp_direct, patient_llh_scratch, tstat, traj_out, stats_out, n_dev, steps_out, place_out); \
    else                                                                                                      \
        hipLaunchKernelGGL((popk_traj_kernel<PKT, POPK_LANES, true>), grid, block, block_lds, stream, m, ntraj, lpw, values,  \
                           logp_direct, patient_llh_scratch, tstat, traj_out, stats_out, n_dev, steps_out, place_out)
#ifdef BCM3_DEV_TWO_VEC
    // development build (tools/resource_two_vec.sh): only the C3 kernel, compiled in seconds
    if (m.pk_type != BCM3HIP_PK_TWO || !vec_state || stats_out) return hipErrorInvalidValue;
    hipLaunchKernelGGL((popk_traj_kernel<BCM3HIP_PK_TWO, POPK_VEC, !vec_nostats>), grid, block, block_lds, stream, m, ntraj,
                       lpw, values, logp_direct, patient_llh_scratch, tstat, traj_out, nullptr, n_dev, steps_out, place_out);
#else
    switch (m.pk_type) {
    case BCM3HIP_PK_ONE: LAUNCH(BCM3HIP_PK_ONE); break;
    case BCM3HIP_PK_TWO: LAUNCH(BCM3HIP_PK_TWO); break;
    case BCM3HIP_PK_ONE_BIPHASIC: LAUNCH(BCM3HIP_PK_ONE_BIPHASIC); break;
    case BCM3HIP_PK_TWO_BIPHASIC: LAUNCH(BCM3HIP_PK_TWO_BIPHASIC); break;
    case BCM3HIP_PK_ONE_TRANSIT: LAUNCH(BCM3HIP_PK_ONE_TRANSIT); break;
    case BCM3HIP_PK_TWO_TRANSIT: LAUNCH(BCM3HIP_PK_TWO_TRANSIT); break;
    default: return hipErrorInvalidValue;
    }
#endif
#undef LAUNCH
    if (ev_stop) hipEventRecord(ev_stop, stream);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
    const int tb = 256;
    const unsigned rb = (unsigned)((n + tb - 1) / tb);
    if (!direct) {
        hipLaunchKernelGGL(popk_reduce_kernel, dim3(rb), dim3(tb), 0, stream, n, m.P, patient_llh_scratch,
                           traj_status_scratch, logp, status, n_dev);
    }
    return hipGetLastError();
}

}  // namespace bcm3hip
