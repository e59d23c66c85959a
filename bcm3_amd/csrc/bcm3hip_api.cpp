// bcm3hip_api.cpp -- C-ABI of libbcm3hip.so (include/bcm3hip.h).
//
// Owns one HIP stream, the device copy of the model data and grow-only scratch buffers per
// context. The batched evaluation replaces the reference's per-chain TaskManager fan-out
// (SamplerPT::DoMutateMove, src/sampler/SamplerPT.cpp:308-319): one launch evaluates every
// chain's proposal of a mutate step.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <new>
#include <vector>

#include <algorithm>

#include "../../include/bcm3hip.h"
#include "libm_exact.h"
#include "popk_kernel.h"

const xm::GlibcPow* bcm3_pow_tables(int* from_libm);  // libm_tables.cpp

using namespace bcm3hip;

namespace bcm3hip {
struct CellPopDev;
int cellpop_create(int device, const bcm3hip_cellpop_model* m, CellPopDev** out);
int cellpop_precompile(const bcm3hip_cellpop_model* m);
void cellpop_destroy(CellPopDev* c);
int cellpop_launch(CellPopDev* c, size_t n, const double* values, double* logp, int32_t* status, hipStream_t s,
                   hipEvent_t e0, hipEvent_t e1);
int cellpop_cells(CellPopDev* c, size_t item, int32_t* count, bcm3hip_cell_record* rec, double* values, double* end_y);
hipError_t launch_cp_accumulate(int32_t n, double* logp, int32_t* status, const double* x, const int32_t* xstatus,
                                hipStream_t s);
hipError_t launch_cp_assign(int32_t n_problems, int32_t R, int32_t nsim, const double* lik, unsigned char* ws_global,
                            size_t ws_stride, int32_t* match, double* sum, int32_t* ok, hipStream_t s);
size_t cp_assign_ws_bytes(int n);
// the dynamic workspace plus the larger kernel's static LDS (cp_timepoints_kernel, ~8.4 KB) stay within
// 64 KB, the workgroup limit of parts smaller than gfx950's 160 KB
inline bool cp_assign_lds_fits(int n) { return cp_assign_ws_bytes(n) <= 52 * 1024; }
}  // namespace bcm3hip

struct bcm3hip_ctx {
    int device = 0;
    int kind = 0;  // 1 popk, 2 analytic, 3 expm pk, 4 cell population
    bcm3hip::CellPopDev* cp = nullptr;
    std::vector<bcm3hip::CellPopDev*> cp_more;  // experiments 1.. of a cell-population likelihood
    double* cp_logp = nullptr;                  // their per-experiment logp / status
    int32_t *cp_status = nullptr, *cp_status0 = nullptr;
    size_t cap_cp = 0, cap_cp_status = 0, cap_cp_status0 = 0;
    int d = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t last0 = nullptr, last1 = nullptr;  // pair of the most recent launch
    bool timed = false;
    // kernel-time log (BCM3HIP_OPT_TIMING_LOG): one event pair per launch, resolved lazily
    bool log_timing = false;
    std::vector<hipEvent_t> log_ev;
    size_t log_used = 0;
    PopPKDevModel pm{};
    AnalyticDevModel am{};
    ExpmPKDevModel xm{};
    std::vector<void*> model_allocs;
    // grow-only scratch
    double* values = nullptr;
    size_t cap_values = 0;
    double* logp = nullptr;
    int32_t* status = nullptr;
    size_t cap_n = 0;
    double* pllh = nullptr;
    int32_t* tstatus = nullptr;
    size_t cap_traj = 0, cap_tstatus = 0, cap_status = 0;
    double* traj = nullptr;
    size_t cap_trajout = 0;
    double* exps = nullptr;  // expm pk: [n][n_jobs][n*n]
    size_t cap_exps = 0;
    bcm3hip_traj_stats* stats = nullptr;
    size_t cap_stats = 0;
    // the grow-only scratch above is shared by every launch of the context: a launch on another
    // stream than the previous one waits for that one (scratch_ev), so concurrent callers on
    // different streams cannot overwrite each other's exponentials / per-patient results
    hipEvent_t scratch_ev = nullptr;
    hipStream_t scratch_stream = nullptr;
    bool scratch_used = false;
    int lanes_per_wave = 0;  // 0 = auto (auto_lanes_per_wave)
    int uni_solver = 0;      // BCM3HIP_OPT_UNI_SOLVER
    int block_waves = 1;
    int block_lds = 0;  // BCM3HIP_OPT_BLOCK_LDS
    bool place_log = false;  // BCM3HIP_OPT_PLACEMENT_LOG
    uint64_t* place = nullptr;
    size_t cap_place = 0;
    int64_t place_n = 0;
    hipStream_t place_stream = nullptr;
};

#define HIPCHK(x)                                                                                          \
    do {                                                                                                   \
        hipError_t e_ = (x);                                                                               \
        if (e_ != hipSuccess) {                                                                            \
            fprintf(stderr, "bcm3hip: %s failed: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            return BCM3HIP_ERR_HIP;                                                                        \
        }                                                                                                  \
    } while (0)

template <class T>
static int grow(T*& p, size_t& cap, size_t need)
{
    if (need <= cap) return 0;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    size_t n = need < 256 ? 256 : need;
    if (hipMalloc((void**)&p, n * sizeof(T)) != hipSuccess) return BCM3HIP_ERR_ALLOC;
    cap = n;
    return 0;
}

template <class T>
static int upload(bcm3hip_ctx* c, const T* host, size_t count, const T** dev_out)
{
    *dev_out = nullptr;
    if (count == 0) return 0;
    if (!host) return BCM3HIP_ERR_ARG;
    void* p = nullptr;
    HIPCHK(hipMalloc(&p, count * sizeof(T)));
    c->model_allocs.push_back(p);
    HIPCHK(hipMemcpy(p, host, count * sizeof(T), hipMemcpyHostToDevice));
    *dev_out = (const T*)p;
    return 0;
}

static int ctx_common_init(bcm3hip_ctx* c, int device)
{
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return BCM3HIP_ERR_NODEVICE;
    if (device < 0 || device >= count) return BCM3HIP_ERR_ARG;
    c->device = device;
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipEventCreate(&c->ev0));
    HIPCHK(hipEventCreate(&c->ev1));
    HIPCHK(hipEventCreateWithFlags(&c->scratch_ev, hipEventDisableTiming));
    return 0;
}

extern "C" {

int bcm3hip_device_count(void)
{
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) return 0;
    return count;
}

int bcm3hip_current_device_simds(void)
{
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    return 4 * cus;
}

const char* bcm3hip_error_string(int code)
{
    switch (code) {
    case BCM3HIP_OK: return "success";
    case BCM3HIP_ERR_ARG: return "invalid argument";
    case BCM3HIP_ERR_HIP: return "HIP runtime error";
    case BCM3HIP_ERR_NODEVICE: return "no HIP device";
    case BCM3HIP_ERR_MODEL: return "invalid model description";
    case BCM3HIP_ERR_ALLOC: return "device allocation failed";
    default: return "unknown error";
    }
}

int bcm3hip_libm_pow_tables(void)
{
    // the tables popk_prepare_device uploads (BCM3_POW=computed included)
    int from_libm = 0;
    bcm3_pow_tables(&from_libm);
    return from_libm;
}

int bcm3hip_open_popk(int device, const bcm3hip_popk_model* m, bcm3hip_ctx** out)
{
    if (!m || !out) return BCM3HIP_ERR_ARG;
    *out = nullptr;
    if (m->pk_type < BCM3HIP_PK_ONE || m->pk_type > BCM3HIP_PK_TWO_TRANSIT) return BCM3HIP_ERR_MODEL;
    const bool two = m->pk_type == BCM3HIP_PK_TWO || m->pk_type == BCM3HIP_PK_TWO_BIPHASIC ||
                     m->pk_type == BCM3HIP_PK_TWO_TRANSIT;
    const bool transit = m->pk_type == BCM3HIP_PK_ONE_TRANSIT || m->pk_type == BCM3HIP_PK_TWO_TRANSIT;
    const bool biphasic = m->pk_type == BCM3HIP_PK_ONE_BIPHASIC || m->pk_type == BCM3HIP_PK_TWO_BIPHASIC;
    if (m->N != (two ? 3 : 2)) return BCM3HIP_ERR_MODEL;
    if (m->d <= 0 || m->P <= 0 || m->T < 0 || m->sd_ix < 0 || m->sd_ix + 1 >= m->d) return BCM3HIP_ERR_MODEL;
    if (m->param_map == BCM3HIP_PARAM_MAP_POPULATION) {
        if (m->num_pk_params + m->num_pk_pop_params * m->P + 1 >= m->d) return BCM3HIP_ERR_MODEL;
    } else if (m->param_map == BCM3HIP_PARAM_MAP_SINGLE) {
        // one patient; the variables read by fixed index (LikelihoodPharmacokineticTrajectory.cpp:226-259)
        int need = std::isnan(m->fixed_vod) ? 4 : 3;
        if (two && std::isnan(m->fixed_kf)) need = 6;
        if (biphasic) need = 8;
        if (m->P != 1 || m->d < need) return BCM3HIP_ERR_MODEL;
        if (biphasic && (m->biphasic_time_ix != 6 || m->absorption2_ix != 7)) return BCM3HIP_ERR_MODEL;
    } else {
        return BCM3HIP_ERR_MODEL;
    }
    if (transit && (m->n_transit_ix >= m->d || m->transit_time_ix >= m->d)) return BCM3HIP_ERR_MODEL;
    if (transit && (m->n_transit_ix < 0 || m->transit_time_ix < 0)) return BCM3HIP_ERR_MODEL;
    if (biphasic && (m->biphasic_time_ix < 0 || m->absorption2_ix < 0)) return BCM3HIP_ERR_MODEL;
    for (int j = 0; j < m->P; j++) {
        if (m->simulate_until[j] < 0 || m->simulate_until[j] > m->T) return BCM3HIP_ERR_MODEL;
        // ODESolver::SetDiscontinuity ignores t <= 0 (history-dependent in the reference): reject
        if (!(m->dosing_interval[j] > 0.0)) return BCM3HIP_ERR_MODEL;
    }
    bcm3hip_ctx* c = new (std::nothrow) bcm3hip_ctx();
    if (!c) return BCM3HIP_ERR_ALLOC;
    int r = ctx_common_init(c, device);
    if (r) {
        bcm3hip_close(c);
        return r;
    }
    if (popk_prepare_device(nullptr) != hipSuccess) {
        bcm3hip_close(c);
        return BCM3HIP_ERR_HIP;
    }
    c->kind = 1;
    c->d = m->d;
    PopPKDevModel& pm = c->pm;
    pm.pk_type = m->pk_type;
    pm.N = m->N;
    pm.num_pk_params = m->num_pk_params;
    pm.num_pk_pop_params = m->num_pk_pop_params;
    pm.d = m->d;
    pm.P = m->P;
    pm.T = m->T;
    pm.sd_ix = m->sd_ix;
    pm.n_transit_ix = m->n_transit_ix;
    pm.transit_time_ix = m->transit_time_ix;
    pm.biphasic_time_ix = m->biphasic_time_ix;
    pm.absorption2_ix = m->absorption2_ix;
    pm.max_steps = m->max_steps;
    pm.param_map = m->param_map;
    pm.rtol = m->rtol;
    pm.atol = m->atol;
    pm.MW = m->MW;
    pm.fixed_vod = m->fixed_vod;
    pm.fixed_kf = m->fixed_kf;
    pm.fixed_kb = m->fixed_kb;
    pm.unity = 1.0;
    const size_t P = m->P, T = m->T;
    if ((r = upload(c, m->transforms, (size_t)m->d, &pm.transforms)) ||
        (r = upload(c, m->time, T, &pm.time)) || (r = upload(c, m->observed, P * T, &pm.observed)) ||
        (r = upload(c, m->dose, P, &pm.dose)) || (r = upload(c, m->dosing_interval, P, &pm.dosing_interval)) ||
        (r = upload(c, m->dose_after_dose_change, P, &pm.dose_after_dose_change)) ||
        (r = upload(c, m->dose_change_time, P, &pm.dose_change_time)) ||
        (r = upload(c, m->intermittent, P, &pm.intermittent)) ||
        (r = upload(c, m->skipped_days, P * 29, &pm.skipped_days)) ||
        (r = upload(c, m->simulate_until, P, &pm.simulate_until))) {
        bcm3hip_close(c);
        return r;
    }
    *out = c;
    return 0;
}

int bcm3hip_open_analytic(int device, const bcm3hip_analytic_model* m, bcm3hip_ctx** out)
{
    if (!m || !out) return BCM3HIP_ERR_ARG;
    *out = nullptr;
    if (m->kind != BCM3HIP_ANALYTIC_BANANA && m->kind != BCM3HIP_ANALYTIC_CIRCULAR && m->kind != BCM3HIP_ANALYTIC_DUMMY)
        return BCM3HIP_ERR_MODEL;
    if (m->d < (m->kind == BCM3HIP_ANALYTIC_BANANA ? 2 : 1)) return BCM3HIP_ERR_MODEL;
    bcm3hip_ctx* c = new (std::nothrow) bcm3hip_ctx();
    if (!c) return BCM3HIP_ERR_ALLOC;
    int r = ctx_common_init(c, device);
    if (r) {
        bcm3hip_close(c);
        return r;
    }
    c->kind = 2;
    c->d = m->d;
    c->am.kind = m->kind;
    c->am.d = m->d;
    c->am.p0 = m->p0;
    c->am.p1 = m->p1;
    c->am.p2 = m->p2;
    *out = c;
    return 0;
}

// Eigen::LLT<MatrixXd>::compute for small matrices (llt_inplace<double, Lower>::unblocked, LLT.h): the
// lower triangle of A (row-major, n x n) is factorised in place column by column,
//   L(k,k) = sqrt(A(k,k) - sum_j<k L(k,j)^2),  L(i,k) = (A(i,k) - sum_j<k L(i,j) L(k,j)) / L(k,k);
// false (Eigen's info() != Success) when a pivot is not > 0. The strict upper triangle is zeroed.
static bool llt_lower(int n, double* A)
{
    for (int k = 0; k < n; k++) {
        double x = A[k * n + k];
        for (int j = 0; j < k; j++) x -= A[k * n + j] * A[k * n + j];
        if (!(x > 0.0)) return false;
        x = std::sqrt(x);
        A[k * n + k] = x;
        for (int i = k + 1; i < n; i++) {
            double s = A[i * n + k];
            for (int j = 0; j < k; j++) s -= A[i * n + j] * A[k * n + j];
            A[i * n + k] = s / x;
        }
    }
    for (int i = 0; i < n; i++)
        for (int j = i + 1; j < n; j++) A[i * n + j] = 0.0;
    return true;
}

int bcm3hip_open_mixture(int device, const bcm3hip_mixture_model* m, bcm3hip_ctx** out)
{
    if (!m || !out) return BCM3HIP_ERR_ARG;
    *out = nullptr;
    if (m->kind != BCM3HIP_MIXTURE_NORMAL && m->kind != BCM3HIP_MIXTURE_T) return BCM3HIP_ERR_MODEL;
    if (m->d < 1 || m->d > BCM3HIP_MIXTURE_DMAX || m->K < 1 || m->K > BCM3HIP_MIXTURE_KMAX) return BCM3HIP_ERR_MODEL;
    if (!m->log_weights || !m->means || !m->covariances || (m->kind == BCM3HIP_MIXTURE_T && !m->nus))
        return BCM3HIP_ERR_ARG;
    const int d = m->d, K = m->K;
    std::vector<double> chol((size_t)K * d * d), cst((size_t)K * 3);
    for (int k = 0; k < K; k++) {
        double* L = &chol[(size_t)k * d * d];
        std::copy(m->covariances + (size_t)k * d * d, m->covariances + (size_t)(k + 1) * d * d, L);
        const double nu = (m->kind == BCM3HIP_MIXTURE_T) ? m->nus[k] : 0.0;
        double logc;
        if (m->kind == BCM3HIP_MIXTURE_T && !(nu > 0.0)) return BCM3HIP_ERR_MODEL;
        if (m->kind == BCM3HIP_MIXTURE_T && d == 1) {
            // dmvt with p = 1 is LogPdfT(x, mu, sigma(0,0), nu) (mvt.cpp:129-134), whose constant is
            // -log(sigma sqrt(nu) B(nu/2, 1/2)) (ProbabilityDistributions.cpp:176; boost::math::beta
            // there, its lgamma form here -- parity of this constant unpinned, Boost absent)
            const double sigma = L[0];
            const double beta = std::exp(std::lgamma(0.5 * nu) + std::lgamma(0.5) - std::lgamma(0.5 * nu + 0.5));
            logc = -std::log(sigma * std::sqrt(nu) * beta);
        } else {
            if (!llt_lower(d, L)) return BCM3HIP_ERR_MODEL;
            double det = 0.0;
            for (int i = 0; i < d; i++) det += std::log(L[i * d + i]);
            if (m->kind == BCM3HIP_MIXTURE_NORMAL)
                logc = -det - 0.5 * d * std::log(2.0 * M_PI);  // mvn.cpp:22
            else
                logc = std::lgamma(0.5 * (d + nu)) - (std::lgamma(0.5 * nu) + det + 0.5 * d * std::log(M_PI * nu));  // mvt.cpp:145
        }
        cst[3 * k] = m->log_weights[k];
        cst[3 * k + 1] = logc;
        cst[3 * k + 2] = nu;
    }
    bcm3hip_ctx* c = new (std::nothrow) bcm3hip_ctx();
    if (!c) return BCM3HIP_ERR_ALLOC;
    int r = ctx_common_init(c, device);
    if (r == 0) r = upload(c, m->means, (size_t)K * d, &c->am.mean);
    if (r == 0) r = upload(c, (const double*)chol.data(), chol.size(), &c->am.chol);
    if (r == 0) r = upload(c, (const double*)cst.data(), cst.size(), &c->am.cst);
    if (r) {
        bcm3hip_close(c);
        return r;
    }
    c->kind = 2;
    c->d = d;
    c->am.kind = bcm3hip::kAnalyticMixtureBase + m->kind;
    c->am.d = d;
    c->am.K = K;
    *out = c;
    return 0;
}

int bcm3hip_open_cellpop_experiments(int device, const bcm3hip_cellpop_model* m, int n_experiments, bcm3hip_ctx** out)
{
    if (!m || !out || n_experiments < 1) return BCM3HIP_ERR_ARG;
    *out = nullptr;
    for (int k = 1; k < n_experiments; k++)
        if (m[k].d != m[0].d) return BCM3HIP_ERR_ARG;  // one parameter vector for every experiment
    bcm3hip_ctx* c = new (std::nothrow) bcm3hip_ctx();
    if (!c) return BCM3HIP_ERR_ALLOC;
    int r = ctx_common_init(c, device);
    if (r == 0) r = bcm3hip::cellpop_create(device, &m[0], &c->cp);
    for (int k = 1; k < n_experiments && r == 0; k++) {
        bcm3hip::CellPopDev* e = nullptr;
        r = bcm3hip::cellpop_create(device, &m[k], &e);
        if (r == 0) c->cp_more.push_back(e);
    }
    if (r) {
        bcm3hip_close(c);
        return r;
    }
    c->kind = 4;
    c->d = m[0].d;
    *out = c;
    return 0;
}

int bcm3hip_open_cellpop(int device, const bcm3hip_cellpop_model* m, bcm3hip_ctx** out)
{
    return bcm3hip_open_cellpop_experiments(device, m, 1, out);
}

int bcm3hip_cellpop_precompile(const bcm3hip_cellpop_model* m) { return bcm3hip::cellpop_precompile(m); }

int bcm3hip_cellpop_cells(bcm3hip_ctx* c, size_t item, int32_t* count, bcm3hip_cell_record* records, double* values,
                          double* end_y)
{
    if (!c || c->kind != 4 || !count) return BCM3HIP_ERR_ARG;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipDeviceSynchronize());
    return bcm3hip::cellpop_cells(c->cp, item, count, records, values, end_y);
}

int bcm3hip_open_expm_pk(int device, const bcm3hip_expm_pk_model* m, bcm3hip_ctx** out)
{
    if (!m || !out) return BCM3HIP_ERR_ARG;
    *out = nullptr;
    const int n = 2 + (m->peripheral ? 1 : 0) + (m->metabolite ? 1 : 0) + (m->n_transit > 0 ? m->n_transit : 0);
    if (m->n_transit < 0 || n > BCM3HIP_EXPM_NMAX || m->d <= 0) return BCM3HIP_ERR_MODEL;
    if (m->n_treat < 1 || m->n_obs < 1 || !(m->MW > 0.0)) return BCM3HIP_ERR_MODEL;
    const bool single = m->param_map == BCM3HIP_PARAM_MAP_SINGLE;
    if (!single && m->param_map != BCM3HIP_PARAM_MAP_POPULATION) return BCM3HIP_ERR_MODEL;
    const int P = m->P;
    if (P < 1 || (single && P != 1)) return BCM3HIP_ERR_MODEL;
    if (P > 1 && (!m->treat_offset || !m->obs_offset)) return BCM3HIP_ERR_MODEL;
    // per-patient ranges: at least one dose and one observation each, observations sorted
    std::vector<int32_t> toff(P + 1), ooff(P + 1);
    for (int j = 0; j <= P; j++) {
        toff[j] = m->treat_offset ? m->treat_offset[j] : (j ? m->n_treat : 0);
        ooff[j] = m->obs_offset ? m->obs_offset[j] : (j ? m->n_obs : 0);
    }
    if (toff[0] != 0 || ooff[0] != 0 || toff[P] != m->n_treat || ooff[P] != m->n_obs) return BCM3HIP_ERR_MODEL;
    for (int j = 0; j < P; j++) {
        if (toff[j + 1] - toff[j] < 1 || ooff[j + 1] - ooff[j] < 1) return BCM3HIP_ERR_MODEL;
        for (int i = ooff[j] + 1; i < ooff[j + 1]; i++)
            if (m->obs_times[i] < m->obs_times[i - 1]) return BCM3HIP_ERR_MODEL;  // PharmacoPatient.cpp:98-100
    }
    std::vector<int32_t> pix(6 * (size_t)P, -1);
    if (!single) {
        if (m->biphasic || m->metabolite) return BCM3HIP_ERR_MODEL;  // not options of the population model
        for (int w = 0; w < 5; w++) {
            if (m->sigma_ix[w] >= m->d) return BCM3HIP_ERR_MODEL;
            if (m->sigma_ix[w] >= 0 && !m->patient_ix) return BCM3HIP_ERR_MODEL;
        }
        if (m->patient_ix) {
            for (size_t k = 0; k < pix.size(); k++) {
                pix[k] = m->patient_ix[k];
                if (pix[k] >= m->d) return BCM3HIP_ERR_MODEL;
            }
            for (int w = 0; w < 5; w++)
                for (int j = 0; j < P && m->sigma_ix[w] >= 0; j++)
                    if (pix[w * P + j] < 0) return BCM3HIP_ERR_MODEL;
        }
    }
    auto bad = [&](int32_t ix, bool required) { return required ? (ix < 0 || ix >= m->d) : (ix >= m->d); };
    if (bad(m->absorption_ix, true) || bad(m->clearance_ix, true) || bad(m->vod_ix, true) ||
        bad(m->excretion_ix, false) || bad(m->additive_sd_ix, false) || bad(m->proportional_sd_ix, false) ||
        bad(m->pf_ix, m->peripheral != 0) || bad(m->pb_ix, m->peripheral != 0) || bad(m->mtt_ix, m->n_transit > 0) ||
        bad(m->direct_ix, m->biphasic != 0) || bad(m->metab_conv_ix, m->metabolite != 0))
        return BCM3HIP_ERR_MODEL;
    if (m->additive_sd_ix < 0 && m->proportional_sd_ix < 0) return BCM3HIP_ERR_MODEL;
    bcm3hip_ctx* c = new (std::nothrow) bcm3hip_ctx();
    if (!c) return BCM3HIP_ERR_ALLOC;
    int r = ctx_common_init(c, device);
    if (r) {
        bcm3hip_close(c);
        return r;
    }
    if (expm_prepare_device() != hipSuccess) {
        bcm3hip_close(c);
        return BCM3HIP_ERR_HIP;
    }
    c->kind = 3;
    c->d = m->d;
    ExpmPKDevModel& x = c->xm;
    x.d = m->d;
    x.n = n;
    x.n_transit = m->n_transit;
    x.peripheral = m->peripheral != 0;
    x.biphasic = m->biphasic != 0;
    x.metabolite = m->metabolite != 0;
    x.additive_sd_ix = m->additive_sd_ix;
    x.proportional_sd_ix = m->proportional_sd_ix;
    x.absorption_ix = m->absorption_ix;
    x.clearance_ix = m->clearance_ix;
    x.vod_ix = m->vod_ix;
    x.excretion_ix = m->excretion_ix;
    x.pf_ix = m->pf_ix;
    x.pb_ix = m->pb_ix;
    x.mtt_ix = m->mtt_ix;
    x.direct_ix = m->direct_ix;
    x.metab_conv_ix = m->metab_conv_ix;
    x.n_treat = m->n_treat;
    x.n_obs = m->n_obs;
    x.MW = m->MW;
    x.param_map = m->param_map;
    x.P = P;
    for (int w = 0; w < 5; w++) x.sigma_ix[w] = single ? -1 : m->sigma_ix[w];
    // the step lengths PharmacokineticModel::Solve (.cpp:127-174) will exponentiate, per patient,
    // by the loop's own arithmetic; equal values share one job
    std::vector<double> job_dt;
    std::vector<int32_t> job_patient, interval_job(m->n_treat, -1), obs_job(m->n_obs, -1);
    for (int j = 0; j < P; j++) {
        const size_t first = job_dt.size();
        auto job = [&](double dt) -> int32_t {
            for (size_t k = first; k < job_dt.size(); k++)
                if (job_dt[k] == dt) return (int32_t)k;
            job_dt.push_back(dt);
            job_patient.push_back(j);
            return (int32_t)(job_dt.size() - 1);
        };
        const double* tt = m->treat_times + toff[j];
        const double* ot = m->obs_times + ooff[j];
        const int nt = toff[j + 1] - toff[j], no = ooff[j + 1] - ooff[j];
        const double until = ot[no - 1];
        int tti = 0, oti = 0;
        double cur = 0.0;
        while (tti < nt && cur < until) {
            const double target = (tti < nt - 1) ? tt[tti + 1] : until;
            while (oti < no && ot[oti] <= target) {
                obs_job[ooff[j] + oti] = job(ot[oti] - cur);
                oti++;
            }
            interval_job[toff[j] + tti] = job(target - cur);
            cur = target;
            tti++;
        }
    }
    x.n_jobs = (int32_t)job_dt.size();
    if ((r = upload(c, job_dt.data(), job_dt.size(), &x.job_dt)) ||
        (r = upload(c, job_patient.data(), job_patient.size(), &x.job_patient)) ||
        (r = upload(c, interval_job.data(), interval_job.size(), &x.interval_job)) ||
        (r = upload(c, obs_job.data(), obs_job.size(), &x.obs_job)) ||
        (r = upload(c, pix.data(), pix.size(), &x.patient_ix)) ||
        (r = upload(c, toff.data(), toff.size(), &x.treat_offset)) ||
        (r = upload(c, ooff.data(), ooff.size(), &x.obs_offset)) ||
        (r = upload(c, m->transforms, (size_t)m->d, &x.transforms)) ||
        (r = upload(c, m->treat_times, (size_t)m->n_treat, &x.treat_times)) ||
        (r = upload(c, m->treat_doses, (size_t)m->n_treat, &x.treat_doses)) ||
        (r = upload(c, m->obs_times, (size_t)m->n_obs, &x.obs_times)) ||
        (r = upload(c, m->obs_conc, (size_t)m->n_obs, &x.obs_conc))) {
        bcm3hip_close(c);
        return r;
    }
    *out = c;
    return 0;
}

int bcm3hip_close(bcm3hip_ctx* c)
{
    if (!c) return 0;
    if (c->stream) hipSetDevice(c->device);
    if (c->cp) bcm3hip::cellpop_destroy(c->cp);
    for (auto* e : c->cp_more) bcm3hip::cellpop_destroy(e);
    hipFree(c->cp_logp);
    hipFree(c->cp_status);
    hipFree(c->cp_status0);
    for (void* p : c->model_allocs) hipFree(p);
    hipFree(c->values);
    hipFree(c->logp);
    hipFree(c->status);
    hipFree(c->pllh);
    hipFree(c->exps);
    hipFree(c->tstatus);
    hipFree(c->traj);
    hipFree(c->stats);
    hipFree(c->place);
    if (c->ev0) hipEventDestroy(c->ev0);
    if (c->ev1) hipEventDestroy(c->ev1);
    if (c->scratch_ev) hipEventDestroy(c->scratch_ev);
    for (hipEvent_t e : c->log_ev) hipEventDestroy(e);
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
    return 0;
}

int bcm3hip_set_option(bcm3hip_ctx* c, int option, int64_t value)
{
    if (!c) return BCM3HIP_ERR_ARG;
    switch (option) {
    case BCM3HIP_OPT_LANES_PER_WAVE:
        if (value < 0 || value > 64) return BCM3HIP_ERR_ARG;
        c->lanes_per_wave = (int)value;
        return 0;
    case BCM3HIP_OPT_BLOCK_WAVES:
        if (value < 1 || value > 4) return BCM3HIP_ERR_ARG;
        c->block_waves = (int)value;
        return 0;
    case BCM3HIP_OPT_TIMING_LOG:
        if (value != 0 && value != 1) return BCM3HIP_ERR_ARG;
        c->log_timing = value != 0;
        c->log_used = 0;
        return 0;
    case BCM3HIP_OPT_UNI_SOLVER:
        if (value != 0 && value != 1) return BCM3HIP_ERR_ARG;
        c->uni_solver = (int)value;
        return 0;
    case BCM3HIP_OPT_BLOCK_LDS:
        if (value < 0 || value > 65536) return BCM3HIP_ERR_ARG;
        c->block_lds = (int)value;
        return 0;
    case BCM3HIP_OPT_PLACEMENT_LOG:
        if (value != 0 && value != 1) return BCM3HIP_ERR_ARG;
        c->place_log = value != 0;
        return 0;
    default: return BCM3HIP_ERR_ARG;
    }
}

int bcm3hip_num_variables(const bcm3hip_ctx* c) { return c ? c->d : -1; }

int64_t bcm3hip_placement_log(bcm3hip_ctx* c, int64_t n_max, uint64_t* host_out)
{
    if (!c || n_max < 0 || (n_max > 0 && !host_out)) return BCM3HIP_ERR_ARG;
    if (!c->place || c->place_n == 0) return 0;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->place_stream));
    const int64_t m = n_max < c->place_n ? n_max : c->place_n;
    if (m > 0) HIPCHK(hipMemcpy(host_out, c->place, (size_t)m * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return m;
}

int bcm3hip_assign_cells(int32_t n_problems, int32_t R, int32_t nsim, const double* lik, int32_t* match, double* sum,
                         int32_t* ok, void* stream)
{
    if (n_problems < 0 || R < 1 || R > 1024 || nsim < 1 || nsim > 65535 || (n_problems > 0 && (!lik || !match || !sum || !ok)))
        return BCM3HIP_ERR_ARG;
    if (n_problems == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const int nw = R > nsim ? R : nsim;
    unsigned char* ws = nullptr;
    size_t stride = 0;
    if (!bcm3hip::cp_assign_lds_fits(nw)) {
        stride = (bcm3hip::cp_assign_ws_bytes(nw) + 255) / 256 * 256;
        HIPCHK(hipMalloc((void**)&ws, stride * n_problems));
    }
    hipError_t e = bcm3hip::launch_cp_assign(n_problems, R, nsim, lik, ws, stride, match, sum, ok, s);
    if (ws) {
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        hipFree(ws);
    }
    HIPCHK(e);
    return 0;
}

static int ensure_traj_scratch(bcm3hip_ctx* c, size_t n)
{
    size_t ntraj = n * (size_t)c->pm.P;
    if (grow(c->pllh, c->cap_traj, ntraj)) return BCM3HIP_ERR_ALLOC;
    if (grow(c->tstatus, c->cap_tstatus, ntraj)) return BCM3HIP_ERR_ALLOC;
    return 0;
}

// Measured on MI355X (profiles/r01_lpw_sweep.txt): one trajectory per wavefront (the UNI
// solver) is fastest up to ~4k trajectories (16 waves per CU); beyond that packing 16+
// trajectories per wavefront (lane solver, ~1k wavefronts in flight) gives the highest rate.
static int auto_lanes_per_wave(size_t ntraj)
{
    if (ntraj <= 4608) return 1;
    int lpw = 16;
    while (lpw < 64 && ntraj > (size_t)lpw * 1024) lpw *= 2;
    return lpw;
}

// scratch of the matrix-exponential path per launch: exps[n][n_jobs][n^2]; larger batches run in
// chunks of evaluations so that it stays under this many bytes
static const size_t kExpmScratchBytes = (size_t)1 << 30;

static int launch(bcm3hip_ctx* c, size_t n, const double* dvalues, double* dlogp, int32_t* dstatus,
                  double* dtraj, bcm3hip_traj_stats* dstats, hipStream_t s, const int32_t* n_dev = nullptr,
                  int32_t* dsteps = nullptr)
{
    if ((n_dev || dsteps) && c->kind != 1) return BCM3HIP_ERR_ARG;  // PopPK launches only
    hipError_t e;
    if (c->scratch_used && c->scratch_stream != s) HIPCHK(hipStreamWaitEvent(s, c->scratch_ev, 0));
    hipEvent_t e0 = c->ev0, e1 = c->ev1;
    if (c->log_timing) {
        if (c->log_ev.size() < 2 * (c->log_used + 1)) {
            for (int k = 0; k < 2; k++) {
                hipEvent_t ev;
                HIPCHK(hipEventCreate(&ev));
                c->log_ev.push_back(ev);
            }
        }
        e0 = c->log_ev[2 * c->log_used];
        e1 = c->log_ev[2 * c->log_used + 1];
        c->log_used++;
    }
    if (c->kind == 1) {
        int r = ensure_traj_scratch(c, n);
        if (r) return r;
        uint64_t* place = nullptr;
        if (c->place_log) {
            if (grow(c->place, c->cap_place, 4 * n * (size_t)c->pm.P)) return BCM3HIP_ERR_ALLOC;
            HIPCHK(hipMemsetAsync(c->place, 0, 4 * n * (size_t)c->pm.P * sizeof(uint64_t), s));
            place = c->place;
            c->place_n = (int64_t)(n * (size_t)c->pm.P);
            c->place_stream = s;
        }
        e = launch_popk(c->pm, (int64_t)n, dvalues, dlogp, dstatus, c->pllh, c->tstatus, dtraj, dstats,
                        c->lanes_per_wave ? c->lanes_per_wave : auto_lanes_per_wave(n * (size_t)c->pm.P),
                        c->block_waves, c->uni_solver, s, e0, e1, c->block_lds, n_dev, dsteps, place);
    } else if (c->kind == 3) {
        const size_t per_eval = (size_t)c->xm.n_jobs * (size_t)(c->xm.n * c->xm.n);
        const size_t chunk = per_eval == 0 ? n : std::max<size_t>(1, kExpmScratchBytes / (per_eval * sizeof(double)));
        const size_t nc = std::min(n, chunk);
        if (grow(c->exps, c->cap_exps, std::max<size_t>(nc * per_eval, 1))) return BCM3HIP_ERR_ALLOC;
        e = hipSuccess;
        for (size_t i0 = 0; i0 < n && e == hipSuccess; i0 += nc) {
            const size_t m = std::min(nc, n - i0);
            e = launch_expm_pk(c->xm, (int64_t)m, dvalues + i0 * (size_t)c->d, dlogp + i0, dstatus ? dstatus + i0 : nullptr,
                               c->exps, s, i0 == 0 ? e0 : nullptr, i0 + m >= n ? e1 : nullptr);
        }
    } else if (c->kind == 4) {
        // experiment 0 into logp, every further one into scratch, summed in experiment order
        int32_t* st = dstatus;
        if (!c->cp_more.empty()) {
            if (!st && grow(c->cp_status0, c->cap_cp_status0, n)) return BCM3HIP_ERR_ALLOC;
            if (!st) st = c->cp_status0;
            if (grow(c->cp_logp, c->cap_cp, n) || grow(c->cp_status, c->cap_cp_status, n)) return BCM3HIP_ERR_ALLOC;
        }
        int r = bcm3hip::cellpop_launch(c->cp, n, dvalues, dlogp, st, s, e0, c->cp_more.empty() ? e1 : nullptr);
        if (r) return r;
        e = hipSuccess;
        for (size_t k = 0; k < c->cp_more.size() && e == hipSuccess; k++) {
            r = bcm3hip::cellpop_launch(c->cp_more[k], n, dvalues, c->cp_logp, c->cp_status, s, nullptr, nullptr);
            if (r) return r;
            e = bcm3hip::launch_cp_accumulate((int32_t)n, dlogp, st, c->cp_logp, c->cp_status, s);
        }
        if (e == hipSuccess && e1 && !c->cp_more.empty()) e = hipEventRecord(e1, s);
    } else {
        e = launch_analytic(c->am, (int64_t)n, dvalues, dlogp, dstatus, s, e0, e1);
    }
    if (e != hipSuccess) {
        fprintf(stderr, "bcm3hip: kernel launch failed: %s\n", hipGetErrorString(e));
        return BCM3HIP_ERR_HIP;
    }
    HIPCHK(hipEventRecord(c->scratch_ev, s));
    c->scratch_stream = s;
    c->scratch_used = true;
    c->last0 = e0;
    c->last1 = e1;
    c->timed = true;
    return 0;
}

int bcm3hip_eval_batch_device(bcm3hip_ctx* c, size_t n, const double* values_dev, double* logp_dev,
                              int32_t* status_dev, void* stream)
{
    if (!c || (n > 0 && (!values_dev || !logp_dev))) return BCM3HIP_ERR_ARG;
    HIPCHK(hipSetDevice(c->device));
    // the caller's stream as given (NULL = the null/default stream, e.g. torch's default stream)
    return launch(c, n, values_dev, logp_dev, status_dev, nullptr, nullptr, (hipStream_t)stream);
}

int bcm3hip_eval_batch_device_counted(bcm3hip_ctx* c, size_t n_max, const int32_t* n_dev, const double* values_dev,
                                      double* logp_dev, int32_t* status_dev, int32_t* steps_dev, void* stream)
{
    if (!c || !n_dev || (n_max > 0 && (!values_dev || !logp_dev))) return BCM3HIP_ERR_ARG;
    if (c->kind != 1) return BCM3HIP_ERR_ARG;
    HIPCHK(hipSetDevice(c->device));
    return launch(c, n_max, values_dev, logp_dev, status_dev, nullptr, nullptr, (hipStream_t)stream, n_dev, steps_dev);
}

int bcm3hip_last_kernel_ms(bcm3hip_ctx* c, float* ms)
{
    if (!c || !ms || !c->timed) return BCM3HIP_ERR_ARG;
    HIPCHK(hipEventSynchronize(c->last1));
    HIPCHK(hipEventElapsedTime(ms, c->last0, c->last1));
    return 0;
}

int bcm3hip_kernel_time_log(bcm3hip_ctx* c, double* total_ms, int64_t* launches, double* max_ms)
{
    if (!c || !total_ms || !launches) return BCM3HIP_ERR_ARG;
    double tot = 0.0, mx = 0.0;
    for (size_t i = 0; i < c->log_used; i++) {
        float ms = 0.0f;
        HIPCHK(hipEventSynchronize(c->log_ev[2 * i + 1]));
        HIPCHK(hipEventElapsedTime(&ms, c->log_ev[2 * i], c->log_ev[2 * i + 1]));
        tot += ms;
        mx = ms > mx ? ms : mx;
    }
    *total_ms = tot;
    *launches = (int64_t)c->log_used;
    if (max_ms) *max_ms = mx;
    c->log_used = 0;
    return 0;
}

int bcm3hip_eval_batch_detail(bcm3hip_ctx* c, size_t n, size_t d, const double* values, double* logp,
                              int32_t* status, double* patient_llh, double* traj, bcm3hip_traj_stats* stats)
{
    if (!c || (int)d != c->d || (n > 0 && (!values || !logp))) return BCM3HIP_ERR_ARG;
    if (n == 0) return 0;
    if ((patient_llh || traj || stats) && c->kind != 1) return BCM3HIP_ERR_ARG;
    HIPCHK(hipSetDevice(c->device));
    if (grow(c->values, c->cap_values, n * d)) return BCM3HIP_ERR_ALLOC;
    if (grow(c->logp, c->cap_n, n)) return BCM3HIP_ERR_ALLOC;
    if (grow(c->status, c->cap_status, n)) return BCM3HIP_ERR_ALLOC;
    size_t ntraj = (c->kind == 1) ? n * (size_t)c->pm.P : 0;
    double* dtraj = nullptr;
    bcm3hip_traj_stats* dstats = nullptr;
    if (traj) {
        if (grow(c->traj, c->cap_trajout, ntraj * (size_t)c->pm.N * (size_t)c->pm.T)) return BCM3HIP_ERR_ALLOC;
        dtraj = c->traj;
    }
    if (stats) {
        if (grow(c->stats, c->cap_stats, ntraj)) return BCM3HIP_ERR_ALLOC;
        dstats = c->stats;
    }
    HIPCHK(hipMemcpyAsync(c->values, values, n * d * sizeof(double), hipMemcpyHostToDevice, c->stream));
    int r = launch(c, n, c->values, c->logp, c->status, dtraj, dstats, c->stream);
    if (r) return r;
    HIPCHK(hipMemcpyAsync(logp, c->logp, n * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (status) HIPCHK(hipMemcpyAsync(status, c->status, n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    if (patient_llh)
        HIPCHK(hipMemcpyAsync(patient_llh, c->pllh, ntraj * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (traj)
        HIPCHK(hipMemcpyAsync(traj, dtraj, ntraj * c->pm.N * c->pm.T * sizeof(double), hipMemcpyDeviceToHost,
                              c->stream));
    if (stats)
        HIPCHK(hipMemcpyAsync(stats, dstats, ntraj * sizeof(bcm3hip_traj_stats), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

int bcm3hip_eval_batch(bcm3hip_ctx* c, size_t n, size_t d, const double* values, double* logp, int32_t* status)
{
    return bcm3hip_eval_batch_detail(c, n, d, values, logp, status, nullptr, nullptr, nullptr);
}

}  // extern "C"
