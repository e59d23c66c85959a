/*
 * bcm3.h -- C-ABI of the host library libbcm3.so: the bcm3::Likelihood / LikelihoodFactory
 * plugin surface of the reference (src/sampler/Likelihood.h:9-35,
 * src/likelihoods/LikelihoodFactory.cpp:31-100, wired as in src/bcminf/main.cpp:47-121) built
 * from the reference's own input files (prior.xml, likelihood.xml), backed by libbcm3hip.so.
 *
 * Replaces, for a caller that cannot link C++ (Python/ctypes, R .C(), Go cgo ...):
 *   VariableSet::LoadFromXML (src/sampler/VariableSet.cpp:16-69)
 *   LikelihoodFactory::CreateLikelihood + Likelihood::Initialize/PostInitialize
 *   Likelihood::EvaluateLogProbability (single vector) and the batched fan-out of
 *   SamplerPT::DoMutateMove (src/sampler/SamplerPT.cpp:308-319).
 * Return codes: 0 ok, < 0 error (message in bcm3_last_error()). EvaluateLogProbability's
 * "return false" maps to a negative return; logp = -inf is a legal result.
 */
#ifndef BCM3_H
#define BCM3_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bcm3_likelihood bcm3_likelihood;

/* Load prior.xml (variable set) + likelihood.xml, create and initialise the likelihood on HIP
 * device `device` (-1: $BCM3_DEVICE or 0). */
int bcm3_likelihood_create(const char* likelihood_xml, const char* prior_xml, int device, bcm3_likelihood** out);
/* Same with options "key=value;key=value" (config.txt keys; "device=N", "backend=none" to
 * initialise without a device -- evaluation then fails; used to test the host logic on CPU). */
int bcm3_likelihood_create_ex(const char* likelihood_xml, const char* prior_xml, const char* options,
                              bcm3_likelihood** out);
/* The flat PopPK model derived by LikelihoodPopPKTrajectory::Initialize (type
 * pop_pk_trajectory only). Pointers stay valid while the likelihood lives. `model` points to a
 * bcm3hip_popk_model (bcm3hip.h). */
int bcm3_likelihood_popk_model(const bcm3_likelihood* ll, void* model);
/* The flat matrix-exponential PK model a pharmaco_single likelihood hands to the device: the
 * treatment schedule and filtered observations of PharmacoPatient::Load
 * (src/pharmaco/PharmacoPatient.cpp:8-116) and the variable indices of
 * PharmacoLikelihoodSingle::PostInitialize (.cpp:78-147), into a bcm3hip_expm_pk_model. Returns
 * -2 for other likelihood types. */
int bcm3_likelihood_expm_pk_model(const bcm3_likelihood* ll, void* model);
/* cell_population: the generated_derivative body (SBMLModel::GenerateCode, src/sbml/SBMLModel.cpp:
 * 291-367) this likelihood compiled; returns its length (buf may be NULL), < 0 for other types */
int bcm3_likelihood_generated_code(const bcm3_likelihood* ll, char* buf, size_t buflen);
/* VariabilityPseudoRandomIterator's sequence (boost::random::sobol through uniform_01, restated):
 * points x dims, row-major */
int bcm3_sobol_points(size_t points, size_t dims, double* out);
/* cell_population: compile the cell kernel into the code-object cache without a device (build time;
 * create the likelihood with options "backend=none") */
int bcm3_likelihood_cellpop_precompile(const bcm3_likelihood* ll);
/* cell_population: the cells of item `item` of the last batch (bcm3hip_cellpop_cells) */
int bcm3_likelihood_cellpop_cells(bcm3_likelihood* ll, size_t item, int32_t* count, void* records /*bcm3hip_cell_record*/,
                                  double* values, double* end_y);
void bcm3_likelihood_destroy(bcm3_likelihood* ll);
int bcm3_likelihood_num_variables(const bcm3_likelihood* ll);
/* PriorIndependence::LoadFromXML (src/sampler/PriorIndependence.cpp:20-115) as the device sampler
 * holds it: per variable the BCM3HIP_PRIOR_* kind, (p0, p1, p2), (lower, upper) bounds and the
 * marginal (mean, variance) (Dirichlet groups: MultivariateMarginal.cpp:47-180). Fills up to
 * max_vars entries (any array may be NULL); returns the number of variables or < 0. */
int bcm3_prior_marginals(const char* prior_xml, int max_vars, int32_t* kind, double* params, double* bounds,
                         double* moments);
/* name of variable i (prior.xml order, repeat-expanded); returns the name length or < 0 */
int bcm3_likelihood_variable_name(const bcm3_likelihood* ll, int i, char* buf, size_t buflen);
/* VariableSet::TransformVariable code of variable i (0 none, 1 log, 2 log10, 3 logit) */
int bcm3_likelihood_variable_transform(const bcm3_likelihood* ll, int i);
int bcm3_likelihood_set_learning_rate(bcm3_likelihood* ll, double learning_rate);

/* EvaluateLogProbability(threadix, values[d], logp) */
int bcm3_likelihood_evaluate(bcm3_likelihood* ll, size_t threadix, const double* values, double* logp);
/* batched: values[n*d] row-major host buffers; status may be NULL */
int bcm3_likelihood_evaluate_batch(bcm3_likelihood* ll, size_t n, const double* values, double* logp,
                                   int32_t* status);
/* batched on device buffers, asynchronous on `stream` (hipStream_t; NULL = null stream) */
int bcm3_likelihood_evaluate_batch_device(bcm3_likelihood* ll, size_t n, const double* values_dev,
                                          double* logp_dev, int32_t* status_dev, void* stream);
/* duration of the last kernel launch in ms (HIP events on the launch stream) */
int bcm3_likelihood_last_kernel_ms(bcm3_likelihood* ll, float* ms);
/* kernel time log (enable with option BCM3HIP_OPT_TIMING_LOG): summed / max kernel ms and the
 * number of launches since the previous call; synchronises on the logged launches */
int bcm3_likelihood_kernel_time_log(bcm3_likelihood* ll, double* total_ms, int64_t* launches, double* max_ms);
/* backend option (BCM3HIP_OPT_* of bcm3hip.h) */
int bcm3_likelihood_set_option(bcm3_likelihood* ll, int option, int64_t value);

const char* bcm3_last_error(void);
/* A data or output file as the likelihoods' loaders see it (NetCDFDataFile::Open's role): netCDF
 * classic, netCDF-4 through a run-time loaded libnetcdf, or the JSON sidecar, as JSON text
 * {"<group>": {"<variable>": {"dims": [...], "data": nested arrays}}} (fill values -> null).
 * Writes at most cap bytes (NUL-terminated) and returns the full length, < 0 on error. */
int64_t bcm3_data_file_json(const char* filename, char* out, int64_t cap);

/* ---- proposal adaptation (host C++, GMM.cpp) ----
 * SamplerPTChain::AdaptProposal (src/sampler/SamplerPTChain.cpp:120-178) for the C chains of a rank:
 * Proposal::Initialize's history thinning to max_history_samples (Proposal.cpp:92-121), then
 *   BCM3_PROPOSAL_GAUSSIAN_MIXTURE: ProposalGaussianMixture::InitializeImpl
 *     (ProposalGaussianMixture.cpp:125-254): ESS from autocorrelations, GMM::Fit for 1, 2, 3, 4, 5,
 *     8, 13 components (k-means++ + EM, src/stats/GMM.cpp:48-158), lowest AIC (adjusted_aic != 0:
 *     the gaussian_mixture_adjustedAIC selection), else the prior's moments;
 *   BCM3_PROPOSAL_GLOBAL_COVARIANCE: ProposalGlobalCovariance::InitializeImpl (:64-104).
 * history[C][H][d] float rings with counts[C] samples stored (bcm3hip_history_add); active[C]
 * (may be NULL) selects the chains to adapt (T != 0). Outputs per chain, sized for kmax
 * components (kmax >= 13 for every candidate of the mixture fit): ncomp[C], weights[C][kmax],
 * means[C][kmax][d], chol[C][kmax][d][d] (lower Cholesky factors, row-major; identity for unused
 * slots), logc[C][kmax], fitted[C] (may be NULL; 0 = prior fallback). Random numbers: counter
 * based, keyed by (seed, adaptation, chain0 + c). nthreads host threads. */
enum { BCM3_PROPOSAL_GLOBAL_COVARIANCE = 0, BCM3_PROPOSAL_GAUSSIAN_MIXTURE = 1 };
int bcm3_adapt_proposals(int kind, int adjusted_aic, int C, int H, int d, int kmax, const float* history,
                         const int64_t* counts, const uint8_t* active, size_t max_history_samples,
                         const double* prior_mean, const double* prior_var, uint64_t seed, uint64_t adaptation,
                         int64_t chain0, int nthreads, int32_t* ncomp, double* weights, double* means, double* chol,
                         double* logc, int32_t* fitted);
/* GMM::Set + LogPdf + CalculateResponsibilities (src/stats/GMM.cpp:14-45, 160-186) of K components
 * (covariances[K][d][d]) at n points x[n][d]: logpdf[n], resp[n][K], and the Cholesky factors /
 * log normalisers the device proposal state holds (chol_out[K][d][d], logc_out[K]); any output
 * may be NULL. */
int bcm3_gmm_eval(int K, int d, const double* weights, const double* means, const double* covariances, int n,
                  const double* x, double* logpdf, double* resp, double* chol_out, double* logc_out);

/* ---- the PT-MH sampler loop of one rank, in C++ (SamplerPTDevice.cpp) ----
 * SamplerPT::Initialize / Run (src/sampler/SamplerPT.cpp:97-260) with SamplerPTChain's
 * MutateMove / ExchangeMove / AdaptProposal (src/sampler/SamplerPTChain.cpp:120-381): the rank owns
 * the contiguous ladder slice [rank * C, (rank + 1) * C) of num_chains = world * C chains, chain
 * state in HBM, one batched likelihood launch per mutate step on `stream`, proposal adaptation on
 * host threads (bcm3_adapt_proposals), the PT swap of slice-boundary pairs over RCCL. Random
 * numbers are counter based, so a run is identical for any number of ranks (and to
 * bcm3_amd.sampler.PTMHDevice). Not thread-safe per handle. */
enum { BCM3_PTMH_GLOBAL_COVARIANCE = 0, BCM3_PTMH_GAUSSIAN_MIXTURE = 1, BCM3_PTMH_GAUSSIAN_MIXTURE_ADJUSTED_AIC = 2,
       BCM3_PTMH_RANDOM_WALK = 3 };
enum { BCM3_PTMH_DETERMINISTIC_EVEN_ODD = 0, BCM3_PTMH_STOCHASTIC_EVEN_ODD = 1, BCM3_PTMH_STOCHASTIC_RANDOM = 2 };
enum { BCM3_PTMH_TRANSPORT_NONE = 0, BCM3_PTMH_TRANSPORT_RCCL = 1, BCM3_PTMH_TRANSPORT_LOCAL = 2,
       BCM3_PTMH_TRANSPORT_SOCKET = 3 };
typedef struct bcm3_ptmh bcm3_ptmh;
typedef struct bcm3_ptmh_group bcm3_ptmh_group; /* in-process ranks (tests): host-staged transport */
typedef struct {
    int64_t num_chains;          /* ptmhsampler.num_chains, over all ranks */
    int32_t rank, world;
    double temperature_power;    /* ptmhsampler.temperature_schedule_power (3) */
    double temperature_max;      /* 1 */
    uint64_t seed;               /* sampler.rngseed */
    double learning_rate;
    int32_t exploration_steps;   /* ptmhsampler.num_exploration_steps */
    int32_t proposal;            /* BCM3_PTMH_* proposal type */
    double t_dof;                /* ptmhsampler.proposal_t_dof */
    int32_t kmax;                /* mixture component slots, 0 = 13 */
    int32_t adapt_proposal_samples, adapt_proposal_times, max_history_size;
    int32_t adapt_proposal_max_history_samples, use_every_nth;
    int32_t swapping_scheme;     /* BCM3_PTMH_*_EVEN_ODD / _RANDOM */
    double exchange_probability;
    int32_t initial_position_tries;
    int32_t nan_check_every;     /* bcm3_ptmh_run checks for NaN likelihoods every n iterations */
    int32_t host_threads;        /* proposal adaptation threads, 0 = all cores (max 16) */
    int32_t speculate;           /* 1 (default): pairs of iterations in one likelihood launch when the
                                    likelihood supports it (SamplerPTDevice, bcm3hip_ptmh_spec_*);
                                    bit-identical to 0, the one-launch-per-iteration loop */
    int32_t transport;           /* BCM3_PTMH_TRANSPORT_*, world > 1 */
    uint8_t nccl_id[128];        /* BCM3_PTMH_TRANSPORT_RCCL: bcm3_ptmh_nccl_unique_id of rank 0 */
    bcm3_ptmh_group* group;      /* BCM3_PTMH_TRANSPORT_LOCAL */
    char socket_dir[256];        /* BCM3_PTMH_TRANSPORT_SOCKET: a directory every rank's process can
                                    reach; rank r listens on <socket_dir>/bcm3_rank<r>.sock (ranks in
                                    separate processes on one host, e.g. sharing one GPU) */
} bcm3_ptmh_config;
enum { BCM3_PTMH_NUM_COUNTERS = 10 }; /* attempted / accepted mutate, attempted / accepted exchange,
                                         samples done, adaptations done, iterations, exchange rounds,
                                         likelihood launches, trajectories they evaluated (speculative
                                         candidates included) */
void bcm3_ptmh_config_default(bcm3_ptmh_config* cfg);
int bcm3_ptmh_nccl_unique_id(void* id /* 128 bytes */);
int bcm3_ptmh_group_create(int world, bcm3_ptmh_group** out);
void bcm3_ptmh_group_destroy(bcm3_ptmh_group* g);
/* prior_xml: the prior.xml the likelihood was created with (PriorIndependence marginals);
 * stream: hipStream_t, NULL = a stream of its own. Finds the starting positions
 * (SamplerPTChain::FindStartingPosition). */
int bcm3_ptmh_create(bcm3_likelihood* ll, const char* prior_xml, const bcm3_ptmh_config* cfg, void* stream,
                     bcm3_ptmh** out);
/* n iterations of SamplerPT::Run's loop (exchange + mutate moves, adaptation when due), no host
 * synchronisation except at adaptations; last_at_end marks the final iteration as the last sample */
int bcm3_ptmh_iterate(bcm3_ptmh* s, int64_t n, int last_at_end);
/* num_samples * use_every_nth iterations with the NaN check every nan_check_every (fatal, as
 * Sampler::EvaluateLikelihood, src/sampler/Sampler.cpp:172-178) */
int bcm3_ptmh_run(bcm3_ptmh* s, int64_t num_samples);
int bcm3_ptmh_adapt(bcm3_ptmh* s);
/* diagnostics of the speculative iteration pairs (bcm3_ptmh_config.speculate): the last pair's
 * likelihood launch in dispatch order -- entry sources (c < C: chain c's proposal; C + 6c + k:
 * candidate k of chain c, bcm3hip_spec) and BDF steps (src / steps: [7 C], may be NULL); returns the
 * entry count, -1 when the sampler does not speculate */
int64_t bcm3_ptmh_spec_batch_info(bcm3_ptmh* s, int32_t* src, int32_t* steps);
/* wait for the stream; < 0 if a likelihood returned NaN */
int bcm3_ptmh_synchronize(bcm3_ptmh* s);
int bcm3_ptmh_num_chains(const bcm3_ptmh* s); /* chains of this rank */
/* host copies of the rank's chains (any may be NULL): values[C][d], llh[C], lprior[C], lpp[C] */
int bcm3_ptmh_get_state(bcm3_ptmh* s, double* values, double* llh, double* lprior, double* lpp);
int bcm3_ptmh_get_components(bcm3_ptmh* s, int32_t* ncomp /* [C] */);
int bcm3_ptmh_get_counters(bcm3_ptmh* s, int64_t* out /* [BCM3_PTMH_NUM_COUNTERS] */);
void* bcm3_ptmh_stream(const bcm3_ptmh* s);
void bcm3_ptmh_destroy(bcm3_ptmh* s);
/* SampleHandlerNetCDF for the rank (SampleHandlerNetCDF.cpp:24-110, SamplerPT::EmitSample
 * SamplerPT.cpp:321-330): every use_every_nth-th iteration the rank's chains (values, log prior,
 * log likelihood, weight 1) go to `filename` (bcm3_samples_* format below; the ranks of a sharded
 * ladder share one file), staged on the device and written every flush_every samples, at the end of
 * bcm3_ptmh_run and on bcm3_ptmh_flush_output / destroy. Call before the first iteration. */
int bcm3_ptmh_set_output(bcm3_ptmh* s, const char* filename, int64_t num_samples, int32_t flush_every);
int bcm3_ptmh_flush_output(bcm3_ptmh* s);
/* ptmhsampler.output_proposal_adaptation (SamplerPTChain.cpp:149-166): after every adaptation the
 * highest-temperature chain's proposal (group adapt<k>/block1: variable_indices, gmm_weights,
 * cluster<i>_mean / cluster<i>_covariance or covariance, and the fitted history from the second
 * adaptation on) is (re)written to `filename` in the NetCDFBundler layout, netCDF classic
 * (nested groups named "adapt<k>.block1.<name>"); written by the rank holding that chain. */
int bcm3_ptmh_set_adaptation_output(bcm3_ptmh* s, const char* filename);

/* ---- config.txt (bcminf's configuration file) ----
 * boost::program_options::parse_config_file over the options bcminf registers
 * (src/bcminf/main.cpp:293-320; Sampler.cpp:142-149; SamplerPT.cpp:147-171;
 * LikelihoodFactory.cpp:103-111), read as Sampler::LoadSettings / SamplerPT::LoadSettings do
 * (SamplerPT.cpp:40-95): "[section]" lines prefix "section.", '#' comments, the registered
 * defaults for every key the file omits; an unknown or repeated key, a value of the wrong type, an
 * unknown swapping scheme or proposal type (e.g. "parametric_mixture": SamplerPTChain.cpp:428-444)
 * fail (< 0, message in bcm3_last_error). sampler.rngseed = 0 becomes a time-based seed
 * (Sampler.cpp:91-94). rank / world / transport are left at their defaults. */
typedef struct {
    bcm3_ptmh_config ptmh;
    int64_t num_samples;                /* sampler.num_samples (2500): bcm3_ptmh_run's argument */
    int32_t output_proposal_adaptation; /* ptmhsampler.output_proposal_adaptation */
    int32_t pad_;
    int64_t sampling_threads, evaluation_threads;
    char sampler_type[64];
    char prior[1024], likelihood[1024], output_folder[1024];
    char likelihood_options[2048];      /* "key=value;..." for bcm3_likelihood_create_ex */
} bcm3_run_config;
int bcm3_run_config_from_file(const char* path, bcm3_run_config* out);
/* the sampler part of the same file (bcm3_ptmh_config_default, then the file's settings) */
int bcm3_ptmh_config_from_file(const char* path, bcm3_ptmh_config* cfg);

/* ---- netCDF classic files (NetCDFClassic.h): the sampler's output.nc ----
 * The reference's output.nc schema (group "samples", SampleHandlerNetCDF.cpp:41-58) in a netCDF
 * classic (CDF-2) file, group members named "samples.<name>": dims sample_ix, temperature,
 * variable; variables sample_ix, variable (names), temperature, variable_transform,
 * variable_values[sample_ix][temperature][variable], log_prior / log_likelihood / weights
 * [sample_ix][temperature], NC_FILL_DOUBLE where no sample was written. A process writes the
 * temperature columns [first, first + own) (all processes of a sharded ladder open the same file);
 * the process with first == 0 writes the coordinate variables. tools/nc_convert.py makes the
 * netCDF-4 group file the reference's R tooling (R/load.r) opens. */
typedef struct bcm3_samples bcm3_samples;
int bcm3_samples_open(const char* filename, int64_t num_samples, int32_t d, const char* const* names,
                      const int32_t* transforms, int32_t num_temperatures, const double* temperatures, int32_t first,
                      int32_t own, bcm3_samples** out);
/* sample sample_ix of temperatures [first + t0, first + t0 + nt): values[nt][d], lprior / llh /
 * weight [nt] */
int bcm3_samples_write(bcm3_samples* h, int64_t sample_ix, int32_t t0, int32_t nt, const double* values,
                       const double* lprior, const double* llh, const double* weight);
int bcm3_samples_sync(bcm3_samples* h);
void bcm3_samples_close(bcm3_samples* h);

#ifdef __cplusplus
}
#endif
#endif
