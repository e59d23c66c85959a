/*
 * bcm3hip.h -- C-ABI of the MI355X likelihood-evaluation library (libbcm3hip.so).
 *
 * This is the drop-in boundary for BCM3's per-chain likelihood fan-out. It replaces, for the
 * batched GPU path:
 *   - the per-chain task fan-out SamplerPT::DoMutateMove -> TaskManager::AddTask ->
 *     SamplerPTChain::MutateMove -> Sampler::EvaluateLikelihood ->
 *     bcm3::Likelihood::EvaluateLogProbability
 *     (src/sampler/SamplerPT.cpp:308-319, src/utils/TaskManager.cpp:36-116,
 *      src/sampler/Sampler.cpp:164-180, src/sampler/Likelihood.h:29);
 *   - LikelihoodPopPKTrajectory::EvaluateLogProbability and its CVODE solve
 *     (src/likelihoods/LikelihoodPopPKTrajectory.cpp:259-718,
 *      src/odecommon/ODESolverCVODE.cpp:322-463, dependencies/cvode-5.3.0/src/cvode/cvode.c);
 *   - TestLikelihoodBanana / TestLikelihoodCircular::EvaluateLogProbability
 *     (src/likelihoods/TestLikelihoodBanana.cpp:42-55, TestLikelihoodCircular.cpp:42-53).
 * The reference's own C-ABI plugin (LikelihoodDLL: initialize_likelihood /
 * evaluate_log_probability, src/likelihoods/LikelihoodDLL.cpp:34-116) is single-vector; its
 * replacement symbols live in bcm3_dll.h on top of this header.
 *
 * Plain C types only; no torch / HIP types in signatures. Streams are passed as void*.
 * Return codes: 0 = success, < 0 = fatal error (see bcm3hip_error_string). A fatal error maps
 * to EvaluateLogProbability returning false in the host layer. Per-item model failures
 * (solver failure / max_steps) are NOT errors: logp = -inf and status = 1, exactly as the
 * reference (LikelihoodPopPKTrajectory.cpp:400-408).
 * Threading: a context is not thread-safe; use one context per host thread / GPU.
 * Determinism: logp[i] depends only on values[i] and the model (no batch coupling).
 */
#ifndef BCM3HIP_H
#define BCM3HIP_H

#if !defined(__HIPCC_RTC__)  /* (the run-time compiled cell kernel: hipRTC defines these types itself) */
#include <stddef.h>
#include <stdint.h>
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define BCM3HIP_OK 0
#define BCM3HIP_ERR_ARG (-1)
#define BCM3HIP_ERR_HIP (-2)
#define BCM3HIP_ERR_NODEVICE (-3)
#define BCM3HIP_ERR_MODEL (-4)
#define BCM3HIP_ERR_ALLOC (-5)

/* per-item status */
#define BCM3HIP_STATUS_OK 0
#define BCM3HIP_STATUS_SOLVER_FAIL 1 /* CVODE error or max_steps: logp = -inf */

/* PKModelType after the reference's string mapping (LikelihoodPopPKTrajectory.h:28-36,
 * .cpp:69-83; "one_biphasic_uptake" maps to TWO_BIPHASIC there). */
enum {
    BCM3HIP_PK_ONE = 0,
    BCM3HIP_PK_TWO = 1,
    BCM3HIP_PK_ONE_BIPHASIC = 2,
    BCM3HIP_PK_TWO_BIPHASIC = 3,
    BCM3HIP_PK_ONE_TRANSIT = 4,
    BCM3HIP_PK_TWO_TRANSIT = 5
};

/* VariableSet::TransformVariable codes (src/sampler/VariableSet.cpp:97-124). */
enum { BCM3HIP_TF_NONE = 0, BCM3HIP_TF_LOG = 1, BCM3HIP_TF_LOG10 = 2, BCM3HIP_TF_LOGIT = 3 };

/* Parameter maps (values -> PK rate constants) of the two CVODE PK likelihoods:
 * POPULATION = LikelihoodPopPKTrajectory::EvaluateLogProbability (.cpp:263-310): non-centred random
 *   effects per patient, NaN concentrations give -inf;
 * SINGLE = LikelihoodPharmacokineticTrajectory::EvaluateLogProbability
 *   (src/likelihoods/LikelihoodPharmacokineticTrajectory.cpp:215-262): the rates are the
 *   (transformed) variables themselves, biphasic time / absorption at variables 6 / 7, P = 1. */
enum { BCM3HIP_PARAM_MAP_POPULATION = 0, BCM3HIP_PARAM_MAP_SINGLE = 1 };

/* Flat PopPK model: everything LikelihoodPopPKTrajectory::Initialize derives from
 * likelihood.xml + prior.xml + the pkdata file (.cpp:50-252). Host pointers; the arrays are
 * copied to device memory by bcm3hip_open_popk and need not outlive the call. */
typedef struct {
    int32_t pk_type;           /* BCM3HIP_PK_* */
    int32_t N;                 /* ODE states: 2 or 3 */
    int32_t num_pk_params;     /* .cpp:99-120 */
    int32_t num_pk_pop_params; /* 2 */
    int32_t d;                 /* number of sampled variables */
    int32_t P;                 /* patients */
    int32_t T;                 /* time points */
    int32_t sd_ix;             /* index of "standard_deviation" */
    int32_t n_transit_ix;      /* "n_transit" or -1 */
    int32_t transit_time_ix;   /* "mean_transit_time" or -1 */
    int32_t biphasic_time_ix;  /* "biphasic_uptake_time" or -1 */
    int32_t absorption2_ix;    /* "mean_absorption2" or -1 */
    int32_t max_steps;         /* 2000 (ODESolverCVODE.cpp:45) */
    int32_t param_map;         /* BCM3HIP_PARAM_MAP_*: which likelihood's parameter map */
    double rtol;               /* (double)1e-6f */
    double atol;               /* min dose * (double)1e-6f */
    double MW;                 /* molecular weight of the drug */
    double fixed_vod;          /* NaN if sampled */
    double fixed_kf;           /* NaN if sampled */
    double fixed_kb;           /* NaN if sampled */
    const int32_t* transforms; /* [d] BCM3HIP_TF_* */
    const double* time;        /* [T] */
    const double* observed;    /* [P*T], NaN = unobserved */
    const double* dose;        /* [P] */
    const double* dosing_interval;        /* [P] */
    const double* dose_after_dose_change; /* [P] (NaN = none) */
    const double* dose_change_time;       /* [P] (NaN = none) */
    const int32_t* intermittent;          /* [P] 0..3 */
    const uint8_t* skipped_days;          /* [P*29] treatment_interruptions flags */
    const int32_t* simulate_until;        /* [P] number of time points simulated */
} bcm3hip_popk_model;

/* BANANA TestLikelihoodBanana, CIRCULAR TestLikelihoodCircular, DUMMY LikelihoodDummy
 * (src/likelihoods/LikelihoodDummy.cpp:18-32: LogPdfTnu4(values[0], 0, 1)) */
enum { BCM3HIP_ANALYTIC_BANANA = 1, BCM3HIP_ANALYTIC_CIRCULAR = 2, BCM3HIP_ANALYTIC_DUMMY = 3 };
typedef struct {
    int32_t kind; /* BCM3HIP_ANALYTIC_* */
    int32_t d;    /* dimension */
    double p0;    /* banana: sd1 ; circular: radius */
    double p1;    /* banana: sd2 ; circular: offset */
    double p2;    /* circular: width */
} bcm3hip_analytic_model;

/* Mixture test likelihoods: logp = logsum_k (log w_k + log density_k(values)), summed with
 * bcm3::logsum in component order from -inf.
 *   NORMAL  TestLikelihoodMultimodalGaussians (TestLikelihoodMultimodalGaussians.cpp:36-42), each
 *           component bcm3::dmvnormal (src/stats/mvn.cpp:9-33)
 *   T       TestLikelihoodTruncatedT (TestLikelihoodTruncatedT.cpp:81-90), each component
 *           bcm3::dmvt (src/stats/mvt.cpp:119-157; d = 1 goes through LogPdfT with the 1x1
 *           "covariance" as the scale, ProbabilityDistributions.cpp:159-180, as the reference does)
 * The Cholesky factors and log normalising constants are computed once at open time
 * (Eigen::LLT reads the lower triangle of each covariance). */
enum { BCM3HIP_MIXTURE_NORMAL = 1, BCM3HIP_MIXTURE_T = 2 };
#define BCM3HIP_MIXTURE_DMAX 16
#define BCM3HIP_MIXTURE_KMAX 64
typedef struct {
    int32_t kind;               /* BCM3HIP_MIXTURE_* */
    int32_t d;                  /* dimension, 1..BCM3HIP_MIXTURE_DMAX */
    int32_t K;                  /* components, 1..BCM3HIP_MIXTURE_KMAX */
    const double* log_weights;  /* [K] log of each component's weight, added as given */
    const double* means;        /* [K][d] */
    const double* covariances;  /* [K][d][d] row-major; the lower triangle is used */
    const double* nus;          /* [K] degrees of freedom (T), > 0; NULL for NORMAL */
} bcm3hip_mixture_model;

/* Linear-compartment PK model solved by matrix exponentials: the pharmaco_single likelihood
 * (src/pharmaco/PharmacoLikelihoodSingle.cpp:149-218) over PharmacokineticModel::Solve /
 * ConstructMatrix (src/pharmaco/PharmacokineticModel.cpp:111-247) with Eigen's
 * MatrixBase::exp (Pade 3..13 + scaling and squaring, unsupported/Eigen/src/MatrixFunctions/
 * MatrixExponential.h:65-366). Compartments: 2 (+1 peripheral) (+1 metabolite) (+n_transit),
 * at most BCM3HIP_EXPM_NMAX. Treatment and observation arrays are what Patient::Load derives
 * (src/pharmaco/PharmacoPatient.cpp:8-116): doses at treat_times, observations with NaN
 * concentrations removed, sorted times. Variable indices are -1 when the variable is absent. */
enum { BCM3HIP_EXPM_NMAX = 16 };
typedef struct {
    int32_t d;                  /* number of sampled variables */
    int32_t n_transit;          /* num_transit_compartments, 0 = none */
    int32_t peripheral;         /* 0/1 */
    int32_t biphasic;           /* 0/1: direct_absorption */
    int32_t metabolite;         /* 0/1 (metabolite elimination fixed at 1.0) */
    int32_t additive_sd_ix;     /* additive_error_standard_deviation or -1 (sd 0) */
    int32_t proportional_sd_ix; /* proportional_error_standard_deviation or -1 (sd 0) */
    int32_t absorption_ix, clearance_ix, vod_ix; /* required */
    int32_t excretion_ix;       /* -1: excretion 0 */
    int32_t pf_ix, pb_ix;       /* peripheral_forward_rate / peripheral_backward_rate */
    int32_t mtt_ix;             /* mean_transit_time */
    int32_t direct_ix;          /* direct_absorption */
    int32_t metab_conv_ix;      /* metabolite_conversion_rate */
    int32_t n_treat;            /* >= 1 */
    int32_t n_obs;              /* >= 1 */
    double MW;                  /* molecular weight of the drug */
    const int32_t* transforms;  /* [d] BCM3HIP_TF_* */
    const double* treat_times;  /* [n_treat] ascending */
    const double* treat_doses;  /* [n_treat] */
    const double* obs_times;    /* [n_obs] ascending */
    const double* obs_conc;     /* [n_obs] */
    /* pharmaco_population (src/pharmaco/PharmacoLikelihoodPopulation.cpp:202-340). With param_map
     * POPULATION, absorption_ix / clearance_ix / vod_ix / excretion_ix / mtt_ix name the mean_*
     * variables, each patient's rate is fastpow10(QuantileNormal(p<i>_<rate>, mean, sigma)) when
     * sigma_ix[] of that rate is >= 0 (else fastpow10(mean); transit time: TransformVariable), and
     * the P per-patient log-likelihoods are summed in patient order. For pharmaco_single: param_map
     * SINGLE, P = 1, offsets may be NULL. */
    int32_t param_map;          /* BCM3HIP_PARAM_MAP_SINGLE or BCM3HIP_PARAM_MAP_POPULATION */
    int32_t P;                  /* patients (1 for single) */
    int32_t sigma_ix[5];        /* sigma_absorption, _excretion, _clearance, _volume_of_distribution,
                                   _transit_time; -1 = no random effect */
    const int32_t* patient_ix;  /* [6][P]: p<i>_absorption, _excretion, _clearance,
                                   _volume_of_distribution, _transit_time, _bioavailability; -1 = absent */
    const int32_t* treat_offset; /* [P+1]: patient j's doses are treat_*[treat_offset[j], treat_offset[j+1]) */
    const int32_t* obs_offset;   /* [P+1]: likewise for obs_* */
} bcm3hip_expm_pk_model;

/* ---- cell-population likelihood (type "cell_population", src/cellpop) ----------------------
 * One Experiment of CellPopulationLikelihood (src/cellpop/CellPopulationLikelihood.cpp:82-101,
 * Experiment.cpp:239-372, 635-782): heterogeneous cells of an SBML model integrated with CVODE
 * BDF, dividing cells spawning two daughters, a population-average time-course data likelihood.
 * The host layer (libbcm3.so, LikelihoodCellPopulation) derives everything below from
 * likelihood.xml + prior.xml + the SBML file + the data file. */
typedef struct {
    int32_t kind; /* BCM3HIP_REF_VARIABLE: transformed variable `index`; BCM3HIP_REF_FIXED: `value`;
                     BCM3HIP_REF_NONE: absent (offset 0, scale 1) */
    int32_t index;
    double value;
} bcm3hip_value_ref;
enum { BCM3HIP_REF_NONE = 0, BCM3HIP_REF_VARIABLE = 1, BCM3HIP_REF_FIXED = 2 };

/* VariabilityDescriptionVariable::Apply types (VariabilityDescriptionVariable.cpp) */
enum {
    BCM3HIP_APPLY_ADDITIVE = 0, BCM3HIP_APPLY_ADDITIVE_LOG = 1, BCM3HIP_APPLY_ADDITIVE_LOG2 = 2,
    BCM3HIP_APPLY_MULTIPLICATIVE = 3, BCM3HIP_APPLY_MULTIPLICATIVE_LOG = 4, BCM3HIP_APPLY_MULTIPLICATIVE_LOG2 = 5,
    BCM3HIP_APPLY_REPLACE = 6
};
/* One application of a variability dimension in Cell::Initialize order (Cell.cpp:162-176):
 * description by description, the sampled variables in order, then the ODE species in order. */
typedef struct {
    int32_t dim;          /* Sobol / pseudorandom-vector dimension */
    int32_t target_kind;  /* 0 = sampled variable (cell parameter), 1 = ODE species initial condition */
    int32_t target_index;
    int32_t apply;        /* BCM3HIP_APPLY_* */
    int32_t negate;
    int32_t only_initial_cells;
} bcm3hip_variability_action;

/* A data likelihood: DataLikelihoodTimeCoursePopulationAverage (kind 0) or DataLikelihoodTimeCourse
 * (kind 1, one species, no observed lineage, no synchronisation), or DataLikelihoodTimePoints (kind 2,
 * src/cellpop/DataLikelihoodTimePoints.cpp: L species columns, each a sum of species, matched cell by
 * cell at every time point, no synchronisation). */
typedef struct {
    int32_t T;                /* time points */
    int32_t R;                /* population average: replicates; time course / time points: observed cells */
    const double* observed;   /* [R*T] (time points: [R*T*MK]), NaN = missing */
    const int32_t* entry;     /* [T] output entry (sorted simulation time point) of each time point
                                 (time points: of column 0's first term) */
    bcm3hip_value_ref stdev, offset, scale;
    double weight;
    int32_t error_model;      /* BCM3HIP_CP_ERR_*: DataLikelihoodBase::Load's error_model */
    bcm3hip_value_ref proportional_stdev; /* proportional_stdev (BCM3HIP_REF_NONE = 0) */
    int32_t relative_to_time_average;     /* log(x / time mean of x) before the data likelihood */
    int32_t kind;                         /* BCM3HIP_CP_DATA_* */
    int32_t stdev_relative_to_scale;      /* stdev_relative_to_scale: stdev *= scale */
    bcm3hip_value_ref missing_stdev;      /* time course: missing_simulation_time_stdev (NONE = 300) */
    /* time points only (zero otherwise) */
    int32_t L;                            /* species columns ("a;b+c" -> 2) */
    int32_t MK;                           /* markers per observed cell (1 for 2-D data); columns read 0..L-1 */
    const int32_t* term_offset;           /* [L+1] terms of each column */
    const int32_t* term_entry;            /* [terms*T] output entry of term k at time point i */
    const bcm3hip_value_ref* col_ref;     /* [3L] stdev, offset, scale of each column */
    int32_t relative_ix;                  /* value_relative_to_timepoint_ix, -1 = none */
    int32_t only_nondivided;              /* use_only_nondivided: daughters are not simulated cells */
    /* time courses with observed lineages (the data group's "cell_id" / "parent" variables,
     * DataLikelihoodTimeCourse.cpp:132-167; CalculateCellLikelihood's recursion, :431-563): the
     * observed cells without a parent in data order, and each observed cell's children in
     * ascending order (CSR); n_roots = 0: no lineage, every observed cell is a root */
    int32_t n_roots;
    const int32_t* roots;      /* [n_roots] */
    const int32_t* child_off;  /* [R + 1] */
    const int32_t* child_ix;   /* [child_off[R]] */
} bcm3hip_cellpop_data;
enum { BCM3HIP_CP_DATA_POPULATION_AVERAGE = 0, BCM3HIP_CP_DATA_TIME_COURSE = 1, BCM3HIP_CP_DATA_TIME_POINTS = 2 };
enum { BCM3HIP_CP_ERR_NORMAL = 0, BCM3HIP_CP_ERR_T4 = 1, BCM3HIP_CP_ERR_PROPORTIONAL = 2,
       BCM3HIP_CP_ERR_ADDITIVE_PROPORTIONAL = 3 };

typedef struct {
    const char* derivative_body; /* SBMLModel::GenerateCode's generated_derivative body */
    int32_t NS;                  /* ODE-integrated species (<= 64) */
    int32_t NC;                  /* constant species */
    int32_t d;                   /* sampled variables */
    int32_t M;                   /* output entries: the experiment's simulation time points, sorted */
    const int32_t* transforms;   /* [d] BCM3HIP_TF_* */
    const double* y_init;        /* [NS] SBML initial amounts */
    const double* constant_species; /* [NC] */
    const double* output_times;  /* [M] */
    const int32_t* output_species; /* [M] ODE species read at each entry (-1 = none) */
    double rtol, atol, hmin;     /* solver_relative/absolute_tolerance, solver_min_timestep */
    int32_t max_steps;           /* solver_max_steps */
    int32_t divide_cells;
    double end_time;             /* last time point + trailing_simulation_time */
    double past_cs;              /* simulate_past_chromatid_separation_time */
    int32_t events[7];           /* replicating_DNA, replicated_DNA, PCNA_gfp, nuclear_envelope,
                                    chromatid_separation, cytokinesis, apoptosis (-1 = absent) */
    int32_t n_reset;             /* daughter initial conditions (SetInitialConditionsFromOtherCell) */
    const int32_t* reset_index;
    const double* reset_value;
    int32_t num_cells, max_cells;
    bcm3hip_value_ref entry_time;
    int32_t sobol_dims, sobol_points;
    const double* sobol;         /* [sobol_points*sobol_dims] uniforms */
    const bcm3hip_value_ref* scales; /* [sobol_dims] log-scale of each dimension (diagonal_gaussian) */
    int32_t n_actions;
    const bcm3hip_variability_action* actions;
    int32_t n_data;
    const bcm3hip_cellpop_data* data;
    /* <treatment_trajectory type="pulses"> (TreatmentTrajectoryPulses, src/cellpop/
     * TreatmentTrajectoryPulses.cpp): the constant species treat_species[i] follows pulses starting at
     * treat_times[treat_offset[i] .. treat_offset[i+1]) (sorted), with the solver's discontinuities at
     * the pulse corners (Cell.cpp:212-229, 447-461); n_treat = 0: none */
    int32_t n_treat;
    const int32_t* treat_species;  /* [n_treat] constant-species index */
    const int32_t* treat_offset;   /* [n_treat + 1] */
    const double* treat_times;     /* [treat_offset[n_treat]] */
    /* <cell_variability distribution="full_gaussian" covar_base_name="b"> (VariabilityDescription.cpp:
     * 69-128, 184-212): the group's pseudorandom vector is L z, z_i = QuantileNormal(sobol_i) and L the
     * spherical (Pinheiro & Bates) Cholesky factor from exp(scale_i) and the references b<j+1>_<i+1>
     * (j < i) times pi; diagonal_gaussian groups (the rest) use z_i exp(scale_i). n_full = 0: none. */
    int32_t n_full;
    const int32_t* full_groups;          /* [n_full][2]: first sobol dimension, D */
    const bcm3hip_value_ref* covariance; /* the full groups' D(D-1)/2 references each, in order, entry
                                            (i-1)i/2 + k of a group for the pair (k, i), k < i */
    /* synchronised time courses / time points (<data synchronize="...">, Experiment.cpp:265-292,
     * Cell.cpp:280-390): output_sync[M] is the ESynchronizeCellTrajectory of each entry
     * (BCM3HIP_CP_SYNC_*); NULL or every entry BCM3HIP_CP_SYNC_NONE: no synchronisation. With any
     * entry synchronised every cell stores its integration points (Cell.cpp:152, 232-233): event
     * times are bisections of the step's interpolant, a dividing cell ends at its interpolated
     * division time and state, and every entry's value is read from the stored steps
     * (ODESolverCVODE::GetInterpolatedY, ODESolverCVODE.cpp:183-242) at data time + sync_offset +
     * the cell's event time (none: - creation time). */
    const int32_t* output_sync;
    bcm3hip_value_ref sync_offset;  /* synchronization_time_offset (a sampled variable; NONE = 0) */
    int32_t solver;                 /* solver_type: BCM3HIP_CP_SOLVER_CVODE (0) or _DP5 (ODESolverDP5: explicit
                                       Dormand-Prince 5(4), Hairer's dense output; not with synchronised
                                       data or treatment trajectories) */
    double hmax;                    /* solver_max_timestep: DP5's max_dt (> 0, inf = none); CVODE: inf only */
} bcm3hip_cellpop_model;
enum { BCM3HIP_CP_SOLVER_CVODE = 0, BCM3HIP_CP_SOLVER_DP5 = 1 };
enum { BCM3HIP_CP_SYNC_DNA_REPLICATION_START = 0, BCM3HIP_CP_SYNC_PCNA_GFP_INCREASE = 1,
       BCM3HIP_CP_SYNC_NUCLEAR_ENVELOPE_BREAKDOWN = 2, BCM3HIP_CP_SYNC_ANAPHASE_ONSET = 3, BCM3HIP_CP_SYNC_NONE = 4 };

/* Per-cell results of the last evaluation (bcm3hip_cellpop_cells), one record per cell slot. */
typedef struct {
    double creation, sim_end, achieved;
    int32_t flags;   /* bit0 ok, bit1 divided, bit2 died, bit3 entered mitosis, bit4 spawned daughters */
    int32_t nsteps;
} bcm3hip_cell_record;

typedef struct bcm3hip_ctx bcm3hip_ctx;

/* Per-trajectory solver counters (parity/diagnostics), one record per (item, patient). */
typedef struct {
    int32_t nst, nfe, nni, nsetups, nje, netf, ncfn, nreinit;
} bcm3hip_traj_stats;

/* Options (bcm3hip_set_option) */
enum {
    BCM3HIP_OPT_LANES_PER_WAVE = 1, /* trajectories per wavefront: 1..64, 0 = auto (default) */
    BCM3HIP_OPT_BLOCK_WAVES = 2,    /* wavefronts per workgroup: 1..4 (default 1) */
    BCM3HIP_OPT_TIMING_LOG = 3,     /* 1: keep one HIP event pair per launch (see kernel_time_log) */
    BCM3HIP_OPT_UNI_SOLVER = 4,     /* one-trajectory-per-wavefront launches: 0 = state vectors across
                                       lanes (bdf_vec.h, default), 1 = scalar state (bdf_uni.h);
                                       same results */
    BCM3HIP_OPT_BLOCK_LDS = 5,      /* bytes of LDS reserved per workgroup of the PopPK launch (0..65536,
                                       default 0): caps the workgroups resident per CU, so a launch
                                       with more wavefronts than SIMDs queues the rest instead of
                                       sharing a SIMD */
    BCM3HIP_OPT_PLACEMENT_LOG = 6   /* diagnostics, PopPK one-trajectory-per-wavefront launches: 1 = each
                                       trajectory records where and when it ran (see placement_log) */
};

int bcm3hip_device_count(void);
/* 1 when PopPK contexts run on the pow / exp tables of the host libm this process loaded
 * (bcm3_amd/csrc/libm_tables.cpp): CVODE's step-size roots and the exps are then glibc's own
 * results (libm_exact.h pow_glibc / exp_glibc, bit-identical to the reference's libm calls);
 * 0 when tables of the same layout were computed instead (~1 ulp from glibc) -- no such libm, or
 * BCM3_POW=computed in the environment. Host-only query, no device needed. */
int bcm3hip_libm_pow_tables(void);
/* SIMDs of the calling thread's current device (compute units x 4), 0 on error: the wavefronts a
 * launch of one-wavefront workgroups runs one per SIMD */
int bcm3hip_current_device_simds(void);
const char* bcm3hip_error_string(int code);

int bcm3hip_open_popk(int device, const bcm3hip_popk_model* model, bcm3hip_ctx** out);
int bcm3hip_open_analytic(int device, const bcm3hip_analytic_model* model, bcm3hip_ctx** out);
/* multimodal_gaussians / truncated_t; BCM3HIP_ERR_MODEL when a covariance is not positive
 * definite (the reference's LLT fails and its ASSERT is compiled out) or a nu is not > 0 */
int bcm3hip_open_mixture(int device, const bcm3hip_mixture_model* model, bcm3hip_ctx** out);
/* pharmaco_single (PharmacoLikelihoodSingle::EvaluateLogProbability); per-item status 1 when
 * PharmacokineticModel::Solve fails (NaN state): logp = -inf */
int bcm3hip_open_expm_pk(int device, const bcm3hip_expm_pk_model* model, bcm3hip_ctx** out);
/* cell_population (CellPopulationLikelihood::EvaluateLogProbability with one experiment): the
 * cell ODE kernel is compiled at open time with hipRTC for this model's generated right-hand
 * side (the reference compiles its generated code with cmake + make and dlopen()s it,
 * src/cellpop/SolverCodeGenerator.cpp:32-431); code objects are cached on disk
 * ($BCM3_CODEGEN_DIR, default <library dir>/codegen). Per-item status 1 when the experiment fails
 * (solver failure, too many cells): logp = -inf. */
int bcm3hip_open_cellpop(int device, const bcm3hip_cellpop_model* model, bcm3hip_ctx** out);
/* cell_population with several <experiment>s (CellPopulationLikelihood::EvaluateLogProbability,
 * src/cellpop/CellPopulationLikelihood.cpp:82-101): one compiled cell kernel per experiment model,
 * logp = the sum of the experiments' log-likelihoods in experiment order; -inf (status 1) from
 * the first experiment that fails, as the reference returns there. bcm3hip_cellpop_cells reads
 * experiment 0. */
int bcm3hip_open_cellpop_experiments(int device, const bcm3hip_cellpop_model* models, int n_experiments,
                                     bcm3hip_ctx** out);
/* compile (or find in the cache) the model's cell kernel without a device (build time) */
int bcm3hip_cellpop_precompile(const bcm3hip_cellpop_model* model);
/* cells of item `item` of the last cellpop evaluation: *count cells, records / values[count*M]
 * (the data likelihood's values per output entry) / end_y[count*NS] may be NULL. In the reference's
 * cell numbering; for an evaluation that failed (logp -inf) under the device work queue the list ends
 * where that evaluation stopped enqueueing. */
int bcm3hip_cellpop_cells(bcm3hip_ctx* ctx, size_t item, int32_t* count, bcm3hip_cell_record* records,
                          double* values, double* end_y);
int bcm3hip_close(bcm3hip_ctx* ctx);
int bcm3hip_set_option(bcm3hip_ctx* ctx, int option, int64_t value);
int bcm3hip_num_variables(const bcm3hip_ctx* ctx);

/* Host-buffer batch: values[n*d] row-major (one sampler-space vector per row, prior.xml order),
 * logp[n], status[n] (may be NULL). Synchronous. */
int bcm3hip_eval_batch(bcm3hip_ctx* ctx, size_t n, size_t d, const double* values, double* logp,
                       int32_t* status);

/* Device-resident batch on a caller stream (hipStream_t as void*; NULL = the null stream):
 * values_dev[n*d], logp_dev[n], status_dev[n] (may be NULL) are device pointers.
 * Asynchronous; the kernel time of the launch is readable by bcm3hip_last_kernel_ms after the
 * stream has synchronised. */
int bcm3hip_eval_batch_device(bcm3hip_ctx* ctx, size_t n, const double* values_dev, double* logp_dev,
                              int32_t* status_dev, void* stream);
/* PopPK only: as bcm3hip_eval_batch_device for the first *n_dev (a device int32, <= n_max) items of
 * values_dev, the count read on the device (the launch covers n_max; the items beyond *n_dev return
 * at once), so a batch sized by a kernel needs no host round trip; steps_dev[i] (may be NULL) =
 * BDF steps of item i's solve (one patient per evaluation; left unwritten for P > 1). SamplerPTDevice's speculative iteration pairs. */
int bcm3hip_eval_batch_device_counted(bcm3hip_ctx* ctx, size_t n_max, const int32_t* n_dev, const double* values_dev,
                                      double* logp_dev, int32_t* status_dev, int32_t* steps_dev, void* stream);
int bcm3hip_last_kernel_ms(bcm3hip_ctx* ctx, float* ms);
/* With BCM3HIP_OPT_PLACEMENT_LOG on: the placement of the trajectories of the most recent PopPK
 * launch, 4 words per trajectory in launch order: word 0 packs the wavefront's HW_ID register (wave,
 * SIMD, CU, shader array, shader engine fields) in its low 32 bits and the shader-clock cycles the
 * trajectory took (s_memtime difference) in its high 32 bits; word 1 its XCC_ID register; words 2 and
 * 3 the constant-rate wall clock (100 MHz) when the trajectory started and when it finished. Copies min(n_max, trajectories) rows
 * (synchronises with the launch) and returns that count, or a negative error. */
int64_t bcm3hip_placement_log(bcm3hip_ctx* ctx, int64_t n_max, uint64_t* host_out);
/* The observed-to-simulated cell assignment of the time-course data likelihood alone
 * (DataLikelihoodTimeCourse.cpp:287-360 with dependencies/hungarian2's
 * hungarianMinimumWeightPerfectMatching), on the current device, for n_problems matrices of cell
 * log-likelihoods lik[p][i][j] (observed cell i, simulated cell j, -inf = not matchable, R <= 1024).
 * Device pointers: match[p][R] receives the simulated cell of every observed cell (-1 when none),
 * sum[p] the matched likelihoods summed in observed-cell order (-inf when the routine finds no
 * matching), ok[p] Evaluate's result (0: a NaN likelihood). Runs on `stream`, no synchronisation. */
int bcm3hip_assign_cells(int32_t n_problems, int32_t R, int32_t nsim, const double* lik, int32_t* match, double* sum,
                         int32_t* ok, void* stream);
/* With BCM3HIP_OPT_TIMING_LOG on: synchronises on every launch logged since the last call and
 * returns the summed / maximum kernel time (HIP events recorded on each launch's own stream) and
 * the number of launches, then clears the log. Lets a timed loop run without host syncs. */
int bcm3hip_kernel_time_log(bcm3hip_ctx* ctx, double* total_ms, int64_t* launches, double* max_ms);

/* ---- PT-MH iteration kernels (device buffers, asynchronous on `stream`, current device) ----
 * One sampler iteration of C chains of d variables = bcm3hip_pt_exchange_local (+ cross-rank
 * pairs on the host over RCCL), then bcm3hip_ptmh_propose -> bcm3hip_eval_batch_device ->
 * bcm3hip_ptmh_accept. Random numbers are counter based: splitmix64 of (seed, iter, global chain
 * index chain0 + c, slot). Replaces SamplerPT::DoMutateMove / DoExchangeMove's per-chain loops
 * (src/sampler/SamplerPT.cpp:277-319, src/sampler/SamplerPTChain.cpp:217-381). */
/* UnivariateMarginal distribution types (src/sampler/UnivariateMarginal.cpp:25-101) and their
 * parameters (p0, p1, p2): uniform (lower, upper), normal (mu, sigma), exponential (lambda),
 * gamma (k, theta), beta (a, b), half_cauchy (scale), beta_prime (a, b, scale),
 * exponential_mix (lambda, lambda2, mix). bcm3hip_ptmh_propose supports uniform and normal;
 * the adaptive proposal kernels support all. */
enum {
    BCM3HIP_PRIOR_UNIFORM = 0,
    BCM3HIP_PRIOR_NORMAL = 1,
    BCM3HIP_PRIOR_EXPONENTIAL = 2,
    BCM3HIP_PRIOR_GAMMA = 3,
    BCM3HIP_PRIOR_BETA = 4,
    BCM3HIP_PRIOR_HALF_CAUCHY = 5,
    BCM3HIP_PRIOR_BETA_PRIME = 6,
    BCM3HIP_PRIOR_EXPONENTIAL_MIX = 7,
    /* member of a Dirichlet group (MultivariateMarginal, src/sampler/MultivariateMarginal.cpp:23-180;
     * PriorIndependence.cpp:40-77): p0 = alpha_i, p1 = index of the group's first variable, p2 =
     * the group's log normalisation constant lgamma(sum alpha) - sum lgamma(alpha_i). Members are
     * consecutive; the last one is the residual 1 - sum(others) the proposals overwrite
     * (SamplerPTChain.cpp:270-278). Adaptive proposal kernels only. */
    BCM3HIP_PRIOR_DIRICHLET = 8
};
/* prior_kind[d], prior_p0[d] (lower | mu), prior_p1[d] (upper | sigma), scale[d] random-walk sd,
 * temps[C], values[C*d] -> prop[C*d], lprior_prop[C]. T == 0 chains draw from the prior. */
int bcm3hip_ptmh_propose(int C, int d, const int32_t* prior_kind, const double* prior_p0, const double* prior_p1,
                         const double* scale, const double* temps, const double* values, double* prop,
                         double* lprior_prop, int64_t chain0, uint64_t seed, uint64_t iter, void* stream);
/* TestSample + state update with llh_prop from the likelihood launch (times learning_rate);
 * accept_out[C] (may be NULL), *accepted += number accepted (may be NULL). A NaN llh (after the
 * learning rate) is fatal as in Sampler::EvaluateLikelihood (src/sampler/Sampler.cpp:172-178): the
 * chain is left unchanged and *nan_llh (may be NULL) is set to 1 for the caller to stop on. */
int bcm3hip_ptmh_accept(int C, int d, const double* temps, const double* prop, const double* lprior_prop,
                        const double* llh_prop, double learning_rate, double* values, double* lprior, double* llh,
                        double* lpp, uint8_t* accept_out, uint64_t* accepted, int32_t* nan_llh, int64_t chain0,
                        uint64_t seed, uint64_t iter, void* stream);
/* Exchange round `round` (start = round % 2) for the pairs inside chains [g0, g0+C) of the ladder;
 * wrap_local: also the pair (C-1, 0) (single-rank ladder). acc_mask[C] marks accepted first chains. */
int bcm3hip_pt_exchange_local(int C, int d, int64_t g0, int start, int wrap_local, const double* temps,
                              double* values, double* llh, double* lprior, double* lpp, uint8_t* acc_mask,
                              uint64_t* accepted, uint64_t seed, uint64_t round, void* stream);

/* ---- Adaptive proposals (one_block blocking), state resident in device memory ----
 * Replace SamplerPTChain::MutateMove's per-block Proposal::Update / GetNewSample /
 * CalculateMHRatio / NotifyAccepted (src/sampler/SamplerPTChain.cpp:241-310) for
 * ProposalGlobalCovariance (src/sampler/ProposalGlobalCovariance.cpp:20-47) and
 * ProposalGaussianMixture (src/sampler/ProposalGaussianMixture.cpp:20-103), and
 * SampleHistory::AddSample (src/sampler/SampleHistory.cpp:32-45). All pointers in the struct are
 * device pointers; per-chain arrays are indexed by the rank-local chain c in [0, C). */
enum { BCM3HIP_PROPOSAL_GLOBAL_COVARIANCE = 0, BCM3HIP_PROPOSAL_GAUSSIAN_MIXTURE = 1 };
enum { BCM3HIP_PROPOSAL_KMAX = 16 };
typedef struct {
    int32_t kind;                 /* BCM3HIP_PROPOSAL_* (ptmhsampler.proposal_type) */
    int32_t kmax;                 /* component slots per chain, 1..BCM3HIP_PROPOSAL_KMAX */
    double t_dof;                 /* ptmhsampler.proposal_t_dof, 0 = normal proposals */
    double target_acceptance;     /* Proposal::Initialize: 0.44 / 0.35 / 0.3 / 0.234 by d */
    double scaling_learning_rate; /* 0.05 (Proposal.cpp:22) */
    double scaling_ema_period;    /* 1000 (Proposal.cpp:21) */
    const double* lower;          /* [d] prior bounds for ReflectOnBounds (-inf / +inf if unbounded) */
    const double* upper;          /* [d] */
    int32_t* ncomp;               /* [C] mixture components in use (1 for global_covariance) */
    double* weights;              /* [C][kmax] mixture weights */
    double* mean;                 /* [C][kmax][d] component means */
    double* chol;                 /* [C][kmax][d][d] lower Cholesky factors, row-major */
    double* logc;                 /* [C][kmax] -sum log L_jj - d/2 log(2 pi) */
    double* scale;                /* [C][kmax] adaptive scales */
    double* ema;                  /* [C][kmax] acceptance-rate EMAs */
    int32_t* selected;            /* [C] component of the last proposal, -1 before the first */
    double* work;                 /* [C][2*kmax + 2*d] scratch */
} bcm3hip_proposal;
/* As bcm3hip_ptmh_propose, with the proposal's scale update, the mixture component choice and
 * log_mh[C] = log Metropolis-Hastings ratio (0 for global_covariance). */
int bcm3hip_ptmh_propose_adaptive(int C, int d, const int32_t* prior_kind, const double* prior_p0,
                                  const double* prior_p1, const double* prior_p2, const double* temps,
                                  const double* values, double* prop,
                                  double* lprior_prop, double* log_mh, const bcm3hip_proposal* proposal,
                                  int64_t chain0, uint64_t seed, uint64_t iter, void* stream);
/* As bcm3hip_ptmh_accept, with log_mh added to the transition and the acceptance EMA update. */
int bcm3hip_ptmh_accept_adaptive(int C, int d, const double* temps, const double* prop, const double* lprior_prop,
                                 const double* llh_prop, const double* log_mh, double learning_rate, double* values,
                                 double* lprior, double* llh, double* lpp, uint8_t* accept_out, uint64_t* accepted,
                                 int32_t* nan_llh, const bcm3hip_proposal* proposal, int64_t chain0, uint64_t seed,
                                 uint64_t iter, void* stream);
/* ---- speculative iteration pairs (SamplerPTDevice) ----
 * Iteration r+1's proposal of chain c starts from the state exchange round r+1 leaves in slot c: its
 * own state after iteration r (old = values[c], or prop[c] if accepted) or its exchange partner's
 * (values[p] / prop[p]), with the acceptance EMA the accept of r leaves (it decides Proposal::Update's
 * scale branch). With counter-based random numbers every such proposal is determined now, so one
 * launch evaluates iteration r's proposals AND every candidate of r+1; after accept r and exchange
 * r+1, bcm3hip_ptmh_spec_select picks the candidate that happened and its log-likelihood, so the
 * accept of r+1 needs no launch -- bit-identical to the sequential iteration.
 * Candidate slots per chain (k): 0 old_c (own reject), 1 prop_c (own accept), 2 old_p, 3 prop_p
 * (swapped; own reject -- or either outcome when Update's branch does not depend on it), 4 old_p,
 * 5 prop_p (swapped, own accept; only when the branch differs). T == 0 chains: slot 0 (a prior
 * draw). All pointers are device pointers sized for C chains (slots [C][6]). */
enum { BCM3HIP_SPEC_SLOTS = 6 };
/* partner codes besides local chain indices: -1 none, and the neighbour ranks' boundary chains of a
 * sharded ladder (my last chain pairs with the next rank's first, my first with the previous rank's
 * last) whose (state, proposal) rows arrive in `remote` = [next: state d | proposal d][prev: ...] */
enum { BCM3HIP_SPEC_REMOTE_NEXT = -2, BCM3HIP_SPEC_REMOTE_PREV = -3 };
typedef struct {
    double* cand_x;       /* [C][6][d] candidate proposals */
    double* cand_lp;      /* [C][6] their log prior */
    double* cand_lmh;     /* [C][6] log MH ratio */
    double* cand_llh;     /* [C][6] log-likelihood (scattered from the batch) */
    int32_t* cand_sel;    /* [C][6] selected component */
    int32_t* cand_upd;    /* [C][6] component whose scale Update changed (-1 none) */
    double* cand_sc;      /* [C][6] its new scale */
    uint8_t* cand_active; /* [C][6] */
    int32_t* cand_steps;  /* [C][6] BDF steps of the candidate's solve */
    int32_t* steps_hint;  /* [C] BDF steps of the solve of the state in each slot (dispatch order) */
    int32_t* steps_prop;  /* [C] steps of the proposals being accepted or rejected */
    double* batch_x;      /* [7C][d] the launch's vectors, longest predicted solve first */
    double* batch_llh;    /* [7C] */
    int32_t* batch_status;/* [7C] */
    int32_t* batch_steps; /* [7C] */
    int32_t* batch_src;   /* [7C] source of each batch entry: c < C proposal of chain c, C + 6c + k candidate */
    int32_t* batch_n;     /* [1] entries in use (0 before the first launch) */
    int32_t* pred_steps;  /* [7C] predicted solve length of each entry (batch order key) */
    int64_t* batch_total; /* [1] running sum of the entries of every batch built (NULL: not kept) */
    int32_t* batch_pos;   /* [7C] batch position of each entry (-1: not in the batch), the inverse of
                             batch_src; NULL: not kept. When kept, bcm3hip_ptmh_spec_commit with
                             select = 0 takes the batch's results itself (no spec_scatter launch) */
    float* batch_xs;      /* [7C][d] the launch's vectors in single precision, scaled by 1 / prior sd
                             (the dispatch-order predictor's distances); NULL: not kept */
} bcm3hip_spec;
/* candidates of iteration iter_next = r + 1 (after bcm3hip_ptmh_propose_adaptive of iteration r, whose
 * proposals are in prop); partner[c] = exchange partner of chain c in round r + 1 (-1 none) */
int bcm3hip_ptmh_spec_candidates(int C, int d, const int32_t* prior_kind, const double* prior_p0,
                                 const double* prior_p1, const double* prior_p2, const double* temps,
                                 const double* values, const double* prop, const int32_t* partner,
                                 const double* remote, const bcm3hip_proposal* proposal, const bcm3hip_spec* spec,
                                 int64_t chain0, uint64_t seed, uint64_t iter_next, void* stream);
/* the launch's batch: iteration r's C proposals + the active candidates, ordered by the predicted
 * length of their solves, longest first (C <= 585): the mean BDF steps of the entry's 4 nearest
 * neighbours among the previous launch's entries, distances scaled by inv_scale[d] (1 / prior sd);
 * before any launch, the steps_hint of the slot the entry starts from. first_round > 0: the
 * wavefronts the device runs one per SIMD (its SIMD count); a batch larger than that puts its
 * shortest entries on the SIMDs that take two wavefronts (positions p and p + first_round), so the
 * longest run alone; 0: plain longest-first order */
int bcm3hip_ptmh_spec_batch(int C, int d, const double* prop, const int32_t* partner, const double* inv_scale,
                            int first_round, const bcm3hip_spec* spec, void* stream);
/* batch results back: llh_prop[c] (iteration r), cand_llh / cand_steps, steps_prop */
int bcm3hip_ptmh_spec_scatter(int C, const bcm3hip_spec* spec, double* llh_prop, void* stream);
/* after accept r (accept_out = acc_mutate[C]) and exchange r + 1 (accept_out = acc_exchange, indexed
 * by the first chain of each pair; pair_first[c] = that chain for c's pair in round r + 1; for a
 * sharded ladder cross_acc[2] = pt_cross_accept's flags, remote / values as in spec_candidates and
 * after the exchange): iteration
 * r + 1's proposal, log prior, MH ratio and log-likelihood of each chain, and the proposal state
 * writes its propose would have made (scale Update, selected component). *error != 0 if a needed
 * candidate was not evaluated (never expected). */
int bcm3hip_ptmh_spec_select(int C, int d, const double* temps, const int32_t* partner, const int32_t* pair_first,
                             const uint8_t* acc_mutate, const uint8_t* acc_exchange, const uint8_t* cross_acc,
                             const double* remote, const double* values, const bcm3hip_spec* spec, double* prop,
                             double* lprior_prop, double* log_mh, double* llh_prop, const bcm3hip_proposal* proposal,
                             int32_t* error, void* stream);
/* The end of one iteration of a pair in ONE launch, one thread per chain: with select != 0 first
 * bcm3hip_ptmh_spec_select (iteration r + 1; acc_prev = the accept flags of iteration r, a different
 * buffer than accept_out), then bcm3hip_ptmh_accept_adaptive (flags to accept_out), the accept's
 * bcm3hip_ptmh_spec_track and bcm3hip_history_add (mask NULL; skipped when history is NULL) -- per
 * chain the same operations in the same order as those launches. */
int bcm3hip_ptmh_spec_commit(int C, int d, int select, const double* temps, const int32_t* partner,
                             const int32_t* pair_first, const uint8_t* acc_prev, const uint8_t* acc_exchange,
                             const uint8_t* cross_acc, const double* remote, const bcm3hip_spec* spec, double* prop,
                             double* lprior_prop, double* log_mh, double* llh_prop, double learning_rate, double* values,
                             double* lprior, double* llh, double* lpp, uint8_t* accept_out, uint64_t* accepted,
                             int32_t* nan_llh, const bcm3hip_proposal* proposal, int64_t chain0, uint64_t seed,
                             uint64_t iter, int H, int subsampling, float* history, int64_t* counters, int32_t* error,
                             void* stream);
/* One exchange round of a single-rank ladder whose pairs cover every chain once (even C), and what
 * follows it in a pair, in ONE workgroup: bcm3hip_pt_exchange_local (accept flags to acc_exchange),
 * the round's bcm3hip_ptmh_spec_track and bcm3hip_history_add of every chain (skipped when history
 * is NULL); C <= 4096. */
int bcm3hip_ptmh_spec_exchange(int C, int d, int64_t g0, int start, int wrap_local, const double* temps,
                               double* values, double* llh, double* lprior, double* lpp, uint8_t* acc_exchange,
                               uint64_t* accepted, uint64_t seed, uint64_t round, const int32_t* partner,
                               const int32_t* pair_first, const bcm3hip_spec* spec, int H, int subsampling,
                               float* history, int64_t* counters, void* stream);
/* dispatch-order bookkeeping (steps_hint = BDF steps of the solve of the state in each slot): after an
 * accept (acc_mutate: the proposals' steps, steps_prop, become the states') or, with acc_mutate NULL,
 * after an exchange round (acc_exchange indexed by pair_first, partner as in spec_select) */
/* The end of a speculative pair on a single-rank ladder whose exchange pairs cover every chain (the
 * condition of bcm3hip_ptmh_spec_exchange) in ONE launch: bcm3hip_ptmh_spec_commit(select = 0,
 * iteration `iter`, flags to acc_mut), bcm3hip_ptmh_spec_exchange(start, wrap_local, round; flags to
 * acc_exc) and bcm3hip_ptmh_spec_commit(select = 1, iteration iter + 1, acc_prev = acc_mut, flags to
 * acc_mut2) -- bit-identical to the three launches (SamplerPT.cpp:203-212 twice). spec->batch_pos is
 * required (the first commit reads the batch through it); C <= 4096. */
int bcm3hip_ptmh_spec_tail(int C, int d, int64_t g0, int start, int wrap_local, const double* temps,
                           const int32_t* partner, const int32_t* pair_first, uint8_t* acc_mut, uint8_t* acc_mut2,
                           uint8_t* acc_exc, const uint8_t* cross_acc, const double* remote, uint64_t* accepted_mutate,
                           uint64_t* accepted_exchange, const bcm3hip_spec* spec, double* prop, double* lprior_prop,
                           double* log_mh, double* llh_prop, double learning_rate, double* values, double* lprior,
                           double* llh, double* lpp, int32_t* nan_llh, const bcm3hip_proposal* proposal, uint64_t seed,
                           uint64_t iter, uint64_t round, int H, int subsampling, float* history, int64_t* counters,
                           int32_t* error, void* stream);
int bcm3hip_ptmh_spec_track(int C, const uint8_t* acc_mutate, const int32_t* partner, const int32_t* pair_first,
                            const uint8_t* acc_exchange, const bcm3hip_spec* spec, void* stream);
/* The propose kernel's mixture arithmetic (GMM::CalculateResponsibilities, src/stats/GMM.cpp:172-186,
 * with the component densities of GMM::LogPdfMVN :392-398) at n points x[n][d] (device buffers,
 * d <= 64, K <= 64): logpdf[n] = log sum_k w_k N(x; mean_k, L_k L_k^T), resp[n][K]; either may be
 * NULL. mean[K][d], chol[K][d][d] (lower, row-major), logc[K], weights[K] as in bcm3hip_proposal. */
int bcm3hip_gmm_eval(int n, int d, int K, const double* x, const double* mean, const double* chol, const double* logc,
                     const double* weights, double* logpdf, double* resp, void* stream);
/* SampleHistory::AddSample for chains with T != 0 and (mask == NULL or mask[c] != 0):
 * history[C][H][d] float ring, counters[C][2] = {samples stored, calls since the last store}. */
int bcm3hip_history_add(int C, int d, int H, int subsampling, const double* temps, const double* values,
                        const uint8_t* mask, float* history, int64_t* counters, void* stream);

/* One exchange between local chains i1 and i2 (stochastic_random swapping, SamplerPT.cpp:300-305;
 * g1 = global index of i1, keys the uniform); *acc_out (may be NULL) = 1 if swapped. */
int bcm3hip_pt_exchange_pair(int C, int d, int i1, int i2, int64_t g1, const double* temps, double* values,
                             double* llh, double* lprior, double* lpp, uint8_t* acc_out, uint64_t* accepted,
                             uint64_t seed, uint64_t round, void* stream);

/* Slice-boundary exchange of a sharded ladder (rank r owns global chains [g0, g0 + C)).
 * bcm3hip_pt_pack_boundary: the records {values[d], llh, lprior, lpp, T} (d + 4 doubles) of the
 * last and the first local chain (either output may be NULL), sent to the next / previous rank.
 * bcm3hip_pt_cross_accept: ExchangeMove (SamplerPTChain.cpp:328-381) of pair A = (my chain C-1,
 * the next rank's first chain = recv_next; uniform keyed by g0 + C - 1) when do_next, and of
 * pair B = (the previous rank's last chain = recv_prev, my chain 0; keyed by gp, its global index)
 * when do_prev; each rank keeps its side; acc_out[2] (may be NULL) = {A, B} accepted; *accepted
 * counts pair A (the rank of a pair's first chain counts it). */
int bcm3hip_pt_pack_boundary(int C, int d, const double* temps, const double* values, const double* llh,
                             const double* lprior, const double* lpp, double* send_last, double* send_first,
                             void* stream);
int bcm3hip_pt_cross_accept(int C, int d, int64_t g0, int64_t gp, int do_next, int do_prev, const double* temps,
                            double* values, double* llh, double* lprior, double* lpp, const double* recv_next,
                            const double* recv_prev, uint8_t* acc_out, uint64_t* accepted, uint64_t seed,
                            uint64_t round, void* stream);

/* ---- device runtime for the host sampler (runtime.hip) ---- */
enum { BCM3HIP_H2D = 1, BCM3HIP_D2H = 2, BCM3HIP_D2D = 3 };
int bcm3hip_set_device(int device);
int bcm3hip_malloc(void** ptr, size_t bytes);
int bcm3hip_free(void* ptr);
int bcm3hip_memcpy_async(void* dst, const void* src, size_t bytes, int kind, void* stream);
int bcm3hip_memset_async(void* dst, int value, size_t bytes, void* stream);
int bcm3hip_stream_create(void** stream);
int bcm3hip_stream_destroy(void* stream);
int bcm3hip_stream_synchronize(void* stream);
/* RCCL point-to-point for the PT swap between neighbouring ranks (replaces the reference's
 * single-process exchange loop). The unique id is an opaque
 * BCM3HIP_NCCL_ID_BYTES-byte blob made on one rank and broadcast by the caller. */
#define BCM3HIP_NCCL_ID_BYTES 128
int bcm3hip_nccl_get_unique_id(void* id);
int bcm3hip_nccl_comm_init(const void* id, int rank, int world, void** comm);
int bcm3hip_nccl_comm_destroy(void* comm);
int bcm3hip_nccl_exchange(void* comm, int n_send, const double* const* send, const int* send_peer, int n_recv,
                          double* const* recv, const int* recv_peer, size_t count, void* stream);

/* Parity/diagnostic batch (host buffers, any output may be NULL):
 * patient_llh[n*P], traj[n*P*N*T] (states at output times, NaN where not simulated),
 * stats[n*P]. PopPK contexts only. */
int bcm3hip_eval_batch_detail(bcm3hip_ctx* ctx, size_t n, size_t d, const double* values, double* logp,
                              int32_t* status, double* patient_llh, double* traj, bcm3hip_traj_stats* stats);

#ifdef __cplusplus
}
#endif
#endif
