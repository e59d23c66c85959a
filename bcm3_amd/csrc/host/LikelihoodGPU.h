// LikelihoodGPU.h -- MI355X-backed implementations of the reference's likelihood types on the
// hot path, behind the bcm3::Likelihood interface:
//   pop_pk_trajectory  LikelihoodPopPKTrajectory (src/likelihoods/LikelihoodPopPKTrajectory.h:10-115)
//   pharmacokinetic_trajectory  LikelihoodPharmacokineticTrajectory
//                      (src/likelihoods/LikelihoodPharmacokineticTrajectory.h; one patient, same solver)
//   pharmaco_single    PharmacoLikelihoodSingle  (src/pharmaco/PharmacoLikelihoodSingle.h; matrix-exponential PK)
//   banana             TestLikelihoodBanana      (src/likelihoods/TestLikelihoodBanana.cpp)
//   circular           TestLikelihoodCircular    (src/likelihoods/TestLikelihoodCircular.cpp)
//   multimodal_gaussians TestLikelihoodMultimodalGaussians (src/likelihoods/TestLikelihoodMultimodalGaussians.cpp)
//   truncated_t        TestLikelihoodTruncatedT  (src/likelihoods/TestLikelihoodTruncatedT.cpp)
//   dummy              LikelihoodDummy           (src/likelihoods/LikelihoodDummy.cpp)
// Each owns one libbcm3hip context (include/bcm3hip.h) on the configured device. There is no
// CPU fallback: without a GPU, Initialize fails.
#pragma once
#include <cmath>
#include <condition_variable>
#include <mutex>
#include <set>
#include <vector>

#include "../../../include/bcm3hip.h"
#include "Likelihood.h"

namespace bcm3 {

class LikelihoodGPUBase : public Likelihood {
public:
    ~LikelihoodGPUBase() override;
    // Reentrant: concurrent single evaluations from the reference's sampling threads (TaskManager,
    // one task per chain) are combined into batched launches -- the threads that arrive while a
    // launch runs go into the next one -- so the drop-in single-vector route (EvaluateLogProbability,
    // and the LikelihoodDLL C plugin on top of it) approaches the batched rate when there are
    // many sampling threads. Each result depends only on its own vector.
    bool IsReentrant() override { return true; }
    bool EvaluateLogProbability(size_t threadix, const VectorReal& values, Real& logp) override;
    bool EvaluateLogProbabilityBatch(size_t n, const Real* values, Real* logp, int32_t* status) override;
    bool EvaluateLogProbabilityBatchDevice(size_t n, const Real* values_dev, Real* logp_dev, int32_t* status_dev,
                                           void* stream) override;
    bool EvaluateLogProbabilityBatchDeviceCounted(size_t n_max, const int32_t* n_dev, const Real* values_dev,
                                                  Real* logp_dev, int32_t* status_dev, int32_t* steps_dev,
                                                  void* stream) override;
    float LastKernelMilliseconds() override;
    bool KernelTimeLog(double& total_ms, int64_t& launches, double& max_ms) override;
    bool SetBackendOption(int option, int64_t value) override;
    bcm3hip_ctx* Context() const { return ctx; }

protected:
    bool OpenDevice(const OptionsMap& vm);
    virtual bool CheckEvaluable() { return true; }
    int device = 0;
    bcm3hip_ctx* ctx = nullptr;
    std::mutex mutex;

private:
    struct Request {
        const Real* values;
        Real logp;
        bool done, ok;
    };
    std::mutex comb_mutex;
    std::condition_variable comb_cv;
    std::vector<Request*> comb_queue;
    bool comb_busy = false;
};

class LikelihoodPopPKTrajectory : public LikelihoodGPUBase {
public:
    LikelihoodPopPKTrajectory(size_t sampling_threads, size_t evaluation_threads);
    bool Initialize(std::shared_ptr<const VariableSet> varset, const XmlNode& likelihood_node,
                    const OptionsMap& vm) override;
    bool PostInitialize() override { return true; }
    bool SupportsCountedBatch() const override { return ctx != nullptr; }

    size_t GetNumPatients() const { return patient_ids.size(); }
    const std::vector<Real>& GetTimepoints() const { return time; }
    // the flat model handed to the device (for diagnostics / tests)
    const bcm3hip_popk_model& GetDeviceModel() const { return model; }

protected:
    bool CheckEvaluable() override;

private:
    enum PKModelType {
        PKMT_OneCompartment,
        PKMT_TwoCompartment,
        PKMT_OneCompartmentBiphasicUptake,
        PKMT_TwoCompartmentBiphasicUptake,
        PKMT_OneCompartmentTransit,
        PKMT_TwoCompartmentTransit,
        PKMT_Undefined
    };
    size_t sampling_threads;
    std::string drug;
    PKModelType pk_type = PKMT_Undefined;
    size_t num_pk_params = 0, num_pk_pop_params = 0;
    Real fixed_vod, fixed_periphery_fwd, fixed_periphery_bwd;
    std::vector<Real> time;
    std::vector<std::string> patient_ids;
    std::vector<Real> observed, dose, dosing_interval, dose_after_dose_change, dose_change_time;
    std::vector<int32_t> intermittent, simulate_until, transforms;
    std::vector<uint8_t> skipped_days;
    Real MW;
    bcm3hip_popk_model model{};
};

// One patient's trajectory (LikelihoodPharmacokineticTrajectory.cpp:85-340): the PopPK kernel with
// the single-patient parameter map (BCM3HIP_PARAM_MAP_SINGLE)
class LikelihoodPharmacokineticTrajectory : public LikelihoodGPUBase {
public:
    LikelihoodPharmacokineticTrajectory(size_t sampling_threads, size_t evaluation_threads) {}
    bool Initialize(std::shared_ptr<const VariableSet> varset, const XmlNode& likelihood_node,
                    const OptionsMap& vm) override;
    bool PostInitialize() override { return true; }
    bool SupportsCountedBatch() const override { return ctx != nullptr; }
    const std::string& GetPatientID() const { return patient_id; }
    const bcm3hip_popk_model& GetDeviceModel() const { return model; }

protected:
    bool CheckEvaluable() override;

private:
    std::string drug, patient_id;
    Real fixed_vod = NAN, fixed_periphery_fwd = NAN, fixed_periphery_bwd = NAN, MW = NAN;
    std::vector<Real> time, observed, dose, dosing_interval, dose_after_dose_change, dose_change_time;
    std::vector<int32_t> intermittent, simulate_until, transforms;
    std::vector<uint8_t> skipped_days;
    bcm3hip_popk_model model{};
};

// Patient::Load's result (src/pharmaco/PharmacoPatient.h)
struct PharmacoPatient {
    std::string patient_id;
    std::vector<Real> treatment_timepoints, treatment_doses, observation_timepoints, observed_concentrations;
};

// One patient, linear compartment model solved by matrix exponentials
// (PharmacoLikelihoodSingle.cpp:36-218, PharmacoPatient.cpp:8-116, PharmacokineticModel.cpp:111-247).
// Initialize loads the patient (JSON sidecar of the reference's pkdata.nc); PostInitialize resolves
// the variables by name and opens the device context, as the reference resolves them there.
class PharmacoLikelihoodSingle : public LikelihoodGPUBase {
public:
    PharmacoLikelihoodSingle(size_t sampling_threads, size_t evaluation_threads) {}
    bool Initialize(std::shared_ptr<const VariableSet> varset, const XmlNode& likelihood_node,
                    const OptionsMap& vm) override;
    bool PostInitialize() override;
    const PharmacoPatient& GetPatient() const { return patient; }
    const bcm3hip_expm_pk_model& GetDeviceModel() const { return model; }

private:
    std::string drug;
    PharmacoPatient patient;
    bool use_peripheral_compartment = false, biphasic_absorption = false, use_metabolite = false;
    size_t num_transit_compartments = 0;
    Real MW = NAN;
    std::vector<int32_t> transforms;
    OptionsMap options;
    bcm3hip_expm_pk_model model{};
};

// Every patient of the trial, rates drawn per patient from the population distribution
// (PharmacoLikelihoodPopulation.cpp:43-340), log-likelihoods summed in patient order. The
// reference's exact-match result cache (likelihood_cache_size, .cpp:356-393) only returns values
// the solve reproduces bit for bit; the batched device path evaluates every patient.
class PharmacoLikelihoodPopulation : public LikelihoodGPUBase {
public:
    PharmacoLikelihoodPopulation(size_t sampling_threads, size_t evaluation_threads) {}
    bool Initialize(std::shared_ptr<const VariableSet> varset, const XmlNode& likelihood_node,
                    const OptionsMap& vm) override;
    bool PostInitialize() override;
    size_t GetNumPatients() const { return patients.size(); }
    const bcm3hip_expm_pk_model& GetDeviceModel() const { return model; }

private:
    bool InitializePatientMarginals(const std::string& name, int which);
    std::string drug;
    std::vector<PharmacoPatient> patients;
    bool use_peripheral_compartment = false, use_bioavailability = false;
    size_t num_transit_compartments = 0;
    Real MW = NAN;
    std::vector<int32_t> transforms, patient_ix, treat_offset, obs_offset;
    std::vector<Real> treat_times, treat_doses, obs_times, obs_conc;
    OptionsMap options;
    bcm3hip_expm_pk_model model{};
};

class TestLikelihoodBanana : public LikelihoodGPUBase {
public:
    TestLikelihoodBanana(size_t sampling_threads, size_t evaluation_threads) {}
    bool Initialize(std::shared_ptr<const VariableSet> varset, const XmlNode& likelihood_node,
                    const OptionsMap& vm) override;

private:
    size_t dim = 0;
    Real sd1 = 0, sd2 = 0;
};

class TestLikelihoodCircular : public LikelihoodGPUBase {
public:
    TestLikelihoodCircular(size_t sampling_threads, size_t evaluation_threads) {}
    bool Initialize(std::shared_ptr<const VariableSet> varset, const XmlNode& likelihood_node,
                    const OptionsMap& vm) override;

private:
    size_t dimension = 0;
    Real r = 2.0, offset = 3.5, w = 0.1;
};

class TestLikelihoodMultimodalGaussians : public LikelihoodGPUBase {
public:
    TestLikelihoodMultimodalGaussians(size_t sampling_threads, size_t evaluation_threads) {}
    bool Initialize(std::shared_ptr<const VariableSet> varset, const XmlNode& likelihood_node,
                    const OptionsMap& vm) override;
};

class TestLikelihoodTruncatedT : public LikelihoodGPUBase {
public:
    TestLikelihoodTruncatedT(size_t sampling_threads, size_t evaluation_threads) {}
    bool Initialize(std::shared_ptr<const VariableSet> varset, const XmlNode& likelihood_node,
                    const OptionsMap& vm) override;

private:
    size_t dimensions = 0, num_clusters = 0;
};

class LikelihoodDummy : public LikelihoodGPUBase {
public:
    LikelihoodDummy(size_t sampling_threads, size_t evaluation_threads) {}
    bool Initialize(std::shared_ptr<const VariableSet> varset, const XmlNode& likelihood_node,
                    const OptionsMap& vm) override;
};

// bcm3::ParseVectorFromString (src/utils/VectorUtils.cpp:204-219: ';'-separated, empty tokens kept,
// each converted by boost::lexical_cast<Real>) and ParseMatrixFromString (VectorUtils.h:39-67: rows
// separated by ';', columns by ','; every row as long as the first). Errors are logged.
bool ParseVectorFromString(const std::string& str, std::vector<Real>& v);
bool ParseMatrixFromString(const std::string& str, std::vector<std::vector<Real>>& m);

}  // namespace bcm3
