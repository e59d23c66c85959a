// Likelihood.h -- the bcm3::Likelihood plugin surface (src/sampler/Likelihood.h:9-35) and
// LikelihoodFactory (src/likelihoods/LikelihoodFactory.h:8-19), Boost-free, plus one batched
// virtual used by the MI355X fan-out: EvaluateLogProbabilityBatch evaluates all chains' proposals
// of one mutate step in one launch (replacing SamplerPT::DoMutateMove's per-chain TaskManager
// tasks, src/sampler/SamplerPT.cpp:308-319).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "VariableSet.h"
#include "xml.h"

namespace bcm3 {

// boost::program_options::variables_map stand-in (key -> value as written in config.txt / CLI)
using OptionsMap = std::map<std::string, std::string>;

class Likelihood {
public:
    virtual ~Likelihood();

    bool SetLearningRate(Real learning_rate);
    Real GetLearningRate() const { return learning_rate; }

    virtual bool Initialize(std::shared_ptr<const VariableSet> varset, const XmlNode& likelihood_node,
                            const OptionsMap& vm);
    virtual bool AddNonSampledParameters(const std::vector<std::string>& variable_names);
    virtual void SetNonSampledParameters(const VectorReal& values);
    virtual bool PostInitialize();
    virtual bool IsReentrant() = 0;
    virtual void OutputEvaluationStatistics(const std::string& path) const {}

    //! Evaluate the log likelihood of one parameter vector (sampler space, prior.xml order).
    //! @return false on a non-recoverable error (the sampler stops); logp = -inf is legal.
    virtual bool EvaluateLogProbability(size_t threadix, const VectorReal& values, Real& logp) = 0;

    //! Batched evaluation: values[n*d] row-major, logp[n], status[n] (may be null; 0 = ok,
    //! 1 = model failure -> -inf). Default: loop over EvaluateLogProbability on thread 0.
    virtual bool EvaluateLogProbabilityBatch(size_t n, const Real* values, Real* logp, int32_t* status);
    //! Device-resident batch on a HIP stream (void* hipStream_t); false if unsupported.
    virtual bool EvaluateLogProbabilityBatchDevice(size_t n, const Real* values_dev, Real* logp_dev,
                                                   int32_t* status_dev, void* stream);
    //! Device-resident batch whose size *n_dev (<= n_max) is a device value, with the solver steps
    //! of each item in steps_dev (may be null): the speculative iteration pairs of SamplerPTDevice.
    //! False if unsupported (only latency-bound likelihoods -- the PopPK BDF kernel -- provide it).
    virtual bool EvaluateLogProbabilityBatchDeviceCounted(size_t n_max, const int32_t* n_dev, const Real* values_dev,
                                                          Real* logp_dev, int32_t* status_dev, int32_t* steps_dev,
                                                          void* stream)
    {
        return false;
    }
    virtual bool SupportsCountedBatch() const { return false; }
    //! Duration of the last kernel launch (HIP events), < 0 if unknown.
    virtual float LastKernelMilliseconds() { return -1.0f; }
    //! Summed / max kernel time and launch count since the last call (BCM3HIP_OPT_TIMING_LOG).
    virtual bool KernelTimeLog(double& total_ms, int64_t& launches, double& max_ms) { return false; }
    //! Backend tuning option (bcm3hip_set_option); false if unsupported.
    virtual bool SetBackendOption(int option, int64_t value) { return false; }

    size_t GetNumVariables() const { return varset ? varset->GetNumVariables() : 0; }
    const VariableSet* GetVariableSet() const { return varset.get(); }

protected:
    Likelihood();

    Real learning_rate;
    std::shared_ptr<const VariableSet> varset;
};

class LikelihoodFactory {
public:
    // LikelihoodFactory::CreateLikelihood (LikelihoodFactory.cpp:31-100): type string of
    // <bcm_likelihood type="..."> -> class; then Initialize(varset, node, vm).
    static std::shared_ptr<Likelihood> CreateLikelihood(const std::string& likelihood_xml_fn,
                                                        std::shared_ptr<const VariableSet> varset,
                                                        const OptionsMap& vm, size_t sampling_threads,
                                                        size_t evaluation_threads, bool running_inference = true);
    static std::vector<std::string> SupportedTypes();
};

// helper: option lookup with default
std::string option_get(const OptionsMap& vm, const std::string& key, const std::string& def);

}  // namespace bcm3
