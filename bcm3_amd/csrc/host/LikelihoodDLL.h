// LikelihoodDLL.h -- the reference's `type="dll"` likelihood (src/likelihoods/LikelihoodDLL.h:
// 9-34, .cpp:34-116): a user plugin .so exporting initialize_likelihood / evaluate_log_probability
// (include/bcm3_dll.h), evaluated on host threads. It is the user's own CPU code, kept so that a
// likelihood.xml naming type="dll" keeps working with this framework; the MI355X path is the GPU
// likelihood types. Batches are spread over host threads (the plugin must be re-entrant,
// README.md:77); the device-buffer batch stages through host memory.
#pragma once
#include <string>
#include <vector>

#include "Likelihood.h"

namespace bcm3 {

class LikelihoodDLL : public Likelihood {
public:
    LikelihoodDLL(size_t sampling_threads, size_t evaluation_threads);
    ~LikelihoodDLL() override;
    bool Initialize(std::shared_ptr<const VariableSet> varset, const XmlNode& likelihood_node,
                    const OptionsMap& vm) override;
    bool PostInitialize() override;
    bool IsReentrant() override { return true; }
    bool EvaluateLogProbability(size_t threadix, const VectorReal& values, Real& logp) override;
    bool EvaluateLogProbabilityBatch(size_t n, const Real* values, Real* logp, int32_t* status) override;
    bool EvaluateLogProbabilityBatchDevice(size_t n, const Real* values_dev, Real* logp_dev, int32_t* status_dev,
                                           void* stream) override;

private:
    using initialize_fn = bool (*)(size_t, const char* const*);
    using likelihood_fn = bool (*)(size_t, const double*, const char* const*, double*);
    void* handle = nullptr;
    initialize_fn initialize = nullptr;
    likelihood_fn likelihood = nullptr;
    std::vector<std::string> names;
    std::vector<const char*> name_ptrs;
    size_t threads = 1;
};

}  // namespace bcm3
