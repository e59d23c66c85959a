// Likelihood.cpp -- bcm3::Likelihood defaults (src/sampler/Likelihood.cpp:1-44) and the factory.
#include "Likelihood.h"
#include "LikelihoodCellPopulation.h"

#include <cmath>

#include "LikelihoodDLL.h"
#include "LikelihoodGPU.h"
#include "log.h"

namespace bcm3 {

Likelihood::Likelihood() : learning_rate(1.0) {}
Likelihood::~Likelihood() {}

bool Likelihood::SetLearningRate(Real lr)
{
    if (lr <= 0.0 || lr > 1.0) {
        LOGERROR("Learning rate should be in (0, 1], got %g", lr);
        return false;
    }
    learning_rate = lr;
    return true;
}

bool Likelihood::Initialize(std::shared_ptr<const VariableSet> vs, const XmlNode&, const OptionsMap&)
{
    varset = vs;
    return true;
}

bool Likelihood::AddNonSampledParameters(const std::vector<std::string>&) { return false; }
void Likelihood::SetNonSampledParameters(const VectorReal&) {}
bool Likelihood::PostInitialize() { return true; }

bool Likelihood::EvaluateLogProbabilityBatch(size_t n, const Real* values, Real* logp, int32_t* status)
{
    const size_t d = GetNumVariables();
    VectorReal v(d);
    for (size_t i = 0; i < n; i++) {
        v.assign(values + i * d, values + (i + 1) * d);
        Real lp = -std::numeric_limits<Real>::infinity();
        if (!EvaluateLogProbability(0, v, lp)) return false;
        logp[i] = lp;
        if (status) status[i] = 0;
    }
    return true;
}

bool Likelihood::EvaluateLogProbabilityBatchDevice(size_t, const Real*, Real*, int32_t*, void*) { return false; }

std::string option_get(const OptionsMap& vm, const std::string& key, const std::string& def)
{
    auto it = vm.find(key);
    return it == vm.end() ? def : it->second;
}

std::vector<std::string> LikelihoodFactory::SupportedTypes()
{
    return {"pop_pk_trajectory", "pharmacokinetic_trajectory", "pharmaco_single", "pharmaco_population", "banana", "circular",
            "multimodal_gaussians", "truncated_t", "dummy", "cell_population", "dll"};
}

std::shared_ptr<Likelihood> LikelihoodFactory::CreateLikelihood(const std::string& fn,
                                                                 std::shared_ptr<const VariableSet> varset,
                                                                 const OptionsMap& vm, size_t sampling_threads,
                                                                 size_t evaluation_threads, bool running_inference)
{
    std::shared_ptr<Likelihood> ll;
    std::unique_ptr<XmlNode> root;
    try {
        root = xml_load(fn);
    } catch (XmlError& e) {
        LOGERROR("Error loading likelihood file: %s", e.what.c_str());
        return ll;
    }
    const XmlNode* node = root->child("bcm_likelihood");
    if (!node) {
        LOGERROR("Error parsing likelihood file: No such node (bcm_likelihood)");
        return ll;
    }
    std::string type;
    try {
        type = node->get("type");
    } catch (XmlError& e) {
        LOGERROR("Error parsing likelihood file: %s", e.what.c_str());
        return ll;
    }
    OptionsMap opts = vm;
    if (!opts.count("likelihood_dir")) {
        size_t slash = fn.find_last_of('/');
        opts["likelihood_dir"] = (slash == std::string::npos) ? "." : fn.substr(0, slash);
    }
    if (type == "pop_pk_trajectory") {
        ll = std::make_shared<LikelihoodPopPKTrajectory>(sampling_threads, evaluation_threads);
    } else if (type == "pharmacokinetic_trajectory") {
        ll = std::make_shared<LikelihoodPharmacokineticTrajectory>(sampling_threads, evaluation_threads);
    } else if (type == "pharmaco_single") {
        ll = std::make_shared<PharmacoLikelihoodSingle>(sampling_threads, evaluation_threads);
    } else if (type == "pharmaco_population") {
        ll = std::make_shared<PharmacoLikelihoodPopulation>(sampling_threads, evaluation_threads);
    } else if (type == "banana") {
        ll = std::make_shared<TestLikelihoodBanana>(sampling_threads, evaluation_threads);
    } else if (type == "circular") {
        ll = std::make_shared<TestLikelihoodCircular>(sampling_threads, evaluation_threads);
    } else if (type == "multimodal_gaussians") {
        ll = std::make_shared<TestLikelihoodMultimodalGaussians>(sampling_threads, evaluation_threads);
    } else if (type == "truncated_t") {
        ll = std::make_shared<TestLikelihoodTruncatedT>(sampling_threads, evaluation_threads);
    } else if (type == "dummy") {
        ll = std::make_shared<LikelihoodDummy>(sampling_threads, evaluation_threads);
    } else if (type == "cell_population") {
        ll = std::make_shared<LikelihoodCellPopulation>(sampling_threads, evaluation_threads);
    } else if (type == "dll") {
        ll = std::make_shared<LikelihoodDLL>(sampling_threads, evaluation_threads);
    } else {
        LOGERROR("Unknown likelihood type \"%s\" (supported on this backend: pop_pk_trajectory, pharmacokinetic_trajectory, pharmaco_single, pharmaco_population, banana, circular, multimodal_gaussians, truncated_t, dummy, cell_population, dll)",
                 type.c_str());
        return ll;
    }
    if (!ll->Initialize(varset, *node, opts)) ll.reset();
    return ll;
}

}  // namespace bcm3
