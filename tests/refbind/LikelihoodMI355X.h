// LikelihoodMI355X.h -- the bcm3::Likelihood subclass a BCM3 maintainer adds to the reference
// (src/likelihoods/) to route a likelihood through this repository's MI355X path
// (include/bcm3.h, libbcm3.so). INTEGRATION.md §2-3 quote this file; tests/test_refbind.py compiles
// it against the reference's plugin interface (src/sampler/Likelihood.h:9-35) and runs it.
#pragma once

#include <cstdint>

#include "Likelihood.h"
#include "bcm3.h"

namespace bcm3 {

class LikelihoodMI355X : public Likelihood {
public:
    // LikelihoodFactory::CreateLikelihood constructs every likelihood with these two counts
    // (src/likelihoods/LikelihoodFactory.cpp:45-86)
    LikelihoodMI355X(size_t sampling_threads, size_t evaluation_threads);
    ~LikelihoodMI355X() override;

    // <bcm_likelihood type="mi355x" config="likelihood_popk.xml" [device="0"] [options="k=v;..."]/>:
    // config names the reference's own pop_pk_trajectory / pharmaco / cell_population / banana /
    // circular XML; the prior is bcminf's --prior (src/bcminf/main.cpp:297)
    bool Initialize(std::shared_ptr<const VariableSet> varset, boost::property_tree::ptree likelihood_node,
                    const boost::program_options::variables_map& vm) override;
    bool IsReentrant() override { return true; }
    bool EvaluateLogProbability(size_t threadix, const VectorReal& values, Real& logp) override;

    // the batched fan-out: n vectors of the sampler's VariableSet, row-major; status[i] = 1 for a
    // solver failure (logp[i] = -inf, a legal zero likelihood)
    bool EvaluateLogProbabilityBatch(size_t n, const Real* values, Real* logp, int32_t* status);

private:
    std::shared_ptr<const VariableSet> varset;
    size_t sampling_threads;
    bcm3_likelihood* h;
};

// SamplerPT::DoMutateMove (src/sampler/SamplerPT.cpp:308-319) queues one task per chain, each
// calling EvaluateLogProbability once. Batched: the chains' proposals in ONE launch, then the
// caller's accept step with llh * learning_rate, as Sampler::EvaluateLikelihood applies it
// (src/sampler/Sampler.cpp:164-180; a NaN is fatal there, so it is here).
bool EvaluateProposalsBatched(LikelihoodMI355X& ll, const std::vector<VectorReal>& proposals, Real learning_rate,
                              std::vector<Real>& llh);

}  // namespace bcm3
