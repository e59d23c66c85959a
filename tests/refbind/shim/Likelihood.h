// Test infrastructure: the plugin interface bcm3::Likelihood with the virtual functions, argument
// types and access of the reference's src/sampler/Likelihood.h:9-35 (bodies as Likelihood.cpp:6-40),
// so that tests/refbind/LikelihoodMI355X.{h,cpp} -- the subclass INTEGRATION.md §2 tells a
// maintainer to add -- is compiled and run against that exact interface.
#pragma once

#include "VariableSet.h"

namespace bcm3 {

class Likelihood {
public:
    virtual ~Likelihood() {}

    bool SetLearningRate(Real lr)
    {
        if (lr < 0.0 || lr > 1.0) {
            LOGERROR("Learning rate must be >= 0 and <= 1.0");
            return false;
        }
        learning_rate = lr;
        return true;
    }
    inline Real GetLearningRate() const { return learning_rate; }

    virtual bool Initialize(std::shared_ptr<const VariableSet> varset, boost::property_tree::ptree likelihood_node,
                            const boost::program_options::variables_map& vm)
    {
        return true;
    }
    virtual bool AddNonSampledParameters(const std::vector<std::string>& variable_names) { return true; }
    virtual void SetNonSampledParameters(const VectorReal& values) {}
    virtual bool PostInitialize() { return true; }
    virtual bool IsReentrant() = 0;
    virtual void OutputEvaluationStatistics(const std::string& path) const {}
    virtual bool EvaluateLogProbability(size_t threadix, const VectorReal& values, Real& logp) = 0;

protected:
    Likelihood() : learning_rate(1.0) {}

    Real learning_rate;
};

}  // namespace bcm3
