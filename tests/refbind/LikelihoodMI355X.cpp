// LikelihoodMI355X.cpp -- see LikelihoodMI355X.h
#include "Utils.h"
#include "LikelihoodMI355X.h"

#include <cmath>

namespace bcm3 {

LikelihoodMI355X::LikelihoodMI355X(size_t sampling_threads, size_t evaluation_threads)
    : sampling_threads(sampling_threads), h(nullptr)
{
}

LikelihoodMI355X::~LikelihoodMI355X()
{
    if (h) bcm3_likelihood_destroy(h);
}

bool LikelihoodMI355X::Initialize(std::shared_ptr<const VariableSet> varset, boost::property_tree::ptree likelihood_node,
                                  const boost::program_options::variables_map& vm)
{
    this->varset = varset;
    const std::string xml = likelihood_node.get<std::string>("<xmlattr>.config");
    const std::string prior = vm["prior"].as<std::string>();
    std::string options = "device=" + likelihood_node.get<std::string>("<xmlattr>.device", "0");
    const std::string extra = likelihood_node.get<std::string>("<xmlattr>.options", "");
    if (!extra.empty()) options += ";" + extra;
    if (bcm3_likelihood_create_ex(xml.c_str(), prior.c_str(), options.c_str(), &h) != 0) {
        LOGERROR("bcm3_likelihood_create_ex(%s): %s", xml.c_str(), bcm3_last_error());
        return false;
    }
    // the wrapped likelihood must see the sampler's variables, in the sampler's order
    const int d = bcm3_likelihood_num_variables(h);
    if (d < 0 || (size_t)d != varset->GetNumVariables()) {
        LOGERROR("mi355x likelihood: %d variables, the sampler has %zu", d, varset->GetNumVariables());
        return false;
    }
    char name[256];
    for (int i = 0; i < d; i++) {
        if (bcm3_likelihood_variable_name(h, i, name, sizeof(name)) < 0 || varset->GetVariableName(i) != name) {
            LOGERROR("mi355x likelihood: variable %d is \"%s\", the sampler's is \"%s\"", i, name,
                     varset->GetVariableName(i).c_str());
            return false;
        }
    }
    return true;
}

bool LikelihoodMI355X::EvaluateLogProbability(size_t threadix, const VectorReal& values, Real& logp)
{
    if ((size_t)values.size() != varset->GetNumVariables() || threadix >= sampling_threads) return false;
    return bcm3_likelihood_evaluate(h, threadix, values.data(), &logp) == 0;
}

bool LikelihoodMI355X::EvaluateLogProbabilityBatch(size_t n, const Real* values, Real* logp, int32_t* status)
{
    return bcm3_likelihood_evaluate_batch(h, n, values, logp, status) == 0;
}

bool EvaluateProposalsBatched(LikelihoodMI355X& ll, const std::vector<VectorReal>& proposals, Real learning_rate,
                              std::vector<Real>& llh)
{
    const size_t n = proposals.size();
    const size_t d = n ? (size_t)proposals[0].size() : 0;
    std::vector<Real> values(n * d), logp(n);
    std::vector<int32_t> status(n);
    for (size_t c = 0; c < n; c++) Eigen::Map<VectorReal>(&values[c * d], d) = proposals[c];
    if (!ll.EvaluateLogProbabilityBatch(n, values.data(), logp.data(), status.data())) return false;
    llh.resize(n);
    for (size_t c = 0; c < n; c++) {
        llh[c] = logp[c] * learning_rate;
        if (std::isnan(llh[c])) {
            LOGERROR("Likelihood evaluation returned NaN");
            return false;
        }
    }
    return true;
}

}  // namespace bcm3
