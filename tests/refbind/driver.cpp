// Test infrastructure: bcminf's wiring of a likelihood (src/bcminf/main.cpp:47-58, 83-121) around
// the maintainer's LikelihoodMI355X, compiled against the reference-interface shim:
// LikelihoodFactory's branch for type="mi355x" (src/likelihoods/LikelihoodFactory.cpp:45-86),
// Initialize / PostInitialize / SetLearningRate, then either one EvaluateLogProbability per vector
// from `threads` sampling threads with their threadix (TaskManager's fan-out), or the batched fan-out
// EvaluateProposalsBatched.
//
//   refbind_driver <config.xml> <prior.xml> <options> <single|batch> <threads> <draws.f64> <n> <out.f64>
//
// draws.f64: n*d doubles (row-major); out.f64: n doubles of llh. Exit 0 on success.
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <thread>

#include "LikelihoodMI355X.h"

namespace bcm3 {

// LikelihoodFactory::CreateLikelihood's type dispatch (src/likelihoods/LikelihoodFactory.cpp:45-86)
// with the one branch INTEGRATION.md §2 adds
std::shared_ptr<Likelihood> CreateLikelihood(const boost::property_tree::ptree& likelihood_node, size_t sampling_threads,
                                             size_t evaluation_threads)
{
    std::shared_ptr<Likelihood> ll;
    const std::string type = likelihood_node.get<std::string>("<xmlattr>.type");
    if (type == "dll") {
        LOGERROR("type=\"dll\" is not part of this test");
    } else if (type == "mi355x") {
        ll = std::make_shared<LikelihoodMI355X>(sampling_threads, evaluation_threads);
    }
    return ll;
}

}  // namespace bcm3

int main(int argc, char** argv)
{
    if (argc != 9) {
        std::fprintf(stderr, "usage: %s config.xml prior.xml options single|batch threads draws n out\n", argv[0]);
        return 2;
    }
    const std::string cfg = argv[1], prior = argv[2], opts = argv[3], mode = argv[4];
    const size_t threads = (size_t)std::atoi(argv[5]), n = (size_t)std::atoll(argv[7]);

    // the VariableSet bcminf loads from prior.xml: names read through the library without a device
    bcm3_likelihood* names = nullptr;
    if (bcm3_likelihood_create_ex(cfg.c_str(), prior.c_str(), "backend=none", &names) != 0) {
        std::fprintf(stderr, "prior: %s\n", bcm3_last_error());
        return 1;
    }
    auto varset = std::make_shared<bcm3::VariableSet>();
    char buf[256];
    for (int i = 0; i < bcm3_likelihood_num_variables(names); i++) {
        bcm3_likelihood_variable_name(names, i, buf, sizeof(buf));
        varset->AddVariable(buf);
    }
    bcm3_likelihood_destroy(names);
    const size_t d = varset->GetNumVariables();

    boost::property_tree::ptree node;
    node.data["<xmlattr>.type"] = "mi355x";
    node.data["<xmlattr>.config"] = cfg;
    if (!opts.empty() && opts != "-") node.data["<xmlattr>.options"] = opts;
    boost::program_options::variables_map vm;
    vm.values["prior"].text = prior;

    std::shared_ptr<bcm3::Likelihood> ll = bcm3::CreateLikelihood(node, threads, 1);
    if (!ll || !ll->Initialize(varset, node, vm) || !ll->PostInitialize() || !ll->SetLearningRate(1.0)) return 1;

    std::vector<double> x(n * d), out(n);
    std::ifstream in(argv[6], std::ios::binary);
    if (!in.read((char*)x.data(), (std::streamsize)(x.size() * sizeof(double)))) {
        std::fprintf(stderr, "cannot read %zu x %zu draws\n", n, d);
        return 1;
    }
    bool ok = true;
    if (mode == "batch") {
        std::vector<bcm3::VectorReal> proposals(n);
        for (size_t i = 0; i < n; i++) proposals[i] = Eigen::Map<const bcm3::VectorReal>(&x[i * d], d);
        std::vector<bcm3::Real> llh;
        ok = bcm3::EvaluateProposalsBatched(*std::static_pointer_cast<bcm3::LikelihoodMI355X>(ll), proposals,
                                            ll->GetLearningRate(), llh);
        if (ok) out = llh;
    } else {
        std::vector<std::thread> pool;
        std::vector<int> good(threads, 1);
        for (size_t t = 0; t < threads; t++)
            pool.emplace_back([&, t] {
                for (size_t i = t; i < n; i += threads) {
                    bcm3::VectorReal v = Eigen::Map<const bcm3::VectorReal>(&x[i * d], d);
                    bcm3::Real lp;
                    if (!ll->EvaluateLogProbability(t, v, lp)) {
                        good[t] = 0;
                        return;
                    }
                    out[i] = lp * ll->GetLearningRate();
                }
            });
        for (auto& th : pool) th.join();
        for (int g : good) ok &= g != 0;
    }
    if (!ok) {
        std::fprintf(stderr, "evaluation failed: %s\n", bcm3_last_error());
        return 1;
    }
    std::ofstream o(argv[8], std::ios::binary);
    o.write((const char*)out.data(), (std::streamsize)(out.size() * sizeof(double)));
    return o ? 0 : 1;
}
