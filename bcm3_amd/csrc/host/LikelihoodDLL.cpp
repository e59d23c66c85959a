// LikelihoodDLL.cpp -- see LikelihoodDLL.h.
#include "LikelihoodDLL.h"

#include <dlfcn.h>

#include <atomic>
#include <cmath>
#include <limits>
#include <thread>

#include "../../../include/bcm3hip.h"
#include "log.h"

namespace bcm3 {

LikelihoodDLL::LikelihoodDLL(size_t sampling_threads, size_t)
    : threads(sampling_threads > 0 ? sampling_threads : 1)
{
}

LikelihoodDLL::~LikelihoodDLL()
{
    if (handle) dlclose(handle);
}

// LikelihoodDLL::Initialize (LikelihoodDLL.cpp:34-88): dll_filename_base [+ include_build_dir,
// default true: "build/" prefix], ".so" appended, dlopen(RTLD_NOW), the two unmangled symbols
bool LikelihoodDLL::Initialize(std::shared_ptr<const VariableSet> vs, const XmlNode& node, const OptionsMap& vm)
{
    varset = vs;
    names = vs->GetVariableNames();
    name_ptrs.clear();
    for (auto& s : names) name_ptrs.push_back(s.c_str());
    std::string fn;
    bool include_build_dir = true;
    try {
        fn = node.get("dll_filename_base");
        include_build_dir = node.get_bool("include_build_dir", true);
    } catch (XmlError& e) {
        LOGERROR("Error parsing likelihood file: %s", e.what.c_str());
        return false;
    }
    fn += ".so";
    if (include_build_dir) fn = "build/" + fn;
    handle = dlopen(fn.c_str(), RTLD_NOW);
    if (!handle) {
        LOGERROR("Can't find dll for likelihood function \"%s\".", fn.c_str());
        return false;
    }
    initialize = (initialize_fn)dlsym(handle, "initialize_likelihood");
    likelihood = (likelihood_fn)dlsym(handle, "evaluate_log_probability");
    if (!likelihood) {
        LOGERROR("Unable to find evaluate_log_probability function in dll \"%s\".", fn.c_str());
        return false;
    }
    if (threads < 2) threads = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    return true;
}

bool LikelihoodDLL::PostInitialize()
{
    if (initialize && !initialize(names.size(), name_ptrs.data())) {
        LOGERROR("DLL initialize function returning false; halting inference.");
        return false;
    }
    return true;
}

// LikelihoodDLL::EvaluateLogProbability (.cpp:101-116): false or NaN -> error
bool LikelihoodDLL::EvaluateLogProbability(size_t, const VectorReal& values, Real& logp)
{
    double lp = std::numeric_limits<double>::quiet_NaN();
    if (!likelihood(names.size(), values.data(), name_ptrs.data(), &lp)) return false;
    logp = lp;
    return !std::isnan(logp);
}

bool LikelihoodDLL::EvaluateLogProbabilityBatch(size_t n, const Real* values, Real* logp, int32_t* status)
{
    const size_t d = names.size();
    std::atomic<bool> ok{true};
    auto work = [&](size_t t, size_t nt) {
        for (size_t i = t; i < n; i += nt) {
            double lp = std::numeric_limits<double>::quiet_NaN();
            if (!likelihood(d, values + i * d, name_ptrs.data(), &lp) || std::isnan(lp)) ok = false;
            logp[i] = lp;
            if (status) status[i] = 0;
        }
    };
    const size_t nt = std::max<size_t>(1, std::min(threads, n));
    std::vector<std::thread> th;
    for (size_t t = 1; t < nt; t++) th.emplace_back(work, t, nt);
    work(0, nt);
    for (auto& x : th) x.join();
    return ok;
}

bool LikelihoodDLL::EvaluateLogProbabilityBatchDevice(size_t n, const Real* values_dev, Real* logp_dev,
                                                      int32_t* status_dev, void* stream)
{
    const size_t d = names.size();
    std::vector<Real> v(n * d), lp(n);
    std::vector<int32_t> st(n, 0);
    if (bcm3hip_memcpy_async(v.data(), values_dev, v.size() * sizeof(Real), BCM3HIP_D2H, stream) != 0 ||
        bcm3hip_stream_synchronize(stream) != 0)
        return false;
    const bool ok = EvaluateLogProbabilityBatch(n, v.data(), lp.data(), st.data());
    if (bcm3hip_memcpy_async(logp_dev, lp.data(), n * sizeof(Real), BCM3HIP_H2D, stream) != 0) return false;
    if (status_dev && bcm3hip_memcpy_async(status_dev, st.data(), n * sizeof(int32_t), BCM3HIP_H2D, stream) != 0)
        return false;
    return bcm3hip_stream_synchronize(stream) == 0 && ok;
}

}  // namespace bcm3
