/*
 * bcm3_dll.h -- the reference's own C plugin ABI for likelihoods, served by libbcm3_dll.so.
 *
 * LikelihoodDLL (src/likelihoods/LikelihoodDLL.cpp:34-116, template examples/dll_likelihood/
 * code.cpp:1-13) dlopen()s "build/<dll_filename_base>.so" and dlsym()s these two unmangled
 * symbols. Pointing a reference likelihood.xml at this library
 *     <bcm_likelihood type="dll" dll_filename_base="libbcm3_dll"/>
 * (with the .so copied or linked into the run's build/ directory) evaluates the likelihood
 * described by $BCM3_LIKELIHOOD_XML / $BCM3_PRIOR_XML on the MI355X, one vector per call.
 * Environment: BCM3_LIKELIHOOD_XML, BCM3_PRIOR_XML (required), BCM3_DEVICE (default 0),
 * BCM3_OPTIONS ("key=value;..." as for bcm3_likelihood_create_ex).
 * The ABI is single-vector by design (no batching); the fast path is include/bcm3.h.
 * Re-entrant: concurrent calls from the reference's sampling threads are serialised per GPU.
 */
#ifndef BCM3_DLL_H
#define BCM3_DLL_H
#include <stdbool.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* LikelihoodDLL::PostInitialize (LikelihoodDLL.cpp:90-99): variable names in prior.xml order;
 * fails if they differ from $BCM3_PRIOR_XML's. */
bool initialize_likelihood(size_t num_variables, const char* const* variable_names);
/* LikelihoodDLL::EvaluateLogProbability (LikelihoodDLL.cpp:101-116). */
bool evaluate_log_probability(size_t num_variables, const double* values, const char* const* variable_names,
                              double* log_p);

#ifdef __cplusplus
}
#endif
#endif
