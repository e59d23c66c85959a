// bcm3_dll.cpp -- include/bcm3_dll.h: the reference's LikelihoodDLL plugin ABI on top of
// include/bcm3.h (see the header for the contract).
#include "../../../include/bcm3_dll.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "../../../include/bcm3.h"

namespace {
std::mutex g_mutex;
bcm3_likelihood* g_ll = nullptr;
size_t g_d = 0;
}  // namespace

extern "C" {

bool initialize_likelihood(size_t num_variables, const char* const* variable_names)
{
    std::lock_guard<std::mutex> lock(g_mutex);
    const char* lik = std::getenv("BCM3_LIKELIHOOD_XML");
    const char* prior = std::getenv("BCM3_PRIOR_XML");
    if (!lik || !prior) {
        std::fprintf(stderr, "bcm3_dll: BCM3_LIKELIHOOD_XML and BCM3_PRIOR_XML must be set\n");
        return false;
    }
    std::string opts = std::getenv("BCM3_OPTIONS") ? std::getenv("BCM3_OPTIONS") : "";
    if (const char* dev = std::getenv("BCM3_DEVICE")) opts += std::string(opts.empty() ? "" : ";") + "device=" + dev;
    if (g_ll) {
        bcm3_likelihood_destroy(g_ll);
        g_ll = nullptr;
    }
    if (bcm3_likelihood_create_ex(lik, prior, opts.c_str(), &g_ll) != 0) {
        std::fprintf(stderr, "bcm3_dll: %s\n", bcm3_last_error());
        return false;
    }
    g_d = (size_t)bcm3_likelihood_num_variables(g_ll);
    if (g_d != num_variables) {
        std::fprintf(stderr, "bcm3_dll: %zu variables given, the prior has %zu\n", num_variables, g_d);
        return false;
    }
    char buf[512];
    for (size_t i = 0; i < num_variables; i++) {
        bcm3_likelihood_variable_name(g_ll, (int)i, buf, sizeof(buf));
        if (!variable_names || !variable_names[i] || std::strcmp(buf, variable_names[i]) != 0) {
            std::fprintf(stderr, "bcm3_dll: variable %zu is '%s' in the prior\n", i, buf);
            return false;
        }
    }
    return true;
}

bool evaluate_log_probability(size_t num_variables, const double* values, const char* const* variable_names,
                              double* log_p)
{
    (void)variable_names;
    if (!g_ll || num_variables != g_d || !values || !log_p) return false;
    return bcm3_likelihood_evaluate(g_ll, 0, values, log_p) == 0;
}

}  // extern "C"
