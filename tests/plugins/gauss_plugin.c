/* gauss_plugin.c -- TEST FIXTURE: a LikelihoodDLL plugin in the reference's template form
 * (examples/dll_likelihood/code.cpp: initialize_likelihood / evaluate_log_probability, here with
 * extern "C"-compatible C linkage) for tests/test_dll_route.py: an isotropic Gaussian
 * log-density sum_i -0.5 (x_i - i)^2 / 4 over the variables; initialize checks the names. */
#include <math.h>
#include <stdbool.h>
#include <stddef.h>
#include <string.h>

static size_t g_n = 0;

bool initialize_likelihood(size_t num_variables, const char* const* variable_names)
{
    g_n = num_variables;
    return num_variables > 0 && variable_names && variable_names[0] && strlen(variable_names[0]) > 0;
}

bool evaluate_log_probability(size_t num_variables, const double* values, const char* const* variable_names,
                              double* log_p)
{
    (void)variable_names;
    if (num_variables != g_n) return false;
    double s = 0.0;
    for (size_t i = 0; i < num_variables; i++) {
        const double z = values[i] - (double)i;
        s += -0.5 * z * z / 4.0;
    }
    *log_p = (values[0] > 1e6) ? NAN : s;
    return true;
}
