// capi.cpp -- include/bcm3.h on top of the C++ host layer.
#include <algorithm>
#include <cstring>
#include <memory>

#include "../../../include/bcm3.h"
#include "../../../include/bcm3hip.h"
#include "Likelihood.h"
#include "LikelihoodGPU.h"
#include "NetCDFClassic.h"
#include "Prior.h"
#include "log.h"

#include "capi_internal.h"
#include "LikelihoodCellPopulation.h"

extern "C" {

static int create(const char* likelihood_xml, const char* prior_xml, const bcm3::OptionsMap& vm,
                  bcm3_likelihood** out)
{
    if (!likelihood_xml || !prior_xml || !out) return -1;
    *out = nullptr;
    auto h = std::make_unique<bcm3_likelihood>();
    h->varset = std::make_shared<bcm3::VariableSet>();
    if (!h->varset->LoadFromXML(prior_xml)) return -2;
    h->ll = bcm3::LikelihoodFactory::CreateLikelihood(likelihood_xml, h->varset, vm, 1, 1, true);
    if (!h->ll) return -3;
    if (!h->ll->PostInitialize()) return -4;
    *out = h.release();
    return 0;
}

int bcm3_likelihood_create(const char* likelihood_xml, const char* prior_xml, int device, bcm3_likelihood** out)
{
    bcm3::OptionsMap vm;
    if (device >= 0) vm["device"] = std::to_string(device);
    return create(likelihood_xml, prior_xml, vm, out);
}

int bcm3_likelihood_create_ex(const char* likelihood_xml, const char* prior_xml, const char* options,
                              bcm3_likelihood** out)
{
    bcm3::OptionsMap vm;
    std::string s = options ? options : "";
    size_t p = 0;
    while (p < s.size()) {
        size_t e = s.find(';', p);
        if (e == std::string::npos) e = s.size();
        std::string kv = s.substr(p, e - p);
        size_t eq = kv.find('=');
        if (eq != std::string::npos) vm[kv.substr(0, eq)] = kv.substr(eq + 1);
        p = e + 1;
    }
    return create(likelihood_xml, prior_xml, vm, out);
}

int bcm3_likelihood_generated_code(const bcm3_likelihood* h, char* buf, size_t buflen)
{
    if (!h || !h->ll) return -1;
    auto* p = dynamic_cast<bcm3::LikelihoodCellPopulation*>(h->ll.get());
    if (!p) return -2;
    const std::string& code = p->GetGeneratedCode();
    if (buf && buflen) {
        const size_t n = std::min(buflen - 1, code.size());
        memcpy(buf, code.data(), n);
        buf[n] = '\0';
    }
    return (int)code.size();
}

int bcm3_sobol_points(size_t points, size_t dims, double* out)
{
    const std::vector<double> v = bcm3::SobolPoints(points, dims);
    std::copy(v.begin(), v.end(), out);
    return 0;
}

int bcm3_likelihood_cellpop_precompile(const bcm3_likelihood* h)
{
    if (!h || !h->ll) return -1;
    auto* p = dynamic_cast<bcm3::LikelihoodCellPopulation*>(h->ll.get());
    if (!p) return -2;
    for (const bcm3hip_cellpop_model* m : p->GetDeviceModels()) {
        const int r = bcm3hip_cellpop_precompile(m);
        if (r) return r;
    }
    return 0;
}

int bcm3_likelihood_cellpop_cells(bcm3_likelihood* h, size_t item, int32_t* count, void* records, double* values,
                                  double* end_y)
{
    if (!h || !h->ll) return -1;
    auto* p = dynamic_cast<bcm3::LikelihoodCellPopulation*>(h->ll.get());
    if (!p || !p->Context()) return -2;
    return bcm3hip_cellpop_cells(p->Context(), item, count, (bcm3hip_cell_record*)records, values, end_y);
}

int bcm3_likelihood_popk_model(const bcm3_likelihood* h, void* model)
{
    if (!h || !model) return -1;
    if (auto* p = dynamic_cast<bcm3::LikelihoodPopPKTrajectory*>(h->ll.get())) {
        *(bcm3hip_popk_model*)model = p->GetDeviceModel();
        return 0;
    }
    if (auto* p = dynamic_cast<bcm3::LikelihoodPharmacokineticTrajectory*>(h->ll.get())) {
        *(bcm3hip_popk_model*)model = p->GetDeviceModel();
        return 0;
    }
    return -2;
}

int bcm3_likelihood_expm_pk_model(const bcm3_likelihood* h, void* model)
{
    if (!h || !model) return -1;
    if (auto* p = dynamic_cast<bcm3::PharmacoLikelihoodSingle*>(h->ll.get())) {
        *(bcm3hip_expm_pk_model*)model = p->GetDeviceModel();
        return 0;
    }
    if (auto* p = dynamic_cast<bcm3::PharmacoLikelihoodPopulation*>(h->ll.get())) {
        *(bcm3hip_expm_pk_model*)model = p->GetDeviceModel();
        return 0;
    }
    return -2;
}

void bcm3_likelihood_destroy(bcm3_likelihood* h) { delete h; }

int bcm3_prior_marginals(const char* prior_xml, int max_vars, int32_t* kind, double* params /*[max][3]*/,
                         double* bounds /*[max][2]*/, double* moments /*[max][2]*/)
{
    if (!prior_xml) return -1;
    std::vector<bcm3::Marginal> m;
    if (!bcm3::LoadPriorMarginals(prior_xml, m)) return -2;
    const int d = (int)m.size();
    for (int i = 0; i < d && i < max_vars; i++) {
        if (kind) kind[i] = m[i].kind;
        if (params) {
            params[3 * i] = m[i].p0;
            params[3 * i + 1] = m[i].p1;
            params[3 * i + 2] = m[i].p2;
        }
        if (bounds) {
            bounds[2 * i] = m[i].lower;
            bounds[2 * i + 1] = m[i].upper;
        }
        if (moments) {
            moments[2 * i] = m[i].mean;
            moments[2 * i + 1] = m[i].var;
        }
    }
    return d;
}

int bcm3_likelihood_num_variables(const bcm3_likelihood* h) { return h ? (int)h->varset->GetNumVariables() : -1; }

int bcm3_likelihood_variable_name(const bcm3_likelihood* h, int i, char* buf, size_t buflen)
{
    if (!h || i < 0 || (size_t)i >= h->varset->GetNumVariables()) return -1;
    const std::string& n = h->varset->GetVariableName((size_t)i);
    if (buf && buflen) {
        std::strncpy(buf, n.c_str(), buflen - 1);
        buf[buflen - 1] = 0;
    }
    return (int)n.size();
}

int bcm3_likelihood_variable_transform(const bcm3_likelihood* h, int i)
{
    if (!h || i < 0 || (size_t)i >= h->varset->GetNumVariables()) return -1;
    return (int)h->varset->GetVariableTransform((size_t)i);
}

int bcm3_likelihood_set_learning_rate(bcm3_likelihood* h, double lr)
{
    return (h && h->ll->SetLearningRate(lr)) ? 0 : -1;
}

int bcm3_likelihood_evaluate(bcm3_likelihood* h, size_t threadix, const double* values, double* logp)
{
    if (!h || !values || !logp) return -1;
    bcm3::VectorReal v(values, values + h->varset->GetNumVariables());
    return h->ll->EvaluateLogProbability(threadix, v, *logp) ? 0 : -2;
}

int bcm3_likelihood_evaluate_batch(bcm3_likelihood* h, size_t n, const double* values, double* logp, int32_t* status)
{
    if (!h || (n && (!values || !logp))) return -1;
    return h->ll->EvaluateLogProbabilityBatch(n, values, logp, status) ? 0 : -2;
}

int bcm3_likelihood_evaluate_batch_device(bcm3_likelihood* h, size_t n, const double* values_dev, double* logp_dev,
                                          int32_t* status_dev, void* stream)
{
    if (!h) return -1;
    return h->ll->EvaluateLogProbabilityBatchDevice(n, values_dev, logp_dev, status_dev, stream) ? 0 : -2;
}

int bcm3_likelihood_last_kernel_ms(bcm3_likelihood* h, float* ms)
{
    if (!h || !ms) return -1;
    *ms = h->ll->LastKernelMilliseconds();
    return *ms < 0 ? -2 : 0;
}

int bcm3_likelihood_kernel_time_log(bcm3_likelihood* h, double* total_ms, int64_t* launches, double* max_ms)
{
    if (!h || !total_ms || !launches) return -1;
    double mx = 0.0;
    if (!h->ll->KernelTimeLog(*total_ms, *launches, mx)) return -2;
    if (max_ms) *max_ms = mx;
    return 0;
}

int bcm3_likelihood_set_option(bcm3_likelihood* h, int option, int64_t value)
{
    return (h && h->ll->SetBackendOption(option, value)) ? 0 : -1;
}

const char* bcm3_last_error(void) { return bcm3::log_last_error(); }

int64_t bcm3_data_file_json(const char* filename, char* out, int64_t cap)
{
    if (!filename) return -1;
    std::string text;
    try {
        bcm3::Json doc = bcm3::NcIsClassic(filename) ? bcm3::NcClassicRead(filename) : bcm3::LoadDataFile(filename);
        text = bcm3::json_dump(doc);
    } catch (bcm3::JsonError& e) {
        LOGERROR("%s: %s", filename, e.what.c_str());
        return -2;
    }
    if (out && cap > 0) {
        const size_t n = std::min<size_t>((size_t)cap - 1, text.size());
        std::memcpy(out, text.data(), n);
        out[n] = '\0';
    }
    return (int64_t)text.size();
}

}  // extern "C"
