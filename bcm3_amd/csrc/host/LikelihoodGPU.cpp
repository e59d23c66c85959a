// LikelihoodGPU.cpp -- see LikelihoodGPU.h
#include "LikelihoodGPU.h"

#include <cmath>
#include <cstdlib>
#include <fstream>
#include <limits>

#include "json.h"
#include "log.h"

namespace bcm3 {

static const Real NaN = std::numeric_limits<Real>::quiet_NaN();

// ---------------------------------------------------------------------------------------------
LikelihoodGPUBase::~LikelihoodGPUBase()
{
    if (ctx) bcm3hip_close(ctx);
}

bool LikelihoodGPUBase::OpenDevice(const OptionsMap& vm)
{
    if (option_get(vm, "backend", "") == "none") return true;  // host-logic only (tests)
    std::string dev = option_get(vm, "device", "");
    if (dev.empty()) {
        const char* e = getenv("BCM3_DEVICE");
        dev = e ? e : "0";
    }
    device = std::atoi(dev.c_str());
    int count = bcm3hip_device_count();
    if (count <= 0) {
        LOGERROR("No MI355X/HIP device available (this backend has no CPU fallback)");
        return false;
    }
    return true;
}

bool LikelihoodGPUBase::EvaluateLogProbability(size_t threadix, const VectorReal& values, Real& logp)
{
    int32_t st = 0;
    return EvaluateLogProbabilityBatch(1, values.data(), &logp, &st);
}

bool LikelihoodGPUBase::EvaluateLogProbabilityBatch(size_t n, const Real* values, Real* logp, int32_t* status)
{
    if (!CheckEvaluable()) return false;
    if (!ctx) {
        LOGERROR("No GPU context (backend=none)");
        return false;
    }
    std::lock_guard<std::mutex> lock(mutex);
    int r = bcm3hip_eval_batch(ctx, n, GetNumVariables(), values, logp, status);
    if (r != 0) {
        LOGERROR("GPU likelihood evaluation failed: %s", bcm3hip_error_string(r));
        return false;
    }
    return true;
}

bool LikelihoodGPUBase::EvaluateLogProbabilityBatchDevice(size_t n, const Real* values_dev, Real* logp_dev,
                                                          int32_t* status_dev, void* stream)
{
    if (!CheckEvaluable()) return false;
    if (!ctx) {
        LOGERROR("No GPU context (backend=none)");
        return false;
    }
    std::lock_guard<std::mutex> lock(mutex);
    int r = bcm3hip_eval_batch_device(ctx, n, values_dev, logp_dev, status_dev, stream);
    if (r != 0) {
        LOGERROR("GPU likelihood evaluation failed: %s", bcm3hip_error_string(r));
        return false;
    }
    return true;
}

float LikelihoodGPUBase::LastKernelMilliseconds()
{
    float ms = -1.0f;
    if (bcm3hip_last_kernel_ms(ctx, &ms) != 0) return -1.0f;
    return ms;
}

bool LikelihoodGPUBase::KernelTimeLog(double& total_ms, int64_t& launches, double& max_ms)
{
    std::lock_guard<std::mutex> lock(mutex);
    return ctx && bcm3hip_kernel_time_log(ctx, &total_ms, &launches, &max_ms) == 0;
}

bool LikelihoodGPUBase::SetBackendOption(int option, int64_t value) { return bcm3hip_set_option(ctx, option, value) == 0; }

// ---------------------------------------------------------------------------------------------
// LikelihoodPopPKTrajectory

LikelihoodPopPKTrajectory::LikelihoodPopPKTrajectory(size_t sampling_threads, size_t)
    : sampling_threads(sampling_threads), fixed_vod(NaN), fixed_periphery_fwd(NaN), fixed_periphery_bwd(NaN), MW(NaN)
{
}

static bool file_exists(const std::string& p)
{
    std::ifstream f(p);
    return (bool)f;
}

// LikelihoodPopPKTrajectory::Initialize (LikelihoodPopPKTrajectory.cpp:50-252)
bool LikelihoodPopPKTrajectory::Initialize(std::shared_ptr<const VariableSet> vs, const XmlNode& likelihood_node,
                                           const OptionsMap& vm)
{
    bool result = true;
    varset = vs;
    std::string trial, pkdata_file, pk_type_str;
    try {
        const XmlNode* modelnode = likelihood_node.child("pk_model");
        if (!modelnode) throw XmlError{"No such node (pk_model)"};
        drug = modelnode->get("drug");
        pk_type_str = modelnode->get("type");
        trial = modelnode->get("trial");
        pkdata_file = modelnode->get("pkdata_file");
        fixed_vod = modelnode->get_double("volume_of_distribution", NaN);
        fixed_periphery_fwd = modelnode->get_double("k_periphery_fwd", NaN);
        fixed_periphery_bwd = modelnode->get_double("k_periphery_bwd", NaN);
    } catch (XmlError& e) {
        LOGERROR("Error parsing likelihood file: %s", e.what.c_str());
        return false;
    }
    if (pk_type_str == "one") pk_type = PKMT_OneCompartment;
    else if (pk_type_str == "two") pk_type = PKMT_TwoCompartment;
    else if (pk_type_str == "one_biphasic_uptake") pk_type = PKMT_TwoCompartmentBiphasicUptake;  // as the reference
    else if (pk_type_str == "two_biphasic_uptake") pk_type = PKMT_TwoCompartmentBiphasicUptake;
    else if (pk_type_str == "one_transit") pk_type = PKMT_OneCompartmentTransit;
    else if (pk_type_str == "two_transit") pk_type = PKMT_TwoCompartmentTransit;
    else pk_type = PKMT_Undefined;

    // data file: relative paths are tried against the working directory, then the likelihood
    // file's directory
    std::string path = pkdata_file;
    if (!file_exists(path)) {
        std::string alt = option_get(vm, "likelihood_dir", ".") + "/" + pkdata_file;
        if (file_exists(alt)) path = alt;
    }
    Json data;
    try {
        data = json_load(path);
    } catch (JsonError& e) {
        LOGERROR("Failed to open data file %s: %s", pkdata_file.c_str(), e.what.c_str());
        return false;
    }
    const Json* g = data.find(trial);
    if (!g) {
        LOGERROR("Group \"%s\" not found in %s", trial.c_str(), path.c_str());
        return false;
    }
    auto var = [&](const std::string& name) -> const Json* {
        const Json* v = g->find(name);
        if (!v) {
            LOGERROR("Variable \"%s\" not found in group \"%s\"", name.c_str(), trial.c_str());
            result = false;
        }
        return v;
    };
    const Json* jt = var("time");
    const Json* jp = var("patients");
    if (!jt || !jp) return false;
    const size_t num_timepoints = jt->arr.size(), num_patients = jp->arr.size();
    for (auto& p : jp->arr) patient_ids.push_back(p.type == Json::String ? p.str : std::to_string((long)p.num));

    switch (pk_type) {
    case PKMT_OneCompartment: num_pk_params = 4; break;
    case PKMT_TwoCompartment: num_pk_params = 6; break;
    case PKMT_OneCompartmentBiphasicUptake: num_pk_params = 7; break;
    case PKMT_TwoCompartmentBiphasicUptake: num_pk_params = 7; break;
    case PKMT_OneCompartmentTransit: num_pk_params = 6; break;
    case PKMT_TwoCompartmentTransit: num_pk_params = 8; break;
    default: LOGERROR("Invalid PK model type"); return false;
    }
    num_pk_pop_params = 2;

    size_t fixed_var_count = 0;
    if (!std::isnan(fixed_vod)) fixed_var_count++;
    if (!std::isnan(fixed_periphery_fwd)) fixed_var_count++;
    if (!std::isnan(fixed_periphery_bwd)) fixed_var_count++;
    if (varset->GetNumVariables() != num_pk_params - fixed_var_count + num_pk_pop_params * (num_patients + 1) + 2) {
        LOGERROR("Incorrect number of variables in prior");
        return false;
    }

    time.resize(num_timepoints);
    for (size_t i = 0; i < num_timepoints; i++) time[i] = jt->arr[i].as_double();

    const Json* jc = var(drug + "_plasma_concentration");
    const Json* jd = var(drug + "_dose");
    const Json* jda = var(drug + "_dose_after_dose_change");
    const Json* jdt = var(drug + "_dose_change_time");
    const Json* jdi = var(drug + "_dosing_interval");
    const Json* jin = var(drug + "_intermittent");
    const Json* jti = var("treatment_interruptions");
    if (!result) return false;

    const size_t P = num_patients, T = num_timepoints;
    observed.assign(P * T, NaN);
    dose.resize(P);
    dose_after_dose_change.resize(P);
    dose_change_time.resize(P);
    dosing_interval.resize(P);
    intermittent.assign(P, 0);
    skipped_days.assign(P * 29, 0);
    simulate_until.assign(P, 0);
    Real minimum_dose = std::numeric_limits<Real>::max();
    try {
        for (size_t j = 0; j < P; j++) {
            for (size_t i = 0; i < T; i++) observed[j * T + i] = jc->arr.at(j).arr.at(i).as_double();
            dose[j] = jd->arr.at(j).as_double();
            dose_after_dose_change[j] = jda->arr.at(j).as_double();
            dose_change_time[j] = jdt->arr.at(j).as_double();
            dosing_interval[j] = jdi->arr.at(j).as_double();
            intermittent[j] = (int32_t)jin->arr.at(j).as_double();
            for (int i = 0; i < 29; i++)
                if (jti->arr.at(j).arr.at(i).as_double() != 0.0) skipped_days[j * 29 + i] = 1;

            // patients marked as intermittent from day 2: simulate only the first day (.cpp:163-174)
            if (skipped_days[j * 29 + 1]) {
                for (size_t i = 0; i < T; i++)
                    if (time[i] >= 24.0) {
                        simulate_until[j] = (int32_t)i;
                        break;
                    }
            } else {
                simulate_until[j] = (int32_t)T;
            }
            // first measurement later than day 15: do not simulate (.cpp:176-184)
            for (size_t i = 0; i < T; i++) {
                if (!std::isnan(observed[j * T + i])) {
                    if (time[i] > 15 * 24) simulate_until[j] = 0;
                    break;
                }
            }
            if (!std::isnan(dose_after_dose_change[j])) {
                if (std::isnan(dose_change_time[j])) {
                    LOGERROR("Patient %zu has dose change, but time of dose change is not specified.", j);
                    return false;
                }
                if (std::abs(dose_change_time[j] / dosing_interval[j]) < 1e-6) {
                    LOGERROR("Dose change time for patient  %zu is not an exact multiple of the dosing interval.", j);
                    return false;
                }
            }
            if (dose[j] < minimum_dose) minimum_dose = dose[j];
            if (!std::isnan(dose_after_dose_change[j]) && dose_after_dose_change[j] < minimum_dose)
                minimum_dose = dose_after_dose_change[j];
        }
    } catch (std::out_of_range&) {
        LOGERROR("PopPK data arrays have inconsistent dimensions");
        return false;
    } catch (JsonError& e) {
        LOGERROR("PopPK data: %s", e.what.c_str());
        return false;
    }

    if (drug == "lapatinib") MW = 581.06;
    else if (drug == "dacomitinib") MW = 469.95;
    else if (drug == "afatinib") MW = 485.94;
    else if (drug == "trametinib") MW = 615.404;
    else if (drug == "mirdametinib") MW = 482.19;
    else if (drug == "selumetinib") MW = 457.68;
    else MW = NaN;  // the reference reports "Unknown drug" at evaluation time (.cpp:390-392)

    // flat device model
    transforms.resize(varset->GetNumVariables());
    for (size_t i = 0; i < transforms.size(); i++) transforms[i] = (int32_t)varset->GetVariableTransform(i);
    auto ix = [&](const char* n) -> int32_t {
        size_t i = varset->GetVariableIndex(n, false);
        return i == std::numeric_limits<size_t>::max() ? -1 : (int32_t)i;
    };
    model.pk_type = (int32_t)pk_type;
    model.N = (pk_type == PKMT_TwoCompartment || pk_type == PKMT_TwoCompartmentBiphasicUptake ||
               pk_type == PKMT_TwoCompartmentTransit) ? 3 : 2;
    model.num_pk_params = (int32_t)num_pk_params;
    model.num_pk_pop_params = (int32_t)num_pk_pop_params;
    model.d = (int32_t)varset->GetNumVariables();
    model.P = (int32_t)P;
    model.T = (int32_t)T;
    model.sd_ix = ix("standard_deviation");
    model.n_transit_ix = ix("n_transit");
    model.transit_time_ix = ix("mean_transit_time");
    model.biphasic_time_ix = ix("biphasic_uptake_time");
    model.absorption2_ix = ix("mean_absorption2");
    model.max_steps = 2000;  // ODESolverCVODE.cpp:45
    // SetTolerance(1e-6f, minimum_dose * 1e-6f) (.cpp:238)
    model.rtol = (double)1e-6f;
    model.atol = minimum_dose * (double)1e-6f;
    model.MW = std::isnan(MW) ? 1.0 : MW;
    model.fixed_vod = fixed_vod;
    model.fixed_kf = fixed_periphery_fwd;
    model.fixed_kb = fixed_periphery_bwd;
    model.transforms = transforms.data();
    model.time = time.data();
    model.observed = observed.data();
    model.dose = dose.data();
    model.dosing_interval = dosing_interval.data();
    model.dose_after_dose_change = dose_after_dose_change.data();
    model.dose_change_time = dose_change_time.data();
    model.intermittent = intermittent.data();
    model.skipped_days = skipped_days.data();
    model.simulate_until = simulate_until.data();
    if (model.sd_ix < 0) {
        LOGERROR("Could not find variable \"standard_deviation\"");
        return false;
    }
    if (!OpenDevice(vm)) return false;
    if (option_get(vm, "backend", "") == "none") return true;
    int r = bcm3hip_open_popk(device, &model, &ctx);
    if (r != 0) {
        LOGERROR("Opening the PopPK GPU context failed: %s", bcm3hip_error_string(r));
        return false;
    }
    return true;
}

bool LikelihoodPopPKTrajectory::CheckEvaluable()
{
    if (std::isnan(MW)) {
        LOGERROR("Unknown drug \"%s\"", drug.c_str());
        return false;
    }
    return true;
}

// ---------------------------------------------------------------------------------------------
// LikelihoodPharmacokineticTrajectory

static int32_t pk_type_code(const std::string& t)
{
    // SetPKModelType (LikelihoodPharmacokineticTrajectory.cpp:66-83), after its string mapping
    if (t == "one") return BCM3HIP_PK_ONE;
    if (t == "two") return BCM3HIP_PK_TWO;
    if (t == "one_biphasic_uptake" || t == "two_biphasic_uptake") return BCM3HIP_PK_TWO_BIPHASIC;
    if (t == "one_transit") return BCM3HIP_PK_ONE_TRANSIT;
    if (t == "two_transit") return BCM3HIP_PK_TWO_TRANSIT;
    return -1;
}

static Real molecular_weight(const std::string& drug)
{
    if (drug == "lapatinib") return 581.06;
    if (drug == "dacomitinib") return 469.95;
    if (drug == "afatinib") return 485.94;
    if (drug == "trametinib") return 615.404;
    if (drug == "mirdametinib") return 482.19;
    if (drug == "selumetinib") return 457.68;
    return NaN;
}

// LikelihoodPharmacokineticTrajectory::Initialize (.cpp:85-213). The reference opens "pkdata.nc";
// this build reads the same arrays from a JSON sidecar (pkdata_file attribute, default
// "pkdata.json"), as for pop_pk_trajectory.
bool LikelihoodPharmacokineticTrajectory::Initialize(std::shared_ptr<const VariableSet> vs,
                                                     const XmlNode& likelihood_node, const OptionsMap& vm)
{
    varset = vs;
    std::string trial, pk_type_str, pkdata_file;
    try {
        const XmlNode* modelnode = likelihood_node.child("pk_model");
        if (!modelnode) throw XmlError{"No such node (pk_model)"};
        drug = modelnode->get("drug");
        pk_type_str = modelnode->get("type");
        trial = modelnode->get("trial");
        patient_id = modelnode->has_attr("patient") ? modelnode->get("patient") : std::string();
        pkdata_file = modelnode->has_attr("pkdata_file") ? modelnode->get("pkdata_file") : std::string("pkdata.json");
        fixed_vod = modelnode->get_double("volume_of_distribution", NaN);
        fixed_periphery_fwd = modelnode->get_double("k_periphery_fwd", NaN);
        fixed_periphery_bwd = modelnode->get_double("k_periphery_bwd", NaN);
    } catch (XmlError& e) {
        LOGERROR("Error parsing likelihood file: %s", e.what.c_str());
        return false;
    }
    const std::string use_patient = option_get(vm, "pk.patient", "");
    if (!use_patient.empty()) patient_id = use_patient;
    if (patient_id.empty()) {
        LOGERROR("Patient ID has not been specified in either the likelihood or as command-line option.");
        return false;
    }
    const int32_t pk_type = pk_type_code(pk_type_str);
    if (pk_type < 0) {
        LOGERROR("Invalid PK model type");
        return false;
    }

    std::string path = pkdata_file;
    if (!file_exists(path)) {
        std::string alt = option_get(vm, "likelihood_dir", ".") + "/" + pkdata_file;
        if (file_exists(alt)) path = alt;
    }
    Json data;
    try {
        data = json_load(path);
    } catch (JsonError& e) {
        LOGERROR("Failed to open data file %s: %s", pkdata_file.c_str(), e.what.c_str());
        return false;
    }
    const Json* g = data.find(trial);
    if (!g) {
        LOGERROR("Group \"%s\" not found in %s", trial.c_str(), path.c_str());
        return false;
    }
    bool result = true;
    auto var = [&](const std::string& name) -> const Json* {
        const Json* v = g->find(name);
        if (!v) {
            LOGERROR("Variable \"%s\" not found in group \"%s\"", name.c_str(), trial.c_str());
            result = false;
        }
        return v;
    };
    const Json* jt = var("time");
    const Json* jp = var("patients");
    const Json* jc = var(drug + "_plasma_concentration");
    const Json* jd = var(drug + "_dose");
    const Json* jda = var(drug + "_dose_after_dose_change");
    const Json* jdt = var(drug + "_dose_change_time");
    const Json* jdi = var(drug + "_dosing_interval");
    const Json* jin = var(drug + "_intermittent");
    const Json* jti = var("treatment_interruptions");
    if (!result) return false;
    size_t pix = jp->arr.size();
    for (size_t j = 0; j < jp->arr.size(); j++) {
        const Json& p = jp->arr[j];
        const std::string id = p.type == Json::String ? p.str : std::to_string((long)p.num);
        if (id == patient_id) {
            pix = j;
            break;
        }
    }
    if (pix == jp->arr.size()) {
        LOGERROR("Cannot find patient \"%s\" in data file", patient_id.c_str());
        return false;
    }
    const size_t T = jt->arr.size();
    time.resize(T);
    observed.resize(T);
    skipped_days.assign(29, 0);
    try {
        for (size_t i = 0; i < T; i++) {
            time[i] = jt->arr[i].as_double();
            observed[i] = jc->arr.at(pix).arr.at(i).as_double();
        }
        dose = {jd->arr.at(pix).as_double()};
        dose_after_dose_change = {jda->arr.at(pix).as_double()};
        dose_change_time = {jdt->arr.at(pix).as_double()};
        dosing_interval = {jdi->arr.at(pix).as_double()};
        // `intermittent` is read as a bool here (.cpp:183-185)
        intermittent = {jin->arr.at(pix).as_double() != 0.0 ? 1 : 0};
        for (int i = 0; i < 29; i++)
            if (jti->arr.at(pix).arr.at(i).as_double() != 0.0) skipped_days[i] = 1;
    } catch (std::out_of_range&) {
        LOGERROR("PK data arrays have inconsistent dimensions");
        return false;
    } catch (JsonError& e) {
        LOGERROR("PK data: %s", e.what.c_str());
        return false;
    }
    simulate_until = {(int32_t)T};  // every time point (SolveReturnSolution over `time`, .cpp:311)
    MW = molecular_weight(drug);

    transforms.resize(varset->GetNumVariables());
    for (size_t i = 0; i < transforms.size(); i++) transforms[i] = (int32_t)varset->GetVariableTransform(i);
    auto ix = [&](const char* n) -> int32_t {
        size_t i = varset->GetVariableIndex(n, false);
        return i == std::numeric_limits<size_t>::max() ? -1 : (int32_t)i;
    };
    const bool two = pk_type == BCM3HIP_PK_TWO || pk_type == BCM3HIP_PK_TWO_BIPHASIC || pk_type == BCM3HIP_PK_TWO_TRANSIT;
    const bool biphasic = pk_type == BCM3HIP_PK_ONE_BIPHASIC || pk_type == BCM3HIP_PK_TWO_BIPHASIC;
    model = bcm3hip_popk_model{};
    model.pk_type = pk_type;
    model.N = two ? 3 : 2;
    model.num_pk_params = 0;  // (no variable-count check: it is compiled out in the reference, .cpp:118-150)
    model.num_pk_pop_params = 0;
    model.d = (int32_t)varset->GetNumVariables();
    model.P = 1;
    model.T = (int32_t)T;
    model.sd_ix = ix("standard_deviation");
    model.n_transit_ix = ix("n_transit");
    model.transit_time_ix = ix("mean_transit_time");
    model.biphasic_time_ix = biphasic ? 6 : -1;  // fixed indices (.cpp:252-253)
    model.absorption2_ix = biphasic ? 7 : -1;
    model.max_steps = 2000;
    model.param_map = BCM3HIP_PARAM_MAP_SINGLE;
    // SetTolerance(1e-6f, dose * 1e-6f) (.cpp:205)
    model.rtol = (double)1e-6f;
    model.atol = dose[0] * (double)1e-6f;
    model.MW = std::isnan(MW) ? 1.0 : MW;
    model.fixed_vod = fixed_vod;
    model.fixed_kf = fixed_periphery_fwd;
    model.fixed_kb = fixed_periphery_bwd;
    model.transforms = transforms.data();
    model.time = time.data();
    model.observed = observed.data();
    model.dose = dose.data();
    model.dosing_interval = dosing_interval.data();
    model.dose_after_dose_change = dose_after_dose_change.data();
    model.dose_change_time = dose_change_time.data();
    model.intermittent = intermittent.data();
    model.skipped_days = skipped_days.data();
    model.simulate_until = simulate_until.data();
    if (model.sd_ix < 0) {
        LOGERROR("Could not find variable \"standard_deviation\"");
        return false;
    }
    if (!OpenDevice(vm)) return false;
    if (option_get(vm, "backend", "") == "none") return true;
    int r = bcm3hip_open_popk(device, &model, &ctx);
    if (r != 0) {
        LOGERROR("Opening the PK GPU context failed: %s", bcm3hip_error_string(r));
        return false;
    }
    return true;
}

bool LikelihoodPharmacokineticTrajectory::CheckEvaluable()
{
    if (std::isnan(MW)) {
        LOGERROR("Unknown drug \"%s\"", drug.c_str());
        return false;
    }
    return true;
}

// ---------------------------------------------------------------------------------------------
// TestLikelihoodBanana::Initialize (TestLikelihoodBanana.cpp:13-39)
bool TestLikelihoodBanana::Initialize(std::shared_ptr<const VariableSet> vs, const XmlNode& node, const OptionsMap& vm)
{
    varset = vs;
    try {
        dim = (size_t)node.get_long("dimension", -1);
        if (!node.has_attr("dimension")) throw XmlError{"No such node (<xmlattr>.dimension)"};
        if (dim != varset->GetNumVariables()) {
            LOGERROR("Dimension %zd does not match number of variables in prior (%zd)", dim, varset->GetNumVariables());
            return false;
        }
        if (dim < 2) {
            LOGERROR("Dimension is %zd but should be at least 2", dim);
            return false;
        }
        sd1 = node.get_double("sd1");
        sd2 = node.get_double("sd2");
        if (sd1 <= 0.0 || sd2 <= 0.0) {
            LOGERROR("Standard deviations should be greater than 0");
            return false;
        }
    } catch (XmlError& e) {
        LOGERROR("Error parsing likelihood file: %s", e.what.c_str());
        return false;
    }
    if (!OpenDevice(vm)) return false;
    if (option_get(vm, "backend", "") == "none") return true;
    bcm3hip_analytic_model m{BCM3HIP_ANALYTIC_BANANA, (int32_t)dim, sd1, sd2, 0.0};
    int r = bcm3hip_open_analytic(device, &m, &ctx);
    if (r != 0) {
        LOGERROR("Opening the banana GPU context failed: %s", bcm3hip_error_string(r));
        return false;
    }
    return true;
}

// TestLikelihoodCircular::Initialize (TestLikelihoodCircular.cpp:13-37)
bool TestLikelihoodCircular::Initialize(std::shared_ptr<const VariableSet> vs, const XmlNode& node,
                                        const OptionsMap& vm)
{
    varset = vs;
    try {
        if (!node.has_attr("dimension")) throw XmlError{"No such node (<xmlattr>.dimension)"};
        dimension = (size_t)node.get_long("dimension", 0);
        r = node.get_double("radius", 2.0);
        offset = node.get_double("offset", 3.5);
        w = node.get_double("width", 0.1);  // width="=0.1" falls back to 0.1 like Boost's get-with-default
    } catch (XmlError& e) {
        LOGERROR("Error parsing likelihood file: %s", e.what.c_str());
        return false;
    }
    if (varset->GetNumVariables() != dimension) {
        LOGERROR("Inconsistent prior and likelihood (%zu variables and %zu dimensions)", varset->GetNumVariables(),
                 dimension);
        return false;
    }
    if (!OpenDevice(vm)) return false;
    if (option_get(vm, "backend", "") == "none") return true;
    bcm3hip_analytic_model m{BCM3HIP_ANALYTIC_CIRCULAR, (int32_t)dimension, r, offset, w};
    int rr = bcm3hip_open_analytic(device, &m, &ctx);
    if (rr != 0) {
        LOGERROR("Opening the circular GPU context failed: %s", bcm3hip_error_string(rr));
        return false;
    }
    return true;
}

}  // namespace bcm3
