// LikelihoodGPU.cpp -- see LikelihoodGPU.h
#include "LikelihoodGPU.h"

#include <cctype>
#include <cmath>
#include <cstdlib>
#include <exception>
#include <fstream>
#include <limits>

#include "NetCDFClassic.h"
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
    // request combining: the caller that finds no launch in flight takes every queued request
    // (its own included) into one batched launch; the others wait for their results
    if (values.size() != GetNumVariables()) return false;
    Request me{values.data(), 0.0, false, false};
    std::unique_lock<std::mutex> lk(comb_mutex);
    comb_queue.push_back(&me);
    while (!me.done) {
        if (comb_busy) {
            comb_cv.wait(lk);
            continue;
        }
        comb_busy = true;
        std::vector<Request*> batch;
        batch.swap(comb_queue);
        lk.unlock();
        // whatever happens in the launch (a bad_alloc included), the batch is marked done and the
        // waiting threads are woken, so no caller waits on a launch that will never finish
        bool ok = false;
        const size_t d = GetNumVariables(), n = batch.size();
        std::vector<Real> out;
        std::vector<int32_t> st;
        try {
            std::vector<Real> v(n * d);
            out.assign(n, -std::numeric_limits<Real>::infinity());
            st.assign(n, BCM3HIP_STATUS_SOLVER_FAIL);
            for (size_t i = 0; i < n; i++) std::copy(batch[i]->values, batch[i]->values + d, v.begin() + i * d);
            ok = EvaluateLogProbabilityBatch(n, v.data(), out.data(), st.data());
        } catch (const std::exception& e) {
            LOGERROR("Batched likelihood evaluation failed: %s", e.what());
            ok = false;
        }
        lk.lock();
        for (size_t i = 0; i < n; i++) {
            // per request: a model failure (status 1) is a legal -inf, anything else a failed call
            const bool item_ok = ok && i < st.size() && (st[i] == BCM3HIP_STATUS_OK || st[i] == BCM3HIP_STATUS_SOLVER_FAIL);
            batch[i]->logp = item_ok ? out[i] : std::numeric_limits<Real>::quiet_NaN();
            batch[i]->ok = item_ok;
            batch[i]->done = true;
        }
        comb_busy = false;
        comb_cv.notify_all();
    }
    lk.unlock();
    logp = me.logp;
    return me.ok;
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

bool LikelihoodGPUBase::EvaluateLogProbabilityBatchDeviceCounted(size_t n_max, const int32_t* n_dev,
                                                                 const Real* values_dev, Real* logp_dev,
                                                                 int32_t* status_dev, int32_t* steps_dev, void* stream)
{
    if (!SupportsCountedBatch() || !CheckEvaluable() || !ctx) return false;
    std::lock_guard<std::mutex> lock(mutex);
    int r = bcm3hip_eval_batch_device_counted(ctx, n_max, n_dev, values_dev, logp_dev, status_dev, steps_dev, stream);
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
        data = LoadDataFile(path);
        UnwrapDataVariables(data);
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
        data = LoadDataFile(path);
        UnwrapDataVariables(data);
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
// Patient::Load (PharmacoPatient.cpp:8-116) from group g of the JSON sidecar of pkdata.nc:
// treatment schedule up to 696 h, observations sorted with NaN concentrations dropped
static bool load_pharmaco_patient(const Json* g, const std::string& trial, const std::string& drug, size_t pix,
                                  PharmacoPatient& out)
{
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
    const Json* jc = var(drug + "_plasma_concentration");
    const Json* jd = var(drug + "_dose");
    const Json* jdi = var(drug + "_dosing_interval");
    const Json* jda = var(drug + "_dose_after_dose_change");
    const Json* jdt = var(drug + "_dose_change_time");
    const Json* jin = var(drug + "_intermittent");
    const Json* jti = var("treatment_interruptions");
    if (!result) return false;
    std::vector<Real> tp, conc;
    Real dose, dosing_interval, dose_after_dose_change, dose_change_time;
    unsigned int intermittent;
    std::set<int> skipped_days;
    try {
        for (size_t i = 0; i < jt->arr.size(); i++) {
            tp.push_back(jt->arr[i].as_double());
            conc.push_back(jc->arr.at(pix).arr.at(i).as_double());
        }
        dose = jd->arr.at(pix).as_double();
        dosing_interval = jdi->arr.at(pix).as_double();
        dose_after_dose_change = jda->arr.at(pix).as_double();
        dose_change_time = jdt->arr.at(pix).as_double();
        intermittent = (unsigned int)jin->arr.at(pix).as_double();
        for (int i = 0; i < 29; i++)
            if (jti->arr.at(pix).arr.at(i).as_double() != 0.0) skipped_days.insert(i);
    } catch (std::out_of_range&) {
        LOGERROR("PK data arrays have inconsistent dimensions");
        return false;
    } catch (JsonError& e) {
        LOGERROR("PK data: %s", e.what.c_str());
        return false;
    }
    if (!(dosing_interval > 0.0)) {
        LOGERROR("Dosing interval must be positive");  // the reference loops forever otherwise
        return false;
    }
    out.treatment_timepoints.clear();
    out.treatment_doses.clear();
    const Real last_time = 696;
    for (Real t = 0; t < last_time; t += dosing_interval) {
        bool give_treatment = true;
        const int day = static_cast<int>(floor(t / 24.0));
        if (skipped_days.count(day)) give_treatment = false;
        if (intermittent == 1) {
            const Real time_in_week = t - 7.0 * 24.0 * floor(t / (7.0 * 24.0));
            if (time_in_week >= 5.0 * 24.0) give_treatment = false;
        } else if (intermittent == 2) {
            const Real time_in_course = t - 28.0 * 24.0 * floor(t / (28.0 * 24.0));
            if (time_in_course >= 21.0 * 24.0) give_treatment = false;
        } else if (intermittent == 3) {
            const Real time_in_week = t - 7.0 * 24.0 * floor(t / (7.0 * 24.0));
            if (time_in_week >= 4.0 * 24.0) give_treatment = false;
        }
        if (give_treatment) out.treatment_timepoints.push_back(t);
    }
    for (Real t : out.treatment_timepoints)
        out.treatment_doses.push_back((!std::isnan(dose_change_time) && t >= dose_change_time) ? dose_after_dose_change
                                                                                              : dose);
    out.observation_timepoints.clear();
    out.observed_concentrations.clear();
    Real prev_time = -std::numeric_limits<Real>::infinity();
    for (size_t i = 0; i < tp.size(); i++) {
        if (tp[i] < prev_time) {
            LOGERROR("Observation timepoints need to be sorted");
            return false;
        }
        prev_time = tp[i];
        if (!std::isnan(conc[i])) {
            out.observation_timepoints.push_back(tp[i]);
            out.observed_concentrations.push_back(conc[i]);
        }
    }
    if (out.observation_timepoints.empty() || out.treatment_timepoints.empty()) {
        // (the reference reads observation_timepoints.tail(1) and stale scratch here)
        LOGERROR("Patient \"%s\" has no observations or no treatments", out.patient_id.c_str());
        return false;
    }
    return true;
}

static const Json* load_pharmaco_group(const OptionsMap& vm, const std::string& pkdata_file, const std::string& trial,
                                       Json& data)
{
    std::string path = pkdata_file;
    if (!file_exists(path)) {
        std::string alt = option_get(vm, "likelihood_dir", ".") + "/" + pkdata_file;
        if (file_exists(alt)) path = alt;
    }
    try {
        data = LoadDataFile(path);
        UnwrapDataVariables(data);
    } catch (JsonError& e) {
        LOGERROR("Failed to open data file %s: %s", pkdata_file.c_str(), e.what.c_str());
        return nullptr;
    }
    const Json* g = data.find(trial);
    if (!g) LOGERROR("Group \"%s\" not found in %s", trial.c_str(), path.c_str());
    if (g && !g->find("patients")) {
        LOGERROR("Variable \"patients\" not found in group \"%s\"", trial.c_str());
        return nullptr;
    }
    return g;
}

static std::string patient_name(const Json& p) { return p.type == Json::String ? p.str : std::to_string((long)p.num); }

// PharmacoLikelihoodSingle::Initialize (PharmacoLikelihoodSingle.cpp:36-76). The reference opens
// "pkdata.nc"; this build reads the same variables from the JSON sidecar named by pkdata_file
// (default "pkdata.json").
bool PharmacoLikelihoodSingle::Initialize(std::shared_ptr<const VariableSet> vs, const XmlNode& likelihood_node,
                                          const OptionsMap& vm)
{
    varset = vs;
    options = vm;
    std::string trial, pkdata_file;
    try {
        const XmlNode* modelnode = likelihood_node.child("pk_model");
        if (!modelnode) throw XmlError{"No such node (pk_model)"};
        drug = modelnode->get("drug");
        trial = modelnode->get("trial");
        patient.patient_id = modelnode->has_attr("patient") ? modelnode->get("patient") : std::string();
        use_peripheral_compartment = modelnode->get_bool("peripheral_compartment", false);
        const long nt = modelnode->get_long("num_transit_compartments", 0);
        if (nt < 0) throw XmlError{"num_transit_compartments must be >= 0"};
        num_transit_compartments = (size_t)nt;
        biphasic_absorption = modelnode->get_bool("biphasic_absorption", false);
        use_metabolite = modelnode->get_bool("metabolite", false);
        pkdata_file = modelnode->has_attr("pkdata_file") ? modelnode->get("pkdata_file") : std::string("pkdata.json");
    } catch (XmlError& e) {
        LOGERROR("Error parsing likelihood file: %s", e.what.c_str());
        return false;
    }
    const std::string use_patient = option_get(vm, "pharmacosingle.patient", "");
    if (!use_patient.empty()) patient.patient_id = use_patient;
    if (patient.patient_id.empty()) {
        LOGERROR("Patient ID has not been specified in either the likelihood or as command-line option.");
        return false;
    }
    Json data;
    const Json* g = load_pharmaco_group(vm, pkdata_file, trial, data);
    if (!g) return false;
    const Json* jp = g->find("patients");
    size_t pix = jp->arr.size();
    for (size_t j = 0; j < jp->arr.size(); j++) {
        if (patient_name(jp->arr[j]) == patient.patient_id) {
            pix = j;
            break;
        }
    }
    if (pix == jp->arr.size()) {
        LOGERROR("Cannot find patient \"%s\" in data file", patient.patient_id.c_str());
        return false;
    }
    if (!load_pharmaco_patient(g, trial, drug, pix, patient)) return false;
    MW = molecular_weight(drug);
    if (std::isnan(MW)) {
        LOGERROR("Unknown drug \"%s\"", drug.c_str());
        return false;
    }
    return true;
}

// PharmacoLikelihoodSingle::PostInitialize (.cpp:78-147)
bool PharmacoLikelihoodSingle::PostInitialize()
{
    const size_t none = std::numeric_limits<size_t>::max();
    auto ix = [&](const char* n, bool required) -> int32_t {
        const size_t i = varset->GetVariableIndex(n, required);
        return i == none ? -1 : (int32_t)i;
    };
    model = bcm3hip_expm_pk_model{};
    model.additive_sd_ix = ix("additive_error_standard_deviation", false);
    model.proportional_sd_ix = ix("proportional_error_standard_deviation", false);
    if (model.additive_sd_ix < 0 && model.proportional_sd_ix < 0) {
        LOGERROR("Neither \"additive_error_standard_deviation\" nor \"proportional_error_standard_deviation\" has been "
                 "specified in the prior; at least one of these variables should be included.");
        return false;
    }
    model.absorption_ix = ix("absorption", true);
    model.clearance_ix = ix("clearance", true);
    model.vod_ix = ix("volume_of_distribution", true);
    if (model.absorption_ix < 0 || model.clearance_ix < 0 || model.vod_ix < 0) return false;
    model.excretion_ix = ix("excretion", false);
    model.pf_ix = model.pb_ix = model.mtt_ix = model.direct_ix = model.metab_conv_ix = -1;
    if (use_peripheral_compartment) {
        model.pf_ix = ix("peripheral_forward_rate", true);
        model.pb_ix = ix("peripheral_backward_rate", true);
        if (model.pf_ix < 0 || model.pb_ix < 0) {
            LOGERROR("Peripheral compartmant was specified, but forward or backward rates have not both been specified in prior.");
            return false;
        }
    }
    if (num_transit_compartments > 0) {
        model.mtt_ix = ix("mean_transit_time", true);
        if (model.mtt_ix < 0) {
            LOGERROR("Transit compartmants were specified, but mean transit time has not been specified in prior.");
            return false;
        }
    }
    if (biphasic_absorption) {
        model.direct_ix = ix("direct_absorption", true);
        if (model.direct_ix < 0) {
            LOGERROR("Biphasic absorption was specified, but direct absorption rate has not been specified in prior.");
            return false;
        }
    }
    if (use_metabolite) {
        model.metab_conv_ix = ix("metabolite_conversion_rate", true);
        if (model.metab_conv_ix < 0) {
            LOGERROR("Use of metabolite was specified, but metabolite conversion rate has not been specified in prior.");
            return false;
        }
    }
    transforms.resize(varset->GetNumVariables());
    for (size_t i = 0; i < transforms.size(); i++) transforms[i] = (int32_t)varset->GetVariableTransform(i);
    model.d = (int32_t)varset->GetNumVariables();
    model.n_transit = (int32_t)num_transit_compartments;
    model.peripheral = use_peripheral_compartment;
    model.biphasic = biphasic_absorption;
    model.metabolite = use_metabolite;
    model.n_treat = (int32_t)patient.treatment_timepoints.size();
    model.n_obs = (int32_t)patient.observation_timepoints.size();
    model.MW = MW;
    model.transforms = transforms.data();
    model.treat_times = patient.treatment_timepoints.data();
    model.treat_doses = patient.treatment_doses.data();
    model.obs_times = patient.observation_timepoints.data();
    model.obs_conc = patient.observed_concentrations.data();
    model.param_map = BCM3HIP_PARAM_MAP_SINGLE;
    model.P = 1;
    for (int w = 0; w < 5; w++) model.sigma_ix[w] = -1;
    const int ncomp = 2 + (use_peripheral_compartment ? 1 : 0) + (use_metabolite ? 1 : 0) + (int)num_transit_compartments;
    if (ncomp > BCM3HIP_EXPM_NMAX) {
        LOGERROR("%d compartments; this backend supports at most %d", ncomp, (int)BCM3HIP_EXPM_NMAX);
        return false;
    }
    if (!OpenDevice(options)) return false;
    if (option_get(options, "backend", "") == "none") return true;
    const int r = bcm3hip_open_expm_pk(device, &model, &ctx);
    if (r != 0) {
        LOGERROR("Opening the pharmaco_single GPU context failed: %s", bcm3hip_error_string(r));
        return false;
    }
    return true;
}

// ---------------------------------------------------------------------------------------------
// PharmacoLikelihoodPopulation::Initialize (PharmacoLikelihoodPopulation.cpp:43-98): every patient
// of the trial, loaded as Patient::Load does, concatenated for the device (offsets per patient)
bool PharmacoLikelihoodPopulation::Initialize(std::shared_ptr<const VariableSet> vs, const XmlNode& likelihood_node,
                                              const OptionsMap& vm)
{
    varset = vs;
    options = vm;
    std::string trial, pkdata_file;
    try {
        const XmlNode* modelnode = likelihood_node.child("pk_model");
        if (!modelnode) throw XmlError{"No such node (pk_model)"};
        drug = modelnode->get("drug");
        trial = modelnode->get("trial");
        use_peripheral_compartment = modelnode->get_bool("peripheral_compartment", false);
        const long nt = modelnode->get_long("num_transit_compartments", 0);
        if (nt < 0) throw XmlError{"num_transit_compartments must be >= 0"};
        num_transit_compartments = (size_t)nt;
        use_bioavailability = modelnode->get_bool("bioavailability", false);
        // likelihood_cache_size: the reference's exact-match cache; nothing to size here
        if (modelnode->get_long("likelihood_cache_size", 16) < 0) throw XmlError{"likelihood_cache_size must be >= 0"};
        pkdata_file = modelnode->has_attr("pkdata_file") ? modelnode->get("pkdata_file") : std::string("pkdata.json");
    } catch (XmlError& e) {
        LOGERROR("Error parsing likelihood file: %s", e.what.c_str());
        return false;
    }
    Json data;
    const Json* g = load_pharmaco_group(vm, pkdata_file, trial, data);
    if (!g) return false;
    const Json* jp = g->find("patients");
    patients.assign(jp->arr.size(), PharmacoPatient{});
    if (patients.empty()) {
        LOGERROR("No patients in group \"%s\"", trial.c_str());
        return false;
    }
    treat_times.clear();
    treat_doses.clear();
    obs_times.clear();
    obs_conc.clear();
    treat_offset.assign(1, 0);
    obs_offset.assign(1, 0);
    for (size_t i = 0; i < patients.size(); i++) {
        patients[i].patient_id = patient_name(jp->arr[i]);
        if (!load_pharmaco_patient(g, trial, drug, i, patients[i])) return false;
        const PharmacoPatient& p = patients[i];
        treat_times.insert(treat_times.end(), p.treatment_timepoints.begin(), p.treatment_timepoints.end());
        treat_doses.insert(treat_doses.end(), p.treatment_doses.begin(), p.treatment_doses.end());
        obs_times.insert(obs_times.end(), p.observation_timepoints.begin(), p.observation_timepoints.end());
        obs_conc.insert(obs_conc.end(), p.observed_concentrations.begin(), p.observed_concentrations.end());
        treat_offset.push_back((int32_t)treat_times.size());
        obs_offset.push_back((int32_t)obs_times.size());
    }
    MW = molecular_weight(drug);
    if (std::isnan(MW)) {
        LOGERROR("Unknown drug \"%s\"", drug.c_str());
        return false;
    }
    return true;
}

// PharmacoLikelihoodPopulation::InitializePatientMarginals (.cpp:345-356): p<i>_<name>, i from 1
bool PharmacoLikelihoodPopulation::InitializePatientMarginals(const std::string& name, int which)
{
    const size_t P = patients.size();
    for (size_t i = 0; i < P; i++) {
        const std::string varname = "p" + std::to_string(i + 1) + "_" + name;
        const size_t ix = varset->GetVariableIndex(varname, false);
        if (ix == std::numeric_limits<size_t>::max()) {
            LOGERROR("Standard deviation found for \"%s\", but could not find prior variable for \"%s\"", name.c_str(),
                     varname.c_str());
            return false;
        }
        patient_ix[which * P + i] = (int32_t)ix;
    }
    return true;
}

// PharmacoLikelihoodPopulation::PostInitialize (.cpp:100-183)
bool PharmacoLikelihoodPopulation::PostInitialize()
{
    const size_t none = std::numeric_limits<size_t>::max();
    auto ix = [&](const std::string& n, bool required) -> int32_t {
        const size_t i = varset->GetVariableIndex(n, required);
        return i == none ? -1 : (int32_t)i;
    };
    model = bcm3hip_expm_pk_model{};
    model.additive_sd_ix = ix("additive_error_standard_deviation", false);
    model.proportional_sd_ix = ix("proportional_error_standard_deviation", false);
    if (model.additive_sd_ix < 0 && model.proportional_sd_ix < 0) {
        LOGERROR("Neither \"additive_error_standard_deviation\" nor \"proportional_error_standard_deviation\" has been "
                 "specified in the prior; at least one of these variables should be included.");
        return false;
    }
    model.absorption_ix = ix("mean_absorption", true);
    model.clearance_ix = ix("mean_clearance", true);
    model.vod_ix = ix("mean_volume_of_distribution", true);
    if (model.absorption_ix < 0 || model.clearance_ix < 0 || model.vod_ix < 0) return false;
    model.excretion_ix = ix("mean_excretion", false);
    const size_t P = patients.size();
    patient_ix.assign(6 * P, -1);
    static const char* rates[5] = {"absorption", "excretion", "clearance", "volume_of_distribution", "transit_time"};
    for (int w = 0; w < 5; w++) {
        model.sigma_ix[w] = ix(std::string("sigma_") + rates[w], false);
        if (model.sigma_ix[w] >= 0 && !InitializePatientMarginals(rates[w], w)) return false;
    }
    model.pf_ix = model.pb_ix = model.mtt_ix = model.direct_ix = model.metab_conv_ix = -1;
    if (use_peripheral_compartment) {
        model.pf_ix = ix("peripheral_forward_rate", true);
        model.pb_ix = ix("peripheral_backward_rate", true);
        if (model.pf_ix < 0 || model.pb_ix < 0) {
            LOGERROR("Peripheral compartmant was specified, but forward or backward rates have not both been specified in prior.");
            return false;
        }
    }
    if (num_transit_compartments > 0) {
        model.mtt_ix = ix("mean_transit_time", true);
        if (model.mtt_ix < 0) {
            LOGERROR("Transit compartmants were specified, but mean transit time has not been specified in prior.");
            return false;
        }
    } else {
        model.sigma_ix[4] = -1;  // the reference reads sigma_transit_time only with transit compartments
    }
    if (use_bioavailability && !InitializePatientMarginals("bioavailability", 5)) return false;
    transforms.resize(varset->GetNumVariables());
    for (size_t i = 0; i < transforms.size(); i++) transforms[i] = (int32_t)varset->GetVariableTransform(i);
    model.d = (int32_t)varset->GetNumVariables();
    model.n_transit = (int32_t)num_transit_compartments;
    model.peripheral = use_peripheral_compartment;
    model.n_treat = (int32_t)treat_times.size();
    model.n_obs = (int32_t)obs_times.size();
    model.MW = MW;
    model.transforms = transforms.data();
    model.treat_times = treat_times.data();
    model.treat_doses = treat_doses.data();
    model.obs_times = obs_times.data();
    model.obs_conc = obs_conc.data();
    model.param_map = BCM3HIP_PARAM_MAP_POPULATION;
    model.P = (int32_t)P;
    model.patient_ix = patient_ix.data();
    model.treat_offset = treat_offset.data();
    model.obs_offset = obs_offset.data();
    const int ncomp = 2 + (use_peripheral_compartment ? 1 : 0) + (int)num_transit_compartments;
    if (ncomp > BCM3HIP_EXPM_NMAX) {
        LOGERROR("%d compartments; this backend supports at most %d", ncomp, (int)BCM3HIP_EXPM_NMAX);
        return false;
    }
    if (!OpenDevice(options)) return false;
    if (option_get(options, "backend", "") == "none") return true;
    const int r = bcm3hip_open_expm_pk(device, &model, &ctx);
    if (r != 0) {
        LOGERROR("Opening the pharmaco_population GPU context failed: %s", bcm3hip_error_string(r));
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

// ---------------------------------------------------------------------------------------------
// bcm3::tokenize (src/utils/Utils.cpp:7-25): boost::char_separator with keep_empty_tokens, one
// trailing newline dropped; an empty string gives no tokens
static std::vector<std::string> tokenize_keep_empty(std::string str, char delim)
{
    std::vector<std::string> t;
    if (str.empty()) return t;
    if (str.back() == '\n') str.pop_back();
    size_t b = 0;
    for (;;) {
        size_t e = str.find(delim, b);
        t.push_back(str.substr(b, e == std::string::npos ? std::string::npos : e - b));
        if (e == std::string::npos) break;
        b = e + 1;
    }
    return t;
}

// boost::lexical_cast<double>: the whole token, no surrounding whitespace, no hexadecimal form
static bool lexical_cast_real(const std::string& s, Real& v)
{
    if (s.empty() || std::isspace((unsigned char)s.front()) || std::isspace((unsigned char)s.back())) return false;
    if (s.find_first_of("xX") != std::string::npos) return false;
    char* e = nullptr;
    v = std::strtod(s.c_str(), &e);
    return e && *e == 0;
}

bool ParseVectorFromString(const std::string& str, std::vector<Real>& v)
{
    const std::vector<std::string> tok = tokenize_keep_empty(str, ';');
    v.assign(tok.size(), 0.0);
    for (size_t i = 0; i < tok.size(); i++) {
        if (!lexical_cast_real(tok[i], v[i])) {
            LOGERROR("Could not cast value \"%s\" to a constant real value: bad lexical cast", tok[i].c_str());
            return false;
        }
    }
    return true;
}

bool ParseMatrixFromString(const std::string& str, std::vector<std::vector<Real>>& m)
{
    const std::vector<std::string> rows = tokenize_keep_empty(str, ';');
    m.clear();
    if (rows.empty()) {  // the reference reads rows[0] of an empty list
        LOGERROR("Empty matrix");
        return false;
    }
    const size_t cols = tokenize_keep_empty(rows[0], ',').size();
    for (const std::string& r : rows) {
        const std::vector<std::string> row = tokenize_keep_empty(r, ',');
        if (row.size() != cols) {
            LOGERROR("Inconsistent matrix");
            return false;
        }
        std::vector<Real> vals(cols);
        for (size_t j = 0; j < cols; j++) {
            if (!lexical_cast_real(row[j], vals[j])) {
                LOGERROR("Could not cast string to a Real value: bad lexical cast");
                return false;
            }
        }
        m.push_back(vals);
    }
    return true;
}

static bool open_mixture_ctx(int device, int kind, size_t d, const std::vector<Real>& log_w,
                             const std::vector<std::vector<Real>>& mus, const std::vector<std::vector<std::vector<Real>>>& sigmas,
                             const std::vector<Real>& nus, bcm3hip_ctx** ctx, const char* what)
{
    const size_t K = log_w.size();
    std::vector<double> mean, cov;
    for (size_t k = 0; k < K; k++) {
        mean.insert(mean.end(), mus[k].begin(), mus[k].end());
        for (size_t i = 0; i < d; i++) cov.insert(cov.end(), sigmas[k][i].begin(), sigmas[k][i].end());
    }
    bcm3hip_mixture_model m{kind, (int32_t)d, (int32_t)K, log_w.data(), mean.data(), cov.data(),
                            nus.empty() ? nullptr : nus.data()};
    const int r = bcm3hip_open_mixture(device, &m, ctx);
    if (r != 0) {
        LOGERROR("Opening the %s GPU context failed: %s%s", what, bcm3hip_error_string(r),
                 r == BCM3HIP_ERR_MODEL ? " (a covariance that is not positive definite, a nu <= 0, or more than "
                                          "16 dimensions / 64 clusters)"
                                        : "");
        return false;
    }
    return true;
}

// TestLikelihoodMultimodalGaussians::Initialize (TestLikelihoodMultimodalGaussians.cpp:15-34): two
// fixed 2-D components, weights 1/2: means (-5,-5), (5,5), covariances [1 -0.9; -0.9 1], [2 -0.5; -0.5 1]
bool TestLikelihoodMultimodalGaussians::Initialize(std::shared_ptr<const VariableSet> vs, const XmlNode& node,
                                                   const OptionsMap& vm)
{
    varset = vs;
    if (varset->GetNumVariables() != 2) {
        LOGERROR("Inconsistent prior and likelihood (%zu variables and %zu dimensions)", varset->GetNumVariables(),
                 (size_t)2);
        return false;
    }
    if (!OpenDevice(vm)) return false;
    if (option_get(vm, "backend", "") == "none") return true;
    const std::vector<Real> lw = {std::log(0.5), std::log(0.5)};
    const std::vector<std::vector<Real>> mus = {{-5, -5}, {5, 5}};
    const std::vector<std::vector<std::vector<Real>>> sig = {{{1, -0.9}, {-0.9, 1}}, {{2, -0.5}, {-0.5, 1}}};
    return open_mixture_ctx(device, BCM3HIP_MIXTURE_NORMAL, 2, lw, mus, sig, {}, &ctx, "multimodal_gaussians");
}

// TestLikelihoodTruncatedT::Initialize (TestLikelihoodTruncatedT.cpp:20-79): num_clusters components
// mu<i> / sigma<i> (1-based), nus, weights normalised to sum 1 (log taken per evaluation there, once here)
bool TestLikelihoodTruncatedT::Initialize(std::shared_ptr<const VariableSet> vs, const XmlNode& node,
                                          const OptionsMap& vm)
{
    varset = vs;
    std::vector<std::vector<Real>> mus;
    std::vector<std::vector<std::vector<Real>>> sigmas;
    std::vector<Real> nus, weights;
    try {
        if (!node.has_attr("dimensions")) throw XmlError{"No such node (<xmlattr>.dimensions)"};
        if (!node.has_attr("num_clusters")) throw XmlError{"No such node (<xmlattr>.num_clusters)"};
        const long dl = node.get_long("dimensions", -1), kl = node.get_long("num_clusters", -1);
        if (dl < 0 || kl < 0) throw XmlError{"conversion of data to type \"size_t\" failed"};
        dimensions = (size_t)dl;
        num_clusters = (size_t)kl;
        if (varset->GetNumVariables() != dimensions) {
            LOGERROR("Incorrect number of variables in prior for samples a %zu-dimensional space", dimensions);
            return false;
        }
        mus.resize(num_clusters);
        sigmas.resize(num_clusters);
        for (size_t i = 0; i < num_clusters; i++) {
            if (!ParseVectorFromString(node.get("mu" + std::to_string(i + 1)), mus[i])) return false;
            if (mus[i].size() != dimensions) {
                LOGERROR("Inconsistent dimension for mu%zu", i);
                return false;
            }
            if (!ParseMatrixFromString(node.get("sigma" + std::to_string(i + 1)), sigmas[i])) return false;
            if (sigmas[i].size() != dimensions || sigmas[i][0].size() != dimensions) {
                LOGERROR("Inconsistent dimension for sigma%zu", i);
                return false;
            }
        }
        if (!ParseVectorFromString(node.get("nus"), nus)) return false;
        if (nus.size() != num_clusters) {
            LOGERROR("Inconsistent number of nus");
            return false;
        }
        if (!ParseVectorFromString(node.get("weights"), weights)) return false;
        if (weights.size() != num_clusters) {
            LOGERROR("Inconsistent number of weights");
            return false;
        }
    } catch (XmlError& e) {
        LOGERROR("Error parsing likelihood file: %s", e.what.c_str());
        return false;
    }
    if (num_clusters == 0) {
        LOGERROR("truncated_t needs at least one cluster (the reference's logp is -inf for every sample)");
        return false;
    }
    Real wsum = 0.0;
    for (Real w : weights) wsum += w;
    std::vector<Real> lw(num_clusters);
    for (size_t i = 0; i < num_clusters; i++) lw[i] = std::log(weights[i] / wsum);
    if (!OpenDevice(vm)) return false;
    if (option_get(vm, "backend", "") == "none") return true;
    return open_mixture_ctx(device, BCM3HIP_MIXTURE_T, dimensions, lw, mus, sigmas, nus, &ctx, "truncated_t");
}

// LikelihoodDummy::Initialize / EvaluateLogProbability (LikelihoodDummy.cpp:13-32): LogPdfTnu4(values[0], 0, 1)
bool LikelihoodDummy::Initialize(std::shared_ptr<const VariableSet> vs, const XmlNode& node, const OptionsMap& vm)
{
    varset = vs;
    if (varset->GetNumVariables() < 1) {
        LOGERROR("The dummy likelihood reads the first variable; the prior has none");
        return false;
    }
    if (!OpenDevice(vm)) return false;
    if (option_get(vm, "backend", "") == "none") return true;
    bcm3hip_analytic_model m{BCM3HIP_ANALYTIC_DUMMY, (int32_t)varset->GetNumVariables(), 0.0, 0.0, 0.0};
    const int r = bcm3hip_open_analytic(device, &m, &ctx);
    if (r != 0) {
        LOGERROR("Opening the dummy GPU context failed: %s", bcm3hip_error_string(r));
        return false;
    }
    return true;
}

}  // namespace bcm3
