// LikelihoodCellPopulation.cpp -- see LikelihoodCellPopulation.h. File:line citations are to the
// reference's src/cellpop unless stated otherwise.
#include "LikelihoodCellPopulation.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <fstream>
#include <functional>
#include <limits>

#include "NetCDFClassic.h"
#include "json.h"
#include "log.h"

namespace bcm3 {

namespace {
constexpr double NaN = std::numeric_limits<double>::quiet_NaN();

bool file_exists(const std::string& p)
{
    std::ifstream f(p);
    return (bool)f;
}

std::string resolve(const std::string& fn, const OptionsMap& vm)
{
    if (file_exists(fn)) return fn;
    const std::string alt = option_get(vm, "likelihood_dir", ".") + "/" + fn;
    return file_exists(alt) ? alt : fn;
}

bool parse_double(const std::string& s, double& v)
{
    char* end = nullptr;
    v = strtod(s.c_str(), &end);
    if (end == s.c_str()) return false;
    while (*end && std::isspace((unsigned char)*end)) end++;
    return *end == '\0';
}

// bcm3::tokenize (src/utils/Utils.cpp:7-25): boost char_separator with keep_empty_tokens, a trailing
// newline dropped, nothing for an empty string
std::vector<std::string> tokenize(std::string s, char delim)
{
    std::vector<std::string> out;
    if (s.empty()) return out;
    if (s.back() == '\n') s.pop_back();
    size_t p0 = 0;
    for (;;) {
        const size_t p1 = s.find(delim, p0);
        out.push_back(s.substr(p0, p1 == std::string::npos ? std::string::npos : p1 - p0));
        if (p1 == std::string::npos) break;
        p0 = p1 + 1;
    }
    return out;
}

std::string trim(const std::string& s)
{
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) a++;
    while (b > a && std::isspace((unsigned char)s[b - 1])) b--;
    return s.substr(a, b - a);
}

// Joe & Kuo (2008) new-joe-kuo-6.21201, dimensions 2..13: (s, a, m_1..m_s)
struct JK {
    int s, a;
    unsigned m[5];
};
const JK kJoeKuo[] = {{1, 0, {1}},          {2, 1, {1, 3}},          {3, 1, {1, 3, 1}},        {3, 2, {1, 1, 1}},
                      {4, 1, {1, 1, 3, 3}}, {4, 4, {1, 3, 5, 13}},   {5, 2, {1, 1, 5, 5, 17}}, {5, 4, {1, 1, 5, 5, 5}},
                      {5, 7, {1, 1, 7, 11, 19}}, {5, 11, {1, 1, 5, 1, 1}}, {5, 13, {1, 1, 1, 3, 11}}, {5, 14, {1, 3, 5, 5, 31}}};
}  // namespace

std::vector<double> SobolPoints(size_t points, size_t dims)
{
    std::vector<double> out(points * dims);
    if (dims == 0) return out;
    const int bits = 64;
    std::vector<std::vector<uint64_t>> v(dims, std::vector<uint64_t>(bits));
    for (size_t d = 0; d < dims; d++) {
        if (d == 0) {
            for (int k = 0; k < bits; k++) v[d][k] = (uint64_t)1 << (bits - 1 - k);
            continue;
        }
        const JK& jk = kJoeKuo[d - 1];
        std::vector<uint64_t> m(jk.m, jk.m + jk.s);
        for (int k = jk.s; k < bits; k++) {
            uint64_t x = m[k - jk.s] ^ (m[k - jk.s] << jk.s);
            for (int j = 1; j < jk.s; j++)
                if ((jk.a >> (jk.s - 1 - j)) & 1) x ^= m[k - j] << j;
            m.push_back(x);
        }
        for (int k = 0; k < bits; k++) v[d][k] = m[k] << (bits - 1 - k);
    }
    std::vector<uint64_t> state(dims, 0);
    for (size_t i = 0; i < points; i++) {
        int c = 0;
        for (size_t x = i; x & 1; x >>= 1) c++;
        for (size_t d = 0; d < dims; d++) {
            state[d] ^= v[d][c];
            out[i * dims + d] = (double)state[d] * 5.42101086242752217e-20;  // 2^-64
        }
    }
    return out;
}

LikelihoodCellPopulation::LikelihoodCellPopulation(size_t sampling_threads, size_t evaluation_threads) {}

// the synchronize attribute of time courses / time points (DataLikelihoodTimeCourse.cpp:27-41,
// DataLikelihoodTimePoints.cpp:29-43)
static bool parse_sync(const std::string& s, int32_t& sync)
{
    if (s.empty() || s == "none")
        sync = BCM3HIP_CP_SYNC_NONE;
    else if (s == "DNA_replication_start")
        sync = BCM3HIP_CP_SYNC_DNA_REPLICATION_START;
    else if (s == "PCNA_gfp_increase")
        sync = BCM3HIP_CP_SYNC_PCNA_GFP_INCREASE;
    else if (s == "mitosis" || s == "nuclear_envelope_breakdown")
        sync = BCM3HIP_CP_SYNC_NUCLEAR_ENVELOPE_BREAKDOWN;
    else if (s == "anaphase" || s == "anaphase_onset")
        sync = BCM3HIP_CP_SYNC_ANAPHASE_ONSET;
    else {
        LOGERROR("Synchronization is specified as \"%s\" which is not a recognized synchronization point", s.c_str());
        return false;
    }
    return true;
}

bool LikelihoodCellPopulation::ParseRef(const std::string& s, bcm3hip_value_ref& r) const
{
    // ValueReference::Load (ValueReference.cpp:16-41): sampled variable, else a number
    const size_t ix = varset->GetVariableIndex(s, false);
    if (ix != SIZE_MAX) {
        r = bcm3hip_value_ref{BCM3HIP_REF_VARIABLE, (int32_t)ix, 0.0};
        return true;
    }
    double v;
    if (!parse_double(s, v)) {
        LOGERROR("Could not find variable for parameter \"%s\", and also could not cast it to a constant real value", s.c_str());
        return false;
    }
    r = bcm3hip_value_ref{BCM3HIP_REF_FIXED, -1, v};
    return true;
}

// CellPopulationLikelihood::Initialize (CellPopulationLikelihood.cpp:19-44)
bool LikelihoodCellPopulation::Initialize(std::shared_ptr<const VariableSet> vs, const XmlNode& likelihood_node,
                                          const OptionsMap& vm)
{
    varset = vs;
    host_only = option_get(vm, "backend", "") == "none";
    std::vector<const XmlNode*> exps = likelihood_node.children_named("experiment");
    if (exps.empty()) {
        LOGERROR("cell_population: no <experiment> in the likelihood");
        return false;
    }
    try {
        if (!LoadExperiment(*exps[0], vm)) return false;
        for (size_t k = 1; k < exps.size(); k++) {
            auto e = std::make_unique<LikelihoodCellPopulation>(1, 1);
            e->varset = vs;
            e->host_only = true;
            if (!e->LoadExperiment(*exps[k], vm)) return false;
            more_experiments.push_back(std::move(e));
        }
    } catch (XmlError& e) {
        LOGERROR("Error parsing likelihood file: %s", e.what.c_str());
        return false;
    }
    return OpenDevice(vm);
}

// Experiment::Load + Initialize (Experiment.cpp:404-633)
bool LikelihoodCellPopulation::LoadExperiment(const XmlNode& ex, const OptionsMap& vm)
{
    name = ex.get("name");
    const std::string model_file = resolve(ex.get("model_file"), vm);
    const std::string data_file = ex.has_attr("data_file") ? ex.get("data_file") : std::string();
    const std::string solver_type = ex.has_attr("solver_type") ? ex.get("solver_type") : std::string("CVODE");
    // Cell::AllocateSolver (Cell.cpp:57-66)
    if (solver_type == "DP5")
        solver = BCM3HIP_CP_SOLVER_DP5;
    else if (solver_type == "CVODE")
        solver = BCM3HIP_CP_SOLVER_CVODE;
    else {
        LOGERROR("Unknown solver type \"%s\"; accepted options are \"DP5\" or \"CVODE\"", solver_type.c_str());
        return false;
    }
    const double feps4 = 4 * (double)std::numeric_limits<float>::epsilon();
    hmin = ex.get_double("solver_min_timestep", 1e-8);
    hmax = ex.get_double("solver_max_timestep", std::numeric_limits<double>::infinity());
    // DP5's max_dt (ODESolverDP5::SetSolverParameter, :81-87: must be positive); the CVODE kernel
    // has no hmax clamp (CVodeSetMaxStep)
    if (solver == BCM3HIP_CP_SOLVER_DP5 && !(hmax > 0.0)) {
        LOGERROR("max_dt should be strictly positive, but %g was provided", hmax);
        return false;
    }
    if (solver != BCM3HIP_CP_SOLVER_DP5 && !std::isinf(hmax)) {
        LOGERROR("cell_population: a finite solver_max_timestep is not supported");
        return false;
    }
    max_steps = (int32_t)ex.get_long("solver_max_steps", 10000);
    atol = ex.get_double("solver_absolute_tolerance", feps4);
    rtol = ex.get_double("solver_relative_tolerance", feps4);

    std::string err;
    if (!sbml.LoadSBML(model_file, err)) {
        LOGERROR("%s", err.c_str());
        return false;
    }
    num_cells = (int32_t)ex.get_long("num_cells", 1);
    max_cells = (int32_t)ex.get_long("max_cells", 20);
    divide_cells = ex.get_bool("divide_cells", true);
    trailing = ex.get_double("trailing_simulation_time", 0.0);
    past_cs = ex.get_double("simulate_past_chromatid_separation_time", 0.0);

    treat_names.clear();
    treat_times.clear();
    treat_offset.assign(1, 0);
    for (const auto& c : ex.children) {
        if (c->name == "set_parameter") {
            const std::string p = c->get("parameter_name");
            if (!sbml.HasParameter(p)) {
                LOGERROR("Fixed parameter value requested for \"%s\", but there is no parameter with that ID in the SBML model", p.c_str());
                return false;
            }
            forced[p] = c->get_double("value");
        } else if (c->name == "set_species" || c->name == "experiment_specific_parameter") {
            LOGERROR("cell_population: <%s> is not supported", c->name.c_str());
            return false;
        } else if (c->name == "treatment_trajectory") {
            // Experiment::Load (Experiment.cpp:571-584) + TreatmentTrajectory::Create / Load
            const std::string type = c->get("type");
            if (type == "from_data") {
                // TreatmentTrajectoryFromData::Load fails in the reference (its data read is #if TODO)
                LOGERROR("Treatment trajectory type \"from_data\" cannot be loaded (the reference's loader returns failure)");
                return false;
            }
            if (type != "pulses") {
                LOGERROR("Unknown trajectory type \"%s\"", type.c_str());
                return false;
            }
            treat_names.push_back(c->get("species_name"));
            // TreatmentTrajectoryPulses::Load: comma-separated times, sorted
            std::vector<double> t;
            const std::string ts = c->get("times");
            size_t p0 = 0;
            while (p0 <= ts.size()) {
                size_t p1 = ts.find(',', p0);
                if (p1 == std::string::npos) p1 = ts.size();
                std::string tok = ts.substr(p0, p1 - p0);
                tok.erase(0, tok.find_first_not_of(" \t"));
                tok.erase(tok.find_last_not_of(" \t") + 1);
                char* end = nullptr;
                const double v = strtod(tok.c_str(), &end);
                if (tok.empty() || *end) {
                    LOGERROR("Treatment trajectory: could not read pulse time \"%s\"", tok.c_str());
                    return false;
                }
                t.push_back(v);
                p0 = p1 + 1;
            }
            std::sort(t.begin(), t.end());
            treat_times.insert(treat_times.end(), t.begin(), t.end());
            treat_offset.push_back((int32_t)treat_times.size());
        }
    }
    // cell variabilities (VariabilityDescription::Load, VariabilityDescriptionVariable::Load)
    for (const XmlNode* cv : ex.children_named("cell_variability")) {
        const std::string dist = cv->get("distribution");
        if (dist != "diagonal_gaussian" && dist != "full_gaussian") {
            LOGERROR("Unknown distribution \"%s\" in variability description", dist.c_str());
            return false;
        }
        std::vector<VarVariable> vv;
        for (const XmlNode* v : cv->children_named("variable")) {
            VarVariable x;
            x.species = v->has_attr("initial_condition_species") ? v->get("initial_condition_species") : "";
            x.parameter = v->has_attr("model_parameter") ? v->get("model_parameter") : "";
            x.entry_time = v->has_attr("entry_time") && !v->get("entry_time").empty();
            const int count = (!x.species.empty()) + (!x.parameter.empty()) + (x.entry_time ? 1 : 0);
            if (count != 1) {
                LOGERROR("Cell variability description needs exactly one of initial_condition_species, model_parameter, entry_time");
                return false;
            }
            x.only_initial = v->get_bool("only_initial_cells", x.entry_time);
            const std::string a = v->get("apply");
            static const std::map<std::string, int32_t> apply = {
                {"additive", BCM3HIP_APPLY_ADDITIVE}, {"additive_log", BCM3HIP_APPLY_ADDITIVE_LOG},
                {"additive_log2", BCM3HIP_APPLY_ADDITIVE_LOG2}, {"multiplicative", BCM3HIP_APPLY_MULTIPLICATIVE},
                {"multiplicative_log", BCM3HIP_APPLY_MULTIPLICATIVE_LOG},
                {"multiplicative_log2", BCM3HIP_APPLY_MULTIPLICATIVE_LOG2}, {"replace", BCM3HIP_APPLY_REPLACE}};
            auto it = apply.find(a);
            if (it == apply.end()) {
                LOGERROR("Unknown variability application type \"%s\"", a.c_str());
                return false;
            }
            x.apply = it->second;
            x.negate = v->get_bool("negate", false);
            if (!ParseRef(v->get("scale"), x.scale)) return false;
            vv.push_back(x);
        }
        variabilities.push_back(vv);
        std::vector<bcm3hip_value_ref> cov;
        if (dist == "full_gaussian") {
            // the covariance references covar_base_name + (j + 1) + "_" + (i + 1), j < i, resolved in
            // PostInitialize as a sampled variable or a number (ValueReference::Load)
            const std::string base_name = cv->get("covar_base_name");
            for (size_t i = 0; i < vv.size(); i++)
                for (size_t j = 0; j < i; j++) {
                    bcm3hip_value_ref r{};
                    if (!ParseRef(base_name + std::to_string(j + 1) + "_" + std::to_string(i + 1), r)) {
                        LOGERROR("Missing parameter for covariance");
                        return false;
                    }
                    cov.push_back(r);
                }
        }
        variability_full.push_back(dist == "full_gaussian" ? 1 : 0);
        variability_cov.push_back(cov);
    }
    if (!ParseRef(ex.get("entry_time"), entry_time)) return false;
    // synchronization_time_offset (Experiment::Initialize / PostInitialize, Experiment.cpp:172-185,
    // 619): a sampled variable; a number is written to fixed_entry_time in the reference (so it
    // replaces a constant entry time) and leaves the offset at 0
    sync_offset = bcm3hip_value_ref{BCM3HIP_REF_NONE, -1, 0.0};
    if (ex.has_attr("synchronization_time_offset") && !ex.get("synchronization_time_offset").empty()) {
        const std::string so = ex.get("synchronization_time_offset");
        const size_t ix = varset->GetVariableIndex(so, false);
        double v;
        if (ix != SIZE_MAX) {
            sync_offset = bcm3hip_value_ref{BCM3HIP_REF_VARIABLE, (int32_t)ix, 0.0};
        } else if (parse_double(so, v)) {
            if (entry_time.kind == BCM3HIP_REF_FIXED) entry_time.value = v;
        } else {
            LOGERROR("Synchronization time offset was specified as \"%s\", but could not find variable and also could not cast it to a constant real value",
                     so.c_str());
            return false;
        }
    }

    // data (DataLikelihoodBase::Load, DataLikelihoodTimeCourseBase::Load,
    // DataLikelihoodTimeCoursePopulationAverage::Load); the sidecar holds the netCDF group
    // {"<experiment>": {"<var>": {"dims": [...], "data": [...]}}}
    if (data_file.empty()) {
        LOGERROR("cell_population: a data_file is required");
        return false;
    }
    Json doc;
    try {
        doc = LoadDataFile(resolve(data_file, vm));
    } catch (JsonError& e) {
        LOGERROR("Failed to open data file %s: %s", data_file.c_str(), e.what.c_str());
        return false;
    }
    const Json* group = doc.find(name);
    if (!group) {
        LOGERROR("Group \"%s\" not found in %s", name.c_str(), data_file.c_str());
        return false;
    }
    for (const XmlNode* dn : ex.children_named("data")) {
        // DataLikelihoodBase::Create (DataLikelihoodBase.cpp:20-36): time_course by default
        const std::string type = dn->has_attr("type") ? dn->get("type") : std::string("time_course");
        DataLikelihood d;
        if (type == "time_course")
            d.kind = BCM3HIP_CP_DATA_TIME_COURSE;
        else if (type == "time_course_population_average")
            d.kind = BCM3HIP_CP_DATA_POPULATION_AVERAGE;
        else if (type == "time_points") {
            d.kind = BCM3HIP_CP_DATA_TIME_POINTS;
            if (!LoadTimePoints(*dn, d, *group, vm)) return false;
            data.push_back(d);
            continue;
        } else if (type == "duration") {
            // DataLikelihoodDuration::Evaluate fills likelihoods(i, count) but reads likelihoods(i, j)
            // with the simulated-cell index j (DataLikelihoodDuration.cpp:95-110): past its matrix
            LOGERROR("cell_population: data type \"duration\" is not supported (the reference reads past its likelihood matrix)");
            return false;
        } else {
            LOGERROR("Unknown data likelihood type \"%s\"", type.c_str());
            return false;
        }
        d.data_name = dn->get("data_name");
        d.weight = dn->get_double("weight", 1.0);
        const std::string em = dn->has_attr("error_model") ? dn->get("error_model") : std::string("normal");
        // DataLikelihoodBase::Load (src/cellpop/DataLikelihoodBase.cpp:51-70)
        if (em == "normal" || em == "additive_normal")
            d.error_model = BCM3HIP_CP_ERR_NORMAL;
        else if (em == "proportional_normal")
            d.error_model = BCM3HIP_CP_ERR_PROPORTIONAL;
        else if (em == "additive_proportional_normal")
            d.error_model = BCM3HIP_CP_ERR_ADDITIVE_PROPORTIONAL;
        else if (em == "student_t4" || em == "t4")
            d.error_model = BCM3HIP_CP_ERR_T4;
        else {
            LOGERROR("cell_population: error model \"%s\" is not supported", em.c_str());
            return false;
        }
        d.relative_to_time_average = (d.kind == BCM3HIP_CP_DATA_POPULATION_AVERAGE &&
                                      dn->get_bool("relative_to_time_average", false)) ? 1 : 0;
        d.stdev_relative_to_scale = dn->get_bool("stdev_relative_to_scale", false) ? 1 : 0;
        // include_only_cells_that_went_through_mitosis is read by DataLikelihoodTimeCourseBase::Load
        // but used by neither likelihood built here; the population average of this restatement
        // refuses it as before
        if (dn->get_bool("use_log_ratio", false) || dn->get_bool("optimize_offset_scale", false) ||
            (d.kind == BCM3HIP_CP_DATA_POPULATION_AVERAGE && dn->get_bool("include_only_cells_that_went_through_mitosis", false)) ||
            dn->has_attr("saturation_scale")) {
            LOGERROR("cell_population: unsupported option on data \"%s\"", d.data_name.c_str());
            return false;
        }
        if (d.kind == BCM3HIP_CP_DATA_TIME_COURSE) {
            // DataLikelihoodTimeCourse::Load (DataLikelihoodTimeCourse.cpp:27-41)
            if (!parse_sync(dn->has_attr("synchronize") ? dn->get("synchronize") : std::string(), d.sync)) return false;
            // missing_simulation_time_stdev (DataLikelihoodTimeCourseBase.cpp:93-110): a variable
            // or a number, 300 when absent
            d.missing_stdev = bcm3hip_value_ref{BCM3HIP_REF_FIXED, -1, 300.0};
            if (dn->has_attr("missing_simulation_time_stdev") && !dn->get("missing_simulation_time_stdev").empty() &&
                !ParseRef(dn->get("missing_simulation_time_stdev"), d.missing_stdev))
                return false;
        }
        if (!ParseRef(dn->get("stdev"), d.stdev)) return false;
        const std::string ps = dn->has_attr("proportional_stdev") ? dn->get("proportional_stdev") : std::string();
        if ((d.error_model == BCM3HIP_CP_ERR_PROPORTIONAL || d.error_model == BCM3HIP_CP_ERR_ADDITIVE_PROPORTIONAL) &&
            ps.empty()) {
            LOGERROR("Proportional error model is selected, but proportional stdev has not been specified.");
            return false;
        }
        // GetCurrentProportionalSTDev: 0 when not given
        d.proportional_stdev = bcm3hip_value_ref{BCM3HIP_REF_NONE, -1, 0.0};
        if (!ps.empty() && !ParseRef(ps, d.proportional_stdev)) return false;
        d.offset = bcm3hip_value_ref{BCM3HIP_REF_NONE, -1, 0.0};
        d.scale = bcm3hip_value_ref{BCM3HIP_REF_NONE, -1, 1.0};
        if (dn->has_attr("offset") && !ParseRef(dn->get("offset"), d.offset)) return false;
        if (dn->has_attr("scale") && !ParseRef(dn->get("scale"), d.scale)) return false;
        const Json* var = group->find(d.data_name);
        const Json* dims = var ? var->find("dims") : nullptr;
        const Json* values = var ? var->find("data") : nullptr;
        if (!dims || !values || dims->arr.empty()) {
            LOGERROR("Data \"%s\" not found in group \"%s\"", d.data_name.c_str(), name.c_str());
            return false;
        }
        const Json* tvar = group->find(dims->arr[0].str);
        const Json* tdata = tvar ? tvar->find("data") : nullptr;
        if (!tdata) {
            LOGERROR("Time dimension \"%s\" not found", dims->arr[0].str.c_str());
            return false;
        }
        for (const auto& t : tdata->arr) d.times.push_back(t.as_double());
        const size_t T = d.times.size();
        const size_t nd = dims->arr.size();
        if (d.kind == BCM3HIP_CP_DATA_POPULATION_AVERAGE) {
            if (nd > 2) {
                LOGERROR("Time course population likelihood for data %s; data has %zu dimensions but can only handle 1 or 2 dimensions.",
                         d.data_name.c_str(), nd);
                return false;
            }
            d.R = nd == 1 ? 1 : (int32_t)values->arr[0].arr.size();
            d.observed.assign((size_t)d.R * T, NaN);
            for (size_t i = 0; i < T && i < values->arr.size(); i++)
                for (int j = 0; j < d.R; j++)
                    d.observed[(size_t)j * T + i] = nd == 1 ? values->arr[i].as_double() : values->arr[i].arr[j].as_double();
        } else {
            // DataLikelihoodTimeCourse::Load (DataLikelihoodTimeCourse.cpp:43-130): time x cells
            // (x markers, of which one species reads the first); use_only_cell_ix picks cells
            if (nd < 1 || nd > 3) {
                LOGERROR("Time course likelihood for data %s; data has %zu dimensions but can only handle 1, 2 or 3 dimensions.",
                         d.data_name.c_str(), nd);
                return false;
            }
            const std::string only = option_get(vm, "cellpop.use_only_cell_ix", "-1");
            const size_t ncells_data = nd == 1 ? 1 : values->arr.empty() ? 0 : values->arr[0].arr.size();
            std::vector<size_t> pick;
            if (only == "-1") {
                for (size_t j = 0; j < ncells_data; j++) pick.push_back(j);
            } else {
                if (nd == 1) {
                    LOGERROR("use_only_cell_ix has been specified, but there is only 1 cell in the data.");
                    return false;
                }
                size_t p0 = 0;
                while (p0 <= only.size()) {
                    size_t p1 = only.find(',', p0);
                    if (p1 == std::string::npos) p1 = only.size();
                    const std::string tok = only.substr(p0, p1 - p0);
                    char* end = nullptr;
                    const long ix = strtol(tok.c_str(), &end, 10);
                    if (tok.empty() || *end || ix < 0) {
                        LOGERROR("cellpop.use_only_cell_ix: could not read \"%s\"", tok.c_str());
                        return false;
                    }
                    if ((size_t)ix >= ncells_data) {
                        LOGERROR("Requested to use cell %ld, but data contains only %zu cells", ix, ncells_data);
                        return false;
                    }
                    pick.push_back((size_t)ix);
                    p0 = p1 + 1;
                }
            }
            d.R = (int32_t)pick.size();
            d.observed.assign((size_t)d.R * T, NaN);
            for (size_t i = 0; i < T && i < values->arr.size(); i++)
                for (int j = 0; j < d.R; j++) {
                    const Json& row = values->arr[i];
                    d.observed[(size_t)j * T + i] = nd == 1   ? row.as_double()
                                                    : nd == 2 ? row.arr[pick[j]].as_double()
                                                              : row.arr[pick[j]].arr[0].as_double();
                }
            // observed lineage (DataLikelihoodTimeCourse.cpp:132-167): "parent" holds the parent's
            // "cell_id" (INT_MIN: none); children are kept per parent in ascending order
            if (const Json* par = group->find("parent")) {
                const Json* pd = par->find("data");
                const Json* idv = group->find("cell_id");
                const Json* id = idv ? idv->find("data") : nullptr;
                if (!pd || !id) {
                    LOGERROR("cell_population: data group \"%s\" has \"parent\" but no \"cell_id\"", name.c_str());
                    return false;
                }
                std::vector<long long> ids(d.R);
                for (int j = 0; j < d.R; j++) ids[j] = (long long)id->arr.at(pick[j]).as_double();
                std::vector<std::vector<int32_t>> children(d.R);
                d.roots.clear();
                for (int j = 0; j < d.R; j++) {
                    const long long p = (long long)pd->arr.at(pick[j]).as_double();
                    if (p != (long long)std::numeric_limits<int>::min()) {
                        const auto it = std::find(ids.begin(), ids.end(), p);
                        if (it == ids.end()) {
                            LOGERROR("Could not find cell %lld for parent of cell %d", p, j);
                            return false;
                        }
                        children[it - ids.begin()].push_back(j);
                    } else {
                        d.roots.push_back(j);
                    }
                }
                d.child_off.assign(1, 0);
                d.child_ix.clear();
                for (int j = 0; j < d.R; j++) {
                    d.child_ix.insert(d.child_ix.end(), children[j].begin(), children[j].end());
                    d.child_off.push_back((int32_t)d.child_ix.size());
                }
                // the device recursion is unrolled to 8 generations of observed cells
                std::function<int(int)> depth = [&](int c) {
                    int m = 0;
                    for (int32_t ch : children[c]) m = std::max(m, depth(ch));
                    return m + 1;
                };
                for (int32_t r : d.roots)
                    if (depth(r) > 8) {
                        LOGERROR("cell_population: observed lineages deeper than 8 generations are not supported");
                        return false;
                    }
                if (d.roots.size() != (size_t)d.R) {
                    // a cell in a parent cycle is nobody's descendant of a root: refuse
                    size_t reach = 0;
                    std::function<void(int)> walk = [&](int c) {
                        reach++;
                        for (int32_t ch : children[c]) walk(ch);
                    };
                    for (int32_t r : d.roots) walk(r);
                    if (reach != (size_t)d.R) {
                        LOGERROR("cell_population: the observed lineage of data \"%s\" has a parent cycle", d.data_name.c_str());
                        return false;
                    }
                }
            }
            if (max_cells < d.R) {
                LOGERROR("Maximum number of simulated cells (%d) in the experiment is not sufficient for the amount of cells in the data (%d)",
                         max_cells, d.R);
                return false;
            }
            if (max_cells > d.R) {
                LOGERROR("Simulating more cells (%d) than there are cells in the data (%d) - currently not supported.", max_cells, d.R);
                return false;
            }
            if (num_cells > max_cells || d.R > 1024) {
                LOGERROR("cell_population: time course with %d initial cells for %d observed cells (at most max_cells, 1024) is not supported",
                         num_cells, d.R);
                return false;
            }
        }
        // species reference (RequestSimulationInfo): ODE species, else constant species
        d.species_name = dn->get("species_name");
        size_t six = sbml.GetODEIntegratedSpeciesByName(d.species_name);
        if (six == SIZE_MAX) {
            LOGERROR("cell_population: \"%s\" is not an ODE-integrated species (sums, ratios and constant species are not supported)",
                     d.species_name.c_str());
            return false;
        }
        d.species_ix = (int32_t)six;
        data.push_back(d);
    }
    return true;
}

// DataLikelihoodBase::Load + DataLikelihoodTimePoints::Load (DataLikelihoodBase.cpp:38-75,
// DataLikelihoodTimePoints.cpp:19-201) and the per-column references of PostInitialize (:77-127)
bool LikelihoodCellPopulation::LoadTimePoints(const XmlNode& dn, DataLikelihood& d, const Json& group,
                                              const OptionsMap& vm) const
{
    d.data_name = dn.get("data_name");
    d.weight = dn.get_double("weight", 1.0);
    const std::string em = dn.has_attr("error_model") ? dn.get("error_model") : std::string("normal");
    if (em == "normal" || em == "additive_normal")
        d.error_model = BCM3HIP_CP_ERR_NORMAL;
    else if (em == "student_t4" || em == "t4")
        d.error_model = BCM3HIP_CP_ERR_T4;
    else if (em == "proportional_normal" || em == "additive_proportional_normal") {
        // Evaluate handles normal and t4 only; the other models give a NaN cell likelihood
        // (DataLikelihoodTimePoints.cpp:283-290, assert compiled out)
        LOGERROR("cell_population: time points data \"%s\": error model \"%s\" gives NaN cell likelihoods in the reference (not supported)",
                 d.data_name.c_str(), em.c_str());
        return false;
    } else {
        LOGERROR("Unknown error model \"%s\"", em.c_str());
        return false;
    }
    d.stdev_relative_to_scale = dn.get_bool("stdev_relative_to_scale", false) ? 1 : 0;
    d.only_nondivided = dn.get_bool("use_only_nondivided", false) ? 1 : 0;
    if (!parse_sync(dn.has_attr("synchronize") ? dn.get("synchronize") : std::string(), d.sync)) return false;
    // data: time x cells (x markers)
    const Json* var = group.find(d.data_name);
    const Json* dims = var ? var->find("dims") : nullptr;
    const Json* values = var ? var->find("data") : nullptr;
    if (!dims || !values || dims->arr.empty()) {
        LOGERROR("Data \"%s\" not found in group \"%s\"", d.data_name.c_str(), name.c_str());
        return false;
    }
    const size_t nd = dims->arr.size();
    if (nd != 2 && nd != 3) {
        LOGERROR("Need 2 or 3 dimensional data");
        return false;
    }
    const Json* tvar = group.find(dims->arr[0].str);
    const Json* tdata = tvar ? tvar->find("data") : nullptr;
    if (!tdata) {
        LOGERROR("Time dimension \"%s\" not found", dims->arr[0].str.c_str());
        return false;
    }
    d.times.clear();
    for (const auto& t : tdata->arr) d.times.push_back(t.as_double());
    const size_t T = d.times.size();
    if (T == 0 || values->arr.size() < T) {
        LOGERROR("Data \"%s\": fewer rows than time points", d.data_name.c_str());
        return false;
    }
    const size_t ncells_data = values->arr[0].arr.size();
    const std::string only = option_get(vm, "cellpop.use_only_cell_ix", "-1");
    std::vector<size_t> pick;
    if (only == "-1") {
        for (size_t j = 0; j < ncells_data; j++) pick.push_back(j);
    } else if (nd == 3) {
        LOGERROR("Not implemented yet");  // use_only_cell_ix on 3-D data (.cpp:112-114)
        return false;
    } else {
        for (const std::string& tok : tokenize(only, ',')) {
            char* end = nullptr;
            const long ix = strtol(tok.c_str(), &end, 10);
            if (tok.empty() || *end || ix < 0) {
                LOGERROR("cellpop.use_only_cell_ix: could not read \"%s\"", tok.c_str());
                return false;
            }
            if ((size_t)ix >= ncells_data) {
                LOGERROR("Requested to use cell %ld, but data contains only %zu cells", ix, ncells_data);
                return false;
            }
            pick.push_back((size_t)ix);
        }
    }
    d.R = (int32_t)pick.size();
    d.MK = nd == 3 ? (int32_t)(ncells_data ? values->arr[0].arr[0].arr.size() : 0) : 1;
    if (d.R < 1 || d.MK < 1) {
        LOGERROR("Data \"%s\" holds no cells", d.data_name.c_str());
        return false;
    }
    d.observed.assign((size_t)d.R * T * d.MK, NaN);
    for (size_t i = 0; i < T; i++)
        for (int j = 0; j < d.R; j++)
            for (int m = 0; m < d.MK; m++) {
                const Json& c = values->arr[i].arr[pick[j]];
                d.observed[((size_t)j * T + i) * d.MK + m] = nd == 2 ? c.as_double() : c.arr[m].as_double();
            }
    // species columns: "a;b" -> columns, "a+b" -> sums; a species is registered for simulation once,
    // at its first use (species_map, .cpp:139-188)
    d.species_name = dn.get("species_name");
    std::vector<std::string> cols;
    if (d.species_name.find(';') != std::string::npos) {
        for (const std::string& c : tokenize(d.species_name, ';')) cols.push_back(trim(c));
    } else {
        cols.push_back(d.species_name);
    }
    d.L = (int32_t)cols.size();
    d.term_offset.assign(1, 0);
    d.term_species.clear();
    d.species_order.clear();
    for (const std::string& col : cols) {
        std::vector<std::string> terms;
        if (col.find('+') != std::string::npos) {
            for (const std::string& t : tokenize(col, '+')) terms.push_back(trim(t));
        } else if (col.find('/') != std::string::npos) {
            LOGERROR("Division currently not supported for time points data");
            return false;
        } else {
            terms.push_back(col);
        }
        for (const std::string& t : terms) {
            const size_t six = sbml.GetODEIntegratedSpeciesByName(t);
            if (six == SIZE_MAX) {
                if (sbml.GetConstantSpeciesByName(t) == SIZE_MAX)
                    LOGERROR("Could not find species \"%s\" as either an dynamic or constant species", t.c_str());
                else
                    LOGERROR("cell_population: time points of the constant species \"%s\" are not supported", t.c_str());
                return false;
            }
            d.term_species.push_back((int32_t)six);
            if (std::find(d.species_order.begin(), d.species_order.end(), (int32_t)six) == d.species_order.end())
                d.species_order.push_back((int32_t)six);
        }
        d.term_offset.push_back((int32_t)d.term_species.size());
    }
    // Evaluate reads observed(i, l) for l < L: the data need that many markers
    if (d.L > 8) {
        LOGERROR("cell_population: time points data \"%s\" with %d species columns (at most 8) are not supported",
                 d.data_name.c_str(), d.L);
        return false;
    }
    if (d.L > d.MK) {
        LOGERROR("cell_population: time points data \"%s\" has %d marker(s) for %d species columns", d.data_name.c_str(),
                 d.MK, d.L);
        return false;
    }
    if (max_cells < d.R) {
        LOGERROR("Maximum number of simulated cells (%d) in the experiment is not sufficient for the amount of cells in the data (%d)",
                 max_cells, d.R);
        return false;
    }
    if (d.R > 1024) {
        LOGERROR("cell_population: time points with %d observed cells (at most 1024) are not supported", d.R);
        return false;
    }
    // value_relative_to_timepoint_ix (DataLikelihoodBase.cpp:49): a time point index of these data
    d.relative_ix = -1;
    if (dn.has_attr("value_relative_to_timepoint_ix")) {
        const std::string s = dn.get("value_relative_to_timepoint_ix");
        char* end = nullptr;
        const long ix = strtol(s.c_str(), &end, 10);
        if (s.empty() || *end || ix < 0 || (size_t)ix >= T) {
            LOGERROR("cell_population: value_relative_to_timepoint_ix \"%s\" is not a time point of data \"%s\"", s.c_str(),
                     d.data_name.c_str());
            return false;
        }
        d.relative_ix = (int32_t)ix;
    }
    // stdev / offset / scale: one value for every column or one per column (GetCurrentSTDev & co.,
    // DataLikelihoodBase.cpp:130-215: an index past a longer list gives NaN)
    auto refs = [&](const std::string& attr, bcm3hip_value_ref none, int slot) {
        const std::string s = dn.has_attr(attr) ? dn.get(attr) : std::string();
        const std::vector<std::string> toks = tokenize(s, ';');
        for (int l = 0; l < d.L; l++) {
            bcm3hip_value_ref r = none;
            if (toks.size() == 1) {
                if (!ParseRef(toks[0], r)) return false;
            } else if ((size_t)l < toks.size()) {
                if (!ParseRef(toks[l], r)) return false;
            } else if (!toks.empty()) {
                r = bcm3hip_value_ref{BCM3HIP_REF_FIXED, -1, NaN};
            }
            d.col_ref[(size_t)l * 3 + slot] = r;
        }
        for (size_t k = (size_t)d.L; k < toks.size(); k++) {  // parsed by PostInitialize all the same
            bcm3hip_value_ref r;
            if (!ParseRef(toks[k], r)) return false;
        }
        return true;
    };
    d.col_ref.assign((size_t)d.L * 3, bcm3hip_value_ref{BCM3HIP_REF_NONE, -1, 0.0});
    if (!dn.has_attr("stdev")) {
        LOGERROR("cell_population: data \"%s\" needs a stdev", d.data_name.c_str());
        return false;
    }
    if (!refs("stdev", bcm3hip_value_ref{BCM3HIP_REF_NONE, -1, 0.0}, 0) ||
        !refs("offset", bcm3hip_value_ref{BCM3HIP_REF_NONE, -1, 0.0}, 1) ||
        !refs("scale", bcm3hip_value_ref{BCM3HIP_REF_NONE, -1, 1.0}, 2))
        return false;
    d.stdev = d.col_ref[0];
    d.offset = d.col_ref[1];
    d.scale = d.col_ref[2];
    d.proportional_stdev = bcm3hip_value_ref{BCM3HIP_REF_NONE, -1, 0.0};
    d.missing_stdev = bcm3hip_value_ref{BCM3HIP_REF_NONE, -1, 0.0};
    d.species_ix = d.term_species[0];
    return true;
}

// Experiment::PostInitialize (Experiment.cpp:145-237) + the flat device model
std::vector<const bcm3hip_cellpop_model*> LikelihoodCellPopulation::GetDeviceModels() const
{
    std::vector<const bcm3hip_cellpop_model*> v{&model};
    for (const auto& e : more_experiments) v.push_back(&e->model);
    return v;
}

bool LikelihoodCellPopulation::PostInitialize()
{
    for (auto& e : more_experiments)
        if (!e->PostInitialize()) return false;
    std::string err;
    if (!sbml.GenerateDerivative(varset->GetVariableNames(), forced, derivative_body, err)) {
        LOGERROR("%s", err.c_str());
        return false;
    }
    const size_t NS = sbml.GetNumODEIntegratedSpecies(), NC = sbml.GetNumConstantSpecies();
    if (NS < 1 || NS > 64) {
        LOGERROR("cell_population: %zu ODE species (1..64 supported)", NS);
        return false;
    }
    // simulation time points: (data likelihood, time, time index, species), sorted stably by time
    // (time points data: one run per species in first-use order, DataLikelihoodTimePoints.cpp:139-188)
    struct TP {
        int dl;
        double t;
        int ti;
        int species;
        int order;
        int sync;
    };
    std::vector<TP> tps;
    for (size_t k = 0; k < data.size(); k++) {
        const DataLikelihood& d = data[k];
        if (d.kind == BCM3HIP_CP_DATA_TIME_POINTS) {
            for (size_t o = 0; o < d.species_order.size(); o++)
                for (size_t i = 0; i < d.times.size(); i++)
                    tps.push_back(TP{(int)k, d.times[i], (int)i, d.species_order[o], (int)o, d.sync});
        } else {
            for (size_t i = 0; i < d.times.size(); i++) tps.push_back(TP{(int)k, d.times[i], (int)i, d.species_ix, 0, d.sync});
        }
        // a synchronised course also simulates its full duration, for negative time points
        // (DataLikelihoodTimeCourse.cpp:192-199, DataLikelihoodTimePoints.cpp:190-197): an entry
        // without species
        if (d.sync != BCM3HIP_CP_SYNC_NONE && !d.times.empty()) {
            const double last_tp = d.times.back(), full_duration = last_tp - d.times.front();
            if (full_duration > last_tp) tps.push_back(TP{(int)k, full_duration, -1, -1, 0, d.sync});
        }
    }
    std::stable_sort(tps.begin(), tps.end(), [](const TP& a, const TP& b) { return a.t < b.t; });
    if (tps.empty()) {
        LOGERROR("cell_population: no data time points");
        return false;
    }
    output_times.clear();
    output_species.clear();
    output_sync.clear();
    std::vector<std::vector<int32_t>> order_entry(data.size());  // time points: [order][T]
    for (size_t k = 0; k < data.size(); k++) {
        data[k].entry.assign(data[k].times.size(), -1);
        order_entry[k].assign(std::max<size_t>(1, data[k].species_order.size()) * data[k].times.size(), -1);
    }
    for (size_t k = 0; k < tps.size(); k++) {
        output_times.push_back(tps[k].t);
        output_species.push_back(tps[k].species);
        output_sync.push_back(tps[k].sync);
        if (tps[k].ti < 0) continue;
        DataLikelihood& d = data[tps[k].dl];
        if (d.kind == BCM3HIP_CP_DATA_TIME_POINTS)
            order_entry[tps[k].dl][(size_t)tps[k].order * d.times.size() + tps[k].ti] = (int32_t)k;
        else
            d.entry[tps[k].ti] = (int32_t)k;
    }
    // a column's terms are summed in the order their values are notified: the order of the entries
    // (DataLikelihoodTimePoints::NotifySimulatedValue, .cpp:345-370, over the sorted time points)
    for (size_t k = 0; k < data.size(); k++) {
        DataLikelihood& d = data[k];
        if (d.kind != BCM3HIP_CP_DATA_TIME_POINTS) continue;
        const size_t T = d.times.size();
        d.term_entry.assign(d.term_species.size() * T, -1);
        for (int l = 0; l < d.L; l++) {
            std::vector<int32_t> ord;
            for (int q = d.term_offset[l]; q < d.term_offset[l + 1]; q++)
                ord.push_back((int32_t)(std::find(d.species_order.begin(), d.species_order.end(), d.term_species[q]) -
                                        d.species_order.begin()));
            std::stable_sort(ord.begin(), ord.end());  // entries at one time follow the species order
            for (size_t q = 0; q < ord.size(); q++)
                for (size_t i = 0; i < T; i++)
                    d.term_entry[(d.term_offset[l] + q) * T + i] = order_entry[k][(size_t)ord[q] * T + i];
        }
        for (size_t i = 0; i < T; i++) d.entry[i] = d.term_entry[i];
    }
    transforms.clear();
    for (size_t i = 0; i < varset->GetNumVariables(); i++) transforms.push_back((int32_t)varset->GetVariableTransform(i));
    y_init.clear();
    for (size_t i = 0; i < NS; i++) y_init.push_back(sbml.GetODEIntegratedSpecies(i).initial);
    constant_init.clear();
    for (size_t i = 0; i < NC; i++) constant_init.push_back(sbml.GetConstantSpecies(i).initial);
    // daughters (Cell::SetInitialConditionsFromOtherCell, Cell.cpp:127-133): these species must exist
    reset_index.clear();
    reset_value.clear();
    if (divide_cells) {
        const std::pair<const char*, double> resets[] = {{"cytokinesis", 0.0}, {"nuclear_envelope", 1.0}, {"G1S_break", 1.0},
                                                         {"G2_break", 1.0}, {"spindle_components", 0.0},
                                                         {"assembled_spindle", 0.0}, {"chromatid_separation", 0.0}};
        for (auto& r : resets) {
            const size_t ix = sbml.GetODEIntegratedSpeciesByName(r.first);
            if (ix == SIZE_MAX) {
                LOGERROR("cell_population: dividing cells need an ODE species \"%s\" (Cell.cpp:127-133)", r.first);
                return false;
            }
            reset_index.push_back((int32_t)ix);
            reset_value.push_back(r.second);
        }
    }
    // event species: SIMULATED-species indices applied to the ODE state, as Cell's constructor
    // looks them up (Cell.cpp:44-50) and integration_step_cb reads them (:467-533)
    const char* ev_names[7] = {"replicating_DNA", "replicated_DNA", "PCNA_gfp", "nuclear_envelope",
                               "chromatid_separation", "cytokinesis", "apoptosis"};
    int32_t events[7];
    for (int k = 0; k < 7; k++) {
        const size_t ix = sbml.GetSimulatedSpeciesByName(ev_names[k]);
        events[k] = ix == SIZE_MAX ? -1 : (int32_t)ix;
    }
    // variabilities: Sobol table, per-dimension scales, application list in Cell::Initialize order
    scales.clear();
    actions.clear();
    full_groups.clear();
    covariance.clear();
    int dim0 = 0;
    for (size_t g = 0; g < variabilities.size(); g++) {
        const auto& vv = variabilities[g];
        if (variability_full[g]) {
            full_groups.push_back(dim0);
            full_groups.push_back((int32_t)vv.size());
            covariance.insert(covariance.end(), variability_cov[g].begin(), variability_cov[g].end());
        }
        // an entry_time variable takes its dimension of the pseudorandom vector (GetPseudorandomVector
        // covers every variable) but changes nothing: the reference never calls
        // ApplyVariabilityEntryTime (VariabilityDescriptionVariable.cpp:66-78; Cell::Initialize,
        // Cell.cpp:150-176, applies parameters and initial conditions only), so it gets no action
        for (size_t k = 0; k < vv.size(); k++) scales.push_back(vv[k].scale);
        for (size_t i = 0; i < varset->GetNumVariables(); i++)
            for (size_t k = 0; k < vv.size(); k++)
                if (!vv[k].parameter.empty() && vv[k].parameter == varset->GetVariableName(i))
                    actions.push_back(bcm3hip_variability_action{dim0 + (int32_t)k, 0, (int32_t)i, vv[k].apply, vv[k].negate,
                                                                 vv[k].only_initial});
        for (size_t i = 0; i < NS; i++)
            for (size_t k = 0; k < vv.size(); k++)
                if (!vv[k].species.empty() && vv[k].species == sbml.GetODEIntegratedSpecies(i).name)
                    actions.push_back(bcm3hip_variability_action{dim0 + (int32_t)k, 1, (int32_t)i, vv[k].apply, vv[k].negate,
                                                                 vv[k].only_initial});
        for (size_t k = 0; k < vv.size(); k++) {
            if (!vv[k].parameter.empty() && varset->GetVariableIndex(vv[k].parameter, false) == SIZE_MAX) {
                LOGERROR("Variability has been specified for parameter \"%s\", but the parameter is not sampled",
                         vv[k].parameter.c_str());
                return false;
            }
            if (!vv[k].species.empty() && sbml.GetODEIntegratedSpeciesByName(vv[k].species) == SIZE_MAX) {
                LOGERROR("Could not find species \"%s\"", vv[k].species.c_str());
                return false;
            }
        }
        dim0 += (int)vv.size();
    }
    const int sobol_points = scales.empty() ? 0 : num_cells * 100;
    sobol = SobolPoints(sobol_points, scales.size());

    // treatment trajectories: the species must be a constant species (Experiment.cpp:573-577); every
    // cell must see its own first discontinuity: the reference's solver keeps the last one across the
    // cells of its pool when a cell sets none (ODESolver::SetDiscontinuity is skipped, Cell.cpp:226),
    // which this restatement does not reproduce, so pulses must run past the experiment's end
    treat_species.clear();
    for (size_t i = 0; i < treat_names.size(); i++) {
        const size_t ix = sbml.GetConstantSpeciesByName(treat_names[i]);
        if (ix == SIZE_MAX) {
            LOGERROR("Cannot find \"%s\" as a constant species for treatment trajectory (the species needs to be constant).",
                     treat_names[i].c_str());
            return false;
        }
        treat_species.push_back((int32_t)ix);
        const int n = treat_offset[i + 1] - treat_offset[i];
        if (n == 0 || treat_times[treat_offset[i + 1] - 1] + 14.0 <= output_times.back() + trailing) {
            LOGERROR("Treatment trajectory for \"%s\": the pulses end before the experiment does; cells created after "
                     "the last pulse would inherit another cell's solver discontinuity in the reference (not supported)",
                     treat_names[i].c_str());
            return false;
        }
    }
    data_flat.clear();
    for (const auto& d : data) {
        const bool tp = d.kind == BCM3HIP_CP_DATA_TIME_POINTS;
        data_flat.push_back(bcm3hip_cellpop_data{(int32_t)d.times.size(), d.R, d.observed.data(), d.entry.data(), d.stdev,
                                                 d.offset, d.scale, d.weight, d.error_model,
                                                 d.proportional_stdev, d.relative_to_time_average, d.kind,
                                                 d.stdev_relative_to_scale, d.missing_stdev, tp ? d.L : 0,
                                                 tp ? d.MK : 0, tp ? d.term_offset.data() : nullptr,
                                                 tp ? d.term_entry.data() : nullptr, tp ? d.col_ref.data() : nullptr,
                                                 tp ? d.relative_ix : -1, tp ? d.only_nondivided : 0,
                                                 (int32_t)d.roots.size(), d.roots.data(), d.child_off.data(),
                                                 d.child_ix.data()});
    }
    model = bcm3hip_cellpop_model{};
    model.derivative_body = derivative_body.c_str();
    model.NS = (int32_t)NS;
    model.NC = (int32_t)NC;
    model.d = (int32_t)varset->GetNumVariables();
    model.M = (int32_t)output_times.size();
    model.transforms = transforms.data();
    model.y_init = y_init.data();
    model.constant_species = constant_init.data();
    model.output_times = output_times.data();
    model.output_species = output_species.data();
    model.output_sync = output_sync.data();
    model.sync_offset = sync_offset;
    // a sampled synchronization_time_offset without synchronised data: the reference then reads every
    // value by an exact-time lookup at data time + offset among the cell's output times
    // (Cell.cpp:328-335), which misses (NaN) unless the offset happens to be 0 -- refused, not restated
    if (sync_offset.kind == BCM3HIP_REF_VARIABLE &&
        std::all_of(output_sync.begin(), output_sync.end(), [](int32_t x) { return x == BCM3HIP_CP_SYNC_NONE; })) {
        LOGERROR("cell_population: a sampled synchronization_time_offset needs synchronised data (without it the reference's exact-time lookups at data time + offset return NaN); not supported");
        return false;
    }
    model.solver = solver;
    model.hmax = hmax;
    // DP5 (ODESolverDP5.cpp): GetInterpolatedY and get_threshold_crossing_time are not implemented in
    // the reference (NaN, ASSERT compiled out), so synchronised data would read NaN everywhere; its
    // discontinuity handling (:123-135, 239-254) is not built here
    if (solver == BCM3HIP_CP_SOLVER_DP5) {
        for (int32_t x : output_sync)
            if (x != BCM3HIP_CP_SYNC_NONE) {
                LOGERROR("cell_population: synchronised data with solver_type DP5 (the reference's DP5 solver does not implement GetInterpolatedY) is not supported");
                return false;
            }
        if (!treat_species.empty()) {
            LOGERROR("cell_population: treatment trajectories with solver_type DP5 are not supported");
            return false;
        }
    }
    model.rtol = rtol;
    model.atol = atol;
    model.hmin = hmin;
    model.max_steps = max_steps;
    model.divide_cells = divide_cells ? 1 : 0;
    model.end_time = output_times.back() + trailing;
    model.past_cs = past_cs;
    for (int k = 0; k < 7; k++) model.events[k] = events[k];
    model.n_reset = (int32_t)reset_index.size();
    model.reset_index = reset_index.data();
    model.reset_value = reset_value.data();
    model.num_cells = num_cells;
    model.max_cells = max_cells;
    model.entry_time = entry_time;
    model.sobol_dims = (int32_t)scales.size();
    model.sobol_points = sobol_points;
    model.sobol = sobol.data();
    model.scales = scales.data();
    model.n_actions = (int32_t)actions.size();
    model.actions = actions.data();
    model.n_full = (int32_t)(full_groups.size() / 2);
    model.full_groups = full_groups.data();
    model.covariance = covariance.data();
    model.n_data = (int32_t)data_flat.size();
    model.data = data_flat.data();
    model.n_treat = (int32_t)treat_species.size();
    model.treat_species = treat_species.data();
    model.treat_offset = treat_offset.data();
    model.treat_times = treat_times.data();
    if (host_only) return true;
    std::vector<bcm3hip_cellpop_model> models{model};
    for (const auto& e : more_experiments) models.push_back(e->model);
    const int r = bcm3hip_open_cellpop_experiments(device, models.data(), (int)models.size(), &ctx);
    if (r) {
        LOGERROR("bcm3hip_open_cellpop failed: %s", bcm3hip_error_string(r));
        return false;
    }
    return true;
}

}  // namespace bcm3
