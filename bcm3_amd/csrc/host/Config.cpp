// Config.cpp -- see Config.h
#include "Config.h"

#include <algorithm>
#include <cctype>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <fstream>
#include <limits>

#include "../../../include/bcm3.h"
#include "log.h"

namespace bcm3 {

namespace {

std::string Trim(const std::string& s)
{
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) a++;
    while (b > a && std::isspace((unsigned char)s[b - 1])) b--;
    return s.substr(a, b - a);
}

std::string Lower(std::string s)
{
    for (auto& c : s) c = (char)std::tolower((unsigned char)c);
    return s;
}

// boost::program_options' bool validator: "", on, yes, 1, true -> true; off, no, 0, false -> false
bool ParseBool(const std::string& v, bool& out)
{
    const std::string s = Lower(v);
    if (s.empty() || s == "on" || s == "yes" || s == "1" || s == "true") {
        out = true;
        return true;
    }
    if (s == "off" || s == "no" || s == "0" || s == "false") {
        out = false;
        return true;
    }
    return false;
}

// lexical_cast of the whole text (no trailing characters)
bool ParseReal(const std::string& v, double& out)
{
    if (v.empty()) return false;
    char* end = nullptr;
    out = std::strtod(v.c_str(), &end);
    return end && *end == '\0';
}

bool ParseUnsigned(const std::string& v, uint64_t& out)
{
    if (v.empty() || v[0] == '-') return false;  // a negative size_t is refused here, not wrapped
    char* end = nullptr;
    errno = 0;
    out = std::strtoull(v.c_str(), &end, 10);
    return end && *end == '\0' && errno == 0;
}

bool ParseInt(const std::string& v, int64_t& out)
{
    if (v.empty()) return false;
    char* end = nullptr;
    errno = 0;
    out = std::strtoll(v.c_str(), &end, 10);
    return end && *end == '\0' && errno == 0;
}

}  // namespace

ConfigFile::ConfigFile()
{
    struct Opt {
        const char* key;
        Kind kind;
        const char* def;
    };
    static const Opt opts[] = {
        // bcminf (src/bcminf/main.cpp:294-307)
        {"sampling_threads", SIZE, "0"},
        {"evaluation_threads", SIZE, "1"},
        {"prior", STRING, "prior.xml"},
        {"likelihood", STRING, "likelihood.xml"},
        {"learning_rate", REAL, "1.0"},
        {"output.folder", STRING, "output"},
        {"predict", STRING, ""},
        {"predict.input", STRING, "output.nc"},
        {"predict.output", STRING, "prediction.nc"},
        {"predict.skip_n", SIZE, "0"},
        {"predict.specific_temperature", SIZE, "18446744073709551615"},
        {"progress_update_time", REAL, "0.5"},
        // SamplerFactory / Sampler (SamplerFactory.cpp:42-44, Sampler.cpp:144-148)
        {"sampler.type", STRING, "ptmh"},
        {"sampler.num_samples", SIZE, "2500"},
        {"sampler.use_every_nth", SIZE, "1"},
        {"sampler.rngseed", U64, "0"},
        // SamplerPT (SamplerPT.cpp:149-170)
        {"ptmhsampler.num_chains", SIZE, "6"},
        {"ptmhsampler.blocking_strategy", STRING, "one_block"},
        {"ptmhsampler.proposal_type", STRING, "gaussian_mixture"},
        {"ptmhsampler.proposal_transform_to_unbounded", BOOL, "false"},
        {"ptmhsampler.adapt_proposal_samples", SIZE, "2000"},
        {"ptmhsampler.adapt_proposal_times", SIZE, "2"},
        {"ptmhsampler.max_history_size", SIZE, "2000"},
        {"ptmhsampler.adapt_proposal_max_history_samples", SIZE, "2000"},
        {"ptmhsampler.adapt_proposal_max_clustering_samples", SIZE, "1000"},
        {"ptmhsampler.stop_proposal_scaling", SIZE, "6000"},
        {"ptmhsampler.sample_clustering_kernel_nn", SIZE, "3"},
        {"ptmhsampler.sample_clustering_kernel_nn2", SIZE, "7"},
        {"ptmhsampler.sample_clustering_num_clusters", SIZE, "4"},
        {"ptmhsampler.swapping_scheme", STRING, "deterministic_even_odd"},
        {"ptmhsampler.exchange_probability", REAL, "0.5"},
        {"ptmhsampler.num_exploration_steps", SIZE, "1"},
        {"ptmhsampler.temperature_schedule_power", REAL, "3.0"},
        {"ptmhsampler.temperature_schedule_max", REAL, "1.0"},
        {"ptmhsampler.output_proposal_adaptation", BOOL, "false"},
        {"ptmhsampler.proposal_t_dof", REAL, "0.0"},
        {"ptmhsampler.initial_position_tries", SIZE, "100"},
        // LikelihoodFactory (LikelihoodFactory.cpp:103-111): CellPopulationLikelihood.cpp:116,
        // LikelihoodCellCycleMarker.cpp:95, LikelihoodPharmacokineticTrajectory.cpp:617,
        // PharmacoLikelihoodSingle.cpp:234
        {"cellpop.use_only_cell_ix", STRING, "-1"},
        {"ccm.track_ix", INT, "0"},
        {"pk.patient", STRING, ""},
        {"pharmacosingle.patient", STRING, ""},
    };
    for (const Opt& o : opts) {
        kinds_[o.key] = o.kind;
        values_[o.key] = o.def;
    }
}

bool ConfigFile::Store(const std::string& key, const std::string& value, int line)
{
    auto k = kinds_.find(key);
    if (k == kinds_.end()) {
        LOGERROR("config file line %d: unrecognised option '%s'", line, key.c_str());
        return false;
    }
    if (set_.count(key)) {
        LOGERROR("config file line %d: option '%s' cannot be specified more than once (first on line %d)", line,
                 key.c_str(), set_[key]);
        return false;
    }
    bool okv = true, b;
    double r;
    uint64_t u;
    int64_t i;
    switch (k->second) {
    case STRING: break;
    case SIZE:
    case U64: okv = ParseUnsigned(value, u); break;
    case INT: okv = ParseInt(value, i); break;
    case REAL: okv = ParseReal(value, r); break;
    case BOOL: okv = ParseBool(value, b); break;
    }
    if (!okv) {
        LOGERROR("config file line %d: the argument ('%s') for option '%s' is invalid", line, value.c_str(), key.c_str());
        return false;
    }
    values_[key] = value;
    set_[key] = line;
    return true;
}

bool ConfigFile::Load(const std::string& path)
{
    std::ifstream f(path);
    if (!f) {
        LOGERROR("Could not open config file \"%s\"", path.c_str());
        return false;
    }
    // boost::program_options::detail::common_config_file_iterator: '#' starts a comment anywhere
    // on a line; "[section]" prefixes the following names with "section."; "name = value"
    std::string line, prefix;
    int ln = 0;
    while (std::getline(f, line)) {
        ln++;
        const size_t hash = line.find('#');
        if (hash != std::string::npos) line.erase(hash);
        line = Trim(line);
        if (line.empty()) continue;
        if (line.front() == '[' && line.back() == ']') {
            prefix = Trim(line.substr(1, line.size() - 2));
            if (!prefix.empty()) prefix += '.';
            continue;
        }
        const size_t eq = line.find('=');
        if (eq == std::string::npos) {
            LOGERROR("config file line %d: invalid syntax '%s'", ln, line.c_str());
            return false;
        }
        const std::string name = Trim(line.substr(0, eq)), value = Trim(line.substr(eq + 1));
        if (name.empty()) {
            LOGERROR("config file line %d: invalid syntax '%s'", ln, line.c_str());
            return false;
        }
        if (!Store(prefix + name, value, ln)) return false;
    }
    return true;
}

const std::string& ConfigFile::String(const std::string& key) const { return values_.at(key); }

double ConfigFile::Real(const std::string& key) const
{
    double r = 0.0;
    ParseReal(values_.at(key), r);
    return r;
}

int64_t ConfigFile::Int(const std::string& key) const
{
    const std::string& v = values_.at(key);
    if (kinds_.at(key) == INT) {
        int64_t i = 0;
        ParseInt(v, i);
        return i;
    }
    uint64_t u = 0;
    ParseUnsigned(v, u);
    return (u > (uint64_t)std::numeric_limits<int64_t>::max()) ? std::numeric_limits<int64_t>::max() : (int64_t)u;
}

uint64_t ConfigFile::ULL(const std::string& key) const
{
    uint64_t u = 0;
    ParseUnsigned(values_.at(key), u);
    return u;
}

bool ConfigFile::Bool(const std::string& key) const
{
    bool b = false;
    ParseBool(values_.at(key), b);
    return b;
}

bool LoadRunConfig(const std::string& path, RunConfig& out)
{
    ConfigFile cf;
    if (!cf.Load(path)) return false;
    RunConfig rc;
    PTMHConfig& p = rc.ptmh;

    // SamplerFactory::Create (SamplerFactory.cpp:10-37)
    rc.sampler_type = cf.String("sampler.type");
    if (rc.sampler_type != "ptmh" && rc.sampler_type != "parallel_tempered_Metropolis_Hastings") {
        if (rc.sampler_type == "is" || rc.sampler_type == "importance_sampling")
            LOGERROR("sampler.type \"%s\": importance sampling is not part of this PT-MH path", rc.sampler_type.c_str());
        else
            LOGERROR("Unknown sampler type \"%s\"", rc.sampler_type.c_str());
        return false;
    }
    // Sampler::LoadSettings (Sampler.cpp:55-62) + seeding (:91-94): 0 = a time-based seed
    rc.num_samples = cf.Int("sampler.num_samples");
    p.use_every_nth = (int)std::min<int64_t>(cf.Int("sampler.use_every_nth"), std::numeric_limits<int>::max());
    p.seed = cf.ULL("sampler.rngseed");
    if (p.seed == 0) {
        p.seed = (uint64_t)std::chrono::high_resolution_clock::now().time_since_epoch().count();
        LOG("sampler.rngseed = 0: using the time-based seed %llu", (unsigned long long)p.seed);
    }

    // SamplerPT::LoadSettings (SamplerPT.cpp:40-95)
    const std::string blocking = cf.String("ptmhsampler.blocking_strategy");
    if (blocking != "one_block") {
        LOGERROR("ptmhsampler.blocking_strategy \"%s\": only one_block is built (DESIGN.md §8)", blocking.c_str());
        return false;
    }
    if (cf.Bool("ptmhsampler.proposal_transform_to_unbounded")) {
        // Proposal::Initialize asserts !transform_to_unbounded (Proposal.cpp:131-135)
        LOGERROR("ptmhsampler.proposal_transform_to_unbounded = true is not supported (the reference asserts it off)");
        return false;
    }
    // SamplerPTChain::CreateProposalInstance (SamplerPTChain.cpp:428-444)
    const std::string prop = cf.String("ptmhsampler.proposal_type");
    if (prop == "global_covariance") {
        p.proposal = BCM3_PTMH_GLOBAL_COVARIANCE;
    } else if (prop == "gaussian_mixture") {
        p.proposal = BCM3_PTMH_GAUSSIAN_MIXTURE;
    } else if (prop == "gaussian_mixture_adjustedAIC") {
        p.proposal = BCM3_PTMH_GAUSSIAN_MIXTURE_ADJUSTED_AIC;
    } else if (prop == "gaussian_mixture_fit_in_r" || prop == "clustered_covariance") {
        LOGERROR("ptmhsampler.proposal_type \"%s\" is not built here (DESIGN.md §8)", prop.c_str());
        return false;
    } else {
        LOGERROR("Unknown proposal type \"%s\"", prop.c_str());
        return false;
    }
    const std::string scheme = cf.String("ptmhsampler.swapping_scheme");
    if (scheme == "stochastic_random") {
        p.swapping_scheme = BCM3_PTMH_STOCHASTIC_RANDOM;
    } else if (scheme == "stochastic_even_odd") {
        p.swapping_scheme = BCM3_PTMH_STOCHASTIC_EVEN_ODD;
    } else if (scheme == "deterministic_even_odd") {
        p.swapping_scheme = BCM3_PTMH_DETERMINISTIC_EVEN_ODD;
    } else {
        LOGERROR("Unknown swapping scheme \"%s\"", scheme.c_str());
        return false;
    }
    auto as_int = [&](const char* key, int& dst) {
        const int64_t v = cf.Int(key);
        if (v > std::numeric_limits<int>::max()) {
            LOGERROR("%s = %lld is out of range", key, (long long)v);
            return false;
        }
        dst = (int)v;
        return true;
    };
    const int64_t chains = cf.Int("ptmhsampler.num_chains");
    if (chains < 1) {
        LOGERROR("ptmhsampler.num_chains must be at least 1");
        return false;
    }
    p.num_chains = chains;
    if (!as_int("ptmhsampler.adapt_proposal_samples", p.adapt_proposal_samples) ||
        !as_int("ptmhsampler.adapt_proposal_times", p.adapt_proposal_times) ||
        !as_int("ptmhsampler.max_history_size", p.max_history_size) ||
        !as_int("ptmhsampler.adapt_proposal_max_history_samples", p.adapt_proposal_max_history_samples) ||
        !as_int("ptmhsampler.num_exploration_steps", p.exploration_steps) ||
        !as_int("ptmhsampler.initial_position_tries", p.initial_position_tries))
        return false;
    p.exchange_probability = cf.Real("ptmhsampler.exchange_probability");
    p.temperature_power = cf.Real("ptmhsampler.temperature_schedule_power");
    p.temperature_max = cf.Real("ptmhsampler.temperature_schedule_max");
    p.t_dof = cf.Real("ptmhsampler.proposal_t_dof");
    rc.output_proposal_adaptation = cf.Bool("ptmhsampler.output_proposal_adaptation");

    // bcminf (main.cpp:47-58, 83-121): learning rate to the sampler, file names, threads
    p.learning_rate = cf.Real("learning_rate");
    rc.sampling_threads = cf.Int("sampling_threads");
    rc.evaluation_threads = cf.Int("evaluation_threads");
    if (rc.sampling_threads > 0) p.host_threads = (int)std::min<int64_t>(rc.sampling_threads, 1024);
    rc.prior = cf.String("prior");
    rc.likelihood = cf.String("likelihood");
    rc.output_folder = cf.String("output.folder");

    // the likelihood factory's options, as bcm3_likelihood_create_ex's "key=value;..." string:
    // only those the file sets (the likelihoods apply the same defaults themselves)
    for (const char* key : {"pk.patient", "pharmacosingle.patient", "cellpop.use_only_cell_ix", "ccm.track_ix"}) {
        if (!cf.Set(key)) continue;
        const std::string& v = cf.String(key);
        if (v.find(';') != std::string::npos) {
            LOGERROR("%s: ';' is not allowed in a likelihood option value", key);
            return false;
        }
        if (!rc.likelihood_options.empty()) rc.likelihood_options += ';';
        rc.likelihood_options += std::string(key) + "=" + v;
    }
    out = rc;
    return true;
}

}  // namespace bcm3
