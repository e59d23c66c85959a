// Config.h -- bcminf's configuration file (config.txt) for the PT-MH path.
//
// The reference parses config.txt with boost::program_options::parse_config_file against the
// options registered by bcminf (src/bcminf/main.cpp:293-320), the sampler factory
// (src/sampler/SamplerFactory.cpp:40-49), Sampler (Sampler.cpp:142-149), SamplerPT
// (SamplerPT.cpp:147-171) and the likelihood factory (LikelihoodFactory.cpp:103-111), then reads
// them in Sampler::LoadSettings / SamplerPT::LoadSettings (SamplerPT.cpp:40-95). ConfigFile
// restates that parser (INI sections as "section.key" prefixes, '#' comments, typed values with
// the registered defaults, unknown or repeated keys rejected) without Boost; RunConfig is what the
// PT-MH path reads out of it.
#pragma once

#include <cstdint>
#include <map>
#include <string>

#include "SamplerPTDevice.h"

namespace bcm3 {

class ConfigFile {
public:
    enum Kind { STRING, SIZE, INT, REAL, BOOL, U64 };
    // every option bcminf registers, with its default (as text, parsed like a file value)
    ConfigFile();
    // parse `path`; false (with LOGERROR) on a syntax error, an unknown or repeated option or a
    // value that does not parse as the option's type
    bool Load(const std::string& path);
    bool Has(const std::string& key) const { return values_.count(key) != 0; }
    bool Set(const std::string& key) const { return set_.count(key) != 0; }  // given in the file
    const std::string& String(const std::string& key) const;
    double Real(const std::string& key) const;
    int64_t Int(const std::string& key) const;
    uint64_t ULL(const std::string& key) const;
    bool Bool(const std::string& key) const;
    const std::map<std::string, std::string>& Values() const { return values_; }

private:
    bool Store(const std::string& key, const std::string& value, int line);
    std::map<std::string, Kind> kinds_;
    std::map<std::string, std::string> values_;
    std::map<std::string, int> set_;
};

struct RunConfig {
    PTMHConfig ptmh;
    int64_t num_samples = 2500;
    bool output_proposal_adaptation = false;
    int64_t sampling_threads = 0, evaluation_threads = 1;
    std::string sampler_type, prior, likelihood, output_folder;
    std::string likelihood_options;  // "key=value;..." (bcm3_likelihood_create_ex)
};

// SamplerPT::LoadSettings + bcminf's option reads for the device sampler; false on settings the
// reference rejects (unknown swapping scheme / proposal type) or this path does not build
// (importance sampling, blocking strategies other than one_block, clustered / R-fitted proposals,
// proposal_transform_to_unbounded).
bool LoadRunConfig(const std::string& path, RunConfig& out);

}  // namespace bcm3
