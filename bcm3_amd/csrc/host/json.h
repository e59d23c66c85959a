// json.h -- minimal JSON reader for the PopPK data sidecar (the netCDF-4 group schema of
// LikelihoodPopPKTrajectory::Initialize, src/likelihoods/LikelihoodPopPKTrajectory.cpp:89-204,
// stored as {"<trial>": {"time": [...], "patients": [...], "<drug>_dose": [...], ...}};
// null = NaN). netCDF/HDF5 are not available to this build.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace bcm3 {

struct Json {
    enum Type { Null, Bool, Number, String, Array, Object } type = Null;
    double num = 0.0;
    bool b = false;
    std::string str;
    std::vector<Json> arr;
    std::map<std::string, Json> obj;

    const Json* find(const std::string& k) const;
    double as_double() const;  // null -> NaN
};

struct JsonError {
    std::string what;
};

Json json_parse(const std::string& text);
Json json_load(const std::string& filename);
// compact text, numbers round-trip (%.17g), NaN / inf as null
std::string json_dump(const Json& j);

}  // namespace bcm3
