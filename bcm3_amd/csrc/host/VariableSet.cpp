// VariableSet.cpp -- see VariableSet.h
#include "VariableSet.h"

#include <cmath>

#include "log.h"

namespace bcm3 {

bool VariableSet::LoadFromXML(const std::string& filename)
{
    try {
        auto root = xml_load(filename);
        std::string name = filename;
        size_t dot = name.find_last_of('.');
        if (dot != std::string::npos) name[dot] = '_';
        return LoadFromXML(*root, name);
    } catch (XmlError& e) {
        LOGERROR("Error loading variable file: %s", e.what.c_str());
        return false;
    }
}

// VariableSet::LoadFromXML (VariableSet.cpp:16-69): <prior> or <variableset> root; each
// <variable name [repeat] [logspace] [logistic]>; repeat > 1 expands to name_0, name_1, ...
bool VariableSet::LoadFromXML(const XmlNode& root, const std::string& name)
{
    Name = name;
    const XmlNode* node = root.child("prior");
    if (!node) node = root.child("variableset");
    if (!node) {
        LOGERROR("Incorrect prior XML format");
        return false;
    }
    try {
        for (auto& var : node->children) {
            if (var->name != "variable") continue;
            std::string vname = var->get("name");
            long repeat = var->get_long("repeat", 1);
            bool logspace = var->get_bool("logspace", false);
            bool logistic = var->get_bool("logistic", false);
            for (long i = 0; i < repeat; i++) {
                variables.push_back(repeat > 1 ? vname + "_" + std::to_string(i) : vname);
                transforms.push_back(logspace ? Transform_Log10 : (logistic ? Transform_Logit : Transform_None));
            }
        }
    } catch (XmlError& e) {
        LOGERROR("Error parsing variable file: %s", e.what.c_str());
        return false;
    }
    return true;
}

void VariableSet::AddVariable(const std::string& name, bool logspace, bool logistic)
{
    variables.push_back(name);
    transforms.push_back(logspace ? Transform_Log10 : (logistic ? Transform_Logit : Transform_None));
}

size_t VariableSet::GetVariableIndex(const std::string& name, bool log_error) const
{
    for (size_t vi = 0; vi < variables.size(); vi++)
        if (variables[vi] == name) return vi;
    if (log_error) LOGERROR("Could not find variable \"%s\"", name.c_str());
    return std::numeric_limits<size_t>::max();
}

Real VariableSet::TransformVariable(size_t i, Real x) const
{
    switch (transforms[i]) {
    case Transform_None: return x;
    case Transform_Log: return std::exp(x);
    case Transform_Log10: return std::exp(x * 2.3025850929940459);  // bcm3::fastpow10
    case Transform_Logit:
        if (x > 0) {
            Real z = std::exp(-x);
            return 1.0 / (1.0 + z);
        } else {
            Real z = std::exp(x);
            return z / (1.0 + z);
        }
    default: return x;
    }
}

}  // namespace bcm3
