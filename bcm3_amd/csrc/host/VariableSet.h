// VariableSet.h -- bcm3::VariableSet (src/sampler/VariableSet.h / .cpp:16-124), Boost-free.
#pragma once
#include <cstddef>
#include <limits>
#include <memory>
#include <string>
#include <vector>

#include "xml.h"

namespace bcm3 {

using Real = double;
using VectorReal = std::vector<Real>;

class VariableSet {
public:
    enum Transform { Transform_None = 0, Transform_Log = 1, Transform_Log10 = 2, Transform_Logit = 3 };

    bool LoadFromXML(const std::string& filename);
    bool LoadFromXML(const XmlNode& root, const std::string& name);
    void AddVariable(const std::string& name, bool logspace = false, bool logistic = false);

    size_t GetNumVariables() const { return variables.size(); }
    const std::string& GetVariableName(size_t i) const { return variables[i]; }
    const std::vector<std::string>& GetVariableNames() const { return variables; }
    // GetVariableIndex (VariableSet.cpp:83-95): max size_t when absent
    size_t GetVariableIndex(const std::string& name, bool log_error = true) const;
    Transform GetVariableTransform(size_t i) const { return transforms[i]; }
    Real TransformVariable(size_t i, Real x) const;  // VariableSet.cpp:97-124
    const std::string& GetName() const { return Name; }

private:
    std::string Name;
    std::vector<std::string> variables;
    std::vector<Transform> transforms;
};

}  // namespace bcm3
