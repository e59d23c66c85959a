// Test infrastructure: the members of the reference's bcm3::VariableSet (src/sampler/VariableSet.h:5-33)
// a likelihood plugin reads; variables are added by name (prior.xml order).
#pragma once

#include "Utils.h"

namespace bcm3 {

class VariableSet {
public:
    void AddVariable(const std::string& name) { variables.push_back(name); }
    size_t GetNumVariables() const { return variables.size(); }
    const std::string& GetVariableName(size_t i) const { return variables[i]; }
    const std::vector<std::string>& GetAllVariableNames() const { return variables; }

private:
    std::vector<std::string> variables;
};

}  // namespace bcm3
