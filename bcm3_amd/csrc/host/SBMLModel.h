// SBMLModel.h -- the subset of an SBML cell model that BCM3's cell-population likelihood uses,
// read without libsbml, and the right-hand-side code generator.
//   SBMLModel::LoadSBML         src/sbml/SBMLModel.cpp:22-180  (species and reactions keyed by id
//                               -> sorted; ODE-integrated species = reactants/products; the rest
//                               are constant species)
//   SBMLSpecies::Initialize     src/sbml/SBMLSpecies.cpp:14-93 (CellDesigner class DEGRADED = sink)
//   SBMLReaction::Initialize    src/sbml/SBMLReaction.cpp:16-77
//   SBMLRatelawElement::Generate / GenerateEquation  src/sbml/SBMLRatelaws.cpp:79-1100
//   SBMLModel::GenerateCode     src/sbml/SBMLModel.cpp:291-367 (the derivative; cells integrate
//                               with a difference-quotient Jacobian, Cell.cpp:57-76)
// MathML node types: apply plus / minus / times / divide / power / exp / ln, ci, cn (integer,
// real, e-notation) and calls of hill / mm / synthcap / tQSSA -- the set the reference handles.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "xml.h"

namespace bcm3 {

class SBMLModel {
public:
    struct Species {
        std::string id, name;
        double initial;
        bool sink;
    };
    struct Reaction {
        std::string id;
        std::vector<std::string> reactants, products;
        std::vector<double> reactant_stoichiometry, product_stoichiometry;
        const XmlNode* law = nullptr;  // the <math> element's expression (owned by doc)
    };

    bool LoadSBML(const std::string& filename, std::string& error);

    // name lookups (by species *name*, SBMLModel.cpp:606-643); SIZE_MAX if absent
    size_t GetSimulatedSpeciesByName(const std::string& name) const;
    size_t GetODEIntegratedSpeciesByName(const std::string& name) const;
    size_t GetConstantSpeciesByName(const std::string& name) const;
    size_t GetNumODEIntegratedSpecies() const { return ode.size(); }
    size_t GetNumConstantSpecies() const { return constant.size(); }
    const Species& GetODEIntegratedSpecies(size_t i) const { return species.at(ode[i]); }
    const Species& GetConstantSpecies(size_t i) const { return species.at(constant[i]); }
    bool HasParameter(const std::string& id) const { return parameters.count(id) > 0; }

    //! Body of generated_derivative (SBMLModel::GenerateCode): ratelaws[] then out[i] per species.
    //! variables = the sampled variable names (parameters[] index), forced = <set_parameter>.
    bool GenerateDerivative(const std::vector<std::string>& variables, const std::map<std::string, double>& forced,
                            std::string& code, std::string& error) const;

private:
    std::shared_ptr<XmlNode> doc;
    std::map<std::string, Species> species;  // by id (sorted, as the reference's std::map)
    std::map<std::string, double> parameters;
    std::map<std::string, Reaction> reactions;
    std::vector<std::string> simulated, ode, constant;
};

}  // namespace bcm3
