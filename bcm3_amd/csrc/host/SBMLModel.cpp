// SBMLModel.cpp -- see SBMLModel.h. The equation strings are the reference's, character for
// character (tests/test_cellpop.py compares them with oracle/sbml_codegen.py), because the
// generated code IS the model's arithmetic: constants go through std::to_string(long double)
// ("%Lf", six decimals), integer Hill exponents select the fixed-n helpers.
#include "SBMLModel.h"

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <set>

namespace bcm3 {

namespace {

std::string local_name(const std::string& n)
{
    const size_t c = n.find(':');
    return c == std::string::npos ? n : n.substr(c + 1);
}

std::string trim(const std::string& s)
{
    size_t b = 0, e = s.size();
    while (b < e && std::isspace((unsigned char)s[b])) b++;
    while (e > b && std::isspace((unsigned char)s[e - 1])) e--;
    return s.substr(b, e - b);
}

const XmlNode* first_named(const XmlNode& n, const std::string& local)
{
    for (const auto& c : n.children)
        if (local_name(c->name) == local) return c.get();
    return nullptr;
}

// std::to_string((long double)x)
std::string ld_string(double x)
{
    char buf[512];
    snprintf(buf, sizeof(buf), "%Lf", (long double)x);
    return buf;
}

// the CellDesigner species class of <species><annotation>...<celldesigner:class>X</...>
std::string celldesigner_class(const XmlNode& n)
{
    if (local_name(n.name) == "class") return trim(n.text);
    for (const auto& c : n.children) {
        const std::string r = celldesigner_class(*c);
        if (!r.empty()) return r;
    }
    return "";
}

struct Gen {
    const std::vector<std::string>& variables;
    const std::map<std::string, double>& forced;
    const std::vector<std::string>& ode;
    const std::vector<std::string>& constant;
    const std::map<std::string, double>& parameters;
    std::string error;

    static size_t index_of(const std::vector<std::string>& v, const std::string& x)
    {
        for (size_t i = 0; i < v.size(); i++)
            if (v[i] == x) return i;
        return SIZE_MAX;
    }

    // SBMLRatelawElement::Generate + GenerateEquation in one pass
    bool eqn(const XmlNode& e, std::string& out)
    {
        const std::string t = local_name(e.name);
        if (t == "ci") {
            const std::string name = trim(e.text);
            auto f = forced.find(name);
            if (f != forced.end()) {
                out = ld_string(f->second);
                return true;
            }
            size_t ix = index_of(variables, name);
            if (ix != SIZE_MAX) {
                out = "parameters[" + std::to_string(ix) + "]";
                return true;
            }
            ix = index_of(ode, name);
            if (ix != SIZE_MAX) {
                out = "species[" + std::to_string(ix) + "]";
                return true;
            }
            ix = index_of(constant, name);
            if (ix != SIZE_MAX) {
                out = "constant_species[" + std::to_string(ix) + "]";
                return true;
            }
            auto p = parameters.find(name);
            if (p != parameters.end()) {
                out = ld_string(p->second);
                return true;
            }
            error = "AST_NAME name \"" + name + "\" does not map to either a species id or a parameter";
            return false;
        }
        if (t == "cn") {
            const std::string type = e.has_attr("type") ? e.attr.at("type") : "real";
            double v;
            if (type == "e-notation") {
                // <cn type="e-notation"> m <sep/> e </cn>: our reader keeps the text around <sep/>
                std::string txt = trim(e.text);
                char* end = nullptr;
                const double m = strtod(txt.c_str(), &end);
                const double x = strtod(end, nullptr);
                v = m * std::pow(10.0, x);
            } else if (type == "integer") {
                v = (double)strtol(trim(e.text).c_str(), nullptr, 10);
            } else {
                v = strtod(trim(e.text).c_str(), nullptr);
            }
            out = ld_string(v);
            return true;
        }
        if (t != "apply" || e.children.empty()) {
            error = "MathML element <" + t + "> not implemented";
            return false;
        }
        const XmlNode& head = *e.children[0];
        const std::string op = local_name(head.name);
        std::vector<std::string> a;
        for (size_t i = 1; i < e.children.size(); i++) {
            std::string s;
            if (!eqn(*e.children[i], s)) return false;
            a.push_back(s);
        }
        auto join = [&](const char* sep) {
            std::string r = "(" + a[0];
            for (size_t i = 1; i < a.size(); i++) r += sep + a[i];
            return r + ")";
        };
        if (op == "plus") {
            if (a.size() < 2) return fail_arity(op);
            out = join("+");
        } else if (op == "minus") {
            if (a.size() == 1)
                out = "(-" + a[0] + ")";
            else if (a.size() == 2)
                out = "(" + a[0] + "-" + a[1] + ")";
            else
                return fail_arity(op);
        } else if (op == "times") {
            if (a.size() < 2) return fail_arity(op);
            out = join("*");
        } else if (op == "divide") {
            if (a.size() != 2) return fail_arity(op);
            out = "(" + a[0] + "/" + a[1] + ")";
        } else if (op == "power") {
            if (a.size() != 2) return fail_arity(op);
            out = "safepow(" + a[0] + "," + a[1] + ")";
        } else if (op == "exp") {
            if (a.size() != 1) return fail_arity(op);
            out = "exp(" + a[0] + ")";
        } else if (op == "ln") {
            if (a.size() != 1) return fail_arity(op);
            out = "log(" + a[0] + ")";
        } else if (op == "ci") {
            const std::string fn = trim(head.text);
            if (fn == "hill") {
                if (a.size() != 3) return fail_arity(fn);
                static const std::map<std::string, std::string> fixed = {
                    {"2.000000", "2"}, {"4.000000", "4"}, {"10.000000", "10"}, {"16.000000", "16"}, {"100.000000", "100"}};
                auto f = fixed.find(a[2]);
                if (f != fixed.end())
                    out = "hill_function_fixedn" + f->second + "(" + a[0] + "," + a[1] + ")";
                else
                    out = "hill_function(" + a[0] + "," + a[1] + "," + a[2] + ")";
            } else if (fn == "mm") {
                if (a.size() != 4) return fail_arity(fn);
                out = "michaelis_menten_function(" + a[0] + "," + a[1] + "," + a[2] + "," + a[3] + ")";
            } else if (fn == "synthcap") {
                if (a.size() != 1) return fail_arity(fn);
                out = "synthcap(" + a[0] + ")";
            } else if (fn == "tQSSA") {
                if (a.size() != 4) return fail_arity(fn);
                out = "tQSSA(" + a[0] + "," + a[1] + "," + a[2] + "," + a[3] + ")";
            } else {
                error = "AST function with unknown name " + fn;
                return false;
            }
        } else {
            error = "SBML AST node <" + op + "> not implemented";
            return false;
        }
        return true;
    }
    bool fail_arity(const std::string& op)
    {
        error = "wrong number of arguments for " + op;
        return false;
    }
};

}  // namespace

bool SBMLModel::LoadSBML(const std::string& filename, std::string& error)
{
    std::unique_ptr<XmlNode> root;
    try {
        root = xml_load(filename);
    } catch (const XmlError& e) {
        error = "Errors reading SBML file " + filename + ": " + e.what;
        return false;
    }
    doc = std::shared_ptr<XmlNode>(root.release());
    const XmlNode* sbml = nullptr;
    for (const auto& c : doc->children)
        if (local_name(c->name) == "sbml") sbml = c.get();
    const XmlNode* model = sbml ? first_named(*sbml, "model") : nullptr;
    if (!model) {
        error = "Unable to load SBML model";
        return false;
    }
    species.clear();
    parameters.clear();
    reactions.clear();
    if (const XmlNode* ls = first_named(*model, "listOfSpecies")) {
        for (const auto& sp : ls->children) {
            if (local_name(sp->name) != "species") continue;
            Species s;
            s.id = sp->get("id");
            s.name = sp->has_attr("name") ? sp->attr.at("name") : "";
            s.initial = sp->has_attr("initialAmount") ? strtod(sp->attr.at("initialAmount").c_str(), nullptr)
                                                      : std::numeric_limits<double>::quiet_NaN();
            const std::string cls = celldesigner_class(*sp);
            s.sink = (cls == "DEGRADED");
            if (cls == "RNA") s.name += "_mRNA";
            if (species.count(s.id)) {
                error = "Duplicate species id " + s.id;
                return false;
            }
            species[s.id] = s;
        }
    }
    if (const XmlNode* lp = first_named(*model, "listOfParameters")) {
        for (const auto& p : lp->children)
            if (local_name(p->name) == "parameter")
                parameters[p->get("id")] = p->has_attr("value") ? strtod(p->attr.at("value").c_str(), nullptr)
                                                                 : std::numeric_limits<double>::quiet_NaN();
    }
    if (const XmlNode* lr = first_named(*model, "listOfReactions")) {
        for (const auto& r : lr->children) {
            if (local_name(r->name) != "reaction") continue;
            Reaction re;
            re.id = r->get("id");
            for (const auto& part : r->children) {
                const std::string pt = local_name(part->name);
                if (pt == "listOfReactants" || pt == "listOfProducts") {
                    for (const auto& ref : part->children) {
                        const std::string sid = ref->has_attr("species") ? ref->attr.at("species") : "";
                        auto it = species.find(sid);
                        if (it == species.end() || it->second.sink) continue;
                        const double st = ref->has_attr("stoichiometry") ? strtod(ref->attr.at("stoichiometry").c_str(), nullptr) : 1.0;
                        if (pt == "listOfReactants") {
                            re.reactants.push_back(sid);
                            re.reactant_stoichiometry.push_back(st);
                        } else {
                            re.products.push_back(sid);
                            re.product_stoichiometry.push_back(st);
                        }
                    }
                } else if (pt == "kineticLaw") {
                    const XmlNode* math = first_named(*part, "math");
                    if (math && !math->children.empty()) re.law = math->children[0].get();
                }
            }
            if (!re.law) {
                error = "Reaction \"" + re.id + "\" does not have a kinetic law";
                return false;
            }
            if (reactions.count(re.id)) {
                error = "Duplicate reaction id " + re.id;
                return false;
            }
            reactions[re.id] = re;
        }
    }
    simulated.clear();
    ode.clear();
    constant.clear();
    std::set<std::string> used;
    for (const auto& kv : reactions) {
        used.insert(kv.second.reactants.begin(), kv.second.reactants.end());
        used.insert(kv.second.products.begin(), kv.second.products.end());
    }
    for (const auto& kv : species) {
        if (kv.second.sink) continue;
        simulated.push_back(kv.first);
        (used.count(kv.first) ? ode : constant).push_back(kv.first);
    }
    return true;
}

static size_t by_name(const std::map<std::string, SBMLModel::Species>& sp, const std::vector<std::string>& ids,
                      const std::string& name)
{
    for (size_t i = 0; i < ids.size(); i++)
        if (sp.at(ids[i]).name == name) return i;
    return SIZE_MAX;
}
size_t SBMLModel::GetSimulatedSpeciesByName(const std::string& name) const { return by_name(species, simulated, name); }
size_t SBMLModel::GetODEIntegratedSpeciesByName(const std::string& name) const { return by_name(species, ode, name); }
size_t SBMLModel::GetConstantSpeciesByName(const std::string& name) const { return by_name(species, constant, name); }

bool SBMLModel::GenerateDerivative(const std::vector<std::string>& variables, const std::map<std::string, double>& forced,
                                   std::string& code, std::string& error) const
{
    Gen g{variables, forced, ode, constant, parameters, ""};
    code = "\tOdeReal ratelaws[" + std::to_string(reactions.size()) + "];\n";
    std::vector<const Reaction*> rs;
    size_t i = 0;
    for (const auto& kv : reactions) {
        std::string e;
        if (!g.eqn(*kv.second.law, e)) {
            error = "reaction " + kv.first + ": " + g.error;
            return false;
        }
        code += "\tratelaws[" + std::to_string(i) + "] = " + (e.empty() ? std::string("0.0") : e) + ";\n";
        rs.push_back(&kv.second);
        i++;
    }
    for (size_t s = 0; s < ode.size(); s++) {
        std::string eqn;
        for (size_t r = 0; r < rs.size(); r++) {
            const Reaction& re = *rs[r];
            for (size_t p = 0; p < re.products.size(); p++) {
                if (re.products[p] != ode[s]) continue;
                const double st = re.product_stoichiometry[p];
                if (st == 1.0)
                    eqn += "+ratelaws[" + std::to_string(r) + "]";
                else if (st != 0.0)
                    eqn += "+" + std::to_string(st) + "*ratelaws[" + std::to_string(r) + "]";
            }
            for (size_t p = 0; p < re.reactants.size(); p++) {
                if (re.reactants[p] != ode[s]) continue;
                const double st = re.reactant_stoichiometry[p];
                if (st == 1.0)
                    eqn += "-ratelaws[" + std::to_string(r) + "]";
                else if (st != 0.0)
                    eqn += "-" + std::to_string(st) + "*ratelaws[" + std::to_string(r) + "]";
            }
        }
        code += "\tout[" + std::to_string(s) + "] = " + (eqn.empty() ? std::string("0.0") : eqn) + ";\n";
    }
    return true;
}

}  // namespace bcm3
