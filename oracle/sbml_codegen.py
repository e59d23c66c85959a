"""TEST INFRASTRUCTURE (oracle). Never imported by the product path.

Restatement of the reference's SBML model loading order and right-hand-side code generation:
  SBMLModel::LoadSBML            src/sbml/SBMLModel.cpp:22-180   (species / reactions keyed by id in
                                                                  std::map -> sorted; ODE-integrated =
                                                                  species that are a reactant or product;
                                                                  the others are constant species)
  SBMLSpecies::Initialize        src/sbml/SBMLSpecies.cpp:14-93   (CellDesigner class; DEGRADED = sink)
  SBMLReaction::Initialize       src/sbml/SBMLReaction.cpp:16-77  (sink reactants/products dropped)
  SBMLRatelawElement::Generate   src/sbml/SBMLRatelaws.cpp:79-350 (name lookup order: forced parameter,
                                                                  sampled variable, species, constant
                                                                  species, non-sampled parameter, SBML
                                                                  parameter value)
  *::GenerateEquation            src/sbml/SBMLRatelaws.cpp:380-1100 (constants printed by
                                                                  std::to_string(long double) = "%Lf";
                                                                  integer-n hill specialisations)
  SBMLModel::GenerateCode        src/sbml/SBMLModel.cpp:291-367  (derivative part)
  SolverCodeGenerator            src/cellpop/SolverCodeGenerator.cpp:109-295 (helper functions)
with libsbml's MathML -> AST mapping for the node types the reference handles (apply plus / minus /
times / divide / power / exp / ln, ci, cn, user function calls). Used to check the product's C++
code generator text (tests/test_cellpop.py) and to compile the host copy of the generated
derivative the CPU oracle integrates (oracle/cellpop.py).
"""
import xml.etree.ElementTree as ET

MATHML = "{http://www.w3.org/1998/Math/MathML}"


def _local(tag):
    return tag.split("}", 1)[1] if "}" in tag else tag


def _to_string_ld(x):
    # std::to_string((long double)x) == "%Lf"
    return "%f" % float(x)


class Node:
    def __init__(self, kind, children=(), value=None):
        self.kind = kind  # plus minus negate times divide species const_species param nsparam const exp log pow hill mm synthcap tqssa
        self.children = list(children)
        self.value = value

    def eqn(self):
        k, c = self.kind, self.children
        if k == "plus":
            return "(" + "+".join(x.eqn() for x in c) + ")"
        if k == "minus":
            return "(" + c[0].eqn() + "-" + c[1].eqn() + ")"
        if k == "negate":
            return "(-" + c[0].eqn() + ")"
        if k == "times":
            return "(" + "*".join(x.eqn() for x in c) + ")"
        if k == "divide":
            return "(" + c[0].eqn() + "/" + c[1].eqn() + ")"
        if k == "species":
            return f"species[{self.value}]"
        if k == "const_species":
            return f"constant_species[{self.value}]"
        if k == "param":
            return f"parameters[{self.value}]"
        if k == "nsparam":
            return f"non_sampled_parameters[{self.value}]"
        if k == "const":
            return _to_string_ld(self.value)
        if k == "exp":
            return "exp(" + c[0].eqn() + ")"
        if k == "log":
            return "log(" + c[0].eqn() + ")"
        if k == "pow":
            return "safepow(" + c[0].eqn() + "," + c[1].eqn() + ")"
        if k == "hill":
            n = c[2].eqn()
            fixed = {"2.000000": 2, "4.000000": 4, "10.000000": 10, "16.000000": 16, "100.000000": 100}
            if n in fixed:
                return f"hill_function_fixedn{fixed[n]}(" + c[0].eqn() + "," + c[1].eqn() + ")"
            return "hill_function(" + c[0].eqn() + "," + c[1].eqn() + "," + n + ")"
        if k == "mm":
            return "michaelis_menten_function(" + ",".join(x.eqn() for x in c) + ")"
        if k == "synthcap":
            return "synthcap(" + c[0].eqn() + ")"
        if k == "tqssa":
            return "tQSSA(" + ",".join(x.eqn() for x in c) + ")"
        raise ValueError(k)


class SBMLModel:
    def __init__(self, filename):
        root = ET.parse(filename).getroot()
        model = next(e for e in root if _local(e.tag) == "model")
        self.species = {}  # id -> dict(name, initial, sink)
        self.parameters = {}
        self.reactions = {}  # id -> dict(reactants, rstoich, products, pstoich, law (xml element))
        for lst in model:
            t = _local(lst.tag)
            if t == "listOfSpecies":
                for sp in lst:
                    sid = sp.get("id")
                    cls = None
                    for ann in sp.iter():
                        if _local(ann.tag) == "class" and ann.text:
                            cls = ann.text.strip()
                    init = sp.get("initialAmount")
                    self.species[sid] = dict(name=sp.get("name", ""), initial=float(init) if init is not None else float("nan"),
                                             sink=(cls == "DEGRADED"))
            elif t == "listOfParameters":
                for p in lst:
                    self.parameters[p.get("id")] = float(p.get("value", "nan"))
        for lst in model:
            if _local(lst.tag) != "listOfReactions":
                continue
            for r in lst:
                rid = r.get("id")
                rec = dict(reactants=[], rstoich=[], products=[], pstoich=[], law=None)
                for part in r:
                    pt = _local(part.tag)
                    if pt in ("listOfReactants", "listOfProducts"):
                        for ref in part:
                            s = ref.get("species")
                            if s in self.species and not self.species[s]["sink"]:
                                key = "reactants" if pt == "listOfReactants" else "products"
                                rec[key].append(s)
                                rec["rstoich" if key == "reactants" else "pstoich"].append(float(ref.get("stoichiometry", "1")))
                    elif pt == "kineticLaw":
                        rec["law"] = next(m for m in part if _local(m.tag) == "math")[0]
                if rec["law"] is None:
                    raise ValueError(f'Reaction "{rid}" does not have a kinetic law')
                self.reactions[rid] = rec
        self.simulated = sorted(s for s, v in self.species.items() if not v["sink"])
        used = set()
        for rec in self.reactions.values():
            used.update(rec["reactants"])
            used.update(rec["products"])
        self.ode = [s for s in self.simulated if s in used]
        self.constant = [s for s in self.simulated if s not in used]

    # SBMLModel::GetODEIntegratedSpeciesByName (by species *name*)
    def ode_index(self, name):
        for i, s in enumerate(self.ode):
            if self.species[s]["name"] == name:
                return i
        return None

    def constant_index(self, name):
        for i, s in enumerate(self.constant):
            if self.species[s]["name"] == name:
                return i
        return None

    def _ast(self, e, variables, forced, nonsampled):
        t = _local(e.tag)
        if t == "ci":
            name = e.text.strip()
            if name in forced:
                return Node("const", value=forced[name])
            if name in variables:
                return Node("param", value=variables.index(name))
            if name in self.ode:
                return Node("species", value=self.ode.index(name))
            if name in self.constant:
                return Node("const_species", value=self.constant.index(name))
            if name in nonsampled:
                return Node("nsparam", value=nonsampled.index(name))
            if name in self.parameters:
                return Node("const", value=self.parameters[name])
            raise ValueError(f'AST_NAME name "{name}" does not map to either a species id or a parameter')
        if t == "cn":
            txt = (e.text or "").strip()
            if e.get("type") == "e-notation":
                parts = [txt] + [x.tail.strip() for x in e if x.tail]
                return Node("const", value=float(parts[0]) * 10.0 ** float(parts[1]))
            return Node("const", value=float(int(txt)) if e.get("type") == "integer" else float(txt))
        if t != "apply":
            raise ValueError(f"MathML element {t} not implemented")
        head, *args = list(e)
        ht = _local(head.tag)
        kids = [self._ast(a, variables, forced, nonsampled) for a in args]
        if ht == "plus":
            return Node("plus", kids)
        if ht == "minus":
            return Node("negate", kids) if len(kids) == 1 else Node("minus", kids)
        if ht == "times":
            return Node("times", kids)
        if ht == "divide":
            return Node("divide", kids)
        if ht == "power":
            return Node("pow", kids)
        if ht == "exp":
            return Node("exp", kids)
        if ht == "ln":
            return Node("log", kids)
        if ht == "ci":
            fname = head.text.strip()
            m = {"hill": ("hill", 3), "mm": ("mm", 4), "synthcap": ("synthcap", 1), "tQSSA": ("tqssa", 4)}
            if fname not in m or len(kids) != m[fname][1]:
                raise ValueError(f"AST function {fname} with {len(kids)} arguments")
            return Node(m[fname][0], kids)
        raise ValueError(f"MathML operator {ht} not implemented")

    def generate_derivative(self, variables, forced=None, nonsampled=()):
        """Text of generated_derivative's body as SBMLModel::GenerateCode writes it."""
        forced = forced or {}
        rids = sorted(self.reactions)
        code = "\tOdeReal ratelaws[%d];\n" % len(rids)
        for i, rid in enumerate(rids):
            eqn = self._ast(self.reactions[rid]["law"], list(variables), forced, list(nonsampled)).eqn()
            code += "\tratelaws[%d] = %s;\n" % (i, eqn if eqn else "0.0")
        for i, s in enumerate(self.ode):
            eqn = ""
            for ri, rid in enumerate(rids):
                rec = self.reactions[rid]
                for p, st in zip(rec["products"], rec["pstoich"]):
                    if p == s:
                        if st == 1.0:
                            eqn += "+ratelaws[%d]" % ri
                        elif st != 0.0:
                            eqn += "+" + _to_string_ld(st) + "*ratelaws[%d]" % ri
                for p, st in zip(rec["reactants"], rec["rstoich"]):
                    if p == s:
                        if st == 1.0:
                            eqn += "-ratelaws[%d]" % ri
                        elif st != 0.0:
                            eqn += "-" + _to_string_ld(st) + "*ratelaws[%d]" % ri
            code += "\tout[%d] = %s;\n" % (i, eqn if eqn else "0.0")
        return code


# SolverCodeGenerator.cpp:122-294 (the helper functions of the generated translation unit), as
# host C++ for the oracle's copy of the derivative
HELPERS = r"""
#include <cmath>
#include <limits>
typedef double OdeReal;
inline OdeReal square(OdeReal x) { return x * x; }
inline OdeReal hill_function(OdeReal x, OdeReal k, OdeReal n)
{
	if (x <= 0.0) return 0.0;
	OdeReal xn = pow(x, n);
	OdeReal kn = pow(k, n);
	OdeReal xnpkn = xn + kn;
	if (xnpkn < std::numeric_limits<OdeReal>::min()) return 0.0;
	if (xnpkn > 3e38f) return 1.0;
	return xn / xnpkn;
}
inline OdeReal hill_function_fixedn2(OdeReal x, OdeReal k)
{
	if (x <= 0.0) return 0.0;
	OdeReal x2 = x * x;
	OdeReal k2 = k * k;
	OdeReal xnpkn = x2 + k2;
	if (xnpkn < std::numeric_limits<OdeReal>::min()) return 0.0;
	if (xnpkn > 3e38f) return 10.0;
	return x2 / xnpkn;
}
inline OdeReal hill_function_fixedn4(OdeReal x, OdeReal k)
{
	if (x <= 0.0) return 0.0;
	OdeReal x2 = x * x;
	OdeReal x4 = x2 * x2;
	OdeReal k2 = k * k;
	OdeReal k4 = k2 * k2;
	OdeReal xnpkn = x4 + k4;
	if (xnpkn < std::numeric_limits<OdeReal>::min()) return 0.0;
	if (xnpkn > 3e38f) return 1.0;
	return x4 / xnpkn;
}
inline OdeReal hill_function_fixedn10(OdeReal x, OdeReal k)
{
	if (x <= 0.0) return 0.0;
	OdeReal x2 = x * x;
	OdeReal x4 = x2 * x2;
	OdeReal x8 = x4 * x4;
	OdeReal x10 = x2 * x8;
	OdeReal k2 = k * k;
	OdeReal k4 = k2 * k2;
	OdeReal k8 = k4 * k4;
	OdeReal k10 = k2 * k8;
	OdeReal xnpkn = x10 + k10;
	if (xnpkn < std::numeric_limits<OdeReal>::min()) return 0.0;
	if (xnpkn > 3e38f) return 1.0;
	return x10 / xnpkn;
}
inline OdeReal hill_function_fixedn16(OdeReal x, OdeReal k)
{
	if (x <= 0.0) return 0.0;
	OdeReal x2 = x * x;
	OdeReal x4 = x2 * x2;
	OdeReal x8 = x4 * x4;
	OdeReal x16 = x8 * x8;
	OdeReal k2 = k * k;
	OdeReal k4 = k2 * k2;
	OdeReal k8 = k4 * k4;
	OdeReal k16 = k8 * k8;
	OdeReal xnpkn = x16 + k16;
	if (xnpkn < std::numeric_limits<OdeReal>::min()) return 0.0;
	return x16 / xnpkn;
}
inline OdeReal hill_function_fixedn100(OdeReal x, OdeReal k)
{
	if (x <= 0.0) return 0.0;
	OdeReal x2 = x * x;
	OdeReal x4 = x2 * x2;
	OdeReal x8 = x4 * x4;
	OdeReal x16 = x8 * x8;
	OdeReal x32 = x16 * x16;
	OdeReal x64 = x32 * x32;
	OdeReal x100 = x64 * x32 * x4;
	OdeReal k2 = k * k;
	OdeReal k4 = k2 * k2;
	OdeReal k8 = k4 * k4;
	OdeReal k16 = k8 * k8;
	OdeReal k32 = k16 * k16;
	OdeReal k64 = k32 * k32;
	OdeReal k100 = k64 * k32 * k4;
	OdeReal xnpkn = x100 + k100;
	if (xnpkn < std::numeric_limits<OdeReal>::min()) return 0.0;
	if (xnpkn > 3e38f) return 1.0;
	return x100 / xnpkn;
}
inline OdeReal michaelis_menten_function(OdeReal kcat, OdeReal KM, OdeReal e, OdeReal s)
{
	if (e <= 0) return 0.0;
	if (s + KM < 0.1 * KM) {
		OdeReal bound = -KM + 0.1 * KM;
		OdeReal offset = (e * kcat * bound / (0.01 * KM) - e * kcat * bound / (KM + bound));
		return e * kcat * s / (0.01 * KM) - offset;
	}
	return kcat * e * s / (KM + s);
}
inline OdeReal safepow(OdeReal x, OdeReal n)
{
	if (x <= 0) {
		return 0.0;
	} else {
		return pow(x, n);
	}
}
inline OdeReal synthcap(OdeReal x)
{
	if (x <= 0) {
		return 1.0;
	} else {
		OdeReal x2 = x * x;
		OdeReal x4 = x2 * x2;
		OdeReal x8 = x4 * x4;
		return 1.0 - x8 * x2;
	}
}
inline OdeReal tQSSA(OdeReal k, OdeReal km, OdeReal e, OdeReal s)
{
	OdeReal ekms = e + km + s;
	return 0.5 * k * (ekms - sqrt(ekms * ekms - 4 * e * s));
}
"""


def host_translation_unit(body):
    return (HELPERS + '\nextern "C" void generated_derivative(OdeReal* out, const OdeReal* species, '
            'const OdeReal* constant_species, const OdeReal* parameters, const OdeReal* non_sampled_parameters)\n{\n'
            + body + "}\n")
