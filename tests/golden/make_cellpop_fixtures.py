"""Writes the config-C4 problem (cellpop SBML model, heterogeneous cells with division)
used by the cellpop parity tests and the bench's C4 line.

The reference ships no cellpop model or data (src/cellpop needs a CellDesigner SBML file and a
netCDF data file the user provides), so this is a synthetic cell-cycle model in the reference's
SBML dialect: kinetic laws in MathML with the reference's function names (hill, mm, synthcap;
src/sbml/SBMLRatelaws.cpp:285-350), the species names Cell.cpp hard-codes for division and phase
events (cytokinesis, nuclear_envelope, G1S_break, G2_break, spindle_components, assembled_spindle,
chromatid_separation: Cell.cpp:44-50, 119-133; replicating_DNA / replicated_DNA / PCNA_gfp
thresholds Cell.cpp:467-484). Time unit: hours. One cycle takes ~10 h at the "true" parameters.

    python tests/golden/make_cellpop_fixtures.py          # model, prior, likelihood XML
    python tests/golden/make_cellpop_fixtures.py --data   # + data sidecar simulated by the oracle

The data (population-average PCNA_gfp, 3 replicates x 21 time points) are simulated by the
oracle (oracle/cellpop.py, the reference's vendored CVODE 5.3.0 + its PartialPivLU) at TRUE below
plus Gaussian noise (seed 20251017).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))

# species: id -> initial amount (ids = names; the model sorts them by id like SBMLModel's std::map)
SPECIES = {
    "APC": 0.0, "CycB": 0.0, "CycD": 0.2, "CycE": 0.0, "G1S_break": 1.0, "G2_break": 1.0, "PCNA_gfp": 0.0,
    "assembled_spindle": 0.0, "chromatid_separation": 0.0, "cytokinesis": 0.0, "licensed_DNA": 2.0,
    "mitogen": 1.0, "nuclear_envelope": 1.0, "replicated_DNA": 0.0, "replicating_DNA": 0.0,
    "spindle_components": 0.0,
}
# SBML constant parameters (printed by the reference's code generator with 6 decimals, so all of
# them are exact at that precision)
PARAMETERS = {
    "kd_D": 0.5, "k_g1s": 0.3, "kd_E": 0.5, "k_rep": 0.3, "k_fin": 0.5, "k_pcna": 1.0, "kd_pcna": 0.5,
    "kd_B": 2.0, "k_g2": 0.5, "k_neb": 1.0, "k_sp": 1.0, "k_as": 1.0, "kd_apc": 0.5, "k_sep": 1.0,
    "k_cyt": 1.0, "k_lic": 1.0, "K_B": 1.5, "K_gate": 0.5, "K_apc": 0.5,
    # sampled in the prior (the SBML value is the default when a variable is absent)
    "k_D": 0.5, "k_E": 1.0, "k_B": 1.0, "k_apc": 2.0,
}


# kinetic-law DSL -> MathML: ("op", args...) with op in plus/minus/times/divide/power/exp/ln or a
# function name (hill, mm, synthcap, tQSSA); str = <ci>, int/float = <cn>
def mathml(e):
    if isinstance(e, str):
        return f"<ci> {e} </ci>"
    if isinstance(e, bool):
        raise TypeError(e)
    if isinstance(e, int):
        return f'<cn type="integer"> {e} </cn>'
    if isinstance(e, float):
        return f"<cn> {e!r} </cn>"
    op, *args = e
    inner = "".join(mathml(a) for a in args)
    if op in ("plus", "minus", "times", "divide", "power", "exp", "ln"):
        return f"<apply><{op}/>{inner}</apply>"
    return f"<apply><ci> {op} </ci>{inner}</apply>"


def gate_off(x):  # 1 - hill(x, K_gate, 16): on once x drops below ~K_gate
    return ("minus", 1, ("hill", x, "K_gate", 16))


# reaction id -> (reactants, products, kinetic law)
REACTIONS = {
    "r01_CycD_synthesis": ([], ["CycD"], ("times", "k_D", "mitogen")),
    "r02_CycD_degradation": (["CycD"], [], ("times", "kd_D", "CycD")),
    "r03_G1S_release": (["G1S_break"], [], ("times", "k_g1s", "CycD", "G1S_break")),
    "r04_CycE_synthesis": ([], ["CycE"], ("times", "k_E", ("synthcap", "G1S_break"))),
    "r05_CycE_degradation": (["CycE"], [], ("times", "kd_E", "CycE")),
    "r06_replication_start": (["licensed_DNA"], ["replicating_DNA"], ("times", "k_rep", "CycE", "licensed_DNA")),
    "r07_replication_finish": (["replicating_DNA"], ["replicated_DNA"], ("times", "k_fin", "replicating_DNA")),
    "r08_PCNA_synthesis": ([], ["PCNA_gfp"], ("times", "k_pcna", "replicating_DNA")),
    "r09_PCNA_degradation": (["PCNA_gfp"], [], ("times", "kd_pcna", "PCNA_gfp")),
    "r10_CycB_synthesis": ([], ["CycB"], ("times", "k_B", ("hill", "replicated_DNA", "K_B", 4))),
    "r11_CycB_degradation": (["CycB"], [], ("times", "kd_B", "CycB", "APC")),
    "r12_G2_release": (["G2_break"], [], ("times", "k_g2", "CycB", "G2_break")),
    "r13_envelope_breakdown": (["nuclear_envelope"], [], ("times", "k_neb", "CycB", "nuclear_envelope", gate_off("G2_break"))),
    "r14_spindle_synthesis": ([], ["spindle_components"], ("times", "k_sp", gate_off("nuclear_envelope"))),
    "r15_spindle_assembly": (["spindle_components"], ["assembled_spindle"], ("times", "k_as", "spindle_components")),
    "r16_APC_activation": ([], ["APC"], ("times", "k_apc", ("hill", "assembled_spindle", "K_apc", 4), ("minus", 1, "APC"))),
    "r17_APC_inactivation": (["APC"], [], ("times", "kd_apc", "APC")),
    "r18_chromatid_separation": ([], ["chromatid_separation"], ("times", "k_sep", "APC", "assembled_spindle")),
    "r19_cytokinesis": ([], ["cytokinesis"], ("times", "k_cyt", "chromatid_separation")),
    "r20_relicensing": (["replicated_DNA"], ["licensed_DNA"], ("times", "k_lic", "APC", "replicated_DNA")),
}

FUNCTIONS = {  # lambda bodies for SBML validity; the reference maps the names, not the bodies
    "hill": (["x", "k", "n"], ("divide", ("power", "x", "n"), ("plus", ("power", "x", "n"), ("power", "k", "n")))),
    "synthcap": (["x"], ("minus", 1, ("power", "x", 10))),
}

# prior (d = 7): rate constants in log10 space, the variability scale on its log scale
# (VariabilityDescription.cpp:60-67: v = QuantileNormal(sobol) * exp(scale)), the data stdev
PRIOR = [
    ("k_D", -0.8, 0.2, True),
    ("k_E", -0.5, 0.5, True),
    ("k_B", -0.5, 0.5, True),
    ("k_apc", 0.0, 0.7, True),
    ("var_kD", -3.0, -0.5, False),
    ("var_CycD0", -3.0, -0.5, False),
    ("stdev", -2.0, -0.5, True),
]
TRUE = {"k_D": -0.30103, "k_E": 0.0, "k_B": 0.0, "k_apc": 0.30103, "var_kD": -1.6, "var_CycD0": -1.2, "stdev": -1.3}

TIMES = [float(h) for h in range(21)]  # hours 0..20
REPLICATES = 3


def sbml_text():
    out = ['<?xml version="1.0" encoding="UTF-8"?>',
           '<sbml xmlns="http://www.sbml.org/sbml/level2/version4" level="2" version="4">',
           '  <model id="cellcycle_toy" name="synthetic cell cycle (bcm3_amd config C4)">',
           '    <listOfFunctionDefinitions>']
    for name, (args, body) in FUNCTIONS.items():
        bvars = "".join(f"<bvar><ci> {a} </ci></bvar>" for a in args)
        out.append(f'      <functionDefinition id="{name}"><math xmlns="http://www.w3.org/1998/Math/MathML">'
                   f"<lambda>{bvars}{mathml(body)}</lambda></math></functionDefinition>")
    out.append('    </listOfFunctionDefinitions>')
    out.append('    <listOfCompartments><compartment id="cell" size="1"/></listOfCompartments>')
    out.append('    <listOfSpecies>')
    for sid, v in SPECIES.items():
        out.append(f'      <species id="{sid}" name="{sid}" compartment="cell" initialAmount="{v!r}"/>')
    out.append('    </listOfSpecies>')
    out.append('    <listOfParameters>')
    for pid, v in PARAMETERS.items():
        out.append(f'      <parameter id="{pid}" value="{v!r}"/>')
    out.append('    </listOfParameters>')
    out.append('    <listOfReactions>')
    for rid, (re, pr, law) in REACTIONS.items():
        out.append(f'      <reaction id="{rid}" reversible="false">')
        if re:
            out.append("        <listOfReactants>" + "".join(f'<speciesReference species="{s}"/>' for s in re) + "</listOfReactants>")
        if pr:
            out.append("        <listOfProducts>" + "".join(f'<speciesReference species="{s}" stoichiometry="1"/>' for s in pr) + "</listOfProducts>")
        modifiers = sorted({a for a in _names(law) if a in SPECIES and a not in re and a not in pr})
        if modifiers:
            out.append("        <listOfModifiers>" + "".join(f'<modifierSpeciesReference species="{s}"/>' for s in modifiers) + "</listOfModifiers>")
        out.append(f'        <kineticLaw><math xmlns="http://www.w3.org/1998/Math/MathML">{mathml(law)}</math></kineticLaw>')
        out.append('      </reaction>')
    out.append('    </listOfReactions>')
    out.append('  </model>')
    out.append('</sbml>')
    return "\n".join(out) + "\n"


def _names(e):
    if isinstance(e, str):
        yield e
    elif isinstance(e, tuple):
        for a in e[1:]:
            yield from _names(a)


def prior_text():
    rows = ['<?xml version="1.0" encoding="utf-8"?>', "<variableset>"]
    for name, lo, hi, logspace in PRIOR:
        ls = ' logspace="true"' if logspace else ""
        rows.append(f'  <variable name="{name}" distribution="uniform" lower="{lo}" upper="{hi}"{ls}/>')
    rows.append("</variableset>")
    return "\n".join(rows) + "\n"


def likelihood_text(num_cells=500, max_cells=2048, data_file="cellpop_data.json", model_file="cellpop_model.xml",
                    data_attrs='stdev="stdev"', experiment_attrs="", extra="", data_xml=None, entry_time="0",
                    variability_extra=""):
    """extra: further children of the <experiment> (e.g. a <treatment_trajectory>); data_xml: the
    <data> element(s) in place of the population average"""
    if data_xml is None:
        data_xml = f'<data type="time_course_population_average" data_name="pcna_mean" species_name="PCNA_gfp" {data_attrs}/>'
    return f"""<bcm_likelihood type="cell_population">
  <experiment name="exp1" model_file="{model_file}" data_file="{data_file}" num_cells="{num_cells}" max_cells="{max_cells}" entry_time="{entry_time}"{experiment_attrs}>
    <cell_variability distribution="diagonal_gaussian">
      <variable model_parameter="k_D" apply="multiplicative_log" scale="var_kD"/>
      <variable initial_condition_species="CycD" apply="multiplicative_log" scale="var_CycD0"/>{variability_extra}
    </cell_variability>
    {data_xml}{extra}
  </experiment>
</bcm_likelihood>
"""


def write_model_files(d=HERE):
    with open(os.path.join(d, "cellpop_model.xml"), "w") as f:
        f.write(sbml_text())
    with open(os.path.join(d, "cellpop_prior.xml"), "w") as f:
        f.write(prior_text())
    with open(os.path.join(d, "cellpop_likelihood.xml"), "w") as f:
        f.write(likelihood_text())


def true_values():
    return [TRUE[name] for name, *_ in PRIOR]


def write_data(d=HERE):
    import numpy as np
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
    import cellpop as CP
    # the data are needed to set the problem up; simulate with a placeholder data set first
    placeholder = {"exp1": {"time": {"dims": ["time"], "data": TIMES},
                            "pcna_mean": {"dims": ["time", "replicate"], "data": [[0.0] * REPLICATES for _ in TIMES]}}}
    with open(os.path.join(d, "cellpop_data.json"), "w") as f:
        json.dump(placeholder, f)
    prob = CP.load_problem(os.path.join(d, "cellpop_likelihood.xml"), os.path.join(d, "cellpop_prior.xml"))
    sim = CP.simulate(prob, np.array(true_values()))
    avg = sim["population_average"][0]
    rng = np.random.default_rng(20251017)
    sd = 10.0 ** TRUE["stdev"]
    obs = avg[:, None] + sd * rng.standard_normal((len(TIMES), REPLICATES))
    data = {"exp1": {"time": {"dims": ["time"], "data": TIMES},
                     "pcna_mean": {"dims": ["time", "replicate"], "data": obs.tolist()}}}
    with open(os.path.join(d, "cellpop_data.json"), "w") as f:
        json.dump(data, f, indent=1)
    print("cells", sim["num_cells"], "population average", np.round(avg, 3))


TC_CELLS = 16


def write_tc_data(d=HERE):
    """cellpop_tc_data.json: single-cell PCNA_gfp time courses for the time_course likelihood
    (DataLikelihoodTimeCourse): TC_CELLS non-dividing cells simulated at the true parameters plus
    noise, a few observations missing (NaN); the population average of cellpop_data.json
    alongside, a 1-D series (one cell) and a 3-D copy with a second marker"""
    import numpy as np
    import tempfile
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
    import cellpop as CP
    tmp = tempfile.mkdtemp()
    path = os.path.join(tmp, "l.xml")
    with open(path, "w") as f:
        f.write(likelihood_text(num_cells=TC_CELLS, max_cells=TC_CELLS, data_file=os.path.join(d, "cellpop_data.json"),
                                model_file=os.path.join(d, "cellpop_model.xml"), experiment_attrs=' divide_cells="false"'))
    prob = CP.load_problem(path, os.path.join(d, "cellpop_prior.xml"))
    sim = CP.simulate(prob, np.array(true_values()))
    cells = sim["detail"][0]["cells"]
    vals = np.array([c["values"] for c in cells])  # cells x times
    rng = np.random.default_rng(20261017)
    sd = 10.0 ** TRUE["stdev"]
    obs = vals.T + sd * rng.standard_normal((len(TIMES), TC_CELLS))
    for t, c in ((3, 2), (7, 5), (12, 11), (20, 0)):
        obs[t, c] = float("nan")
    with open(os.path.join(d, "cellpop_data.json")) as f:
        group = json.load(f)["exp1"]
    group["pcna_cells"] = {"dims": ["time", "cell"], "data": obs.tolist()}
    group["pcna_cell0"] = {"dims": ["time"], "data": obs[:, 1].tolist()}
    m2 = np.stack([obs, rng.standard_normal(obs.shape)], axis=2)
    group["pcna_cells_markers"] = {"dims": ["time", "cell", "marker"], "data": m2.tolist()}
    with open(os.path.join(d, "cellpop_tc_data.json"), "w") as f:
        json.dump({"exp1": group}, f, indent=1)


def write_tp_data(d=HERE):
    """adds to cellpop_tc_data.json the variants the time-points tests read (DataLikelihoodTimePoints
    takes 2-D or 3-D data only): pcna_cell0_2d (time x 1 cell, the data of pcna_cell0) and
    pcna_cells_late (pcna_cells without the observations of the first two time points)"""
    import math
    fn = os.path.join(d, "cellpop_tc_data.json")
    with open(fn) as f:
        doc = json.load(f)
    g = doc["exp1"]
    cells = g["pcna_cells"]["data"]
    g["pcna_cell0_2d"] = {"dims": ["time", "cell1"], "data": [[row[1]] for row in cells]}
    g["pcna_cells_late"] = {"dims": ["time", "cell"],
                            "data": [[math.nan] * len(row) if t < 2 else list(row) for t, row in enumerate(cells)]}
    with open(fn, "w") as f:
        json.dump(doc, f, indent=1)


if __name__ == "__main__":
    write_model_files()
    if "--data" in sys.argv:
        write_data()
    if "--tc-data" in sys.argv:
        write_tc_data()
    if "--tc-data" in sys.argv or "--tp-data" in sys.argv:
        write_tp_data()
