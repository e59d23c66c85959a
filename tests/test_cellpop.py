"""CPU tests of the cell-population likelihood (config C4): the product's SBML reader and code
generator against the oracle's restatement of the reference's (oracle/sbml_codegen.py), the Sobol
sequence, and the oracle itself (reference CVODE + PartialPivLU, oracle/cellpop.py) on the
reference's cell bookkeeping rules."""
import ctypes as C
import math
import os

import numpy as np
import pytest

import cellpop_helpers as CH
import cellpop as CP
import sbml_codegen as SG


def _lik(path, prior=CH.PRIOR):
    from bcm3_amd.likelihood import Likelihood
    return Likelihood(path, prior, options="backend=none")


def test_generated_code_matches_restatement():
    ll = _lik(os.path.join(CH.GOLDEN, "cellpop_likelihood.xml"))
    code = ll.generated_code()
    model = SG.SBMLModel(os.path.join(CH.GOLDEN, "cellpop_model.xml"))
    assert code == model.generate_derivative(ll.variable_names)
    # the reference's formatting: constants through "%Lf", integer Hill exponents specialised,
    # sampled variables as parameters[], species in id order
    assert "hill_function_fixedn4(species[12],1.500000)" in code
    assert "(1.000000-hill_function_fixedn16(species[5],0.500000))" in code
    assert "ratelaws[0] = (parameters[0]*constant_species[0]);" in code
    ll.close()


def test_generated_code_mathml_forms(tmp_path):
    """every MathML form the reference's generator handles, C++ vs the restatement"""
    model = f"""<?xml version="1.0"?>
<sbml xmlns="http://www.sbml.org/sbml/level2/version4" level="2" version="4"><model id="m">
<listOfSpecies>
 <species id="s2" name="B" initialAmount="1.5"/><species id="s1" name="A" initialAmount="2"/>
 <species id="s3" name="C" initialAmount="0.25"/><species id="sink" name="gone" initialAmount="0">
  <annotation><celldesigner:extension xmlns:celldesigner="http://www.sbml.org/2001/ns/celldesigner">
   <celldesigner:speciesIdentity><celldesigner:class>DEGRADED</celldesigner:class></celldesigner:speciesIdentity>
  </celldesigner:extension></annotation></species>
</listOfSpecies>
<listOfParameters><parameter id="k1" value="0.0001234567"/><parameter id="km" value="3"/></listOfParameters>
<listOfReactions>
 <reaction id="z"><listOfReactants><speciesReference species="s1" stoichiometry="2"/></listOfReactants>
  <listOfProducts><speciesReference species="s2"/><speciesReference species="sink"/></listOfProducts>
  <kineticLaw><math xmlns="http://www.w3.org/1998/Math/MathML"><apply><plus/>
   <apply><times/><ci> k1 </ci><ci> s1 </ci><ci> s3 </ci></apply>
   <apply><minus/><ci> s2 </ci></apply>
   <apply><divide/><apply><exp/><ci> s1 </ci></apply><apply><ln/><ci> s2 </ci></apply></apply>
   <apply><power/><ci> s1 </ci><cn> 2.5 </cn></apply>
   <apply><ci> hill </ci><ci> s2 </ci><ci> km </ci><cn type="integer"> 3 </cn></apply>
   <apply><ci> hill </ci><ci> s2 </ci><ci> km </ci><cn type="integer"> 2 </cn></apply>
   <apply><ci> mm </ci><ci> k2 </ci><ci> km </ci><ci> s1 </ci><ci> s2 </ci></apply>
   <apply><ci> tQSSA </ci><ci> k2 </ci><ci> km </ci><ci> s1 </ci><ci> s2 </ci></apply>
  </apply></math></kineticLaw></reaction>
 <reaction id="a"><listOfProducts><speciesReference species="s1" stoichiometry="0.5"/></listOfProducts>
  <kineticLaw><math xmlns="http://www.w3.org/1998/Math/MathML"><apply><ci> synthcap </ci><ci> s2 </ci></apply></math></kineticLaw></reaction>
</listOfReactions></model></sbml>
"""
    (tmp_path / "m.xml").write_text(model)
    (tmp_path / "prior.xml").write_text('<variableset><variable name="k2" distribution="uniform" lower="0" upper="1"/>'
                                        '<variable name="stdev" distribution="uniform" lower="0.1" upper="1"/></variableset>')
    (tmp_path / "data.json").write_text('{"e": {"time": {"dims": ["time"], "data": [1.0, 2.0]}, '
                                        '"y": {"dims": ["time"], "data": [1.0, 2.0]}}}')
    (tmp_path / "lik.xml").write_text(
        f'<bcm_likelihood type="cell_population"><experiment name="e" model_file="{tmp_path}/m.xml" '
        f'data_file="{tmp_path}/data.json" num_cells="1" divide_cells="false" entry_time="0">'
        '<data type="time_course_population_average" data_name="y" species_name="A" stdev="stdev"/>'
        '</experiment></bcm_likelihood>')
    ll = _lik(str(tmp_path / "lik.xml"), str(tmp_path / "prior.xml"))
    code = ll.generated_code()
    ref = SG.SBMLModel(str(tmp_path / "m.xml")).generate_derivative(ll.variable_names)
    assert code == ref
    assert "constant_species[0]" in code and "0.000123" in code and "hill_function_fixedn2(" in code
    assert "hill_function(species[1],3.000000,3.000000)" in code and "0.500000*ratelaws[0]" in code
    assert "-2.000000*ratelaws[1]" in code and "sink" not in code
    ll.close()


def test_sobol_sequence_matches_restatement():
    from bcm3_amd.likelihood import lib
    L = lib()
    for dims in (1, 2, 5, 13):
        out = np.empty((3000, dims))
        L.bcm3_sobol_points(C.c_size_t(3000), C.c_size_t(dims), out.ctypes.data_as(C.c_void_p))
        assert np.array_equal(out, CP.sobol_points(3000, dims))
    p = CP.sobol_points(8, 2)
    # Gray-code order, the zero point skipped (boost::random::sobol's first point is 0.5)
    assert np.array_equal(p[:4, 0], [0.5, 0.75, 0.25, 0.375])
    # every coordinate of a 2^k prefix + the skipped zero is a permutation of the k-bit grid
    p = CP.sobol_points(255, 3)
    for d in range(3):
        assert np.array_equal(np.sort(np.concatenate([[0.0], p[:, d]])), np.arange(256) / 256.0)


def test_unsupported_options_fail_loudly(tmp_path, capfd):
    path = CH.write_likelihood(tmp_path, 4, 64)
    text = open(path).read()
    # VariabilityDescription::Load (VariabilityDescription.cpp:184-212): an unknown distribution, and
    # full_gaussian without covar_base_name, fail to load
    for bad, msg in ((text.replace('"diagonal_gaussian"', '"lognormal"'), 'Unknown distribution "lognormal"'),
                     (text.replace('"diagonal_gaussian"', '"full_gaussian"'), "covar_base_name")):
        (tmp_path / "bad.xml").write_text(bad)
        with pytest.raises(RuntimeError):
            _lik(str(tmp_path / "bad.xml"))
        assert msg in capfd.readouterr().err


def test_full_gaussian_variability_loads(tmp_path, capfd):
    lik, prior = CH.write_full_gaussian(tmp_path, 4, 64)
    _lik(lik, prior).close()
    e = CP.load_problem(lik, prior)["experiments"][0]
    assert e["variability_cov"] == [[("var", 7)]]
    # the covariance references must be sampled variables or numbers (ValueReference::Load;
    # "Missing parameter for covariance", VariabilityDescription.cpp:40-44)
    lik2, _ = CH.write_full_gaussian(tmp_path, 4, 64, covar_base_name="corr")
    with pytest.raises(RuntimeError):
        _lik(lik2, prior)
    assert "Missing parameter for covariance" in capfd.readouterr().err


def test_oracle_full_gaussian_factor():
    """the oracle's spherical Cholesky factor (VariabilityDescription.cpp:99-118) for D = 2 applied
    additively to two parameters: L = [[e^s0, 0], [e^s1 cos(pi rho), e^s1 sin(pi rho)]], vector L z"""
    import math

    class Model:
        ode, species = [], []
    vv = [dict(scale=("fixed", 0.1), parameter="a", species="", apply="additive", negate=False, only_initial=False),
          dict(scale=("fixed", -0.2), parameter="b", species="", apply="additive", negate=False, only_initial=False)]
    e = {"variabilities": [vv], "variability_cov": [[("fixed", 0.25)]], "sobol": np.array([[0.8, 0.3]]),
         "model": Model}
    params, _ = CP._cell_init(e, {"variables": ["a", "b"]}, [0.0, 0.0], [], 0, True)
    z0, z1 = CP.quantile_normal(0.8), CP.quantile_normal(0.3)
    c, sn = math.cos(0.25 * math.pi), math.sin(0.25 * math.pi)
    want = [math.exp(0.1) * z0, math.exp(-0.2) * c * z0 + math.exp(-0.2) * sn * z1]
    assert np.allclose(params, want, rtol=1e-14)


@pytest.fixture(scope="module")
def small_problem(tmp_path_factory):
    d = tmp_path_factory.mktemp("cellpop")
    return CP.load_problem(CH.write_likelihood(d, 4, 64), CH.PRIOR)


def test_oracle_cell_bookkeeping(small_problem):
    """Experiment::Simulate's rules on the oracle run: FIFO numbering of daughters, daughters start at
    the division step of their parent, reset species, Sobol indices initial + 2*parent + child."""
    r = CP.simulate_experiment(small_problem["experiments"][0], small_problem, np.array(CH.F.true_values()))
    cells = r["cells"]
    assert r["ok"] and len(cells) == 12  # 4 initial cells, each divides once before 20 h
    for c in cells[:4]:
        assert c["parent"] == -1 and c["creation"] == 0.0 and c["divided"]
    for k, c in enumerate(cells[4:]):
        parent = cells[k // 2]
        assert c["parent"] == parent["index"]
        assert c["creation"] == parent["achieved"] == parent["sim_end"]  # created at t_div
        assert c["sobol_ix"] == 4 + parent["sobol_ix"] * 2 + (k % 2)
        assert not c["divided"]
    e = small_problem["experiments"][0]
    for k, c in enumerate(cells[4:]):
        y0 = c["y0"]
        for ix, v in e["reset"]:
            assert y0[ix] == v
    # the data values: NaN before creation and after a division
    for c in cells:
        for k, t in enumerate(e["output_times"]):
            ct = t - c["creation"]
            assert (ct < 0.0 or ct > c["sim_end"]) == math.isnan(c["values"][k])


def test_oracle_max_cells_fails(tmp_path):
    prob = CP.load_problem(CH.write_likelihood(tmp_path, 4, 10), CH.PRIOR)
    r = CP.simulate(prob, np.array([CH.F.true_values()]))
    assert r["logp"][0] == -math.inf


def test_oracle_logp_near_truth_is_higher(small_problem):
    x = CH.draws(6, 3)
    lp = CP.simulate(small_problem, x)["logp"]
    assert np.all(np.isfinite(lp) | (lp == -math.inf))
    assert lp[0] == lp.max()


def test_error_model_options(tmp_path):
    """DataLikelihoodBase::Load's error models: the proportional ones need proportional_stdev;
    unknown names fail, as in the reference"""
    from bcm3_amd.likelihood import Likelihood
    ok = [('stdev="stdev" error_model="proportional_normal" proportional_stdev="0.1"', ""),
          ('stdev="stdev" error_model="additive_proportional_normal" proportional_stdev="stdev"', ""),
          ('stdev="stdev" error_model="student_t4"', ' divide_cells="false"')]
    for i, (da, ea) in enumerate(ok):
        path = CH.write_likelihood(tmp_path, 4, 16, name=f"ok{i}.xml", data_attrs=da, experiment_attrs=ea)
        Likelihood(path, CH.PRIOR, options="backend=none").close()
        prob = CP.load_problem(path, CH.PRIOR)
        assert prob["experiments"][0]["data"][0]["error_model"] in ("proportional", "additive_proportional", "t4")
    for i, da in enumerate(['stdev="stdev" error_model="proportional_normal"', 'stdev="stdev" error_model="laplace"']):
        path = CH.write_likelihood(tmp_path, 4, 16, name=f"bad{i}.xml", data_attrs=da)
        with pytest.raises(RuntimeError):
            Likelihood(path, CH.PRIOR, options="backend=none")


def test_proportional_error_oracle_formula(tmp_path):
    """the oracle's additive-proportional term: LogPdfNormal(x, o, stdev + ps max(o, 0)) per
    replicate, with the population-average data value in the 'simulated' role (argument swap)"""
    import math
    d = dict(stdev=("fixed", 0.2), offset=None, scale=None, relative_to_time_average=False, weight=1.0,
             error_model="additive_proportional", proportional_stdev=("fixed", 0.1),
             observed=np.array([[1.0, -0.5]]), times=[0.0, 1.0])
    avg = np.array([[0.9], [0.1]])
    got = CP._popavg_logp(d, avg, [])
    want = 0.0
    for x, o in ((0.9, 1.0), (0.1, -0.5)):
        s = 0.2 + 0.1 * max(o, 0.0)
        want += -math.log(s) - 0.91893853320467274178032973640562 - (x - o) ** 2 / (2 * s * s)
    assert abs(got - want) < 1e-14


def test_several_experiments_load(tmp_path):
    """CellPopulationLikelihood::Initialize loads every <experiment> (CellPopulationLikelihood.cpp:
    24-35); a likelihood without one is an error"""
    import test_cellpop_experiments_gpu as TE
    from bcm3_amd.likelihood import Likelihood
    _, _, ab = TE.two_experiments(tmp_path)
    Likelihood(ab, CH.PRIOR, options="backend=none").close()
    assert len(CP.load_problem(ab, CH.PRIOR)["experiments"]) == 2
    none = tmp_path / "none.xml"
    none.write_text('<bcm_likelihood type="cell_population">\n</bcm_likelihood>\n')
    with pytest.raises(RuntimeError):
        Likelihood(str(none), CH.PRIOR, options="backend=none")


def test_treatment_trajectory_options(tmp_path):
    """<treatment_trajectory> (Experiment.cpp:571-584, TreatmentTrajectory::Create): pulses load, with
    their times sorted; from_data fails (its loader returns failure in the reference), unknown types
    and non-constant species fail; pulses that end before the experiment does are refused (the
    reference would carry a stale discontinuity between the cells of its pool)"""
    from bcm3_amd.likelihood import Likelihood
    good = '\n    <treatment_trajectory type="pulses" species_name="mitogen" times="13,-1"/>'
    path = CH.write_likelihood(tmp_path, 4, 16, name="treat_ok.xml", extra=good)
    Likelihood(path, CH.PRIOR, options="backend=none").close()
    e = CP.load_problem(path, CH.PRIOR)["experiments"][0]
    assert e["treatments"] == [(0, [-1.0, 13.0])]
    bad = ['\n    <treatment_trajectory type="from_data" species_name="mitogen"/>',
           '\n    <treatment_trajectory type="steps" species_name="mitogen" times="1"/>',
           '\n    <treatment_trajectory type="pulses" species_name="CycD" times="1"/>',
           '\n    <treatment_trajectory type="pulses" species_name="mitogen" times="0,2"/>',
           '\n    <treatment_trajectory type="pulses" species_name="mitogen" times="1,x"/>']
    for i, b in enumerate(bad):
        p = CH.write_likelihood(tmp_path, 4, 16, name=f"treat_bad{i}.xml", extra=b)
        with pytest.raises(RuntimeError):
            Likelihood(p, CH.PRIOR, options="backend=none")


def test_oracle_runs_treatment_trajectory(tmp_path):
    """the oracle with a pulse treatment on mitogen (the constant species of CycD synthesis): mitogen is
    0 outside the pulses, so the treated population divides later than the untreated one (mitogen 1)"""
    good = '\n    <treatment_trajectory type="pulses" species_name="mitogen" times="13,-1"/>'
    treated = CP.load_problem(CH.write_likelihood(tmp_path, 4, 32, name="t.xml", extra=good), CH.PRIOR)
    plain = CP.load_problem(CH.write_likelihood(tmp_path, 4, 32, name="p.xml"), CH.PRIOR)
    x = CH.draws(2, 5)
    rt, rp = CP.simulate(treated, x), CP.simulate(plain, x)
    for i in range(2):
        ct, cp = rt["detail"][i]["cells"], rp["detail"][i]["cells"]
        assert all(c["ok"] for c in ct if "ok" in c)
        first_t = min(c["sim_end"] for c in ct[:4] if c["divided"]) if any(c["divided"] for c in ct[:4]) else 1e9
        first_p = min(c["sim_end"] for c in cp[:4] if c["divided"]) if any(c["divided"] for c in cp[:4]) else 1e9
        assert first_t > first_p, (i, first_t, first_p)


def test_entry_time_variability_takes_a_dimension(tmp_path):
    """<variable entry_time="true" ...> loads, gets a column of the Sobol table and no target
    (VariabilityDescriptionVariable.cpp:66-78 is never called by the reference)"""
    import make_cellpop_fixtures as F
    path = tmp_path / "lik.xml"
    path.write_text(F.likelihood_text(num_cells=4, max_cells=64, data_file=os.path.join(CH.GOLDEN, "cellpop_data.json"),
                                      model_file=os.path.join(CH.GOLDEN, "cellpop_model.xml"),
                                      variability_extra='<variable entry_time="true" apply="additive" scale="var_kD"/>'))
    _lik(str(path)).close()
    e = CP.load_problem(str(path), CH.PRIOR)["experiments"][0]
    assert e["sobol"].shape[1] == 3 and e["variabilities"][0][2]["entry_time"]
