"""CPU tests of the C++ host layer (libbcm3.so, include/bcm3.h) without a device: XML/JSON
loading, VariableSet, LikelihoodFactory dispatch and the restated
LikelihoodPopPKTrajectory::Initialize, compared with the oracle's independent restatement."""
import ctypes as C
import math
import os

import numpy as np
import pytest

import helpers as H
import oracle as O

GOLDEN = H.GOLDEN


def _lik(name, options="backend=none"):
    from bcm3_amd.likelihood import Likelihood
    return Likelihood(os.path.join(GOLDEN, f"{name}_likelihood.xml"), os.path.join(GOLDEN, f"{name}_prior.xml"),
                      options=options)


def _arr(ptr, n, dt):
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dt))), shape=(n,)).copy()


@pytest.mark.parametrize("name,P", [("c3", 1), ("p64", 64)])
def test_popk_initialize_matches_oracle(name, P):
    ll = _lik(name)
    m = ll.popk_model()
    prob = H.c3_problem(P)
    for k in ("pk_type", "N", "num_pk_params", "num_pk_pop_params", "d", "P", "T", "sd_ix", "n_transit_ix",
              "transit_time_ix", "biphasic_time_ix", "absorption2_ix", "max_steps"):
        assert getattr(m, k) == getattr(prob, k), k
    for k in ("rtol", "atol", "MW"):
        assert getattr(m, k) == getattr(prob, k), k
    assert math.isnan(m.fixed_vod) and math.isnan(m.fixed_kf) and math.isnan(m.fixed_kb)
    T, d = prob.T, prob.d
    assert np.array_equal(_arr(m.transforms, d, np.int32), prob.transforms)
    assert np.array_equal(_arr(m.time, T, np.float64), prob.time)
    assert np.array_equal(_arr(m.observed, P * T, np.float64), prob.observed.reshape(-1), equal_nan=True)
    assert np.array_equal(_arr(m.dose, P, np.float64), prob.dose)
    assert np.array_equal(_arr(m.dosing_interval, P, np.float64), prob.dosing_interval)
    assert np.array_equal(_arr(m.simulate_until, P, np.int32), prob.simulate_until)
    assert np.array_equal(_arr(m.skipped_days, P * 29, np.uint8), prob.skipped_days.reshape(-1))
    assert ll.variable_names == [v.name for v in prob.variables]
    ll.close()


def test_tolerances_are_float_literals():
    m = _lik("c3").popk_model()
    # SetTolerance(1e-6f, minimum_dose * 1e-6f) (LikelihoodPopPKTrajectory.cpp:238)
    assert m.rtol == float(np.float32(1e-6))
    assert m.atol == 1250.0 * float(np.float32(1e-6))


def test_wrong_variable_count_is_rejected(tmp_path):
    from bcm3_amd.likelihood import Likelihood
    prior = tmp_path / "prior.xml"
    lines = open(os.path.join(GOLDEN, "c3_prior.xml")).read().splitlines()
    prior.write_text("\n".join(l for l in lines if "patient0_clearance" not in l))
    lik = tmp_path / "lik.xml"
    lik.write_text(open(os.path.join(GOLDEN, "c3_likelihood.xml")).read().replace(
        'pkdata_file="c3_pkdata.json"', f'pkdata_file="{os.path.join(GOLDEN, "c3_pkdata.json")}"'))
    with pytest.raises(RuntimeError, match="Incorrect number of variables in prior"):
        Likelihood(str(lik), str(prior), options="backend=none")


def test_unknown_type_and_missing_node(tmp_path):
    from bcm3_amd.likelihood import Likelihood
    lik = tmp_path / "lik.xml"
    lik.write_text('<bcm_likelihood type="no_such_type"/>')
    with pytest.raises(RuntimeError, match="Unknown likelihood type"):
        Likelihood(str(lik), os.path.join(GOLDEN, "banana_prior.xml"), options="backend=none")
    lik.write_text('<something_else type="banana"/>')
    with pytest.raises(RuntimeError, match="bcm_likelihood"):
        Likelihood(str(lik), os.path.join(GOLDEN, "banana_prior.xml"), options="backend=none")


def test_analytic_configs_load():
    b = _lik("banana")
    c = _lik("circular")  # width="=0.1" falls back to the default 0.1 as in the reference
    assert b.d == 2 and c.d == 2
    assert b.variable_names == ["x1", "x2"]


def test_no_cpu_fallback():
    ll = _lik("c3")
    with pytest.raises(RuntimeError, match="No GPU context"):
        ll.evaluate(np.zeros(12))


def test_repeat_and_transforms(tmp_path):
    from bcm3_amd.likelihood import Likelihood
    prior = tmp_path / "prior.xml"
    prior.write_text('<prior><variable name="a" distribution="uniform" lower="0" upper="1" repeat="3" '
                     'logspace="true"/><variable name="b" distribution="uniform" lower="0" upper="1" '
                     'logistic="true"/></prior>')
    lik = tmp_path / "lik.xml"
    lik.write_text('<bcm_likelihood type="circular" dimension="4"/>')
    ll = Likelihood(str(lik), str(prior), options="backend=none")
    assert ll.variable_names == ["a_0", "a_1", "a_2", "b"]
    assert ll.variable_transforms == [2, 2, 2, 3]


DIRICHLET_PRIOR = """<?xml version="1.0" encoding="utf-8"?>
<variableset>
  <variable name="x" distribution="uniform" lower="-1.0" upper="2.0"/>
  <variable name="w0" multivariate="true" id="1" distribution="dirichlet" alpha="2.0"/>
  <variable name="w1" multivariate="true" id="1" distribution="dirichlet" alpha="3.0"/>
  <variable name="w2" multivariate="true" id="1" distribution="dirichlet" alpha="4.5"/>
  <variable name="y" distribution="normal" mu="0.5" sigma="2.0"/>
  <variable name="v0" multivariate="true" id="2" distribution="dirichlet" alpha="0.5"/>
  <variable name="v1" multivariate="true" id="2" distribution="dirichlet" alpha="1.5"/>
</variableset>
"""


def _host_prior(path, d_max=16):
    import ctypes as C
    from bcm3_amd.likelihood import lib
    L = lib()
    L.bcm3_prior_marginals.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    kind = np.zeros(d_max, dtype=np.int32)
    par, bnd, mom = np.zeros((d_max, 3)), np.zeros((d_max, 2)), np.zeros((d_max, 2))
    d = L.bcm3_prior_marginals(str(path).encode(), d_max, kind.ctypes.data, par.ctypes.data, bnd.ctypes.data,
                               mom.ctypes.data)
    return d, kind[:max(d, 0)], par[:max(d, 0)], bnd[:max(d, 0)], mom[:max(d, 0)]


def test_dirichlet_prior_host_parse(tmp_path):
    """PriorIndependence's multivariate groups (PriorIndependence.cpp:20-115, MultivariateMarginal.cpp):
    libbcm3's parse equals the Python one the GPU tests restate, with the reference's moments, bounds
    and log normalisation constant lgamma(sum a) - sum lgamma(a_i)"""
    import math
    from bcm3_amd.sampler import PRIOR_KINDS, load_prior
    p = tmp_path / "prior.xml"
    p.write_text(DIRICHLET_PRIOR)
    d, kind, par, bnd, mom = _host_prior(p)
    assert d == 7 and kind.tolist() == [0, 8, 8, 8, 1, 8, 8]
    py = load_prior(str(p))
    for i, m in enumerate(py):
        assert PRIOR_KINDS[m.kind] == kind[i]
        # (p2 of a Dirichlet member is lgamma-based: glibc's lgamma here, CPython's own in load_prior)
        np.testing.assert_allclose(par[i], m.p, rtol=4e-16, atol=0)
        assert tuple(bnd[i]) == m.bounds() and tuple(mom[i]) == m.moments()
    a = [2.0, 3.0, 4.5]
    lnc = math.lgamma(sum(a)) - sum(math.lgamma(x) for x in a)
    assert par[1, 2] == par[3, 2] and abs(par[1, 2] - lnc) < 1e-13
    assert par[5, 1] == 5.0 and par[6, 1] == 5.0 and tuple(bnd[6]) == (0.0, 1.0)
    s = sum(a)
    assert abs(mom[2, 0] - 3.0 / s) < 1e-16 and abs(mom[2, 1] - 3.0 * (s - 3.0) / (s * s * (s + 1))) < 1e-16


@pytest.mark.parametrize("body,msg", [
    ('<variable name="w0" multivariate="true" id="1" distribution="dirichlet" alpha="2"/>'
     '<variable name="x" distribution="uniform" lower="0" upper="1"/>'
     '<variable name="w1" multivariate="true" id="1" distribution="dirichlet" alpha="2"/>', "follow each other"),
    ('<variable name="w0" multivariate="true" id="1" distribution="wishart" alpha="2"/>', "only dirichlet"),
    ('<variable name="w0" multivariate="true" id="0" distribution="dirichlet" alpha="2"/>', "start at 1"),
    ('<variable name="w0" multivariate="true" id="1" repeat="2" distribution="dirichlet" alpha="2"/>', "repeat"),
    # ids out of order: group 1's first member still names its distribution
    ('<variable name="v0" multivariate="true" id="2" distribution="dirichlet" alpha="2"/>'
     '<variable name="w0" multivariate="true" id="1" distribution="wishart" alpha="2"/>', "only dirichlet"),
])
def test_dirichlet_prior_errors(tmp_path, body, msg):
    from bcm3_amd.likelihood import lib
    p = tmp_path / "prior.xml"
    p.write_text(f'<?xml version="1.0"?>\n<variableset>{body}</variableset>\n')
    d = _host_prior(p)[0]
    assert d < 0 and msg in lib().bcm3_last_error().decode()
