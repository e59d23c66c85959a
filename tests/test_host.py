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
