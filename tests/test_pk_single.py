"""The single-patient CVODE PK likelihood (type "pharmacokinetic_trajectory",
src/likelihoods/LikelihoodPharmacokineticTrajectory.cpp): the PopPK kernel with the single-patient
parameter map (BCM3HIP_PARAM_MAP_SINGLE).

CPU: the oracle's restatement equals the vendored CVODE built from the reference sources
(FMA off) bit for bit on every PK model and dosing rule, and the host layer's Initialize builds
the same device model as the oracle's restatement. GPU (marked): the kernel against the oracle
within the parity envelope (tests/parity.py), and through the host layer."""
import math
import os

import numpy as np
import pytest

import helpers as H
import oracle as O
import parity

GOLDEN = H.GOLDEN
HAVE_REF = os.path.exists(O.LIB_REF_NOFMA)
needs_ref = pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built (needs /root/reference)")
TYPES = ["one", "two", "one_biphasic_uptake", "two_biphasic_uptake", "one_transit", "two_transit"]


def _rule_kw(rule):
    return {"plain": {}, "intermittent1": dict(intermittent=1, T_days=10), "skipped": dict(skipped=(2, 3)),
            "dose_change": dict(dose_change=(500.0, 72.0)), "interval12": dict(interval=12.0)}[rule]


@needs_ref
@pytest.mark.parametrize("pk_type", TYPES)
@pytest.mark.parametrize("rule", ["plain", "intermittent1", "skipped", "dose_change", "interval12"])
def test_single_restated_bit_exact_vs_reference_cvode(pk_type, rule):
    prob, lo, hi, _ = H.make_single_problem(pk_type, **_rule_kw(rule))
    vals = H.draws(lo, hi, 48, 21)
    a = O.Oracle("restated").popk_eval(prob, vals, nthreads=4)
    b = O.Oracle("ref_nofma").popk_eval(prob, vals, nthreads=4)
    assert np.array_equal(a["traj"], b["traj"], equal_nan=True)
    assert np.array_equal(a["logp"], b["logp"], equal_nan=True)
    assert np.array_equal(a["ok"], b["ok"])
    # solver counters of the successful solves (a switch time past the dosing interval puts tstop
    # behind t after the switch: both fail with CV_ILL_INPUT, their RHS counts differ by one there)
    ok = a["ok"][:, 0] == 1
    assert np.array_equal(a["stats"][ok], b["stats"][ok])


def test_single_biphasic_switch_not_clamped():
    """The single-patient likelihood does not clamp the switch time into the dosing interval (the
    population one does, LikelihoodPopPKTrajectory.cpp:303-305): a switch after 30 h with a 24 h
    interval sets the next discontinuity (24 h) behind t, which CVode rejects -> -inf."""
    prob, lo, hi, _ = H.make_single_problem("two_biphasic_uptake", T_days=3)
    v = (lo + hi) / 2
    v[6] = math.log10(30.0)
    r = O.Oracle("restated").popk_eval(prob, v[None], nthreads=1)
    assert r["logp"][0] == -np.inf and r["ok"][0, 0] == 0
    v[6] = math.log10(10.0)
    assert np.isfinite(O.Oracle("restated").popk_eval(prob, v[None], nthreads=1)["logp"][0])


def _lik(options="backend=none", **kw):
    from bcm3_amd.likelihood import Likelihood
    return Likelihood(os.path.join(GOLDEN, "pk_single_likelihood.xml"), os.path.join(GOLDEN, "pk_single_prior.xml"),
                      options=options)


def _golden_single_problem():
    pk = O.load_pkdata(os.path.join(GOLDEN, "c3_pkdata.json"))
    import xml.etree.ElementTree as ET
    variables = []
    for v in ET.parse(os.path.join(GOLDEN, "pk_single_prior.xml")).getroot().iter("variable"):
        variables.append(O.Variable(v.get("name"), float(v.get("lower")), float(v.get("upper")),
                                    O.TF_LOG10 if v.get("logspace") == "true" else O.TF_NONE))
    return O.build_single_problem(pk, "SYN", "lapatinib", "two", variables, "P000")


def test_host_initialize_matches_oracle():
    import ctypes as C
    ll = _lik()
    m = ll.popk_model()
    prob = _golden_single_problem()
    for k in ("pk_type", "N", "d", "P", "T", "sd_ix", "n_transit_ix", "transit_time_ix", "biphasic_time_ix",
              "absorption2_ix", "max_steps", "param_map"):
        assert getattr(m, k) == getattr(prob, k), k
    assert m.rtol == prob.rtol and m.atol == prob.atol == 1250.0 * float(np.float32(1e-6)) and m.MW == prob.MW

    def arr(ptr, n, dt):
        return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dt))), shape=(n,)).copy()

    assert np.array_equal(arr(m.observed, prob.T, np.float64), prob.observed.reshape(-1), equal_nan=True)
    assert np.array_equal(arr(m.simulate_until, 1, np.int32), [prob.T])
    ll.close()


def test_host_patient_selection(tmp_path):
    from bcm3_amd.likelihood import Likelihood
    xml = tmp_path / "lik.xml"
    src = open(os.path.join(GOLDEN, "pk_single_likelihood.xml")).read()
    xml.write_text(src.replace('patient="P000"', 'patient="NOPE"').replace(
        'pkdata_file="c3_pkdata.json"', f'pkdata_file="{os.path.join(GOLDEN, "c3_pkdata.json")}"'))
    with pytest.raises(Exception):
        Likelihood(str(xml), os.path.join(GOLDEN, "pk_single_prior.xml"), options="backend=none")
    # the pk.patient option overrides the XML attribute (LikelihoodPharmacokineticTrajectory.cpp:101-104)
    ll = Likelihood(str(xml), os.path.join(GOLDEN, "pk_single_prior.xml"), options="backend=none;pk.patient=P000")
    assert ll.popk_model().param_map == 1
    ll.close()


@pytest.mark.gpu
@pytest.mark.parametrize("pk_type", TYPES)
@pytest.mark.parametrize("lpw", [1, 64])
def test_single_gpu_vs_oracle(pk_type, lpw):
    prob, lo, hi, _ = H.make_single_problem(pk_type, T_days=10)
    vals = H.draws(lo, hi, 512, 33)
    ctx = H.gpu_context(prob, lanes_per_wave=lpw)
    g = ctx.eval(vals, detail=True)
    o = O.Oracle("restated").popk_eval(prob, vals, nthreads=8)
    e = parity.y1_rel_err(g["traj"][:, 0, 1], o["traj"][:, 0, 1], prob.atol)
    le = parity.llh_err(g["logp"], o["logp"])
    ok_g = (g["status"] == 0).astype(np.int32)
    parity.assert_parity(e, le, g["stats"]["nst"][:, 0], o["stats"][:, 0, 0], ok_g, o["ok"][:, 0])


@pytest.mark.gpu
def test_single_host_layer_gpu():
    ll = _lik(options="device=0")
    prob = _golden_single_problem()
    lo = np.array([v.lower for v in prob.variables])
    hi = np.array([v.upper for v in prob.variables])
    vals = H.draws(lo, hi, 128, 5)
    logp, status = ll.evaluate_batch(vals)
    ref = O.Oracle("restated").popk_eval(prob, vals, nthreads=8)["logp"]
    le = parity.llh_err(logp, ref)
    assert np.mean(le <= parity.LLH_T1) >= 0.95 and np.all(le[np.isfinite(ref)] <= parity.LLH_T2)
    ll.close()
