"""pharmaco_population: every patient of a trial, rates drawn per patient from the population
distribution, linear compartment PK by matrix exponentials, log-likelihoods summed in patient order
(src/pharmaco/PharmacoLikelihoodPopulation.cpp:43-356, PharmacokineticModel.cpp:111-247).

CPU: the restated likelihood (oracle/expm_pk.py, param_map 0) against the golden fixture made with
the reference's vendored Eigen (tests/golden/make_pharmaco_population_fixtures.py); the host
layer's Initialize/PostInitialize (all patients concatenated, p<i>_* indices, sigma_* switches)
against the restatement; its error behaviour (missing p<i>_ variable, missing means).
GPU (marked): the HIP kernel (expm_pk_kernel.hip: one wavefront per (evaluation, patient), then a
patient-ordered sum) through the host layer and the C-ABI against the golden fixture.
Tolerance |dlogp| <= 1e-9 (1 + |logp|) as for pharmaco_single; QuantileNormal is Boost's in the
reference, a rational guess + 3 Halley steps on the device and scipy's ndtri in the restatement
(all within a few ulp of the exact quantile)."""
import json
import os

import numpy as np
import pytest

import expm_pk as X
import make_pharmaco_population_fixtures as F

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
PKDATA = os.path.join(GOLDEN, "pharmaco_pkdata.json")
GOLD = np.load(os.path.join(GOLDEN, "pharmaco_population_golden.npz"))
LLH_TOL = 1e-9


def _pkdata():
    with open(PKDATA) as f:
        return json.load(f)


def _files(tmp_path, variant, prior_text=None):
    lx = tmp_path / f"pop_{variant}.xml"
    lx.write_text(F.likelihood_xml(variant, PKDATA))
    px = tmp_path / f"pop_{variant}_prior.xml"
    px.write_text(prior_text if prior_text is not None else F.prior_xml(variant))
    return str(lx), str(px)


def _close(a, b, tol=LLH_TOL):
    a, b = np.asarray(a), np.asarray(b)
    fin = np.isfinite(b)
    return np.array_equal(np.isfinite(a), fin) and np.all(np.abs(a[fin] - b[fin]) <= tol * (1 + np.abs(b[fin])))


def _read(ptr, n, dtype):
    import ctypes
    ct = ctypes.c_int32 if dtype == np.int32 else ctypes.c_double
    return np.array((ct * n).from_address(ptr), dtype=dtype)


@pytest.mark.parametrize("variant", list(F.VARIANTS))
def test_restated_population_matches_golden(variant):
    m = F.model_fields(variant, _pkdata())
    v = GOLD[f"{variant}_values"]
    logp, ok = X.evaluate(m, v)
    assert np.array_equal(ok, GOLD[f"{variant}_ok"])
    assert _close(logp, GOLD[f"{variant}_logp"], 1e-12)


def test_population_is_the_sum_of_single_patients():
    """with no random effect every patient sees the mean rates: the population logp is the sum of
    the pharmaco_single logps of its patients at those rates"""
    import make_pharmaco_fixtures as S
    pk = _pkdata()
    m = F.model_fields("mean_only", pk)
    v = GOLD["mean_only_values"][:6]
    nm = F.names("mean_only")
    want = np.zeros(len(v))
    for pid in pk[S.TRIAL]["patients"]:
        s = S.model_fields("plain", pid, pk)
        sv = np.zeros((len(v), s["d"]))
        for k, n in enumerate(["absorption", "clearance", "volume_of_distribution", "excretion"]):
            sv[:, [p[0] for p in S.PRIOR].index(n)] = v[:, nm.index("mean_" + n)]
        for n in ("additive_error_standard_deviation", "proportional_error_standard_deviation"):
            sv[:, [p[0] for p in S.PRIOR].index(n)] = v[:, nm.index(n)]
        want += X.evaluate(s, sv)[0]
    assert _close(X.evaluate(m, v)[0], want, 1e-13)


def test_quantile_normal():
    assert X.quantile_normal(0.5, 1.25, 0.3) == 1.25
    assert abs(X.quantile_normal(0.975, 0.0, 1.0) - 1.959963984540054) < 1e-15


@pytest.mark.parametrize("variant", ["mean_only", "random", "all"])
def test_host_layer_builds_the_restated_model(tmp_path, variant):
    from bcm3_amd.likelihood import Likelihood
    ll = Likelihood(*_files(tmp_path, variant), options="backend=none")
    m = ll.expm_pk_model()
    want = F.model_fields(variant, _pkdata())
    P = want["P"]
    sizes = {"transforms": m.d, "treat_times": m.n_treat, "treat_doses": m.n_treat, "obs_times": m.n_obs,
             "obs_conc": m.n_obs, "patient_ix": 6 * P, "treat_offset": P + 1, "obs_offset": P + 1}
    for k, v in want.items():
        if k in sizes:
            ct = np.float64 if k in ("treat_times", "treat_doses", "obs_times", "obs_conc") else np.int32
            assert np.array_equal(_read(getattr(m, k), sizes[k], ct), np.asarray(v, dtype=ct)), k
        elif k == "sigma_ix":
            assert list(m.sigma_ix) == v, k
        else:
            assert getattr(m, k) == v, k
    ll.close()


def test_host_layer_errors(tmp_path):
    from bcm3_amd.likelihood import Likelihood
    # sigma_clearance present, p2_clearance missing (InitializePatientMarginals)
    bad = F.prior_xml("random").replace('name="p2_clearance"', 'name="q2_clearance"')
    with pytest.raises(RuntimeError):
        Likelihood(*_files(tmp_path, "random", bad), options="backend=none")
    # no mean_clearance
    bad = F.prior_xml("mean_only").replace('name="mean_clearance"', 'name="clearance"')
    with pytest.raises(RuntimeError):
        Likelihood(*_files(tmp_path, "mean_only", bad), options="backend=none")
    # bioavailability requested, p<i>_bioavailability missing
    bad = F.prior_xml("all").replace('name="p1_bioavailability"', 'name="p1_ba"')
    with pytest.raises(RuntimeError):
        Likelihood(*_files(tmp_path, "all", bad), options="backend=none")


# ---------------------------------------------------------------------------------------------
# GPU

@pytest.mark.gpu
@pytest.mark.parametrize("variant", list(F.VARIANTS))
def test_gpu_matches_golden(tmp_path, variant):
    from bcm3_amd.likelihood import Likelihood
    ll = Likelihood(*_files(tmp_path, variant), device=0)
    v = GOLD[f"{variant}_values"]
    logp, status = ll.evaluate_batch(v)
    assert np.all(status == 0)
    ref = GOLD[f"{variant}_logp"]
    assert _close(logp, ref), np.max(np.abs(logp - ref) / (1 + np.abs(ref)))
    ll.close()


@pytest.mark.gpu
def test_gpu_c_abi_batch_invariance_and_failures():
    from bcm3_amd import _hip
    m = F.model_fields("all", _pkdata())
    ctx = _hip.Context.expm_pk(m, device=0)
    v = F.draws("all", 1024, 11)
    a = ctx.eval(v)[0]
    b = ctx.eval(v[300:333])[0]
    assert np.array_equal(a[300:333], b)
    ref, _ = X.evaluate(m, v[:48])
    assert _close(a[:48], ref)
    # a non-finite rate in one patient makes the whole evaluation -inf
    w = v[:4].copy()
    w[1, F.names("all").index("p2_clearance")] = np.nan
    w[2, F.names("all").index("mean_volume_of_distribution")] = 400.0
    logp, status = ctx.eval(w)[:2]
    ref, _ = X.evaluate(m, w)
    assert np.array_equal(np.isfinite(logp), np.isfinite(ref))
    assert _close(logp[[0, 3]], ref[[0, 3]])
    assert ctx.eval(v[:0])[0].shape == (0,)
