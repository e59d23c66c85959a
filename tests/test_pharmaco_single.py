"""pharmaco_single: one patient, linear compartment PK solved by matrix exponentials
(src/pharmaco/PharmacoLikelihoodSingle.cpp, PharmacokineticModel.cpp, PharmacoPatient.cpp).

CPU: the restated Eigen matrix exponential (oracle/expm_pk.py) against the vendored Eigen itself
(oracle/_ref/libexpmref.so) on every Pade branch; the restated likelihood against the golden
fixture made with the Eigen build; the host layer's Initialize/PostInitialize (treatment schedule,
observation filter, variable indices) against the restatement; its error behaviour.
GPU (marked): the HIP kernel (expm_pk_kernel.hip) through the host layer and through the C-ABI
against the golden fixture. Tolerance: |dlogp| <= 1e-9 (1 + |logp|) -- the kernel's sums use
fused multiply-adds and Eigen's vectorised products round differently, nothing else differs."""
import os

import numpy as np
import pytest

import expm_pk as X
import make_pharmaco_fixtures as F

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
PKDATA = os.path.join(GOLDEN, "pharmaco_pkdata.json")
PRIOR = os.path.join(GOLDEN, "pharmaco_prior.xml")
GOLD = np.load(os.path.join(GOLDEN, "pharmaco_single_golden.npz"))
HAVE_REF = os.path.exists(X.LIB_EXPM_REF)
needs_ref = pytest.mark.skipif(not HAVE_REF, reason="oracle/_ref not built (needs /root/reference)")
CASES = [(v, p) for v in F.VARIANTS for p in F.PATIENTS]
LLH_TOL = 1e-9


def _pkdata():
    import json
    with open(PKDATA) as f:
        return json.load(f)


def _xml(tmp_path, variant, patient):
    p = tmp_path / f"{variant}_{patient}.xml"
    p.write_text(F.likelihood_xml(variant, patient, PKDATA))
    return str(p)


def _close(a, b, tol=LLH_TOL):
    a, b = np.asarray(a), np.asarray(b)
    same_inf = np.array_equal(np.isfinite(a), np.isfinite(b))
    fin = np.isfinite(b)
    return same_inf and np.all(np.abs(a[fin] - b[fin]) <= tol * (1 + np.abs(b[fin])))


def _random_matrix(n, scale, seed):
    r = np.random.default_rng(seed)
    return (r.standard_normal((n, n)) * scale)


@needs_ref
@pytest.mark.parametrize("n", [2, 3, 5, 8])
@pytest.mark.parametrize("scale", [1e-3, 2e-2, 0.1, 0.3, 1.0, 8.0, 60.0])
def test_restated_expm_matches_eigen(n, scale):
    for s in range(4):
        M = _random_matrix(n, scale / n, 100 * n + s)
        a = X.expm(M)
        b = X.expm_ref(M)
        assert np.max(np.abs(a - b)) <= 1e-12 * max(1.0, np.max(np.abs(b))), (n, scale, s)


@needs_ref
def test_expm_every_pade_degree_matches_eigen():
    # 1-norms inside each of Eigen's double-precision branches (MatrixExponential.h:245-258)
    R = _random_matrix(4, 1.0, 5)
    R /= np.max(np.sum(np.abs(R), axis=0))
    for target in (0.01, 0.1, 0.5, 1.5, 5.0, 300.0):
        M = R * target
        a, b = X.expm(M), X.expm_ref(M)
        assert np.max(np.abs(a - b)) <= 1e-12 * max(1.0, np.max(np.abs(b))), target


def test_expm_known_values():
    # exp of a diagonal and of a nilpotent matrix
    D = np.diag([-0.5, -2.0, -30.0])
    assert np.allclose(X.expm(D), np.diag(np.exp([-0.5, -2.0, -30.0])), rtol=1e-13, atol=0)
    N = np.array([[0.0, 1.0], [0.0, 0.0]]) * 5.0
    assert np.allclose(X.expm(N), [[1.0, 5.0], [0.0, 1.0]], rtol=1e-14, atol=1e-14)
    assert np.array_equal(X.expm(np.zeros((3, 3))), np.eye(3))


@pytest.mark.parametrize("variant,patient", CASES)
def test_restated_likelihood_matches_golden(variant, patient):
    m = F.model_fields(variant, patient, _pkdata())
    v = GOLD[f"{variant}_{patient}_values"][:16]
    logp, ok = X.evaluate(m, v)
    assert np.array_equal(ok, GOLD[f"{variant}_{patient}_ok"][:16])
    assert _close(logp, GOLD[f"{variant}_{patient}_logp"][:16])


@needs_ref
def test_ref_solve_reproduces_golden():
    m = F.model_fields("all", "B2", _pkdata())
    v = GOLD["all_B2_values"][:8]
    logp, _ = X.evaluate(m, v, backend="ref")
    assert np.array_equal(logp, GOLD["all_B2_logp"][:8])


def test_treatment_schedule_rules():
    # PharmacoPatient::Load: doses every interval up to 696 h, skipped days, intermittent
    # schedules, dose change at / after the change time
    t, d = X.treatment_schedule(1250.0, 24.0)
    assert len(t) == 29 and t[-1] == 672.0 and np.all(d == 1250.0)
    t, d = X.treatment_schedule(500.0, 12.0, 250.0, 96.0, 1, (3,))
    assert 72.0 not in t and 84.0 not in t  # day 3 skipped
    assert 120.0 not in t and 156.0 not in t  # days 6-7 of the week off
    assert np.all(d[t >= 96.0] == 250.0) and np.all(d[t < 96.0] == 500.0)
    t, _ = X.treatment_schedule(100.0, 24.0, intermittent=2)
    assert 21 * 24.0 not in t and 20 * 24.0 in t
    t, _ = X.treatment_schedule(100.0, 24.0, intermittent=3)
    assert 4 * 24.0 not in t and 3 * 24.0 in t


@pytest.mark.parametrize("variant,patient", [("all", "B2"), ("plain", "A1"), ("transit1", "B2")])
def test_host_layer_builds_the_restated_model(tmp_path, variant, patient):
    from bcm3_amd.likelihood import Likelihood
    ll = Likelihood(_xml(tmp_path, variant, patient), PRIOR, options="backend=none")
    m = ll.expm_pk_model()
    want = F.model_fields(variant, patient, _pkdata())
    for k, v in want.items():
        if k in ("transforms", "treat_times", "treat_doses", "obs_times", "obs_conc"):
            n = {"transforms": m.d, "treat_times": m.n_treat, "treat_doses": m.n_treat, "obs_times": m.n_obs,
                 "obs_conc": m.n_obs}[k]
            ct = np.int32 if k == "transforms" else np.float64
            got = _read(getattr(m, k), n, ct)
            assert np.array_equal(got, np.asarray(v, dtype=ct)), k
        else:
            assert getattr(m, k) == v, k
    ll.close()


def _read(ptr, n, dtype):
    import ctypes
    ct = ctypes.c_int32 if dtype == np.int32 else ctypes.c_double
    return np.array((ct * n).from_address(ptr), dtype=dtype)


def test_host_layer_errors(tmp_path):
    from bcm3_amd.likelihood import Likelihood
    # unknown patient
    p = tmp_path / "l.xml"
    p.write_text(F.likelihood_xml("plain", "ZZ", PKDATA))
    with pytest.raises(RuntimeError):
        Likelihood(str(p), PRIOR, options="backend=none")
    # peripheral compartment without its rates in the prior
    prior = tmp_path / "prior.xml"
    prior.write_text(F.prior_xml().replace("peripheral_forward_rate", "pfr"))
    with pytest.raises(RuntimeError):
        Likelihood(_xml(tmp_path, "peripheral", "A1"), str(prior), options="backend=none")
    # more compartments than the device supports
    p.write_text(F.likelihood_xml("plain", "A1", PKDATA).replace("pk_model ", 'pk_model num_transit_compartments="20" '))
    with pytest.raises(RuntimeError):
        Likelihood(str(p), PRIOR, options="backend=none")


# ---------------------------------------------------------------------------------------------
# GPU

@pytest.mark.gpu
@pytest.mark.parametrize("variant,patient", CASES)
def test_gpu_matches_golden(tmp_path, variant, patient):
    from bcm3_amd.likelihood import Likelihood
    ll = Likelihood(_xml(tmp_path, variant, patient), PRIOR, device=0)
    v = GOLD[f"{variant}_{patient}_values"]
    logp, status = ll.evaluate_batch(v)
    assert np.all(status == 0)
    assert _close(logp, GOLD[f"{variant}_{patient}_logp"]), np.max(
        np.abs(logp - GOLD[f"{variant}_{patient}_logp"]) / (1 + np.abs(GOLD[f"{variant}_{patient}_logp"])))
    ll.close()


@pytest.mark.gpu
def test_gpu_c_abi_context_and_batch_invariance():
    from bcm3_amd import _hip
    m = F.model_fields("all", "B2", _pkdata())
    ctx = _hip.Context.expm_pk(m, device=0)
    v = F.draws(1024, 7)
    a = ctx.eval(v)[0]
    b = ctx.eval(v[100:140])[0]
    assert np.array_equal(a[100:140], b)
    ref, _ = X.evaluate(m, v[:64])
    assert _close(a[:64], ref)
    assert ctx.eval(v[:0])[0].shape == (0,)


@pytest.mark.gpu
def test_gpu_nonfinite_rates_give_minus_inf():
    from bcm3_amd import _hip
    m = F.model_fields("plain", "A1", _pkdata())
    ctx = _hip.Context.expm_pk(m, device=0)
    v = F.draws(4, 3)
    v[1, 1] = 400.0  # clearance 1e400 = inf -> NaN state
    v[2, 0] = np.nan
    logp, status = ctx.eval(v)[:2]
    ref, ok = X.evaluate(m, v)
    assert np.array_equal(np.isfinite(logp), np.isfinite(ref))
    assert _close(logp[[0, 3]], ref[[0, 3]])
