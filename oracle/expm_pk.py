"""CPU oracle for the pharmaco_single likelihood (TEST INFRASTRUCTURE ONLY: imported by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the product path).

Restates, in plain numpy/Python:
  * Patient::Load's treatment schedule and observation filter (src/pharmaco/PharmacoPatient.cpp:48-113);
  * PharmacoLikelihoodSingle::EvaluateLogProbability's parameter map and observation model
    (src/pharmaco/PharmacoLikelihoodSingle.cpp:149-218);
  * PharmacokineticModel::ConstructMatrix / Solve (src/pharmaco/PharmacokineticModel.cpp:111-247);
  * Eigen 3.4-rc1 MatrixBase::exp for double (third-party, vendored at
    dependencies/eigen-3.4-rc1, unsupported/Eigen/src/MatrixFunctions/MatrixExponential.h:65-366):
    Pade 3/5/7/9 by the 1-norm thresholds, Pade 13 on M / 2^s beyond, (V - U)^-1 (V + U) by
    PartialPivLU (unblocked_lu, Eigen/src/LU/PartialPivLU.h) and s squarings.

Pinning: oracle/expm_ref.cpp computes the same solve with the vendored Eigen itself (compiled from
/root/reference/dependencies/eigen-3.4-rc1 into oracle/_ref/libexpmref.so by oracle/Makefile);
tests/test_pharmaco_single.py checks this restatement against it (relative 1e-12) when it is
built, and tests/golden/pharmaco_single_golden.npz holds its outputs for the GPU box.
"""
import ctypes as C
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_EXPM_REF = os.path.join(HERE, "_ref", "libexpmref.so")

MW = {"lapatinib": 581.06, "dacomitinib": 469.95, "afatinib": 485.94, "trametinib": 615.404,
      "mirdametinib": 482.19, "selumetinib": 457.68}

# Pade coefficients b[0..m] (MatrixExponential.h:69-149)
PADE = {
    3: [120.0, 60.0, 12.0, 1.0],
    5: [30240.0, 15120.0, 3360.0, 420.0, 30.0, 1.0],
    7: [17297280.0, 8648640.0, 1995840.0, 277200.0, 25200.0, 1512.0, 56.0, 1.0],
    9: [17643225600.0, 8821612800.0, 2075673600.0, 302702400.0, 30270240.0, 2162160.0, 110880.0, 3960.0,
        90.0, 1.0],
    13: [64764752532480000.0, 32382376266240000.0, 7771770303897600.0, 1187353796428800.0, 129060195264000.0,
         10559470521600.0, 670442572800.0, 33522128640.0, 1323241920.0, 40840800.0, 960960.0, 16380.0, 182.0,
         1.0],
}


def _mm(X, Y):
    n = X.shape[0]
    C_ = np.empty_like(X)
    for i in range(n):
        for j in range(n):
            acc = X[i, 0] * Y[0, j]
            for k in range(1, n):
                acc = acc + X[i, k] * Y[k, j]
            C_[i, j] = acc
    return C_


def _uv(M):
    """matrix_exp_computeUV<MatrixType, double>::run (MatrixExponential.h:235-261)"""
    n = M.shape[0]
    I = np.eye(n)
    l1 = float(np.max(np.sum(np.abs(M), axis=0))) if n else 0.0
    s = 0
    if l1 < 1.495585217958292e-002:
        b = PADE[3]
        A2 = _mm(M, M)
        U = _mm(M, b[3] * A2 + b[1] * I)
        V = b[2] * A2 + b[0] * I
    elif l1 < 2.539398330063230e-001:
        b = PADE[5]
        A2 = _mm(M, M)
        A4 = _mm(A2, A2)
        U = _mm(M, b[5] * A4 + b[3] * A2 + b[1] * I)
        V = b[4] * A4 + b[2] * A2 + b[0] * I
    elif l1 < 9.504178996162932e-001:
        b = PADE[7]
        A2 = _mm(M, M)
        A4 = _mm(A2, A2)
        A6 = _mm(A4, A2)
        U = _mm(M, b[7] * A6 + b[5] * A4 + b[3] * A2 + b[1] * I)
        V = b[6] * A6 + b[4] * A4 + b[2] * A2 + b[0] * I
    elif l1 < 2.097847961257068e+000:
        b = PADE[9]
        A2 = _mm(M, M)
        A4 = _mm(A2, A2)
        A6 = _mm(A4, A2)
        A8 = _mm(A6, A2)
        U = _mm(M, b[9] * A8 + b[7] * A6 + b[5] * A4 + b[3] * A2 + b[1] * I)
        V = b[8] * A8 + b[6] * A6 + b[4] * A4 + b[2] * A2 + b[0] * I
    else:
        b = PADE[13]
        _, e = math.frexp(l1 / 5.371920351148152)
        s = max(e, 0)
        A = np.ldexp(M, -s)
        A2 = _mm(A, A)
        A4 = _mm(A2, A2)
        A6 = _mm(A4, A2)
        V = b[13] * A6 + b[11] * A4 + b[9] * A2
        T = _mm(A6, V)
        T = T + (b[7] * A6 + b[5] * A4 + b[3] * A2 + b[1] * I)
        U = _mm(A, T)
        T = b[12] * A6 + b[10] * A4 + b[8] * A2
        V = _mm(A6, T)
        V = V + (b[6] * A6 + b[4] * A4 + b[2] * A2 + b[0] * I)
    return U, V, s


def _lu_solve(D, B):
    """PartialPivLU(D).solve(B): unblocked_lu with row swaps of the whole row, then the permuted
    right-hand side through the unit-lower and upper triangular solves"""
    D = D.copy()
    B = B.copy()
    n = D.shape[0]
    perm = []
    for k in range(n):
        col = np.abs(D[k:, k])
        row = k + int(np.argmax(col))  # first maximum
        big = col[row - k]
        perm.append(row)
        if big != 0.0:
            if row != k:
                D[[k, row], :] = D[[row, k], :]
            piv = D[k, k]
            for i in range(k + 1, n):
                lik = D[i, k] / piv
                for j in range(k + 1, n):
                    D[i, j] = D[i, j] - lik * D[k, j]
                D[i, k] = lik
    for k, r in enumerate(perm):
        if r != k:
            B[[k, r], :] = B[[r, k], :]
    for j in range(n):
        for k in range(n):
            b = B[k, j]
            for i in range(k + 1, n):
                B[i, j] = B[i, j] - b * D[i, k]
        for k in range(n - 1, -1, -1):
            b = B[k, j] * (1.0 / D[k, k])
            B[k, j] = b
            for i in range(k):
                B[i, j] = B[i, j] - b * D[i, k]
    return B


def expm(M):
    """Eigen's MatrixBase::exp for double (matrix_exp_compute, MatrixExponential.h:354-366)"""
    U, V, s = _uv(np.asarray(M, dtype=np.float64))
    R = _lu_solve(-U + V, U + V)
    for _ in range(s):
        R = _mm(R, R)
    return R


# ---------------------------------------------------------------------------------------------
# the patient (PharmacoPatient.cpp:48-113)

def treatment_schedule(dose, dosing_interval, dose_after_dose_change=float("nan"), dose_change_time=float("nan"),
                       intermittent=0, skipped_days=()):
    times = []
    t = 0.0
    skipped = set(skipped_days)
    while t < 696.0:
        give = math.floor(t / 24.0) not in skipped
        if intermittent == 1:
            if t - 7.0 * 24.0 * math.floor(t / (7.0 * 24.0)) >= 5.0 * 24.0:
                give = False
        elif intermittent == 2:
            if t - 28.0 * 24.0 * math.floor(t / (28.0 * 24.0)) >= 21.0 * 24.0:
                give = False
        elif intermittent == 3:
            if t - 7.0 * 24.0 * math.floor(t / (7.0 * 24.0)) >= 4.0 * 24.0:
                give = False
        if give:
            times.append(t)
        t += dosing_interval
    doses = [dose_after_dose_change if (not math.isnan(dose_change_time) and x >= dose_change_time) else dose
             for x in times]
    return np.array(times), np.array(doses)


def filter_observations(time, conc):
    time = np.asarray(time, dtype=np.float64)
    conc = np.asarray(conc, dtype=np.float64)
    keep = ~np.isnan(conc)
    return time[keep], conc[keep]


# ---------------------------------------------------------------------------------------------
# model (PharmacoLikelihoodSingle.cpp:149-218, PharmacokineticModel.cpp:111-247)

def transform(tf, x):
    """VariableSet::TransformVariable (VariableSet.cpp:97-124): 0 none, 1 log, 2 log10 (fastpow10), 3 logit"""
    if tf == 1:
        return _exp(x)
    if tf == 2:
        return _exp(x * 2.3025850929940459)
    if tf == 3:
        if x > 0:
            z = _exp(-x)
            return 1.0 / (1.0 + z)
        z = _exp(x)
        return z / (1.0 + z)
    return float(x)


def _exp(x):
    try:
        return math.exp(x)
    except OverflowError:
        return math.inf


def quantile_normal(p, mu, sigma):
    """bcm3::QuantileNormal (src/utils/ProbabilityDistributions.cpp:359-363): Boost
    quantile(normal(mu, sigma), p) = mu - sigma sqrt(2) erfc_inv(2p); scipy's ndtri is the same
    function (third-party implementations agree to a few ulp)"""
    from scipy.special import ndtri
    return mu + sigma * float(ndtri(p))


def population_rates(model, v, j):
    """PharmacoLikelihoodPopulation::SetupSimulation (PharmacoLikelihoodPopulation.cpp:271-340) for
    patient j: (absorption, excretion, clearance, vod, transit_time, bioavailability)"""
    P = model["P"]
    sig = model["sigma_ix"]
    pix = model["patient_ix"]

    def pop(which, mean_ix):
        if sig[which] < 0:
            return _exp(v[mean_ix] * 2.3025850929940459)  # fastpow10 (MathFunctions.h:13)
        return _exp(quantile_normal(v[pix[which * P + j]], v[mean_ix], v[sig[which]]) * 2.3025850929940459)

    absorption = pop(0, model["absorption_ix"])
    excretion = pop(1, model["excretion_ix"]) if model["excretion_ix"] >= 0 else 0.0
    clearance = pop(2, model["clearance_ix"])
    vod = pop(3, model["vod_ix"])
    tt = 0.0
    if model["n_transit"] > 0:
        tt = transform(model["transforms"][model["mtt_ix"]], v[model["mtt_ix"]]) if sig[4] < 0 else pop(4, model["mtt_ix"])
    bi = pix[5 * P + j]
    return absorption, excretion, clearance, vod, tt, (v[bi] if bi >= 0 else 1.0)


def construct_matrix(model, v, j=0):
    """(A, conv, additive_sd, proportional_sd, bioavailability) for one parameter vector (and
    patient j of a population model); model = dict of the bcm3hip_expm_pk_model fields"""
    tv = lambda ix: transform(model["transforms"][ix], v[ix])  # noqa: E731
    add_sd = tv(model["additive_sd_ix"]) if model["additive_sd_ix"] >= 0 else 0.0
    prop_sd = tv(model["proportional_sd_ix"]) if model["proportional_sd_ix"] >= 0 else 0.0
    if model.get("param_map", 1) == 0:
        absorption, excretion, clearance, vod, transit_time, bioavailability = population_rates(model, v, j)
    else:
        absorption = tv(model["absorption_ix"])
        clearance = tv(model["clearance_ix"])
        vod = tv(model["vod_ix"])
        excretion = tv(model["excretion_ix"]) if model["excretion_ix"] >= 0 else 0.0
        transit_time = tv(model["mtt_ix"]) if model["n_transit"] > 0 else 0.0
        bioavailability = 1.0
    elimination = clearance / vod
    conv = (1e6 / model["MW"]) / vod
    nc, mi, ft = 2, -1, 0
    nt = model["n_transit"]
    if model["peripheral"]:
        nc += 1
    if model["metabolite"]:
        mi = nc
        nc += 1
    if nt > 0:
        ft = nc
        nc += nt
    A = np.zeros((nc, nc))
    A[0, 0] -= excretion
    A[0, 0] -= absorption
    if nt > 0:
        tr = (nt + 1.0) / transit_time
        A[ft, 0] += absorption
        if nt > 2:
            for i in range(nt - 1):
                A[ft + i, ft + i] -= tr
                A[ft + i + 1, ft + i] += tr
        A[ft + nt - 1, ft + nt - 1] = -tr
        A[1, ft + nt - 1] += tr
    else:
        A[1, 0] += absorption
    if model["peripheral"]:
        pf, pb = tv(model["pf_ix"]), tv(model["pb_ix"])
        A[1, 1] -= pf
        A[2, 1] += pf
        A[1, 2] += pb
        A[2, 2] -= pb
    if model["biphasic"]:
        da = tv(model["direct_ix"])
        A[0, 0] -= da
        A[1, 0] += da
    if model["metabolite"]:
        mc = tv(model["metab_conv_ix"])
        A[1, 1] -= mc
        A[mi, 1] += mc
        A[mi, mi] -= 1.0
    A[1, 1] -= elimination
    return A, conv, add_sd, prop_sd, bioavailability


def solve(A, treat_times, treat_doses, obs_times, expm_fn=expm, bioavailability=1.0):
    """PharmacokineticModel::Solve: (ok, central compartment at the observation times)"""
    n = A.shape[0]
    y = np.zeros(n)
    out = np.full(len(obs_times), np.nan)
    simulate_until = obs_times[-1]
    tti = oti = 0
    t = 0.0
    while tti < len(treat_times) and t < simulate_until:
        target = treat_times[tti + 1] if tti < len(treat_times) - 1 else simulate_until
        y[0] += treat_doses[tti] * bioavailability
        while oti < len(obs_times) and obs_times[oti] <= target:
            E = expm_fn(A * (obs_times[oti] - t))
            out[oti] = (E @ y)[1]
            oti += 1
        E = expm_fn(A * (target - t))
        y = E @ y
        if np.any(np.isnan(y)):
            return False, out
        t = target
        tti += 1
    return True, out


def log_pdf_tnu4(x, mu, sigma):
    xn = (x - mu) / sigma
    return -0.9808292530117262 - 2.5 * math.log1p(0.25 * xn * xn) - math.log(sigma)


def evaluate(model, values, backend="restated"):
    """logp[n], ok[n] for values[n][d]: PharmacoLikelihoodSingle::EvaluateLogProbability
    (PharmacoLikelihoodSingle.cpp:149-218), or with param_map 0 the patient-ordered sum of
    PharmacoLikelihoodPopulation::EvaluateLogProbability (PharmacoLikelihoodPopulation.cpp:202-248;
    ok = every patient's solve succeeded)"""
    values = np.atleast_2d(np.asarray(values, dtype=np.float64))
    tt = np.asarray(model["treat_times"], dtype=np.float64)
    td = np.asarray(model["treat_doses"], dtype=np.float64)
    ot = np.asarray(model["obs_times"], dtype=np.float64)
    oc = np.asarray(model["obs_conc"], dtype=np.float64)
    P = model.get("P", 1)
    toff = model.get("treat_offset") or [0, len(tt)]
    ooff = model.get("obs_offset") or [0, len(ot)]
    logp = np.zeros(len(values))
    ok = np.ones(len(values), dtype=bool)
    with np.errstate(all="ignore"):  # non-finite rates propagate as in the reference
        for j in range(P):
            lp = np.empty(len(values))
            good = np.empty(len(values), dtype=bool)
            _evaluate_into(model, values, j, tt[toff[j]:toff[j + 1]], td[toff[j]:toff[j + 1]],
                           ot[ooff[j]:ooff[j + 1]], oc[ooff[j]:ooff[j + 1]], backend, lp, good)
            logp += lp
            ok &= good
    return logp, ok


def _evaluate_into(model, values, j, tt, td, ot, oc, backend, logp, ok):
    for e, v in enumerate(values):
        A, conv, add_sd, prop_sd, bioavailability = construct_matrix(model, v, j)
        if backend == "ref":
            good, central = solve_ref(A, tt, td * bioavailability, ot)
        else:
            good, central = solve(A, tt, td, ot, bioavailability=bioavailability)
        ok[e] = good
        if not good:
            logp[e] = -np.inf
            continue
        lp = 0.0
        for i in range(len(ot)):
            x = conv * central[i]
            if math.isnan(x) or math.isinf(x):
                lp = -np.inf
                break
            if not math.isnan(oc[i]):
                lp += log_pdf_tnu4(x, oc[i], add_sd + prop_sd * max(x, 0.0))
        logp[e] = lp


# ---------------------------------------------------------------------------------------------
# the vendored Eigen itself (oracle/_ref/libexpmref.so, built from the reference's sources)

_ref = None


def ref_lib():
    global _ref
    if _ref is None:
        if not os.path.exists(LIB_EXPM_REF):
            raise FileNotFoundError(LIB_EXPM_REF)
        L = C.CDLL(LIB_EXPM_REF)
        vp, i = C.c_void_p, C.c_int
        L.eigen_expm.argtypes = [i, vp, vp]
        L.eigen_expm.restype = i
        L.eigen_pk_solve.argtypes = [i, vp, i, vp, vp, i, vp, vp]
        L.eigen_pk_solve.restype = i
        L.eigen_pk_solve_batch.argtypes = [i, i, i, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
        L.eigen_pk_solve_batch.restype = i
        _ref = L
    return _ref


def expm_ref(M):
    M = np.asfortranarray(M, dtype=np.float64)
    out = np.empty_like(M, order="F")
    ref_lib().eigen_expm(M.shape[0], M.ctypes.data, out.ctypes.data)
    return out


def solve_ref(A, treat_times, treat_doses, obs_times):
    A = np.asfortranarray(A, dtype=np.float64)
    tt = np.ascontiguousarray(treat_times, dtype=np.float64)
    td = np.ascontiguousarray(treat_doses, dtype=np.float64)
    ot = np.ascontiguousarray(obs_times, dtype=np.float64)
    out = np.full(len(ot), np.nan)
    ok = ref_lib().eigen_pk_solve(A.shape[0], A.ctypes.data, len(tt), tt.ctypes.data, td.ctypes.data, len(ot),
                                  ot.ctypes.data, out.ctypes.data)
    return bool(ok), out
