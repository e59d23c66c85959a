"""Parity contract for the PopPK path (calibrated -- see DESIGN.md §3).

CVODE output is not bit-stable even CPU-vs-CPU: the reference's own CVODE built with and
without FMA contraction (oracle/_ref/libbcm3ref.so vs libbcm3ref_nofma.so) differs, measured on
8192 C3 prior draws, as
    y1 max rel err per draw:  <=1e-9 for 93.0%, <=1e-6 for 99.0%, <=2e-5 for 99.65%
    llh |d|/(1+|llh|):        <=1e-8 for 99.2%, max 1.4e-5
    BDF step counts equal:    99.3%;  ok/fail status identical for 100%.
(Round 3: with the 3x3 solve of both builds run by the vendored Eigen itself, 8192 draws give 92.8 %,
98.97 %, 99.67 %; llh 99.13 %; steps 99.29 %.)
The device follows the no-FMA build's arithmetic operation for operation (round 4), so
against that build and the C restatement (bit-exact to it) the tiers are absolute: y1 >=92% at 1e-9,
>=98.5% at 1e-6, >=99.5% at 2e-5; llh >=99% at 1e-8 (measured round 4: 99.2 % / 99.95 % / 100 %, llh
99.93 % on 4,096 draws), plus a floor on the fraction of bit-identical llh (bitexact_min()).
Against the FMA build, which no other build reproduces, a test may pass the reference's own
spread measured on the same draws (reference_self_spread): a tier the reference's two builds
themselves miss on that sample is held to their fraction minus two binomial standard deviations.
Every assert_parity call appends its measured fractions to the JSON-lines file named by
$BCM3_PARITY_LOG (committed under profiles/ per round).
"""
from __future__ import annotations

import json
import os

import numpy as np

Y1_TIERS = ((1e-9, 0.92), (1e-6, 0.985), (2e-5, 0.995))  # (tolerance, min fraction of draws)
LLH_T1, LLH_T1_FRAC = 1e-8, 0.99
LLH_T2 = 1e-3  # every draw whose ok/fail status agrees
# The llh tier is a rate near 99 %: on fewer than LLH_FULL_N draws its sampling noise (sigma = 0.44 %
# at 512 draws) exceeds the margin, so smaller samples are held to the binomial bound of a 99 %
# process (expected misses + 2 sigma); the >= 99 % rate itself is asserted on the large samples
# (8,192 golden draws, 4,096 prior draws, 12,288 P64 trajectories, 2,048 C5 chains). The
# reference's own two builds differ on 4 of the 512 c3_golden draws (99.2 %).
LLH_FULL_N = 2048


def llh_min_fraction(n: int) -> float:
    if n >= LLH_FULL_N:
        return LLH_T1_FRAC
    p = 1.0 - LLH_T1_FRAC
    allowed = int(np.floor(n * p + 2.0 * np.sqrt(n * p * (1.0 - p))))
    return 1.0 - allowed / max(1, n)
STEPS_FRACTION = 0.98
# The device computes the reference's operations in the reference's order with glibc's own libm
# results (pow and exp from the loaded libm's tables): against the reference built
# without FMA contraction it is bit-identical on 100 % of C3 draws (profiles/r04h_bitexact_probe.txt,
# r04p_parity.jsonl: 512, 4,096 and 8,192 draws). C3 samples must stay at 100 % when the device runs
# on the loaded libm's tables (bcm3hip_libm_pow_tables() == 1); with computed tables (~1 ulp from
# glibc's pow / exp) the floor is 99 % (88 % was measured with correctly rounded pow / exp in place
# of glibc's, r04b).
BITEXACT_MIN_FALLBACK = 0.99


def bitexact_min() -> float:
    from bcm3_amd import _hip
    return 1.0 if _hip.lib().bcm3hip_libm_pow_tables() == 1 else BITEXACT_MIN_FALLBACK


def bitexact_fraction(a, b) -> float:
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return float(np.mean((a == b) | (np.isnan(a) & np.isnan(b))))


def y1_rel_err(a: np.ndarray, b: np.ndarray, floor: float) -> np.ndarray:
    """max_t |a-b| / max(|b|, floor) per trajectory for the observed compartment; a,b [..., T].
    NaN positions must agree (else inf)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    nan_a, nan_b = np.isnan(a), np.isnan(b)
    mism = nan_a != nan_b
    d = np.abs(np.where(nan_a | nan_b, 0.0, a - b)) / np.maximum(np.abs(np.where(nan_b, 0.0, b)), floor)
    d = np.where(mism, np.inf, d)
    return d.max(axis=-1)


def llh_err(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    same = (a == b) | (np.isnan(a) & np.isnan(b))
    with np.errstate(invalid="ignore"):
        d = np.abs(a - b) / (1.0 + np.abs(b))
    d = np.where(same, 0.0, d)
    return np.where(np.isnan(d), np.inf, d)


def summarize(y1_err, llh_e, steps_a, steps_b) -> dict:
    out = {f"y1_le_{t:g}": float(np.mean(y1_err <= t)) for t, _ in Y1_TIERS}
    out.update(llh_t1=float(np.mean(llh_e <= LLH_T1)), llh_max=float(np.max(llh_e)) if llh_e.size else 0.0,
               steps_equal=float(np.mean(np.asarray(steps_a) == np.asarray(steps_b))))
    return out


def log_summary(s: dict, **extra):
    """Append one JSON line {test, fractions...} to $BCM3_PARITY_LOG (no-op when unset)."""
    path = os.environ.get("BCM3_PARITY_LOG")
    if not path:
        return
    rec = {"test": os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0], **s, **extra}
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "a") as f:
        f.write(json.dumps(rec) + "\n")


def reference_self_spread(prob, values) -> dict | None:
    """The reference's own FMA / no-FMA spread on the SAME draws: the vendored CVODE (and the
    vendored Eigen's 3x3 solve) built with and without FMA contraction (oracle/_ref), compared per
    patient as the GPU is. None when oracle/_ref is not built."""
    import oracle as O
    if not O.have_ref():
        return None
    a = O.Oracle("ref").popk_eval(prob, values, nthreads=8)
    b = O.Oracle("ref_nofma").popk_eval(prob, values, nthreads=8)
    T = prob.T
    y1 = y1_rel_err(a["traj"][:, :, 1, :].reshape(-1, T), b["traj"][:, :, 1, :].reshape(-1, T), prob.atol)
    pa, pb = a["patient_llh"].reshape(-1), b["patient_llh"].reshape(-1)
    ok = ~np.isneginf(pa) & ~np.isneginf(pb)
    out = {f"y1_le_{t:g}": float(np.mean(y1[ok] <= t)) for t, _ in Y1_TIERS}
    out["llh_t1"] = float(np.mean(llh_err(pa, pb) <= LLH_T1))
    out["n"] = int(pa.size)
    return out


def _bar(frac: float, ref_frac: float | None, n: int) -> float:
    """The tier's fraction, or -- when the reference's own two builds fall short of it on these
    draws -- their fraction minus two binomial standard deviations (the GPU must sit inside the
    reference's own envelope measured on the same sample)."""
    if ref_frac is None or ref_frac >= frac:
        return frac
    sd = np.sqrt(max(ref_frac * (1.0 - ref_frac), 1e-6) / max(n, 1))
    return min(frac, ref_frac - 2.0 * sd)


def assert_parity(y1_err, llh_e, steps_a, steps_b, ok_a, ok_b, near_cap=None, ref_self=None, bitexact=None):
    """Assert the GPU-vs-oracle differences are inside the contract's tiers. ref_self
    (reference_self_spread on the same draws) lowers a tier's bar only where the reference's own
    FMA / no-FMA builds miss that tier on this sample (used only against the FMA build, which the
    device does not follow). bitexact (fraction of identical log-likelihoods) is asserted >=
    bitexact_min() when given."""
    s = summarize(y1_err, llh_e, steps_a, steps_b)
    if bitexact is not None:
        s["bitexact"] = bitexact
    log_summary(s, n=int(np.asarray(llh_e).size), **({"ref_self": ref_self} if ref_self else {}))
    if bitexact is not None:
        assert bitexact >= bitexact_min(), s
    rs = ref_self or {}
    ok_a, ok_b = np.asarray(ok_a), np.asarray(ok_b)
    differ = ok_a != ok_b
    if near_cap is not None:
        differ &= ~np.asarray(near_cap)
    assert not differ.any(), ("ok/fail status differs", np.nonzero(differ)[0][:20], s)
    both_ok = (ok_a == 1) & (ok_b == 1)
    nb = int(np.sum(both_ok))
    for t, frac in Y1_TIERS:
        bar = _bar(frac, rs.get(f"y1_le_{t:g}"), nb)
        assert np.mean(y1_err[both_ok] <= t) >= bar, (t, bar, s, rs)
    n = int(np.asarray(llh_e).size)
    bar = _bar(llh_min_fraction(n), rs.get("llh_t1"), n)
    assert np.mean(llh_e <= LLH_T1) >= bar, (bar, s, rs)
    assert np.all(llh_e[both_ok] <= LLH_T2), s
    assert s["steps_equal"] >= STEPS_FRACTION, s
    return s
