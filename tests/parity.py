"""Two-tier parity metrics of SURVEY.md §8(c) (shared by the CPU and GPU tests)."""
from __future__ import annotations

import numpy as np

# Tier 1 / Tier 2 tolerances
TRAJ_T1, TRAJ_T2 = 1e-9, 2e-5
LLH_T1, LLH_T2 = 1e-8, 1e-3
T1_FRACTION = 0.99
STEPS_FRACTION = 0.98


def traj_rel_err(a: np.ndarray, b: np.ndarray, floor: float) -> np.ndarray:
    """max over (state, time) of |a-b| / max(|b|, floor) per trajectory; a,b [..., N, T].
    NaN positions must agree (both NaN) else the error is inf."""
    a = np.asarray(a)
    b = np.asarray(b)
    nan_a, nan_b = np.isnan(a), np.isnan(b)
    mism = nan_a != nan_b
    d = np.abs(np.where(nan_a | nan_b, 0.0, a - b)) / np.maximum(np.abs(np.where(nan_b, 0.0, b)), floor)
    d = np.where(mism, np.inf, d)
    return d.reshape(*d.shape[:-2], -1).max(axis=-1)


def llh_err(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    same_inf = (a == b)
    d = np.abs(a - b) / (1.0 + np.abs(b))
    d = np.where(same_inf, 0.0, d)
    return np.where(np.isnan(d), np.inf, d)


def summarize(traj_err: np.ndarray, llh_e: np.ndarray, steps_a: np.ndarray, steps_b: np.ndarray) -> dict:
    return dict(
        traj_t1_frac=float(np.mean(traj_err <= TRAJ_T1)),
        traj_max=float(np.max(traj_err)) if traj_err.size else 0.0,
        llh_t1_frac=float(np.mean(llh_e <= LLH_T1)),
        llh_max=float(np.max(llh_e)) if llh_e.size else 0.0,
        steps_equal_frac=float(np.mean(steps_a == steps_b)),
    )


def assert_two_tier(traj_err, llh_e, steps_a, steps_b, ok_a=None, ok_b=None, near_cap=None):
    s = summarize(traj_err, llh_e, steps_a, steps_b)
    assert s["traj_t1_frac"] >= T1_FRACTION, s
    assert s["llh_t1_frac"] >= T1_FRACTION, s
    assert s["steps_equal_frac"] >= STEPS_FRACTION, s
    if ok_a is not None:
        differ = np.asarray(ok_a) != np.asarray(ok_b)
        if near_cap is not None:
            differ &= ~np.asarray(near_cap)
        assert not differ.any(), ("ok/fail status differs", np.nonzero(differ))
    fin = np.isfinite(traj_err)
    assert np.all(traj_err[fin] <= TRAJ_T2), s
    assert np.all(llh_e <= LLH_T2), s
    return s
