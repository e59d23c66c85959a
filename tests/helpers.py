"""Test-side helpers: build GPU contexts and oracle problems from the same inputs."""
from __future__ import annotations

import math
import os

import numpy as np

import oracle as O
import synthetic as S

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def variables(P: int):
    return [O.Variable(n, lo, hi, O.TF_LOG10 if ls else O.TF_NONE) for n, lo, hi, ls in S.variables(P)]


def c3_problem(P: int = 1) -> O.PopPKProblem:
    name = "c3" if P == 1 else "p64"
    pk = O.load_pkdata(os.path.join(GOLDEN, f"{name}_pkdata.json"))
    return O.build_problem(pk, S.TRIAL, S.DRUG, S.PK_TYPE, variables(P))


def problem_fields(prob: O.PopPKProblem) -> dict:
    """bcm3hip_popk_model fields from the oracle-side problem description (same inputs)."""
    keys = ("pk_type", "N", "num_pk_params", "num_pk_pop_params", "d", "P", "T", "sd_ix", "n_transit_ix",
            "transit_time_ix", "biphasic_time_ix", "absorption2_ix", "max_steps", "rtol", "atol", "MW",
            "fixed_vod", "fixed_kf", "fixed_kb", "transforms", "time", "observed", "dose", "dosing_interval",
            "dose_after_dose_change", "dose_change_time", "intermittent", "skipped_days", "simulate_until",
            "param_map")
    return {k: getattr(prob, k) for k in keys}


def gpu_context(prob: O.PopPKProblem, lanes_per_wave: int = 64, uni_solver: int = 0):
    """lanes_per_wave 1: one trajectory per wavefront, uni_solver 0 = lane-vector state
    (bdf_vec.h), 1 = scalar state (bdf_uni.h); > 1: lane solver (bdf_lane.h)."""
    from bcm3_amd import _hip
    ctx = _hip.Context.popk(problem_fields(prob))
    ctx.set_option(_hip.OPT_LANES_PER_WAVE, lanes_per_wave)
    if uni_solver:  # (0 is the library default)
        ctx.set_option(_hip.OPT_UNI_SOLVER, uni_solver)
    return ctx


def make_problem(pk_type_str: str, P: int = 2, T_days: int = 7, intermittent=0, skipped=(), dose_change=None,
                 seed: int = 5, interval: float = 24.0):
    """Small synthetic problems covering every PK model variant and dosing rule."""
    rng = np.random.default_rng(seed)
    times = [0.0, 1.0, 2.0, 4.0, 8.0] + [24.0 * d for d in range(1, T_days + 1)]
    T = len(times)
    pk_type = O.PK_TYPES[pk_type_str]
    npk = O.NUM_PK_PARAMS[pk_type]
    names = []
    # population parameters in the reference's index order (LikelihoodPopPKTrajectory.cpp:267-272)
    base = [("pk_absorption_mean", -1.0, 0.0, False), ("k_excretion", -3.0, -1.5, True),
            ("pk_clearance_mean", 0.5, 1.5, False), ("volume_of_distribution", 1.5, 2.5, True)]
    extra = []
    tail = []
    if pk_type in (0, 2, 4):
        extra += [("unused4", 0.0, 1.0, False), ("unused5", 0.0, 1.0, False)]
    if pk_type in (1, 3, 5):
        extra += [("k_periphery_fwd", -2.5, -1.0, True), ("k_periphery_bwd", -2.5, -1.0, True)]
    if pk_type in (2, 3):
        # num_pk_params = 7 leaves one positional slot; the second named biphasic parameter can
        # only be appended (see oracle.build_problem(check_count=False))
        extra += [("biphasic_uptake_time", 0.0, 1.0, True)]
        tail = [("mean_absorption2", -1.5, -0.5, True)]
    if pk_type in (4, 5):
        extra = extra[:4 - len(base) + 2] if pk_type == 4 else extra
        if pk_type == 4:
            extra = [("n_transit", 0.0, 1.0, True), ("mean_transit_time", 0.0, 0.7, True)]
        else:
            extra += [("n_transit", 0.0, 1.0, True), ("mean_transit_time", 0.0, 0.7, True)]
    pop = (base + extra)[:npk]
    while len(pop) < npk:
        pop.append((f"unused{len(pop)}", 0.0, 1.0, False))
    pop += [("pk_absorption_sd", 0.05, 0.3, False), ("pk_clearance_sd", 0.05, 0.3, False)]
    pats = []
    for j in range(P):
        pats += [(f"patient{j}_absorption", 0.05, 0.95, False), (f"patient{j}_clearance", 0.05, 0.95, False)]
    sds = [("standard_deviation", -1.0, 1.0, True), ("standard_deviation_proportional", -2.0, -0.7, True)]
    allv = pop + pats + sds + tail
    variables = [O.Variable(n, lo, hi, O.TF_LOG10 if ls else O.TF_NONE) for n, lo, hi, ls in allv]
    nan = None
    obs = [[nan] + [float(x) for x in rng.uniform(50, 2000, T - 1)] for _ in range(P)]
    ti = [[0] * 29 for _ in range(P)]
    for j in range(P):
        for d in skipped:
            ti[j][d] = 1
    pk = {"TRIAL": {
        "time": times, "patients": [f"p{j}" for j in range(P)],
        "lapatinib_plasma_concentration": obs,
        "lapatinib_dose": [1000.0 + 250 * j for j in range(P)],
        "lapatinib_dose_after_dose_change": [nan if dose_change is None else dose_change[0]] * P,
        "lapatinib_dose_change_time": [nan if dose_change is None else dose_change[1]] * P,
        "lapatinib_dosing_interval": [interval] * P,
        "lapatinib_intermittent": [intermittent] * P,
        "treatment_interruptions": ti,
    }}
    prob = O.build_problem(pk, "TRIAL", "lapatinib", pk_type_str, variables, check_count=not tail)
    lo = np.array([v.lower for v in variables])
    hi = np.array([v.upper for v in variables])
    return prob, lo, hi


def draws(lo, hi, n, seed):
    rng = np.random.default_rng(seed)
    return lo + (hi - lo) * rng.random((n, len(lo)))


def make_single_problem(pk_type_str: str, T_days: int = 7, intermittent=0, skipped=(), dose_change=None, seed: int = 5,
                        interval: float = 24.0, patient: str = "p1"):
    """One patient of make_problem's data for the single-patient likelihood (pharmacokinetic_trajectory):
    variables by the reference's fixed indices (LikelihoodPharmacokineticTrajectory.cpp:221-253)."""
    rng = np.random.default_rng(seed)
    times = [0.0, 1.0, 2.0, 4.0, 8.0] + [24.0 * d for d in range(1, T_days + 1)]
    T = len(times)
    pk_type = O.PK_TYPES[pk_type_str]
    v = [("k_absorption", -1.5, 0.0, True), ("k_excretion", -3.0, -1.5, True), ("clearance", 0.5, 1.5, True),
         ("volume_of_distribution", 1.5, 2.5, True)]
    if pk_type in (1, 3, 5):
        v += [("k_periphery_fwd", -2.5, -1.0, True), ("k_periphery_bwd", -2.5, -1.0, True)]
    else:
        v += [("unused4", 0.0, 1.0, False), ("unused5", 0.0, 1.0, False)]
    if pk_type in (2, 3):
        v += [("biphasic_uptake_time", 0.0, 1.2, True), ("mean_absorption2", -1.5, -0.5, True)]
    if pk_type in (4, 5):
        v += [("n_transit", 0.0, 1.0, True), ("mean_transit_time", 0.0, 0.7, True)]
    v += [("standard_deviation", -1.0, 1.0, True), ("standard_deviation_proportional", -2.0, -0.7, True)]
    variables = [O.Variable(n, lo, hi, O.TF_LOG10 if ls else O.TF_NONE) for n, lo, hi, ls in v]
    nan = None
    obs = [[nan] + [float(x) for x in rng.uniform(50, 2000, T - 1)] for _ in range(2)]
    ti = [[1 if d in skipped else 0 for d in range(29)] for _ in range(2)]
    pk = {"TRIAL": {
        "time": times, "patients": ["p0", "p1"],
        "lapatinib_plasma_concentration": obs,
        "lapatinib_dose": [1000.0, 1250.0],
        "lapatinib_dose_after_dose_change": [nan if dose_change is None else dose_change[0]] * 2,
        "lapatinib_dose_change_time": [nan if dose_change is None else dose_change[1]] * 2,
        "lapatinib_dosing_interval": [interval] * 2,
        "lapatinib_intermittent": [intermittent] * 2,
        "treatment_interruptions": ti,
    }}
    prob = O.build_single_problem(pk, "TRIAL", "lapatinib", pk_type_str, variables, patient)
    lo = np.array([x.lower for x in variables])
    hi = np.array([x.upper for x in variables])
    return prob, lo, hi, pk
