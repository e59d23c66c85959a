"""oracle.py -- TEST INFRASTRUCTURE (the parity oracle). Never imported by the product.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use
this module, and only as the checker / CPU baseline.

Wraps two C libraries through ctypes:

* ``oracle/liboracle.so``       -- plain-C restatement of CVODE 5.3.0 BDF + BCM3 PopPK glue
* ``oracle/_ref/libbcm3ref.so`` -- the same glue on the vendored CVODE 5.3.0 compiled from the
  reference sources (``oracle/Makefile``).

It also restates, in Python, the data-dependent parts of
``LikelihoodPopPKTrajectory::Initialize`` (src/likelihoods/LikelihoodPopPKTrajectory.cpp:50-252)
that turn a pkdata file + prior into the flat model description both libraries consume.
"""
from __future__ import annotations

import ctypes as C
import json
import math
import os
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_RESTATED = os.path.join(HERE, "liboracle.so")
LIB_REF = os.path.join(HERE, "_ref", "libbcm3ref.so")
LIB_REF_NOFMA = os.path.join(HERE, "_ref", "libbcm3ref_nofma.so")


def have_ref() -> bool:
    """True when both reference-CVODE builds (oracle/_ref) are present."""
    return os.path.exists(LIB_REF) and os.path.exists(LIB_REF_NOFMA)
LIB_FLOPS = os.path.join(HERE, "libflops.so")  # op-counting build of the restatement (flopcount.hpp)

ST_COUNT = 8
ST_NAMES = ["nst", "nfe", "nni", "nsetups", "nje", "netf", "ncfn", "nreinit"]

# LikelihoodPopPKTrajectory.cpp:69-83 (string -> PKModelType; note the one_biphasic quirk)
PK_TYPES = {
    "one": 0,
    "two": 1,
    "one_biphasic_uptake": 3,  # reference maps this to PKMT_TwoCompartmentBiphasicUptake
    "two_biphasic_uptake": 3,
    "one_transit": 4,
    "two_transit": 5,
}
# .cpp:99-120
NUM_PK_PARAMS = {0: 4, 1: 6, 2: 7, 3: 7, 4: 6, 5: 8}
NUM_STATES = {0: 2, 1: 3, 2: 2, 3: 3, 4: 2, 5: 3}  # .cpp:210-233 (Initialize(N))
# .cpp:377-393
MOLECULAR_WEIGHT = {
    "lapatinib": 581.06,
    "dacomitinib": 469.95,
    "afatinib": 485.94,
    "trametinib": 615.404,
    "mirdametinib": 482.19,
    "selumetinib": 457.68,
}
TF_NONE, TF_LOG, TF_LOG10, TF_LOGIT = 0, 1, 2, 3


class OrcPopPKModel(C.Structure):
    _fields_ = [
        ("pk_type", C.c_int32), ("N", C.c_int32), ("num_pk_params", C.c_int32),
        ("num_pk_pop_params", C.c_int32), ("d", C.c_int32), ("P", C.c_int32), ("T", C.c_int32),
        ("sd_ix", C.c_int32), ("n_transit_ix", C.c_int32), ("transit_time_ix", C.c_int32),
        ("biphasic_time_ix", C.c_int32), ("absorption2_ix", C.c_int32), ("max_steps", C.c_int32),
        ("param_map", C.c_int32),
        ("rtol", C.c_double), ("atol", C.c_double), ("MW", C.c_double), ("fixed_vod", C.c_double),
        ("fixed_kf", C.c_double), ("fixed_kb", C.c_double),
        ("transforms", C.POINTER(C.c_int32)), ("time", C.POINTER(C.c_double)),
        ("observed", C.POINTER(C.c_double)), ("dose", C.POINTER(C.c_double)),
        ("dosing_interval", C.POINTER(C.c_double)), ("dose_after_dose_change", C.POINTER(C.c_double)),
        ("dose_change_time", C.POINTER(C.c_double)), ("intermittent", C.POINTER(C.c_int32)),
        ("skipped_days", C.POINTER(C.c_uint8)), ("simulate_until", C.POINTER(C.c_int32)),
    ]


@dataclass
class Variable:
    name: str
    lower: float
    upper: float
    transform: int = TF_NONE
    distribution: str = "uniform"


@dataclass
class PopPKProblem:
    """Everything LikelihoodPopPKTrajectory::Initialize derives, in flat arrays."""

    pk_type: int
    N: int
    num_pk_params: int
    num_pk_pop_params: int
    d: int
    P: int
    T: int
    sd_ix: int
    n_transit_ix: int
    transit_time_ix: int
    biphasic_time_ix: int
    absorption2_ix: int
    max_steps: int
    rtol: float
    atol: float
    MW: float
    fixed_vod: float
    fixed_kf: float
    fixed_kb: float
    transforms: np.ndarray
    time: np.ndarray
    observed: np.ndarray
    dose: np.ndarray
    dosing_interval: np.ndarray
    dose_after_dose_change: np.ndarray
    dose_change_time: np.ndarray
    intermittent: np.ndarray
    skipped_days: np.ndarray
    simulate_until: np.ndarray
    variables: List[Variable] = field(default_factory=list)
    param_map: int = 0  # 0 LikelihoodPopPKTrajectory, 1 LikelihoodPharmacokineticTrajectory

    def to_c(self):
        keep = []

        def arr(a, dt):
            a = np.ascontiguousarray(a, dtype=dt)
            keep.append(a)
            return a.ctypes.data_as(C.POINTER(np.ctypeslib.as_ctypes_type(dt)))

        m = OrcPopPKModel()
        for k in ("pk_type", "N", "num_pk_params", "num_pk_pop_params", "d", "P", "T", "sd_ix",
                  "n_transit_ix", "transit_time_ix", "biphasic_time_ix", "absorption2_ix", "max_steps",
                  "param_map"):
            setattr(m, k, int(getattr(self, k)))
        for k in ("rtol", "atol", "MW", "fixed_vod", "fixed_kf", "fixed_kb"):
            setattr(m, k, float(getattr(self, k)))
        m.transforms = arr(self.transforms, np.int32)
        m.time = arr(self.time, np.float64)
        m.observed = arr(self.observed, np.float64)
        m.dose = arr(self.dose, np.float64)
        m.dosing_interval = arr(self.dosing_interval, np.float64)
        m.dose_after_dose_change = arr(self.dose_after_dose_change, np.float64)
        m.dose_change_time = arr(self.dose_change_time, np.float64)
        m.intermittent = arr(self.intermittent, np.int32)
        m.skipped_days = arr(self.skipped_days, np.uint8)
        m.simulate_until = arr(self.simulate_until, np.int32)
        return m, keep


def _f32(x: float) -> float:
    """(double)x for a C float literal such as 1e-6f."""
    return float(np.float32(x))


def build_problem(pkdata: dict, trial: str, drug: str, pk_type_str: str, variables: List[Variable],
                  fixed_vod=math.nan, fixed_kf=math.nan, fixed_kb=math.nan, check_count=True) -> PopPKProblem:
    """Restates LikelihoodPopPKTrajectory::Initialize (.cpp:50-252) for a pkdata dict in the
    JSON sidecar layout (group -> variables, NaN as null).

    check_count=False skips the variable-count check of .cpp:127-130 (needed only to exercise the
    biphasic models, whose named parameters cannot all fit the reference's count formula)."""
    g = pkdata[trial]
    pk_type = PK_TYPES[pk_type_str]
    names = [v.name for v in variables]
    time = np.array(g["time"], dtype=np.float64)
    T = len(time)
    patients = g["patients"]
    P = len(patients)

    def f64(x):
        return np.array([math.nan if v is None else v for v in x], dtype=np.float64)

    obs = np.array([[math.nan if v is None else v for v in row] for row in g[drug + "_plasma_concentration"]],
                   dtype=np.float64).reshape(P, T)
    dose = f64(g[drug + "_dose"])
    dadc = f64(g[drug + "_dose_after_dose_change"])
    dct = f64(g[drug + "_dose_change_time"])
    di = f64(g[drug + "_dosing_interval"])
    inter = np.array(g[drug + "_intermittent"], dtype=np.int32)
    ti = np.array(g["treatment_interruptions"], dtype=np.uint8).reshape(P, 29)
    npk = NUM_PK_PARAMS[pk_type]
    npop = 2
    nfixed = sum(0 if math.isnan(x) else 1 for x in (fixed_vod, fixed_kf, fixed_kb))
    if check_count and len(variables) != npk - nfixed + npop * (P + 1) + 2:
        raise ValueError("Incorrect number of variables in prior")
    sim_until = np.zeros(P, dtype=np.int32)
    min_dose = float(np.finfo(np.float64).max)
    for j in range(P):
        if ti[j, 1]:
            for i in range(T):
                if time[i] >= 24.0:
                    sim_until[j] = i
                    break
        else:
            sim_until[j] = T
        for i in range(T):
            if not math.isnan(obs[j, i]):
                if time[i] > 15 * 24:
                    sim_until[j] = 0
                break
        if dose[j] < min_dose:
            min_dose = dose[j]
        if not math.isnan(dadc[j]) and dadc[j] < min_dose:
            min_dose = dadc[j]

    def idx(name):
        return names.index(name) if name in names else -1

    return PopPKProblem(
        pk_type=pk_type, N=NUM_STATES[pk_type], num_pk_params=npk, num_pk_pop_params=npop,
        d=len(variables), P=P, T=T, sd_ix=idx("standard_deviation"), n_transit_ix=idx("n_transit"),
        transit_time_ix=idx("mean_transit_time"), biphasic_time_ix=idx("biphasic_uptake_time"),
        absorption2_ix=idx("mean_absorption2"), max_steps=2000,
        # SetTolerance(1e-6f, minimum_dose * 1e-6f) (.cpp:238): float * double -> double
        rtol=_f32(1e-6), atol=min_dose * _f32(1e-6), MW=MOLECULAR_WEIGHT[drug],
        fixed_vod=fixed_vod, fixed_kf=fixed_kf, fixed_kb=fixed_kb,
        transforms=np.array([v.transform for v in variables], dtype=np.int32), time=time,
        observed=obs, dose=dose, dosing_interval=di, dose_after_dose_change=dadc, dose_change_time=dct,
        intermittent=inter, skipped_days=ti, simulate_until=sim_until, variables=list(variables))


def build_single_problem(pkdata: dict, trial: str, drug: str, pk_type_str: str, variables: List[Variable],
                         patient: str, fixed_vod=math.nan, fixed_kf=math.nan, fixed_kb=math.nan) -> PopPKProblem:
    """Restates LikelihoodPharmacokineticTrajectory::Initialize (src/likelihoods/
    LikelihoodPharmacokineticTrajectory.cpp:85-213) for one patient of a pkdata dict: no
    variable-count check (compiled out, .cpp:118-150), every time point simulated, tolerances
    SetTolerance(1e-6f, dose * 1e-6f) with the patient's dose (.cpp:205), biphasic switch time
    and second absorption rate at variables 6 and 7 (.cpp:252-253)."""
    g = pkdata[trial]
    pk_type = PK_TYPES[pk_type_str]
    names = [v.name for v in variables]
    patients = [str(p) for p in g["patients"]]
    if patient not in patients:
        raise ValueError(f'Cannot find patient "{patient}" in data file')
    j = patients.index(patient)
    time = np.array(g["time"], dtype=np.float64)
    T = len(time)

    def f(x):
        return math.nan if x is None else float(x)

    obs = np.array([f(v) for v in g[drug + "_plasma_concentration"][j]], dtype=np.float64).reshape(1, T)
    dose = np.array([f(g[drug + "_dose"][j])])
    biphasic = pk_type in (2, 3)

    def idx(name):
        return names.index(name) if name in names else -1

    return PopPKProblem(
        pk_type=pk_type, N=NUM_STATES[pk_type], num_pk_params=0, num_pk_pop_params=0, d=len(variables), P=1,
        T=T, sd_ix=idx("standard_deviation"), n_transit_ix=idx("n_transit"),
        transit_time_ix=idx("mean_transit_time"), biphasic_time_ix=6 if biphasic else -1,
        absorption2_ix=7 if biphasic else -1, max_steps=2000,
        rtol=_f32(1e-6), atol=float(dose[0]) * _f32(1e-6), MW=MOLECULAR_WEIGHT[drug],
        fixed_vod=fixed_vod, fixed_kf=fixed_kf, fixed_kb=fixed_kb,
        transforms=np.array([v.transform for v in variables], dtype=np.int32), time=time, observed=obs,
        dose=dose, dosing_interval=np.array([f(g[drug + "_dosing_interval"][j])]),
        dose_after_dose_change=np.array([f(g[drug + "_dose_after_dose_change"][j])]),
        dose_change_time=np.array([f(g[drug + "_dose_change_time"][j])]),
        # read as a bool (.cpp:183-185)
        intermittent=np.array([1 if g[drug + "_intermittent"][j] else 0], dtype=np.int32),
        skipped_days=np.array(g["treatment_interruptions"][j], dtype=np.uint8).reshape(1, 29),
        simulate_until=np.array([T], dtype=np.int32), variables=list(variables), param_map=1)


class Oracle:
    """ctypes front-end for one oracle library (restated or reference-built)."""

    def __init__(self, which: str = "restated"):
        path = {"restated": LIB_RESTATED, "ref": LIB_REF, "ref_nofma": LIB_REF_NOFMA, "flops": LIB_FLOPS}[which]
        if not os.path.exists(path):
            raise FileNotFoundError(f"oracle library {path} not built (run make -C oracle)")
        self.which = which
        self.lib = C.CDLL(path)
        L = self.lib
        L.orc_popk_eval.argtypes = [C.POINTER(OrcPopPKModel), C.c_int64, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_int32]
        L.orc_popk_eval.restype = C.c_int
        L.orc_banana_eval.argtypes = [C.c_int64, C.c_int32, C.c_double, C.c_double, C.c_void_p, C.c_void_p]
        L.orc_circular_eval.argtypes = [C.c_int64, C.c_int32, C.c_double, C.c_double, C.c_double, C.c_void_p,
                                        C.c_void_p]
        for fn in ("orc_quantile_normal", "orc_log_pdf_tnu4"):
            getattr(L, fn).argtypes = [C.c_double, C.c_double, C.c_double]
            getattr(L, fn).restype = C.c_double
        L.orc_transform.argtypes = [C.c_int32, C.c_double]
        L.orc_transform.restype = C.c_double
        if which == "flops":
            L.orc_flops_take.restype = C.c_longlong

    def popk_flops(self, prob: PopPKProblem, values: np.ndarray) -> np.ndarray:
        """FP64 operations of each evaluation (flops build only; SURVEY.md §8(d) counting rule:
        +, -, *, /, fma, exp, log, pow, sqrt 1 each), one evaluation per call on this thread."""
        if self.which != "flops":
            raise ValueError("popk_flops needs Oracle('flops')")
        values = np.ascontiguousarray(values, dtype=np.float64).reshape(-1, prob.d)
        out = np.empty(values.shape[0], dtype=np.int64)
        self.lib.orc_flops_take()
        for i in range(values.shape[0]):
            self.popk_eval(prob, values[i:i + 1], nthreads=1, full_patients=False, want_traj=False)
            out[i] = self.lib.orc_flops_take()
        return out

    def popk_eval(self, prob: PopPKProblem, values: np.ndarray, nthreads: int = 1, full_patients: bool = True,
                  want_traj: bool = True):
        values = np.ascontiguousarray(values, dtype=np.float64).reshape(-1, prob.d)
        n = values.shape[0]
        m, keep = prob.to_c()
        logp = np.empty(n)
        pllh = np.empty(n * prob.P)
        traj = np.empty(n * prob.P * prob.N * prob.T) if want_traj else None
        stats = np.empty(n * prob.P * ST_COUNT, dtype=np.int64)
        ok = np.empty(n * prob.P, dtype=np.int32)
        r = self.lib.orc_popk_eval(C.byref(m), n, values.ctypes.data, logp.ctypes.data, pllh.ctypes.data,
                                   traj.ctypes.data if traj is not None else None, stats.ctypes.data,
                                   ok.ctypes.data, int(full_patients), int(nthreads))
        if r != 0:
            raise RuntimeError("orc_popk_eval failed")
        del keep
        out = dict(logp=logp, patient_llh=pllh.reshape(n, prob.P), stats=stats.reshape(n, prob.P, ST_COUNT),
                   ok=ok.reshape(n, prob.P))
        if traj is not None:
            out["traj"] = traj.reshape(n, prob.P, prob.N, prob.T)
        return out

    def banana(self, values, d, sd1, sd2):
        values = np.ascontiguousarray(values, dtype=np.float64).reshape(-1, d)
        out = np.empty(values.shape[0])
        self.lib.orc_banana_eval(values.shape[0], d, sd1, sd2, values.ctypes.data, out.ctypes.data)
        return out

    def circular(self, values, d, radius=2.0, offset=3.5, width=0.1):
        values = np.ascontiguousarray(values, dtype=np.float64).reshape(-1, d)
        out = np.empty(values.shape[0])
        self.lib.orc_circular_eval(values.shape[0], d, radius, offset, width, values.ctypes.data, out.ctypes.data)
        return out


def load_pkdata(path: str) -> dict:
    with open(path) as f:
        return json.load(f)
