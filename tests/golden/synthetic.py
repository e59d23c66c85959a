"""Synthetic PopPK workloads of SURVEY.md §8(d) (C3 and its P=64 variant).

The reference ships no PopPK data, so the C3 inputs are synthetic: trial ``SYN``, drug
lapatinib, model ``two`` (3 states), dose 1250 every 24 h, 16 output times to 336 h. This
module only *describes* the workload (times, prior, draws); observations are produced by
``make_fixtures.py`` with the reference-built oracle and committed as a pkdata JSON file.
"""
from __future__ import annotations

import math

import numpy as np

TRIAL = "SYN"
DRUG = "lapatinib"
PK_TYPE = "two"
TIMES = [0, 1, 2, 3, 4, 6, 8, 12, 24, 48, 72, 120, 168, 216, 288, 336]
DOSE = 1250.0
INTERVAL = 24.0

# (name, lower, upper, logspace) in prior.xml order; index meaning per
# LikelihoodPopPKTrajectory.cpp:267-310 for model type "two" (num_pk_params = 6).
POP_VARS = [
    ("pk_absorption_mean", -1.5, 0.5, False),     # 0  mu log10 ka
    ("k_excretion", -4.0, -1.0, True),            # 1  ke
    ("pk_clearance_mean", 0.0, 2.0, False),       # 2  mu log10 CL
    ("volume_of_distribution", 1.5, 3.0, True),   # 3  V
    ("k_periphery_fwd", -3.0, -0.5, True),        # 4  kf
    ("k_periphery_bwd", -3.0, -0.5, True),        # 5  kb
    ("pk_absorption_sd", 0.05, 0.5, False),       # 6  sigma_a
    ("pk_clearance_sd", 0.05, 0.5, False),        # 7  sigma_e
]
SD_VARS = [
    ("standard_deviation", -1.0, 1.5, True),
    ("standard_deviation_proportional", -2.0, -0.5, True),
]


def variables(P: int):
    """List of (name, lower, upper, logspace) for P patients (d = 8 + 2(P+1)... = 12 at P=1)."""
    v = list(POP_VARS)
    for j in range(P):
        v.append((f"patient{j}_absorption", 0.0, 1.0, False))
        v.append((f"patient{j}_clearance", 0.0, 1.0, False))
    v += SD_VARS
    return v


def prior_xml(P: int) -> str:
    lines = ['<?xml version="1.0" encoding="utf-8"?>', "<variableset>"]
    for name, lo, hi, logspace in variables(P):
        ls = ' logspace="true"' if logspace else ""
        lines.append(f'  <variable name="{name}" distribution="uniform" lower="{lo!r}" upper="{hi!r}"{ls}/>')
    lines.append("</variableset>")
    return "\n".join(lines) + "\n"


def likelihood_xml(pkdata_file: str) -> str:
    return (f'<bcm_likelihood type="pop_pk_trajectory">\n'
            f'  <pk_model drug="{DRUG}" type="{PK_TYPE}" trial="{TRIAL}" pkdata_file="{pkdata_file}"/>\n'
            f'</bcm_likelihood>\n')


def prior_draws(P: int, n: int, seed: int) -> np.ndarray:
    """n independent draws from the uniform prior (sampler space, untransformed)."""
    rng = np.random.default_rng(seed)
    v = variables(P)
    lo = np.array([x[1] for x in v])
    hi = np.array([x[2] for x in v])
    return lo + (hi - lo) * rng.random((n, len(v)))


def pkdata_skeleton(P: int) -> dict:
    nan = None
    return {TRIAL: {
        "time": [float(t) for t in TIMES],
        "patients": [f"P{j:03d}" for j in range(P)],
        f"{DRUG}_plasma_concentration": [[nan] * len(TIMES) for _ in range(P)],
        f"{DRUG}_dose": [DOSE] * P,
        f"{DRUG}_dose_after_dose_change": [nan] * P,
        f"{DRUG}_dose_change_time": [nan] * P,
        f"{DRUG}_dosing_interval": [INTERVAL] * P,
        f"{DRUG}_intermittent": [0] * P,
        "treatment_interruptions": [[0] * 29 for _ in range(P)],
    }}


TRUE_POP = [-0.5, math.log10(0.01), 1.2, 2.3, math.log10(0.05), math.log10(0.02), 0.2, 0.2]
TRUE_SD = [0.5, -1.0]
