"""Golden fixtures for the pharmaco_single likelihood (matrix-exponential PK).

Run in the build container (needs oracle/_ref/libexpmref.so, built from the reference's vendored
Eigen by oracle/Makefile):
    python tests/golden/make_pharmaco_fixtures.py

Outputs (data only):
  pharmaco_pkdata.json       two synthetic patients in the JSON sidecar of the reference's pkdata.nc
                             schema (PharmacoPatient.cpp:27-46); observations simulated with the
                             Eigen-built solve at TRUE + t4 noise, some left NaN (unobserved)
  pharmaco_prior.xml         every variable any variant reads (log10 uniforms)
  pharmaco_single_golden.npz per variant x patient: 48 prior draws and the Eigen-built logp
The likelihood XMLs are written by likelihood_xml() below (tests write them to tmp dirs).
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import expm_pk as X  # noqa: E402

TRIAL = "PHS"
DRUG = "lapatinib"
TIME = [0.0, 1.0, 2.0, 4.0, 8.0, 12.0, 24.0, 25.0, 48.0, 72.0, 96.0, 168.0, 240.0, 336.0]
PATIENTS = {
    # id: dose, interval, dose_after_change, change_time, intermittent, skipped days
    "A1": (1250.0, 24.0, float("nan"), float("nan"), 0, ()),
    "B2": (500.0, 12.0, 250.0, 96.0, 1, (3,)),
}
# name, lower, upper (all logspace)
PRIOR = [
    ("absorption", -1.5, 0.5),
    ("clearance", 0.0, 2.0),
    ("volume_of_distribution", 1.5, 3.0),
    ("excretion", -4.0, -1.0),
    ("peripheral_forward_rate", -3.0, -0.5),
    ("peripheral_backward_rate", -3.0, -0.5),
    ("mean_transit_time", -0.5, 1.0),
    ("direct_absorption", -2.0, 0.0),
    ("metabolite_conversion_rate", -3.0, -1.0),
    ("additive_error_standard_deviation", -1.0, 1.5),
    ("proportional_error_standard_deviation", -2.0, -0.5),
]
TRUE = [-0.5, 1.2, 2.3, -2.5, -1.5, -2.0, 0.3, -1.0, -2.0, 0.5, -1.2]
# pk_model attributes of each variant (PharmacoLikelihoodSingle.cpp:42-52)
VARIANTS = {
    "plain": {},
    "peripheral": {"peripheral_compartment": "true"},
    "transit1": {"num_transit_compartments": "1"},
    "transit3": {"num_transit_compartments": "3"},
    "biphasic": {"biphasic_absorption": "true"},
    "metabolite": {"metabolite": "true"},
    "all": {"peripheral_compartment": "true", "num_transit_compartments": "4", "biphasic_absorption": "true",
            "metabolite": "true"},
}
N_DRAWS = 48


def prior_xml() -> str:
    rows = "\n".join(f'  <variable name="{n}" distribution="uniform" lower="{a}" upper="{b}" logspace="true"/>'
                     for n, a, b in PRIOR)
    return f'<?xml version="1.0" encoding="utf-8"?>\n<variableset>\n{rows}\n</variableset>\n'


def likelihood_xml(variant: str, patient: str, pkdata_file: str = "pharmaco_pkdata.json") -> str:
    attrs = " ".join(f'{k}="{v}"' for k, v in VARIANTS[variant].items())
    return (f'<bcm_likelihood type="pharmaco_single">\n  <pk_model drug="{DRUG}" trial="{TRIAL}" patient="{patient}" '
            f'pkdata_file="{pkdata_file}" {attrs}/>\n</bcm_likelihood>\n')


def model_fields(variant: str, patient: str, pkdata: dict) -> dict:
    """The bcm3hip_expm_pk_model the host layer derives (PostInitialize's indices by name)."""
    g = pkdata[TRIAL]
    j = g["patients"].index(patient)
    nan = lambda v: float("nan") if v is None else float(v)  # noqa: E731
    tt, td = X.treatment_schedule(nan(g[f"{DRUG}_dose"][j]), nan(g[f"{DRUG}_dosing_interval"][j]),
                                  nan(g[f"{DRUG}_dose_after_dose_change"][j]), nan(g[f"{DRUG}_dose_change_time"][j]),
                                  int(g[f"{DRUG}_intermittent"][j]),
                                  [i for i, f in enumerate(g["treatment_interruptions"][j]) if f])
    ot, oc = X.filter_observations(g["time"], [nan(c) for c in g[f"{DRUG}_plasma_concentration"][j]])
    names = [p[0] for p in PRIOR]
    a = VARIANTS[variant]
    ix = names.index
    return {
        "d": len(names), "n_transit": int(a.get("num_transit_compartments", 0)),
        "peripheral": int(a.get("peripheral_compartment") == "true"),
        "biphasic": int(a.get("biphasic_absorption") == "true"),
        "metabolite": int(a.get("metabolite") == "true"),
        "additive_sd_ix": ix("additive_error_standard_deviation"),
        "proportional_sd_ix": ix("proportional_error_standard_deviation"),
        "absorption_ix": ix("absorption"), "clearance_ix": ix("clearance"), "vod_ix": ix("volume_of_distribution"),
        "excretion_ix": ix("excretion"),
        "pf_ix": ix("peripheral_forward_rate") if a.get("peripheral_compartment") == "true" else -1,
        "pb_ix": ix("peripheral_backward_rate") if a.get("peripheral_compartment") == "true" else -1,
        "mtt_ix": ix("mean_transit_time") if int(a.get("num_transit_compartments", 0)) > 0 else -1,
        "direct_ix": ix("direct_absorption") if a.get("biphasic_absorption") == "true" else -1,
        "metab_conv_ix": ix("metabolite_conversion_rate") if a.get("metabolite") == "true" else -1,
        "n_treat": len(tt), "n_obs": len(ot), "MW": X.MW[DRUG], "transforms": [2] * len(names),
        "treat_times": tt, "treat_doses": td, "obs_times": ot, "obs_conc": oc,
    }


def draws(n, seed):
    lo = np.array([p[1] for p in PRIOR])
    hi = np.array([p[2] for p in PRIOR])
    return lo + np.random.default_rng(seed).random((n, len(PRIOR))) * (hi - lo)


def main():
    rng = np.random.default_rng(20251017)
    # synthetic observations: the "all" variant's structure is too rich for a realistic drug;
    # simulate with the peripheral model at TRUE
    g = {"time": TIME, "patients": list(PATIENTS), f"{DRUG}_plasma_concentration": [],
         f"{DRUG}_dose": [], f"{DRUG}_dosing_interval": [], f"{DRUG}_dose_after_dose_change": [],
         f"{DRUG}_dose_change_time": [], f"{DRUG}_intermittent": [], "treatment_interruptions": []}
    for pid, (dose, tau, dac, dct, inter, skipped) in PATIENTS.items():
        g[f"{DRUG}_dose"].append(dose)
        g[f"{DRUG}_dosing_interval"].append(tau)
        g[f"{DRUG}_dose_after_dose_change"].append(None if math.isnan(dac) else dac)
        g[f"{DRUG}_dose_change_time"].append(None if math.isnan(dct) else dct)
        g[f"{DRUG}_intermittent"].append(inter)
        g["treatment_interruptions"].append([1 if d in skipped else 0 for d in range(29)])
        g[f"{DRUG}_plasma_concentration"].append([0.0] * len(TIME))
    pk = {TRIAL: g}
    for j, pid in enumerate(PATIENTS):
        m = model_fields("peripheral", pid, pk)
        A, conv, add_sd, prop_sd, _ = X.construct_matrix(m, np.array(TRUE))
        ok, central = X.solve_ref(A, m["treat_times"], m["treat_doses"], np.array(TIME))
        assert ok
        x = conv * central
        y = x + (add_sd + prop_sd * np.maximum(x, 0)) * rng.standard_t(4, len(TIME))
        conc = [float(v) for v in y]
        conc[0] = None  # pre-dose: unobserved
        if pid == "B2":
            conc[5] = None
        g[f"{DRUG}_plasma_concentration"][j] = conc
    with open(os.path.join(HERE, "pharmaco_pkdata.json"), "w") as f:
        json.dump(pk, f)
    with open(os.path.join(HERE, "pharmaco_prior.xml"), "w") as f:
        f.write(prior_xml())
    with open(os.path.join(HERE, "pharmaco_single_likelihood.xml"), "w") as f:  # bench.py's workload
        f.write(likelihood_xml("all", "B2"))
    out = {}
    for k, variant in enumerate(VARIANTS):
        for pid in PATIENTS:
            m = model_fields(variant, pid, pk)
            v = draws(N_DRAWS, 1000 + k)
            v[0] = TRUE
            logp, ok = X.evaluate(m, v, backend="ref")
            out[f"{variant}_{pid}_values"] = v
            out[f"{variant}_{pid}_logp"] = logp
            out[f"{variant}_{pid}_ok"] = ok
            print(variant, pid, "finite", int(np.isfinite(logp).sum()), "of", len(logp))
    np.savez_compressed(os.path.join(HERE, "pharmaco_single_golden.npz"), **out)


if __name__ == "__main__":
    main()
