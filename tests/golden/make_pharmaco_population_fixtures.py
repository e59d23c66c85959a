"""Golden fixtures for the pharmaco_population likelihood (PharmacoLikelihoodPopulation.cpp).

Run in the build container after make_pharmaco_fixtures.py (needs oracle/_ref/libexpmref.so, the
reference's vendored Eigen):
    python tests/golden/make_pharmaco_population_fixtures.py

Inputs: pharmaco_pkdata.json (the two synthetic patients of the pharmaco_single fixtures).
Outputs (data only):
  pharmaco_population_prior.xml   mean_* (log10 values, read raw as the reference does),
                                  sigma_*, and p<i>_* patient quantiles / bioavailabilities
  pharmaco_population_golden.npz  per variant: 48 prior draws and the Eigen-built logp
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, HERE)

import expm_pk as X  # noqa: E402
import make_pharmaco_fixtures as S  # noqa: E402

RATES = ["absorption", "excretion", "clearance", "volume_of_distribution", "transit_time"]
# name, lower, upper, logspace
PRIOR = [
    ("mean_absorption", -1.5, 0.5, False),
    ("mean_excretion", -4.0, -1.0, False),
    ("mean_clearance", 0.0, 2.0, False),
    ("mean_volume_of_distribution", 1.5, 3.0, False),
    ("mean_transit_time", -0.5, 1.0, True),
    ("peripheral_forward_rate", -3.0, -0.5, True),
    ("peripheral_backward_rate", -3.0, -0.5, True),
    ("additive_error_standard_deviation", -1.0, 1.5, True),
    ("proportional_error_standard_deviation", -2.0, -0.5, True),
] + [(f"sigma_{r}", 0.02, 0.5, False) for r in RATES] + \
    [(f"p{i + 1}_{r}", 0.01, 0.99, False) for i in range(len(S.PATIENTS)) for r in RATES] + \
    [(f"p{i + 1}_bioavailability", 0.3, 1.0, False) for i in range(len(S.PATIENTS))]
# (pk_model attributes, the sigma_* variables present) per variant
VARIANTS = {
    "mean_only": ({}, []),
    "random": ({}, ["absorption", "clearance", "volume_of_distribution"]),
    "peripheral": ({"peripheral_compartment": "true"}, ["clearance"]),
    "transit_fixed": ({"num_transit_compartments": "2"}, ["absorption"]),
    "all": ({"peripheral_compartment": "true", "num_transit_compartments": "3", "bioavailability": "true"}, RATES),
}
N_DRAWS = 48


def prior_xml(variant: str | None = None) -> str:
    """all variables; with a variant, the sigma_* it does not use are left out (their presence
    switches the random effect on, PharmacoLikelihoodPopulation.cpp:130-164)"""
    keep = None if variant is None else set(VARIANTS[variant][1])
    rows = []
    for n, a, b, lg in PRIOR:
        if keep is not None and n.startswith("sigma_") and n[6:] not in keep:
            continue
        rows.append(f'  <variable name="{n}" distribution="uniform" lower="{a}" upper="{b}" '
                    f'logspace="{"true" if lg else "false"}"/>')
    return '<?xml version="1.0" encoding="utf-8"?>\n<variableset>\n' + "\n".join(rows) + "\n</variableset>\n"


def names(variant: str) -> list[str]:
    keep = set(VARIANTS[variant][1])
    return [p[0] for p in PRIOR if not (p[0].startswith("sigma_") and p[0][6:] not in keep)]


def likelihood_xml(variant: str, pkdata_file: str = "pharmaco_pkdata.json") -> str:
    attrs = " ".join(f'{k}="{v}"' for k, v in VARIANTS[variant][0].items())
    return (f'<bcm_likelihood type="pharmaco_population">\n  <pk_model drug="{S.DRUG}" trial="{S.TRIAL}" '
            f'pkdata_file="{pkdata_file}" {attrs}/>\n</bcm_likelihood>\n')


def model_fields(variant: str, pkdata: dict) -> dict:
    """The bcm3hip_expm_pk_model the host layer derives for pharmaco_population"""
    a, sig = VARIANTS[variant]
    nm = names(variant)
    ix = lambda n: nm.index(n) if n in nm else -1  # noqa: E731
    pats = pkdata[S.TRIAL]["patients"]
    P = len(pats)
    tt, td, ot, oc, toff, ooff = [], [], [], [], [0], [0]
    for pid in pats:
        m1 = S.model_fields("plain", pid, pkdata)
        tt += list(m1["treat_times"]); td += list(m1["treat_doses"])
        ot += list(m1["obs_times"]); oc += list(m1["obs_conc"])
        toff.append(len(tt)); ooff.append(len(ot))
    nt = int(a.get("num_transit_compartments", 0))
    per = a.get("peripheral_compartment") == "true"
    pix = [-1] * (6 * P)
    for w, r in enumerate(RATES + ["bioavailability"]):
        on = (r in sig) if r != "bioavailability" else a.get("bioavailability") == "true"
        for j in range(P):
            if on:
                pix[w * P + j] = ix(f"p{j + 1}_{r}")
    return {
        "d": len(nm), "n_transit": nt, "peripheral": int(per), "biphasic": 0, "metabolite": 0,
        "additive_sd_ix": ix("additive_error_standard_deviation"),
        "proportional_sd_ix": ix("proportional_error_standard_deviation"),
        "absorption_ix": ix("mean_absorption"), "clearance_ix": ix("mean_clearance"),
        "vod_ix": ix("mean_volume_of_distribution"), "excretion_ix": ix("mean_excretion"),
        "pf_ix": ix("peripheral_forward_rate") if per else -1, "pb_ix": ix("peripheral_backward_rate") if per else -1,
        "mtt_ix": ix("mean_transit_time") if nt > 0 else -1, "direct_ix": -1, "metab_conv_ix": -1,
        "n_treat": len(tt), "n_obs": len(ot), "MW": X.MW[S.DRUG],
        "transforms": [2 if p[3] else 0 for p in PRIOR if p[0] in nm],
        "treat_times": tt, "treat_doses": td, "obs_times": ot, "obs_conc": oc,
        "param_map": 0, "P": P, "sigma_ix": [ix(f"sigma_{r}") for r in RATES], "patient_ix": pix,
        "treat_offset": toff, "obs_offset": ooff,
    }


def draws(variant: str, n: int, seed: int) -> np.ndarray:
    rows = [p for p in PRIOR if p[0] in names(variant)]
    lo = np.array([p[1] for p in rows])
    hi = np.array([p[2] for p in rows])
    return lo + np.random.default_rng(seed).random((n, len(rows))) * (hi - lo)


def main():
    with open(os.path.join(HERE, "pharmaco_pkdata.json")) as f:
        pk = json.load(f)
    with open(os.path.join(HERE, "pharmaco_population_prior.xml"), "w") as f:
        f.write(prior_xml())
    with open(os.path.join(HERE, "pharmaco_population_likelihood.xml"), "w") as f:  # bench.py's workload
        f.write(likelihood_xml("all"))
    out = {}
    for k, variant in enumerate(VARIANTS):
        m = model_fields(variant, pk)
        v = draws(variant, N_DRAWS, 2000 + k)
        logp, ok = X.evaluate(m, v, backend="ref")
        out[f"{variant}_values"] = v
        out[f"{variant}_logp"] = logp
        out[f"{variant}_ok"] = ok
        print(variant, "d", m["d"], "finite", int(np.isfinite(logp).sum()), "of", len(logp))
    np.savez_compressed(os.path.join(HERE, "pharmaco_population_golden.npz"), **out)


if __name__ == "__main__":
    main()
