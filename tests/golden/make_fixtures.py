"""Generate the committed golden fixtures for the PopPK / analytic parity tests.

Run in the build container (needs oracle/_ref built from /root/reference):
    python tests/golden/make_fixtures.py

Outputs (all data; no reference source text):
  c3_pkdata.json / p64_pkdata.json   synthetic pkdata (JSON sidecar of the netCDF schema,
                                     LikelihoodPopPKTrajectory.cpp:94-204) with observations
                                     simulated by the reference-built CVODE at TRUE_* + t4 noise
  c3_prior.xml, c3_likelihood.xml    inputs in the reference's own XML formats
  c3_golden.npz                      512 prior draws (seed 20251016) with the reference-built
                                     oracle's logp, per-patient llh, trajectories, step counters,
                                     from the build with FMA contraction (as the reference's CMake
                                     builds it) and without (`*_nofma`, the arithmetic the GPU follows)
  analytic_golden.npz                banana / circular draws with reference-formula outputs
  c3_golden_llh.npz                  8,192 prior draws (seed 20251021, regenerated from the seed by
                                     synthetic.prior_draws) with the reference-built oracle's logp,
                                     step counts and ok flags, and the same from the reference built
                                     without FMA contraction (its self-spread); `--llh-only` writes
                                     just this file; `--draws-only` rewrites c3_golden.npz and this
                                     file from the committed pkdata (after a change of the reference
                                     build, e.g. the N = 3 solve through the vendored Eigen)
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
sys.path.insert(0, HERE)

import oracle as O  # noqa: E402
import synthetic as S  # noqa: E402


def variables(P):
    return [O.Variable(n, lo, hi, O.TF_LOG10 if ls else O.TF_NONE) for n, lo, hi, ls in S.variables(P)]


def t4_noise(rng, n):
    # Student-t with nu = 4 (the observation model of LogPdfTnu4)
    return rng.standard_t(4, size=n)


def make_pkdata(P: int, seed: int) -> dict:
    rng = np.random.default_rng(seed)
    pk = S.pkdata_skeleton(P)
    prob = O.build_problem(pk, S.TRIAL, S.DRUG, S.PK_TYPE, variables(P))
    true = list(S.TRUE_POP)
    for j in range(P):
        true += [float(rng.uniform(0.2, 0.8)), float(rng.uniform(0.2, 0.8))]
    true += S.TRUE_SD
    true = np.array(true)
    ref = O.Oracle("ref")
    out = ref.popk_eval(prob, true[None, :])
    conv = (1e6 / prob.MW) / (10 ** true[3])
    sd, sd2 = 10 ** true[-2], 10 ** true[-1]
    obs = []
    for j in range(P):
        x = conv * out["traj"][0, j, 1, :]
        y = x + t4_noise(rng, len(x)) * (sd + sd2 * np.maximum(x, 0))
        row = [None if S.TIMES[i] == 0 else float(max(y[i], 0.0)) for i in range(len(x))]
        obs.append(row)
    pk[S.TRIAL][S.DRUG + "_plasma_concentration"] = obs
    return pk


LLH_SEED, LLH_N = 20251021, 8192


def make_llh_fixture():
    pk = O.load_pkdata(os.path.join(HERE, "c3_pkdata.json"))
    prob = O.build_problem(pk, S.TRIAL, S.DRUG, S.PK_TYPE, variables(1))
    draws = S.prior_draws(1, LLH_N, LLH_SEED)
    ref = O.Oracle("ref").popk_eval(prob, draws, nthreads=8, want_traj=False)
    nof = O.Oracle("ref_nofma").popk_eval(prob, draws, nthreads=8, want_traj=False)
    np.savez_compressed(os.path.join(HERE, "c3_golden_llh.npz"), seed=LLH_SEED, n=LLH_N,
                        values_sum=draws.sum(), logp=ref["logp"], nst=ref["stats"][:, 0, 0], ok=ref["ok"][:, 0],
                        logp_nofma=nof["logp"], nst_nofma=nof["stats"][:, 0, 0])


def make_c3_golden():
    pk = O.load_pkdata(os.path.join(HERE, "c3_pkdata.json"))
    prob = O.build_problem(pk, S.TRIAL, S.DRUG, S.PK_TYPE, variables(1))
    draws = S.prior_draws(1, 512, 20251016)
    ref = O.Oracle("ref").popk_eval(prob, draws)
    nof = O.Oracle("ref_nofma").popk_eval(prob, draws)
    np.savez_compressed(os.path.join(HERE, "c3_golden.npz"), values=draws, logp=ref["logp"],
                        patient_llh=ref["patient_llh"], traj=ref["traj"], stats=ref["stats"], ok=ref["ok"],
                        logp_nofma=nof["logp"], patient_llh_nofma=nof["patient_llh"], traj_nofma=nof["traj"],
                        stats_nofma=nof["stats"], ok_nofma=nof["ok"])


def main():
    if "--llh-only" in sys.argv:
        make_llh_fixture()
        return
    if "--draws-only" in sys.argv:
        make_c3_golden()
        make_llh_fixture()
        return
    for P, name, seed in ((1, "c3", 20251015), (64, "p64", 20251017)):
        pk = make_pkdata(P, seed)
        with open(os.path.join(HERE, f"{name}_pkdata.json"), "w") as f:
            json.dump(pk, f)
        with open(os.path.join(HERE, f"{name}_prior.xml"), "w") as f:
            f.write(S.prior_xml(P))
        with open(os.path.join(HERE, f"{name}_likelihood.xml"), "w") as f:
            f.write(S.likelihood_xml(f"{name}_pkdata.json"))

    make_c3_golden()

    # analytic: banana (examples/banana: dimension 2, sd1 2, sd2 1, U(-6,4)xU(-6,20)) and
    # circular (examples/multimodal_circular_ridge: U(-6,6)^2, offset 3.5 radius 2 width 0.1)
    rng = np.random.default_rng(20251018)
    b = np.stack([rng.uniform(-6, 4, 1024), rng.uniform(-6, 20, 1024)], axis=1)
    c = rng.uniform(-6, 6, (1024, 2))
    r = O.Oracle("ref")
    np.savez_compressed(os.path.join(HERE, "analytic_golden.npz"), banana_values=b,
                        banana_logp=r.banana(b, 2, 2.0, 1.0), circular_values=c,
                        circular_logp=r.circular(c, 2, 2.0, 3.5, 0.1))
    make_llh_fixture()
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
