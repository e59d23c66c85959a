"""GPU parity of the cell-population likelihood with solver_type="DP5" (the per-model cell kernel's
CP_DP5 path, cellpop_solver.h) against the oracle's restatement of the reference's ODESolverDP5
(oracle/cellpop_ref.cpp); the cases of tests/test_cellpop_dp5.py.

The device evaluates the same Dormand-Prince stages, error ratio (a NaN-skipping row maximum, exact
in any order) and Hairer dense output as the reference, uncontracted; the step-size factor's pow is
glibc's (xm::pow_glibc_pos on the loaded libm's tables, round 6; round 5 used the device's pow, ~1 ulp
from glibc, so step sequences could part after a near-tie of the acceptance thresholds). Bar: logp within the cell-population envelope (cellpop_helpers.logp_bar: 1e-6 (1 + |logp|)
or 10x the oracle's own FMA / no-FMA difference on the draw) with an identical -inf pattern, the same cell counts and division decisions, simulation ends within 1e-3 h, and the same
step count on >= 99 % of cells."""
import math

import numpy as np
import pytest

import cellpop_helpers as CH
import cellpop as CP
from test_cellpop_dp5 import CASES, dp5_likelihood

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", params=list(CASES))
def dp5_case(request, tmp_path_factory):
    from bcm3_amd.likelihood import Likelihood
    path = dp5_likelihood(tmp_path_factory.mktemp("dp5_gpu"), request.param)
    ll = Likelihood(path, CH.PRIOR, device=0)
    prob = CP.load_problem(path, CH.PRIOR)
    x = CH.draws(8, 11)
    yield request.param, ll, prob, x, path
    ll.close()


def test_dp5_matches_oracle(dp5_case):
    name, ll, prob, x, path = dp5_case
    lp, status = ll.evaluate_batch(x)
    r = CP.simulate(prob, x)
    ref = r["logp"]
    ref_nofma = CP.simulate(CP.load_problem(path, CH.PRIOR, variant="nofma"), x)["logp"]
    CH.check_logp(lp, None, ref, ref_nofma, name=f"dp5 {name}")
    e = prob["experiments"][0]
    M, NS = len(e["output_times"]), len(e["model"].ode)
    same_steps = total = 0
    for i in range(len(x)):
        if status[i] != 0:
            continue
        cells = r["detail"][i]["cells"]
        rec, vals, _ = ll.cellpop_cells(i, M, NS)
        assert len(rec) == len(cells), (name, i)
        for c, oc in enumerate(cells):
            assert bool(rec["flags"][c] & 2) == oc["divided"], (name, i, c)
            assert not rec["flags"][c] & 8  # no crossings: never "entered mitosis"
            assert abs(rec["sim_end"][c] - oc["sim_end"]) <= 1e-3, (name, i, c, rec["sim_end"][c], oc["sim_end"])
            assert (np.isnan(vals[c]) == np.isnan(oc["values"])).all(), (name, i, c)
            same_steps += int(rec["nsteps"][c] == oc["nsteps"])
            total += 1
    import parity
    parity.log_summary({"dp5_steps_equal": same_steps / max(1, total), "cells": total, "case": name}, n=len(x))
    assert total > 0 and same_steps >= 0.99 * total, (name, same_steps, total)
