"""GPU parity of the cell-population likelihood (config C4) against the oracle: the reference's
vendored CVODE 5.3.0 with its PartialPivLU per cell (oracle/_ref/libcellpopref.so) under the
restated Experiment / Cell logic (oracle/cellpop.py).

Parity envelope (stated here, as north_star asks for fp64 work). The device integrates the same BDF
arithmetic with hardware-reciprocal division, a column-oriented LU solve and ocml's pow/exp; the
oracle uses Eigen's blocked triangular solves and glibc. An adaptive solver at rtol = atol =
4*FLT_EPSILON amplifies last-bit differences (a difference-quotient Jacobian with a different
increment, a corrector that converged one ulp apart) into step sizes that differ at ~1e-7, so the
reference is not reproducible to more than that even against ITSELF: the same sources built with
and without FMA contraction (oracle/_ref/libcellpopref_nofma.so) differ by up to ~5e-5 relative in
logp on these draws. The GPU must sit inside that spread:
  * identical cell bookkeeping: cell count, division decisions, daughter numbering;
  * step counts equal for >= 95 % of the cells;
  * creation and division times within 0.1 h (a step flip moves a division by one step),
    data values within 1e-3 relative;
  * logp within cellpop_helpers.logp_bar for every draw: 1e-5 * (1 + |logp|), or 10x the two
    reference builds' own difference on that draw when larger (round 6: the measured envelope,
    profiles/r06b_cellpop_parity.jsonl, not round 5's flat 2e-4), the -inf pattern identical, and
    the median GPU-vs-oracle deviation no larger than 10x the median oracle-vs-oracle(no FMA)
    deviation."""
import math

import numpy as np
import pytest

import cellpop_helpers as CH
import cellpop as CP
import parity

pytestmark = pytest.mark.gpu


TREAT = '\n    <treatment_trajectory type="pulses" species_name="mitogen" times="13,-1"/>'

# (initial cells, max cells, draws, likelihood options): the small case runs many draws; the larger
# one fills several four-cell wavefronts per generation with cells of different dynamics (rows
# diverge); the last two take the other error models (DataLikelihoodBase.cpp:51-70) and a
# population without division
CASES = [(6, 64, 12, {}), (40, 256, 4, {}),
         (8, 64, 6, dict(data_attrs='stdev="stdev" error_model="additive_proportional_normal" proportional_stdev="0.05"')),
         (6, 32, 6, dict(data_attrs='stdev="stdev" error_model="t4"', experiment_attrs=' divide_cells="false"')),
         (6, 64, 6, dict(data_attrs='stdev="stdev" relative_to_time_average="true" offset="0.05"')),
         # a treatment trajectory (TreatmentTrajectoryPulses) on the constant species mitogen: the
         # right-hand side follows the pulses and the solver stops and restarts at every pulse corner
         (8, 64, 6, dict(extra=TREAT)),
         # overlapping pulses: the next corner the reference's NextDiscontinuity gives after a pulse
         # end can lie behind the cell's time; CVode then refuses the stop time and the cell fails
         (6, 64, 4, dict(extra=TREAT.replace('"13,-1"', '"6,-1,13"'))),
         # an entry_time variability variable: it takes a sobol dimension of the group (the table gets
         # three) and is never applied (the reference has no ApplyVariabilityEntryTime call)
         (6, 64, 6, dict(variability_extra='\n      <variable entry_time="true" apply="additive" scale="var_kD"/>'))]


@pytest.fixture(scope="module", params=CASES, ids=["6cells", "40cells", "addprop", "t4_nodiv", "reltime", "pulses",
                                                           "pulses_overlap", "entry_time_var"])
def setup(request, tmp_path_factory):
    from bcm3_amd.likelihood import Likelihood
    nc, mc, nd, attrs = request.param
    d = tmp_path_factory.mktemp("cellpop_gpu")
    path = CH.write_likelihood(d, nc, mc, **attrs)
    ll = Likelihood(path, CH.PRIOR, device=0)
    prob = CP.load_problem(path, CH.PRIOR)
    x = CH.draws(nd, 11)
    ref = CP.simulate(prob, x)
    ref_nofma = CP.simulate(CP.load_problem(path, CH.PRIOR, variant="nofma"), x)
    yield ll, prob, x, ref, ref_nofma
    ll.close()


def test_logp_matches_oracle(setup):
    ll, prob, x, ref, ref_nofma = setup
    lp, status = ll.evaluate_batch(x)
    # per draw: the measured envelope, or 10x the reference's own FMA / no-FMA difference on this
    # draw when that is larger (a division one step earlier moves a small-sigma data likelihood by
    # more; e.g. addprop draw 2: the two reference builds differ by 6.8e-3)
    dev, spread = CH.check_logp(lp, status, ref["logp"], ref_nofma["logp"], name=f"{len(x)} draws")
    if dev:  # (every draw -inf: the overlapping-pulses case)
        assert np.median(dev) <= 10.0 * np.median(spread) + 1e-12, (np.median(dev), np.median(spread))


def test_cells_match_oracle(setup):
    ll, prob, x, ref, _ = setup
    ll.evaluate_batch(x)
    e = prob["experiments"][0]
    M, NS = len(e["output_times"]), len(e["model"].ode)
    same_steps = total = 0
    for i in range(len(x)):
        cells = ref["detail"][i]["cells"]
        if not ref["detail"][i]["ok"]:
            continue
        rec, vals, endy = ll.cellpop_cells(i, M, NS)
        assert len(rec) == len(cells), i
        for k, c in enumerate(cells):
            assert rec["flags"][k] & 1
            assert bool(rec["flags"][k] & 2) == c["divided"], (i, k)
            same_steps += int(rec["nsteps"][k] == c["nsteps"])
            total += 1
            # times in hours: within 0.1 h, a few BDF steps near a division (~0.05 h each). A cell
            # whose step count flips between builds divides one step earlier or later; the
            # reference flips such cells between its own FMA / no-FMA builds too (0.01-0.025 h)
            assert abs(rec["creation"][k] - c["creation"]) <= 0.1, (i, k)
            assert abs(rec["sim_end"][k] - c["sim_end"]) <= 0.1, (i, k)
            if rec["nsteps"][k] != c["nsteps"] or abs(rec["sim_end"][k] - c["sim_end"]) > 1e-3:
                continue  # a flipped step moves the end state; the logp envelope covers these cells
            np.testing.assert_array_equal(np.isnan(vals[k]), np.isnan(c["values"]))
            ok = ~np.isnan(c["values"])
            np.testing.assert_allclose(vals[k][ok], c["values"][ok], rtol=1e-3, atol=1e-9)
            np.testing.assert_allclose(endy[k], c["end_y"], rtol=1e-3, atol=1e-8)
    assert same_steps >= 0.95 * total, (same_steps, total)


def test_batch_invariance(setup):
    """logp[i] depends on values[i] only: a single evaluation equals the batch entry bit for bit"""
    ll, prob, x, ref, _ = setup
    lp, _ = ll.evaluate_batch(x)
    for i in (0, 3):
        one, _ = ll.evaluate_batch(x[i:i + 1])
        assert one[0] == lp[i] or (math.isnan(one[0]) and math.isnan(lp[i]))


def test_bench_size_batch_matches_oracle(tmp_path):
    """Config C4 as benched (tests/golden/cellpop_likelihood.xml: 500 initial cells, max_cells 2048,
    ~1,650 cells per evaluation) with the bench's 64 evaluations in ONE batch, so generation sizes,
    the generation loop and the cell numbering run at the bench's scale; all 64 evaluations checked
    against the oracle (both reference builds) inside the envelope of the module docstring."""
    import os
    import parity
    from bcm3_amd.likelihood import Likelihood
    path = os.path.join(CH.GOLDEN, "cellpop_likelihood.xml")
    ll = Likelihood(path, CH.PRIOR, device=0)
    x = CH.draws(64, 23)
    lp, status = ll.evaluate_batch(x)
    n = len(x)
    nthreads = max(1, min(16, len(os.sched_getaffinity(0))))
    prob = CP.load_problem(path, CH.PRIOR)
    ref = CP.simulate(prob, x[:n], nthreads=nthreads)
    ref_nofma = CP.simulate(CP.load_problem(path, CH.PRIOR, variant="nofma"), x[:n], nthreads=nthreads)
    e = prob["experiments"][0]
    M, NS = len(e["output_times"]), len(e["model"].ode)
    dev, spread = CH.check_logp(lp, status, ref["logp"], ref_nofma["logp"], name="bench-size batch")
    same_steps, total, cells_total = 0, 0, 0
    for i in range(n):
        if ref["logp"][i] == -math.inf:
            continue
        cells = ref["detail"][i]["cells"]
        rec, _, _ = ll.cellpop_cells(i, M, NS)
        assert len(rec) == len(cells), i
        cells_total += len(cells)
        for k, c in enumerate(cells):
            assert bool(rec["flags"][k] & 2) == c["divided"], (i, k)
            same_steps += int(rec["nsteps"][k] == c["nsteps"])
            total += 1
    assert dev, "every checked draw was -inf"
    if dev:  # (every draw -inf: the overlapping-pulses case)
        assert np.median(dev) <= 10.0 * np.median(spread) + 1e-12, (np.median(dev), np.median(spread))
    assert same_steps >= 0.95 * total, (same_steps, total)
    parity.log_summary({"cellpop_draws_checked": n, "finite": len(dev), "cells": cells_total,
                        "steps_equal": same_steps / max(1, total), "logp_dev_median": float(np.median(dev)),
                        "logp_dev_max": float(np.max(dev)), "ref_fma_spread_median": float(np.median(spread))},
                       n=n)
    # the rest of the batch: each entry equals its own single evaluation (no batch coupling)
    for i in (17, 40, 63):
        one, _ = ll.evaluate_batch(x[i:i + 1])
        assert one[0] == lp[i] or (math.isnan(one[0]) and math.isnan(lp[i]))
    ll.close()


def test_full_gaussian_variability_matches_oracle(tmp_path):
    """<cell_variability distribution="full_gaussian" covar_base_name="rho">: the two variability
    dimensions correlated through the sampled rho1_2 (VariabilityDescription.cpp:69-128); the cells'
    parameters / initial conditions and the logp against the reference-CVODE oracle with the same
    envelope as the diagonal cases"""
    from bcm3_amd.likelihood import Likelihood
    lik, prior = CH.write_full_gaussian(tmp_path, 8, 64)
    x = CH.draws_full(8, 17)
    ll = Likelihood(lik, prior, device=0)
    ref = CP.simulate(CP.load_problem(lik, prior), x)
    ref_nofma = CP.simulate(CP.load_problem(lik, prior, variant="nofma"), x)
    lp, status = ll.evaluate_batch(x)
    # the correlation changes the cells: the same draws with rho = 0 give other logp
    x0 = x.copy()
    x0[:, -1] = 0.0
    lp0, _ = ll.evaluate_batch(x0)
    fin = np.isfinite(lp) & np.isfinite(lp0)
    assert fin.any() and np.any(lp[fin] != lp0[fin])
    dev, spread = CH.check_logp(lp, status, ref["logp"], ref_nofma["logp"], name="full_gaussian")
    assert dev and np.median(dev) <= 10.0 * np.median(spread) + 1e-12, (np.median(dev), np.median(spread))
    # every cell's creation time and division decision as the oracle's
    e = CP.load_problem(lik, prior)["experiments"][0]
    M, NS = len(e["output_times"]), len(e["model"].ode)
    ll.evaluate_batch(x)
    for i in range(len(x)):
        if not ref["detail"][i]["ok"]:
            continue
        rec, _, _ = ll.cellpop_cells(i, M, NS)
        cells = ref["detail"][i]["cells"]
        assert len(rec) == len(cells), i
        for k, c in enumerate(cells):
            assert bool(rec["flags"][k] & 2) == c["divided"], (i, k)
            assert abs(rec["creation"][k] - c["creation"]) <= 0.1, (i, k)
    parity.log_summary({"logp_dev_median": float(np.median(dev)), "ref_fma_spread_median": float(np.median(spread))},
                       n=len(dev))
    ll.close()


def test_too_many_cells_is_minus_inf(tmp_path):
    from bcm3_amd.likelihood import Likelihood
    path = CH.write_likelihood(tmp_path, 4, 10, name="small_max.xml")
    ll = Likelihood(path, CH.PRIOR, device=0)
    lp, status = ll.evaluate_batch(np.array([CH.F.true_values()]))
    assert lp[0] == -math.inf and status[0] == 1
    ll.close()


def test_sampler_drives_cell_population(tmp_path):
    """config C4 end to end: the C++ PT-MH sampler (bcm3_ptmh_*) with the cell-population likelihood
    -- proposals, batched evaluation of all chains per mutate step, accept, exchange -- and the
    final chain states' log-likelihoods equal a fresh evaluation of the same values"""
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.ptmh import PTMHNative
    path = CH.write_likelihood(tmp_path, 6, 64)
    ll = Likelihood(path, CH.PRIOR, device=0)
    s = PTMHNative(ll, CH.PRIOR, 8, seed=3, adapt_proposal_samples=0)
    s.iterate(6)
    s.synchronize()
    st = s.state()
    c = s.counters()
    s.close()
    assert c["attempted_mutate"] == 6 * 8 and c["accepted_mutate"] > 0
    lp, _ = ll.evaluate_batch(st["values"])
    fin = np.isfinite(st["llh"])
    assert fin.any()
    np.testing.assert_array_equal(lp[fin], st["llh"][fin])
    ll.close()
