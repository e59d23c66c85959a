"""CPU tests of the cell-population likelihood with solver_type="DP5" (Cell::AllocateSolver,
src/cellpop/Cell.cpp:57-66; ODESolverDP5, src/odecommon/ODESolverDP5.cpp): the oracle's restatement
of the reference's Dormand-Prince solver and its cell-driver semantics, and the product's loader /
kernel build.

The reference's DP5 source cannot be compiled here (Utils.h pulls in Boost), so oracle/cellpop_ref.cpp
restates ApplyRK / Solve statement for statement; parity of that restatement is unpinned beyond the
published Dormand-Prince tableau and Hairer's dense output it transcribes, and checked here against a
fixed-step reference integration of the same ODE."""
import ctypes
import math
import os

import numpy as np
import pytest

import cellpop_helpers as CH
import cellpop as CP

# name -> likelihood kwargs
CASES = {
    "division": dict(num_cells=16, max_cells=64, experiment_attrs=' solver_type="DP5"'),
    "no_division": dict(num_cells=16, max_cells=16, experiment_attrs=' solver_type="DP5" divide_cells="false"'),
    "late_entry": dict(num_cells=8, max_cells=32, experiment_attrs=' solver_type="DP5"', entry_time="1.5"),
    # max_dt (ODESolverDP5::SetSolverParameter: the first step min(max_dt, 1) and the growth clamp)
    "max_dt": dict(num_cells=16, max_cells=64, experiment_attrs=' solver_type="DP5" solver_max_timestep="0.25"'),
}


def dp5_likelihood(directory, name, **extra):
    import make_cellpop_fixtures as F
    kw = dict(CASES[name])
    kw.update(extra)
    path = os.path.join(str(directory), f"dp5_{name}.xml")
    with open(path, "w") as f:
        f.write(F.likelihood_text(data_file=os.path.join(CH.GOLDEN, "cellpop_data.json"),
                                  model_file=os.path.join(CH.GOLDEN, "cellpop_model.xml"), **kw))
    return path


@pytest.mark.parametrize("name", list(CASES))
def test_oracle_builds_agree(tmp_path, name):
    """the restatement built with and without FMA contraction (the reference's two builds)"""
    path = dp5_likelihood(tmp_path, name)
    x = CH.draws(4, 7)
    a = CP.simulate(CP.load_problem(path, CH.PRIOR), x)["logp"]
    b = CP.simulate(CP.load_problem(path, CH.PRIOR, variant="nofma"), x)["logp"]
    assert ((a == -math.inf) == (b == -math.inf)).all()
    fin = np.isfinite(a)
    assert fin.any()
    assert (np.abs(a[fin] - b[fin]) <= 1e-6 * (1 + np.abs(a[fin]))).all()


def test_dp5_semantics(tmp_path):
    """the reference's DP5 cell behaviour: no threshold crossings (the event times stay NaN, so no
    cell "enters mitosis"), a division does not stop the integration (the step callback's result is
    ignored) and the solve resets the outputs before the cell's creation to NaN"""
    prob = CP.load_problem(dp5_likelihood(tmp_path, "division"), CH.PRIOR)
    r = CP.simulate(prob, CH.draws(1, 3))
    cells = r["detail"][0]["cells"]
    assert all(all(math.isnan(v) for v in c["events"]) for c in cells)
    div = [c for c in cells if c["divided"]]
    assert div, "the test model divides within 20 h"
    # the cell keeps integrating past cytokinesis: its simulation end is a later step than the first
    # one with cytokinesis > 1, i.e. one step after the end_time the anaphase callback set
    e = prob["experiments"][0]
    late = CP.load_problem(dp5_likelihood(tmp_path, "late_entry"), CH.PRIOR)
    rl = CP.simulate(late, CH.draws(1, 3))
    ek = late["experiments"][0]
    k0 = [k for k, t in enumerate(ek["timepoints"]) if t[1] - 1.5 < 2.220446049250313e-16]
    assert k0, "time points before the cells' creation"
    for c in rl["detail"][0]["cells"]:
        assert all(math.isnan(c["values"][k]) for k in k0)
    assert e["solver"] == 1


def test_dp5_tracks_a_fine_integration(tmp_path):
    """the restated DP5 solution of one cell against a fine fixed-step RK4 integration of the same
    generated right-hand side (an independent check of the transcribed tableau)"""
    prob = CP.load_problem(dp5_likelihood(tmp_path, "no_division", num_cells=1, max_cells=1), CH.PRIOR)
    e = prob["experiments"][0]
    x = CH.draws(1, 3)[0]
    r = CP.simulate(prob, x[None, :])
    cell = r["detail"][0]["cells"][0]
    tv = [CP.transform(tf, v) for tf, v in zip(prob["transforms"], x)]
    N = len(e["model"].ode)
    f = e["deriv_lib"].generated_derivative
    f.argtypes = [ctypes.c_void_p] * 5
    cs = np.ascontiguousarray(e["constant_init"], dtype=float)
    prm = np.ascontiguousarray(tv, dtype=float)

    def rhs(y):
        out = np.empty(N)
        yy = np.ascontiguousarray(y)
        f(out.ctypes.data, yy.ctypes.data, cs.ctypes.data, prm.ctypes.data, None)
        return out

    y = np.array(cell["y0"], dtype=float)
    h = 1e-3
    t = 0.0
    ks = [k for k, tp in enumerate(e["timepoints"]) if tp[3] >= 0]
    want = {}
    for k in ks:
        tk = e["timepoints"][k][1]
        while t + h <= tk + 1e-12:
            k1 = rhs(y)
            k2 = rhs(y + 0.5 * h * k1)
            k3 = rhs(y + 0.5 * h * k2)
            k4 = rhs(y + h * k3)
            y = y + h / 6 * (k1 + 2 * k2 + 2 * k3 + k4)
            t += h
        want[k] = y[e["timepoints"][k][3]]
    for k in ks:
        if e["timepoints"][k][1] < 1e-12:
            continue
        assert abs(cell["values"][k] - want[k]) <= 1e-4 * (1 + abs(want[k])), (k, cell["values"][k], want[k])


@pytest.mark.parametrize("name", list(CASES))
def test_loader_builds_the_dp5_kernel(tmp_path, name):
    from bcm3_amd import likelihood
    ll = likelihood.Likelihood(dp5_likelihood(tmp_path, name), CH.PRIOR, options="backend=none")
    L = likelihood.lib()
    L.bcm3_likelihood_cellpop_precompile.argtypes = [ctypes.c_void_p]
    assert L.bcm3_likelihood_cellpop_precompile(ll.h) == 0
    ll.close()


def test_loader_refuses_dp5_with_synchronisation_or_treatments_and_unknown_solvers(tmp_path):
    """the reference's DP5 GetInterpolatedY / get_threshold_crossing_time are not implemented (NaN),
    its discontinuity handling is not built here; an unknown solver_type fails as in
    Cell::AllocateSolver"""
    from bcm3_amd import likelihood
    import make_cellpop_fixtures as F
    sync_tc = '<data data_name="pcna_sync" species_name="PCNA_gfp" stdev="stdev" synchronize="mitosis"/>'
    pulses = '\n    <treatment_trajectory type="pulses" species_name="mitogen" times="5"/>'
    bad = [dict(num_cells=16, max_cells=16, data_file=os.path.join(CH.GOLDEN, "cellpop_sync_data.json"), data_xml=sync_tc,
                experiment_attrs=' solver_type="DP5" divide_cells="false"'),
           dict(num_cells=16, max_cells=64, data_file=os.path.join(CH.GOLDEN, "cellpop_data.json"), extra=pulses,
                experiment_attrs=' solver_type="DP5"'),
           dict(num_cells=16, max_cells=64, data_file=os.path.join(CH.GOLDEN, "cellpop_data.json"),
                experiment_attrs=' solver_type="RK4"')]
    for kw in bad:
        path = os.path.join(str(tmp_path), "bad.xml")
        with open(path, "w") as f:
            f.write(F.likelihood_text(model_file=os.path.join(CH.GOLDEN, "cellpop_model.xml"), **kw))
        with pytest.raises(RuntimeError):
            likelihood.Likelihood(path, CH.PRIOR, options="backend=none")
