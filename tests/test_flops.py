"""F_alg: the op-counting build of the oracle computes the same logp as the
restatement, bit for bit, and reproduces the frozen per-draw counts in tests/golden/c3_falg.json
that bench.py's FP64 roofline uses."""
import json
import os

import numpy as np
import pytest

import helpers as H
import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def c3():
    return H.c3_problem(1), np.load(os.path.join(GOLDEN, "c3_golden.npz"))


def test_flops_build_is_the_restatement(c3):
    prob, z = c3
    a = O.Oracle("flops").popk_eval(prob, z["values"][:64], want_traj=True)
    b = O.Oracle("restated").popk_eval(prob, z["values"][:64], want_traj=True)
    assert np.array_equal(a["logp"], b["logp"], equal_nan=True)
    assert np.array_equal(a["traj"], b["traj"], equal_nan=True)
    assert np.array_equal(a["stats"], b["stats"])


def test_frozen_falg(c3):
    prob, z = c3
    with open(os.path.join(GOLDEN, "c3_falg.json")) as f:
        frozen = json.load(f)
    fl = O.Oracle("flops").popk_flops(prob, z["values"])
    assert fl.tolist() == frozen["per_draw"]
    assert fl.mean() == frozen["flops_per_eval_mean"]
    # about 290 flops per BDF step (SURVEY.md §8(d) estimate: ~220)
    assert 150 < frozen["flops_per_bdf_step"] < 500


def test_counter_counts_only_arithmetic():
    # one quantile = a known number of operations, and a second call repeats it exactly
    orc = O.Oracle("flops")
    orc.lib.orc_flops_take()
    orc.lib.orc_log_pdf_tnu4(1.0, 0.5, 2.0)
    n1 = orc.lib.orc_flops_take()
    orc.lib.orc_log_pdf_tnu4(3.0, 0.5, 2.0)
    assert orc.lib.orc_flops_take() == n1 > 0


def test_c4_falg_fixture_matches_the_model():
    """tests/golden/c4_falg.json (bench.py's C4 FP64 roofline): its right-hand-side operation count
    is the count of the committed cell model's generated derivative (make_c4_falg.rhs_ops), and the
    per-cell-step figure is within the model's range (RHS-dominated, N = 15 species)"""
    import sys
    if GOLDEN not in sys.path:
        sys.path.insert(0, GOLDEN)
    import cellpop as CP
    import cellpop_helpers as CH
    import make_c4_falg as F
    with open(os.path.join(GOLDEN, "c4_falg.json")) as f:
        fx = json.load(f)
    prob = CP.load_problem(os.path.join(GOLDEN, "cellpop_likelihood.xml"), CH.PRIOR)
    e = prob["experiments"][0]
    assert fx["species"] == len(e["model"].ode) == 15
    assert fx["f_rhs"] == F.rhs_ops(e["derivative_body"])
    assert 20 * fx["species"] + 70 < fx["flops_per_cell_step"] < 10 * (fx["species"] * fx["f_rhs"])
