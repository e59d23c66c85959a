"""The cell work queue (BCM3_CP_QUEUE=1: one persistent launch of cellpop_solver.h's cp_queue_kernel, the
daughters enqueued as their mothers end -- the reference's aux-thread queue, Experiment.cpp:691-782)
against the generation launches on the same draws: it changes only the order in which cells are
solved, so the bar is bit-identity -- every logp (the -inf pattern included), and for every finite
evaluation the cell list (count, numbering, records, data values, end states). The generation
launches are checked against the oracle by test_cellpop_gpu.py and its siblings. A failed evaluation
stops enqueueing, so its cell list may be shorter than the generation launches' (its logp is -inf
either way)."""
import math
import os

import numpy as np
import pytest

import cellpop as CP
import cellpop_helpers as CH
from test_cellpop_dp5 import dp5_likelihood

pytestmark = pytest.mark.gpu

TREAT = '\n    <treatment_trajectory type="pulses" species_name="mitogen" times="13,-1"/>'


def _pair(path, prior, monkeypatch):
    from bcm3_amd.likelihood import Likelihood
    monkeypatch.setenv("BCM3_CP_QUEUE", "0")
    gen = Likelihood(path, prior, device=0)
    monkeypatch.setenv("BCM3_CP_QUEUE", "1")
    que = Likelihood(path, prior, device=0)
    e = CP.load_problem(path, prior)["experiments"][0]
    gen.shape = que.shape = (len(e["output_times"]), len(e["model"].ode))
    return gen, que


def _same(gen, que, x):
    M, NS = gen.shape
    lp_g, st_g = gen.evaluate_batch(x)
    lp_q, st_q = que.evaluate_batch(x)
    np.testing.assert_array_equal(st_q, st_g)
    assert lp_q.tobytes() == lp_g.tobytes(), np.nonzero(lp_q != lp_g)
    fin = np.isfinite(lp_g)
    for i in np.nonzero(fin)[0]:
        rg, vg, yg = gen.cellpop_cells(int(i), M, NS)
        rq, vq, yq = que.cellpop_cells(int(i), M, NS)
        assert len(rq) == len(rg), i
        assert rq.tobytes() == rg.tobytes() and vq.tobytes() == vg.tobytes() and yq.tobytes() == yg.tobytes(), i
    return int(fin.sum())


CASES = {"6cells": (6, 64, 12, {}), "40cells": (40, 256, 6, {}),
         "nodiv": (6, 32, 6, dict(data_attrs='stdev="stdev" error_model="t4"', experiment_attrs=' divide_cells="false"')),
         "pulses": (8, 64, 6, dict(extra=TREAT)),
         "entry_time_var": (6, 64, 6, dict(variability_extra='\n      <variable entry_time="true" apply="additive" scale="var_kD"/>')),
         # max_cells reached: the evaluation fails (the cap check moves onto the device)
         "cap": (4, 10, 6, {}),
         "late_entry": (8, 32, 6, dict(entry_time="1.5"))}


@pytest.mark.parametrize("case", list(CASES))
def test_queue_matches_generation_launches(case, tmp_path, monkeypatch):
    nc, mc, nd, attrs = CASES[case]
    path = CH.write_likelihood(tmp_path, nc, mc, **attrs)
    gen, que = _pair(path, CH.PRIOR, monkeypatch)
    x = CH.draws(nd, 11)
    _same(gen, que, x)
    # batch sizes: one evaluation, and an odd count
    _same(gen, que, x[:1])
    _same(gen, que, x[:3])
    gen.close()
    que.close()


def test_queue_cap_fails_like_generation_launches(tmp_path, monkeypatch):
    path = CH.write_likelihood(tmp_path, 4, 10, name="small_max.xml")
    gen, que = _pair(path, CH.PRIOR, monkeypatch)
    lp, status = que.evaluate_batch(np.array([CH.F.true_values()]))
    assert lp[0] == -math.inf and status[0] == 1
    gen.close()
    que.close()


def test_queue_full_gaussian(tmp_path, monkeypatch):
    lik, prior = CH.write_full_gaussian(tmp_path, 8, 64)
    gen, que = _pair(lik, prior, monkeypatch)
    _same(gen, que, CH.draws_full(8, 17))
    gen.close()
    que.close()


def test_queue_dp5(tmp_path, monkeypatch):
    path = dp5_likelihood(tmp_path, "division")
    gen, que = _pair(path, CH.PRIOR, monkeypatch)
    _same(gen, que, CH.draws(8, 11))
    gen.close()
    que.close()


def test_queue_bench_size(monkeypatch):
    """config C4 as benched: 64 evaluations of tests/golden/cellpop_likelihood.xml (500 initial cells,
    ~1,650 cells per evaluation) in one persistent launch, twice (the queue's buffers reused)"""
    path = os.path.join(CH.GOLDEN, "cellpop_likelihood.xml")
    gen, que = _pair(path, CH.PRIOR, monkeypatch)
    x = CH.draws(64, 23)
    assert _same(gen, que, x) > 0
    assert _same(gen, que, x[::-1].copy()) > 0
    gen.close()
    que.close()


def test_queue_stall_is_reported(tmp_path, monkeypatch):
    """the queue's bounded wait: with a 0 ms bound every wavefront that finds nothing ready gives up at
    once, the launch drains and the host reports the stall as an error instead of a result (the 60 s
    default is far beyond any cell's solve)"""
    from bcm3_amd.likelihood import Likelihood
    path = CH.write_likelihood(tmp_path, 40, 256)
    monkeypatch.setenv("BCM3_CP_QUEUE", "1")
    monkeypatch.setenv("BCM3_CP_QUEUE_IDLE_MS", "0")
    ll = Likelihood(path, CH.PRIOR, device=0)
    with pytest.raises(Exception):
        ll.evaluate_batch(CH.draws(4, 11))
    ll.close()
    monkeypatch.delenv("BCM3_CP_QUEUE_IDLE_MS")
    gen, que = _pair(path, CH.PRIOR, monkeypatch)
    _same(gen, que, CH.draws(4, 11))  # (a fresh likelihood with the default bound is unaffected)
    gen.close()
    que.close()
