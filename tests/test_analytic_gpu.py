"""GPU parity of the analytic likelihoods (configs C1/C2) against the golden fixtures."""
import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def test_banana_golden(golden_dir):
    from bcm3_amd import _hip
    g = np.load(os.path.join(golden_dir, "analytic_golden.npz"))
    ctx = _hip.Context.analytic(_hip.ANALYTIC_BANANA, 2, 2.0, 1.0)
    lp, st = ctx.eval(g["banana_values"])
    # PdfNormal's rsqrtss + 2 Newton steps (MathFunctions.h:35-48) is CPU-vendor dependent
    err = np.abs(lp - g["banana_logp"]) / (1 + np.abs(g["banana_logp"]))
    assert np.max(err) <= 1e-12
    assert np.all(st == 0)
    ctx.close()


def test_circular_golden(golden_dir):
    from bcm3_amd import _hip
    g = np.load(os.path.join(golden_dir, "analytic_golden.npz"))
    ctx = _hip.Context.analytic(_hip.ANALYTIC_CIRCULAR, 2, 2.0, 3.5, 0.1)
    lp, _ = ctx.eval(g["circular_values"])
    err = np.abs(lp - g["circular_logp"]) / (1 + np.abs(g["circular_logp"]))
    assert np.max(err) <= 1e-14
    ctx.close()


@pytest.mark.parametrize("d", [3, 7])
def test_higher_dimensions_vs_oracle(d):
    from bcm3_amd import _hip
    rng = np.random.default_rng(d)
    v = rng.uniform(-5, 5, (4096, d))
    o = O.Oracle("restated")
    for kind, args, ref in ((_hip.ANALYTIC_BANANA, (2.0, 1.0, 0.0), o.banana(v, d, 2.0, 1.0)),
                            (_hip.ANALYTIC_CIRCULAR, (2.0, 3.5, 0.1), o.circular(v, d, 2.0, 3.5, 0.1))):
        ctx = _hip.Context.analytic(kind, d, *args)
        lp, _ = ctx.eval(v)
        fin = np.isfinite(ref)
        assert np.array_equal(np.isfinite(lp), fin)
        err = np.abs(lp[fin] - ref[fin]) / (1 + np.abs(ref[fin]))
        assert np.max(err) <= 1e-12
        ctx.close()
