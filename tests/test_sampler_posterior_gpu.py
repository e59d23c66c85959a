"""The whole device PT-MH loop (the C++ sampler over the HIP kernels, bcm3_ptmh_*) on the
reference's example problems, as a user runs them: config C1 (examples/banana, 8 chains) and C2
(examples/multimodal_circular_ridge, bimodal), default gaussian_mixture proposal with adaptation,
samples read back from the sampler's output file (SampleHandlerNetCDF schema).

Both targets are 2-D, so their exact posterior moments come from integrating prior x likelihood on
a fine grid (TestLikelihoodBanana.cpp:42-55, TestLikelihoodCircular.cpp:42-53 restated in numpy).
Runs are seeded and bit-reproducible; the tolerances are several Monte-Carlo standard errors of
the retained T = 1 samples."""
import os

import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu


def _run(name, chains, samples, seed, tmp_path, **kw):
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.ptmh import PTMHNative
    from scipy.io import netcdf_file
    lik, pri = (os.path.join(H.GOLDEN, f"{name}_likelihood.xml"), os.path.join(H.GOLDEN, f"{name}_prior.xml"))
    ll = Likelihood(lik, pri, device=0)
    s = PTMHNative(ll, pri, chains, seed=seed, **kw)
    out = str(tmp_path / f"{name}.nc")
    s.set_output(out, samples, flush_every=256)
    s.run(samples)
    c = s.counters()
    s.close()
    with netcdf_file(out, "r", mmap=False) as f:
        x = np.array(f.variables["samples.variable_values"][:])
        temps = np.array(f.variables["samples.temperature"][:])
    assert temps[-1] == 1.0
    return x[:, -1, :], c


def _moments(logp, g1, g2):
    w = np.exp(logp - logp.max())
    w /= w.sum()
    X1, X2 = np.meshgrid(g1, g2, indexing="ij")
    m1, m2 = (w * X1).sum(), (w * X2).sum()
    return m1, m2, np.sqrt((w * (X1 - m1) ** 2).sum()), np.sqrt((w * (X2 - m2) ** 2).sum())


def test_c1_banana_posterior(tmp_path):
    x, c = _run("banana", 8, 8000, 21, tmp_path, adapt_proposal_samples=500, adapt_proposal_times=2)
    assert c["adaptations_done"] == 2 and c["samples_done"] == 8000
    assert 0.05 < c["accepted_mutate"] / c["attempted_mutate"] < 0.9
    post = x[2000:]
    # prior U(-6, 4) x U(-6, 20); x1 ~ N(0, 2), x2 | x1 ~ N(4 x1 + (1 - x1)^2, 1)
    g1, g2 = np.linspace(-6, 4, 1201), np.linspace(-6, 20, 3001)
    X1, X2 = np.meshgrid(g1, g2, indexing="ij")
    logp = -X1 ** 2 / 8.0 - (X2 - (4 * X1 + (1 - X1) ** 2)) ** 2 / 2.0
    m1, m2, s1, s2 = _moments(logp, g1, g2)
    assert abs(post[:, 0].mean() - m1) < 0.25, (post[:, 0].mean(), m1)
    assert abs(post[:, 1].mean() - m2) < 1.0, (post[:, 1].mean(), m2)
    assert abs(post[:, 0].std() - s1) < 0.25, (post[:, 0].std(), s1)
    assert abs(post[:, 1].std() - s2) < 1.0, (post[:, 1].std(), s2)
    assert np.all((post[:, 0] >= -6) & (post[:, 0] <= 4) & (post[:, 1] >= -6) & (post[:, 1] <= 20))


def test_c2_circular_ridge_visits_both_modes(tmp_path):
    x, c = _run("circular", 8, 8000, 5, tmp_path, adapt_proposal_samples=500, adapt_proposal_times=2)
    post = x[2000:]
    # two rings of radius 2 (width 0.1) around (-3.5, 0) and (3.5, 0): symmetric, so half of the
    # mass on each side; every sample close to a ring
    right = post[:, 0] > 0
    assert 0.25 < right.mean() < 0.75, right.mean()
    r = np.where(right, np.hypot(post[:, 0] - 3.5, post[:, 1]), np.hypot(post[:, 0] + 3.5, post[:, 1]))
    assert abs(r.mean() - 2.0) < 0.05 and r.std() < 0.2, (r.mean(), r.std())
    # the ring's angle is uniform: the mean of cos / sin of the angle on each side is near 0
    ang = np.where(right, np.arctan2(post[:, 1], post[:, 0] - 3.5), np.arctan2(post[:, 1], post[:, 0] + 3.5))
    assert abs(np.cos(ang).mean()) < 0.25 and abs(np.sin(ang).mean()) < 0.25
