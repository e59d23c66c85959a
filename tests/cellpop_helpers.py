"""Shared set-up of the config-C4 (cell_population) tests: the committed synthetic cell-cycle model
(tests/golden/make_cellpop_fixtures.py) with a chosen number of initial / maximum cells."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "oracle"), GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)

import make_cellpop_fixtures as F  # noqa: E402

PRIOR = os.path.join(GOLDEN, "cellpop_prior.xml")


def write_likelihood(directory, num_cells, max_cells, name="cellpop_small_likelihood.xml", **attrs):
    """attrs: data_attrs / experiment_attrs of make_cellpop_fixtures.likelihood_text"""
    path = os.path.join(str(directory), name)
    with open(path, "w") as f:
        f.write(F.likelihood_text(num_cells=num_cells, max_cells=max_cells,
                                  data_file=os.path.join(GOLDEN, "cellpop_data.json"),
                                  model_file=os.path.join(GOLDEN, "cellpop_model.xml"), **attrs))
    return path


def draws(n, seed):
    """the true parameters first, then uniform prior draws"""
    rng = np.random.default_rng(seed)
    lo = np.array([p[1] for p in F.PRIOR])
    hi = np.array([p[2] for p in F.PRIOR])
    x = lo + rng.random((n, len(F.PRIOR))) * (hi - lo)
    x[0] = F.true_values()
    return x


# full_gaussian cell variability (VariabilityDescription.cpp:69-128, 184-212): the two variability
# dimensions correlated through the sampled variable rho1_2 (covar_base_name="rho")
FULL_GAUSSIAN = ('<cell_variability distribution="diagonal_gaussian">',
                 '<cell_variability distribution="full_gaussian" covar_base_name="rho">')
RHO = ("rho1_2", -0.45, 0.45)


def write_full_gaussian(directory, num_cells, max_cells, covar_base_name="rho"):
    """(likelihood, prior) paths: the C4 model with a full_gaussian variability and rho1_2 appended
    to the prior"""
    path = write_likelihood(directory, num_cells, max_cells, name="cellpop_full_likelihood.xml")
    text = open(path).read().replace(FULL_GAUSSIAN[0], FULL_GAUSSIAN[1].replace('"rho"', f'"{covar_base_name}"'))
    with open(path, "w") as f:
        f.write(text)
    prior = os.path.join(str(directory), "cellpop_full_prior.xml")
    rows = open(PRIOR).read().replace("</variableset>",
                                      f'  <variable name="{RHO[0]}" distribution="uniform" lower="{RHO[1]}" '
                                      f'upper="{RHO[2]}"/>\n</variableset>')
    with open(prior, "w") as f:
        f.write(rows)
    return path, prior


def draws_full(n, seed):
    """draws() with rho1_2 appended (the first draw: the true parameters and rho = 0.3)"""
    x = draws(n, seed)
    rng = np.random.default_rng(seed + 1)
    rho = RHO[1] + rng.random(n) * (RHO[2] - RHO[1])
    rho[0] = 0.3
    return np.concatenate([x, rho[:, None]], axis=1)
