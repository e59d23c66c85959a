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
