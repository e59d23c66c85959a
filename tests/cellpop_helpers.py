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


# The cell-population parity bar (round 6: the measured envelope instead of round 5's flat 2e-4).
# Measured on MI355X over every C4-family GPU test (profiles/r06b_cellpop_parity.jsonl, ~330 finite
# draws): median deviations 1e-16 .. 1.6e-7 relative; the largest, 3e-5, on draws where the
# reference's own FMA / no-FMA builds differ by as much (a division one step earlier or later); where
# the two builds agree the GPU stays within 3.1e-6 (a step flip of its own in a dividing population).
# Per draw: |logp - oracle| <= max(LOGP_REL (1 + |oracle|), SPREAD_FACTOR x the two reference builds'
# own difference on that draw), with the -inf pattern identical.
LOGP_REL = 1e-5
SPREAD_FACTOR = 10.0


def logp_bar(r, r_nofma=None):
    b = LOGP_REL * (1.0 + abs(r))
    if r_nofma is not None and np.isfinite(r_nofma):
        b = max(b, SPREAD_FACTOR * abs(r_nofma - r))
    return b


def check_logp(lp, status, ref, ref_nofma=None, name=""):
    """Assert the GPU logp of every draw inside the bar (logp_bar) and the -inf / status pattern
    identical (status None: not checked); log the measured deviations (tests/parity.py
    log_summary). Returns (dev, spread): the relative deviations of the finite draws and, with
    ref_nofma, the reference's own."""
    import math
    import parity
    dev, spread, worst = [], [], 0.0
    for i in range(len(ref)):
        r = ref[i]
        if r == -math.inf:
            assert lp[i] == -math.inf and (status is None or status[i] == 1), (name, i, lp[i])
            continue
        rn = None if ref_nofma is None else ref_nofma[i]
        assert status is None or status[i] == 0, (name, i, status[i])
        assert np.isfinite(lp[i]), (name, i, lp[i], r)
        d = abs(lp[i] - r)
        dev.append(d / (1.0 + abs(r)))
        if rn is not None:
            spread.append(abs(rn - r) / (1.0 + abs(r)))
        worst = max(worst, d / logp_bar(r, rn))
    rec = {"cellpop_logp": name, "finite": len(dev), "of": len(ref),
           "logp_dev_median": float(np.median(dev)) if dev else None,
           "logp_dev_max": float(np.max(dev)) if dev else None,
           "ref_fma_spread_median": float(np.median(spread)) if spread else None,
           "ref_fma_spread_max": float(np.max(spread)) if spread else None,
           "worst_fraction_of_bar": worst}
    parity.log_summary(rec, n=len(ref))
    assert worst <= 1.0, rec
    return dev, spread


def write_wide_model(directory, extra=6):
    """the C4 model with `extra` reporter species appended (a chain driven by CycB, each decaying,
    nothing feeding back): NS = 15 + extra ODE species, past the 16-lane row of the four-cell build, so
    the cell kernel takes its one-cell-per-wavefront form (cellpop_solver.h ROW = 64)"""
    text = open(os.path.join(GOLDEN, "cellpop_model.xml")).read()
    sp = "".join(f'      <species id="X{i}" name="X{i}" compartment="cell" initialAmount="0.{i}"/>\n'
                 for i in range(1, extra + 1))
    text = text.replace("    </listOfSpecies>", sp + "    </listOfSpecies>", 1)
    mm = 'xmlns="http://www.w3.org/1998/Math/MathML"'
    rx = []
    for i in range(1, extra + 1):
        src = "CycB" if i == 1 else f"X{i - 1}"
        rx.append(f'      <reaction id="rx{i}_make" reversible="false">\n'
                  f'        <listOfProducts><speciesReference species="X{i}" stoichiometry="1"/></listOfProducts>\n'
                  f'        <listOfModifiers><modifierSpeciesReference species="{src}"/></listOfModifiers>\n'
                  f'        <kineticLaw><math {mm}><apply><times/><cn> 0.{i + 2} </cn><ci> {src} </ci></apply></math></kineticLaw>\n'
                  f'      </reaction>\n'
                  f'      <reaction id="rx{i}_decay" reversible="false">\n'
                  f'        <listOfReactants><speciesReference species="X{i}"/></listOfReactants>\n'
                  f'        <kineticLaw><math {mm}><apply><times/><cn> 0.5 </cn><ci> X{i} </ci></apply></math></kineticLaw>\n'
                  f'      </reaction>\n')
    text = text.replace("    </listOfReactions>", "".join(rx) + "    </listOfReactions>", 1)
    path = os.path.join(str(directory), "cellpop_model_wide.xml")
    with open(path, "w") as f:
        f.write(text)
    return path


def write_wide_likelihood(directory, num_cells, max_cells, extra=6, **attrs):
    """a likelihood on write_wide_model's model (the C4 data and variabilities)"""
    path = os.path.join(str(directory), "cellpop_wide_likelihood.xml")
    with open(path, "w") as f:
        f.write(F.likelihood_text(num_cells=num_cells, max_cells=max_cells,
                                  data_file=os.path.join(GOLDEN, "cellpop_data.json"),
                                  model_file=write_wide_model(directory, extra), **attrs))
    return path
