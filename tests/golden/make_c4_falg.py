"""F_alg of config C4 (the cell-population likelihood, tests/golden/cellpop_likelihood.xml): FP64
operations of one evaluation, from an operation-count model of the reference's per-cell CVODE BDF +
PartialPivLU solve driven by the reference solver's own counters (oracle/_ref/libcellpopref.so:
CVodeGetNumSteps / RhsEvals / NonlinSolvIters / LinSolvSetups / JacEvals / ErrTestFails per cell), over
prior draws of the benchmark problem. Writes tests/golden/c4_falg.json (bench.py's C4 roofline line).

Counted as one operation each: +, -, *, /, and the comparisons-free arithmetic of the generated
right-hand side (its text, tests: oracle/sbml_codegen.py) with the reference's helper functions
(hill_function_fixedn4: 6, hill_function_fixedn16: 10, synthcap: 5 -- their bodies in
SolverCodeGenerator.cpp's emitted helpers). Per event of the solve (N species, q ~ 3):
  RHS evaluation (nfe)             F_rhs
  difference-quotient Jacobian     N F_rhs + N (2N + 8)             (cvLsDQJac: one RHS per column)
  linear-solver setup (nsetups)    2N^3/3 + 2N^2                    (I - gamma J, partial-pivot LU)
  Newton iteration (nni)           2N^2 + 10N                       (residual, LU solve, update, WRMS)
  step (nsteps)                    20N + 70                          (predict, ewt, complete, step control)
  error-test failure (netf)        6N                               (restore the Nordsieck array)
This is a model, not an instrumented count (the reference's CVODE is C and is not rebuilt with a
counting type); it fixes the order of magnitude of the FP64 roofline fraction.

    python tests/golden/make_c4_falg.py
"""
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), HERE]

import cellpop as CP  # noqa: E402
import cellpop_helpers as CH  # noqa: E402

HELPER_OPS = {"hill_function_fixedn4": 6, "hill_function_fixedn16": 10, "synthcap": 5}


def rhs_ops(body: str) -> int:
    ops = 0
    for line in body.splitlines():
        if "=" not in line:
            continue
        rhs = line.split("=", 1)[1]
        for name, cost in HELPER_OPS.items():
            ops += cost * rhs.count(name + "(")
        rhs = re.sub(r"\[[^\]]*\]", "", rhs)  # array indices are not arithmetic
        rhs = re.sub(r"[0-9]\.[0-9]*e[-+][0-9]+", "1", rhs)  # exponents of literals
        n = rhs.count("*") + rhs.count("/")
        terms = re.findall(r"[-+]", rhs.strip().lstrip("+"))
        ops += n + len(terms)
    return ops


def main(n_draws=16, seed=23):
    path = os.path.join(HERE, "cellpop_likelihood.xml")
    prob = CP.load_problem(path, CH.PRIOR)
    e = prob["experiments"][0]
    N = len(e["model"].ode)
    f_rhs = rhs_ops(e["derivative_body"])
    x = CH.draws(n_draws, seed)
    ref = CP.simulate(prob, x, nthreads=8)
    tot, cells, steps, fin = [], [], [], 0
    for i in range(n_draws):
        det = ref["detail"][i]
        f = 0.0
        st = 0
        for c in det["cells"]:
            if "stats" not in c:  # queued but never simulated (the evaluation failed first)
                continue
            s = c["stats"]
            f += (s["nfe"] * f_rhs + s["nje"] * (N * f_rhs + N * (2 * N + 8)) +
                  s["nsetups"] * (2 * N ** 3 / 3 + 2 * N * N) + s["nni"] * (2 * N * N + 10 * N) +
                  c["nsteps"] * (20 * N + 70) + s["netf"] * 6 * N)
            st += c["nsteps"]
        tot.append(f)
        cells.append(sum(1 for c in det["cells"] if "stats" in c))
        steps.append(st)
        fin += int(np.isfinite(ref["logp"][i]))
    out = {"flops_per_eval_mean": float(np.mean(tot)), "flops_per_cell_step": float(np.sum(tot) / np.sum(steps)),
           "cells_per_eval_mean": float(np.mean(cells)), "steps_per_eval_mean": float(np.mean(steps)),
           "f_rhs": f_rhs, "species": N, "draws": n_draws, "seed": seed, "finite_draws": fin,
           "method": "operation-count model over the reference CVODE's per-cell counters (make_c4_falg.py)"}
    with open(os.path.join(HERE, "c4_falg.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(out)


if __name__ == "__main__":
    main()
