"""Freeze F_alg, the algorithmic FP64 work of one C3 likelihood evaluation (SURVEY.md §8(d),
BASELINE.md §3), by op-counting in the CPU restatement: oracle/libflops.so is the restated oracle
compiled with every double operation counted (oracle/flopcount.hpp; +, -, *, /, fma, exp, log,
pow, sqrt = 1 flop). The mean over the 512 committed c3_golden.npz prior draws is what bench.py
divides into its roofline.

    make -C oracle libflops.so && python tests/golden/make_falg.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), HERE]
import oracle as O  # noqa: E402
import helpers as H  # noqa: E402


def count(problem, values):
    return O.Oracle("flops").popk_flops(problem, values)


def main():
    z = np.load(os.path.join(HERE, "c3_golden.npz"))
    prob = H.c3_problem(1)
    fl = count(prob, z["values"])
    nst = z["stats"][:, 0, 0].astype(np.float64)
    out = {
        "workload": "C3 pop_pk_trajectory two-compartment, P=1, T=16 (tests/golden/c3_*.xml)",
        "draws": "tests/golden/c3_golden.npz values (512 uniform prior draws)",
        "rule": "+ - * / fma exp log log1p pow sqrt erf = 1 flop each; compare/fabs/floor/copies = 0",
        "flops_per_eval_mean": float(fl.mean()),
        "flops_per_eval_min": int(fl.min()),
        "flops_per_eval_max": int(fl.max()),
        "flops_per_bdf_step": float(fl.sum() / nst.sum()),
        "per_draw": fl.tolist(),
    }
    with open(os.path.join(HERE, "c3_falg.json"), "w") as f:
        json.dump(out, f, indent=1)
    print({k: v for k, v in out.items() if k != "per_draw"})


if __name__ == "__main__":
    main()
