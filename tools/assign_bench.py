"""Timing of the cell-matching routine on the GPU (bcm3hip_assign_cells: the time-course / time-points
likelihoods' observed-to-simulated assignment, cellpop_kernels.hip hg_match) for growing cell counts.

Matrices shaped like DataLikelihoodTimeCourse's: observed cell i = a simulated cell's trajectory plus
noise over 21 time points, L[i, j] = the normal log-likelihood of cell j's trajectory for cell i's data.

    python tools/assign_bench.py [R ...]        -> one JSON line per R
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def matrices(problems, R, T=21, sd=0.05, seed=0):
    rng = np.random.default_rng(seed + R)
    out = np.empty((problems, R, R))
    for p in range(problems):
        x = np.cumsum(rng.normal(0.0, 0.1, (R, T)), axis=1) + rng.normal(0, 0.3, (R, 1))
        y = x[rng.permutation(R)] + rng.normal(0.0, sd, (R, T))
        d = y[:, None, :] - x[None, :, :]
        out[p] = (-np.log(sd) - 0.91893853320467274 - d * d / (2 * sd * sd)).sum(axis=2)
    return out


def main():
    import torch
    from bcm3_amd import _hip
    Rs = [int(a) for a in sys.argv[1:]] or [16, 64, 128, 256, 512]
    for R in Rs:
        for problems in (1, 64):
            L = torch.tensor(matrices(problems, R), device="cuda")
            _hip.assign_cells(L)  # warm-up (module load)
            reps = 3
            t0 = time.perf_counter()
            for _ in range(reps):
                m, s, ok = _hip.assign_cells(L)
            dt = (time.perf_counter() - t0) / reps
            print(json.dumps({"R": R, "problems": problems, "ms_per_batch": dt * 1e3,
                              "ok": int(ok.sum()), "matched_identity_frac": None}), flush=True)


if __name__ == "__main__":
    main()
