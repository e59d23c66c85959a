"""Diagnostic probe (not a test): GPU vs oracle parity summary + launch-shape timings.

    python tools/popk_probe.py [n_parity] [--timing]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]

import numpy as np  # noqa: E402

import helpers as H  # noqa: E402
import oracle as O  # noqa: E402
import parity  # noqa: E402
import synthetic as S  # noqa: E402
from bcm3_amd import _hip  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 2048
    prob = H.c3_problem(1)
    ctx = H.gpu_context(prob)
    vals = S.prior_draws(1, n, 20251016)
    t = time.time()
    g = ctx.eval(vals, detail=True)
    print(f"gpu detail eval n={n}: {time.time()-t:.3f}s")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "probe_gpu.npz"), values=vals, logp=g["logp"],
                        status=g["status"], traj=g["traj"], nst=g["stats"]["nst"])
    for which in ("restated", "ref"):
        t = time.time()
        o = O.Oracle(which).popk_eval(prob, vals, nthreads=8)
        print(f"oracle {which}: {time.time()-t:.3f}s")
        te = parity.y1_rel_err(g["traj"][:, 0, 1], o["traj"][:, 0, 1], prob.atol)
        le = parity.llh_err(g["logp"], o["logp"])
        s = parity.summarize(te, le, g["stats"]["nst"][:, 0], o["stats"][:, 0, 0])
        print(which, s)
        print("  fail gpu/oracle:", np.mean(g["status"] != 0), np.mean(o["ok"][:, 0] == 0),
              "steps mean gpu/oracle", g["stats"]["nst"].mean(), o["stats"][:, 0, 0].mean())
        bad = np.nonzero(g["stats"]["nst"][:, 0] != o["stats"][:, 0, 0])[0][:10]
        print("  first step mismatches:", bad, g["stats"]["nst"][bad, 0], o["stats"][bad, 0, 0])
    if "--timing" in sys.argv:
        import torch
        for nn, P in ((256, 1), (4096, 1), (16384, 1)):
            v = torch.tensor(S.prior_draws(1, nn, 7), device="cuda", dtype=torch.float64)
            lp = torch.empty(nn, device="cuda", dtype=torch.float64)
            for lpw in (1, 2, 4, 8, 16, 64):
                ctx.set_option(_hip.OPT_LANES_PER_WAVE, lpw)
                ms = []
                for rep in range(3):
                    ctx.eval_device(nn, v.data_ptr(), lp.data_ptr(), None, None)
                    ms.append(ctx.last_kernel_ms())
                print(f"n={nn} lpw={lpw}: kernel ms {min(ms):.3f}  evals/s {nn/min(ms)*1e3:.0f}")
        ctx.set_option(_hip.OPT_LANES_PER_WAVE, 64)


if __name__ == "__main__":
    main()
