"""How often is the GPU bit-identical to the reference's two CVODE builds (oracle/_ref: FMA as the
reference compiles it, and FMA off)? C3 prior draws; prints the fractions of draws whose logp and
whole y1 trajectory are identical, and the same between the two reference builds.
    python tools/bitexact_probe.py [n]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import helpers as H  # noqa: E402
import oracle as O  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
prob = H.c3_problem(1)
vals = H.S.prior_draws(1, n, 20251019)
ctx = H.gpu_context(prob)
g = ctx.eval(vals, detail=True)
ctx.close()
ref = O.Oracle("ref").popk_eval(prob, vals, nthreads=8)
nof = O.Oracle("ref_nofma").popk_eval(prob, vals, nthreads=8)


def same(a_logp, a_traj, b_logp, b_traj):
    lp = (a_logp == b_logp) | (np.isnan(a_logp) & np.isnan(b_logp))
    tr = np.all((a_traj == b_traj) | (np.isnan(a_traj) & np.isnan(b_traj)), axis=-1)
    return float(np.mean(lp)), float(np.mean(tr))


gt = g["traj"][:, 0, 1, :]
print("draws", n)
print("gpu == ref (FMA build)   logp %.4f  y1 %.4f" % same(g["logp"], gt, ref["logp"], ref["traj"][:, 0, 1, :]))
print("gpu == ref_nofma         logp %.4f  y1 %.4f" % same(g["logp"], gt, nof["logp"], nof["traj"][:, 0, 1, :]))
print("ref == ref_nofma         logp %.4f  y1 %.4f" % same(ref["logp"], ref["traj"][:, 0, 1, :], nof["logp"],
                                                           nof["traj"][:, 0, 1, :]))
gs = g["stats"]["nst"][:, 0]
print("steps equal: gpu/ref %.4f gpu/nofma %.4f" % (np.mean(gs == ref["stats"][:, 0, 0]), np.mean(gs == nof["stats"][:, 0, 0])))
