"""Diagnostic (not a test): where the cell kernel's time goes. Run with BCM3_CP_PHASES=1 (the
diagnostic build of cellpop_solver.h): per cell, clock64 cycles in the Newton right-hand sides,
difference-quotient Jacobians, LU factorisations, LU solves, whole BDF steps, the whole kernel,
whole Newton iterations and the next step's size / order choice (returned in end_y[0..7]).

    BCM3_CP_PHASES=1 python tools/cellpop_phases.py [n_evals]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bcm3_amd.likelihood import Likelihood  # noqa: E402
from bcm3_amd.sampler import DevicePrior, load_prior  # noqa: E402

assert os.environ.get("BCM3_CP_PHASES") == "1", "set BCM3_CP_PHASES=1"
G = os.path.join(ROOT, "tests", "golden")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
dev = torch.device("cuda", 0)
lik, pri = os.path.join(G, "cellpop_likelihood.xml"), os.path.join(G, "cellpop_prior.xml")
ll = Likelihood(lik, pri, device=0)
gen = torch.Generator(device=dev)
gen.manual_seed(20251018)
x = DevicePrior(load_prior(pri), dev).sample(n, gen).contiguous()
out = torch.empty(n, dtype=torch.float64, device=dev)
ll.evaluate_batch_device(n, x.data_ptr(), out.data_ptr(), None, torch.cuda.current_stream(dev).cuda_stream)
torch.cuda.synchronize()
tot = np.zeros(8)
cells = steps = 0
for i in range(n):
    rec, vals, endy = ll.cellpop_cells(i, 21, 15)
    tot += endy[:, :8].sum(axis=0)
    cells += len(rec)
    steps += int(rec["nsteps"].sum())
names = ["newton rhs", "dq jacobian", "lu factor", "lu solve", "bdf steps (all)", "kernel", "newton (all)",
         "step/order choice"]
print(f"{cells} cells, {steps / cells:.0f} steps/cell; clock64 ticks per cell / per step, share of kernel:")
for k in range(8):
    print(f"  {names[k]:16s} {tot[k] / cells:12.0f} {tot[k] / steps:9.0f}  {tot[k] / tot[5]:6.3f}")
ll.close()
