"""Run-to-run determinism of the C4 batch: the bench's 64 draws evaluated REPS times in one process;
prints how many logp entries differ between repetitions (and from a saved earlier run, argv[2]),
and saves this run's first repetition to argv[1] (.npy).

    python tools/c4_determinism.py out.npy [earlier.npy]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bcm3_amd.likelihood import Likelihood  # noqa: E402
from bcm3_amd.sampler import DevicePrior, load_prior  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
reps = int(os.environ.get("REPS", "4"))
dev = torch.device("cuda", 0)
lik, pri = os.path.join(G, "cellpop_likelihood.xml"), os.path.join(G, "cellpop_prior.xml")
ll = Likelihood(lik, pri, device=0)
gen = torch.Generator(device=dev)
gen.manual_seed(20251018)
x = DevicePrior(load_prior(pri), dev).sample(64, gen).contiguous()
xh = x.cpu().numpy()
runs = []
for r in range(reps):
    lp, st = ll.evaluate_batch(xh)
    runs.append(lp.copy())
    cells = [len(ll.cellpop_cells(i, 21, 15)[0]) for i in range(64)]
    print(f"rep {r}: finite {int(np.isfinite(lp).sum())}, cells {sum(cells)}, "
          f"checksum {float(lp[np.isfinite(lp)].sum()):.17g}", flush=True)
base = runs[0]
for r in range(1, reps):
    d = ~((runs[r] == base) | (np.isnan(runs[r]) & np.isnan(base)))
    print(f"rep {r} vs rep 0: {int(d.sum())} entries differ {np.flatnonzero(d)[:16].tolist()}", flush=True)
np.save(sys.argv[1], base)
if len(sys.argv) > 2 and os.path.exists(sys.argv[2]):
    prev = np.load(sys.argv[2])
    d = ~((prev == base) | (np.isnan(prev) & np.isnan(base)))
    print(f"this process vs {os.path.basename(sys.argv[2])}: {int(d.sum())} entries differ "
          f"{np.flatnonzero(d)[:16].tolist()} max |d| {float(np.nanmax(np.abs(np.where(d, prev - base, 0.0)))):.3g}",
          flush=True)
ll.close()
