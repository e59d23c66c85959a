"""The C4 cell work queue (BCM3_CP_QUEUE=1, cellpop_solver.h cp_queue_kernel) against the generation
launches, in one process on the same draws: per evaluation logp bit for bit, and for every finite
evaluation the cell list (count, records, output values, end states) bit for bit; then the batch time of
both paths, interleaved.

    python tools/c4_queue_check.py [n_evals] [reps]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from bcm3_amd.likelihood import Likelihood  # noqa: E402
from bcm3_amd.sampler import DevicePrior, load_prior  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda", 0)
lik, pri = os.path.join(G, "cellpop_likelihood.xml"), os.path.join(G, "cellpop_prior.xml")
M, NS = 21, 15
# WIDE=1: the C4 workload on the model with six reporter species (NS = 21, one cell per wavefront)
if os.environ.get("WIDE") == "1":
    import tempfile
    sys.path[:0] = [os.path.join(ROOT, "tests"), G, os.path.join(ROOT, "oracle")]
    import cellpop_helpers as CH  # noqa: E402
    lik = CH.write_wide_likelihood(tempfile.mkdtemp(), 500, 2048)
    NS = 21


def make(queue):
    os.environ["BCM3_CP_QUEUE"] = "1" if queue else "0"
    return Likelihood(lik, pri, device=0)


paths = {"generations": make(False), "queue": make(True)}
gen = torch.Generator(device=dev)
gen.manual_seed(20251018)
x = DevicePrior(load_prior(pri), dev).sample(n, gen).contiguous()
stream = torch.cuda.current_stream(dev).cuda_stream
outs = {}
for name, ll in paths.items():
    out = torch.empty(n, dtype=torch.float64, device=dev)
    ll.evaluate_batch_device(n, x.data_ptr(), out.data_ptr(), None, stream)
    torch.cuda.synchronize()
    outs[name] = out.cpu().numpy()
a, b = outs["generations"], outs["queue"]
same = a.view(np.int64) == b.view(np.int64)
fin = np.isfinite(a)
print(f"logp bit-identical {int(same.sum())}/{n} (finite {int(fin.sum())}, queue finite {int(np.isfinite(b).sum())})",
      flush=True)
cells_ok = 0
for i in np.nonzero(fin)[0]:
    ra, va, ya = paths["generations"].cellpop_cells(int(i), M, NS)
    rb, vb, yb = paths["queue"].cellpop_cells(int(i), M, NS)
    ok = len(ra) == len(rb) and ra.tobytes() == rb.tobytes() and va.tobytes() == vb.tobytes() and ya.tobytes() == yb.tobytes()
    cells_ok += ok
    if not ok:
        print(f"  evaluation {i}: cells {len(ra)} vs {len(rb)} differ", flush=True)
print(f"cell lists bit-identical {cells_ok}/{int(fin.sum())} finite evaluations", flush=True)
times = {k: [] for k in paths}
out = torch.empty(n, dtype=torch.float64, device=dev)
for r in range(reps):
    for name, ll in paths.items():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ll.evaluate_batch_device(n, x.data_ptr(), out.data_ptr(), None, stream)
        torch.cuda.synchronize()
        times[name].append(time.perf_counter() - t0)
for name, t in times.items():
    print(f"{name}: median {np.median(t) * 1e3:.2f} ms per batch of {n} ({n / np.median(t):.1f} evals/s), "
          f"all {' '.join(f'{v * 1e3:.2f}' for v in t)}", flush=True)
print(f"speedup {np.median(times['generations']) / np.median(times['queue']):.3f}x", flush=True)
for ll in paths.values():
    ll.close()
