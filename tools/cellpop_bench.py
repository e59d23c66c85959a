"""C4 workload alone (for rocprofv3): 64 chains' proposals of the cell-population likelihood per
launch, repeated. Prints evals/s and cells per eval.

    python tools/cellpop_bench.py [n_evals] [reps]
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
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
lik, pri = os.path.join(G, "cellpop_likelihood.xml"), os.path.join(G, "cellpop_prior.xml")
# CP_SOLVER=DP5: the same C4 experiment with solver_type="DP5" (a temporary copy of the likelihood)
if os.environ.get("CP_SOLVER", "CVODE") == "DP5":
    import tempfile
    text = open(lik).read().replace('<experiment name="exp1" ', '<experiment name="exp1" solver_type="DP5" ')
    text = text.replace('model_file="cellpop_model.xml"', f'model_file="{os.path.join(G, "cellpop_model.xml")}"')
    text = text.replace('data_file="cellpop_data.json"', f'data_file="{os.path.join(G, "cellpop_data.json")}"')
    lik = os.path.join(tempfile.mkdtemp(), "cellpop_dp5.xml")
    with open(lik, "w") as f:
        f.write(text)
ll = Likelihood(lik, pri, device=0)
gen = torch.Generator(device=dev)
gen.manual_seed(20251018)
x = DevicePrior(load_prior(pri), dev).sample(n, gen).contiguous()
out = torch.empty(n, dtype=torch.float64, device=dev)
stream = torch.cuda.current_stream(dev).cuda_stream
ll.evaluate_batch_device(n, x.data_ptr(), out.data_ptr(), None, stream)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(reps):
    ll.evaluate_batch_device(n, x.data_ptr(), out.data_ptr(), None, stream)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / reps
cells = sum(len(ll.cellpop_cells(i, 21, 15)[0]) for i in range(n))
steps = sum(int(ll.cellpop_cells(i, 21, 15)[0]["nsteps"].sum()) for i in range(n))
print(f"n={n}: {dt * 1e3:.2f} ms per batch, {n / dt:.1f} evals/s, {cells / n:.0f} cells/eval, "
      f"{steps / cells:.0f} steps/cell, finite logp {int(torch.isfinite(out).sum())}/{n}", flush=True)
fin = torch.isfinite(out)
print(f"logp checksum {float(out[fin].sum()):.17g}", flush=True)
ll.close()
