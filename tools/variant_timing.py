"""Time build variants of libbcm3hip.so on the C3 workload (one subprocess per library).

    python tools/variant_timing.py lib1.so [lib2.so ...]
Prints kernel ms at n=256 lanes_per_wave=1 (min of 5) and the llh agreement with the oracle.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys
sys.path[:0] = [ROOT, os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]
import numpy as np, torch
import helpers as H, synthetic as S, oracle as O, parity
from bcm3_amd import _hip
prob = H.c3_problem(1)
ctx = H.gpu_context(prob, lanes_per_wave=1)
out = []
for n in (256, 2048):
    v = torch.tensor(S.prior_draws(1, n, 7), device='cuda', dtype=torch.float64)
    lp = torch.empty(n, device='cuda', dtype=torch.float64)
    ms = []
    for _ in range(5):
        ctx.eval_device(n, v.data_ptr(), lp.data_ptr(), None, None)
        ms.append(ctx.last_kernel_ms())
    out.append(f"n={n}: {min(ms):.3f} ms")
vals = S.prior_draws(1, int(os.environ.get("NPAR", "512")), 20251019)
g = ctx.eval(vals)
o = O.Oracle('restated').popk_eval(prob, vals, nthreads=8, want_traj=False)
e = parity.llh_err(g[0] if isinstance(g, tuple) else g['logp'], o['logp'])
print(LIB, ' '.join(out), f"llh<=1e-8 {np.mean(e <= 1e-8):.4f} max {np.max(e):.2e}", flush=True)
"""


def main():
    for lib in sys.argv[1:]:
        env = dict(os.environ, BCM3HIP_LIB=os.path.abspath(lib))
        code = CHILD.replace("ROOT", repr(ROOT)).replace("LIB", repr(os.path.basename(lib)))
        subprocess.run([sys.executable, "-c", code], env=env, check=False, timeout=300)


if __name__ == "__main__":
    main()
