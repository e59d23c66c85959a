"""Time build variants of libbcm3hip.so on the C3 workload (one subprocess per library and round).

    [ROUNDS=3] python tools/variant_timing.py lib1.so [lib2.so ...]
Prints kernel ms at n=256 and 2048 (lanes_per_wave=1, min of 5 launches) and the llh agreement with
the oracle; with ROUNDS > 1 the libraries run interleaved (A B A B ...: the chip's clock drifts
between processes) and a last line gives each library's median over the rounds.
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
    print("RESULT", LIB, n, min(ms), flush=True)
npar = int(os.environ.get("NPAR", "512"))
if npar == 0:
    print(LIB, ' '.join(out), flush=True)
    sys.exit(0)
vals = S.prior_draws(1, npar, 20251019)
g = ctx.eval(vals)
o = O.Oracle('restated').popk_eval(prob, vals, nthreads=8, want_traj=False)
e = parity.llh_err(g[0] if isinstance(g, tuple) else g['logp'], o['logp'])
print(LIB, ' '.join(out), f"llh<=1e-8 {np.mean(e <= 1e-8):.4f} max {np.max(e):.2e}", flush=True)
"""


def main():
    rounds = int(os.environ.get("ROUNDS", "1"))
    res = {}
    for r in range(rounds):
        for lib in sys.argv[1:]:
            env = dict(os.environ, BCM3HIP_LIB=os.path.abspath(lib))
            if r > 0:
                env["NPAR"] = "0"
            code = CHILD.replace("ROOT", repr(ROOT)).replace("LIB", repr(os.path.basename(lib)))
            p = subprocess.run([sys.executable, "-c", code], env=env, check=False, timeout=300,
                               stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
            for line in p.stdout.splitlines():
                if line.startswith("RESULT "):
                    _, name, n, ms = line.split()
                    res.setdefault((name, int(n)), []).append(float(ms))
                elif "amdgpu.ids" not in line:
                    print(line, flush=True)
    if rounds > 1:
        import numpy as np
        for (name, n), v in sorted(res.items(), key=lambda kv: (kv[0][1], kv[0][0])):
            print(f"median over {len(v)} rounds: {name} n={n}: {np.median(v):.3f} ms  ({' '.join(f'{x:.3f}' for x in v)})")


if __name__ == "__main__":
    main()
