"""Diagnostic (not a test): how many BDF steps run in vec::fast_run (build/var/FC.so, built with
-DBCM3_FASTCOUNT: ncfn counts fast-loop steps, nreinit += 1000 per fast_run entry, nje = clock
ticks/16 inside fast_run, nsetups = clock ticks/16 of the whole trajectory,
nni / nfe = clock ticks/16 in cvode_entry / attempt_loop, approximately: their event counts add in).

    BCM3HIP_LIB=build/var/FC.so python tools/fast_count.py [n]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import numpy as np  # noqa: E402

import helpers as H  # noqa: E402
import synthetic as S  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
prob = H.c3_problem(1)
ctx = H.gpu_context(prob, lanes_per_wave=1)
vals = S.prior_draws(1, n, 7)
ctx.eval(vals, detail=True)
g = ctx.eval(vals, detail=True)
st = g["stats"][:, 0]
nst = st["nst"].astype(float)
fast = st["ncfn"].astype(float)
entries = (st["nreinit"].astype(float) - 14) / 1000
print(f"n={n} kernel {ctx.last_kernel_ms():.3f} ms")
print(f"steps mean {nst.mean():.1f} max {nst.max():.0f}; in-loop fast steps mean {fast.mean():.1f} "
      f"({fast.sum() / nst.sum():.3f}); fast_run entries mean {entries.mean():.1f}; netf {st['netf'].mean():.1f} "
      f"nsetups {st['nsetups'].mean():.1f}")
i = int(np.argmax(nst))
tin = st["nje"].astype(float)
tot = st["nsetups"].astype(float)
print(f"time in fast_run: {tin.sum() / tot.sum():.3f}; per fast step {tin.sum() * 16 / (fast.sum() + entries.sum()):.0f} clk, "
      f"per other step {(tot.sum() - tin.sum()) * 16 / (nst.sum() - fast.sum() - entries.sum()):.0f} clk")
te = st["nni"].astype(float)
ta = st["nfe"].astype(float)
print(f"time shares: fast_run {tin.sum()/tot.sum():.3f} cvode_entry {te.sum()/tot.sum():.3f} attempt_loop {ta.sum()/tot.sum():.3f} rest {(tot.sum()-tin.sum()-te.sum()-ta.sum())/tot.sum():.3f}")
print(f"slowest: steps {nst[i]:.0f} fast {fast[i]:.0f} entries {entries[i]:.0f} netf {st['netf'][i]}")
