"""Estimate what a barrier-free (dataflow) PT-MH loop would gain over one global barrier per
iteration: run the C3 PT-MH loop on the CPU (numpy restatement of the device kernels + the
oracle), record each chain's BDF step count per iteration, then compare
  barrier:  sum_k max_c cost(c, k)
  dataflow: T(c, k) = cost(c, k) + max(T(c, k-1), T(partner_k(c), k-1))  (exchange round k pairs
            c with its even/odd neighbour; a chain's mutate k needs only its own and its partner's
            state after mutate k-1).
TEST/ANALYSIS TOOL ONLY (uses the oracle)."""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import oracle as O  # noqa: E402
import helpers as H  # noqa: E402
import ptmh_reference as R  # noqa: E402
import pt_oracle  # noqa: E402
from bcm3_amd.pt import temperature_ladder, exchange_uniform  # noqa: E402
from bcm3_amd.sampler import load_prior  # noqa: E402

C = int(sys.argv[1]) if len(sys.argv) > 1 else 256
K = int(sys.argv[2]) if len(sys.argv) > 2 else 60
seed = 20251016
prob = H.c3_problem(1)
orc = O.Oracle("restated")
pri = load_prior(os.path.join(ROOT, "tests", "golden", "c3_prior.xml"))
kind = np.array([0 if m.kind == "uniform" else 1 for m in pri])
p0 = np.array([m.a if m.kind == "uniform" else m.mu for m in pri])
p1 = np.array([m.b if m.kind == "uniform" else m.sigma for m in pri])
scale = np.where(kind == 0, 0.02 * (p1 - p0), 0.1 * p1)
temps = np.array(temperature_ladder(C))


def ev(x):
    r = orc.popk_eval(prob, x, nthreads=8, want_traj=False)
    return r["logp"], r["stats"][:, 0, 0].astype(float)


values, lprior = R.propose(kind, p0, p1, scale, np.zeros(C), np.zeros((C, len(pri))), 0, seed, (1 << 63) - 1)
llh, _ = ev(values)
lpp = np.where(temps == 0, lprior, lprior + temps * llh)
cost = np.zeros((K, C))
for k in range(K):
    chains = [dict(values=list(values[c]), llh=llh[c], lprior=lprior[c], lpp=lpp[c]) for c in range(C)]
    pt_oracle.exchange_round(chains, list(temps), k, seed, exchange_uniform)
    values = np.array([c["values"] for c in chains])
    llh = np.array([c["llh"] for c in chains]); lprior = np.array([c["lprior"] for c in chains])
    lpp = np.array([c["lpp"] for c in chains])
    prop, lpq = R.propose(kind, p0, p1, scale, temps, values, 0, seed, k)
    lq, st = ev(prop)
    cost[k] = st
    R.accept(temps, prop, lpq, lq, 1.0, values, lprior, llh, lpp, 0, seed, k)
np.save("/tmp/sim/cost.npy", cost)
barrier = cost.max(axis=1).sum()
Tm = np.zeros(C)
for k in range(K):
    start = k % 2
    part = np.arange(C)
    for ci in range(start, C, 2):
        j = (ci + 1) % C
        part[ci], part[j] = j, ci
    Tm = cost[k] + np.maximum(Tm, Tm[part])
print(f"C={C} K={K}: mean steps {cost.mean():.0f}, mean per-iter max {cost.max(axis=1).mean():.0f}")
print(f"barrier makespan {barrier:.0f}  dataflow makespan {Tm.max():.0f}  ideal (mean) {cost.sum(0).max():.0f}")
print(f"gain {barrier / Tm.max():.2f}x")
