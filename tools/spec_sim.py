"""Speculative evaluation, measured before it is built (VERDICT r02 "Next round" 5).

The C3 launch holds 256 trajectories on 1,024 SIMDs and lasts as long as the slowest of them. If
iteration r's launch also evaluated every proposal iteration r+1 can make -- for each chain, one per
outcome of its own accept at r and of its exchange partner's (the state after exchange r+1 is one of
old_i, prop_i, old_p, prop_p: 4 candidates, T = 0 chains 1) -- the accept of r+1 would need no launch
of its own: two iterations per launch. Counter-based random numbers make the candidates' proposals
exactly the ones the sequential sampler would make, so only committed evaluations count.

This script measures the kernel time of one launch of n = k x 256 realistic C3 proposals (chain
states of a running C++ sampler over consecutive iterations) for k = 1..8, with one trajectory per
wavefront (lanes_per_wave 1) and with the library's automatic choice, and prints the committed
evals/s that a 1 + 4 speculative launch would give against the plain loop.

    python tools/spec_sim.py [iterations_warmup]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from bcm3_amd import _hip  # noqa: E402
from bcm3_amd.likelihood import Likelihood  # noqa: E402
from bcm3_amd.ptmh import PTMHNative  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
LIK, PRI = os.path.join(G, "c3_likelihood.xml"), os.path.join(G, "c3_prior.xml")


def kernel_ms(ll, x, lpw, reps=5):
    n = len(x)
    xd = torch.tensor(x, dtype=torch.float64, device="cuda")
    out = torch.empty(n, dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    ll.set_option(_hip.OPT_LANES_PER_WAVE, lpw)
    ll.evaluate_batch_device(n, xd.data_ptr(), out.data_ptr(), None, stream)
    torch.cuda.synchronize()
    best = []
    for _ in range(reps):
        ll.set_option(_hip.OPT_TIMING_LOG, 1)
        ll.evaluate_batch_device(n, xd.data_ptr(), out.data_ptr(), None, stream)
        torch.cuda.synchronize()
        tt, nl, _ = ll.kernel_time_log()
        ll.set_option(_hip.OPT_TIMING_LOG, 0)
        best.append(tt / nl)
    return float(np.median(best))


def main():
    warm = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    ll = Likelihood(LIK, PRI, device=0)
    s = PTMHNative(ll, PRI, 256, seed=20251016, proposal="gaussian_mixture")
    s.iterate(warm)
    states = []
    for _ in range(8):
        s.iterate(1)
        states.append(s.state()["values"].copy())
    s.close()
    res = {}
    for k in range(1, 9):
        x = np.concatenate(states[:k])
        res[k] = {lpw: kernel_ms(ll, x, lpw) for lpw in (1, 0)}
        print(f"n={256 * k:5d}  lpw=1 {res[k][1]:.3f} ms   auto {res[k][0]:.3f} ms", flush=True)
    # launch order and residency: one wavefront per SIMD (LDS reservation: 4 one-wave workgroups per
    # CU), trajectories dispatched longest first (predicted by their own step counts here, by the
    # step count of the state they start from in the sampler) -- the workgroups beyond 1,024 wait
    # for the first SIMDs to free up instead of sharing one
    ctx = _hip.Context.from_popk_model(ll.popk_model(), 0)
    for k in (4, 5, 6, 7, 8):
        x = np.concatenate(states[:k])
        nst = ctx.eval(x, detail=True)["stats"]["nst"].reshape(len(x), -1).sum(axis=1)
        order = np.argsort(-nst, kind="stable")
        xs = np.ascontiguousarray(x[order])
        row = []
        for lds in (0, 40960):
            ll.set_option(_hip.OPT_BLOCK_LDS, lds)
            row.append((lds, kernel_ms(ll, x, 1), kernel_ms(ll, xs, 1)))
        ll.set_option(_hip.OPT_BLOCK_LDS, 0)
        print(f"n={256 * k:5d} steps max {nst.max()} mean {nst.mean():.0f}: " +
              "; ".join(f"lds {l}: as is {a:.3f} ms, longest first {b:.3f} ms" for l, a, b in row), flush=True)
        res[k]["ordered"] = min(b for _, _, b in row)
    ctx.close()
    # the sampler's own speculative launches: kernel time per launch and how well the dispatch order
    # (predicted from the chains' previous solves) follows the real solve lengths
    s = PTMHNative(ll, PRI, 256, seed=20251016, proposal="gaussian_mixture")
    s.iterate(warm)
    ll.set_option(_hip.OPT_TIMING_LOG, 1)
    s.iterate(20)
    s.synchronize()
    tt, nl, mx = ll.kernel_time_log()
    ll.set_option(_hip.OPT_TIMING_LOG, 0)
    src, steps = s.spec_batch_info()
    s.close()
    n = len(steps)
    # the batch layout (ptmh_spec_batch_kernel): predicted rank r -> position; invert it with the
    # device's SIMD count R (positions p and p + R share a SIMD)
    R = _hip.lib().bcm3hip_current_device_simds() if hasattr(_hip.lib(), "bcm3hip_current_device_simds") else 0
    S2 = n - R if 0 < R < n <= 2 * R else 0
    L = n - 2 * S2
    p = np.arange(n)
    pred_rank = np.where(p < S2, L + p, np.where(p < R, p - S2, L + S2 + (p - R))) if S2 else p
    steps = steps[np.argsort(pred_rank)]  # in predicted order, longest first
    rank = np.argsort(np.argsort(-steps, kind="stable"), kind="stable")  # 0 = longest
    top = np.argsort(-steps, kind="stable")[:64]
    print(f"sampler: {nl} launches for 20 iterations, {tt / nl:.3f} ms per launch (max {mx:.3f}); last batch "
          f"{n} entries, steps max {steps.max()} mean {steps.mean():.0f}; the 64 longest solves sit at predicted "
          f"ranks median {np.median(top):.0f} (max {top.max()}); rank correlation "
          f"{np.corrcoef(np.arange(n), rank)[0, 1]:.2f}", flush=True)
    base = res[1][1]
    for k, label in ((5, "1 + 4 candidates"), (7, "1 + 6 candidates")):
        t = min(res[k].values())
        print(f"{label}: launch {t:.3f} ms for 2 committed iterations vs 2 x {base:.3f} ms -> "
              f"{2 * base / t:.2f}x committed evals/s (kernel time only)")
    ll.close()


if __name__ == "__main__":
    main()
