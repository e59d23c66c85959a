"""One rank of a sharded C++ PT-MH sampler in its own OS process (tests/test_ptmh_multiprocess_gpu.py).

    python tests/workers/ptmh_rank.py OUT_NPZ SOCKET_DIR RANK WORLD CHAINS SEED STEPS SPECULATE [OUTPUT_NC]

The ranks exchange the slice-boundary records over BCM3_PTMH_TRANSPORT_SOCKET (Unix domain sockets
under SOCKET_DIR); the final chain state, counters and whether speculative pairs ran go to OUT_NPZ.
With OUTPUT_NC every rank calls set_output (one sample per iteration, flushed every 7): netCDF-4
written by rank 0 from all ranks' rows when $BCM3_LIBNETCDF loads, the shared classic file otherwise."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    out, sock, rank, world, C, seed, steps, spec = sys.argv[1:9]
    out_nc = sys.argv[9] if len(sys.argv) > 9 else None
    rank, world, C, seed, steps, spec = int(rank), int(world), int(C), int(seed), int(steps), int(spec)
    from bcm3_amd.likelihood import Likelihood
    from bcm3_amd.ptmh import TRANSPORT_SOCKET, PTMHNative
    g = os.path.join(ROOT, "tests", "golden")
    lik, pri = os.path.join(g, "c3_likelihood.xml"), os.path.join(g, "c3_prior.xml")
    ll = Likelihood(lik, pri, device=0)
    s = PTMHNative(ll, pri, C, rank=rank, world=world, seed=seed, transport=TRANSPORT_SOCKET, socket_dir=sock,
                   speculate=spec, adapt_proposal_samples=25, adapt_proposal_times=1)
    if out_nc:
        s.set_output(out_nc, steps, flush_every=7)
    s.iterate(steps)
    s.synchronize()
    if out_nc:
        s.flush_output()
    st, cnt = s.state(), s.counters()
    info = s.spec_batch_info()
    s.close()
    np.savez(out, values=st["values"], llh=st["llh"], lprior=st["lprior"], lpp=st["lpp"],
             accepted_mutate=cnt["accepted_mutate"], accepted_exchange=cnt["accepted_exchange"],
             speculated=info is not None)


if __name__ == "__main__":
    main()
