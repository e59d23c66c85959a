"""Launch the PopPK kernel a few times for rocprofv3 (kernel trace / PMC passes).

    python tools/prof_popk.py N LANES_PER_WAVE REPS
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]

import numpy as np  # noqa: E402

import helpers as H  # noqa: E402
import synthetic as S  # noqa: E402
from bcm3_amd import _hip  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    lpw = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    import torch
    prob = H.c3_problem(1)
    ctx = H.gpu_context(prob, lanes_per_wave=lpw)
    v = torch.tensor(S.prior_draws(1, n, 7), device="cuda", dtype=torch.float64)
    lp = torch.empty(n, device="cuda", dtype=torch.float64)
    ms = []
    for _ in range(reps):
        ctx.eval_device(n, v.data_ptr(), lp.data_ptr(), None, None)
        ms.append(ctx.last_kernel_ms())
    if os.environ.get("PROF_NO_DETAIL"):  # (C3-only development libraries have no counting kernel)
        print(f"n={n} lpw={lpw} kernel ms min {min(ms):.3f} med {np.median(ms):.3f}")
        return
    # steps of the slowest lane, for per-step cost
    g = ctx.eval(S.prior_draws(1, n, 7), detail=True)
    print(f"n={n} lpw={lpw} kernel ms min {min(ms):.3f} med {np.median(ms):.3f}; steps max {g['stats']['nst'].max()} "
          f"mean {g['stats']['nst'].mean():.1f}; total steps {g['stats']['nst'].sum()}")


if __name__ == "__main__":
    main()
