"""Differential check of a compiler flag (ADVICE r04 medium / VERDICT r04 item 4): every PK model x
dosing rule of tests/test_popk_gpu.py::test_all_models_and_dosing_rules, in all three solver forms
(lanes_per_wave 1 with vector or scalar state, 64), evaluated with two library builds; logp, every
interpolated output and every solver counter must agree bit for bit.

    python tools/flag_diff.py libA.so libB.so            (each build runs in its own process)
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PK = ["one", "two", "one_biphasic_uptake", "two_biphasic_uptake", "one_transit", "two_transit"]
RULES = ["daily", "intermittent1", "intermittent2", "intermittent3", "skipped", "dose_change", "interval12"]

CHILD = r"""
import os, sys
sys.path[:0] = [ROOT, os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]
import numpy as np
import helpers as H
out = {}
for pk in PK:
    for rule in RULES:
        kw = dict(P=2, T_days=6)
        if rule.startswith('intermittent'):
            kw['intermittent'] = int(rule[-1]); kw['T_days'] = 10
        elif rule == 'skipped':
            kw['skipped'] = (2, 3)
        elif rule == 'dose_change':
            kw['dose_change'] = (500.0, 72.0)
        elif rule == 'interval12':
            kw['interval'] = 12.0
        prob, lo, hi = H.make_problem(pk, **kw)
        vals = H.draws(lo, hi, 256, 91)
        for lpw, uni in ((1, 0), (1, 1), (64, 0)):
            ctx = H.gpu_context(prob, lanes_per_wave=lpw, uni_solver=uni)
            g = ctx.eval(vals, detail=True)
            ctx.close()
            key = f'{pk}/{rule}/{lpw}/{uni}'
            out[key + '/logp'] = g['logp']
            out[key + '/traj'] = g['traj']
            for k in g['stats'].dtype.names:
                out[key + '/' + k] = g['stats'][k]
np.savez(OUT, **out)
"""


def run(lib, out):
    code = (CHILD.replace("ROOT", repr(ROOT)).replace("OUT", repr(out)).replace("PK", repr(PK))
            .replace("RULES", repr(RULES)))
    env = dict(os.environ, BCM3HIP_LIB=os.path.abspath(lib))
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=900)


def main():
    a, b = sys.argv[1], sys.argv[2]
    run(a, "/tmp/flag_diff_a.npz")
    run(b, "/tmp/flag_diff_b.npz")
    A, B = np.load("/tmp/flag_diff_a.npz"), np.load("/tmp/flag_diff_b.npz")
    bad, cases = [], set()
    for k in A.files:
        cases.add(k.rsplit("/", 1)[0])
        if not np.array_equal(A[k], B[k], equal_nan=True):
            bad.append(k)
    # the three solver forms against each other within each build, as the test does
    forms_bad = []
    for X, name in ((A, os.path.basename(a)), (B, os.path.basename(b))):
        for pk in PK:
            for rule in RULES:
                for f in ("1/1", "64/0"):
                    for k in ("logp", "traj", "nst"):
                        if not np.array_equal(X[f"{pk}/{rule}/1/0/{k}"], X[f"{pk}/{rule}/{f}/{k}"], equal_nan=True):
                            forms_bad.append(f"{name}:{pk}/{rule}/{f}/{k}")
    print(f"{os.path.basename(a)} vs {os.path.basename(b)}: {len(cases)} cases (6 PK models x 7 dosing rules x 3 "
          f"solver forms, 256 draws, P = 2), {len(A.files)} arrays compared")
    print("differences between the builds:", bad if bad else "none (bit-identical)")
    print("solver forms disagreeing within a build:", forms_bad if forms_bad else "none")


if __name__ == "__main__":
    main()
