"""C3 parity of libbcm3hip.so builds against BOTH reference builds (one subprocess per library):
the 8,192-draw golden fixture (tests/golden/c3_golden_llh.npz: the reference's CVODE built with and
without FMA contraction) evaluated by each library, and the fractions the parity contract asserts
(tests/parity.py: llh within 1e-8 (1 + |llh|), bit-identical llh, equal BDF step counts, identical
ok / fail pattern) against each build, next to the two builds' own spread.

    python tools/contract_parity.py lib1.so [lib2.so ...]      (env ARITH=contract: the product
    library's contract-arithmetic kernel, BCM3HIP_OPT_ARITHMETIC)
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
sys.path[:0] = [ROOT, os.path.join(ROOT, 'oracle'), os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]
import numpy as np
import helpers as H, parity
from bcm3_amd import _hip
prob = H.c3_problem(1)
ctx = H.gpu_context(prob)
if os.environ.get('ARITH') == 'contract':
    ctx.set_option(_hip.OPT_ARITHMETIC, 1)
z = np.load(os.path.join(H.GOLDEN, 'c3_golden_llh.npz'))
vals = H.S.prior_draws(1, int(z['n']), int(z['seed']))
g = ctx.eval(vals, detail=True)
ok_g = g['status'] == 0
out = {'lib': LIB, 'arith': os.environ.get('ARITH', 'exact'), 'n': int(len(vals))}
for tag, lp, nst in (('fma', z['logp'], z['nst']), ('nofma', z['logp_nofma'], z['nst_nofma'])):
    e = parity.llh_err(g['logp'], lp)
    ok_r = z['ok'].astype(bool)
    out[tag] = {'llh_t1': float(np.mean(e <= parity.LLH_T1)), 'llh_max_both_ok': float(e[ok_g & ok_r].max()),
                'bitexact': parity.bitexact_fraction(g['logp'], lp),
                'steps_equal': float(np.mean(g['stats']['nst'][:, 0] == nst)),
                'status_differs': int(np.sum(ok_g != ok_r))}
s = parity.llh_err(z['logp_nofma'], z['logp'])
out['ref_self_llh_t1'] = float(np.mean(s <= parity.LLH_T1))
print('RESULT ' + json.dumps(out), flush=True)
"""


def main():
    for lib in sys.argv[1:]:
        env = dict(os.environ, BCM3HIP_LIB=os.path.abspath(lib))
        code = CHILD.replace("ROOT", repr(ROOT)).replace("LIB", repr(os.path.basename(lib)))
        p = subprocess.run([sys.executable, "-c", code], env=env, check=False, timeout=300,
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        for line in p.stdout.splitlines():
            if line.startswith("RESULT "):
                print(json.dumps(json.loads(line[7:])), flush=True)
            elif "amdgpu.ids" not in line:
                print(line, flush=True)


if __name__ == "__main__":
    main()
