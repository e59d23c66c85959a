"""CPU rate of the oracle's cell-population evaluation (the reference's CVODE, or the restated DP5
with CP_SOLVER=DP5) on the C4 experiment: n prior draws on `threads` host threads, one evaluation
per thread like the reference's sampling threads (test infrastructure: the oracle is the checker).

    [CP_SOLVER=DP5] python tools/cellpop_cpu_rate.py [n] [threads]
"""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tests", "golden")]
import cellpop as CP  # noqa: E402
import cellpop_helpers as CH  # noqa: E402

G = os.path.join(ROOT, "tests", "golden")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
threads = int(sys.argv[2]) if len(sys.argv) > 2 else 16
lik = os.path.join(G, "cellpop_likelihood.xml")
if os.environ.get("CP_SOLVER", "CVODE") == "DP5":
    text = open(lik).read().replace('<experiment name="exp1" ', '<experiment name="exp1" solver_type="DP5" ')
    text = text.replace('model_file="cellpop_model.xml"', f'model_file="{os.path.join(G, "cellpop_model.xml")}"')
    text = text.replace('data_file="cellpop_data.json"', f'data_file="{os.path.join(G, "cellpop_data.json")}"')
    lik = os.path.join(tempfile.mkdtemp(), "cellpop_dp5.xml")
    with open(lik, "w") as f:
        f.write(text)
prob = CP.load_problem(lik, CH.PRIOR)
x = CH.draws(n, 20251018)
t0 = time.perf_counter()
r = CP.simulate(prob, x, nthreads=threads)
dt = time.perf_counter() - t0
print(f"{os.environ.get('CP_SOLVER', 'CVODE')}: {n} evals on {threads} threads in {dt:.2f} s = {n / dt:.2f} evals/s, "
      f"{sum(r['num_cells']) / n:.0f} cells/eval", flush=True)
