cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03h
mkdir -p $O
export BCM3_PARITY_LOG=$O/parity.jsonl
# test failures (exit 1) are reported and the run goes on; a fault, abort, timeout or hang ends it
step() { "$@"; rc=$?; if [ $rc -gt 1 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; return 0; }
step timeout -k 10 600 python -u -m pytest tests/test_ptmh_native_gpu.py tests/test_refbind.py -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
grep -E "passed|failed" $O/pytest_gpu.log | tail -3
grep -E "FAILED|ERROR|^E " $O/pytest_gpu.log | head -20
timeout -k 10 400 python tools/spec_sim.py > $O/spec_sim.txt 2>&1 || { echo spec_sim failed; tail -20 $O/spec_sim.txt; exit 1; }
tail -4 $O/spec_sim.txt
timeout -k 10 120 python tools/phase_probe.py 256 1 > $O/phases.txt 2>&1 || { echo phases failed; tail -20 $O/phases.txt; exit 1; }
cat $O/phases.txt
timeout -k 10 60 tools/ubench/build/handoff > $O/handoff.txt 2>&1 || { echo handoff failed; exit 1; }
cat $O/handoff.txt
timeout -k 10 300 python bench.py --steps 40 --warmup 6 --cpu-seconds 0 --throughput-batch 0 --extras 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['config']['sampler_loop'])"
