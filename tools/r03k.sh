cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
export BCM3_PARITY_LOG=$O/parity.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 60 --warmup 6 --cpu-seconds 0 --throughput-batch 0 --extras 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 40 --warmup 4 --cpu-seconds 0 --throughput-batch 0 --extras 0 --issue-probe 0 > $O/kt.log 2>&1 || { tail -5 $O/kt.log; exit 1; }
python - <<'PY'
import csv
for r in sorted(csv.DictReader(open('gpurun_out/r03k/kt/kt_kernel_stats.csv')), key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:8.1f} us")
PY
timeout -k 10 400 python tools/spec_sim.py > $O/spec_sim.txt 2>&1 || { tail -20 $O/spec_sim.txt; exit 1; }
grep sampler $O/spec_sim.txt
timeout -k 10 400 python tools/variant_timing.py varlib/old_fast.so varlib/new_plain.so varlib/old_fast.so varlib/new_plain.so
