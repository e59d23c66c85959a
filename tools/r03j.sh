cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
export BCM3_PARITY_LOG=$O/parity.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python tools/prof_popk.py 256 1 5 > $O/popk256.txt 2>&1 || { cat $O/popk256.txt; exit 1; }
cat $O/popk256.txt
timeout -k 10 300 python bench.py --steps 60 --warmup 6 --cpu-seconds 0 --throughput-batch 0 --extras 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], d['roofline']['issue']['kernel_ms'] if d['roofline']['issue'] else None)"
