#!/bin/bash
# One gpurun call: GPU tests, smoke, bench, rocprofv3 kernel trace + PMC passes of the bench.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r01
mkdir -p $O
STEPS=${STEPS:-20}
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
cat $O/smoke.log | tail -2
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
cat $O/bench.json
BENCH="bench.py --steps $STEPS --warmup 3 --cpu-seconds 0 --throughput-batch 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $BENCH > $O/kt.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 $BENCH > $O/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 $BENCH > $O/pmc_write.log 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sq -o pmc -- python3 $BENCH > $O/pmc_sq.log 2>&1
echo done
