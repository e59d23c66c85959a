#!/bin/bash
# One gpurun call collecting a round's evidence into gpurun_out/$TAG: GPU tests, smoke, bench,
# rocprofv3 kernel-trace stats of the bench, PMC passes (FETCH_SIZE, WRITE_SIZE, SQ counters) --
# one counter group per run, as MI355X_MICROARCH.md prescribes. tools/collect_profiles.py $TAG
# then copies the summaries into profiles/.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r01}
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "$PROFILES_ONLY" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  tail -1 $O/smoke.log
  timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
  cat $O/bench.json
fi
BENCH="bench.py --steps 40 --warmup 4 --cpu-seconds 0 --throughput-batch 0 --extras 0 --issue-probe 0 --strong-chains 0"
# the SQ passes count instructions per BDF step on plain 256-proposal launches (one trajectory per wave)
SQRUN="tools/prof_popk.py 256 1 3"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 $BENCH > $O/kt.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_extras -o kt -- python3 bench.py --steps 5 --warmup 1 --cpu-seconds 0 --throughput-batch 0 --extras 1 --strong-chains 0 > $O/kt_extras.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 $BENCH > $O/pmc_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 $BENCH > $O/pmc_write.log 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sq -o pmc -- python3 $SQRUN > $O/pmc_sq.log 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 --output-format csv -d $O/pmc_sq2 -o pmc -- python3 $SQRUN > $O/pmc_sq2.log 2>&1
echo done
