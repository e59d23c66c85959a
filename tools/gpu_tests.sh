#!/bin/bash
# One GPU call: tests (+ parity summary log), smoke and the default bench line into gpurun_out/$TAG,
# then the optional extras the environment asks for:
#   VARIANTS="varlib/a.so varlib/b.so ..."  A/B kernel timing of library builds (tools/variant_timing.py)
#   PHASES=1                                 plain-step phase attribution (tools/phase_probe.py; needs
#                                            make -C bcm3_amd/csrc phases beforehand)
#   SQ=1                                     SQ instruction counters of plain 256-proposal launches
#   NOTESTS=1 / NOBENCH=1                    skip the tests + smoke / the bench
# usage: TAG=r05a [VARIANTS=...] [PHASES=1] [SQ=1] bash tools/gpu_tests.sh
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r05}
O=gpurun_out/$TAG
mkdir -p $O
export BCM3_PARITY_LOG=$O/parity.jsonl
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
  head -c 1500 $O/bench.json
fi
if [ -n "$VARIANTS" ]; then
  timeout -k 10 600 python tools/variant_timing.py $VARIANTS > $O/variants.txt 2>&1
  cat $O/variants.txt
fi
if [ -n "$PHASES" ]; then
  timeout -k 10 180 python tools/phase_probe.py 256 > $O/phases.txt 2>&1
  tail -24 $O/phases.txt
fi
if [ -n "$SQ" ]; then
  SQRUN="tools/prof_popk.py 256 1 3"
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sq -o pmc -- python3 $SQRUN > $O/pmc_sq.log 2>&1
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 --output-format csv -d $O/pmc_sq2 -o pmc -- python3 $SQRUN > $O/pmc_sq2.log 2>&1
fi
echo done
