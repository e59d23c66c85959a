#!/bin/bash
# GPU tests + smoke + bench, the phase attribution, and the SQ instruction counters of the BDF kernel
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04j}
O=gpurun_out/$TAG
mkdir -p $O
TAG=$TAG bash tools/gpu_tests.sh
timeout -k 10 180 python tools/phase_probe.py 256 > $O/phases.txt 2>&1
tail -24 $O/phases.txt
SQRUN="tools/prof_popk.py 256 1 3"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_sq -o pmc -- python3 $SQRUN > $O/pmc_sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 --output-format csv -d $O/pmc_sq2 -o pmc -- python3 $SQRUN > $O/pmc_sq2.log 2>&1
echo done
