#!/bin/bash
# C4: SQ counters of the generation launches' cell kernel and of the work queue's (same batches)
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06r${TAG:-}; mkdir -p $O
for qm in 0 1; do
  BCM3_CP_QUEUE=$qm timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_BRANCH --output-format csv -d $O/q$qm -o pmc -- python3 tools/cellpop_bench.py 64 2 > $O/q$qm.log 2>&1
  BCM3_CP_QUEUE=$qm timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_FLAT --output-format csv -d $O/q${qm}b -o pmc -- python3 tools/cellpop_bench.py 64 2 > $O/q${qm}b.log 2>&1
done
echo ok
