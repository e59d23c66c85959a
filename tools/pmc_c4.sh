# SQ counters of the C4 cell kernel (tools/cellpop_bench.py), one counter group per pass
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-c4pmc}; mkdir -p $O
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_BRANCH --output-format csv -d $O/p1 -o pmc -- python3 tools/cellpop_bench.py 64 2 > $O/p1.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU_FMA_F64 SQ_LDS_BANK_CONFLICT --output-format csv -d $O/p2 -o pmc -- python3 tools/cellpop_bench.py 64 2 > $O/p2.log 2>&1
echo ok
