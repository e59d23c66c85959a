set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/ic; mkdir -p $O
B="bench.py --steps 20 --warmup 3 --cpu-seconds 0 --throughput-batch 0 --extras 0"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_INSTS_SALU --output-format csv -d $O/p1 -o pmc -- python3 $B > $O/p1.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_IFETCH_LEVEL --output-format csv -d $O/p2 -o pmc -- python3 $B > $O/p2.log 2>&1
echo ok
