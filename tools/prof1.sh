set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof1
timeout -k 10 300 python tools/prof_popk.py 256 1 3 > gpurun_out/prof1/plain.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1/kt -o kt -- python3 tools/prof_popk.py 256 1 3 > gpurun_out/prof1/kt.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/prof1/pmc1 -o pmc1 -- python3 tools/prof_popk.py 256 1 3 > gpurun_out/prof1/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/prof1/pmc2 -o pmc2 -- python3 tools/prof_popk.py 256 1 3 > gpurun_out/prof1/pmc2.log 2>&1
echo done
