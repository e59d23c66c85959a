set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/prof2
mkdir -p $O
timeout -k 10 300 python tools/prof_popk.py 256 1 3 > $O/plain.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH --output-format csv -d $O/pmc1 -o pmc1 -- python3 tools/prof_popk.py 256 1 3 > $O/pmc1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE SQ_INSTS_SMEM --output-format csv -d $O/pmc2 -o pmc2 -- python3 tools/prof_popk.py 256 1 3 > $O/pmc2.log 2>&1
echo done
