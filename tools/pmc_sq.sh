#!/bin/bash
# SQ / SQC counter passes of the BDF kernel at 256 chains (one pass per counter group).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmcsq}
mkdir -p $O
P="python3 tools/prof_popk.py 256 1 3"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_LDS" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_INSTS_VMEM GRBM_GUI_ACTIVE" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_FLAT SQ_INSTS_VALU_FMA_F64"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o p -- $P > $O/p$i.log 2>&1 || echo "pass $i failed"
done
python3 - "$O" <<'PY'
import csv, collections, glob, sys
o = sys.argv[1]
for f in sorted(glob.glob(o + "/p*/p_counter_collection.csv")):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "popk_traj" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(f"{k:28s} {sum(v)/len(v):14.4g}  per-wave {sum(v)/len(v)/256:12.4g}")
PY
