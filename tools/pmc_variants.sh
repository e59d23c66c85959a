#!/bin/bash
# SQ counters of the C3 kernel (256 prior draws, seed 7: 254,710 BDF steps per launch) for several
# library builds, two passes each; prints per-step instruction counts and the wait shares:
#   TAG=r05g bash tools/pmc_variants.sh varlib/a.so varlib/b.so ...
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PROF_NO_DETAIL=1
O=gpurun_out/${TAG:-pmcvar}
mkdir -p $O
for lib in "$@"; do
  n=$(basename $lib .so)
  i=0; mkdir -p $O/$n
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INSTS_SMEM" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_LDS" \
             ${ICACHE:+"SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVES"}; do
    i=$((i+1))
    BCM3HIP_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/$n/p$i -o p -- python3 tools/prof_popk.py 256 1 3 > $O/$n/p$i.log 2>&1 || { echo "$n pass $i failed"; tail -5 $O/$n/p$i.log; exit 1; }
  done
done
python3 - "$O" "$@" <<'PY'
import csv, collections, glob, os, sys
o = sys.argv[1]
STEPS = 254710.0
for lib in sys.argv[2:]:
    n = os.path.basename(lib)[:-3]
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{o}/{n}/p*/p_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "popk_traj" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    a = {k: sum(v) / len(v) for k, v in agg.items()}
    wc = a.get("SQ_WAVE_CYCLES", 1.0)
    print(f"{n:18s} per step: VALU {a.get('SQ_INSTS_VALU',0)/STEPS:6.1f} SALU {a.get('SQ_INSTS_SALU',0)/STEPS:6.1f} "
          f"SMEM {a.get('SQ_INSTS_SMEM',0)/STEPS:5.2f} LDS {a.get('SQ_INSTS_LDS',0)/STEPS:5.2f} branch {a.get('SQ_INSTS_BRANCH',0)/STEPS:5.1f} "
          f"wave-cycles(x4) {4*wc/STEPS:7.1f} | WAIT_ANY {a.get('SQ_WAIT_ANY',0)/wc:5.3f} WAIT_INST {a.get('SQ_WAIT_INST_ANY',0)/wc:5.3f} "
          f"ACTIVE {a.get('SQ_ACTIVE_INST_ANY',0)/wc:5.3f} VALU-active {a.get('SQ_ACTIVE_INST_VALU',0)/wc:5.3f} SCA {a.get('SQ_ACTIVE_INST_SCA',0)/wc:5.3f}")
    if "SQC_ICACHE_MISSES" in a:
        print(f"{'':18s} icache per step: misses {a['SQC_ICACHE_MISSES']/STEPS:6.3f} dup {a.get('SQC_ICACHE_MISSES_DUPLICATE',0)/STEPS:6.3f} "
              f"hits {a['SQC_ICACHE_HITS']/STEPS:6.1f} ifetch {a.get('SQ_IFETCH',0)/STEPS:6.1f} ifetch-level/ifetch {a.get('SQ_IFETCH_LEVEL',0)/max(a.get('SQ_IFETCH',1),1):6.2f}")
PY
