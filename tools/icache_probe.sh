#!/bin/bash
# Instruction-cache pressure of the C3 kernel vs the number of wavefronts sharing the chip's
# instruction caches: SQ / SQC counters per BDF step at n = 32, 256, 1024 prior draws (product library).
#   TAG=r05j bash tools/icache_probe.sh
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-icache}
mkdir -p $O
for n in 32 256 1024; do
  i=0; mkdir -p $O/n$n
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
             "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVES"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $O/n$n/p$i -o p -- python3 tools/prof_popk.py $n 1 3 > $O/n$n/p$i.log 2>&1 || { echo "n=$n pass $i failed"; exit 1; }
  done
done
python3 - "$O" <<'PY'
import csv, collections, glob, re, sys
o = sys.argv[1]
for n in (32, 256, 1024):
    steps = None
    for line in open(f"{o}/n{n}/p1.log"):
        m = re.search(r"total steps (\d+)", line)
        if m: steps = float(m.group(1))
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(f"{o}/n{n}/p*/p_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "popk_traj_kernelILi1ELi2ELb0E" in r["Kernel_Name"] or "popk_traj_kernel<1, 2, false>" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    a = {k: sum(v) / len(v) for k, v in agg.items()}
    wc = a["SQ_WAVE_CYCLES"]
    print(f"n={n:5d} steps/launch {steps:.0f}: VALU {a['SQ_INSTS_VALU']/steps:6.1f} SALU {a['SQ_INSTS_SALU']/steps:6.1f} "
          f"cycles(x4) {4*wc/steps:7.1f} WAIT {a['SQ_WAIT_ANY']/wc:5.3f} ACTIVE {a['SQ_ACTIVE_INST_ANY']/wc:5.3f} | "
          f"icache misses/step {a['SQC_ICACHE_MISSES']/steps:6.3f} dup {a['SQC_ICACHE_MISSES_DUPLICATE']/steps:6.3f} ifetch/step {a['SQ_IFETCH']/steps:6.1f}")
PY
