# C4 cell kernel built with extra hipRTC options (BCM3_CP_OPTS): ms per 64-evaluation batch and the
# logp checksum (the options must not change a bit)
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-cpopts}; mkdir -p $O
# SWEEP="opts1|opts2|...": the option sets (default: the round-3 r03zd set)
SWEEP=${SWEEP:-"|-fno-unroll-loops|-mllvm -unroll-threshold=100|-fno-unroll-loops -mllvm -amdgpu-sched-strategy=max-ilp|-mllvm -amdgpu-sched-strategy=max-ilp"}
IFS='|' read -r -a SETS <<< "$SWEEP"
i=0
for opts in "${SETS[@]}"; do
  BCM3_CP_OPTS="$opts" timeout -k 10 200 python tools/cellpop_bench.py 64 5 > $O/v$i.txt 2>&1
  echo "[$opts] $(tr '\n' ' ' < $O/v$i.txt)"
  i=$((i+1))
done
