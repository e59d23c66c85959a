# C4 occupancy sweep: the cell kernel built for 1 / 2 / 3 wavefronts per SIMD (BCM3_CP_WAVES)
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/${TAG:-waves}; mkdir -p $O
for w in ${WAVES:-1 2 3}; do BCM3_CP_WAVES=$w timeout -k 10 200 python tools/cellpop_bench.py 64 5 > $O/w$w.txt 2>&1; echo "waves $w: $(grep n=64 $O/w$w.txt)"; done
