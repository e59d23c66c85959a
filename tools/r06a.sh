#!/bin/bash
# round 6, first lease: C3 arithmetic variants (parity against both reference builds, bench line)
# and C4 with FMA contraction in the hipRTC cell kernel
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; O=gpurun_out/r06a; mkdir -p $O
V="gpuvar/product.so gpuvar/v_rootcr.so gpuvar/v_fma.so gpuvar/v_rootcr_fma.so gpuvar/v_rootcr_fma_fdiv.so"
timeout -k 10 400 python tools/contract_parity.py $V > $O/parity.txt 2>&1
cat $O/parity.txt
ROUNDS=2 timeout -k 10 600 bash tools/bench_variants.sh $V > $O/bench_variants.txt 2>&1
cat $O/bench_variants.txt
timeout -k 10 200 python tools/cellpop_bench.py 64 5 > $O/c4_default.txt 2>&1
cat $O/c4_default.txt
BCM3_CP_OPTS="-ffp-contract=fast" timeout -k 10 200 python tools/cellpop_bench.py 64 5 > $O/c4_fma.txt 2>&1
cat $O/c4_fma.txt
timeout -k 10 200 python tools/cellpop_bench.py 64 5 > $O/c4_default2.txt 2>&1
cat $O/c4_default2.txt
