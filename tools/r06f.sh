#!/bin/bash
# round 6, lease f: profiles at HEAD -- C3 kernel trace + PMC traffic / SQ passes (tools/evidence.sh,
# PROFILES_ONLY), C4 SQ passes (tools/pmc_c4.sh) and the C4 phase split (BCM3_CP_PHASES=1)
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
PROFILES_ONLY=1 TAG=r06f bash tools/evidence.sh
TAG=r06f bash tools/pmc_c4.sh
BCM3_CP_PHASES=1 timeout -k 10 200 python tools/cellpop_phases.py 16 > gpurun_out/r06f/c4_phases.txt 2>&1
cat gpurun_out/r06f/c4_phases.txt
