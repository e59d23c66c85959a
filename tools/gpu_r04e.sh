#!/bin/bash
# Round-4 evidence in one call: GPU tests + smoke + bench (tools/gpu_tests.sh), the fast-loop phase
# attribution (profiling build), then the rocprofv3 kernel-trace and PMC passes of tools/evidence.sh.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${TAG:-r04e}
O=gpurun_out/$TAG
mkdir -p $O
TAG=$TAG bash tools/gpu_tests.sh
timeout -k 10 180 python tools/phase_probe.py 256 > $O/phases.txt 2>&1
tail -22 $O/phases.txt
TAG=$TAG PROFILES_ONLY=1 bash tools/evidence.sh
