#!/bin/bash
# Strip-kernel timing breakdown: ablate.py on the 1080p D=128 r=20 batch-8 workload for each lib (timing only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; LIBS=$2; R=${3:-20}
SM_AB_B=8 SM_AB_R=$R timeout -k 10 500 python tools/ab.py $LIBS > gpurun_out/${TAG}_ab.txt 2>&1 || { tail -5 gpurun_out/${TAG}_ab.txt; exit 2; }
cat gpurun_out/${TAG}_ab.txt
