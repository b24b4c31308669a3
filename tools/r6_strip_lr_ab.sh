#!/bin/bash
# Box + LR at wide radii, strip right view against the separable path: tools/r6_strip_lr_ab.sh TAG "libs" RADII
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; LIBS=$2; shift 2
for r in "$@"; do
  SM_AB_B=8 SM_AB_R=$r SM_AB_LR=1 timeout -k 10 500 python tools/ab.py $LIBS > gpurun_out/${TAG}_lr_r$r.txt 2>&1 || { tail -5 gpurun_out/${TAG}_lr_r$r.txt; exit 2; }
  echo "== LR r=$r"; cat gpurun_out/${TAG}_lr_r$r.txt
done
