#!/bin/bash
# One GPU iteration: parity tests of the in-tree build for the touched paths, then same-box A/B timings.
#   tools/gpu_iter.sh TAG "pytest files" "guided A/B libs" "segtree A/B libs"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=$1; TESTS=$2; GLIBS=$3; SLIBS=$4
if [ -n "$TESTS" ]; then
  timeout -k 10 500 python -u -m pytest $TESTS -x -q --timeout 170 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1; rc=$?
  tail -4 gpurun_out/${TAG}_pytest.txt
  if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_pytest.txt | head -20; echo "pytest rc=$rc: stopping"; exit $rc; fi
fi
if [ -n "$GLIBS" ]; then
  SM_AB_AGG=guided SM_AB_B=32 timeout -k 10 400 python tools/ab.py $GLIBS > gpurun_out/${TAG}_ab_guided.txt 2>&1 || { cat gpurun_out/${TAG}_ab_guided.txt; exit 3; }
  cat gpurun_out/${TAG}_ab_guided.txt
  SM_AB_AGG=guided SM_AB_LR=1 SM_AB_B=32 timeout -k 10 400 python tools/ab.py $GLIBS > gpurun_out/${TAG}_ab_guided_lr.txt 2>&1 || { cat gpurun_out/${TAG}_ab_guided_lr.txt; exit 3; }
  cat gpurun_out/${TAG}_ab_guided_lr.txt
fi
for L in $SLIBS; do
  SM_LIB=$L timeout -k 10 300 python tools/segtree_timing.py >> gpurun_out/${TAG}_segtree.txt 2>&1 || { cat gpurun_out/${TAG}_segtree.txt; exit 4; }
done
[ -n "$SLIBS" ] && cat gpurun_out/${TAG}_segtree.txt
exit 0
