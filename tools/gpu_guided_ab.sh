#!/bin/bash
# Guided-kernel iteration on the GPU box: parity tests of the product build, then same-box A/B timing
# of the variant libraries under tools/ab/ (guided and guided+LR at 1080p D=128 r=5, 32 frames/call).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-gab}; shift
LIBS="$*"
timeout -k 10 400 python -u -m pytest tests/test_gpu_guided.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.txt 2>&1; rc=$?
tail -4 gpurun_out/${TAG}_pytest.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
grep -E "^(FAILED|ERROR)|Error" gpurun_out/${TAG}_pytest.txt | head -20
SM_AB_AGG=guided SM_AB_B=32 timeout -k 10 400 python tools/ab.py $LIBS > gpurun_out/${TAG}_ab_guided.txt 2>&1 || { cat gpurun_out/${TAG}_ab_guided.txt; exit 3; }
cat gpurun_out/${TAG}_ab_guided.txt
SM_AB_AGG=guided SM_AB_LR=1 SM_AB_B=32 timeout -k 10 400 python tools/ab.py $LIBS > gpurun_out/${TAG}_ab_guided_lr.txt 2>&1 || { cat gpurun_out/${TAG}_ab_guided_lr.txt; exit 3; }
cat gpurun_out/${TAG}_ab_guided_lr.txt
exit $rc
