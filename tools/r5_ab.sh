# tools/r5_ab.sh TAG "libA libB ..." [tests...]: parity tests on the in-tree build, then same-box A/B timings
# (box 1080p / 4K, optionally box+LR and guided via SM_R5_AB_EXTRA="lr guided")
set -o pipefail
mkdir -p gpurun_out
TAG=$1; LIBS=$2; shift 2
if [ $# -gt 0 ]; then
  timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread "$@" > gpurun_out/${TAG}_tests.txt 2>&1; rc=$?
  tail -3 gpurun_out/${TAG}_tests.txt
  [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_tests.txt | head -20; exit 1; }
fi
SM_AB_B=32 timeout -k 10 300 python tools/ab.py $LIBS > gpurun_out/${TAG}_ab_box.txt 2>&1 && cat gpurun_out/${TAG}_ab_box.txt || exit 2
SM_AB_B=8 SM_AB_W=3840 SM_AB_H=2160 SM_AB_D=192 timeout -k 10 300 python tools/ab.py $LIBS > gpurun_out/${TAG}_ab_box4k.txt 2>&1 && cat gpurun_out/${TAG}_ab_box4k.txt || exit 3
for X in $SM_R5_AB_EXTRA; do
  if [ "$X" = lr ]; then SM_AB_B=32 SM_AB_LR=1 timeout -k 10 300 python tools/ab.py $LIBS > gpurun_out/${TAG}_ab_lr.txt 2>&1 && cat gpurun_out/${TAG}_ab_lr.txt || exit 4; fi
  if [ "$X" = guided ]; then SM_AB_B=32 SM_AB_AGG=guided timeout -k 10 400 python tools/ab.py $LIBS > gpurun_out/${TAG}_ab_guided.txt 2>&1 && cat gpurun_out/${TAG}_ab_guided.txt || exit 5; fi
  if [ "$X" = guidedlr ]; then SM_AB_B=32 SM_AB_AGG=guided SM_AB_LR=1 timeout -k 10 400 python tools/ab.py $LIBS > gpurun_out/${TAG}_ab_guidedlr.txt 2>&1 && cat gpurun_out/${TAG}_ab_guidedlr.txt || exit 6; fi
done
exit 0
