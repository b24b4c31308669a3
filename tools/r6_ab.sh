#!/bin/bash
# Round-6 same-box A/B: tools/r6_ab.sh TAG "libA libB ..." MODES — bit-compare the guided maps of the builds
# (tools/variant_diff.py), then time each MODE (box | lr | guided | guidedlr | box4k | lr4k | guidedlr4k) with
# tools/ab.py, every lib in its own process, rounds alternated.  Each step under its own time limit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; LIBS=$2; MODES=$3
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SM_AB_NODIFF" ]; then
  timeout -k 10 400 python tools/variant_diff.py $LIBS > gpurun_out/${TAG}_diff.txt 2>&1 || { tail -20 gpurun_out/${TAG}_diff.txt; exit 1; }
  cat gpurun_out/${TAG}_diff.txt
fi
for X in $MODES; do
  case $X in
    box) E="SM_AB_B=32";;
    lr) E="SM_AB_B=32 SM_AB_LR=1";;
    guided) E="SM_AB_B=32 SM_AB_AGG=guided";;
    guidedlr) E="SM_AB_B=32 SM_AB_AGG=guided SM_AB_LR=1";;
    box4k) E="SM_AB_B=8 SM_AB_W=3840 SM_AB_H=2160 SM_AB_D=192";;
    lr4k) E="SM_AB_B=8 SM_AB_W=3840 SM_AB_H=2160 SM_AB_D=192 SM_AB_LR=1";;
    guidedlr4k) E="SM_AB_B=8 SM_AB_W=3840 SM_AB_H=2160 SM_AB_D=192 SM_AB_AGG=guided SM_AB_LR=1";;
    wide20) E="SM_AB_B=8 SM_AB_R=20";;
    wide127lr) E="SM_AB_B=8 SM_AB_R=127 SM_AB_LR=1";;
    *) echo "unknown mode $X"; exit 9;;
  esac
  env $E timeout -k 10 500 python tools/ab.py $LIBS > gpurun_out/${TAG}_ab_${X}.txt 2>&1 || { tail -5 gpurun_out/${TAG}_ab_${X}.txt; exit 2; }
  echo "== $X"; cat gpurun_out/${TAG}_ab_${X}.txt
done
exit 0
