# round 4: guided 96-row tiles on one 12-wave workgroup per CU (SM_G_TALL=2) against the kept 32-row tiles:
# maps bit-compared, then same-box timing (1080p D=128 r=5, 32 frames per call; 4K D=192 8 frames), counters
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=tools/abv
timeout -k 10 300 python tools/variant_diff.py $V/g32.so $V/g96.so $V/g96r.so > gpurun_out/r4j_diff.txt 2>&1; rc=$?; cat gpurun_out/r4j_diff.txt; [ $rc -eq 0 ] || exit $rc
SM_AB_AGG=guided SM_AB_B=32 timeout -k 10 400 python tools/ab.py $V/g32.so $V/g96.so > gpurun_out/r4j_ab.txt 2>&1 || { cat gpurun_out/r4j_ab.txt; exit 3; }
cat gpurun_out/r4j_ab.txt
SM_AB_AGG=guided SM_AB_B=8 SM_AB_W=3840 SM_AB_H=2160 SM_AB_D=192 timeout -k 10 400 python tools/ab.py $V/g32.so $V/g96.so > gpurun_out/r4j_ab_4k.txt 2>&1 || { cat gpurun_out/r4j_ab_4k.txt; exit 3; }
cat gpurun_out/r4j_ab_4k.txt
SM_AB_AGG=guided SM_AB_LR=1 SM_AB_B=32 timeout -k 10 400 python tools/ab.py $V/g32.so $V/g96r.so > gpurun_out/r4j_ab_lr.txt 2>&1 || { cat gpurun_out/r4j_ab_lr.txt; exit 3; }
cat gpurun_out/r4j_ab_lr.txt
SM_VALU_JOBS=guided_r5_1080p_d128_b32 SM_LIB=$V/g96.so SM_TAG=_g96 timeout -k 10 400 python tools/valu_counts.py > gpurun_out/r4j_valu_g96.txt 2>&1 || { tail -5 gpurun_out/r4j_valu_g96.txt; exit 4; }
cat gpurun_out/r4j_valu_g96.txt
