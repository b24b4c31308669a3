set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/variant_diff.py tools/ab/rr_new.so tools/ab/g_mix.so tools/ab/g_rr3.so > gpurun_out/r3t_diff.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r3t_diff.txt; [ $rc -eq 0 ] || exit $rc
SM_AB_AGG=guided SM_AB_LR=1 SM_AB_B=32 timeout -k 10 400 python tools/ab.py tools/ab/rr_new.so tools/ab/g_mix.so tools/ab/g_rr3.so > gpurun_out/r3t_ab_glr.txt 2>&1; rc=$?; cat gpurun_out/r3t_ab_glr.txt; [ $rc -eq 0 ] || exit $rc
SM_AB_AGG=guided SM_AB_B=32 timeout -k 10 400 python tools/ab.py tools/ab/rr_new.so tools/ab/g_mix.so > gpurun_out/r3t_ab_g.txt 2>&1; rc=$?; cat gpurun_out/r3t_ab_g.txt; [ $rc -eq 0 ] || exit $rc
SM_AB_AGG=guided SM_AB_LR=1 SM_AB_B=8 SM_AB_W=3840 SM_AB_H=2160 SM_AB_D=192 timeout -k 10 500 python tools/ab.py tools/ab/rr_new.so tools/ab/g_rr3.so > gpurun_out/r3t_ab_glr4k.txt 2>&1; rc=$?; cat gpurun_out/r3t_ab_glr4k.txt; exit $rc
