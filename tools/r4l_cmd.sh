# round 4: guided right-view keys by saturating conversion (rk1, one v_min) against the clamped keys (rk0)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=tools/abv
timeout -k 10 300 python tools/variant_diff.py $V/rk0.so $V/rk1.so > gpurun_out/r4l_diff.txt 2>&1; cat gpurun_out/r4l_diff.txt
SM_AB_AGG=guided SM_AB_LR=1 SM_AB_B=32 timeout -k 10 400 python tools/ab.py $V/rk0.so $V/rk1.so --rounds 5 > gpurun_out/r4l_ab.txt 2>&1 || { cat gpurun_out/r4l_ab.txt; exit 3; }
cat gpurun_out/r4l_ab.txt
SM_AB_AGG=guided SM_AB_LR=1 SM_AB_B=8 SM_AB_W=3840 SM_AB_H=2160 SM_AB_D=192 timeout -k 10 400 python tools/ab.py $V/rk0.so $V/rk1.so > gpurun_out/r4l_ab_4k.txt 2>&1 || { cat gpurun_out/r4l_ab_4k.txt; exit 3; }
cat gpurun_out/r4l_ab_4k.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_guided.py tests/test_gpu_headline.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r4l_pytest.txt 2>&1; rc=$?
tail -3 gpurun_out/r4l_pytest.txt
exit $rc
