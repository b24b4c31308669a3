set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_guided.py tests/test_gpu_literal.py > gpurun_out/r5d_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/r5d_tests.txt
[ $rc -eq 0 ] || exit 1
A="tools/abv/base5.so tools/abv/skip5.so"
SM_AB_B=32 timeout -k 10 300 python tools/ab.py $A > gpurun_out/r5d_ab_box.txt 2>&1 && cat gpurun_out/r5d_ab_box.txt || exit 2
SM_AB_B=8 SM_AB_W=3840 SM_AB_H=2160 SM_AB_D=192 timeout -k 10 300 python tools/ab.py $A > gpurun_out/r5d_ab_box4k.txt 2>&1 && cat gpurun_out/r5d_ab_box4k.txt || exit 3
SM_AB_B=32 SM_AB_AGG=guided timeout -k 10 400 python tools/ab.py $A > gpurun_out/r5d_ab_guided.txt 2>&1 && cat gpurun_out/r5d_ab_guided.txt || exit 4
