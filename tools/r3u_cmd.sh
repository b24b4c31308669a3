set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
P=gpu_stereo_matching_amd/libsm_hip.so
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r3u_pytest_gpu.txt 2>&1; rc=$?; tail -3 gpurun_out/r3u_pytest_gpu.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/variant_diff.py tools/ab/rr_new.so $P > gpurun_out/r3u_diff.txt 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/r3u_diff.txt; [ $rc -eq 0 ] || exit $rc
SM_AB_AGG=guided SM_AB_LR=1 SM_AB_B=32 timeout -k 10 400 python tools/ab.py tools/ab/rr_new.so $P > gpurun_out/r3u_ab.txt 2>&1; rc=$?; cat gpurun_out/r3u_ab.txt; [ $rc -eq 0 ] || exit $rc
for r in 1 2 4; do SM_AB_R=$r SM_AB_AGG=guided SM_AB_LR=1 SM_AB_B=32 timeout -k 10 400 python tools/ab.py tools/ab/rr_new.so $P > gpurun_out/r3u_ab_r$r.txt 2>&1; rc=$?; echo "r=$r"; cat gpurun_out/r3u_ab_r$r.txt; [ $rc -eq 0 ] || exit $rc; done
timeout -k 10 300 python bench.py > gpurun_out/r3u_bench.json 2> gpurun_out/r3u_bench.err && cut -c1-300 gpurun_out/r3u_bench.json
