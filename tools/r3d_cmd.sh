set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "ad_volume or staged or sad_volume" --timeout 120 --timeout-method thread > gpurun_out/r3d_pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r3d_pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab_staged_kernels.py tools/ab/adv16.so tools/ab/adv64.so > gpurun_out/r3d_adv.txt 2>&1; cat gpurun_out/r3d_adv.txt
for L in tools/ab/stp4.so tools/ab/stp8.so tools/ab/stp16.so tools/ab/stp4.so tools/ab/stp8.so tools/ab/stp16.so; do SM_LIB=$L timeout -k 10 200 python tools/segtree_timing.py >> gpurun_out/r3d_stp.txt 2>&1 || break; done; grep -v amdgpu.ids gpurun_out/r3d_stp.txt
