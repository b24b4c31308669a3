set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_iter.sh r3e "tests/test_gpu_guided.py" "tools/ab/g3off.so tools/ab/g3.so" "" || exit $?
timeout -k 10 400 python tools/ab_staged_kernels.py tools/ab/adv16.so tools/ab/adv64.so > gpurun_out/r3e_adv.txt 2>&1; cat gpurun_out/r3e_adv.txt
for L in tools/ab/stp4.so tools/ab/stp8.so tools/ab/stp16.so tools/ab/stp4.so tools/ab/stp8.so tools/ab/stp16.so; do SM_LIB=$L timeout -k 10 200 python tools/segtree_timing.py >> gpurun_out/r3e_stp.txt 2>&1 || break; done; grep -v amdgpu.ids gpurun_out/r3e_stp.txt
