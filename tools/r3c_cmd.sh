set -o pipefail
bash tools/gpu_iter.sh r3c "tests/test_gpu_guided.py tests/test_gpu_parity.py" "tools/ab/st1.so tools/ab/g2.so" "" || exit $?
timeout -k 10 300 python tools/roundtrip_ab.py > gpurun_out/r3c_roundtrip.txt 2>&1; cat gpurun_out/r3c_roundtrip.txt
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3c_prof -o st -- python3 tools/segtree_timing.py > gpurun_out/r3c_segprof.txt 2>&1; tail -3 gpurun_out/r3c_segprof.txt; find gpurun_out/r3c_prof -name "*stats*" | head
timeout -k 10 400 python tools/ab_staged_kernels.py tools/ab/adv16.so tools/ab/adv64.so > gpurun_out/r3c_adv.txt 2>&1; cat gpurun_out/r3c_adv.txt
