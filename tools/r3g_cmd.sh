set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/variant_diff.py tools/ab/g4.so tools/ab/g4rr.so > gpurun_out/r3g_diff.txt 2>&1; tail -4 gpurun_out/r3g_diff.txt
SM_AB_AGG=guided SM_AB_LR=1 SM_AB_B=32 timeout -k 10 400 python tools/ab.py tools/ab/g4.so tools/ab/g4rr.so > gpurun_out/r3g_ab_lr.txt 2>&1; cat gpurun_out/r3g_ab_lr.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3g_prof -o st --output-format csv -- python3 tools/segtree_timing.py > gpurun_out/r3g_segprof.txt 2>&1; grep -v amdgpu.ids gpurun_out/r3g_segprof.txt | grep ST; find gpurun_out/r3g_prof -name "*kernel_stats.csv" | head -2
