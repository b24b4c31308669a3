#!/bin/bash
# Round-end evidence in one GPU call: SQ counters of the compute-bound kernels (VALU roofline input),
# PMC HBM traffic of the box kernel, the staged kernels' HBM roofline, the bench line (with the fresh
# counts), and a rocprofv3 kernel-stats summary of `bench.py --profile`.  Every step has its own time
# limit; the chain stops at the first failure.  Outputs under gpurun_out/ (copied to profiles/ by hand).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r03}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python tools/valu_counts.py > gpurun_out/${TAG}_valu.txt 2>&1 \
 && timeout -k 10 600 python tools/pmc_traffic.py box_r5_1080p > gpurun_out/${TAG}_pmc.txt 2>&1 \
 && timeout -k 10 500 python tools/staged_roofline.py > gpurun_out/${TAG}_staged.txt 2>&1 \
 && timeout -k 10 600 python bench.py --valu-json gpurun_out/valu_counts.json > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
 && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o bench --output-format csv -- python3 bench.py --profile --valu-json gpurun_out/valu_counts.json > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof_bench.err \
 && echo PROFILE_OK
