#!/bin/bash
# Round-end evidence: bench line (with CPU baseline), rocprofv3 kernel stats of the bench, PMC traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
mkdir -p gpurun_out profiles
export TMPDIR=/tmp
timeout -k 10 900 python tools/pmc_traffic.py box_r5_1080p > gpurun_out/${TAG}_pmc.txt 2>&1 \
 && timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
 && cat gpurun_out/${TAG}_bench.json \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o bench --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2>&1 \
 \
 && cp $(find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' | head -1) profiles/${TAG}_bench_kernel_stats.csv \
 && cp gpurun_out/${TAG}_prof_bench.json profiles/${TAG}_bench_under_rocprof.json \
 && echo PROFILE_OK
