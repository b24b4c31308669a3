#!/bin/bash
# Round-end evidence: PMC HBM traffic of the box kernel, the bench line (with CPU baseline and the
# per-config table), and a rocprofv3 kernel-stats summary of `bench.py --profile` (only the timed
# 4-frame steps, so its box_match_kernel average is the bench's kernel_ms_per_launch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python tools/pmc_traffic.py box_r5_1080p > gpurun_out/${TAG}_pmc.txt 2>&1 \
 && timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
 && cat gpurun_out/${TAG}_bench.json \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o bench --output-format csv -- python3 bench.py --profile > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof_bench.err \
 && cat gpurun_out/${TAG}_prof_bench.json \
 && cat $(find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' | head -1) | cut -c1-180 \
 && echo PROFILE_OK
