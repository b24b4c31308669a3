#!/bin/bash
# One GPU session: build check, parity tests, smoke, bench, rocprof kernel-trace of the bench.
# Every GPU step has its own time limit; steps are chained with && so a failure stops the run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-run}
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/${TAG}_pytest_gpu.txt 2>&1 \
 && tail -3 gpurun_out/${TAG}_pytest_gpu.txt \
 && timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 \
 && tail -1 gpurun_out/${TAG}_smoke.txt \
 && timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
 && cat gpurun_out/${TAG}_bench.json \
 && export TMPDIR=/tmp \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o bench --output-format csv -- python3 bench.py --no-cpu-baseline --steps 50 > gpurun_out/${TAG}_prof_bench.json 2>&1 \
 && cat $(find gpurun_out/${TAG}_prof -name '*kernel_stats.csv') | cut -c1-200
