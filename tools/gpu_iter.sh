#!/bin/bash
# Fast iteration: GPU parity tests + bench (no CPU baseline) + kernel-trace stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-it}
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/${TAG}_pytest.txt 2>&1; rc=$?
tail -3 gpurun_out/${TAG}_pytest.txt
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/${TAG}_pytest.txt | head -20; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && cat gpurun_out/${TAG}_bench.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('value', d['value'], 'ms/frame', d['ms_per_frame'], 'kern_ms', d['roofline']['kernel_ms_per_launch'], 'frac', d['roofline']['frac'], d.get('variants'))"
