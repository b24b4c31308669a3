#!/bin/bash
# Round-6 targeted GPU checks: the touched test files, then an N=2 gloo rehearsal of bench.py (one GPU, two
# ranks) that records the split parity checks.  Each GPU step under its own time limit; the chain stops at
# the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?usage: r6_check.sh TAG}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_gpu_dslice_lr.py tests/test_gpu_group.py tests/test_gpu_guided.py \
  "tests/test_gpu_parity.py::test_two_streams_one_handle_wide" "tests/test_gpu_parity.py::test_two_streams_one_handle" \
  > gpurun_out/${TAG}_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -3 gpurun_out/${TAG}_tests.txt
SM_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --no-variants \
  > gpurun_out/${TAG}_n2_gloo.json 2> gpurun_out/${TAG}_n2_gloo.err || { tail -20 gpurun_out/${TAG}_n2_gloo.err; exit 2; }
python - <<PY
import json
ln = [l for l in open("gpurun_out/${TAG}_n2_gloo.json") if l.lstrip().startswith("{")][-1]
d = json.loads(ln[ln.index("{"):])
print(json.dumps({k: d.get(k) for k in ("value", "rccl_world", "split_parity")}))
print(json.dumps(d["dslice"].get("check")), json.dumps(d["rowband"].get("check")))
print(json.dumps(d["cfg5_guided_lr"].get("dslice_guided_lr", {}).get("check")))
PY
