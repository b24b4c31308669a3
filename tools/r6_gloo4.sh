#!/bin/bash
# The new d-slice LR fuzz test, then a 4-rank gloo rehearsal of bench.py on one GPU (uneven d splits:
# 256 / 4, 192 / 4, row bands of 270 rows) with the split parity checks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?usage: r6_gloo4.sh TAG}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
  tests/test_gpu_dslice_lr.py -k "fuzz" > gpurun_out/${TAG}_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_tests.txt
SM_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 \
  --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --steps 8 --warmup 2 --no-variants --batch 32 \
  > gpurun_out/${TAG}_n4_gloo.json 2> gpurun_out/${TAG}_n4_gloo.err || { tail -20 gpurun_out/${TAG}_n4_gloo.err; exit 2; }
python - <<PY
import json
ln = [l for l in open("gpurun_out/${TAG}_n4_gloo.json") if "{" in l][-1]
d = json.loads(ln[ln.index("{"):])
print(json.dumps({k: d.get(k) for k in ("value", "rccl_world", "split_parity")}))
print(json.dumps(d["dslice"].get("check")), json.dumps(d["rowband"].get("check")))
print(json.dumps(d["cfg5_guided_lr"].get("dslice_guided_lr", {}).get("check")))
PY
