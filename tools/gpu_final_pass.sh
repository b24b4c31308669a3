#!/bin/bash
# Round-end evidence on the product in one GPU call (replaces the per-call r3*/r4*_cmd.sh copies):
#   tools/gpu_final_pass.sh TAG [STEPS]
# STEPS (default "tests,smoke,valu,staged,bench,prof") picks the steps, in this order:
#   tests   full `pytest -m gpu` suite            -> gpurun_out/TAG_pytest_gpu.txt
#   smoke   __graft_entry__.smoke()               -> gpurun_out/TAG_smoke.txt
#   valu    SQ counters of the compute-bound kernels (tools/valu_counts.py, VALU roofline input)
#   staged  HBM roofline of the staged AD / SAD / WTA kernels (tools/staged_roofline.py, SM_TAG=_TAG)
#   bench   bench.py with the fresh counts        -> gpurun_out/TAG_bench.json
#   prof    rocprofv3 --kernel-trace --stats of `bench.py --profile` -> gpurun_out/TAG_prof/
# Every GPU step has its own time limit, and the chain stops at the first failure (exit code = step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:?usage: gpu_final_pass.sh TAG [STEPS]}
STEPS=",${2:-tests,smoke,valu,staged,bench,prof},"
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out/${TAG}
has() { [[ "$STEPS" == *",$1,"* ]]; }
if has tests; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > ${O}_pytest_gpu.txt 2>&1; rc=$?
  tail -3 ${O}_pytest_gpu.txt
  [ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" ${O}_pytest_gpu.txt | head -20; exit 1; }
fi
if has smoke; then
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.txt 2>&1 && tail -1 ${O}_smoke.txt || exit 2
fi
VJ=""
if has valu; then
  timeout -k 10 600 python tools/valu_counts.py > ${O}_valu.txt 2>&1 || { tail -5 ${O}_valu.txt; exit 3; }
  VJ="--valu-json gpurun_out/valu_counts.json"
fi
if has staged; then
  SM_TAG=_${TAG} timeout -k 10 300 python tools/staged_roofline.py > ${O}_staged.txt 2>&1 || { tail -5 ${O}_staged.txt; exit 4; }
fi
if has bench; then
  timeout -k 10 500 python bench.py $VJ > ${O}_bench.json 2> ${O}_bench.err || { tail -5 ${O}_bench.err; exit 5; }
  python -c "
import json; d=json.load(open('${O}_bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'])
for k,v in d['variants'].items():
    if 'round trip' in k or 'lr' in k or 'guided' in k or 'segment' in k: print(k, v)"
fi
if has prof; then
  timeout -k 10 500 rocprofv3 --kernel-trace --stats -d ${O}_prof -o bench --output-format csv -- python3 bench.py --profile $VJ > ${O}_prof_bench.json 2> ${O}_prof_bench.err || { tail -5 ${O}_prof_bench.err; exit 6; }
  echo PROFILE_OK
fi
exit 0
