# round 4, final pass on the product: full GPU suite, smoke, bench line, rocprofv3 kernel stats of the bench,
# staged roofline, PMC counts of the compute-bound kernels (VALU roofline input)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/r4ag_pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/r4ag_pytest_gpu.txt
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/r4ag_pytest_gpu.txt | head -20; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4ag_smoke.txt 2>&1 && tail -1 gpurun_out/r4ag_smoke.txt || exit 1
timeout -k 10 600 python tools/valu_counts.py > gpurun_out/r4ag_valu.txt 2>&1 || { tail -5 gpurun_out/r4ag_valu.txt; exit 2; }
SM_TAG=_r4ag timeout -k 10 300 python tools/staged_roofline.py > gpurun_out/r4ag_staged.txt 2>&1 || { tail -5 gpurun_out/r4ag_staged.txt; exit 4; }
timeout -k 10 400 python bench.py --valu-json gpurun_out/valu_counts.json > gpurun_out/r4ag_bench.json 2> gpurun_out/r4ag_bench.err || { tail -5 gpurun_out/r4ag_bench.err; exit 5; }
python -c "
import json; d=json.load(open('gpurun_out/r4ag_bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'])
for k,v in d['variants'].items():
    if 'round trip' in k or 'lr' in k or 'guided' in k or 'segment' in k: print(k, v)"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r4ag_prof -o bench --output-format csv -- python3 bench.py --profile --valu-json gpurun_out/valu_counts.json > gpurun_out/r4ag_prof_bench.json 2> gpurun_out/r4ag_prof_bench.err || { tail -5 gpurun_out/r4ag_prof_bench.err; exit 6; }
echo PROFILE_OK
