# round 4, fourth GPU pass: full GPU suite on the product (skew fix, AD 2x2), smoke, the staged roofline,
# bench line and a rocprofv3 kernel-stats summary of the bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/r4d_pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/r4d_pytest_gpu.txt
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/r4d_pytest_gpu.txt | head -20; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4d_smoke.txt 2>&1 && tail -1 gpurun_out/r4d_smoke.txt || exit 1
SM_TAG=_r4d timeout -k 10 300 python tools/staged_roofline.py > gpurun_out/r4d_staged.txt 2>&1 || { tail -5 gpurun_out/r4d_staged.txt; exit 4; }
python -c "
import json; d=json.load(open('gpurun_out/staged_roofline_1080p_r4d.json'))
for k,x in d['kernels'].items(): print(k, x['avg_ms'], x['frac_of_peak'], round(x['hbm_bytes_pmc']/x['algorithmic_bytes'],4))"
timeout -k 10 400 python bench.py > gpurun_out/r4d_bench.json 2> gpurun_out/r4d_bench.err || { tail -5 gpurun_out/r4d_bench.err; exit 5; }
python -c "
import json; d=json.load(open('gpurun_out/r4d_bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'])
for k,v in d['variants'].items():
    if 'round trip' in k or 'lr' in k or 'guided' in k or 'segment' in k: print(k, v)"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r4d_prof -o bench --output-format csv -- python3 bench.py --profile > gpurun_out/r4d_prof_bench.json 2> gpurun_out/r4d_prof_bench.err || { tail -5 gpurun_out/r4d_prof_bench.err; exit 6; }
echo PROFILE_OK
