# round 4, first GPU pass: full GPU suite, smoke, guided A/B of the M0 change, bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/r4a_pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/r4a_pytest_gpu.txt
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/r4a_pytest_gpu.txt | head -30; [ $rc -eq 1 ] || exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a_smoke.txt 2>&1 && tail -1 gpurun_out/r4a_smoke.txt || exit 1
SM_AB_AGG=guided SM_AB_B=32 timeout -k 10 400 python tools/ab.py tools/abv/g_r3.so tools/abv/g_t48L.so tools/abv/g_t48.so > gpurun_out/r4a_ab_guided.txt 2>&1 || { cat gpurun_out/r4a_ab_guided.txt; exit 3; }
cat gpurun_out/r4a_ab_guided.txt
SM_AB_AGG=guided SM_AB_LR=1 SM_AB_B=32 timeout -k 10 400 python tools/ab.py tools/abv/g_r3.so tools/abv/g_t48L.so tools/abv/g_t48.so > gpurun_out/r4a_ab_guided_lr.txt 2>&1 || { cat gpurun_out/r4a_ab_guided_lr.txt; exit 3; }
cat gpurun_out/r4a_ab_guided_lr.txt
for v in st_old st_new; do
  SM_LIB=tools/abv/$v.so SM_TAG=_$v timeout -k 10 400 python tools/staged_roofline.py > gpurun_out/r4a_staged_$v.txt 2>&1 || { tail -5 gpurun_out/r4a_staged_$v.txt; exit 4; }
  python -c "
import json; d=json.load(open('gpurun_out/staged_roofline_1080p_$v.json'))
for k,v in d['kernels'].items(): print('$v', k, v['avg_ms'], v['frac_of_peak'], round(v['hbm_bytes_pmc']/v['algorithmic_bytes'],4))"
done
timeout -k 10 300 python bench.py > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err && python -c "
import json; d=json.load(open('gpurun_out/r4a_bench.json'))
print(d['value'], d['ms_per_step'])
for k,v in d['variants'].items():
    if 'round trip' in k: print(k, v)"
exit $rc
