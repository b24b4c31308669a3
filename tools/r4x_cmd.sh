# round 4: full GPU suite and the bench line with 8-wave tiles for batch-1 mid-size launches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/r4x_pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/r4x_pytest_gpu.txt
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|Error" gpurun_out/r4x_pytest_gpu.txt | head -20; exit $rc; }
timeout -k 10 400 python bench.py > gpurun_out/r4x_bench.json 2> gpurun_out/r4x_bench.err || { tail -5 gpurun_out/r4x_bench.err; exit 5; }
python -c "
import json; d=json.load(open('gpurun_out/r4x_bench.json'))
print(d['value'], d['ms_per_step'], d['latency_ms_batch1'])
for k,v in d['variants'].items():
    if 'round trip' in k or 'segment' in k: print(k, v.get('ms_per_frame'))"
