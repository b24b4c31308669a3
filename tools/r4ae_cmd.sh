# round 4: host round trip without the unconditional start event (A/B), stage-timing test
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q  --timeout 120 --timeout-method thread > gpurun_out/r4ae_pytest.txt 2>&1; rc=$?
tail -2 gpurun_out/r4ae_pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/roundtrip_ab.py > gpurun_out/r4ae_rt.txt 2>&1 || { tail -5 gpurun_out/r4ae_rt.txt; exit 3; }
cat gpurun_out/r4ae_rt.txt
