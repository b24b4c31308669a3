set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "ad_volume or staged or sad_volume" --timeout 120 --timeout-method thread > gpurun_out/r3i_pytest.txt 2>&1; rc=$?; tail -2 gpurun_out/r3i_pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab_staged_kernels.py tools/ab/adv16old.so tools/ab/adv16.so tools/ab/adv64.so > gpurun_out/r3i_adv.txt 2>&1; cat gpurun_out/r3i_adv.txt
