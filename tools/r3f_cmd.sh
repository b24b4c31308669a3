set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "pinned or zero_copy or reference_entry" --timeout 120 --timeout-method thread > gpurun_out/r3f_pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/r3f_pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/roundtrip_ab.py > gpurun_out/r3f_roundtrip.txt 2>&1; cat gpurun_out/r3f_roundtrip.txt
SM_LIB=tools/ab/g3off.so SM_TAG=_r3_before timeout -k 10 600 python tools/valu_counts.py > gpurun_out/r3f_valu_before.txt 2>&1 && SM_TAG=_r3_after timeout -k 10 600 python tools/valu_counts.py > gpurun_out/r3f_valu_after.txt 2>&1; tail -2 gpurun_out/r3f_valu_after.txt
