# round 4: box edge tiles mask only the pairs that need it (dfree) against tile-wide masking (dedge)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=tools/abv
SM_AB_B=32 timeout -k 10 400 python tools/ab.py $V/dedge.so $V/dfree.so > gpurun_out/r4m_ab.txt 2>&1 || { cat gpurun_out/r4m_ab.txt; exit 3; }
cat gpurun_out/r4m_ab.txt
SM_AB_LR=1 SM_AB_B=32 timeout -k 10 400 python tools/ab.py $V/dedge.so $V/dfree.so > gpurun_out/r4m_ab_lr.txt 2>&1 || { cat gpurun_out/r4m_ab_lr.txt; exit 3; }
cat gpurun_out/r4m_ab_lr.txt
SM_AB_B=8 SM_AB_W=3840 SM_AB_H=2160 SM_AB_D=192 timeout -k 10 400 python tools/ab.py $V/dedge.so $V/dfree.so > gpurun_out/r4m_ab_4k.txt 2>&1 || { cat gpurun_out/r4m_ab_4k.txt; exit 3; }
cat gpurun_out/r4m_ab_4k.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r4m_pytest.txt 2>&1; rc=$?
tail -3 gpurun_out/r4m_pytest.txt
exit $rc
