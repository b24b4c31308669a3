# round 4, third GPU pass: box + LR right-key row skew A/B (1080p and 4K), AD order-3 / low-split sweep,
# box + LR PMC with the skew, full GPU suite on the product
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=tools/abv
SM_AB_LR=1 SM_AB_B=32 timeout -k 10 400 python tools/ab.py $V/skew0.so $V/skew1.so > gpurun_out/r4c_ab_skew.txt 2>&1 || { cat gpurun_out/r4c_ab_skew.txt; exit 3; }
cat gpurun_out/r4c_ab_skew.txt
SM_AB_LR=1 SM_AB_B=8 SM_AB_W=3840 SM_AB_H=2160 SM_AB_D=192 timeout -k 10 400 python tools/ab.py $V/skew0.so $V/skew1.so > gpurun_out/r4c_ab_skew_4k.txt 2>&1 || { cat gpurun_out/r4c_ab_skew_4k.txt; exit 3; }
cat gpurun_out/r4c_ab_skew_4k.txt
timeout -k 10 600 python tools/ab_staged_kernels.py $V/ad_o0.so $V/ad_o0s8.so $V/ad_o3.so $V/ad_o3s8.so $V/ad_o3s4.so $V/ad_o0s2.so $V/ad_o0s2r2.so $V/ad_o0s4r2.so > gpurun_out/r4c_ab_staged.txt 2>&1 || { tail -20 gpurun_out/r4c_ab_staged.txt; exit 4; }
cat gpurun_out/r4c_ab_staged.txt
for v in ad_o0 ad_o0s8 ad_o3 ad_o3s8 ad_o3s4 ad_o0s2 ad_o0s2r2 ad_o0s4r2; do
  SM_LIB=$V/$v.so SM_TAG=_$v timeout -k 10 300 python tools/staged_roofline.py > gpurun_out/r4c_staged_$v.txt 2>&1 || { tail -5 gpurun_out/r4c_staged_$v.txt; exit 5; }
  python -c "
import json; d=json.load(open('gpurun_out/staged_roofline_1080p_$v.json'))
x=d['kernels']['ad_volume_kernel']; print('$v', 'ad_volume_kernel', x['avg_ms'], x['frac_of_peak'], round(x['hbm_bytes_pmc']/x['algorithmic_bytes'],4))"
done
SM_VALU_JOBS=box_lr_r5_1080p_d128_b32 SM_TAG=_boxlr_skew timeout -k 10 400 python tools/valu_counts.py > gpurun_out/r4c_valu_boxlr.txt 2>&1 || { tail -5 gpurun_out/r4c_valu_boxlr.txt; exit 6; }
cat gpurun_out/r4c_valu_boxlr.txt
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/r4c_pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/r4c_pytest_gpu.txt
exit $rc
