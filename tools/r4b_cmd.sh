# round 4, second GPU pass: AD block-order / chunk sweep and SAD walk A/B (HIP events, then rocprof
# bytes), box + LR and tall-guided PMC counts, full GPU suite on the product
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=tools/abv
timeout -k 10 600 python tools/ab_staged_kernels.py $V/ad_o0.so $V/ad_o1.so $V/ad_o2g1.so $V/ad_o2g2.so $V/ad_o2g4.so $V/ad_o0s8.so $V/ad_o0s4.so $V/ad_o0s8r8.so $V/sad_z0.so $V/sad_z1.so > gpurun_out/r4b_ab_staged.txt 2>&1 || { tail -20 gpurun_out/r4b_ab_staged.txt; exit 3; }
cat gpurun_out/r4b_ab_staged.txt
for v in ad_o0 ad_o1 ad_o2g2 ad_o2g4 ad_o0s8 ad_o0s4 sad_z0; do
  SM_LIB=$V/$v.so SM_TAG=_$v timeout -k 10 300 python tools/staged_roofline.py > gpurun_out/r4b_staged_$v.txt 2>&1 || { tail -5 gpurun_out/r4b_staged_$v.txt; exit 4; }
  python -c "
import json; d=json.load(open('gpurun_out/staged_roofline_1080p_$v.json'))
for k,x in d['kernels'].items(): print('$v', k, x['avg_ms'], x['frac_of_peak'], round(x['hbm_bytes_pmc']/x['algorithmic_bytes'],4))"
done
SM_VALU_JOBS=box_lr_r5_1080p_d128_b32,box_lr_reduce_1080p_d128_b32 SM_TAG=_boxlr timeout -k 10 400 python tools/valu_counts.py > gpurun_out/r4b_valu_boxlr.txt 2>&1 || { tail -5 gpurun_out/r4b_valu_boxlr.txt; exit 5; }
cat gpurun_out/r4b_valu_boxlr.txt
SM_VALU_JOBS=guided_r5_1080p_d128_b32 SM_LIB=$V/g_t48.so SM_TAG=_tall timeout -k 10 400 python tools/valu_counts.py > gpurun_out/r4b_valu_tall.txt 2>&1 || { tail -5 gpurun_out/r4b_valu_tall.txt; exit 6; }
SM_VALU_JOBS=guided_r5_1080p_d128_b32 SM_TAG=_g32 timeout -k 10 400 python tools/valu_counts.py > gpurun_out/r4b_valu_g32.txt 2>&1 || { tail -5 gpurun_out/r4b_valu_g32.txt; exit 6; }
cat gpurun_out/r4b_valu_tall.txt gpurun_out/r4b_valu_g32.txt
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 150 --timeout-method thread > gpurun_out/r4b_pytest_gpu.txt 2>&1; rc=$?
tail -3 gpurun_out/r4b_pytest_gpu.txt
exit $rc
