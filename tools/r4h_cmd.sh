# round 4: staged pipeline A/B of the AD band height at 2 d chunks (the SAD kernel's speed follows it)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python tools/ab_staged_kernels.py tools/abv/ad_s2r4.so tools/abv/ad_s2r2.so tools/abv/ad_s2r4_z0.so --rounds 5 > gpurun_out/r4h_ab_staged.txt 2>&1 || { tail -20 gpurun_out/r4h_ab_staged.txt; exit 3; }
cat gpurun_out/r4h_ab_staged.txt
