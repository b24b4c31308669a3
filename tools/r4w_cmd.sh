# round 4: batch-1 latency with 8-wave tiles for small launches (SM_BOX_MID) against 4-wave tiles
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/latency_ab.py "SM_BOX_MID=0" "SM_BOX_MID=1 SM_BOX_MID_MAX=8" "SM_BOX_MID=1 SM_BOX_MID_MAX=3" "SM_BOX_MID=0" > gpurun_out/r4w_lat.txt 2>&1 || { tail -5 gpurun_out/r4w_lat.txt; exit 3; }
grep -v amdgpu.ids gpurun_out/r4w_lat.txt
