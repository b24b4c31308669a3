# round 4: segment-tree A/B (edge chunks + page-locked trees vs before), alternated rounds
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in st_r4pre st_r4new st_r4new2; do
    SM_LIB=tools/abv/$v.so timeout -k 10 300 python tools/segtree_timing.py 2>&1 | grep Art >> gpurun_out/r4f_segtree_ab.txt || exit 3
  done
done
cat gpurun_out/r4f_segtree_ab.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_segtree.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r4f_pytest_segtree.txt 2>&1; rc=$?
tail -2 gpurun_out/r4f_pytest_segtree.txt
exit $rc
