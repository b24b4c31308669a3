# round 4: segment-tree BFS on the device: GPU tests of the segment tree, A/B against the host BFS, kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_segtree.py -x -v --timeout 150 --timeout-method thread > gpurun_out/r4ac_pytest.txt 2>&1; rc=$?
tail -25 gpurun_out/r4ac_pytest.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/segtree_bfs_ab.py > gpurun_out/r4ac_ab.txt 2>&1 || { tail -5 gpurun_out/r4ac_ab.txt; exit 3; }
cat gpurun_out/r4ac_ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4ac_prof -o st --output-format csv -- python3 tools/segtree_timing.py > gpurun_out/r4ac_prof.log 2>&1 || { tail -5 gpurun_out/r4ac_prof.log; exit 4; }
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r4ac_prof/**/*kernel_stats.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        print(row["Name"][:70], row["Calls"], round(float(row["AverageNs"]) / 1e3, 1), "us", round(float(row["TotalDurationNs"]) / 1e6, 2), "ms total")
PY
