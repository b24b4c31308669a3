# round 4: guided right reduce with a fixed trip count (rrvec) against the covering-tile loop (rrold)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
V=tools/abv
SM_AB_AGG=guided SM_AB_LR=1 SM_AB_B=32 timeout -k 10 400 python tools/ab.py $V/rrold.so $V/rrvec.so > gpurun_out/r4o_ab.txt 2>&1 || { cat gpurun_out/r4o_ab.txt; exit 3; }
cat gpurun_out/r4o_ab.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4o_glr -o glr --output-format csv -- python3 tools/kernel_driver.py --agg guided --lr --batch 32 --iters 5 > gpurun_out/r4o_glr.log 2>&1 || { tail -5 gpurun_out/r4o_glr.log; exit 4; }
python3 - <<'PY'
import csv, glob
for f in glob.glob("gpurun_out/r4o_glr/**/*kernel_stats.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        print(row["Name"][:80], row["Calls"], round(float(row["AverageNs"]) / 1e3, 1), "us")
PY
timeout -k 10 400 python -u -m pytest tests/test_gpu_guided.py tests/test_gpu_parity.py tests/test_gpu_segtree.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r4o_pytest.txt 2>&1; rc=$?
tail -3 gpurun_out/r4o_pytest.txt
exit $rc
