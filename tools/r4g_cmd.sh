# round 4: host segment-tree phase times on the box's CPU (prefetch variants), guided + LR kernel split
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do for v in v0 v1 v2 v3; do tools/abv/st_host_bench_$v tools/abv/art_bgr.bin $v 20 >> gpurun_out/r4g_st_host.txt || exit 2; done; done
cat gpurun_out/r4g_st_host.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4g_glr -o glr --output-format csv -- python3 tools/kernel_driver.py --agg guided --lr --batch 32 --iters 5 > gpurun_out/r4g_glr.log 2>&1 || { tail -5 gpurun_out/r4g_glr.log; exit 3; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r4g_blr -o blr --output-format csv -- python3 tools/kernel_driver.py --agg box --lr --batch 32 --iters 5 > gpurun_out/r4g_blr.log 2>&1 || { tail -5 gpurun_out/r4g_blr.log; exit 4; }
python3 - <<'PY'
import csv, glob
for d in ("gpurun_out/r4g_glr", "gpurun_out/r4g_blr"):
    for f in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            print(d[-3:], row["Name"][:80], row["Calls"], round(float(row["AverageNs"]) / 1e3, 1), "us")
PY
