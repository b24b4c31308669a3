"""Collect HBM traffic for the bench configuration with rocprofv3 PMC passes (one counter group
per pass, no tracing domains), per MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of the bytes of
wide coalesced streams on gfx950 (doubled below; other widths are uncalibrated, so the corrected
figure is an upper bound), WRITE_SIZE is exact for 16-B stores.  Writes profiles/pmc_<tag>.json."""
import csv, glob, json, os, subprocess, sys, statistics
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1] if len(sys.argv) > 1 else "box_r5_1080p"
W, H, D, r = 1920, 1080, 128, 5
B = int(os.environ.get("SM_PMC_BATCH", "128"))   # bench.py's default frames per step
out = os.path.join(ROOT, "gpurun_out", "pmc_" + tag)
env = dict(os.environ, TMPDIR="/tmp")
vals = {}
for i, ctr in enumerate(["FETCH_SIZE", "WRITE_SIZE", "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"]):
    d = os.path.join(out, f"p{i}")
    cmd = ["timeout", "-k", "10", "240", "rocprofv3", "--pmc"] + ctr.split() + ["-d", d, "-o", "pmc", "--output-format", "csv",
           "--", sys.executable, os.path.join(ROOT, "tools", "kernel_driver.py"), "--iters", "10", "--batch", str(B)]
    subprocess.run(cmd, check=True, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "box_match_kernel" in row["Kernel_Name"]:
                vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
med = {k: statistics.median(v) for k, v in vals.items()}
fetch_kb, write_kb = med.get("FETCH_SIZE", 0.0), med.get("WRITE_SIZE", 0.0)
res = {
    "workload": [W, H, D, r, B],
    "kernel": f"box_match_kernel<{r}, 128>",
    "counters_median_per_launch": med,
    "fetch_bytes_raw": fetch_kb * 1024, "write_bytes": write_kb * 1024,
    "hbm_bytes_per_launch": round(2 * fetch_kb * 1024 + write_kb * 1024),
    "hbm_bytes_per_launch_uncorrected": round(fetch_kb * 1024 + write_kb * 1024),
    "note": "FETCH_SIZE doubled per the gfx950 calibration for wide coalesced reads; the kernel's loads are "
            "4-B dwords (uncalibrated width), so hbm_bytes_per_launch is an upper bound. Compulsory: "
            f"{3 * W * H * B} B (L+R in, disparity out).",
}
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "profiles", f"pmc_{tag}.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
