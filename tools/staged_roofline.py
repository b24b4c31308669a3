"""Per-kernel HBM roofline of the staged box path (AD u8 -> SAD u16 -> WTA) at 1080p D=128 r=5,
8 frames per launch (one launch group of run_staged; SM_STAGED_FRAMES overrides).
Runs rocprofv3 kernel stats and one --pmc pass per counter (FETCH_SIZE, WRITE_SIZE) on
tools/kernel_driver.py --agg box-staged, and writes profiles/staged_roofline_1080p.json with each
kernel's duration, algorithmic bytes, measured HBM bytes (gfx950 FETCH correction x2) and GB/s."""
import csv, glob, json, os, statistics, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, D, r = 1920, 1080, 128, 5
F = int(os.environ.get("SM_STAGED_FRAMES", "8"))
P = W * H
out = os.path.join(ROOT, "gpurun_out", "staged_roofline")
env = dict(os.environ, TMPDIR="/tmp")
drv = [sys.executable, os.path.join(ROOT, "tools", "kernel_driver.py"), "--agg", "box-staged", "--batch", str(F),
       "--iters", "10"] + (["--lib", os.environ["SM_LIB"]] if os.environ.get("SM_LIB") else [])
out = out + os.environ.get("SM_TAG", "")
subprocess.run(["timeout", "-k", "10", "240", "rocprofv3", "--kernel-trace", "--stats", "-d", os.path.join(out, "kt"),
                "-o", "k", "--output-format", "csv", "--"] + drv, check=True, env=env,
               stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
dur = {}
for f in glob.glob(os.path.join(out, "kt", "**", "*kernel_stats.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        dur[row["Name"]] = float(row["AverageNs"]) * 1e-9
pmc = {}
for i, ctr in enumerate(["FETCH_SIZE", "WRITE_SIZE"]):
    d = os.path.join(out, f"p{i}")
    subprocess.run(["timeout", "-k", "10", "240", "rocprofv3", "--pmc", ctr, "-d", d, "-o", "pmc", "--output-format",
                    "csv", "--"] + drv, check=True, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            pmc.setdefault(row["Kernel_Name"], {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
alg = {"ad_volume_kernel": F * P * (D + 2), "box_sad_kernel": F * 3 * P * D, "volume_wta_kernel": F * (2 * P * D + P)}
res = {"workload": [W, H, D, r], "frames_per_launch": F, "peak_GBs": 8000.0, "achievable_GBs_guide": 6300.0, "kernels": {}}
for name, t in dur.items():
    key = next((k for k in alg if k in name), None)
    if key is None:
        continue
    c = {k: statistics.median(v) for k, v in pmc.get(name, {}).items()}
    hbm = 2 * c.get("FETCH_SIZE", 0.0) * 1024 + c.get("WRITE_SIZE", 0.0) * 1024
    res["kernels"][key] = {"avg_ms": round(t * 1e3, 4), "algorithmic_bytes": alg[key],
                           "achieved_GBs": round(alg[key] / t / 1e9, 1),
                           "frac_of_peak": round(alg[key] / t / 8e12, 3),
                           "hbm_bytes_pmc": round(hbm), "hbm_GBs_pmc": round(hbm / t / 1e9, 1)}
tot = sum(v["avg_ms"] for v in res["kernels"].values())
res["staged_ms_per_frame"] = round(tot / F, 4)
os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
json.dump(res, open(os.path.join(ROOT, "gpurun_out", "staged_roofline_1080p%s.json" % os.environ.get("SM_TAG", "")), "w"),
          indent=1)
print(json.dumps(res, indent=1))
