"""Same-box A/B of the staged box path's three kernels (1080p D=128 r=5, one frame per call) for
several libsm_hip.so builds: rocprofv3 --kernel-trace --stats per build, average ns per kernel and
the HBM fraction of its algorithmic bytes.  usage: python tools/ab_staged.py lib1.so lib2.so ..."""
import csv, glob, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P, D = 1920 * 1080, 128
ALG = {"ad_volume_kernel": P * (D + 2), "box_sad_kernel": 3 * P * D, "volume_wta_kernel": 2 * P * D + P}
env = dict(os.environ, TMPDIR="/tmp")
for rnd in range(2):
    for lib in sys.argv[1:]:
        tag = os.path.basename(lib).replace(".so", "")
        d = os.path.join(ROOT, "gpurun_out", "ab_staged", f"{tag}_{rnd}")
        subprocess.run(["timeout", "-k", "10", "120", "rocprofv3", "--kernel-trace", "--stats", "-d", d, "-o", "k",
                        "--output-format", "csv", "--", sys.executable, os.path.join(ROOT, "tools", "kernel_driver.py"),
                        "--agg", "box-staged", "--batch", "1", "--iters", "20", "--lib", lib],
                       check=True, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        res = []
        for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                for k, b in ALG.items():
                    if k in row["Name"]:
                        ns = float(row["AverageNs"])
                        res.append(f"{k.split('_kernel')[0]} {ns / 1e3:7.1f} us {b / ns / 8e3:5.3f}")
        print(f"{tag:10s} " + " | ".join(sorted(res)), flush=True)
