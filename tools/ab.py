"""Interleaved A/B timing of libsm_hip.so builds in ONE process per lib, rounds alternated.
usage: python tools/ab.py lib1.so lib2.so ... [--rounds 3]"""
import subprocess, sys, os, json, statistics
libs = [a for a in sys.argv[1:] if a.endswith(".so")]
rounds = 3
res = {l: [] for l in libs}
here = os.path.dirname(os.path.abspath(__file__))
for r in range(rounds):
    for l in libs:
        out = subprocess.run([sys.executable, os.path.join(here, "ablate.py"), l], capture_output=True, text=True, timeout=200)
        line = [x for x in out.stdout.splitlines() if "ms/frame" in x]
        if not line:
            print(out.stdout, out.stderr); sys.exit(1)
        res[l].append(float(line[-1].split()[-1]) * 1000)
for l in libs:
    print(f"{os.path.basename(l):24s} us/frame  median {statistics.median(res[l]):7.2f}  min {min(res[l]):7.2f}  all {[round(v,1) for v in res[l]]}")
