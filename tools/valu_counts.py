"""VALU / LDS instruction counts per launch of the bench's compute-bound kernels, for bench.py's
`roofline` (bound "valu").  One rocprofv3 --pmc pass per workload (SQ counters only, no tracing
domains: MI355X_MICROARCH.md §PMC), on tools/kernel_driver.py with the bench's exact configuration
(1080p D=128 r=5; the box kernel at the headline's 128 frames per launch, guided at 32).  SQ_INSTS_VALU is a chip total of wave64 instructions and
does not depend on timing, so bench.py divides it by the live HIP-event kernel time.

    python tools/valu_counts.py            # writes profiles/valu_counts.json
"""
import csv, glob, json, os, statistics, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CTRS = "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
# name, kernel-name substring, driver args; workload = [W, H, D, r, frames per launch]
# name, kernel-name substring (rocprof's demangled name), driver args, workload, mangled-name substring (the
# symbol whose machine code tools/codeobj.py hashes into the entry: bench.py reports frac null when the library
# it loads carries other code for that kernel)
JOBS = (
    ("box_r5_1080p_d128_b128", "box_match_kernel<5, 128, false, 4>", ["--agg", "box", "--batch", "128"],
     [1920, 1080, 128, 5, 128], "box_match_kernelILi5ELi128ELb0ELi4E"),
    ("guided_r5_1080p_d128_b32", "guided_fused_kernel<5, false", ["--agg", "guided", "--batch", "32"],
     [1920, 1080, 128, 5, 32], "guided_fused_kernelILi5ELb0E"),
    ("guided_lr_r5_1080p_d128_b32", "guided_fused_kernel<5, true", ["--agg", "guided", "--lr", "--batch", "32"],
     [1920, 1080, 128, 5, 32], "guided_fused_kernelILi5ELb1E"),
    # box + LR: the right-view matcher and its reduce, from the same runs
    ("box_lr_r5_1080p_d128_b32", "box_match_kernel<5, 128, true", ["--agg", "box", "--lr", "--batch", "32"],
     [1920, 1080, 128, 5, 32], "box_match_kernelILi5ELi128ELb1E"),
    ("box_lr_reduce_1080p_d128_b32", "right_reduce_lr_vec_kernel", ["--agg", "box", "--lr", "--batch", "32"],
     [1920, 1080, 128, 5, 32], "right_reduce_lr_vec_kernelILi4E"),
)
# SM_VALU_JOBS=name1,name2: only those jobs
if os.environ.get("SM_VALU_JOBS"):
    JOBS = tuple(j for j in JOBS if j[0] in os.environ["SM_VALU_JOBS"].split(","))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import codeobj  # noqa: E402


# issue / wait breakdown of the guided kernels: wave cycles spent waiting at
# s_waitcnt / barriers (SQ_WAIT_ANY), stalled on issue (SQ_WAIT_INST_ANY; SQ_WAIT_INST_LDS its LDS part)
# and issuing (SQ_ACTIVE_INST_ANY), which add up to SQ_WAVE_CYCLES
WAIT_CTRS = "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"


def main():
    env = dict(os.environ, TMPDIR="/tmp")
    tag = os.environ.get("SM_TAG", "")
    res = {"counters": CTRS.split(), "note": "chip totals per launch (median over launches); SQ_INSTS_VALU counts "
           "wave64 VALU instructions, SQ_LDS_IDX_ACTIVE LDS-array cycles summed over CUs", "kernels": {}}
    lib = os.environ.get("SM_LIB") or codeobj.default_lib()
    for name, kname, args, wl, sym in JOBS:
        d = os.path.join(ROOT, "gpurun_out", "valu_counts" + tag, name)
        cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc"] + CTRS.split() + [
            "-d", d, "-o", "pmc", "--output-format", "csv", "--", sys.executable,
            os.path.join(ROOT, "tools", "kernel_driver.py"), "--iters", "3"] + args
        if os.environ.get("SM_LIB"):
            cmd += ["--lib", os.environ["SM_LIB"]]
        subprocess.run(cmd, check=True, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        vals = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if kname in row["Kernel_Name"]:
                    vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
        if "guided" in name or "box_lr" in name or name.startswith("box_r5"):   # + the headline
            d2 = d + "_wait"
            cmd2 = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc"] + WAIT_CTRS.split() + [
                "-d", d2, "-o", "pmc", "--output-format", "csv", "--", sys.executable,
                os.path.join(ROOT, "tools", "kernel_driver.py"), "--iters", "3"] + args
            if os.environ.get("SM_LIB"):
                cmd2 += ["--lib", os.environ["SM_LIB"]]
            subprocess.run(cmd2, check=True, env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
            for f in glob.glob(os.path.join(d2, "**", "*counter_collection.csv"), recursive=True):
                for row in csv.DictReader(open(f)):
                    if kname in row["Kernel_Name"]:
                        vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
        med = {k: statistics.median(v) for k, v in vals.items()}
        if "SQ_WAVE_CYCLES" in med and med["SQ_WAVE_CYCLES"] > 0:
            wc = med["SQ_WAVE_CYCLES"]
            med["share_wait_any"] = med.get("SQ_WAIT_ANY", 0) / wc
            med["share_wait_inst_any"] = med.get("SQ_WAIT_INST_ANY", 0) / wc
            med["share_active_inst_any"] = med.get("SQ_ACTIVE_INST_ANY", 0) / wc
        res["kernels"][name] = {"kernel": kname, "workload": wl, "per_launch": med, "code_symbol": sym,
                                "code_sha256": codeobj.kernel_sha256(lib, sym)}
        print(name, json.dumps(med), flush=True)
    out = os.path.join(ROOT, "gpurun_out", "valu_counts%s.json" % tag)
    json.dump(res, open(out, "w"), indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main()
