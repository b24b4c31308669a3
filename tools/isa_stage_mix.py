"""Per-stage VALU mix of guided_fused_kernel: build bm_guided.hip with SM_G_MARK=1, whose
`;@stage NAME` / `;@stage end` comments bracket S1V, S1H, S2V and S2H in the ISA, and sum each stage's VALU
instructions and issue cycles (tools/isa_mix.py's measured weights) per instance.  Counts are static, per wave and
per disparity: one instance of a stage's code is what one wave executes for one d (the stages are fully unrolled).

    python tools/isa_stage_mix.py [--json] [R] [RIGHT]    # default R = 5, RIGHT = 0
    SM_G_FLAGS="-DSM_G_ACC=1" python tools/isa_stage_mix.py   # a variant's mix
"""
import collections
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
from isa_mix import kernel_lines, weight  # noqa: E402


def build_marked(out):
    src = os.path.join(ROOT, "gpu_stereo_matching_amd", "csrc", "bm_guided.hip")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-fvisibility=hidden",
                    "-DSM_G_MARK=1", *os.environ.get("SM_G_FLAGS", "").split(), "--cuda-device-only", "-S", src,
                    "-o", out], check=True,
                   stderr=subprocess.DEVNULL)


def stage_mix(path, name):
    lines = kernel_lines(path, name)
    inst, cur = [], None
    for ln in lines:
        m = re.search(r";@stage (\w+)", ln)
        if m:
            if m.group(1) == "end":
                cur = None
            else:
                cur = {"stage": m.group(1), "valu": 0, "cycles": 0.0, "lds": 0, "mix": collections.Counter()}
                inst.append(cur)
            continue
        if cur is None:
            continue
        m = re.match(r"^\s+(v_\w+)\s*(.*)", ln)
        if m:
            cur["valu"] += 1
            cur["cycles"] += weight(m.group(1), m.group(2))
            cur["mix"][m.group(1)] += 1
        elif re.match(r"^\s+ds_", ln):
            cur["lds"] += 1
    return inst


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    R = int(args[0]) if args else 5
    right = int(args[1]) if len(args) > 1 else 0
    out = os.path.join(ROOT, "gpu_stereo_matching_amd", "csrc", "build", "bm_guided_marked.s")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    build_marked(out)
    name = f"guided_fused_kernelILi{R}ELb{right}E"
    inst = stage_mix(out, name)
    # the d loop's instances: the largest instance of each stage (stats / masked variants are smaller or equal)
    best = {}
    for i in inst:
        if i["stage"] not in best or i["valu"] > best[i["stage"]]["valu"]:
            best[i["stage"]] = i
    res = {"kernel": name, "radius": R, "right_view": bool(right),
           "note": "static VALU and LDS instructions per wave and disparity for each stage (largest instance: the "
                   "masked / limited variant), issue cycles weighted as tools/isa_mix.py; SM_G_MARK=1 build",
           "instances": [{k: (v if k != "mix" else None) for k, v in i.items() if k != "mix"} for i in inst],
           "stages": {k: {"valu": v["valu"], "issue_cycles": round(v["cycles"], 1), "lds": v["lds"],
                          "avg_cycles_per_valu": round(v["cycles"] / max(v["valu"], 1), 3),
                          "mix": dict(v["mix"].most_common())} for k, v in best.items()}}
    # per tile and d at the phase-1 roles (R <= 5 left view: S1V and S2V on 2 waves each, S1H and S2H on all 4):
    # the interior instance of S1V (no column masks) is the smallest non-stats one
    s1v_int = sorted(i["valu"] for i in inst if i["stage"] == "S1V")[1:2] or [best["S1V"]["valu"]]
    waves = {"S1V": 2, "S2V": 2, "S1H": 4, "S2H": 4}
    per = {k: waves[k] * (s1v_int[0] if k == "S1V" else best[k]["valu"]) for k in waves if k in best}
    TW, TH = 64 - 4 * R, 32
    res["per_tile_and_d"] = {
        "wave_instructions": per, "total": sum(per.values()), "outputs": TW * TH,
        "lane_ops_per_output_and_d": {k: round(v * 64 / (TW * TH), 2) for k, v in per.items()},
        "lane_ops_per_output_and_d_total": round(sum(per.values()) * 64 / (TW * TH), 2),
        "halo": {"P_region_over_outputs": round(64 * (TH + 4 * R) / (TW * TH), 3),
                 "A_region_over_outputs": round((TW + 2 * R) * (TH + 2 * R) / (TW * TH), 3),
                 "S2V_region_over_outputs": round(64 * TH / (TW * TH), 3)},
        "algorithmic_minimum_note": "about 25 VALU per (pixel, d) with no halo and no idle lanes: AD 1, packed "
                                    "vertical sum 2, horizontal sums 5 (packed add/sub + Sp unpack), SIp 1, a and b 7, "
                                    "float box sums of a and b 8, q + WTA 3"}
    if "--json" in sys.argv:
        print(json.dumps(res, indent=1))
    else:
        for k, v in res["stages"].items():
            print(k, v["valu"], "VALU", v["issue_cycles"], "cycles", v["lds"], "LDS",
                  list(v["mix"].items())[:12])


if __name__ == "__main__":
    main()
