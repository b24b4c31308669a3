"""VALU instruction mix of a kernel's loops from the gfx950 assembly (`make -C gpu_stereo_matching_amd/csrc asm`):
per loop (a label reached by a backward s_cbranch / s_branch), the VALU opcodes and their issue-cycle weight
from the measured per-instruction rates on this part (profiles/microbench/r02_valu_issue_cycles_pmc.txt:
32-bit-encoded VOP1/VOP2 ~2.37 cycles per wave64 instruction per SIMD, VOP3 / VOP3P / DPP-free 64-bit
encodings ~4.25, conversions 3.9, v_cndmask 3.24).

    python tools/isa_mix.py build/bm_box.s 'box_match_kernelILi5ELi128ELb0ELi4E'
    python tools/isa_mix.py --json build/bm_box.s 'box_match_kernelILi5ELi128ELb0ELi4E' > profiles/isa_mix_box.json
"""
import collections
import re
import sys

# ops measured at ~2.37 cycles (32-bit encodings: VOP1 / VOP2 with VGPR, SGPR or inline-constant operands)
FAST = {"v_add_u32", "v_sub_u32", "v_subrev_u32", "v_add_f32", "v_sub_f32", "v_mul_f32", "v_fmac_f32", "v_fma_f32",
        "v_and_b32", "v_or_b32", "v_xor_b32", "v_lshlrev_b32", "v_lshrrev_b32", "v_ashrrev_i32", "v_mov_b32",
        "v_add_co_u32", "v_sub_co_u32", "v_subrev_co_u32", "v_addc_co_u32", "v_max_f32", "v_min_f32", "v_not_b32",
        "v_mac_f32", "v_readfirstlane_b32", "v_mul_u32_u24", "v_mul_i32_i24"}
SLOW_VOP3 = 4.25
CVT = 3.9


def weight(op, operands):
    if op.startswith("v_cvt"):
        return CVT
    if op.startswith("v_cndmask"):
        return 3.24
    base = op.replace("_e32", "").replace("_e64", "")
    if op.endswith("_e64"):
        return SLOW_VOP3
    if base in ("v_min_u32", "v_max_u32", "v_min_i32", "v_max_i32"):
        return SLOW_VOP3   # measured MinI 4.24
    if base in ("v_mul_u32_u24", "v_mul_i32_i24", "v_mad_u32_u24", "v_mad_i32_i24"):
        return SLOW_VOP3   # measured 4.19-4.27
    if base in FAST:
        # a 32-bit literal operand forces the 64-bit form
        if re.search(r"0x[0-9a-f]{3,}", operands):
            return SLOW_VOP3
        return 2.37
    return SLOW_VOP3


def kernel_lines(path, name):
    out, on = [], False
    for ln in open(path):
        if re.match(r"^_Z\S*" + re.escape(name) + r"\S*:", ln):
            on = True
            continue
        if on and ln.startswith("\t.section"):
            break
        if on:
            out.append(ln.rstrip("\n"))
    return out


def loop_blocks(lines, a, b):
    """basic blocks of lines[a..b]: (label, VALU count, issue cycles, opcode Counter)"""
    blocks, cur = [], None
    for ln in lines[a:b + 1]:
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            cur = [m.group(1), 0, 0.0, collections.Counter()]
            blocks.append(cur)
            continue
        m = re.match(r"^\s+(v_\w+)\s*(.*)", ln)
        if m and cur is not None:
            cur[1] += 1
            cur[2] += weight(m.group(1), m.group(2))
            cur[3][m.group(1)] += 1
    return blocks


def hot_path(path, name, exclude_op="v_cmp_lt_i32_e64"):
    """The largest loop's blocks without `exclude_op` (for box_match_kernel: the unmasked pair iteration,
    the masked phase-H blocks compare every output's d against its validity limit): VALU per iteration,
    issue cycles, average cycles per VALU instruction and the opcode mix."""
    lines = kernel_lines(path, name)
    labels = {m.group(1): i for i, ln in enumerate(lines) for m in [re.match(r"^(\.LBB\S+):", ln)] if m}
    loops = []
    for i, ln in enumerate(lines):
        m = re.match(r"^\s+s_(cbranch_\w+|branch)\s+(\.LBB\S+)", ln)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            loops.append((labels[m.group(2)], i))
    a, b = max(loops, key=lambda t: t[1] - t[0])
    n, cyc, mix = 0, 0.0, collections.Counter()
    for lab, cnt, c, ops in loop_blocks(lines, a, b):
        if exclude_op in ops:
            continue
        n += cnt
        cyc += c
        mix += ops
    return {"kernel": name, "valu_per_iteration": n, "issue_cycles_per_iteration": round(cyc, 1),
            "avg_cycles_per_valu": round(cyc / n, 4), "mix": dict(mix.most_common()),
            "excluded_blocks_with": exclude_op}


def main():
    if sys.argv[1] == "--json":
        import json
        print(json.dumps(hot_path(sys.argv[2], sys.argv[3]), indent=1))
        return
    path, name = sys.argv[1], sys.argv[2]
    lines = kernel_lines(path, name)
    labels = {}
    for i, ln in enumerate(lines):
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            labels[m.group(1)] = i
    loops = []
    for i, ln in enumerate(lines):
        m = re.match(r"^\s+s_(cbranch_\w+|branch)\s+(\.LBB\S+)", ln)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            loops.append((labels[m.group(2)], i))
    total = collections.Counter()
    for ln in lines:
        m = re.match(r"^\s+(v_\w+)\s*(.*)", ln)
        if m:
            total[m.group(1)] += 1
    print(f"kernel {name}: {sum(total.values())} VALU instructions in the whole body, {len(loops)} loops")
    for a, b in sorted(loops, key=lambda t: -(t[1] - t[0])):
        mix = collections.Counter()
        cyc = 0.0
        for ln in lines[a:b + 1]:
            m = re.match(r"^\s+(v_\w+)\s*(.*)", ln)
            if m:
                mix[m.group(1)] += 1
                cyc += weight(m.group(1), m.group(2))
        n = sum(mix.values())
        if n == 0:
            continue
        nlds = sum(1 for ln in lines[a:b + 1] if re.match(r"^\s+ds_", ln))
        nsalu = sum(1 for ln in lines[a:b + 1] if re.match(r"^\s+s_", ln))
        print(f"loop lines {a}-{b}: {n} VALU, {cyc:.0f} issue cycles (avg {cyc / n:.2f}), LDS {nlds}, SALU {nsalu}")
        for op, c in mix.most_common(25):
            print(f"   {c:5d} {op}")
        break   # the largest loop only


if __name__ == "__main__":
    main()
