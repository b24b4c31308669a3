"""Static check of the gfx950 ISA: every s_barrier that follows an inline-asm LDS store
(ds_write_addtid_b32 / ds_write_b64, which the compiler's wait-count pass does not track) must be
preceded by an s_waitcnt lgkmcnt(0) issued after that store.  A missing wait lets another wave read
the rows before they land (a rare, timing-dependent wrong result).

Second check: every ds_write_addtid_b32 reads M0, so it must follow the
`s_mov_b32 m0, ...; s_nop 0` of its own asm statement with nothing but other add-TID stores in
between; a compiler-generated M0 write in the gap would redirect the stores.

usage: python tools/check_lds_barriers.py [source.hip ...]   (default: every csrc/*.hip)"""
import glob, os, subprocess, sys, tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASM_STORES = ("ds_write_addtid", "ds_write_b64")


def unguarded_barriers(asm_text: str):
    bad, total, waited, kernel = [], 0, True, "?"
    for line in asm_text.split("\n"):
        t = line.strip()
        if line and not line[0].isspace() and t.endswith(":") and not t.startswith("."):
            kernel = t.split(":")[0]
        if t.startswith(ASM_STORES):
            waited = False
        elif t.startswith("s_waitcnt") and "lgkmcnt(0)" in t:
            waited = True
        elif t.startswith("s_barrier"):
            total += 1
            if not waited:
                bad.append(kernel)
        elif t.startswith("s_endpgm"):
            waited = True
    return total, bad


def unguarded_addtid(asm_text: str):
    """(add-TID stores, those not directly behind their own `s_mov_b32 m0` + `s_nop 0`)"""
    ins = []
    for line in asm_text.split("\n"):
        t = line.split(";")[0].strip()
        if not t or t.startswith(".") or t.endswith(":"):
            continue
        ins.append(t)
    total, bad = 0, 0
    for i, t in enumerate(ins):
        if not t.startswith("ds_write_addtid"):
            continue
        total += 1
        j = i - 1
        while j >= 0 and ins[j].startswith("ds_write_addtid"):
            j -= 1
        if not (j >= 1 and ins[j].startswith("s_nop") and ins[j - 1].replace(" ", "").startswith("s_mov_b32m0,")):
            bad += 1
    return total, bad


def check(src: str, m0: bool = False):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                        "-S", "-o", out, src], check=True, capture_output=True)
        text = open(out).read()
        return unguarded_addtid(text) if m0 else unguarded_barriers(text)


if __name__ == "__main__":
    m0 = "--m0" in sys.argv
    srcs = [a for a in sys.argv[1:] if a != "--m0"] or sorted(glob.glob(os.path.join(ROOT, "gpu_stereo_matching_amd", "csrc", "*.hip")))
    rc = 0
    for s in srcs:
        if m0:
            total, nbad = check(s, m0=True)
            print(f"{os.path.basename(s)}: {total} add-TID stores, {nbad} not behind their own M0 write")
            rc |= bool(nbad)
            continue
        total, bad = check(s)
        print(f"{os.path.basename(s)}: {total} barriers, {len(bad)} after an unwaited asm LDS store"
              + (f" in {sorted(set(bad))[:3]}" if bad else ""))
        rc |= bool(bad)
    sys.exit(rc)
