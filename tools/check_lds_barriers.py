"""Static check of the gfx950 ISA: every s_barrier that follows an inline-asm LDS store
(ds_write_addtid_b32 / ds_write_b64, which the compiler's wait-count pass does not track) must be
preceded by an s_waitcnt lgkmcnt(0) issued after that store.  A missing wait lets another wave read
the rows before they land (a rare, timing-dependent wrong result).

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


def check(src: str):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only",
                        "-S", "-o", out, src], check=True, capture_output=True)
        return unguarded_barriers(open(out).read())


if __name__ == "__main__":
    srcs = sys.argv[1:] or sorted(glob.glob(os.path.join(ROOT, "gpu_stereo_matching_amd", "csrc", "*.hip")))
    rc = 0
    for s in srcs:
        total, bad = check(s)
        print(f"{os.path.basename(s)}: {total} barriers, {len(bad)} after an unwaited asm LDS store"
              + (f" in {sorted(set(bad))[:3]}" if bad else ""))
        rc |= bool(bad)
    sys.exit(rc)
