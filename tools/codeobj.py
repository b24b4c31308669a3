"""Identity of a kernel's machine code inside libsm_hip.so.

The counters the bench's roofline reads (profiles/valu_counts.json, profiles/isa_mix_box.json) describe one
build of one kernel.  kernel_sha256() hashes that kernel's gfx950 machine code: the bytes of its function
symbol in the device code object that the host library carries in its `.hip_fatbin` section (clang offload
bundles, one per object file).  The tools that write those files stamp the hash; bench.py recomputes it from
the library it loads and reports `frac: null` when the two differ, so an edit to the kernel without a
re-count cannot leave stale numbers on the bench line.

    python tools/codeobj.py gpu_stereo_matching_amd/libsm_hip.so 'box_match_kernelILi5ELi128ELb0ELi4E'
"""
from __future__ import annotations

import hashlib
import struct
import sys

BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf: bytes):
    """name -> (sh_addr, sh_offset, sh_size, sh_link, sh_entsize) of a little-endian ELF64 image."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        raise ValueError("not an ELF64 image")
    e_shoff, = struct.unpack_from("<Q", elf, 0x28)
    e_shentsize, e_shnum, e_shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = []
    for i in range(e_shnum):
        o = e_shoff + i * e_shentsize
        name, typ, _flags, addr, off, size, link, _info, _align, entsize = struct.unpack_from("<IIQQQQIIQQ", elf, o)
        hdrs.append((name, typ, addr, off, size, link, entsize))
    stroff = hdrs[e_shstrndx][3]
    out = {}
    for name, typ, addr, off, size, link, entsize in hdrs:
        end = elf.index(b"\0", stroff + name)
        out[elf[stroff + name:end].decode()] = (addr, off, size, link, entsize, typ)
    return out, hdrs


def device_code_objects(lib_path: str, arch: str = "gfx950"):
    """The `arch` code objects of every offload bundle in the library's .hip_fatbin section."""
    with open(lib_path, "rb") as f:
        host = f.read()
    secs, _ = _sections(host)
    if ".hip_fatbin" not in secs:
        raise ValueError(f"{lib_path}: no .hip_fatbin section")
    _, off, size = secs[".hip_fatbin"][:3]
    fat = host[off:off + size]
    objs = []
    pos = fat.find(BUNDLE_MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fat, pos + 24)
        p = pos + 32
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if triple.endswith(arch) and esize:
                objs.append(fat[pos + eoff:pos + eoff + esize])
        pos = fat.find(BUNDLE_MAGIC, pos + 1)
    return objs


def kernel_code(lib_path: str, symbol_part: str, arch: str = "gfx950") -> bytes:
    """Machine code of the one FUNC symbol whose mangled name contains `symbol_part` (its `.kd`
    descriptor excluded).  Raises when none or several match."""
    found = []
    for co in device_code_objects(lib_path, arch):
        secs, hdrs = _sections(co)
        symtab = secs.get(".symtab")
        if symtab is None:
            continue
        _, soff, ssize, slink, sent, _ = symtab
        stroff = hdrs[slink][3]
        for i in range(ssize // sent):
            st_name, st_info, _other, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", co, soff + i * sent)
            if st_info & 0xF != 2 or st_size == 0:   # STT_FUNC
                continue
            end = co.index(b"\0", stroff + st_name)
            name = co[stroff + st_name:end].decode()
            if symbol_part not in name:
                continue
            _n, _t, addr, off, _s, _l, _e = hdrs[st_shndx]
            start = off + (st_value - addr)
            found.append((name, co[start:start + st_size]))
    if len(found) != 1:
        raise ValueError(f"{symbol_part}: {len(found)} matching kernels in {lib_path}: {[n for n, _ in found][:4]}")
    return found[0][1]


def kernel_sha256(lib_path: str, symbol_part: str, arch: str = "gfx950") -> str:
    return hashlib.sha256(kernel_code(lib_path, symbol_part, arch)).hexdigest()


def default_lib() -> str:
    import os
    return os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu_stereo_matching_amd",
                        "libsm_hip.so")


def stamp(json_path: str, symbol_part: str, lib_path: str = None) -> str:
    """Write the kernel's code hash into a single-kernel counts file (e.g. profiles/isa_mix_box.json)."""
    import json
    lib_path = lib_path or default_lib()
    h = kernel_sha256(lib_path, symbol_part)
    with open(json_path) as f:
        d = json.load(f)
    d["code_symbol"] = symbol_part
    d["code_sha256"] = h
    with open(json_path, "w") as f:
        json.dump(d, f, indent=1)
    return h


if __name__ == "__main__":
    if sys.argv[1] == "--stamp":          # --stamp JSON SYMBOL [LIB]
        print(stamp(sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else None))
    else:
        lib, sym = sys.argv[1], sys.argv[2]
        code = kernel_code(lib, sym)
        print(hashlib.sha256(code).hexdigest(), len(code), "bytes")
