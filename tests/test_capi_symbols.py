"""CPU tests: libsm_hip.so loads and exports every symbol include/sm_hip.h declares;
calls that need no GPU behave."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "sm_hip.h")).read()
    return sorted(set(re.findall(r"SM_API\s+[\w\s\*]+?\b(sm_\w+)\s*\(", txt)))


def test_header_declares_expected_set():
    from gpu_stereo_matching_amd import _capi
    assert set(declared_symbols()) == set(_capi.EXPORTED)


def test_library_exports_all_symbols():
    from gpu_stereo_matching_amd import _capi
    lib = _capi.load()
    for name in declared_symbols():
        assert hasattr(lib, name), name


def test_version_and_errors_without_device():
    from gpu_stereo_matching_amd import _capi
    lib = _capi.load()
    assert b"gfx950" in lib.sm_version()
    n = ctypes.c_int(-1)
    assert lib.sm_device_count(ctypes.byref(n)) == 0 and n.value >= 0
    h = ctypes.c_void_p()
    assert lib.sm_create(0, 0, 10, 64, ctypes.byref(h)) == _capi.SM_ERR_INVALID_ARG
    assert lib.sm_create(0, 64, 64, 300, ctypes.byref(h)) == _capi.SM_ERR_INVALID_ARG
    assert lib.sm_block_match_u8(None, None, None, 10, 10, 10, 1, 8, 0, None, 10) == _capi.SM_ERR_INVALID_ARG
    assert b"null handle" in lib.sm_last_error_string()
    if n.value == 0:
        assert lib.sm_create(0, 64, 64, 64, ctypes.byref(h)) == _capi.SM_ERR_DEVICE


def test_group_errors_without_device():
    """The multi-GPU group handle: argument checks, and member creation failing cleanly (the
    partially built group is torn down, its worker threads joined) when no device is visible."""
    from gpu_stereo_matching_amd import _capi
    lib = _capi.load()
    g = ctypes.c_void_p()
    assert lib.sm_create_group(0, None, 64, 64, 64, ctypes.byref(g)) == _capi.SM_ERR_INVALID_ARG
    assert lib.sm_create_group(2, None, 64, 64, 64, None) == _capi.SM_ERR_INVALID_ARG
    assert lib.sm_group_block_match_u8(None, None, None, 8, 8, 8, 1, 8, 0, None, 8) == _capi.SM_ERR_INVALID_ARG
    assert lib.sm_group_block_match_batch_u8(None, None, None, 1, 8, 8, 8, 1, 8, 0, None, 8) == _capi.SM_ERR_INVALID_ARG
    assert lib.sm_destroy_group(None) == _capi.SM_OK
    n = ctypes.c_int(-1)
    lib.sm_device_count(ctypes.byref(n))
    if n.value == 0:
        assert lib.sm_create_group(2, None, 64, 64, 64, ctypes.byref(g)) == _capi.SM_ERR_DEVICE
        assert b"group member 0" in lib.sm_last_error_string()
        assert not g.value


def test_no_cpu_fallback_in_product():
    """The product package must not import or load the oracle (test infrastructure only)."""
    pkg = os.path.join(ROOT, "gpu_stereo_matching_amd")
    bad = re.compile(r"^\s*(from\s+oracle|import\s+oracle)|libsm_oracle|ora_[a-z_]+\(", re.M)
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".h", ".cpp")):
                txt = open(os.path.join(dirpath, f)).read()
                assert not bad.search(txt), f


def test_missing_library_fails_loudly(tmp_path):
    from gpu_stereo_matching_amd import _capi
    with pytest.raises(ImportError):
        saved = _capi._lib
        _capi._lib = None
        try:
            _capi.load(str(tmp_path / "nope.so"))
        finally:
            _capi._lib = saved


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc absent")
def test_asm_lds_stores_are_waited_before_barriers():
    """The guided kernel writes LDS rows with inline asm (ds_write_addtid_b32, ds_write_b64), which the
    compiler's wait-count pass does not track.  Every s_barrier after such a store must follow an
    s_waitcnt lgkmcnt(0), or another wave may read the rows before they land (tools/check_lds_barriers.py
    on the gfx950 ISA)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("check_lds_barriers",
                                                  os.path.join(ROOT, "tools", "check_lds_barriers.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    total, bad = mod.check(os.path.join(ROOT, "gpu_stereo_matching_amd", "csrc", "bm_guided.hip"))
    assert total > 0 and not bad, f"{len(bad)} of {total} barriers follow an unwaited asm LDS store: {sorted(set(bad))[:3]}"


def test_host_alloc_rejects_bad_args():
    """sm_host_alloc validates its arguments before touching the HIP runtime."""
    import ctypes
    from gpu_stereo_matching_amd import _capi
    L = _capi.load()
    assert L.sm_host_alloc(16, None) != 0
    p = ctypes.c_void_p()
    assert L.sm_host_alloc(0, ctypes.byref(p)) != 0 and not p.value
    assert L.sm_host_free(None) == 0


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc absent")
def test_addtid_stores_follow_their_own_m0_write():
    """ds_write_addtid_b32 addresses LDS through M0.  Each such store must sit in the asm statement
    that writes M0 (s_mov_b32 m0 + s_nop 0 right before it), so no compiler-generated M0
    use can fall between the write and the store (tools/check_lds_barriers.py --m0 on the ISA)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("check_lds_barriers",
                                                  os.path.join(ROOT, "tools", "check_lds_barriers.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    total, bad = mod.check(os.path.join(ROOT, "gpu_stereo_matching_amd", "csrc", "bm_guided.hip"), m0=True)
    assert total > 0 and bad == 0, f"{bad} of {total} add-TID stores are not behind their own M0 write"
