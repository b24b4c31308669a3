"""ctypes binding of ``libsm_hip.so`` (the C ABI declared in ``include/sm_hip.h``).

The HIP library is the only compute path: if it is missing or fails to load this module
raises, it never falls back to a CPU implementation.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsm_hip.so")

SM_OK = 0
SM_ERR_INVALID_ARG = 1
SM_ERR_OUT_OF_MEMORY = 2
SM_ERR_DEVICE = 3
SM_ERR_LAUNCH = 4
SM_ERR_CAPACITY = 5

SM_AGG_BOX = 0
SM_AGG_GUIDED = 1
SM_LR_CHECK = 2
SM_MEDIAN = 4
SM_STAGED = 8
SM_DEVICE_CU_GRID = 16

SM_PARAM_GUIDED_EPS = 1
SM_PARAM_STAGED_GROUP = 2
SM_PARAM_STAGE_TIMING = 3

# every symbol include/sm_hip.h declares (checked by tests/test_capi_symbols.py)
EXPORTED = (
    "sm_version", "sm_last_error_string", "sm_device_count", "sm_create", "sm_destroy",
    "sm_set_param_f", "sm_block_match_u8", "sm_block_match_lr_u8", "sm_last_stage_ms",
    "sm_last_staged_kernel_ms",
    "sm_match_device", "sm_slice_keys_device", "sm_keys_to_disp_device", "sm_stream_sync",
    "sm_bgr_to_gray_device", "sm_remap_u8_device", "sm_block_match_bgr_u8", "sm_median_u8_device",
    "sm_bgr_to_gray_u8", "sm_remap_u8", "sm_ad_volume_device", "sm_ad_volume_u8", "sm_sad_volume_device",
    "sm_all_sad_device", "sm_all_sad_u8",
    "sm_stereo_rectify", "sm_init_rectify_map_device", "sm_init_rectify_map",
    "sm_create_group", "sm_destroy_group", "sm_group_size", "sm_group_set_param_f", "sm_group_block_match_u8",
    "sm_group_block_match_lr_u8", "sm_group_block_match_batch_u8", "sm_group_dslice_block_match_u8", "sm_guided_slice_keys_device",
    "sm_guided_keys_to_disp_device", "sm_segment_tree_match_bgr_u8", "sm_segment_tree_refined_bgr_u8",
    "sm_last_segment_tree_stats", "sm_last_segment_tree_arrays", "sm_host_alloc", "sm_host_free",
    "sm_dslice_plan", "sm_dslice_rehearse_u8", "sm_slice_keys_lr_device", "sm_right_keys_to_disp_device",
    "sm_lr_check_device",
)


class SMError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[sm error {code}] {msg}")
        self.code = code


_lib = None
_u8p = ctypes.c_void_p


def load(path: str = LIB_PATH):
    """Load and type the library once; raises if the HIP build is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C gpu_stereo_matching_amd/csrc` (hipcc, gfx950)")
    # One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64.so.7.  Loading torch
    # first makes our DT_NEEDED libamdhip64.so.7 resolve to that already-loaded copy (same soname)
    # instead of mapping /opt/rocm's second runtime next to it (two HSA runtimes cannot share a GPU).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    vp, i, i64, u = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint
    L.sm_version.restype = ctypes.c_char_p
    L.sm_last_error_string.restype = ctypes.c_char_p
    L.sm_device_count.argtypes = [ctypes.POINTER(i)]
    L.sm_create.argtypes = [i, i, i, i, ctypes.POINTER(vp)]
    L.sm_destroy.argtypes = [vp]
    L.sm_set_param_f.argtypes = [vp, i, ctypes.c_float]
    L.sm_block_match_u8.argtypes = [vp, vp, vp, i, i, i, i, i, u, vp, i]
    L.sm_block_match_lr_u8.argtypes = [vp, vp, vp, i, i, i, i, i, u, vp, vp, vp, i]
    L.sm_last_stage_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                                   ctypes.POINTER(ctypes.c_float)]
    L.sm_last_staged_kernel_ms.argtypes = L.sm_last_stage_ms.argtypes
    L.sm_match_device.argtypes = [vp, vp, vp, i, i, i, i, i64, i, i, u, vp, i, i64, vp]
    L.sm_slice_keys_device.argtypes = [vp, vp, vp, i, i, i, i, i, i, vp, vp]
    L.sm_keys_to_disp_device.argtypes = [vp, vp, i, i, i, vp, i, vp]
    L.sm_guided_slice_keys_device.argtypes = [vp, vp, vp, i, i, i, i, i, i, vp, vp]
    L.sm_guided_keys_to_disp_device.argtypes = [vp, vp, i, i, vp, i, vp]
    L.sm_stream_sync.argtypes = [vp, vp]
    L.sm_host_alloc.argtypes = [ctypes.c_size_t, ctypes.POINTER(vp)]
    L.sm_host_free.argtypes = [vp]
    L.sm_median_u8_device.argtypes = [vp, vp, i, i, i, i, vp, i, vp]
    L.sm_bgr_to_gray_u8.argtypes = [vp, vp, i, i, i, i, vp, i]
    L.sm_remap_u8.argtypes = [vp, vp, i, i, i, vp, vp, i, vp, i]
    L.sm_ad_volume_device.argtypes = [vp, vp, vp, i, i, i, i, vp, vp]
    L.sm_ad_volume_u8.argtypes = [vp, vp, vp, i, i, i, i, vp]
    L.sm_sad_volume_device.argtypes = [vp, vp, vp, i, i, i, i, i, vp, vp]
    L.sm_all_sad_device.argtypes = [vp, vp, vp, i, i, i, i, i, vp, vp]
    L.sm_all_sad_u8.argtypes = [vp, vp, vp, i, i, i, i, i, vp]
    L.sm_bgr_to_gray_device.argtypes = [vp, vp, i, i, i, i, vp, i, vp]
    L.sm_remap_u8_device.argtypes = [vp, vp, i, i, i, vp, vp, i, vp, i, vp]
    L.sm_block_match_bgr_u8.argtypes = [vp, vp, vp, i, i, i, i, i, i, u, vp, i]
    L.sm_segment_tree_match_bgr_u8.argtypes = [vp, vp, vp, i, i, i, i, i, ctypes.c_float, vp, i]
    L.sm_segment_tree_refined_bgr_u8.argtypes = [vp, vp, vp, i, i, i, i, i, ctypes.c_float, vp, i]
    L.sm_last_segment_tree_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                                             ctypes.POINTER(ctypes.c_int)]
    L.sm_last_segment_tree_arrays.argtypes = [vp, vp, i64, vp, i64, ctypes.POINTER(ctypes.c_int)]
    L.sm_stereo_rectify.argtypes = [vp, vp, i, vp, vp, i, i, i, vp, i, vp, vp, vp, vp, vp, vp]
    L.sm_init_rectify_map_device.argtypes = [vp, vp, vp, i, vp, vp, i, i, vp, vp, i, vp]
    L.sm_init_rectify_map.argtypes = [vp, vp, vp, i, vp, vp, i, i, vp, vp, i]
    L.sm_create_group.argtypes = [i, vp, i, i, i, vp]
    L.sm_destroy_group.argtypes = [vp]
    L.sm_group_size.argtypes = [vp, vp]
    L.sm_group_set_param_f.argtypes = [vp, i, ctypes.c_float]
    L.sm_group_block_match_u8.argtypes = [vp, vp, vp, i, i, i, i, i, u, vp, i]
    L.sm_group_block_match_lr_u8.argtypes = [vp, vp, vp, i, i, i, i, i, u, vp, vp, vp, i]
    L.sm_group_block_match_batch_u8.argtypes = [vp, vp, vp, i, i, i, i, i, i, u, vp, i]
    L.sm_group_dslice_block_match_u8.argtypes = [vp, vp, vp, i, i, i, i, i, u, vp, i]
    L.sm_dslice_plan.argtypes = [i64, i, i, i, ctypes.POINTER(i), ctypes.POINTER(i), ctypes.POINTER(i64),
                                 ctypes.POINTER(i64)]
    L.sm_dslice_rehearse_u8.argtypes = [vp, vp, vp, i, i, i, i, i, u, i, vp, i]
    L.sm_slice_keys_lr_device.argtypes = [vp, vp, vp, i, i, i, i, i, i, u, vp, vp, vp]
    L.sm_right_keys_to_disp_device.argtypes = [vp, vp, i64, vp, vp]
    L.sm_lr_check_device.argtypes = [vp, vp, vp, i, i, i, vp, vp, i, vp]
    for name in EXPORTED:
        if name not in ("sm_version", "sm_last_error_string"):
            getattr(L, name).restype = ctypes.c_int
    _lib = L
    return L


def check(rc: int):
    if rc != SM_OK:
        msg = load().sm_last_error_string()
        raise SMError(rc, msg.decode() if msg else "")
