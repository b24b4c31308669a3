"""ctypes front-end for the CPU oracle (``oracle/bm_oracle.c``).

TEST INFRASTRUCTURE ONLY: imported by ``tests/``, by ``__graft_entry__.smoke()``
(as the checker) and by ``bench.py``'s ``cpu_baseline`` leg.  The product
package ``gpu_stereo_matching_amd`` never imports this module.

Every function mirrors one routine of the reference's CPU path; see the C file
for the reference file:line each one restates.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libsm_oracle.so")
_lib = None

_u8p = ctypes.POINTER(ctypes.c_uint8)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_f64p = ctypes.POINTER(ctypes.c_double)


def build(force: bool = False) -> str:
    """Compile the oracle with the committed Makefile (gcc -O2)."""
    src = os.path.join(_HERE, "bm_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.ora_bgr_to_gray.argtypes = [_u8p, ctypes.c_int64, ctypes.c_int, _u8p]
        L.ora_precal.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p]
        L.ora_get_disp.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p, _u8p]
        L.ora_get_disp.restype = ctypes.c_int
        L.ora_box_disp.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p, _i32p, _u32p]
        L.ora_box_disp.restype = ctypes.c_int
        L.ora_box_cost.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _i32p]
        L.ora_box_cost.restype = ctypes.c_int
        L.ora_box_keys_slice.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u32p]
        L.ora_box_keys_slice.restype = ctypes.c_int
        L.ora_right_wta.argtypes = [_i32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p]
        L.ora_lr_check.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, _u8p, _u8p]
        L.ora_guided_disp.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_double, _u8p, _f64p, _f64p]
        L.ora_guided_disp.restype = ctypes.c_int
        L.ora_box_mean_f64.argtypes = [_f64p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _f64p]
        L.ora_remap.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float),
                                ctypes.POINTER(ctypes.c_float), _u8p]
        L.ora_median_u8.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p]
        L.ora_synth_pair.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p, _u8p]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t) if a is not None else None


def _img(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    assert a.ndim == 2
    return a


def bgr_to_gray(bgr: np.ndarray) -> np.ndarray:
    """OpenCV-2.4 ``cvtColor(BGR2GRAY)`` on an HxWxC (C=3 or 4) BGR(A) image."""
    bgr = np.ascontiguousarray(bgr, dtype=np.uint8)
    h, w, c = bgr.shape
    out = np.empty((h, w), np.uint8)
    lib().ora_bgr_to_gray(_p(bgr, _u8p), h * w, c, _p(out, _u8p))
    return out


def precal(left, right, D):
    left, right = _img(left), _img(right)
    H, W = left.shape
    dif = np.empty((D, H, W), np.uint8)
    lib().ora_precal(_p(left, _u8p), _p(right, _u8p), W, H, D, _p(dif, _u8p))
    return dif


def get_disp(left, right, sad_window_size: int, search_range: int) -> np.ndarray:
    """Literal restatement of ``getDisp`` (BlockMatching.cpp:111-189)."""
    left, right = _img(left), _img(right)
    H, W = left.shape
    out = np.empty((H, W), np.uint8)
    rc = lib().ora_get_disp(_p(left, _u8p), _p(right, _u8p), W, H, sad_window_size, search_range, _p(out, _u8p), None)
    if rc != 0:
        raise MemoryError("ora_get_disp")
    return out


def box_disp(left, right, radius: int, D: int, want_cost: bool = False, want_keys: bool = False):
    """Box-sum restatement; returns disp [, cost [D,H,W] int32] [, keys u32]."""
    left, right = _img(left), _img(right)
    H, W = left.shape
    out = np.empty((H, W), np.uint8)
    cost = np.empty((D, H, W), np.int32) if want_cost else None
    keys = np.empty((H, W), np.uint32) if want_keys else None
    rc = lib().ora_box_disp(_p(left, _u8p), _p(right, _u8p), W, H, radius, D, _p(out, _u8p),
                            _p(cost, _i32p), _p(keys, _u32p))
    if rc != 0:
        raise MemoryError("ora_box_disp")
    res = [out]
    if want_cost:
        res.append(cost)
    if want_keys:
        res.append(keys)
    return res[0] if len(res) == 1 else tuple(res)


def box_cost(left, right, radius: int, D: int) -> np.ndarray:
    left, right = _img(left), _img(right)
    H, W = left.shape
    cost = np.empty((D, H, W), np.int32)
    lib().ora_box_cost(_p(left, _u8p), _p(right, _u8p), W, H, radius, D, _p(cost, _i32p))
    return cost


def box_keys_slice(left, right, radius: int, d_lo: int, d_hi: int) -> np.ndarray:
    left, right = _img(left), _img(right)
    H, W = left.shape
    keys = np.empty((H, W), np.uint32)
    lib().ora_box_keys_slice(_p(left, _u8p), _p(right, _u8p), W, H, radius, d_lo, d_hi, _p(keys, _u32p))
    return keys


def right_wta(cost: np.ndarray) -> np.ndarray:
    cost = np.ascontiguousarray(cost, dtype=np.int32)
    D, H, W = cost.shape
    out = np.empty((H, W), np.uint8)
    lib().ora_right_wta(_p(cost, _i32p), W, H, D, _p(out, _u8p))
    return out


def lr_check(left_disp, right_disp):
    left_disp, right_disp = _img(left_disp), _img(right_disp)
    H, W = left_disp.shape
    checked = np.empty((H, W), np.uint8)
    mask = np.empty((H, W), np.uint8)
    lib().ora_lr_check(_p(left_disp, _u8p), _p(right_disp, _u8p), W, H, _p(checked, _u8p), _p(mask, _u8p))
    return checked, mask


def box_lr(left, right, radius: int, D: int):
    """Full box + LR pipeline: (left disp, right disp, checked disp, valid mask)."""
    disp, cost = box_disp(left, right, radius, D, want_cost=True)
    rdisp = right_wta(cost)
    checked, mask = lr_check(disp, rdisp)
    return disp, rdisp, checked, mask


def guided_disp(left, right, radius: int, D: int, eps: float, want_q: bool = False):
    """fp64 guided-filter aggregation (this build's definition; parity unpinned)."""
    left, right = _img(left), _img(right)
    H, W = left.shape
    out = np.empty((H, W), np.uint8)
    q = np.empty((D, H, W), np.float64) if want_q else None
    best = np.empty((H, W), np.float64)
    rc = lib().ora_guided_disp(_p(left, _u8p), _p(right, _u8p), W, H, radius, D, float(eps),
                               _p(out, _u8p), _p(q, _f64p), _p(best, _f64p))
    if rc != 0:
        raise MemoryError("ora_guided_disp")
    return (out, q, best) if want_q else (out, best)


def remap(src, mapx, mapy):
    """CPU_Remap restatement (Utility.cpp:239-264)."""
    src = _img(src)
    H, W = src.shape
    mapx = np.ascontiguousarray(mapx, dtype=np.float32)
    mapy = np.ascontiguousarray(mapy, dtype=np.float32)
    out = np.empty((H, W), np.uint8)
    fp = ctypes.POINTER(ctypes.c_float)
    lib().ora_remap(_p(src, _u8p), W, H, mapx.ctypes.data_as(fp), mapy.ctypes.data_as(fp), _p(out, _u8p))
    return out


def median(src, r: int):
    """ctmf (STMatching/ctmf.c) restatement: (2r+1)^2 median, replicate borders."""
    src = _img(src)
    H, W = src.shape
    out = np.empty((H, W), np.uint8)
    lib().ora_median_u8(_p(src, _u8p), W, H, r, _p(out, _u8p))
    return out


def synth_pair(seed: int, W: int, H: int, D: int):
    L = np.empty((H, W), np.uint8)
    R = np.empty((H, W), np.uint8)
    lib().ora_synth_pair(ctypes.c_uint64(seed), W, H, D, _p(L, _u8p), _p(R, _u8p))
    return L, R
