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
    srcs = [os.path.join(_HERE, f) for f in ("bm_oracle.c", "st_oracle.c")]
    if force or not os.path.exists(_LIB_PATH) or any(os.path.getmtime(_LIB_PATH) < os.path.getmtime(f) for f in srcs):
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
        L.ora_get_all_sad.argtypes = L.ora_get_disp.argtypes
        L.ora_device_cu_literal.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p]
        L.ora_device_cu_literal.restype = ctypes.c_int
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
        L.ora_init_rectify_map.argtypes = [_f64p, _f64p, ctypes.c_int, _f64p, _f64p, ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]
        L.ora_synth_pair.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p, _u8p]
        L.ora_guided_probe.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_double, _u8p, _u8p, _u8p, _f64p, _f64p, _f64p, _f64p]
        L.ora_guided_probe.restype = ctypes.c_int
        L.ora_box_lr_probe.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _u8p, _u8p]
        L.ora_box_lr_probe.restype = ctypes.c_int
        L.ora_st_cost.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_float)]
        L.ora_st_tree.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_float, _i32p, _i32p, _u8p, _i32p, _u8p,
                                  _u8p]
        L.ora_st_tree.restype = ctypes.c_int
        L.ora_st_disp.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                  ctypes.c_float, _u8p]
        L.ora_st_disp.restype = ctypes.c_int
        _fp = ctypes.POINTER(ctypes.c_float)
        L.ora_st_right_cost.argtypes = [_fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, _fp]
        L.ora_st_tree_depth.argtypes = [_u8p, _u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                        _i32p, _i32p, _u8p, _i32p, _u8p, _u8p]
        L.ora_st_tree_depth.restype = ctypes.c_int
        L.ora_st2_disp.argtypes = [_u8p, _u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                   ctypes.c_float, _u8p, _u8p, _u8p, _u8p]
        L.ora_st2_disp.restype = ctypes.c_int
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


def device_cu_literal(left, right, sad_window_size: int, search_range: int) -> np.ndarray:
    """Device.cu's map as its fixed launch geometry produces it (blockMatching_gpu, Device.cu:173-301):
    the AD volume only for rows < 256 and cols < 320 (grid (8,10,D) x block (32,32), :231-233; 0 elsewhere
    from the memset, :193-194), the all-zero map for cols > 1024 (the <<<rows, cols>>> launch fails, :253).
    Raises ValueError for rows < 256 or cols < 320, where the reference reads and writes out of bounds."""
    left, right = _img(left), _img(right)
    H, W = left.shape
    out = np.empty((H, W), np.uint8)
    rc = lib().ora_device_cu_literal(_p(left, _u8p), _p(right, _u8p), W, H, sad_window_size, search_range,
                                     _p(out, _u8p))
    if rc == -2:
        raise ValueError(f"{W}x{H}: the Device.cu launch grid is out of bounds below 320x256")
    if rc != 0:
        raise MemoryError("ora_device_cu_literal")
    return out


def device_cu_literal_integral(left, right, radius: int, D: int) -> np.ndarray:
    """Second, independent formulation of device_cu_literal (numpy, for cross-checking the C loop nest):
    the AD planes masked to the grid's 256 x 320 coverage, 2-D integral images, clipped window sums by
    four lookups, then the strict-< WTA from 50 * win^2 with the col + d > W break."""
    L = _img(left).astype(np.int64)
    Rr = _img(right).astype(np.int64)
    H, W = L.shape
    if W < 320 or H < 256:
        raise ValueError("below 320x256")
    out = np.zeros((H, W), np.uint8)
    if W > 1024:
        return out
    win = 2 * radius + 1
    best = np.full((H, W), 50 * win * win, np.int64)
    dm = np.full((H, W), -256, np.int64)
    ys, xs = np.mgrid[0:H, 0:W]
    y0, y1 = np.clip(ys - radius, 0, H), np.clip(ys + radius + 1, 0, H)
    x0, x1 = np.clip(xs - radius, 0, W), np.clip(xs + radius + 1, 0, W)
    for d in range(D):
        ad = np.zeros((H, W), np.int64)
        ad[:256, d:320] = np.abs(L[:256, d:320] - Rr[:256, 0:320 - d]) if d < 320 else 0
        I = np.zeros((H + 1, W + 1), np.int64)
        I[1:, 1:] = ad.cumsum(0).cumsum(1)
        sad = I[y1, x1] - I[y0, x1] - I[y1, x0] + I[y0, x0]
        upd = (sad < best) & (xs + d <= W)
        best = np.where(upd, sad, best)
        dm = np.where(upd, d, dm)
    return (dm & 0xFF).astype(np.uint8)


def get_all_sad(left, right, sad_window_size: int, search_range: int) -> np.ndarray:
    """Literal restatement of ``getAllSAD`` (BlockMatching.cpp:191-261): uint8 [H, W, D] (pixel-major
    ``data_dm[p * D + d]``), each window SAD truncated to uchar, 255 where col + d > W."""
    left, right = _img(left), _img(right)
    H, W = left.shape
    out = np.empty((H, W, search_range), np.uint8)
    rc = lib().ora_get_all_sad(_p(left, _u8p), _p(right, _u8p), W, H, sad_window_size, search_range,
                               _p(out, _u8p), None)
    if rc != 0:
        raise MemoryError("ora_get_all_sad")
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


def box_right_keys_slice(left, right, radius: int, d_lo: int, d_hi: int, cost: np.ndarray = None) -> np.ndarray:
    """Right-view d-slice keys (the contract of sm_slice_keys_lr_device's right map, box): for right pixel u
    the minimum over d in [d_lo, d_hi) with u + d < W of (C_L(u + d, d) << 8 | d), C_R(u, d) = C_L(u + d, d)
    (StereoHelper.cpp:156-180), with the sign bit flipped (^ 0x80000000: a wide window's key passes 2^31, and
    the flip makes a signed MIN order the keys at every radius); 0x7FFFFFFF where no d of the slice reaches u.
    uint32 bit patterns [H, W]: combine slices with a MIN on their int32 view.  `cost`: a box_cost volume of
    at least d_hi planes (computed when None)."""
    if cost is None:
        cost = box_cost(left, right, radius, d_hi)
    _, H, W = cost.shape
    best = np.full((H, W), 0xFFFFFFFF, np.int64)
    for d in range(d_lo, d_hi):
        if d >= W:
            break
        k = (cost[d][:, d:].astype(np.int64) << 8) | d
        best[:, :W - d] = np.minimum(best[:, :W - d], k)
    return (best ^ 0x80000000).astype(np.uint32)


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


def box_lr_probe(left, right, radius: int, D: int):
    """box_lr in O(P) memory per thread (full-size LR checks): (left disp, right disp, checked, mask)."""
    left, right = _img(left), _img(right)
    H, W = left.shape
    disp = np.empty((H, W), np.uint8)
    rdisp = np.empty((H, W), np.uint8)
    if lib().ora_box_lr_probe(_p(left, _u8p), _p(right, _u8p), W, H, radius, D, _p(disp, _u8p), _p(rdisp, _u8p)) != 0:
        raise MemoryError("ora_box_lr_probe")
    checked, mask = lr_check(disp, rdisp)
    return disp, rdisp, checked, mask


def guided_probe(left, right, radius: int, D: int, eps: float, disp_left, disp_right=None):
    """The fp64 guided filter probed at given maps in O(P) memory (full-size checks):
    (oracle disparity, best left cost, left cost at disp_left, best right cost, right cost at
    disp_right); the right costs follow StereoHelper.cpp:156-180 (None without disp_right)."""
    left, right = _img(left), _img(right)
    H, W = left.shape
    dl = _img(disp_left)
    dr = _img(disp_right) if disp_right is not None else None
    out = np.empty((H, W), np.uint8)
    best, qL = np.empty((H, W), np.float64), np.empty((H, W), np.float64)
    bestR = np.empty((H, W), np.float64) if dr is not None else None
    qR = np.empty((H, W), np.float64) if dr is not None else None
    rc = lib().ora_guided_probe(_p(left, _u8p), _p(right, _u8p), W, H, radius, D, float(eps), _p(dl, _u8p),
                                _p(dr, _u8p), _p(out, _u8p), _p(best, _f64p), _p(qL, _f64p), _p(bestR, _f64p),
                                _p(qR, _f64p))
    if rc != 0:
        raise MemoryError("ora_guided_probe")
    return out, best, qL, bestR, qR


def right_cost_from_left(cost: np.ndarray) -> np.ndarray:
    """GetRightMatchingCostFromLeft (STMatching/StereoHelper.cpp:156-180) on a [D][H][W] float volume:
    C_R(y, u, d) = C_L(y, u + d, d) if u + d < W, else C_R(y, u, d - 1)."""
    cost = np.asarray(cost, np.float64)
    D, H, W = cost.shape
    out = np.empty_like(cost)
    u = np.arange(W)
    prev = None
    for d in range(D):
        src = np.minimum(u + d, W - 1)
        cur = cost[d][:, src]
        if prev is not None:
            cur = np.where((u + d < W)[None, :], cur, prev)
        out[d] = cur
        prev = cur
    return out


def right_wta_float(cost: np.ndarray):
    """Right-view WTA (StereoHelper.cpp:131-154: strict < from d = 0, no threshold) of the right
    cost derived from a float left volume.  Returns (right disparity, C_R volume, best C_R)."""
    cr = right_cost_from_left(cost)
    disp = np.argmin(cr, axis=0).astype(np.uint8)   # first minimum = strict < from d = 0
    return disp, cr, cr.min(axis=0)


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


def _bgr(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    assert a.ndim == 3 and a.shape[2] == 3
    return a


def st_cost(left_bgr, right_bgr, D: int) -> np.ndarray:
    """STMatching GetMatchingCost (StereoHelper.cpp:75-129): float [H, W, D] colour + gradient cost."""
    L, R = _bgr(left_bgr), _bgr(right_bgr)
    H, W = L.shape[:2]
    out = np.empty((H, W, D), np.float32)
    lib().ora_st_cost(_p(L, _u8p), _p(R, _u8p), W, H, D, out.ctypes.data_as(ctypes.POINTER(ctypes.c_float)))
    return out


def st_tree(left_bgr, tau: float = 1200.0):
    """STMatching BuildSegmentTree with CColorWeight (SegmentTree.cpp:38-139): the tree in BFS order.
    Returns dict(node, parent, pdist, first, nchild, cdist [P, 4], levels)."""
    L = _bgr(left_bgr)
    H, W = L.shape[:2]
    P = W * H
    t = dict(node=np.empty(P, np.int32), parent=np.empty(P, np.int32), pdist=np.empty(P, np.uint8),
             first=np.empty(P, np.int32), nchild=np.empty(P, np.uint8), cdist=np.zeros((P, 4), np.uint8))
    t["levels"] = lib().ora_st_tree(_p(L, _u8p), W, H, tau, _p(t["node"], _i32p), _p(t["parent"], _i32p),
                                    _p(t["pdist"], _u8p), _p(t["first"], _i32p), _p(t["nchild"], _u8p),
                                    _p(t["cdist"], _u8p))
    return t


def st_disp(left_bgr, right_bgr, D: int = 60, scale: int = 4, sigma: float = 0.1, tau: float = 1200.0):
    """STMatching stereo_disparity_normal (ST-1, StereoDisparity.cpp:57-89); returns (disp, levels)."""
    L, R = _bgr(left_bgr), _bgr(right_bgr)
    H, W = L.shape[:2]
    out = np.empty((H, W), np.uint8)
    levels = lib().ora_st_disp(_p(L, _u8p), _p(R, _u8p), W, H, D, scale, sigma, tau, _p(out, _u8p))
    return out, levels


def st_right_cost(cost) -> np.ndarray:
    """STMatching GetRightMatchingCostFromLeft (StereoHelper.cpp:156-180) of a float [H, W, D] volume."""
    c = np.ascontiguousarray(cost, dtype=np.float32)
    H, W, D = c.shape
    out = np.empty_like(c)
    fp = ctypes.POINTER(ctypes.c_float)
    lib().ora_st_right_cost(c.ctypes.data_as(fp), W, H, D, out.ctypes.data_as(fp))
    return out


def st_tree_depth(left_bgr, disp, mask, level: int, tau: float = 1200.0):
    """BuildSegmentTree with CColorDepthWeight (SegmentTree.cpp:196-219): same dict as st_tree."""
    L = _bgr(left_bgr)
    H, W = L.shape[:2]
    P = W * H
    d, m = _img(disp), _img(mask)
    t = dict(node=np.empty(P, np.int32), parent=np.empty(P, np.int32), pdist=np.empty(P, np.uint8),
             first=np.empty(P, np.int32), nchild=np.empty(P, np.uint8), cdist=np.zeros((P, 4), np.uint8))
    t["levels"] = lib().ora_st_tree_depth(_p(L, _u8p), _p(d, _u8p), _p(m, _u8p), W, H, level, tau,
                                          _p(t["node"], _i32p), _p(t["parent"], _i32p), _p(t["pdist"], _u8p),
                                          _p(t["first"], _i32p), _p(t["nchild"], _u8p), _p(t["cdist"], _u8p))
    return t


def st2_disp(left_bgr, right_bgr, D: int = 60, scale: int = 4, sigma: float = 0.1, tau: float = 1200.0):
    """STMatching stereo_disparity_iteration (ST-2, StereoDisparity.cpp:91-160).
    Returns (disp, levels, first-pass left map, first-pass right map, LR mask)."""
    L, R = _bgr(left_bgr), _bgr(right_bgr)
    H, W = L.shape[:2]
    out, l1, r1, mk = (np.empty((H, W), np.uint8) for _ in range(4))
    levels = lib().ora_st2_disp(_p(L, _u8p), _p(R, _u8p), W, H, D, scale, sigma, tau, _p(out, _u8p), _p(l1, _u8p),
                                _p(r1, _u8p), _p(mk, _u8p))
    return out, levels, l1, r1, mk


def synth_pair(seed: int, W: int, H: int, D: int):
    L = np.empty((H, W), np.uint8)
    R = np.empty((H, W), np.uint8)
    lib().ora_synth_pair(ctypes.c_uint64(seed), W, H, D, _p(L, _u8p), _p(R, _u8p))
    return L, R


# ---------------------------------------------------------------------------------------------
# Rectification (the caller-side step before remap: Rectify, BlockMatching/Utility.cpp:228-234,
# called from remapTest, Caller.cpp:50-51).  The reference delegates to OpenCV 2.4.12's
# stereoRectify(..., CV_CALIB_ZERO_DISPARITY) with the C++ defaults alpha = -1 and
# newImageSize = Size(), then initUndistortRectifyMap(..., CV_32FC1).  OpenCV is a third-party
# dependency absent from the reference tree and from this image; the functions below restate its
# published calib3d/src/calibration.cpp (cvStereoRectify, cvRodrigues2, cvUndistortPoints,
# cvProjectPoints2) in numpy, fp64, with the float32 point buffers OpenCV uses (CV_32FC2) rounded
# where it rounds them.  Parity with OpenCV itself: UNPINNED (no OpenCV output exists here).
# This numpy formulation is deliberately independent of the product's C++ one
# (gpu_stereo_matching_amd/csrc/bm_rectify.hip): different SVD, different code.
# ---------------------------------------------------------------------------------------------
def rodrigues_to_vec(R: np.ndarray) -> np.ndarray:
    """cvRodrigues2 3x3 -> 3x1: orthogonalise by SVD (R = U V^T), then axis * angle."""
    U, _, Vt = np.linalg.svd(np.asarray(R, np.float64))
    R = U @ Vt
    rx, ry, rz = R[2, 1] - R[1, 2], R[0, 2] - R[2, 0], R[1, 0] - R[0, 1]
    s = np.sqrt((rx * rx + ry * ry + rz * rz) * 0.25)
    c = min(1.0, max(-1.0, (R[0, 0] + R[1, 1] + R[2, 2] - 1) * 0.5))
    theta = np.arccos(c)
    if s < 1e-5:
        if c > 0:
            return np.zeros(3)
        t = (R + np.eye(3)) * 0.5          # theta ~ pi (OpenCV's branch)
        rx, ry, rz = (np.sqrt(max(t[i, i], 0.0)) for i in range(3))
        if R[0, 1] < 0:
            ry = -ry
        if R[0, 2] < 0:
            rz = -rz
        if abs(rx) < abs(ry) and abs(rx) < abs(rz) and (R[1, 2] > 0) != (ry * rz > 0):
            rz = -rz
        v = np.array([rx, ry, rz])
        return v * (theta / np.linalg.norm(v))
    return np.array([rx, ry, rz]) * (theta / (2 * s))


def rodrigues_to_mat(r: np.ndarray) -> np.ndarray:
    """cvRodrigues2 3x1 -> 3x3: R = cos I + (1 - cos) n n^T + sin [n]x."""
    r = np.asarray(r, np.float64).reshape(3)
    theta = np.linalg.norm(r)
    if theta < np.finfo(np.float64).eps:
        return np.eye(3)
    n = r / theta
    c, s = np.cos(theta), np.sin(theta)
    nx = np.array([[0, -n[2], n[1]], [n[2], 0, -n[0]], [-n[1], n[0], 0]])
    return c * np.eye(3) + (1 - c) * np.outer(n, n) + s * nx


def undistort_points(pts: np.ndarray, K: np.ndarray, dist: np.ndarray) -> np.ndarray:
    """cvUndistortPoints with R = P = 0: 5 fixed-point iterations (k1..k6, p1, p2), normalised
    output stored as float32 (the CV_32FC2 buffer of cvStereoRectify)."""
    k = np.zeros(8)
    k[:len(dist)] = dist
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    out = np.empty_like(pts, dtype=np.float32)
    for i, (u, v) in enumerate(pts.astype(np.float64)):
        x0 = x = (u - cx) * (1.0 / fx)
        y0 = y = (v - cy) * (1.0 / fy)
        for _ in range(5 if len(dist) else 0):
            r2 = x * x + y * y
            icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
            dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x)
            dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y
            x = (x0 - dx) * icdist
            y = (y0 - dy) * icdist
        out[i] = (x, y)
    return out


def stereo_rectify(K1, dist1, K2, dist2, width: int, height: int, R, T):
    """cvStereoRectify, flags = CV_CALIB_ZERO_DISPARITY, alpha = -1, newImageSize = imageSize.
    R is a 3x3 rotation matrix or a 3-vector; returns (R1, R2, P1, P2, Q) as float64 arrays."""
    K1, K2 = np.asarray(K1, np.float64).reshape(3, 3), np.asarray(K2, np.float64).reshape(3, 3)
    dist1, dist2 = np.asarray(dist1, np.float64).ravel(), np.asarray(dist2, np.float64).ravel()
    R = np.asarray(R, np.float64)
    T = np.asarray(T, np.float64).reshape(3)
    nx, ny = float(width), float(height)
    om = rodrigues_to_vec(R) if R.size == 9 else R.reshape(3)
    r_r = rodrigues_to_mat(om * -0.5)                 # half rotation for each camera
    t = r_r @ T
    idx = 0 if abs(t[0]) > abs(t[1]) else 1
    c = t[idx]
    nt = np.linalg.norm(t)
    uu = np.zeros(3)
    uu[idx] = 1.0 if c > 0 else -1.0
    ww = np.cross(t, uu)
    nw = np.linalg.norm(ww)
    if nw > 0.0:
        ww = ww * (np.arccos(abs(c) / nt) / nw)
    wR = rodrigues_to_mat(ww)
    R1 = wR @ r_r.T
    R2 = wR @ r_r
    t = R2 @ T
    fc_new = np.inf
    for K, dk in ((K1, dist1), (K2, dist2)):
        dk1 = dk[0] if len(dk) else 0.0
        fc = K[idx ^ 1, idx ^ 1]
        if dk1 < 0:
            fc *= 1 + dk1 * (nx * nx + ny * ny) / (4 * fc * fc)
        fc_new = min(fc_new, fc)
    cc = []
    for K, dk, Rk in ((K1, dist1, R1), (K2, dist2, R2)):
        pts = np.array([[(i % 2) * (nx - 1), (i // 2) * (ny - 1)] for i in range(4)], np.float32)
        und = undistort_points(pts, K, dk).astype(np.float64)
        X = np.concatenate([und, np.ones((4, 1))], axis=1)       # convertPointsHomogeneous (float32 values)
        Y = X @ Rk.T
        proj = np.stack([fc_new * Y[:, 0] / Y[:, 2], fc_new * Y[:, 1] / Y[:, 2]], 1).astype(np.float32)
        avg = proj.astype(np.float64).mean(axis=0)
        cc.append([(nx - 1) / 2 - avg[0], (ny - 1) / 2 - avg[1]])
    cx = (cc[0][0] + cc[1][0]) * 0.5                 # CV_CALIB_ZERO_DISPARITY
    cy = (cc[0][1] + cc[1][1]) * 0.5
    cx, cy = nx * cx / nx, ny * cy / ny              # newImgSize == imageSize rescale (rounds)
    P1 = np.array([[fc_new, 0, cx, 0], [0, fc_new, cy, 0], [0, 0, 1, 0]], np.float64)
    P2 = P1.copy()
    P2[idx, 3] = t[idx] * fc_new
    Q = np.array([[1, 0, 0, -cx], [0, 1, 0, -cy], [0, 0, 0, fc_new], [0, 0, -1.0 / t[idx], (cx - cx) / t[idx]]], np.float64)
    return R1, R2, P1, P2, Q


def init_rectify_map(K, dist, R, P, width: int, height: int):
    """initUndistortRectifyMap(..., CV_32FC1) in the C restatement (fp64, OpenCV's op order)."""
    K = np.ascontiguousarray(K, np.float64).reshape(9)
    dist = np.ascontiguousarray(dist, np.float64).ravel()
    R = np.ascontiguousarray(R, np.float64).reshape(9)
    P = np.ascontiguousarray(P, np.float64).reshape(12)
    mx = np.empty((height, width), np.float32)
    my = np.empty((height, width), np.float32)
    fp = ctypes.POINTER(ctypes.c_float)
    lib().ora_init_rectify_map(_p(K, _f64p), _p(dist, _f64p), int(dist.size), _p(R, _f64p), _p(P, _f64p),
                               width, height, mx.ctypes.data_as(fp), my.ctypes.data_as(fp))
    return mx, my
