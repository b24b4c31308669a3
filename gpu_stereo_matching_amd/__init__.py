"""MI355X-native stereo block matching (gfx950 HIP kernels behind a C ABI).

Host-side mirror of the reference's GPU proxy API (ningw42/GPU_Stereo_Matching):

    void blockMatching_gpu(Mat &h_left, Mat &h_right, Mat &h_disparity,
                           int SADWindowSize, int searchRange);      // Device.cuh:50

``blockMatching_gpu(h_left, h_right, SADWindowSize, searchRange)`` takes two uint8 gray
images (numpy, HxW) and returns the uint8 disparity map, with the reference's argument
meaning (SADWindowSize = window radius r, window (2r+1)^2; searchRange = number of
disparities) and output convention (0 where no window SAD is below 50*(2r+1)^2).

``BlockMatcher`` is the handle-based interface (buffers allocated once, device-resident
batched calls on torch tensors, LR check, guided aggregation, d-slice keys for multi-GPU).
All compute runs in ``libsm_hip.so``; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

import numpy as np

from . import _capi
from ._capi import SMError, SM_AGG_BOX, SM_AGG_GUIDED, SM_LR_CHECK, SM_MEDIAN, SM_STAGED, SM_DEVICE_CU_GRID  # noqa: F401
from .synth import synth_pair  # noqa: F401
from .gray import bgr_to_gray  # noqa: F401

__all__ = [
    "BlockMatcher", "BlockMatcherGroup", "blockMatching_gpu", "block_matching_gpu", "SMError", "synth_pair", "bgr_to_gray",
    "SM_AGG_BOX", "SM_AGG_GUIDED", "SM_LR_CHECK", "SM_MEDIAN", "version", "host_empty",
]

DEFAULT_GUIDED_EPS = 1e-4 * 255.0 * 255.0


def version() -> str:
    return _capi.load().sm_version().decode()


def _as_u8_image(a, name: str) -> np.ndarray:
    a = np.asarray(a)
    if a.dtype != np.uint8 or a.ndim != 2:
        raise ValueError(f"{name}: expected a 2-D uint8 (CV_8UC1) image, got {a.dtype} {a.shape}")
    return a if a.flags.c_contiguous else np.ascontiguousarray(a)


def _flags(agg: str, lr_check: bool, median: bool = False) -> int:
    """agg: 'box' (fused), 'box-staged' (through the AD / SAD volumes in HBM), 'guided', or 'device-cu'
    (Device.cu's literal output with its fixed launch geometry: SM_DEVICE_CU_GRID, box only)."""
    if agg not in ("box", "guided", "box-staged", "device-cu"):
        raise ValueError("agg must be 'box', 'box-staged', 'guided' or 'device-cu'")
    f = {"box": SM_AGG_BOX, "guided": SM_AGG_GUIDED, "box-staged": SM_AGG_BOX | SM_STAGED,
         "device-cu": SM_DEVICE_CU_GRID}[agg]
    return f | (SM_LR_CHECK if lr_check else 0) | (SM_MEDIAN if median else 0)


def _check_out(out_t, shape, dtype, device, name: str = "out_t"):
    """A caller-supplied output tensor: the C ABI writes prod(shape) elements through its raw pointer."""
    if out_t.dtype != dtype or tuple(out_t.shape) != tuple(shape) or not out_t.is_contiguous() \
            or out_t.device != device:
        raise ValueError(f"{name} must be a contiguous {dtype} tensor of shape {tuple(shape)} on {device}")


def _check_device_pair(left_t, right_t, keys_t=None):
    """[H, W] uint8 contiguous device frames of one shape (and an int32 [H, W] key map when given):
    the C ABI takes raw pointers and cannot check what they point at."""
    import torch
    if left_t.dtype != torch.uint8 or right_t.dtype != torch.uint8:
        raise ValueError("expected uint8 tensors")
    if left_t.shape != right_t.shape or left_t.dim() != 2:
        raise ValueError("left/right must be equal [H, W] tensors")
    if not (left_t.is_cuda and right_t.is_cuda and left_t.is_contiguous() and right_t.is_contiguous()):
        raise ValueError("expected contiguous device tensors")
    if keys_t is not None and (keys_t.dtype != torch.int32 or tuple(keys_t.shape) != tuple(left_t.shape)
                               or not keys_t.is_contiguous() or keys_t.device != left_t.device):
        raise ValueError("keys_t must be a contiguous int32 [H, W] tensor on the frames' device")


class _PinnedBlock:
    """Owner of one sm_host_alloc block; freed when the last array viewing it goes away."""

    def __init__(self, nbytes: int):
        self._lib = _capi.load()
        p = ctypes.c_void_p()
        _capi.check(self._lib.sm_host_alloc(nbytes, ctypes.byref(p)))
        self.ptr = p.value
        self.nbytes = nbytes

    def __del__(self):
        if getattr(self, "ptr", None):
            self._lib.sm_host_free(ctypes.c_void_p(self.ptr))
            self.ptr = None


def host_empty(shape, dtype=np.uint8) -> np.ndarray:
    """An uninitialised numpy array in page-locked host memory (``sm_host_alloc``): frames and maps
    kept here go to / from HBM as direct DMA in ``BlockMatcher.match`` and friends."""
    dt = np.dtype(dtype)
    n = int(np.prod(shape)) * dt.itemsize
    blk = _PinnedBlock(max(n, 1))
    buf = (ctypes.c_uint8 * max(n, 1)).from_address(blk.ptr)
    buf._sm_owner = blk  # the ctypes buffer keeps the block alive, and the array keeps the buffer
    return np.frombuffer(buf, dtype=dt, count=n // dt.itemsize).reshape(shape)


class BlockMatcher:
    """One device handle: pre-allocated buffers + a HIP stream (``sm_create``)."""

    def __init__(self, device: int = 0, max_width: int = 1920, max_height: int = 1080, max_disp: int = 256):
        self._lib = _capi.load()
        h = ctypes.c_void_p()
        _capi.check(self._lib.sm_create(device, max_width, max_height, max_disp, ctypes.byref(h)))
        self._h = h
        self.device = device
        self.max_width, self.max_height, self.max_disp = max_width, max_height, max_disp

    # -- lifetime ---------------------------------------------------------------------
    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.sm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_guided_eps(self, eps: float):
        _capi.check(self._lib.sm_set_param_f(self._h, _capi.SM_PARAM_GUIDED_EPS, float(eps)))

    def dslice_rehearse(self, left, right, radius: int, num_disp: int, members: int, agg: str = "box",
                        lr_check: bool = False) -> np.ndarray:
        """The d-slice split of BlockMatcherGroup.match_dslice with `members` members, run one after
        another on this device (sm_dslice_rehearse_u8): same slice plan, padding and finalisation, with
        the RCCL MIN reduce-scatter replaced by an elementwise MIN of the members' key maps.  lr_check:
        the right view's keys take a second MIN and the map is LR-checked (StereoDisparity.cpp:136-147)."""
        if agg not in ("box", "guided"):
            raise ValueError("agg must be 'box' or 'guided'")
        L = _as_u8_image(left, "left")
        R = _as_u8_image(right, "right")
        if L.shape != R.shape:
            raise ValueError("left/right sizes differ")
        H, W = L.shape
        out = np.empty((H, W), np.uint8)
        _capi.check(self._lib.sm_dslice_rehearse_u8(self._h, L.ctypes.data, R.ctypes.data, W, H, W, radius, num_disp,
                                                    _flags(agg, lr_check, False), members, out.ctypes.data, W))
        return out

    # -- host-pointer path (blockMatching_gpu replacement) -------------------------------
    def match(self, left, right, radius: int, num_disp: int, agg: str = "box", lr_check: bool = False,
              median: bool = False, out: Optional[np.ndarray] = None) -> np.ndarray:
        """median=True: 7x7 median of the WTA map(s) (STMatching MeanFilter(disp, disp, 3)), before the LR check.
        out: optional contiguous uint8 [H, W] host buffer (e.g. pinned memory) to write the map into."""
        L = _as_u8_image(left, "left")
        R = _as_u8_image(right, "right")
        if L.shape != R.shape:
            raise ValueError("left/right sizes differ")
        H, W = L.shape
        if out is None:
            out = np.empty((H, W), np.uint8)
        elif out.dtype != np.uint8 or out.shape != (H, W) or not out.flags.c_contiguous:
            raise ValueError("out must be a contiguous uint8 array of the frame's shape")
        _capi.check(self._lib.sm_block_match_u8(self._h, L.ctypes.data, R.ctypes.data, W, H, W, radius, num_disp,
                                                _flags(agg, lr_check, median), out.ctypes.data, W))
        return out

    def match_lr(self, left, right, radius: int, num_disp: int, agg: str = "box", median: bool = False
                 ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(checked disparity, right-view disparity, valid mask)."""
        L = _as_u8_image(left, "left")
        R = _as_u8_image(right, "right")
        H, W = L.shape
        out = np.empty((H, W), np.uint8)
        rd = np.empty((H, W), np.uint8)
        mask = np.empty((H, W), np.uint8)
        _capi.check(self._lib.sm_block_match_lr_u8(self._h, L.ctypes.data, R.ctypes.data, W, H, W, radius, num_disp,
                                                   _flags(agg, True, median), out.ctypes.data, rd.ctypes.data,
                                                   mask.ctypes.data, W))
        return out, rd, mask

    def match_bgr(self, left_bgr, right_bgr, radius: int, num_disp: int, agg: str = "box",
                  lr_check: bool = False) -> np.ndarray:
        """imread -> cvtColor(BGR2GRAY) -> blockMatching_gpu in one call (Caller.cpp:12-19): HxWx3/4
        uint8 BGR(A) frames in, uint8 disparity out; the gray conversion runs on the GPU."""
        Lb = np.ascontiguousarray(left_bgr, dtype=np.uint8)
        Rb = np.ascontiguousarray(right_bgr, dtype=np.uint8)
        if Lb.ndim != 3 or Lb.shape[2] not in (3, 4) or Lb.shape != Rb.shape:
            raise ValueError("expected two equal HxWx3 or HxWx4 uint8 BGR(A) frames")
        H, W, C = Lb.shape
        out = np.empty((H, W), np.uint8)
        _capi.check(self._lib.sm_block_match_bgr_u8(self._h, Lb.ctypes.data, Rb.ctypes.data, W, H, W * C, C, radius,
                                                    num_disp, _flags(agg, lr_check), out.ctypes.data, W))
        return out

    def segment_tree(self, left_bgr, right_bgr, max_level: int = 60, scale: int = 4, sigma: float = 0.1,
                     method: int = 0) -> np.ndarray:
        """STMatching's segment-tree stereo on HxWx3 uint8 BGR frames, `method` as STMatching/main.cpp's
        7th argument (defaults as its :49-52):
          0 = ST-1 (stereo_disparity_normal, StereoDisparity.cpp:57-89): colour + gradient cost over
              d < max_level -> tree aggregation on the left view's colour tree -> WTA -> 7x7 median -> x scale;
          1 = ST-2 (stereo_disparity_iteration, :91-160): first-pass left / right maps on colour trees of
              each view, the left-right check, then a colour + depth tree on the left view.
        Cost, filter, WTA, median, LR check and the trees' BFS on the GPU; segment_graph's passes on the
        host (sequential, as the reference's)."""
        Lb = np.ascontiguousarray(left_bgr, dtype=np.uint8)
        Rb = np.ascontiguousarray(right_bgr, dtype=np.uint8)
        if Lb.ndim != 3 or Lb.shape[2] != 3 or Lb.shape != Rb.shape:
            raise ValueError("expected two equal HxWx3 uint8 BGR frames")
        if method not in (0, 1):
            raise ValueError(f"method must be 0 (ST-1) or 1 (ST-2), got {method}")
        H, W, _ = Lb.shape
        out = np.empty((H, W), np.uint8)
        fn = self._lib.sm_segment_tree_refined_bgr_u8 if method else self._lib.sm_segment_tree_match_bgr_u8
        _capi.check(fn(self._h, Lb.ctypes.data, Rb.ctypes.data, W, H, 3 * W, max_level, scale, sigma,
                       out.ctypes.data, W))
        return out

    def segment_tree_stats(self) -> Tuple[float, float, int]:
        """(tree-build ms, whole-call ms, BFS levels of the last tree) of the last segment_tree call."""
        t, a, n = ctypes.c_float(), ctypes.c_float(), ctypes.c_int()
        _capi.check(self._lib.sm_last_segment_tree_stats(self._h, ctypes.byref(t), ctypes.byref(a), ctypes.byref(n)))
        return t.value, a.value, n.value

    def segment_tree_arrays(self, width: int, height: int) -> dict:
        """The last segment_tree call's last tree in BFS order (sm_last_segment_tree_arrays): rank, parent,
        first, child, lev (levels + 1 offsets) and pdist, for a width x height frame."""
        P = int(width) * int(height)
        ints = np.empty(5 * P + 2, np.int32)
        pdist = np.empty(P, np.uint8)
        n = ctypes.c_int()
        _capi.check(self._lib.sm_last_segment_tree_arrays(self._h, ints.ctypes.data, ints.size, pdist.ctypes.data,
                                                          pdist.size, ctypes.byref(n)))
        return {"rank": ints[:P].copy(), "parent": ints[P:2 * P].copy(), "first": ints[2 * P:3 * P].copy(),
                "child": ints[3 * P:4 * P].view(np.uint32).copy(), "lev": ints[4 * P:4 * P + n.value + 1].copy(),
                "pdist": pdist}

    def cvt_color(self, bgr) -> np.ndarray:
        """cvtColor_gpu (Device.cuh:52) on host memory: HxWx3|4 uint8 BGR(A) -> gray, OpenCV 2.4 weights."""
        B = np.ascontiguousarray(bgr, dtype=np.uint8)
        if B.ndim != 3 or B.shape[2] not in (3, 4):
            raise ValueError("expected an HxWx3 or HxWx4 uint8 BGR(A) image")
        H, W, C = B.shape
        out = np.empty((H, W), np.uint8)
        _capi.check(self._lib.sm_bgr_to_gray_u8(self._h, B.ctypes.data, W, H, W * C, C, out.ctypes.data, W))
        return out

    def remap(self, src, mapx, mapy) -> np.ndarray:
        """remap_gpu (Device.cuh:51) on host memory: uint8 [H, W] with CV_32FC1 maps [H, W]."""
        S = _as_u8_image(src, "src")
        mx = np.ascontiguousarray(mapx, dtype=np.float32)
        my = np.ascontiguousarray(mapy, dtype=np.float32)
        if mx.shape != S.shape or my.shape != S.shape:
            raise ValueError("maps must match the image shape")
        H, W = S.shape
        out = np.empty((H, W), np.uint8)
        _capi.check(self._lib.sm_remap_u8(self._h, S.ctypes.data, W, H, W, mx.ctypes.data, my.ctypes.data, W,
                                          out.ctypes.data, W))
        return out

    def ad_volume(self, left, right, num_disp: int) -> np.ndarray:
        """PreCal (BlockMatching.cpp:89-109) on the GPU: uint8 [num_disp, H, W], d-major, 0 where x < d."""
        L = _as_u8_image(left, "left")
        R = _as_u8_image(right, "right")
        H, W = L.shape
        out = np.empty((num_disp, H, W), np.uint8)
        _capi.check(self._lib.sm_ad_volume_u8(self._h, L.ctypes.data, R.ctypes.data, W, H, W, num_disp,
                                              out.ctypes.data))
        return out

    def all_sad(self, left, right, radius: int, num_disp: int) -> np.ndarray:
        """getAllSAD (BlockMatching.cpp:191-261) on the GPU: uint8 [H, W, num_disp] (pixel-major
        ``data_dm[p * D + d]``), each window SAD truncated to uchar, 255 where x + d > W."""
        L = _as_u8_image(left, "left")
        R = _as_u8_image(right, "right")
        H, W = L.shape
        out = np.empty((H, W, num_disp), np.uint8)
        _capi.check(self._lib.sm_all_sad_u8(self._h, L.ctypes.data, R.ctypes.data, W, H, W, radius, num_disp,
                                            out.ctypes.data))
        return out

    def all_sad_device(self, left_t, right_t, radius: int, num_disp: int, out_t=None, stream=None):
        """Device form of :meth:`all_sad`: uint8 [H, W, num_disp] CUDA tensor, async on `stream`."""
        import torch
        H, W = left_t.shape
        if out_t is None:
            out_t = torch.empty((H, W, num_disp), dtype=torch.uint8, device=left_t.device)
        _check_out(out_t, (H, W, num_disp), torch.uint8, left_t.device)
        _capi.check(self._lib.sm_all_sad_device(self._h, left_t.data_ptr(), right_t.data_ptr(), W, H, W, radius,
                                                num_disp, out_t.data_ptr(), self._stream_ptr(stream)))
        return out_t

    def sad_volume_device(self, left_t, right_t, radius: int, num_disp: int, out_t=None, stream=None):
        """u16 SAD volume [num_disp, H, W]: zero-padded (2r+1)^2 window sums of the AD planes."""
        import torch
        H, W = left_t.shape
        if out_t is None:
            out_t = torch.empty((num_disp, H, W), dtype=torch.int16, device=left_t.device)
        _capi.check(self._lib.sm_sad_volume_device(self._h, left_t.data_ptr(), right_t.data_ptr(), W, H, W, radius,
                                                   num_disp, out_t.data_ptr(), self._stream_ptr(stream)))
        return out_t

    def ad_volume_device(self, left_t, right_t, num_disp: int, out_t=None, stream=None):
        import torch
        H, W = left_t.shape
        if out_t is None:
            out_t = torch.empty((num_disp, H, W), dtype=torch.uint8, device=left_t.device)
        _capi.check(self._lib.sm_ad_volume_device(self._h, left_t.data_ptr(), right_t.data_ptr(), W, H, W, num_disp,
                                                  out_t.data_ptr(), self._stream_ptr(stream)))
        return out_t

    def bgr_to_gray_device(self, bgr_t, out_t=None, stream=None):
        """[H, W, 3|4] uint8 cuda tensor -> [H, W] gray (OpenCV 2.4 fixed point), async on `stream`."""
        import torch
        H, W, C = bgr_t.shape
        if out_t is None:
            out_t = torch.empty((H, W), dtype=torch.uint8, device=bgr_t.device)
        _capi.check(self._lib.sm_bgr_to_gray_device(self._h, bgr_t.data_ptr(), W, H, W * C, C, out_t.data_ptr(), W,
                                                    self._stream_ptr(stream)))
        return out_t

    def remap_device(self, src_t, mapx_t, mapy_t, out_t=None, stream=None):
        """Rectification remap (Device.cu:127-167): src [H, W] uint8, maps [H, W] float32 (CV_32FC1)."""
        import torch
        H, W = src_t.shape
        if out_t is None:
            out_t = torch.empty_like(src_t)
        _capi.check(self._lib.sm_remap_u8_device(self._h, src_t.data_ptr(), W, H, W, mapx_t.data_ptr(),
                                                 mapy_t.data_ptr(), W, out_t.data_ptr(), W, self._stream_ptr(stream)))
        return out_t

    @staticmethod
    def _map_args(K, dist, R, P):
        K = np.ascontiguousarray(K, np.float64).reshape(9)
        d = np.ascontiguousarray(dist if dist is not None else [], np.float64).ravel()
        R = np.ascontiguousarray(R, np.float64).reshape(9)
        P = np.ascontiguousarray(P, np.float64).reshape(12)
        return K, d, R, P

    def init_rectify_map(self, K, dist, R, P, width: int, height: int):
        """initUndistortRectifyMap(K, dist, R, P, (width, height), CV_32FC1) computed on the GPU
        (Utility.cpp:232-233): float32 (mapx, mapy) host arrays [height, width]."""
        K, d, R, P = self._map_args(K, dist, R, P)
        mx = np.empty((height, width), np.float32)
        my = np.empty((height, width), np.float32)
        vp = ctypes.c_void_p
        _capi.check(self._lib.sm_init_rectify_map(self._h, K.ctypes.data_as(vp), d.ctypes.data_as(vp) if d.size else None,
                                                  d.size, R.ctypes.data_as(vp), P.ctypes.data_as(vp), width, height,
                                                  mx.ctypes.data, my.ctypes.data, width))
        return mx, my

    def init_rectify_map_device(self, K, dist, R, P, width: int, height: int, mapx_t=None, mapy_t=None, stream=None):
        """Device form of :meth:`init_rectify_map`: float32 [height, width] CUDA tensors."""
        import torch
        K, d, R, P = self._map_args(K, dist, R, P)
        if mapx_t is None:
            mapx_t = torch.empty((height, width), dtype=torch.float32, device=f"cuda:{self.device}")
        if mapy_t is None:
            mapy_t = torch.empty((height, width), dtype=torch.float32, device=f"cuda:{self.device}")
        vp = ctypes.c_void_p
        _capi.check(self._lib.sm_init_rectify_map_device(
            self._h, K.ctypes.data_as(vp), d.ctypes.data_as(vp) if d.size else None, d.size, R.ctypes.data_as(vp),
            P.ctypes.data_as(vp), width, height, mapx_t.data_ptr(), mapy_t.data_ptr(), mapx_t.stride(0),
            self._stream_ptr(stream)))
        return mapx_t, mapy_t

    def median_device(self, src_t, radius: int = 3, out_t=None, stream=None):
        """(2r+1)^2 median, replicate borders (ctmf, STMatching/ctmf.c), r in 1..3; src [H, W] uint8."""
        import torch
        H, W = src_t.shape
        if out_t is None:
            out_t = torch.empty_like(src_t)
        _capi.check(self._lib.sm_median_u8_device(self._h, src_t.data_ptr(), W, H, W, radius, out_t.data_ptr(), W,
                                                  self._stream_ptr(stream)))
        return out_t

    def set_stage_timing(self, on) -> None:
        """Record the host calls' upload / match / download split: True always, False never (stage_ms()
        then reads 0), "auto" (the default) from the first stage_ms() call on.  Each recording costs two
        hipEvent markers between the stages, ~10 us per 1080p call."""
        v = 2.0 if on == "auto" else (1.0 if on else 0.0)
        _capi.check(self._lib.sm_set_param_f(self._h, _capi.SM_PARAM_STAGE_TIMING, v))

    def stage_ms(self) -> Tuple[float, float, float]:
        """(upload, match, download) ms of the last host call (Device.cu:218,238/257,292).  With the
        default "auto" timing the first read arms the recording for the calls after it."""
        u, m, d = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
        _capi.check(self._lib.sm_last_stage_ms(self._h, ctypes.byref(u), ctypes.byref(m), ctypes.byref(d)))
        return u.value, m.value, d.value

    def staged_kernel_ms(self) -> Tuple[float, float, float]:
        """(AD volume, SAD volume, WTA) kernel ms per frame of the last launch group (up to 8 frames) of the
        last 'box-staged' pass."""
        a, b, c = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
        _capi.check(self._lib.sm_last_staged_kernel_ms(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)))
        return a.value, b.value, c.value

    # -- device-resident path (torch tensors in HBM) ------------------------------------
    @staticmethod
    def _stream_ptr(stream):
        if stream is None:
            import torch
            stream = torch.cuda.current_stream()
        return ctypes.c_void_p(stream.cuda_stream)

    def match_device(self, left_t, right_t, radius: int, num_disp: int, out_t=None, agg: str = "box",
                     lr_check: bool = False, stream=None, median: bool = False):
        """left_t/right_t: uint8 cuda tensors [H, W] or [B, H, W] (contiguous). Async on `stream`."""
        import torch
        if left_t.dtype != torch.uint8 or right_t.dtype != torch.uint8:
            raise ValueError("expected uint8 tensors")
        if left_t.shape != right_t.shape or left_t.dim() not in (2, 3):
            raise ValueError("left/right must be equal [H,W] or [B,H,W]")
        if not (left_t.is_cuda and right_t.is_cuda and left_t.is_contiguous() and right_t.is_contiguous()):
            raise ValueError("expected contiguous device tensors")
        if left_t.device != right_t.device or left_t.device.index != self.device:
            raise ValueError(f"frames must be on cuda:{self.device}, the handle's device")
        B = 1 if left_t.dim() == 2 else left_t.shape[0]
        H, W = left_t.shape[-2:]
        if out_t is None:
            out_t = torch.empty_like(left_t)
        _check_out(out_t, left_t.shape, torch.uint8, left_t.device)
        _capi.check(self._lib.sm_match_device(self._h, left_t.data_ptr(), right_t.data_ptr(), W, H, W, B, H * W,
                                              radius, num_disp, _flags(agg, lr_check, median), out_t.data_ptr(), W, H * W,
                                              self._stream_ptr(stream)))
        return out_t

    def slice_keys_device(self, left_t, right_t, radius: int, d_lo: int, d_hi: int, keys_t=None, stream=None):
        """Packed (SAD<<8|d) keys of the d-slice [d_lo, d_hi) as an int32 tensor (bit pattern of uint32)."""
        import torch
        H, W = left_t.shape[-2:]
        if keys_t is None:
            keys_t = torch.empty((H, W), dtype=torch.int32, device=left_t.device)
        _check_device_pair(left_t, right_t, keys_t)
        _capi.check(self._lib.sm_slice_keys_device(self._h, left_t.data_ptr(), right_t.data_ptr(), W, H, W, radius,
                                                   d_lo, d_hi, keys_t.data_ptr(), self._stream_ptr(stream)))
        return keys_t

    def keys_to_disp_device(self, keys_t, radius: int, out_t=None, stream=None):
        import torch
        H, W = keys_t.shape[-2:]
        if keys_t.dtype != torch.int32 or not keys_t.is_cuda or not keys_t.is_contiguous():
            raise ValueError("keys_t must be a contiguous int32 device tensor")
        if out_t is None:
            out_t = torch.empty((H, W), dtype=torch.uint8, device=keys_t.device)
        _check_out(out_t.view(-1) if out_t.is_contiguous() else out_t, (H * W,), torch.uint8, keys_t.device)
        _capi.check(self._lib.sm_keys_to_disp_device(self._h, keys_t.data_ptr(), W, H, radius, out_t.data_ptr(), W,
                                                     self._stream_ptr(stream)))
        return out_t

    def guided_slice_keys_device(self, left_t, right_t, radius: int, d_lo: int, d_hi: int, keys_t=None,
                                 stream=None):
        """Guided-aggregation d-slice keys ((int32)(q * 2^14) << 8 | d, INT32_MAX where no d of the slice
        is valid) as an int32 [H, W] tensor; disjoint slices combine with a signed elementwise min."""
        import torch
        H, W = left_t.shape[-2:]
        if keys_t is None:
            keys_t = torch.empty((H, W), dtype=torch.int32, device=left_t.device)
        _check_device_pair(left_t, right_t, keys_t)
        _capi.check(self._lib.sm_guided_slice_keys_device(self._h, left_t.data_ptr(), right_t.data_ptr(), W, H, W,
                                                          radius, d_lo, d_hi, keys_t.data_ptr(),
                                                          self._stream_ptr(stream)))
        return keys_t

    def slice_keys_lr_device(self, left_t, right_t, radius: int, d_lo: int, d_hi: int, agg: str = "box",
                             keys_t=None, right_keys_t=None, stream=None):
        """Left AND right-view d-slice keys of [d_lo, d_hi) from one fused pass (sm_slice_keys_lr_device): int32
        [H, W] tensors holding the bit patterns of box uint32 keys (combine with an unsigned MIN) or guided
        int32 keys (signed MIN).  The right view's key of u is its best (cost << 8 | d) over the slice's d with
        u + d < W, C_R(u, d) = C_L(u + d, d) (StereoHelper.cpp:156-180)."""
        import torch
        if agg not in ("box", "guided"):
            raise ValueError("agg must be 'box' or 'guided'")
        H, W = left_t.shape[-2:]
        if keys_t is None:
            keys_t = torch.empty((H, W), dtype=torch.int32, device=left_t.device)
        if right_keys_t is None:
            right_keys_t = torch.empty((H, W), dtype=torch.int32, device=left_t.device)
        _check_device_pair(left_t, right_t, keys_t)
        _check_device_pair(left_t, right_t, right_keys_t)
        _capi.check(self._lib.sm_slice_keys_lr_device(self._h, left_t.data_ptr(), right_t.data_ptr(), W, H, W, radius,
                                                      d_lo, d_hi, _flags(agg, False), keys_t.data_ptr(),
                                                      right_keys_t.data_ptr(), self._stream_ptr(stream)))
        return keys_t, right_keys_t

    def right_keys_to_disp_device(self, keys_t, out_t=None, stream=None):
        """Combined right-view keys (any shape, int32) -> dR, the d field of each key (no threshold)."""
        import torch
        if keys_t.dtype != torch.int32 or not keys_t.is_contiguous() or not keys_t.is_cuda:
            raise ValueError("keys_t must be a contiguous int32 device tensor")
        if out_t is None:
            out_t = torch.empty(keys_t.shape, dtype=torch.uint8, device=keys_t.device)
        _check_out(out_t, keys_t.shape, torch.uint8, keys_t.device)
        _capi.check(self._lib.sm_right_keys_to_disp_device(self._h, keys_t.data_ptr(), keys_t.numel(), out_t.data_ptr(),
                                                           self._stream_ptr(stream)))
        return out_t

    def lr_check_device(self, left_disp_t, right_disp_t, out_t=None, mask_t=None, stream=None):
        """StereoDisparity.cpp:136-147 on [H, W] uint8 device maps: occluded (x - d < 0, d == 0 or
        |d - dR(x - d)| > 1) -> 0.  out_t may be left_disp_t (in place)."""
        import torch
        H, W = left_disp_t.shape
        for t in (left_disp_t, right_disp_t):
            _check_out(t, (H, W), torch.uint8, left_disp_t.device, "maps")
        if out_t is None:
            out_t = torch.empty_like(left_disp_t)
        _check_out(out_t, (H, W), torch.uint8, left_disp_t.device)
        if mask_t is not None:
            _check_out(mask_t, (H, W), torch.uint8, left_disp_t.device, "mask_t")
        _capi.check(self._lib.sm_lr_check_device(self._h, left_disp_t.data_ptr(), right_disp_t.data_ptr(), W, H, W,
                                                 out_t.data_ptr(), mask_t.data_ptr() if mask_t is not None else None,
                                                 W, self._stream_ptr(stream)))
        return out_t

    def guided_keys_to_disp_device(self, keys_t, out_t=None, stream=None):
        """Combined guided keys -> uint8 disparity (d where q < 50, else 0)."""
        import torch
        H, W = keys_t.shape[-2:]
        if keys_t.dtype != torch.int32 or not keys_t.is_cuda or not keys_t.is_contiguous():
            raise ValueError("keys_t must be a contiguous int32 device tensor")
        if out_t is None:
            out_t = torch.empty((H, W), dtype=torch.uint8, device=keys_t.device)
        _check_out(out_t.view(-1) if out_t.is_contiguous() else out_t, (H * W,), torch.uint8, keys_t.device)
        _capi.check(self._lib.sm_guided_keys_to_disp_device(self._h, keys_t.data_ptr(), W, H, out_t.data_ptr(), W,
                                                            self._stream_ptr(stream)))
        return out_t


class BlockMatcherGroup:
    """Several GPUs driven from this process through the C ABI's group handle (``sm_create_group``):
    one frame in row bands (one band per device, bit-identical to a single-device pass), or a batch
    of frames spread over the devices.  ``devices`` may repeat an index (several handles on one GPU)."""

    def __init__(self, devices: Sequence[int], max_width: int = 1920, max_height: int = 1080, max_disp: int = 256):
        self._lib = _capi.load()
        devs = (ctypes.c_int * len(devices))(*devices)
        g = ctypes.c_void_p()
        _capi.check(self._lib.sm_create_group(len(devices), devs, max_width, max_height, max_disp, ctypes.byref(g)))
        self._g = g
        self.devices = list(devices)

    def close(self):
        if getattr(self, "_g", None) is not None and self._g.value:
            self._lib.sm_destroy_group(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __len__(self):
        n = ctypes.c_int()
        _capi.check(self._lib.sm_group_size(self._g, ctypes.byref(n)))
        return n.value

    def set_guided_eps(self, eps: float):
        _capi.check(self._lib.sm_group_set_param_f(self._g, _capi.SM_PARAM_GUIDED_EPS, float(eps)))

    def match(self, left, right, radius: int, num_disp: int, agg: str = "box", lr_check: bool = False,
              median: bool = False) -> np.ndarray:
        """One frame, row-banded over the group (sm_group_block_match_u8)."""
        L = _as_u8_image(left, "left")
        R = _as_u8_image(right, "right")
        if L.shape != R.shape:
            raise ValueError("left/right sizes differ")
        H, W = L.shape
        out = np.empty((H, W), np.uint8)
        _capi.check(self._lib.sm_group_block_match_u8(self._g, L.ctypes.data, R.ctypes.data, W, H, W, radius,
                                                      num_disp, _flags(agg, lr_check, median), out.ctypes.data, W))
        return out

    def match_lr(self, left, right, radius: int, num_disp: int, agg: str = "box", median: bool = False
                 ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(checked disparity, right-view disparity, valid mask), row-banded over the group."""
        L = _as_u8_image(left, "left")
        R = _as_u8_image(right, "right")
        H, W = L.shape
        out, rd, mask = (np.empty((H, W), np.uint8) for _ in range(3))
        _capi.check(self._lib.sm_group_block_match_lr_u8(self._g, L.ctypes.data, R.ctypes.data, W, H, W, radius,
                                                         num_disp, _flags(agg, True, median), out.ctypes.data,
                                                         rd.ctypes.data, mask.ctypes.data, W))
        return out, rd, mask

    def match_dslice(self, left, right, radius: int, num_disp: int, agg: str = "box",
                     lr_check: bool = False) -> np.ndarray:
        """One frame sharded over disparities (sm_group_dslice_block_match_u8): each member matches
        its slice of [0, num_disp), RCCL MIN reduce-scatter + all-gather over the members' devices.
        lr_check: the right view's slice keys take a second reduce-scatter + all-gather and the map is
        LR-checked.  Members must be distinct devices."""
        if agg not in ("box", "guided"):
            raise ValueError("agg must be 'box' or 'guided'")
        L = _as_u8_image(left, "left")
        R = _as_u8_image(right, "right")
        if L.shape != R.shape:
            raise ValueError("left/right sizes differ")
        H, W = L.shape
        out = np.empty((H, W), np.uint8)
        _capi.check(self._lib.sm_group_dslice_block_match_u8(self._g, L.ctypes.data, R.ctypes.data, W, H, W, radius,
                                                             num_disp, _flags(agg, lr_check, False), out.ctypes.data, W))
        return out

    def match_batch(self, lefts, rights, radius: int, num_disp: int, agg: str = "box", lr_check: bool = False,
                    median: bool = False):
        """A list of equal-size pairs; frame f runs on member f mod len(group)."""
        Ls = [_as_u8_image(a, "left") for a in lefts]
        Rs = [_as_u8_image(a, "right") for a in rights]
        if len(Ls) != len(Rs) or any(a.shape != Ls[0].shape for a in Ls + Rs):
            raise ValueError("expected equal-size left/right lists")
        if not Ls:
            return []
        H, W = Ls[0].shape
        outs = [np.empty((H, W), np.uint8) for _ in Ls]
        n = len(Ls)
        ptrs = lambda arrs: (ctypes.c_void_p * n)(*[a.ctypes.data for a in arrs])  # noqa: E731
        _capi.check(self._lib.sm_group_block_match_batch_u8(self._g, ptrs(Ls), ptrs(Rs), n, W, H, W, radius,
                                                            num_disp, _flags(agg, lr_check, median), ptrs(outs), W))
        return outs


_default: Optional[BlockMatcher] = None


def _default_matcher(W: int, H: int, D: int) -> BlockMatcher:
    global _default
    if _default is None or W > _default.max_width or H > _default.max_height or D > _default.max_disp:
        if _default is not None:
            _default.close()
        _default = BlockMatcher(0, max(W, 1920), max(H, 1080), 256)
    return _default


def blockMatching_gpu(h_left, h_right, SADWindowSize: int, searchRange: int) -> np.ndarray:
    """Drop-in for ``blockMatching_gpu`` (Device.cu:173): returns the uint8 disparity map.

    Prints the reference's four stage lines in ms, as Device.cu:218,238,257,292 always does:
    "upload data", "pre calculation" (0: the AD cost is fused into the match), "find corr" and
    "download data".  ``SM_QUIET`` in the environment silences them.
    """
    import os
    L = _as_u8_image(h_left, "h_left")
    m = _default_matcher(L.shape[1], L.shape[0], searchRange)
    quiet = bool(os.environ.get("SM_QUIET"))
    if not quiet:
        m.set_stage_timing(True)
    out = m.match(L, h_right, SADWindowSize, searchRange)
    if not quiet:
        u, c, d = m.stage_ms()
        print(f"upload data : {u:g}\npre calculation : 0\nfind corr : {c:g}\ndownload data : {d:g}")
    return out


block_matching_gpu = blockMatching_gpu
