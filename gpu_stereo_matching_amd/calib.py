"""Stereo calibration and rectification maps: the caller-side steps in front of the remap.

Mirrors the reference's remapTest chain (BlockMatching/Caller.cpp:27-74):
  LoadDataBatch  (Utility.cpp:25-42)  -> :func:`load_data_batch` (OpenCV FileStorage YAML, read here
                                          without OpenCV; every matrix converted to float64 as the
                                          reference's ``convertTo(..., CV_64F)`` does)
  Rectify        (Utility.cpp:228-234) -> :func:`rectify` = :func:`stereo_rectify` (host math in the
                                          C ABI, ``sm_stereo_rectify``) + the GPU map kernel
                                          (``sm_init_rectify_map*``) for each camera
  remap_gpu      (Device.cu:303-342)   -> :meth:`BlockMatcher.remap` / ``remap_device``

Rectify is OpenCV 2.4.12 ``stereoRectify(..., CV_CALIB_ZERO_DISPARITY)`` (alpha = -1) followed by
``initUndistortRectifyMap(..., CV_32FC1)``; csrc/bm_rectify.hip restates both.  No CPU fallback:
the maps come from the HIP library or an error is raised.
"""
from __future__ import annotations

import ctypes
import re
from typing import Dict, Tuple

import numpy as np

from . import _capi

_DT = {"f": np.float32, "d": np.float64, "i": np.int32, "u": np.uint8, "c": np.int8, "w": np.uint16, "s": np.int16}


def load_opencv_yaml(path: str) -> Dict[str, np.ndarray]:
    """Every ``!!opencv-matrix`` node of an OpenCV FileStorage YAML file (``%YAML:1.0``), by name.

    Handles the block form OpenCV writes: ``name: !!opencv-matrix`` followed by indented ``rows``,
    ``cols``, ``dt`` and a ``data: [ ... ]`` list that may span lines.  Scalars and other node types
    are skipped."""
    text = open(path, "r", encoding="utf-8", errors="replace").read()
    out: Dict[str, np.ndarray] = {}
    for m in re.finditer(r"^\s*([A-Za-z_][\w]*)\s*:\s*!!opencv-matrix\s*$", text, flags=re.M):
        name = m.group(1)
        body = text[m.end():]
        nxt = re.search(r"^\s*[A-Za-z_][\w]*\s*:\s*!!", body, flags=re.M)
        body = body[:nxt.start()] if nxt else body
        rows = int(re.search(r"\brows\s*:\s*(\d+)", body).group(1))
        cols = int(re.search(r"\bcols\s*:\s*(\d+)", body).group(1))
        dt = re.search(r"\bdt\s*:\s*(\w)", body).group(1)
        data = re.search(r"\bdata\s*:\s*\[(.*?)\]", body, flags=re.S).group(1)
        vals = [float(v) for v in data.replace("\n", " ").split(",") if v.strip()]
        if len(vals) != rows * cols:
            raise ValueError(f"{path}: matrix {name} holds {len(vals)} values, expected {rows}x{cols}")
        out[name] = np.array(vals, dtype=_DT.get(dt, np.float64)).reshape(rows, cols)
    return out


def load_data(path: str, var_name: str) -> np.ndarray:
    """LoadData (Utility.cpp:17-23): one matrix by name, in its stored type."""
    return load_opencv_yaml(path)[var_name]


def load_data_batch(path: str) -> Tuple[np.ndarray, ...]:
    """LoadDataBatch (Utility.cpp:25-42): (camMat1, camMat2, distCoe1, distCoe2, R, T), float64."""
    m = load_opencv_yaml(path)
    names = ("LeftMat", "RightMat", "LeftDist", "RightDist", "RotationVec", "TranslationVec")
    missing = [n for n in names if n not in m]
    if missing:
        raise KeyError(f"{path}: missing {missing}")
    return tuple(m[n].astype(np.float64) for n in names)


def _dptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def stereo_rectify(K1, dist1, K2, dist2, image_size: Tuple[int, int], R, T):
    """OpenCV 2.4 ``stereoRectify`` with CV_CALIB_ZERO_DISPARITY and alpha = -1 (Utility.cpp:230).
    image_size = (width, height) as cv::Size.  Returns (R1, R2, P1, P2, Q) float64 [3x3, 3x3, 3x4, 3x4, 4x4]."""
    K1 = np.ascontiguousarray(K1, np.float64).reshape(9)
    K2 = np.ascontiguousarray(K2, np.float64).reshape(9)
    d1 = np.ascontiguousarray(dist1, np.float64).ravel()
    d2 = np.ascontiguousarray(dist2, np.float64).ravel()
    Rm = np.ascontiguousarray(R, np.float64).ravel()
    Tv = np.ascontiguousarray(T, np.float64).ravel()
    if Tv.size != 3:
        raise ValueError("T must hold 3 values")
    R1, R2 = np.empty(9), np.empty(9)
    P1, P2, Q = np.empty(12), np.empty(12), np.empty(16)
    w, h = image_size
    lib = _capi.load()
    _capi.check(lib.sm_stereo_rectify(_dptr(K1), _dptr(d1) if d1.size else None, d1.size, _dptr(K2),
                                      _dptr(d2) if d2.size else None, d2.size, int(w), int(h), _dptr(Rm), Rm.size,
                                      _dptr(Tv), _dptr(R1), _dptr(R2), _dptr(P1), _dptr(P2), _dptr(Q)))
    return R1.reshape(3, 3), R2.reshape(3, 3), P1.reshape(3, 4), P2.reshape(3, 4), Q.reshape(4, 4)


def rectify(matcher, camMat1, camMat2, distCoe1, distCoe2, R, T, image_size: Tuple[int, int]):
    """Rectify (Utility.cpp:228-234): stereoRectify, then the CV_32FC1 maps of both cameras on the
    GPU.  Returns (mapX1, mapY1, mapX2, mapY2), float32 [height, width] host arrays."""
    R1, R2, P1, P2, _ = stereo_rectify(camMat1, distCoe1, camMat2, distCoe2, image_size, R, T)
    w, h = image_size
    mx1, my1 = matcher.init_rectify_map(camMat1, distCoe1, R1, P1, w, h)
    mx2, my2 = matcher.init_rectify_map(camMat2, distCoe2, R2, P2, w, h)
    return mx1, my1, mx2, my2
