"""BGR(A) -> gray as the reference's caller does it (BlockMatching/Caller.cpp:15-16,
``cvtColor(left, g1, CV_BGR2GRAY)`` under OpenCV 2.4.12): 8-bit fixed point
Y = (1868*B + 9617*G + 4899*R + 8192) >> 14.  Host-side preprocessing, not the hot path.
"""
from __future__ import annotations

import numpy as np


def bgr_to_gray(bgr: np.ndarray) -> np.ndarray:
    bgr = np.asarray(bgr)
    if bgr.ndim != 3 or bgr.shape[2] not in (3, 4) or bgr.dtype != np.uint8:
        raise ValueError("expected HxWx3 or HxWx4 uint8 BGR(A)")
    b = bgr[..., 0].astype(np.uint32)
    g = bgr[..., 1].astype(np.uint32)
    r = bgr[..., 2].astype(np.uint32)
    return ((1868 * b + 9617 * g + 4899 * r + 8192) >> 14).astype(np.uint8)
