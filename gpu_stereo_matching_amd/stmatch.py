"""STMatching's command line (STMatching/main.cpp:40-72, stereo_routine at StereoDisparity.cpp:41-55) on the
GPU segment-tree path:

    python -m gpu_stereo_matching_amd.stmatch leftImgPath rightImgPath dispImgPath [maxLevel] [scale] [sigma] [method]

Same positional arguments and defaults as main.cpp (maxLevel 60, scale 4, sigma 0.1, method 0 = ST-1, any
non-zero method = ST-2).  The images are read as 3-channel BGR, as cv::imread does by default, and the map is
written as an 8-bit image.  Decoding uses PIL, not OpenCV: a JPEG may decode to slightly different pixels
than the reference's cv::imread, so only lossless inputs (PNG, PPM, BMP) are pinned to the reference.
"""
from __future__ import annotations

import sys
from typing import List, Optional

import numpy as np

__all__ = ["stereo_routine"]


def _read_bgr(path: str) -> np.ndarray:
    from PIL import Image
    with Image.open(path) as im:
        rgb = np.asarray(im.convert("RGB"), dtype=np.uint8)
    return np.ascontiguousarray(rgb[:, :, ::-1])


def stereo_routine(left_input: str, right_input: str, output: str, max_dis_level: int = 60, scale: int = 4,
                   sigma: float = 0.1, method: int = 0, device: int = 0) -> np.ndarray:
    """stereo_routine (StereoDisparity.cpp:41-55): read both views, ST-1 (method 0) or ST-2 (otherwise),
    write the map to `output`; returns the map."""
    from PIL import Image
    from . import BlockMatcher

    L, R = _read_bgr(left_input), _read_bgr(right_input)
    if L.shape != R.shape:
        raise ValueError(f"{left_input} and {right_input} differ in size ({L.shape[1]}x{L.shape[0]} vs "
                         f"{R.shape[1]}x{R.shape[0]})")
    H, W = L.shape[:2]
    with BlockMatcher(device, W, H, max(1, min(int(max_dis_level), 256))) as m:
        disp = m.segment_tree(L, R, max_dis_level, scale, sigma, method=1 if method else 0)
    Image.fromarray(disp).save(output)
    return disp


def _main(argv: Optional[List[str]] = None) -> int:
    a = sys.argv[1:] if argv is None else argv
    if len(a) < 3:
        print("*****Segment-Tree based Cost Aggregation for Stereo Matching[CVPR2013]*****\n")
        print("Usage:\npython -m gpu_stereo_matching_amd.stmatch leftImgPath rightImgPath dispImgPath "
              "[maxLevel] [scale] [sigma] [method]")
        print("maxDispLevel: default 60\nscale: default 4\nsigma: default 0.1\nmethod: 0 (default, ST-1) or 1 (ST-2)")
        return 0
    max_level = int(a[3]) if len(a) > 3 else 60
    scale = int(a[4]) if len(a) > 4 else 4
    sigma = float(a[5]) if len(a) > 5 else 0.1
    method = int(a[6]) if len(a) > 6 else 0
    stereo_routine(a[0], a[1], a[2], max_level, scale, sigma, method)
    return 0


if __name__ == "__main__":
    raise SystemExit(_main())
