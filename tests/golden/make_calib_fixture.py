"""Generate the rectification fixtures (run in the build container, where the reference checkout is
mounted read-only at /root/reference; the GPU box never reads it).

* Calib_Data_OpenCV.yml — the reference's own stereo calibration (data file, copied byte for byte),
  read by remapTest through LoadDataBatch (Caller.cpp:50, Utility.cpp:25-42).
* chess_set2_gray.npz — the pair remapTest rectifies (Chess/Set2/{Left,Right}_0.jpg, Caller.cpp:33-34):
  JPEG decoded with PIL, converted to gray with OpenCV 2.4's fixed-point cvtColor weights
  (Caller.cpp:43-44), and stored at full size (1280x800) and at remapTest's 320x200.  The reduction
  to 320x200 is PIL's bilinear resize, not OpenCV's resize (input preparation only: every parity test
  compares the GPU and the oracle on these same bytes).

    python tests/golden/make_calib_fixture.py
"""
from __future__ import annotations

import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

REF = "/root/reference"


def gray_of(path: str, size=None) -> np.ndarray:
    from PIL import Image
    im = Image.open(path).convert("RGB")
    bgr = np.ascontiguousarray(np.array(im)[..., ::-1])
    g = O.bgr_to_gray(bgr)
    if size is not None:
        g = np.array(Image.fromarray(g).resize(size, Image.BILINEAR))
    return g.astype(np.uint8)


def main():
    shutil.copyfile(os.path.join(REF, "Calib_Data_OpenCV.yml"), os.path.join(HERE, "Calib_Data_OpenCV.yml"))
    out = {}
    for side in ("Left", "Right"):
        p = os.path.join(REF, "Chess", "Set2", f"{side}_0.jpg")
        out[f"{side}_full"] = gray_of(p)
        out[f"{side}_320x200"] = gray_of(p, (320, 200))
    np.savez_compressed(os.path.join(HERE, "chess_set2_gray.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
