"""Writes tests/golden/middlebury_bgr.npz: the reference's bundled Art pair (Images/Art/view1.png,
view5.png, 463x370) as BGR uint8 arrays (cv::imread's channel order), the input of the segment-tree
parity test (STMatching takes colour frames: StereoDisparity.cpp:63).  Data only; run here, where
/root/reference exists:  python tests/golden/make_st_fixture.py"""
import os

import numpy as np
from PIL import Image

REF = "/root/reference/Images"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "middlebury_bgr.npz")


def bgr(path):
    return np.ascontiguousarray(np.asarray(Image.open(path).convert("RGB"))[:, :, ::-1])


if __name__ == "__main__":
    np.savez_compressed(OUT, **{"Art/view1": bgr(os.path.join(REF, "Art", "view1.png")),
                                "Art/view5": bgr(os.path.join(REF, "Art", "view5.png"))})
    print("wrote", OUT)
