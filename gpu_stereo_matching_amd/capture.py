"""The reference's capture loop, replayed from files.

`photo()` (Utility.cpp:198-226) grabs left/right frames from two cameras, shows them, and saves the
pairs it is told to keep as ``Left_<n>.jpg`` / ``Right_<n>.jpg`` (Utility.cpp:217-218); ``singleFrame``
(Caller.cpp:9-25) turns one pair into a disparity map and shows it (imshow, Caller.cpp:23-24).  A GPU
box has no camera and no display, so this module keeps the loop and replaces its two ends:

- `PairSequence` replays numbered pairs from a directory (the files photo() writes, or any
  ``<left_prefix><n><ext>`` / ``<right_prefix><n><ext>`` set), in numeric order, as BGR frames
  (cv::imread's channel order), decoded with PIL;
- `run_loop` pushes them through `pipeline.FrameStream`, in batches: BGR -> gray (Caller.cpp:15-16),
  optionally the calibration's rectification (Rectify + remap, Caller.cpp:27-74, Utility.cpp:228-234),
  then block matching (Caller.cpp:19), every step on the GPU.  Each map goes to ``on_map(n, disp)``
  (the imshow slot) and, with ``out_dir``, to ``disp_<n>.png`` (imwrite).

    python -m gpu_stereo_matching_amd.capture PAIRS_DIR --calib Calib_Data_OpenCV.yml --out maps/

Frames are used at their stored size; ``size=(W, H)`` resizes them first with PIL's bilinear filter,
which is not OpenCV's ``resize`` (photo() only resizes for display; remapTest resizes to 320x200,
Caller.cpp:36-43), so resized inputs are not pinned to the reference.
"""
from __future__ import annotations

import argparse
import os
import re
from typing import Callable, Iterator, List, Optional, Tuple

import numpy as np

__all__ = ["PairSequence", "run_loop"]


def _read_bgr(path: str, size: Optional[Tuple[int, int]]) -> np.ndarray:
    from PIL import Image
    with Image.open(path) as im:
        im = im.convert("RGB")
        if size is not None and im.size != tuple(size):
            im = im.resize(tuple(size), Image.BILINEAR)
        rgb = np.asarray(im, dtype=np.uint8)
    return np.ascontiguousarray(rgb[:, :, ::-1])   # BGR, as cv::imread returns


class PairSequence:
    """Numbered stereo pairs in `directory`: ``<left_prefix><n><ext>`` with a matching right file.
    Iterating yields ``(n, left_bgr, right_bgr)`` in increasing n; pairs with a missing right file
    are skipped.  ``size=(W, H)`` resizes (PIL bilinear)."""

    def __init__(self, directory: str, left_prefix: str = "Left_", right_prefix: str = "Right_",
                 exts: Tuple[str, ...] = (".jpg", ".png", ".jpeg", ".bmp"), size: Optional[Tuple[int, int]] = None):
        self.directory = directory
        self.size = size
        pat = re.compile(re.escape(left_prefix) + r"(\d+)(" + "|".join(re.escape(e) for e in exts) + r")$",
                         re.IGNORECASE)
        pairs = []
        for name in os.listdir(directory):
            m = pat.match(name)
            if not m:
                continue
            right = os.path.join(directory, right_prefix + m.group(1) + m.group(2))
            if os.path.exists(right):
                pairs.append((int(m.group(1)), os.path.join(directory, name), right))
        self.pairs = sorted(pairs)

    def __len__(self) -> int:
        return len(self.pairs)

    def __iter__(self) -> Iterator[Tuple[int, np.ndarray, np.ndarray]]:
        for n, lp, rp in self.pairs:
            yield n, _read_bgr(lp, self.size), _read_bgr(rp, self.size)


def _write_png(path: str, disp: np.ndarray) -> None:
    from PIL import Image
    Image.fromarray(disp).save(path)


def run_loop(source, matcher, radius: int = 5, num_disp: int = 64, rectify_maps=None, batch: int = 4,
             agg: str = "box", on_map: Optional[Callable[[int, np.ndarray], None]] = None,
             out_dir: Optional[str] = None) -> List[int]:
    """Match every pair of `source` (an iterable of ``(n, left_bgr, right_bgr)``, e.g. a PairSequence),
    `batch` pairs per GPU launch through FrameStream (BGR -> gray -> [rectify] -> match on the GPU).
    Returns the pair numbers in the order their maps were delivered (the input order).  A short last
    batch is padded with its own last pair, whose extra maps are dropped."""
    from .pipeline import FrameStream

    if out_dir:
        os.makedirs(out_dir, exist_ok=True)
    fs = None
    queued: List[List[int]] = []      # pair numbers of each submitted batch, oldest first
    done: List[int] = []
    cur_n: List[int] = []
    cur_l: List[np.ndarray] = []
    cur_r: List[np.ndarray] = []

    def deliver(maps: np.ndarray) -> None:
        ns = queued.pop(0)
        for i, n in enumerate(ns):
            if on_map is not None:
                on_map(n, maps[i])
            if out_dir:
                _write_png(os.path.join(out_dir, f"disp_{n}.png"), maps[i])
            done.append(n)

    def submit(ns, ls, rs) -> None:
        nonlocal fs
        H, W = ls[0].shape[:2]
        if fs is None:
            fs = FrameStream(matcher, batch, W, H, radius, num_disp, agg=agg, bgr=True, rectify_maps=rectify_maps)
        elif (fs.H, fs.W) != (H, W):
            raise ValueError(f"pair {ns[0]}: frame size {W}x{H} differs from the stream's {fs.W}x{fs.H}")
        while len(ls) < batch:
            ls.append(ls[-1])
            rs.append(rs[-1])
        queued.append(list(ns))
        for maps in fs.submit(np.stack(ls), np.stack(rs)):
            deliver(maps)

    for n, left, right in source:
        if left.shape != right.shape or left.ndim != 3 or left.shape[2] != 3:
            raise ValueError(f"pair {n}: expected two BGR frames of one size")
        cur_n.append(n)
        cur_l.append(left)
        cur_r.append(right)
        if len(cur_n) == batch:
            submit(cur_n, cur_l, cur_r)
            cur_n, cur_l, cur_r = [], [], []
    if cur_n:
        submit(cur_n, cur_l, cur_r)
    if fs is not None:
        for maps in fs.flush():
            deliver(maps)
    return done


def _main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Replay saved stereo pairs (photo()'s Left_<n>/Right_<n> files) "
                                             "through the GPU capture chain and write disparity maps.")
    ap.add_argument("pairs", help="directory of Left_<n>.* / Right_<n>.* files")
    ap.add_argument("--calib", help="OpenCV FileStorage YAML (Calib_Data_OpenCV.yml): rectify first")
    ap.add_argument("--size", help="WxH: resize the frames first (PIL bilinear)")
    ap.add_argument("--radius", type=int, default=5, help="SADWindowSize (the window radius, Caller.cpp:19)")
    ap.add_argument("--disp", type=int, default=64, help="searchRange (number of disparities, Caller.cpp:19)")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--agg", default="box", choices=["box", "guided"])
    ap.add_argument("--out", help="directory for disp_<n>.png")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)
    from . import BlockMatcher, calib

    size = tuple(int(v) for v in a.size.lower().split("x")) if a.size else None
    seq = PairSequence(a.pairs, size=size)
    if not len(seq):
        print(f"no Left_<n>/Right_<n> pairs in {a.pairs}")
        return 1
    first = next(iter(seq))
    H, W = first[1].shape[:2]
    with BlockMatcher(a.device, W, H, max(a.disp, 1)) as m:
        maps = calib.rectify(m, *calib.load_data_batch(a.calib), (W, H)) if a.calib else None
        done = run_loop(seq, m, a.radius, a.disp, rectify_maps=maps, batch=a.batch, agg=a.agg, out_dir=a.out,
                        on_map=lambda n, d: print(f"pair {n}: {W}x{H}, {int((d > 0).sum())} matched pixels"))
    print(f"{len(done)} pairs matched")
    return 0


if __name__ == "__main__":
    raise SystemExit(_main())
