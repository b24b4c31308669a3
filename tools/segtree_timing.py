"""Segment-tree stereo (ST-1) on the bundled Art pair at the app's defaults: GPU path (host tree + GPU
cost / filter / WTA / median) wall time and its stats, beside the C oracle (the restated reference
algorithm, one core) on the same input."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import gpu_stereo_matching_amd as sm
from oracle import oracle as O

g = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "middlebury_bgr.npz"))
L, R = g["Art/view1"], g["Art/view5"]
with sm.BlockMatcher(0, 640, 480, 256) as m:
    for _ in range(2):
        m.segment_tree(L, R)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter(); d = m.segment_tree(L, R); ts.append(time.perf_counter() - t0)
    tree_ms, total_ms, lv = m.segment_tree_stats()
t0 = time.perf_counter(); want, lv_o = O.st_disp(L, R, 60, 4, 0.1); t_o = time.perf_counter() - t0
print(f"ST-1 Art 463x370 D=60: GPU path {sorted(ts)[2]*1e3:.1f} ms/map (host tree {tree_ms:.1f} ms, levels {lv}); "
      f"oracle (1 core) {t_o*1e3:.0f} ms; bit-exact {np.array_equal(d, want)}")
