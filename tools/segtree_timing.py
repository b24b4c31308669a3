"""Segment-tree stereo (ST-1 and ST-2) on the bundled Middlebury pairs at the app's defaults: GPU path
(host trees + GPU cost / filter / WTA / median / LR check) wall time and its stats, beside the C oracle
(the restated reference algorithm, one core) on the same input."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
if os.environ.get("SM_LIB"):      # a variant build (tools/build_variant.sh) instead of the in-tree library
    import gpu_stereo_matching_amd._capi as C
    C.load(os.environ["SM_LIB"])
import gpu_stereo_matching_amd as sm
from oracle import oracle as O

g = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "middlebury_bgr.npz"))
scenes = sorted({k.split("/")[0] for k in g.files})
with sm.BlockMatcher(0, 640, 480, 256) as m:
    for sc in scenes:
        L, R = g[f"{sc}/view1"], g[f"{sc}/view5"]
        for method, name in ((0, "ST-1"), (1, "ST-2")):
            for _ in range(2):
                m.segment_tree(L, R, method=method)
            ts = []
            for _ in range(5):
                t0 = time.perf_counter(); d = m.segment_tree(L, R, method=method); ts.append(time.perf_counter() - t0)
            tree_ms, total_ms, lv = m.segment_tree_stats()
            t0 = time.perf_counter()
            want = O.st2_disp(L, R, 60, 4, 0.1)[0] if method else O.st_disp(L, R, 60, 4, 0.1)[0]
            t_o = time.perf_counter() - t0
            H, W = L.shape[:2]
            print(f"{os.path.basename(os.environ.get('SM_LIB', 'in-tree'))} {name} {sc} {W}x{H} D=60: GPU path {sorted(ts)[2]*1e3:.1f} ms/map (host trees {tree_ms:.1f} ms, "
                  f"levels {lv}); oracle (1 core) {t_o*1e3:.0f} ms; bit-exact {np.array_equal(d, want)}", flush=True)
