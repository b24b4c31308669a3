"""Round 4: segment-tree wall time with the BFS on the device (default) against the host BFS
(SM_ST_HOST_BFS=1, read per call), alternated in one process on the bundled Middlebury pairs at the app's
defaults; maps compared between the two."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import gpu_stereo_matching_amd as sm

g = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                         "middlebury_bgr.npz"))
scenes = sorted({k.split("/")[0] for k in g.files})
with sm.BlockMatcher(0, 640, 480, 256) as m:
    for sc in scenes:
        L, R = g[f"{sc}/view1"], g[f"{sc}/view5"]
        H, W = L.shape[:2]
        for method, name in ((0, "ST-1"), (1, "ST-2")):
            maps = {}
            for rnd in range(3):
                for mode in ("host", "device"):
                    if mode == "host":
                        os.environ["SM_ST_HOST_BFS"] = "1"
                    else:
                        os.environ.pop("SM_ST_HOST_BFS", None)
                    for _ in range(2):
                        m.segment_tree(L, R, method=method)
                    ts = []
                    for _ in range(9):
                        t0 = time.perf_counter()
                        maps[mode] = m.segment_tree(L, R, method=method)
                        ts.append(time.perf_counter() - t0)
                    tree_ms, total_ms, lv = m.segment_tree_stats()
                    print(f"{name} {sc} {W}x{H} round {rnd} {mode:6s} BFS: {np.median(ts) * 1e3:.3f} ms/map "
                          f"(min {min(ts) * 1e3:.3f}; tree {tree_ms:.3f} ms, levels {lv})", flush=True)
            os.environ.pop("SM_ST_HOST_BFS", None)
            print(f"{name} {sc}: maps identical {np.array_equal(maps['host'], maps['device'])}", flush=True)
