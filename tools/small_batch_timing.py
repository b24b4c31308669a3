import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import gpu_stereo_matching_amd as sm
g = np.load("tests/golden/middlebury_gray.npz")
m = sm.BlockMatcher(0, 1920, 1080, 256)
for B in (16, 64, 128, 256):
    sc = ("Art", "Books", "Dolls")
    Lt = torch.from_numpy(np.stack([g[f"{sc[i%3]}/view1"] for i in range(B)])).cuda()
    Rt = torch.from_numpy(np.stack([g[f"{sc[i%3]}/view5"] for i in range(B)])).cuda()
    o = torch.empty_like(Lt)
    for r in (3, 4):
        for _ in range(3): m.match_device(Lt, Rt, r, 64, out_t=o)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20): m.match_device(Lt, Rt, r, 64, out_t=o)
        e1.record(); torch.cuda.synchronize()
        print(B, r, round(e0.elapsed_time(e1) / 20 / B * 1000, 2), "us/frame")
