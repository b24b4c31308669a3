"""Minimal driver for profiling: launch the 1080p box kernel K times on synthetic frames."""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import gpu_stereo_matching_amd as sm

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--batch", type=int, default=4)
ap.add_argument("--W", type=int, default=1920)
ap.add_argument("--H", type=int, default=1080)
ap.add_argument("--D", type=int, default=128)
ap.add_argument("--r", type=int, default=5)
ap.add_argument("--agg", default="box")
ap.add_argument("--lr", action="store_true")
ap.add_argument("--lib", default=None, help="libsm_hip.so build to load (A/B profiling)")
a = ap.parse_args()
if a.lib:
    import gpu_stereo_matching_amd._capi as C
    C.load(a.lib)
m = sm.BlockMatcher(0, a.W, a.H, 256)
pairs = [sm.synth_pair(1234 + i, a.W, a.H, a.D) for i in range(a.batch)]
Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
out = torch.empty_like(Lt)
for _ in range(a.iters):
    m.match_device(Lt, Rt, a.r, a.D, out_t=out, agg=a.agg, lr_check=a.lr)
torch.cuda.synchronize()
print("done")
