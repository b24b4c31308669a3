"""Quick GPU bring-up: parity vs golden fixtures + oracle, and a rough timing."""
import os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpu_stereo_matching_amd as sm
from oracle import oracle as O

G = np.load("tests/golden/middlebury_gray.npz")
E = np.load("tests/golden/bm_expected.npz")
m = sm.BlockMatcher(0, 1920, 1080, 256)
bad = 0
for k in E.files:
    if k.startswith("lr/"):
        continue
    p, r, D = k.split("/")
    r, D = int(r[1:]), int(D[1:])
    got = m.match(G[f"{p}/view1"], G[f"{p}/view5"], r, D)
    n = int((got != E[k]).sum())
    bad += n
    print(f"{k:28s} mismatches {n}", flush=True)
    if n:
        idx = np.argwhere(got != E[k])[:5]
        for (y, x) in idx:
            print("   ", y, x, got[y, x], E[k][y, x])
S = np.load("tests/golden/synth_expected.npz")
for name in sorted({f.split('/')[0] for f in S.files}):
    seed, W, H, r, D = S[f"{name}/meta"]
    got = m.match(S[f"{name}/L"], S[f"{name}/R"], int(r), int(D))
    n = int((got != S[f"{name}/disp"]).sum()); bad += n
    print(f"{name:28s} mismatches {n}", flush=True)
for k in [k for k in E.files if k.startswith("lr/") and k.endswith("/checked")]:
    _, p, r, D, _ = k.split("/")
    r, D = int(r[1:]), int(D[1:])
    out, rd, mask = m.match_lr(G[f"{p}/view1"], G[f"{p}/view5"], r, D)
    n1 = int((rd != E[k.replace("checked", "right")]).sum())
    n2 = int((out != E[k]).sum()); n3 = int((mask != E[k.replace("checked", "mask")]).sum())
    bad += n1 + n2 + n3
    print(f"{k:28s} right {n1} checked {n2} mask {n3}", flush=True)

import torch
L, R = sm.synth_pair(1234, 1920, 1080, 128)
t0 = time.time(); ref = O.box_disp(L, R, 5, 128); print("oracle 1080p", time.time() - t0, flush=True)
Lt = torch.from_numpy(L).cuda(); Rt = torch.from_numpy(R).cuda()
out = m.match_device(Lt, Rt, 5, 128); torch.cuda.synchronize()
n = int((out.cpu().numpy() != ref).sum()); bad += n
print("1080p D128 r5 mismatches", n, flush=True)
for _ in range(5): m.match_device(Lt, Rt, 5, 128, out_t=out)
torch.cuda.synchronize()
e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50): m.match_device(Lt, Rt, 5, 128, out_t=out)
e1.record(); torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 50
print(f"1080p D=128 r=5: {ms:.3f} ms/frame  {1000/ms:.1f} maps/s", flush=True)
print("TOTAL_BAD", bad)
