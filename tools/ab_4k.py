"""A/B of libsm_hip.so builds on the 4K D=192 r=5 box workload (plain and LR), batch 8; one process per lib."""
import os, subprocess, sys
code = r'''
import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import gpu_stereo_matching_amd._capi as C
C.load(sys.argv[1])
import gpu_stereo_matching_amd as sm
m = sm.BlockMatcher(0, 3840, 2160, 256)
B = 8
pairs = [sm.synth_pair(4321 + i, 3840, 2160, 192) for i in range(B)]
Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda(); Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
o = torch.empty_like(Lt)
res = []
for lr in (False, True):
    for _ in range(2): m.match_device(Lt, Rt, 5, 192, out_t=o, lr_check=lr)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): m.match_device(Lt, Rt, 5, 192, out_t=o, lr_check=lr)
    e1.record(); torch.cuda.synchronize()
    res.append(round(e0.elapsed_time(e1) / 10 / B, 4))
print(os.path.basename(sys.argv[1]), "4K D192 ms/frame plain", res[0], "lr", res[1])
'''
for r in range(2):
    for lib in sys.argv[1:]:
        out = subprocess.run([sys.executable, "-c", code, lib], capture_output=True, text=True, timeout=200)
        print(out.stdout.strip() or out.stderr[-500:])
