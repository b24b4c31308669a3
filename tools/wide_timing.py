"""Box matching time per 1080p D=128 frame at wide radii (HIP events, device-resident frames):
    python tools/wide_timing.py LIB.so R1,R2,... [--batch B] [--iters N] [--lr]
(run once per library build, e.g. before / after the wide-window path of bm_wide.hip)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import gpu_stereo_matching_amd._capi as C

C.load(sys.argv[1])
import gpu_stereo_matching_amd as sm  # noqa: E402

radii = [int(v) for v in sys.argv[2].split(",")]
B = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 4
N = int(sys.argv[sys.argv.index("--iters") + 1]) if "--iters" in sys.argv else 10
LR = "--lr" in sys.argv
m = sm.BlockMatcher(0, 1920, 1080, 256)
pairs = [sm.synth_pair(1234 + i, 1920, 1080, 128) for i in range(B)]
Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
out = torch.empty_like(Lt)
for r in radii:
    m.match_device(Lt, Rt, r, 128, out_t=out, lr_check=LR)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(N):
        m.match_device(Lt, Rt, r, 128, out_t=out, lr_check=LR)
    e1.record()
    torch.cuda.synchronize()
    print(f"{os.path.basename(sys.argv[1])} r={r} ({2*r+1}x{2*r+1}) lr={int(LR)} ms/frame {e0.elapsed_time(e1) / N / B:.4f}",
          flush=True)
