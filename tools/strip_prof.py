"""Per-phase shader-clock cycles of one strip-kernel wave (a build with -DSM_STRIP_PROF, timing only: the counters
overwrite the first 40 map bytes of frame 0).  usage: python tools/strip_prof.py lib.so [radius]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import gpu_stereo_matching_amd._capi as C
C.load(sys.argv[1])
import gpu_stereo_matching_amd as sm
R = int(sys.argv[2]) if len(sys.argv) > 2 else 20
m = sm.BlockMatcher(0, 1920, 1080, 256)
pairs = [sm.synth_pair(1234 + i, 1920, 1080, 128) for i in range(8)]
Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda(); Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
out = torch.empty_like(Lt)
for _ in range(3):
    m.match_device(Lt, Rt, R, 128, out_t=out)
torch.cuda.synchronize()
c = out[0].flatten()[:40].cpu().numpy().view(np.uint64)
names = ["stage", "update", "row_wta", "emit", "barrier"]
tot = int(c.sum())
print("cycles per wave over all steps:", {n: int(v) for n, v in zip(names, c)}, "total", tot)
print("fractions:", {n: round(int(v) / max(tot, 1), 3) for n, v in zip(names, c)})
