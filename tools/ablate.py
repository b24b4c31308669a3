"""Time one libsm_hip.so build (path as argv[1]) on the 1080p D=128 workload; env SM_AB_R / SM_AB_D /
SM_AB_B / SM_AB_LR / SM_AB_AGG / SM_AB_W / SM_AB_H select radius, disparities, frames per call, LR and aggregation."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import gpu_stereo_matching_amd._capi as C
C.load(sys.argv[1])
import gpu_stereo_matching_amd as sm
AW, AH = int(os.environ.get('SM_AB_W', '1920')), int(os.environ.get('SM_AB_H', '1080'))
m = sm.BlockMatcher(0, AW, AH, 256)
NB = int(os.environ.get('SM_AB_B', '4'))
pairs = [sm.synth_pair(1234 + i, AW, AH, 128) for i in range(NB)]
Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda(); Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
out = torch.empty_like(Lt)
LR = bool(int(os.environ.get('SM_AB_LR', '0')))
RAD = int(os.environ.get('SM_AB_R', '5'))
AGG = os.environ.get('SM_AB_AGG', 'box')
NIT = 40 if AGG == 'box' else 5
DD = int(os.environ.get('SM_AB_D', '128'))
for _ in range(2 if AGG != 'box' else 5): m.match_device(Lt, Rt, RAD, DD, out_t=out, lr_check=LR, agg=AGG)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(NIT): m.match_device(Lt, Rt, RAD, DD, out_t=out, lr_check=LR, agg=AGG)
e1.record(); torch.cuda.synchronize()
print(sys.argv[1], "ms/frame", e0.elapsed_time(e1) / NIT / NB)
