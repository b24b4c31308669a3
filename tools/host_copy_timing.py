import sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np
import gpu_stereo_matching_amd as sm
m = sm.BlockMatcher(0, 1920, 1080, 256)
m.set_stage_timing(True)   # the default (auto) records the split only once stage_ms() has been read
for (W, H, D, r) in ((463, 370, 64, 4), (464, 370, 64, 4), (1920, 1080, 128, 5)):
    L, R = sm.synth_pair(1, W, H, D)
    for _ in range(3): m.match(L, R, r, D)
    t0 = time.perf_counter()
    for _ in range(20): m.match(L, R, r, D)
    print(W, H, "ms", round((time.perf_counter() - t0) * 50, 4), "stages", [round(v, 4) for v in m.stage_ms()])
# pitched input (ROI of a wider buffer)
big = np.zeros((370, 600), np.uint8); L, R = sm.synth_pair(1, 463, 370, 64)
bl = big.copy(); bl[:, :463] = L; br = big.copy(); br[:, :463] = R
import ctypes
out = np.empty((370, 463), np.uint8)
lib = m._lib
t0 = time.perf_counter()
for _ in range(20):
    lib.sm_block_match_u8(m._h, bl.ctypes.data, br.ctypes.data, 463, 370, 600, 4, 64, 0, out.ctypes.data, 463)
print("pitched ms", round((time.perf_counter() - t0) * 50, 4), [round(v, 4) for v in m.stage_ms()])
