"""Steady-state PCIe-inclusive throughput of pipeline.FrameStream (1080p D=128 r=5) vs slots and
batch size; every slot is filled once before timing so no first-touch cost is measured."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import gpu_stereo_matching_amd as sm
from gpu_stereo_matching_amd.pipeline import FrameStream

W, H, D, r = 1920, 1080, 128, 5
m = sm.BlockMatcher(0, W, H, 256)
L, R = sm.synth_pair(1234, W, H, D)
for B in (4, 8, 16):
    for slots in (2, 3, 4):
        fs = FrameStream(m, B, W, H, r, D, consume=lambda d: None, slots=slots)
        for k in range(slots):
            lv, rv = fs.next_inputs()
            lv[...] = L
            rv[...] = R
            fs.submit()
        fs.flush()
        nb = max(8, 96 // B)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(nb):
            fs.next_inputs()
            fs.submit()
        fs.flush()
        ms = (time.perf_counter() - t0) * 1000 / (nb * B)
        print(f"batch {B:2d} slots {slots}: {ms:.4f} ms/frame  {1000 / ms:8.1f} maps/s")
