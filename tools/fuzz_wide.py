"""Randomised parity sweep of the wide-window path (r 16..127) and the literal Device.cu mode against the
oracle: N cases of random size, radius, d range, batch and LR, each map compared bit for bit.
    python tools/fuzz_wide.py [N] [seed]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import gpu_stereo_matching_amd as sm
from oracle import oracle as O

N = int(sys.argv[1]) if len(sys.argv) > 1 else 40
rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 2026)
m = sm.BlockMatcher(0, 1100, 600, 256)
bad = 0
for i in range(N):
    W = int(rng.integers(4, 420))
    H = int(rng.integers(1, 140))
    r = int(rng.integers(16, 128))
    D = int(rng.integers(1, 80))
    B = int(rng.integers(1, 4))
    lr = bool(rng.integers(0, 2))
    kind = rng.integers(0, 3)
    pairs = []
    for b in range(B):
        if kind == 0:
            L = rng.integers(0, 256, (H, W), dtype=np.uint8)
            R = rng.integers(0, 256, (H, W), dtype=np.uint8)
        elif kind == 1:
            L = (rng.integers(0, 2, (H, W)) * 255).astype(np.uint8)
            R = np.roll(L, int(rng.integers(0, 8)), axis=1)
        else:
            L, R = O.synth_pair(int(rng.integers(0, 1 << 30)), W, H, max(D, 16))
        pairs.append((L, R))
    Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    out = m.match_device(Lt, Rt, r, D, lr_check=lr)
    torch.cuda.synchronize()
    for b, (L, R) in enumerate(pairs):
        want = O.box_lr(L, R, r, D)[2] if lr else O.box_disp(L, R, r, D)
        ok = np.array_equal(out[b].cpu().numpy(), want)
        if not ok:
            bad += 1
            print(f"MISMATCH case {i} frame {b}: W={W} H={H} r={r} D={D} B={B} lr={lr} kind={kind} "
                  f"px={int((out[b].cpu().numpy() != want).sum())}", flush=True)
    if i % 10 == 0:
        print(f"case {i}: W={W} H={H} r={r} D={D} B={B} lr={lr} ok", flush=True)
# literal mode at random sizes >= 320 x 256
for i in range(max(4, N // 8)):
    W = int(rng.integers(320, 1100))
    H = int(rng.integers(256, 600))
    r = int(rng.integers(0, 128))
    D = int(rng.integers(1, 200))
    L, R = O.synth_pair(int(rng.integers(0, 1 << 30)), W, H, max(D, 16))
    got = m.match(L, R, r, D, agg="device-cu")
    want = O.device_cu_literal_integral(L, R, r, D)
    if not np.array_equal(got, want):
        bad += 1
        print(f"LITERAL MISMATCH W={W} H={H} r={r} D={D} px={int((got != want).sum())}", flush=True)
print(f"fuzz done: {N} wide cases + literal cases, {bad} mismatching frames", flush=True)
sys.exit(1 if bad else 0)
