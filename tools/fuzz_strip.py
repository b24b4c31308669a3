"""Randomised parity sweep of the strip kernel (csrc/bm_strip.hip, box r 16..37, LR in every other case) and its neighbours
(r 38..40 on the separable path) against the oracle: N cases of random size, radius, d range, batch, texture and
d-slice, every map / key array compared bit for bit.
    python tools/fuzz_strip.py [N] [seed]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import gpu_stereo_matching_amd as sm
from oracle import oracle as O

N = int(sys.argv[1]) if len(sys.argv) > 1 else 100
rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 2027)
m = sm.BlockMatcher(0, 1100, 320, 256)
bad = 0
for i in range(N):
    W = int(rng.integers(4, 1100))
    H = int(rng.integers(1, 320))
    r = int(rng.integers(16, 41))
    D = int(rng.integers(1, 257))
    B = int(rng.integers(1, 4))
    kind = int(rng.integers(0, 3))
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
    lr = bool(i % 2)
    out = m.match_device(Lt, Rt, r, D, lr_check=lr)
    torch.cuda.synchronize()
    if lr:
        ok = all(np.array_equal(out[b].cpu().numpy(), O.box_lr(L, R, r, D)[2]) for b, (L, R) in enumerate(pairs))
    else:
        ok = all(np.array_equal(out[b].cpu().numpy(), O.box_disp(L, R, r, D)) for b, (L, R) in enumerate(pairs))
    # one d-slice of the first frame
    a = int(rng.integers(0, D))
    e = int(rng.integers(a + 1, D + 1))
    k = m.slice_keys_device(Lt[0], Rt[0], r, a, e)
    torch.cuda.synchronize()
    ok_k = np.array_equal(k.cpu().numpy().view(np.uint32), O.box_keys_slice(pairs[0][0], pairs[0][1], r, a, e))
    if not (ok and ok_k):
        bad += 1
        print(f"MISMATCH case {i}: W={W} H={H} r={r} D={D} B={B} lr={lr} kind={kind} slice=[{a},{e}) maps={ok} keys={ok_k}",
              flush=True)
    if (i + 1) % 20 == 0:
        print(f"{i + 1} cases, {bad} mismatching", flush=True)
print(f"fuzz_strip: {N} cases, {bad} mismatching")
sys.exit(1 if bad else 0)
