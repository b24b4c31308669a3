"""Seeded random stereo pairs for the GPU fuzz parity tests (test infrastructure)."""
import numpy as np


def fuzz_pair(rng, W, H):
    """Random texture with flat patches, saturated 0 / 255 runs and a shifted right view: exercises
    ties (flat regions: equal SADs over many d), the u16 packed sums at their extremes, and borders."""
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    kind = rng.integers(0, 4)
    if kind == 1:
        L[:, : W // 2] = rng.integers(0, 256)                      # flat half: many exact ties
    elif kind == 2:
        L = np.where(rng.random((H, W)) < 0.5, 0, 255).astype(np.uint8)   # saturated values only
    elif kind == 3:
        L = (L // 64 * 64).astype(np.uint8)                         # 4 levels: frequent ties
    s = int(rng.integers(0, 20))
    R = np.roll(L, -s, axis=1)
    noise = rng.integers(-3, 4, (H, W))
    R = np.clip(R.astype(np.int32) + noise * (rng.random((H, W)) < 0.3), 0, 255).astype(np.uint8)
    return np.ascontiguousarray(L), np.ascontiguousarray(R)
