"""Seeded synthetic rectified pairs, the bench and parity-test workload.

SplitMix64(seed) texture T of H x (W + 2D);  L[y][x] = T[y][x + D],
R[y][x] = T[y][x + D + gt(y)] so that R[y][x - gt] = L[y][x], with eight horizontal bands
gt(y) = 8 + floor(8y/H) * floor((D - 16) / 7) (clamped to [0, D-1]).
Byte-identical to oracle/bm_oracle.c:ora_synth_pair (checked in tests).
"""
from __future__ import annotations

import numpy as np

_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _splitmix64_at(seed: int, idx: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx.astype(np.uint64) + np.uint64(1)) * _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def ground_truth_rows(H: int, D: int) -> np.ndarray:
    step = max((D - 16) // 7, 0)
    y = np.arange(H)
    return np.clip(8 + (8 * y // H) * step, 0, D - 1)


def synth_pair(seed: int, W: int, H: int, D: int):
    """Return (L, R) uint8 [H, W] for the given seed."""
    TW = W + 2 * D
    gt = ground_truth_rows(H, D)
    y = np.arange(H, dtype=np.int64)[:, None]
    x = np.arange(W, dtype=np.int64)[None, :]
    iL = y * TW + (x + D)
    iR = y * TW + (x + D + gt[:, None])
    L = (_splitmix64_at(seed, iL) >> np.uint64(56)).astype(np.uint8)
    R = (_splitmix64_at(seed, iR) >> np.uint64(56)).astype(np.uint8)
    return L, R
