"""Tie-aware acceptance rule for the float guided path (used by the guided GPU tests).

Tolerance (absolute, in AD units 0..255): a pixel passes when the GPU disparity equals the fp64
oracle's, or when the oracle cost of the GPU's choice is within TOL of the oracle's best (a
near-tie), or when the oracle best is within TOL of the 50.0 threshold and the GPU reports no
match.
"""
import numpy as np

TOL = 2e-3


def tie_aware_check(gpu, q, best, D, W):
    H = gpu.shape[0]
    xs = np.arange(W)[None, :].repeat(H, 0)
    ys = np.arange(H)[:, None].repeat(W, 1)
    d_g = gpu.astype(np.int64)
    q_g = q[np.clip(d_g, 0, D - 1), ys, xs]
    ok_exact = d_g == best["disp"]
    valid = d_g <= (W - xs)
    near_tie = valid & (q_g <= best["best"] + TOL) & (q_g < 50.0 + TOL)
    no_match = (d_g == 0) & (best["best"] >= 50.0 - TOL)
    ok = ok_exact | near_tie | no_match
    return ok, ok_exact
