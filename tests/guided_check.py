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


def guided_reference(oracle, L, R, r, D, eps):
    """The fp64 oracle's volume and both views' WTA for the tie-aware rules: a dict with the left map
    ("disp"), best left cost ("best"), the q volume ("q"), the right map ("rdisp"), the right cost volume
    C_R ("cr", StereoHelper.cpp:156-180) and its best ("best_r")."""
    disp_o, q, best = oracle.guided_disp(L, R, r, D, eps, want_q=True)
    rd_o, cr, best_r = oracle.right_wta_float(q)
    return {"disp": disp_o, "best": best, "q": q, "rdisp": rd_o, "cr": cr, "best_r": best_r}


def acceptable_left(ref, D, W):
    """acc[d, y, x]: left disparity d at (y, x) passes tie_aware_check's rule."""
    q = ref["q"][:D]
    H = q.shape[1]
    ds = np.arange(D)[:, None, None]
    xs = np.arange(W)[None, None, :]
    acc = (ds == ref["disp"][None]) | ((ds <= W - xs) & (q <= ref["best"][None] + TOL) & (q < 50.0 + TOL))
    acc[0] |= ref["best"] >= 50.0 - TOL
    assert acc.shape == (D, H, W)
    return acc


def acceptable_right(ref, D):
    """acc[d, y, u]: right disparity d at (y, u) is the oracle's or within TOL of its best C_R."""
    cr = ref["cr"][:D]
    ds = np.arange(D)[:, None, None]
    return (ds == ref["rdisp"][None]) | (cr <= ref["best_r"][None] + TOL)


def tie_aware_lr_check(chk, ref, D, W):
    """A checked map (StereoDisparity.cpp:136-147: d kept where x - d >= 0, d != 0 and |d - dR(x - d)| <= 1,
    else 0) is accepted pixel by pixel when SOME left disparity passing the tie-aware rule and SOME right
    disparity at x - d passing the right view's rule produce it.  Exact pixels (both views equal to the
    oracle's) therefore pass only with the oracle's own checked value.  Returns the per-pixel ok map."""
    accL = acceptable_left(ref, D, W)
    accR = acceptable_right(ref, D)
    H = chk.shape[0]
    cntR = accR.sum(axis=0, dtype=np.int32)
    keep_ok = np.zeros((D, H, W), bool)   # value d reachable as "kept"
    zero_ok = np.zeros((H, W), bool)      # value 0 reachable
    for d in range(D):
        cand = accL[d]
        if d == 0:
            zero_ok |= cand
            continue
        zero_ok[:, :d] |= cand[:, :d]                       # x - d < 0: occluded
        if d >= W:
            continue
        # right pixel u = x - d: some acceptable dR within 1 of d ("near") or farther ("far")
        n_near = sum(accR[k][:, :W - d].astype(np.int32) for k in (d - 1, d, d + 1) if 0 <= k < D)
        near = n_near > 0
        far = (cntR[:, :W - d] - n_near) > 0
        keep_ok[d][:, d:] = cand[:, d:] & near
        zero_ok[:, d:] |= cand[:, d:] & far
    c = chk.astype(np.int64)
    ys, xs = np.mgrid[0:H, 0:W]
    ok_keep = (c > 0) & (c < D) & keep_ok[np.clip(c, 0, D - 1), ys, xs]
    return np.where(c == 0, zero_ok, ok_keep)
