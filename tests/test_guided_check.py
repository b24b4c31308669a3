"""CPU tests of the tie-aware acceptance rules the guided GPU tests apply (tests/guided_check.py).

The checked-map rule (tie_aware_lr_check) must accept the oracle's own LR-checked map, the checked map
of any left / right pair that each pass the per-view rules, and nothing else: a pixel whose value no
acceptable pair of disparities produces is rejected."""
import numpy as np

from guided_check import TOL, acceptable_left, guided_reference, tie_aware_check, tie_aware_lr_check

EPS = 1e-4 * 255 * 255


def _ref(oracle, seed=3, W=90, H=40, r=3, D=24):
    L, R = oracle.synth_pair(seed, W, H, max(D, 16))
    return L, R, guided_reference(oracle, L, R, r, D, EPS), D, W


def test_oracle_checked_map_is_accepted(oracle, gray):
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    ref = guided_reference(oracle, L, R, 5, 64, EPS)
    chk = oracle.lr_check(ref["disp"], ref["rdisp"])[0]
    assert tie_aware_lr_check(chk, ref, 64, L.shape[1]).all()


def test_wrong_values_are_rejected(oracle):
    _, _, ref, D, W = _ref(oracle)
    chk = oracle.lr_check(ref["disp"], ref["rdisp"])[0]
    rng = np.random.default_rng(0)
    bad = chk.copy()
    ys, xs = np.nonzero(chk > 2)
    pick = rng.choice(len(ys), size=min(40, len(ys)), replace=False)
    # a value 2 below the kept one: the left view would have to take it, and no near-tie allows that here
    bad[ys[pick], xs[pick]] -= 2
    accL = acceptable_left(ref, D, W)
    justified = accL[bad[ys[pick], xs[pick]].astype(np.int64), ys[pick], xs[pick]]
    ok = tie_aware_lr_check(bad, ref, D, W)
    assert (~justified).sum() > 0
    assert (~ok[ys[pick], xs[pick]])[~justified].all()


def test_near_tie_left_pair_is_accepted(oracle):
    """Swap a left disparity for another within TOL of the best (a near-tie the GPU may pick): the LR rule
    applied to the swapped map is accepted, and tie_aware_check accepts the swapped left map."""
    _, _, ref, D, W = _ref(oracle, seed=8)
    q = ref["q"]
    H = q.shape[1]
    left = ref["disp"].copy()
    for y in range(H):
        for x in range(W):
            for d in range(min(D, W - x + 1)):
                if d != left[y, x] and q[d, y, x] <= ref["best"][y, x] + TOL and q[d, y, x] < 50.0:
                    left[y, x] = d
                    break
    ok_l, _ = tie_aware_check(left, q, {"disp": ref["disp"], "best": ref["best"]}, D, W)
    assert ok_l.all()
    chk = oracle.lr_check(left, ref["rdisp"])[0]
    assert tie_aware_lr_check(chk, ref, D, W).all()
