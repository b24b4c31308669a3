"""GPU median post-filter vs the ctmf restatement (oracle ora_median_u8).

The reference applies MeanFilter(disp, disp, 3) = ctmf(r=3) to its WTA maps
(STMatching/StereoDisparity.cpp:85,119,126,156; Toolkit.cpp:33-48).  Integer, bit-exact.
Parity unpinned w.r.t. ctmf itself: the oracle restates ctmf.c's algorithm.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available()
    return t


@pytest.fixture(scope="module")
def matcher():
    import gpu_stereo_matching_amd as sm
    m = sm.BlockMatcher(0, 2048, 1200, 256)
    yield m
    m.close()


@pytest.mark.parametrize("r", [1, 2, 3])
@pytest.mark.parametrize("W,H", [(1, 1), (5, 3), (64, 32), (65, 33), (333, 77), (1920, 1080)])
def test_median_device(matcher, oracle, torch, r, W, H):
    rng = np.random.default_rng(W * 7 + H + r)
    # disparity-like content: few levels with speckle, plus full-range noise rows
    src = (rng.integers(0, 8, (H, W)) * 9).astype(np.uint8)
    src[::7] = rng.integers(0, 256, src[::7].shape, dtype=np.uint8)
    got = matcher.median_device(torch.from_numpy(src).cuda(), r)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), oracle.median(src, r)), (r, W, H)


def test_median_flag_box(matcher, oracle, gray):
    L, R = gray["Art/view1"], gray["Art/view5"]
    got = matcher.match(L, R, 4, 64, median=True)
    want = oracle.median(oracle.box_disp(L, R, 4, 64), 3)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("r,D", [(5, 64), (3, 48), (8, 32), (16, 24)])
def test_median_then_lr(matcher, oracle, r, D):
    """Both WTA maps median-filtered before the LR check (StereoDisparity.cpp:119-147);
    r = 8 runs the fused right view's u32 window halves, r = 16 the mirrored right view."""
    L, R = oracle.synth_pair(r + D, 301, 97, max(D, 16))
    disp, cost = oracle.box_disp(L, R, r, D, want_cost=True)
    left_m = oracle.median(disp, 3)
    right_m = oracle.median(oracle.right_wta(cost), 3)
    checked, mask = oracle.lr_check(left_m, right_m)
    c, rr, mm = matcher.match_lr(L, R, r, D, median=True)
    assert np.array_equal(rr, right_m) and np.array_equal(c, checked) and np.array_equal(mm, mask)


def test_median_device_batch(matcher, oracle, torch):
    B, W, H, D, r = 3, 250, 64, 64, 5
    pairs = [oracle.synth_pair(40 + b, W, H, D) for b in range(B)]
    Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    out = matcher.match_device(Lt, Rt, r, D, median=True)
    torch.cuda.synchronize()
    for b in range(B):
        assert np.array_equal(out[b].cpu().numpy(), oracle.median(oracle.box_disp(pairs[b][0], pairs[b][1], r, D), 3))


def test_median_guided_lr_properties(matcher, gray):
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    left_m = matcher.match(L, R, 5, 64, agg="guided", median=True)
    chk, rd, mask = matcher.match_lr(L, R, 5, 64, agg="guided", median=True)
    assert ((chk == 0) | (chk == left_m)).all()
    assert (chk[mask == 1] == left_m[mask == 1]).all()


def test_median_bad_radius(sm_mod, matcher, torch):
    x = torch.zeros((8, 8), dtype=torch.uint8, device="cuda")
    with pytest.raises(sm_mod.SMError):
        matcher.median_device(x, 4)


@pytest.fixture(scope="module")
def sm_mod():
    import gpu_stereo_matching_amd as sm
    return sm
