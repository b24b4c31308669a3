"""GPU parity for SM_DEVICE_CU_GRID (Device.cu's literal output, launch geometry included) and for the
wide windows (radius 16-127) of the generic box path.

The literal map: kernalPreCal_V2's fixed grid (8, 10, D) x (32, 32) (Device.cu:231-233) leaves the AD
volume at its memset 0 outside rows < 256, cols < 320 (:193-194), and kernalFindCorr's <<<rows, cols>>>
(:253) does not launch for cols > 1024, leaving the map at 0 (:191-192).  Expected maps come from
oracle.device_cu_literal (the loop nest over that grid, bm_oracle.c), cross-checked at generation time
against a numpy integral-image formulation (tests/golden/make_golden.py --device-cu).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def sm():
    import gpu_stereo_matching_amd as sm
    return sm


@pytest.fixture(scope="module")
def matcher(sm):
    m = sm.BlockMatcher(0, 2048, 1100, 256)
    yield m
    m.close()


@pytest.fixture(scope="module")
def literal_expected():
    return np.load(os.path.join(GOLDEN, "device_cu_expected.npz"))


def test_literal_golden_every_bundled_pair(matcher, gray, literal_expected):
    """All 10 bundled pairs (9 of them 443-463 x 370, where ~50 % of the literal map differs from getDisp)."""
    for k in literal_expected.files:
        p, r, D = k.split("/")
        got = matcher.match(gray[f"{p}/view1"], gray[f"{p}/view5"], int(r[1:]), int(D[1:]), agg="device-cu")
        want = literal_expected[k]
        assert np.array_equal(got, want), f"{k}: {int((got != want).sum())} px differ"


def test_literal_differs_from_getdisp_where_the_reference_does(matcher, gray, bm_expected, literal_expected):
    """SURVEY §8a a1 measured 85,893 / 171,310 pixels of Art (r = 4, D = 64) where Device.cu's real map
    differs from getDisp; the default path stays getDisp, the literal mode reproduces Device.cu."""
    L, R = gray["Art/view1"], gray["Art/view5"]
    lit = matcher.match(L, R, 4, 64, agg="device-cu")
    dflt = matcher.match(L, R, 4, 64)
    assert np.array_equal(dflt, bm_expected["Art/r4/D64"])
    assert int((lit != dflt).sum()) == 85893


def test_literal_equals_default_at_320x256(matcher, gray, bm_expected):
    """At exactly 320 x 256 (singleFrame's Art view1_/view5_) the grid covers every (row, col, d)."""
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    for r, D in ((5, 64), (2, 256)):
        assert np.array_equal(matcher.match(L, R, r, D, agg="device-cu"), bm_expected[f"Art_/r{r}/D{D}"])


def test_literal_synthetic_sizes(matcher, oracle):
    """Odd sizes >= 320 x 256, wide and narrow radii, D up to 256 (d >= 320 - r planes are all zero)."""
    for (W, H, r, D, seed) in ((320, 256, 0, 1, 1), (333, 259, 3, 37, 2), (640, 480, 5, 128, 3),
                               (1024, 300, 17, 256, 4), (400, 700, 9, 64, 5), (512, 256, 31, 16, 6)):
        L, R = oracle.synth_pair(seed, W, H, max(D, 16))
        got = matcher.match(L, R, r, D, agg="device-cu")
        want = oracle.device_cu_literal_integral(L, R, r, D)
        assert np.array_equal(got, want), (W, H, r, D, int((got != want).sum()))


def test_literal_wide_frame_is_all_zero(matcher, oracle):
    """cols > 1024: the <<<rows, cols>>> launch fails, the map keeps the memset 0 (Device.cu:191-192, 253)."""
    L, R = oracle.synth_pair(7, 1025, 260, 64)
    got = matcher.match(L, R, 5, 64, agg="device-cu")
    assert not got.any()
    assert np.array_equal(got, oracle.device_cu_literal(L, R, 5, 64))
    assert matcher.match(L, R, 5, 64).any()   # the default path matches at any width


def test_literal_device_batch(sm, matcher, gray, literal_expected):
    import torch
    L = torch.from_numpy(np.stack([gray["Books/view1"], gray["Dolls/view1"]])).cuda()
    R = torch.from_numpy(np.stack([gray["Books/view5"], gray["Dolls/view5"]])).cuda()
    out = matcher.match_device(L, R, 4, 64, agg="device-cu")
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    assert np.array_equal(got[0], literal_expected["Books/r4/D64"])
    assert np.array_equal(got[1], literal_expected["Dolls/r4/D64"])


def test_literal_rejects_undefined_sizes_and_flags(sm, matcher, gray):
    rng = np.random.default_rng(3)
    small = rng.integers(0, 256, (255, 400), dtype=np.uint8)
    narrow = rng.integers(0, 256, (300, 319), dtype=np.uint8)
    for img in (small, narrow):
        with pytest.raises(sm.SMError):
            matcher.match(img, img, 3, 16, agg="device-cu")
    L, R = gray["Art/view1"], gray["Art/view5"]
    with pytest.raises(sm.SMError):
        matcher.match(L, R, 3, 16, agg="device-cu", lr_check=True)
    with pytest.raises(sm.SMError):
        matcher.match(L, R, 3, 16, agg="device-cu", median=True)
    # the handle still works after the rejected calls
    assert matcher.match(L, R, 3, 16, agg="device-cu").shape == L.shape


# ---- wide windows: radius 16..127 through the generic kernel (Device.cu:46-56's window is unbounded) ----

@pytest.mark.parametrize("r", [17, 31, 64, 127])
def test_wide_radius_bit_exact(matcher, oracle, r):
    rng = np.random.default_rng(500 + r)
    H, W, D = 70, 150, 24
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    R = np.roll(L, -5, axis=1) ^ rng.integers(0, 16, (H, W), dtype=np.uint8)
    assert np.array_equal(matcher.match(L, R, r, D), oracle.box_disp(L, R, r, D))


def test_wide_radius_127_key_headroom(matcher, oracle):
    """r = 127: a window sum reaches 255 * 255^2 = 16,581,375, and (SAD << 8) 4.245e9 of the 4.295e9 u32
    range.  A 255-wide frame of AD 255 puts the centre pixel's full window at that sum."""
    H, W, D = 255, 256, 2
    Lf = np.full((H, W), 255, np.uint8)
    Rz = np.zeros((H, W), np.uint8)
    assert np.array_equal(matcher.match(Lf, Rz, 127, D), oracle.box_disp(Lf, Rz, 127, D))
    rng = np.random.default_rng(127)
    L = (rng.integers(0, 2, (96, 120), dtype=np.uint8) * 255).astype(np.uint8)
    R = (rng.integers(0, 2, (96, 120), dtype=np.uint8) * 255).astype(np.uint8)
    assert np.array_equal(matcher.match(L, R, 127, 6), oracle.box_disp(L, R, 127, 6))


def test_literal_wide_radius_127(matcher, oracle):
    """The literal mode at r = 127, a window larger than the 256 x 320 corner, on 0/255 images."""
    rng = np.random.default_rng(128)
    H, W, D = 260, 330, 16
    L = (rng.integers(0, 2, (H, W), dtype=np.uint8) * 255).astype(np.uint8)
    R = (rng.integers(0, 2, (H, W), dtype=np.uint8) * 255).astype(np.uint8)
    assert np.array_equal(matcher.match(L, R, 127, D, agg="device-cu"), oracle.device_cu_literal_integral(L, R, 127, D))


@pytest.mark.parametrize("r", [17, 40])
def test_wide_radius_lr(matcher, oracle, r):
    """LR at r > 15: the mirrored right-view pass + lr_check (StereoDisparity.cpp:136-147)."""
    rng = np.random.default_rng(900 + r)
    H, W, D = 48, 130, 20
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    R = np.roll(L, -4, axis=1) ^ rng.integers(0, 8, (H, W), dtype=np.uint8)
    chk, rd, mask = matcher.match_lr(L, R, r, D)
    _, rd_o, chk_o, mask_o = oracle.box_lr(L, R, r, D)
    assert np.array_equal(rd, rd_o) and np.array_equal(chk, chk_o) and np.array_equal(mask, mask_o)


# ---- the separable wide-window path (bm_wide.hip, radius 16..127, width <= 4096) ----

@pytest.mark.parametrize("W,H,r,D", [(1920, 1080, 20, 128), (333, 77, 16, 256), (4096, 40, 40, 24), (61, 300, 99, 7)])
def test_wide_path_bit_exact_sizes(matcher, oracle, W, H, r, D):
    """Full HD at r = 20, D = 256, the 4096-column limit (16 outputs per thread), a narrow tall frame."""
    if W > 2048:
        import gpu_stereo_matching_amd as sm
        m = sm.BlockMatcher(0, 4096, 64, 64)
    else:
        m = matcher
    L, R = oracle.synth_pair(40 + r, W, H, max(D, 16))
    assert np.array_equal(m.match(L, R, r, D), oracle.box_disp(L, R, r, D))


def test_wide_path_fallback_past_4096_columns(oracle):
    """Wider than 4096 columns: the strip kernel at r 16..37 (no width limit; the LR check's mirrored right view
    too, valid_mode 1), the direct generic kernel past it (correct, not fast)."""
    import gpu_stereo_matching_amd as sm
    L, R = oracle.synth_pair(9, 4100, 6, 16)
    with sm.BlockMatcher(0, 4100, 8, 16) as m:
        assert np.array_equal(m.match(L, R, 16, 4), oracle.box_disp(L, R, 16, 4))
        assert np.array_equal(m.match(L, R, 40, 4), oracle.box_disp(L, R, 40, 4))
        chk, rd, mask = m.match_lr(L, R, 20, 5)
        _, rd_o, chk_o, mask_o = oracle.box_lr(L, R, 20, 5)
        assert np.array_equal(rd, rd_o) and np.array_equal(chk, chk_o) and np.array_equal(mask, mask_o)
    L2, R2 = oracle.synth_pair(10, 5000, 90, 128)
    with sm.BlockMatcher(0, 5000, 90, 128) as m:
        assert np.array_equal(m.match(L2, R2, 24, 128), oracle.box_disp(L2, R2, 24, 128))
        chk, rd, mask = m.match_lr(L2, R2, 17, 100)
        _, rd_o, chk_o, mask_o = oracle.box_lr(L2, R2, 17, 100)
        assert np.array_equal(rd, rd_o) and np.array_equal(chk, chk_o) and np.array_equal(mask, mask_o)


@pytest.mark.parametrize("r,D", [(16, 64), (31, 48), (127, 12)])
def test_wide_path_lr_and_median_device_batch(sm, matcher, oracle, r, D):
    """The right view from the same row pass (C_R(u, d) = C_L(u + d, d)), with and without the 7x7 median,
    batched on the device: every frame equal to the oracle's LR maps."""
    import torch
    pairs = [oracle.synth_pair(70 + i, 180, 60, max(D, 16)) for i in range(3)]
    Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    out = matcher.match_device(Lt, Rt, r, D, lr_check=True)
    torch.cuda.synchronize()
    for i, (L, R) in enumerate(pairs):
        assert np.array_equal(out[i].cpu().numpy(), oracle.box_lr(L, R, r, D)[2]), i
    chk, rd, mask = matcher.match_lr(pairs[0][0], pairs[0][1], r, D, median=True)
    _, cost = oracle.box_disp(pairs[0][0], pairs[0][1], r, D, want_cost=True)
    left_m = oracle.median(oracle.box_disp(pairs[0][0], pairs[0][1], r, D), 3)
    right_m = oracle.median(oracle.right_wta(cost), 3)
    chk_o, mask_o = oracle.lr_check(left_m, right_m)
    assert np.array_equal(chk, chk_o) and np.array_equal(mask, mask_o)


def test_wide_path_slice_keys(matcher, oracle):
    """d-slice keys at r > 15 (sm_slice_keys_device through the wide path) equal the oracle's keys."""
    import torch
    L, R = oracle.synth_pair(12, 300, 90, 64)
    Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    for a, b in ((0, 20), (20, 64), (63, 64)):
        k = matcher.slice_keys_device(Lt, Rt, 21, a, b)
        torch.cuda.synchronize()
        assert np.array_equal(k.cpu().numpy().view(np.uint32), oracle.box_keys_slice(L, R, 21, a, b)), (a, b)
    assert np.array_equal(matcher.dslice_rehearse(L, R, 21, 64, 3), oracle.box_disp(L, R, 21, 64))


def test_wide_path_frame_groups_partial_last_group(matcher, oracle):
    """Frame groups of the wide path (bm_wide.hip: up to 4 frames per vsum/hwta pair, ceil(2048 / H) of
    them): 5 frames of height 700 run as a group of 3 and a group of 2; every frame, left and right view,
    equal to the oracle."""
    import torch
    pairs = [oracle.synth_pair(300 + i, 96, 700, 32) for i in range(5)]
    Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    out = matcher.match_device(Lt, Rt, 19, 24)
    outlr = matcher.match_device(Lt, Rt, 19, 24, lr_check=True)
    torch.cuda.synchronize()
    for i, (L, R) in enumerate(pairs):
        assert np.array_equal(out[i].cpu().numpy(), oracle.box_disp(L, R, 19, 24)), i
        assert np.array_equal(outlr[i].cpu().numpy(), oracle.box_lr(L, R, 19, 24)[2]), i


@pytest.mark.parametrize("W,H", [(4, 1), (5, 3), (7, 40), (8, 2), (13, 17)])
def test_wide_path_tiny_frames(matcher, oracle, W, H):
    """The wide path's smallest frames (4 <= W < 16, a single row): clamped dword columns and the
    per-lane byte shifts cover every column; left map and LR equal the oracle."""
    rng = np.random.default_rng(W * 100 + H)
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    R = rng.integers(0, 256, (H, W), dtype=np.uint8)
    for D in (1, 3, W + 2):
        assert np.array_equal(matcher.match(L, R, 16, D), oracle.box_disp(L, R, 16, D)), D
        chk, rd, mask = matcher.match_lr(L, R, 16, D)
        _, rd_o, chk_o, mask_o = oracle.box_lr(L, R, 16, D)
        assert np.array_equal(rd, rd_o) and np.array_equal(chk, chk_o) and np.array_equal(mask, mask_o), D
