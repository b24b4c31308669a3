"""GPU parity for the strip kernel (bm_strip.hip, right view in bm_strip_lr.hip): box matching at radius 16..37, lanes =
disparities, vertical sums in registers.  Every map and slice-key array equals the oracle's getDisp
(Device.cu:27-63) bit for bit: every radius the kernel is instantiated for, edge strips (d > x, the last strip
past W), several row bands, frames in a batch, d-slices starting past 0, tie-heavy textures and the key
headroom at r = 37."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sm():
    import gpu_stereo_matching_amd as sm
    return sm


@pytest.fixture(scope="module")
def matcher(sm):
    m = sm.BlockMatcher(0, 2048, 1100, 256)
    yield m
    m.close()


@pytest.mark.parametrize("r", list(range(16, 39)))
def test_strip_every_radius(matcher, oracle, r):
    """Every instantiated radius, and r = 38, the first past the strip range (the separable path)."""
    rng = np.random.default_rng(7000 + r)
    W = int(rng.integers(4, 400))
    H = int(rng.integers(1, 160))
    D = int(rng.choice([1, 7, 63, 64, 65, 128, 200, 256]))
    L, R = oracle.synth_pair(7000 + r, W, H, max(D, 16))
    assert np.array_equal(matcher.match(L, R, r, D), oracle.box_disp(L, R, r, D)), (W, H, D)


@pytest.mark.parametrize("W,H,r,D", [(96, 700, 19, 24), (1000, 333, 37, 256), (130, 64, 16, 192), (54, 90, 37, 100),
                                     (55, 90, 37, 100), (4, 3, 16, 5), (255, 1, 24, 64)])
def test_strip_shapes(matcher, oracle, W, H, r, D):
    """A tall frame over 8 bands; exactly one / just past one strip of 54 outputs; 4 waves of d; a 4-column frame;
    a single row."""
    L, R = oracle.synth_pair(W + 3 * H + r, W, H, max(D, 16))
    assert np.array_equal(matcher.match(L, R, r, D), oracle.box_disp(L, R, r, D))


def test_strip_ties(matcher, oracle):
    """0/1 textures: most windows tie on cost, the smallest d wins as in the key MIN."""
    rng = np.random.default_rng(31)
    for r, D in ((16, 40), (25, 130), (37, 70)):
        L = rng.integers(0, 2, (120, 300), dtype=np.uint8)
        R = rng.integers(0, 2, (120, 300), dtype=np.uint8)
        assert np.array_equal(matcher.match(L, R, r, D), oracle.box_disp(L, R, r, D)), r


def test_strip_key_headroom_r37(matcher, oracle):
    """AD 255 everywhere: V = 75 * 255 in each u16 half, S = 75^2 * 255 < 2^24 (key << 8 in range)."""
    Lf = np.full((160, 200), 255, np.uint8)
    Rz = np.zeros((160, 200), np.uint8)
    assert np.array_equal(matcher.match(Lf, Rz, 37, 9), oracle.box_disp(Lf, Rz, 37, 9))


def test_strip_device_batch(matcher, oracle):
    import torch
    pairs = [oracle.synth_pair(900 + i, 333, 120, 96) for i in range(3)]
    Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    out = matcher.match_device(Lt, Rt, 22, 96)
    torch.cuda.synchronize()
    for i, (L, R) in enumerate(pairs):
        assert np.array_equal(out[i].cpu().numpy(), oracle.box_disp(L, R, 22, 96)), i


def test_strip_slice_keys(matcher, oracle):
    """d-slice keys (no right view) through the strip kernel, slices starting past 0 and past one wave of d."""
    import torch
    L, R = oracle.synth_pair(44, 400, 90, 240)
    Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    for a, b in ((0, 20), (20, 64), (63, 64), (64, 200), (130, 240)):
        k = matcher.slice_keys_device(Lt, Rt, 25, a, b)
        torch.cuda.synchronize()
        assert np.array_equal(k.cpu().numpy().view(np.uint32), oracle.box_keys_slice(L, R, 25, a, b)), (a, b)
    assert np.array_equal(matcher.dslice_rehearse(L, R, 25, 240, 3), oracle.box_disp(L, R, 25, 240))


@pytest.mark.parametrize("r", [16, 22, 29, 37])
def test_strip_lr(matcher, oracle, r):
    """The right view folded in the strip kernel (LDS row + global atomic MIN): checked map, dR and mask equal the
    oracle's box_lr (StereoDisparity.cpp:136-147), edge strips and D past the frame's columns included."""
    rng = np.random.default_rng(8000 + r)
    W = int(rng.integers(60, 700))
    H = int(rng.integers(20, 200))
    D = int(rng.choice([9, 64, 100, 200, 256]))
    L, R = oracle.synth_pair(8000 + r, W, H, max(D, 16))
    chk, rd, mask = matcher.match_lr(L, R, r, D)
    _, rd_o, chk_o, mask_o = oracle.box_lr(L, R, r, D)
    assert np.array_equal(rd, rd_o) and np.array_equal(chk, chk_o) and np.array_equal(mask, mask_o), (W, H, D)


def test_strip_lr_median_device_batch(matcher, oracle):
    """Right keys of several frames in one launch (one right-key plane per frame), with the 7x7 median."""
    import torch
    r, D = 24, 80
    pairs = [oracle.synth_pair(950 + i, 301, 97, D) for i in range(3)]
    Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    out = matcher.match_device(Lt, Rt, r, D, lr_check=True)
    torch.cuda.synchronize()
    for i, (L, R) in enumerate(pairs):
        assert np.array_equal(out[i].cpu().numpy(), oracle.box_lr(L, R, r, D)[2]), i
    L, R = pairs[0]
    chk, rd, mask = matcher.match_lr(L, R, r, D, median=True)
    _, cost = oracle.box_disp(L, R, r, D, want_cost=True)
    chk_o, mask_o = oracle.lr_check(oracle.median(oracle.box_disp(L, R, r, D), 3), oracle.median(oracle.right_wta(cost), 3))
    assert np.array_equal(chk, chk_o) and np.array_equal(mask, mask_o)
