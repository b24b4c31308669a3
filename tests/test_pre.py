"""The steps in front of the matching path: GPU BGR->gray (OpenCV 2.4 fixed point,
Caller.cpp:15-16) and the rectification remap (Device.cu:127-167 / Utility.cpp:239-264)."""
import numpy as np
import pytest


def _maps(H, W, seed, kind):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    if kind == "identity":
        return xx, yy
    if kind == "shift":
        return xx + 0.5, yy + 0.25
    if kind == "random":
        return (rng.uniform(-3, W + 3, (H, W)).astype(np.float32), rng.uniform(-3, H + 3, (H, W)).astype(np.float32))
    # smooth radial-ish warp like an undistort map
    cx, cy = W / 2, H / 2
    r2 = ((xx - cx) ** 2 + (yy - cy) ** 2) / (cx * cx + cy * cy)
    k = 1 + 0.08 * r2
    return (cx + (xx - cx) * k).astype(np.float32), (cy + (yy - cy) * k + 0.3).astype(np.float32)


def test_oracle_remap_identity_quirk(oracle):
    """Identity map: interior copied; last row/column read 0 because the right/bottom tap is out
    of range (Device.cu:155: x2 >= rows || y2 >= cols -> 0)."""
    rng = np.random.default_rng(1)
    src = rng.integers(0, 256, (9, 13), dtype=np.uint8)
    mx, my = _maps(9, 13, 0, "identity")
    out = oracle.remap(src, mx, my)
    assert np.array_equal(out[:-1, :-1], src[:-1, :-1])
    assert (out[-1, :] == 0).all() and (out[:, -1] == 0).all()


def test_oracle_remap_half_pixel_rounds_to_even(oracle):
    src = np.array([[10, 11, 12], [10, 11, 12], [0, 0, 0]], np.uint8)
    mx = np.full((3, 3), 0.5, np.float32)
    my = np.zeros((3, 3), np.float32)
    # 0.5*10 + 0.5*11 = 10.5 -> round half to even -> 10
    assert oracle.remap(src, mx, my)[0, 0] == 10
    mx[:] = 1.5   # 11.5 -> 12
    assert oracle.remap(src, mx, my)[0, 0] == 12


@pytest.mark.gpu
def test_gpu_bgr_to_gray_fixture(gray):
    """GPU gray of the bundled colour pair == the committed gray fixture (Caller.cpp:15-16)."""
    import torch
    import gpu_stereo_matching_amd as sm
    m = sm.BlockMatcher(0, 512, 512, 64)
    for v in ("view1", "view5"):
        bgr = torch.from_numpy(gray[f"Art_/{v}_bgr"]).cuda()
        g = m.bgr_to_gray_device(bgr)
        torch.cuda.synchronize()
        assert np.array_equal(g.cpu().numpy(), gray[f"Art_/{v}"])
    m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("C,W,H", [(3, 97, 31), (4, 64, 8), (3, 1, 5), (4, 1923, 7)])
def test_gpu_bgr_to_gray_random(oracle, C, W, H):
    import torch
    import gpu_stereo_matching_amd as sm
    rng = np.random.default_rng(W * H + C)
    bgr = rng.integers(0, 256, (H, W, C), dtype=np.uint8)
    m = sm.BlockMatcher(0, 2048, 64, 64)
    g = m.bgr_to_gray_device(torch.from_numpy(bgr).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(g.cpu().numpy(), oracle.bgr_to_gray(bgr))
    m.close()


@pytest.mark.gpu
def test_gpu_match_bgr_entry(gray, bm_expected):
    """imread -> cvtColor -> blockMatching_gpu(5, 64) in one call == the singleFrame golden map."""
    import gpu_stereo_matching_amd as sm
    m = sm.BlockMatcher(0, 512, 512, 256)
    got = m.match_bgr(gray["Art_/view1_bgr"], gray["Art_/view5_bgr"], 5, 64)
    assert np.array_equal(got, bm_expected["Art_/r5/D64"])
    m.close()


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["identity", "shift", "random", "warp"])
def test_gpu_remap(oracle, kind):
    import torch
    import gpu_stereo_matching_amd as sm
    H, W = 200, 320     # remapTest's target size (Caller.cpp:35)
    rng = np.random.default_rng(7)
    src = rng.integers(0, 256, (H, W), dtype=np.uint8)
    mx, my = _maps(H, W, 3, kind)
    m = sm.BlockMatcher(0, 512, 512, 64)
    out = m.remap_device(torch.from_numpy(src).cuda(), torch.from_numpy(mx).cuda(), torch.from_numpy(my).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), oracle.remap(src, mx, my))
    m.close()


@pytest.mark.gpu
def test_host_entry_points_cvt_color_and_remap(oracle, gray):
    """sm_bgr_to_gray_u8 / sm_remap_u8: the host-pointer forms behind cvtColor_gpu / remap_gpu."""
    import gpu_stereo_matching_amd as sm
    m = sm.BlockMatcher(0, 640, 480, 64)
    bgr = gray["Art_/view1_bgr"]
    assert np.array_equal(m.cvt_color(bgr), oracle.bgr_to_gray(bgr))
    L = gray["Art/view1"]
    H, W = L.shape
    rng = np.random.default_rng(5)
    mapx = (np.arange(W, dtype=np.float32)[None, :] + rng.uniform(-3, 3, (H, W)).astype(np.float32))
    mapy = (np.arange(H, dtype=np.float32)[:, None] + rng.uniform(-3, 3, (H, W)).astype(np.float32))
    assert np.array_equal(m.remap(L, mapx, mapy), oracle.remap(L, mapx, mapy))
    m.close()
