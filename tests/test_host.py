"""CPU tests of host-side code: synthetic generator, gray conversion, API argument checks."""
import numpy as np
import pytest

import gpu_stereo_matching_amd as sm
from gpu_stereo_matching_amd.synth import ground_truth_rows


@pytest.mark.parametrize("seed,W,H,D", [(1234, 97, 33, 128), (1, 50, 20, 8), (4321, 301, 70, 192)])
def test_synth_matches_c_generator(oracle, seed, W, H, D):
    a = sm.synth_pair(seed, W, H, D)
    b = oracle.synth_pair(seed, W, H, D)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_synth_ground_truth_shift():
    W, H, D = 200, 64, 128
    L, R = sm.synth_pair(9, W, H, D)
    gt = ground_truth_rows(H, D)
    for y in range(H):
        g = int(gt[y])
        assert np.array_equal(R[y, : W - g], L[y, g:])


def test_gray_formula_opencv24(oracle):
    rng = np.random.default_rng(0)
    bgr = rng.integers(0, 256, (17, 23, 3), dtype=np.uint8)
    g = sm.bgr_to_gray(bgr)
    assert np.array_equal(g, oracle.bgr_to_gray(bgr))
    # fixed points of the fixed-point formula
    assert sm.bgr_to_gray(np.full((1, 1, 3), 255, np.uint8))[0, 0] == 255
    assert sm.bgr_to_gray(np.array([[[0, 0, 255]]], np.uint8))[0, 0] == (4899 * 255 + 8192) >> 14
    bgra = np.concatenate([bgr, np.full((17, 23, 1), 9, np.uint8)], axis=2)
    assert np.array_equal(sm.bgr_to_gray(bgra), g)


def test_gray_fixtures_are_gray(gray):
    assert gray["Art_/view1"].shape == (256, 320)
    assert gray["Art/view1"].shape == (370, 463)
    assert gray["Laundry/view1"].shape == (370, 447)
    assert gray["Art_/view1"].dtype == np.uint8


def test_api_rejects_bad_images():
    with pytest.raises(ValueError):
        sm._as_u8_image(np.zeros((4, 4), np.float32), "x")
    with pytest.raises(ValueError):
        sm._as_u8_image(np.zeros((4, 4, 3), np.uint8), "x")
    with pytest.raises(ValueError):
        sm._flags("median", False)
    assert sm._flags("guided", True) == sm.SM_AGG_GUIDED | sm.SM_LR_CHECK


def test_device_pair_checks_reject_bad_inputs():
    """The slice-key wrappers validate what the C ABI cannot (dtype, rank, shape, device, contiguity)."""
    import torch
    import gpu_stereo_matching_amd as sm
    a = torch.zeros((4, 8), dtype=torch.uint8)
    with pytest.raises(ValueError, match="uint8"):
        sm._check_device_pair(a.float(), a)
    with pytest.raises(ValueError, match="equal"):
        sm._check_device_pair(a, torch.zeros((4, 9), dtype=torch.uint8))
    with pytest.raises(ValueError, match="equal"):
        sm._check_device_pair(a[None], a[None])
    with pytest.raises(ValueError, match="device"):
        sm._check_device_pair(a, a)


def test_pair_sequence_order_and_bgr(tmp_path):
    """capture.PairSequence: photo()'s Left_<n>/Right_<n> files (Utility.cpp:217-218) in numeric order
    (10 after 2), unmatched left files skipped, frames returned as BGR like cv::imread."""
    from PIL import Image
    from gpu_stereo_matching_amd.capture import PairSequence
    rng = np.random.default_rng(3)
    frames = {}
    for n in (0, 2, 10):
        lr = [rng.integers(0, 256, (6, 9, 3), dtype=np.uint8) for _ in range(2)]
        frames[n] = lr
        Image.fromarray(lr[0]).save(tmp_path / f"Left_{n}.png")    # written as RGB
        Image.fromarray(lr[1]).save(tmp_path / f"Right_{n}.png")
    Image.fromarray(frames[0][0]).save(tmp_path / "Left_7.png")      # no Right_7
    seq = PairSequence(str(tmp_path))
    assert len(seq) == 3
    got = list(seq)
    assert [g[0] for g in got] == [0, 2, 10]
    for n, left, right in got:
        assert np.array_equal(left, frames[n][0][:, :, ::-1])
        assert np.array_equal(right, frames[n][1][:, :, ::-1])
    small = list(PairSequence(str(tmp_path), size=(3, 2)))
    assert small[0][1].shape == (2, 3, 3)


def test_stmatch_usage(capsys):
    """STMatching's command line prints its usage with fewer than three arguments (main.cpp:41-47)."""
    from gpu_stereo_matching_amd import stmatch
    assert stmatch._main([]) == 0
    assert "leftImgPath rightImgPath dispImgPath" in capsys.readouterr().out
