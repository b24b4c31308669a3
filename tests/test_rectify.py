"""Rectification in front of the remap: remapTest's chain
LoadDataBatch (Utility.cpp:25-42) -> Rectify (Utility.cpp:228-234: OpenCV 2.4 stereoRectify with
CV_CALIB_ZERO_DISPARITY, alpha = -1, then initUndistortRectifyMap CV_32FC1) -> remap_gpu.

Pinning: the calibration is the reference's own Calib_Data_OpenCV.yml (tests/golden, copied as data),
the pair is Chess/Set2 (tests/golden/chess_set2_gray.npz, tests/golden/make_calib_fixture.py).  No
OpenCV output exists in the reference or in this image, so parity with OpenCV itself is UNPINNED:
  * stereoRectify: the product's C++ (sm_stereo_rectify, host-only, no GPU) against the oracle's
    independent numpy restatement (SVD vs Newton polar factor in Rodrigues) — R1/R2 within 1e-12,
    P1/P2/Q to 1e-12 relative — plus the geometric properties the function guarantees;
  * maps: the GPU kernel against the oracle's C loop bit-exact (both fp64 in OpenCV's operation
    order, no contraction, rounded to float once), and the C loop against a vectorised numpy form
    of the same formula within 1e-3 px;
  * remap of the rectified pair: bit-exact with the CPU_Remap restatement.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

YML = os.path.join(GOLDEN, "Calib_Data_OpenCV.yml")


@pytest.fixture(scope="module")
def calib_data():
    from gpu_stereo_matching_amd import calib
    return calib.load_data_batch(YML)


@pytest.fixture(scope="module")
def chess():
    return np.load(os.path.join(GOLDEN, "chess_set2_gray.npz"))


def _rot(rng, scale):
    from oracle import oracle as O
    return O.rodrigues_to_mat(rng.normal(0, scale, 3))


def _cases():
    """(name, K1, d1, K2, d2, (w, h), R, T) synthetic calibrations covering the branches."""
    rng = np.random.default_rng(7)
    K = lambda f, cx, cy: np.array([[f, 0, cx], [0, f * 1.002, cy], [0, 0, 1]], np.float64)  # noqa: E731
    out = []
    out.append(("horizontal_d5", K(800, 330, 250), [0.05, -0.2, 0.001, -0.0005, 0.01], K(810, 320, 245),
                [-0.08, 0.1, -0.0003, 0.0007, 0.0], (640, 480), _rot(rng, 0.01), [-60.0, 0.4, 0.2]))
    out.append(("vertical", K(700, 300, 200), [0.02, -0.1, 0, 0], K(705, 310, 210), [0.01, -0.05, 0, 0],
                (600, 400), _rot(rng, 0.02), [0.5, 55.0, -1.0]))
    out.append(("no_dist_rvec", K(500, 160, 100), [], K(510, 158, 102), [], (320, 200), rng.normal(0, 0.02, 3),
                [30.0, -0.3, 0.1]))
    out.append(("rational_d8", K(900, 480, 270), [-0.3, 0.1, 0.001, 0.002, -0.01, 0.05, 0.01, 0.002],
                K(905, 470, 275), [-0.25, 0.08, 0, 0.001, 0.0, 0.02, 0.0, 0.0], (960, 540), _rot(rng, 0.005),
                [-120.0, 1.0, 2.0]))
    out.append(("identity_R", K(600, 320, 240), [0.0, 0.0, 0.0, 0.0, 0.0], K(600, 320, 240), [0, 0, 0, 0, 0],
                (640, 480), np.eye(3), [-50.0, 0.0, 0.0]))
    return out


CASES = _cases()


def test_load_data_batch_fixture(calib_data):
    """LoadDataBatch: six matrices, float32 values widened to float64 (dt: f, convertTo CV_64F)."""
    K1, K2, d1, d2, R, T = calib_data
    assert K1.shape == K2.shape == R.shape == (3, 3)
    assert d1.shape == d2.shape == (5, 1) and T.shape == (3, 1)
    assert all(a.dtype == np.float64 for a in calib_data)
    assert K1[0, 0] == np.float64(np.float32(1116.744104))
    assert T[0, 0] == np.float64(np.float32(-46.993557))
    assert d2[1, 0] == np.float64(np.float32(-0.311851))


def test_load_data_by_name():
    from gpu_stereo_matching_amd import calib
    assert calib.load_data(YML, "RightDist").shape == (5, 1)
    with pytest.raises(KeyError):
        calib.load_data(YML, "Nope")


def _check_rectify(oracle, K1, d1, K2, d2, size, R, T):
    from gpu_stereo_matching_amd import calib
    got = calib.stereo_rectify(K1, d1, K2, d2, size, R, T)
    want = oracle.stereo_rectify(K1, d1, K2, d2, size[0], size[1], R, T)
    for g, w, name in zip(got, want, ("R1", "R2", "P1", "P2", "Q")):
        tol = 1e-12 * max(1.0, float(np.abs(w).max()))
        assert np.abs(g - w).max() <= tol, (name, np.abs(g - w).max())
    return got


def test_stereo_rectify_fixture_matches_restatement(oracle, calib_data):
    """remapTest's Rectify at 320x200 (Caller.cpp:35) and at the full 1280x800 frame."""
    K1, K2, d1, d2, R, T = calib_data
    for size in ((320, 200), (1280, 800)):
        _check_rectify(oracle, K1, d1, K2, d2, size, R, T)


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_stereo_rectify_cases_match_restatement(oracle, case):
    _check_rectify(oracle, *case[1:])


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_stereo_rectify_geometry(case):
    """What stereoRectify guarantees: R1, R2 rotations; the rectified baseline along one axis; with
    CV_CALIB_ZERO_DISPARITY, equal P1/P2 intrinsics, so a 3-D point lands on the same rectified row
    (horizontal rig) or column (vertical rig) in both views; Q reprojects (x, y, disparity) to it."""
    from gpu_stereo_matching_amd import calib
    from oracle import oracle as O
    _, K1, d1, K2, d2, size, R, T = case
    R = np.asarray(R, np.float64)
    Rm = R if R.size == 9 else O.rodrigues_to_mat(R)
    T = np.asarray(T, np.float64).reshape(3)
    R1, R2, P1, P2, Q = calib.stereo_rectify(K1, d1, K2, d2, size, R, T)
    for Rk in (R1, R2):
        assert np.allclose(Rk @ Rk.T, np.eye(3), atol=1e-12) and abs(np.linalg.det(Rk) - 1) < 1e-12
    idx = 0 if abs(T[0]) > abs(T[1]) else 1
    b = R2 @ T
    assert abs(b[1 - idx]) < 1e-9 * np.linalg.norm(T) and abs(b[2]) < 1e-9 * np.linalg.norm(T)
    assert np.array_equal(P1[:, :3], P2[:, :3])
    rng = np.random.default_rng(3)
    for _ in range(20):
        X = np.array([rng.uniform(-500, 500), rng.uniform(-500, 500), rng.uniform(800, 5000)])
        x1 = P1 @ np.append(R1 @ X, 1.0)
        x2 = P2 @ np.append(R1 @ X, 1.0)            # P2 maps rectified camera-1 coordinates
        assert np.allclose(R2 @ (Rm @ X + T), R1 @ X + R2 @ T, atol=1e-9)
        u1, u2 = x1[:2] / x1[2], x2[:2] / x2[2]
        assert abs(u1[1 - idx] - u2[1 - idx]) < 1e-6
        if idx == 0:
            Xh = Q @ np.array([u1[0], u1[1], u1[0] - u2[0], 1.0])
            assert np.allclose(Xh[:3] / Xh[3], R1 @ X, rtol=1e-8)


def _numpy_map(K, dist, R, P, W, H):
    """initUndistortRectifyMap, vectorised (direct i/j products instead of the running sums)."""
    k = np.zeros(8)
    k[:len(dist)] = np.ravel(dist)
    iR = np.linalg.inv(P[:, :3] @ R)
    jj, ii = np.meshgrid(np.arange(W, dtype=np.float64), np.arange(H, dtype=np.float64))
    X = jj * iR[0, 0] + ii * iR[0, 1] + iR[0, 2]
    Y = jj * iR[1, 0] + ii * iR[1, 1] + iR[1, 2]
    Wh = jj * iR[2, 0] + ii * iR[2, 1] + iR[2, 2]
    x, y = X / Wh, Y / Wh
    r2 = x * x + y * y
    kr = (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2) / (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2)
    u = K[0, 0] * (x * kr + k[2] * 2 * x * y + k[3] * (r2 + 2 * x * x)) + K[0, 2]
    v = K[1, 1] * (y * kr + k[2] * (r2 + 2 * y * y) + k[3] * 2 * x * y) + K[1, 2]
    return u.astype(np.float32), v.astype(np.float32)


def test_oracle_map_vs_vectorised(oracle, calib_data):
    K1, K2, d1, d2, R, T = calib_data
    R1, R2, P1, P2, _ = oracle.stereo_rectify(K1, d1, K2, d2, 320, 200, R, T)
    for K, d, Rk, Pk in ((K1, d1, R1, P1), (K2, d2, R2, P2)):
        mx, my = oracle.init_rectify_map(K, d, Rk, Pk, 320, 200)
        nx, ny = _numpy_map(K, d, Rk, Pk, 320, 200)
        assert np.abs(mx - nx).max() < 1e-3 and np.abs(my - ny).max() < 1e-3


def test_stereo_rectify_rejects_bad_args():
    from gpu_stereo_matching_amd import _capi, calib
    K = np.eye(3)
    with pytest.raises(_capi.SMError) as e:
        calib.stereo_rectify(K, [0.1, 0.2, 0.3], K, [], (64, 48), np.eye(3), [1.0, 0, 0])
    assert e.value.code == _capi.SM_ERR_INVALID_ARG
    with pytest.raises(_capi.SMError):
        calib.stereo_rectify(K, [], K, [], (0, 48), np.eye(3), [1.0, 0, 0])
    with pytest.raises(_capi.SMError):
        calib.stereo_rectify(K, [], K, [], (64, 48), np.eye(2), [1.0, 0, 0])
    with pytest.raises(ValueError):
        calib.stereo_rectify(K, [], K, [], (64, 48), np.eye(3), [1.0, 0])


# ----------------------------------------------------------------------------------------- GPU
MAP_SIZES = [(320, 200), (1280, 800), (97, 65), (1, 1), (64, 129), (1920, 1080)]


@pytest.mark.gpu
@pytest.mark.parametrize("size", MAP_SIZES, ids=[f"{w}x{h}" for w, h in MAP_SIZES])
def test_gpu_rectify_map_bit_exact(oracle, calib_data, size):
    """initUndistortRectifyMap on the GPU == the oracle's fp64 loop, bit for bit, both cameras; host
    form and device form (with a pitched destination)."""
    import torch
    import gpu_stereo_matching_amd as sm
    from gpu_stereo_matching_amd import calib
    W, H = size
    K1, K2, d1, d2, R, T = calib_data
    R1, R2, P1, P2, _ = calib.stereo_rectify(K1, d1, K2, d2, size, R, T)
    with sm.BlockMatcher(0, 64, 64, 16) as m:
        for K, d, Rk, Pk in ((K1, d1, R1, P1), (K2, d2, R2, P2)):
            want_x, want_y = oracle.init_rectify_map(K, d, Rk, Pk, W, H)
            gx, gy = m.init_rectify_map(K, d, Rk, Pk, W, H)
            assert np.array_equal(gx, want_x) and np.array_equal(gy, want_y)
            bx = torch.full((H, W + 7), -1.0, device="cuda:0")
            by = torch.full((H, W + 7), -1.0, device="cuda:0")
            m.init_rectify_map_device(K, d, Rk, Pk, W, H, bx[:, :W], by[:, :W])
            torch.cuda.synchronize()
            assert np.array_equal(bx[:, :W].cpu().numpy(), want_x) and np.array_equal(by[:, :W].cpu().numpy(), want_y)
            assert (bx[:, W:] == -1).all() and (by[:, W:] == -1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_gpu_rectify_map_cases(oracle, case):
    import gpu_stereo_matching_amd as sm
    from gpu_stereo_matching_amd import calib
    _, K1, d1, K2, d2, size, R, T = case
    R1, R2, P1, P2, _ = calib.stereo_rectify(K1, d1, K2, d2, size, R, T)
    with sm.BlockMatcher(0, 64, 64, 16) as m:
        for K, d, Rk, Pk in ((K1, d1, R1, P1), (K2, d2, R2, P2)):
            want = oracle.init_rectify_map(K, d, Rk, Pk, *size)
            got = m.init_rectify_map(K, d, Rk, Pk, *size)
            assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])


@pytest.mark.gpu
@pytest.mark.parametrize("key", ["320x200", "full"])
def test_gpu_remap_test_chain(oracle, calib_data, chess, key):
    """remapTest (Caller.cpp:27-74) in Python: Rectify (GPU maps) then remap_gpu on both views, at
    remapTest's 320x200 and at the calibration's own 1280x800; bit-exact with the oracle chain."""
    import gpu_stereo_matching_amd as sm
    from gpu_stereo_matching_amd import calib
    L, Rimg = chess[f"Left_{key}"], chess[f"Right_{key}"]
    H, W = L.shape
    K1, K2, d1, d2, R, T = calib_data
    with sm.BlockMatcher(0, W, H, 16) as m:
        mx1, my1, mx2, my2 = calib.rectify(m, K1, K2, d1, d2, R, T, (W, H))
        R1, R2, P1, P2, _ = calib.stereo_rectify(K1, d1, K2, d2, (W, H), R, T)
        assert np.array_equal(mx1, oracle.init_rectify_map(K1, d1, R1, P1, W, H)[0])
        for img, mx, my in ((L, mx1, my1), (Rimg, mx2, my2)):
            got = m.remap(img, mx, my)
            assert np.array_equal(got, oracle.remap(img, mx, my))
            assert (got > 0).mean() > 0.5      # the rectified view is mostly inside the source


def test_cpp_adapter_load_data_batch(tmp_path):
    """sm::LoadDataBatch / sm::LoadData in include/stereo_bm.hpp (Utility.cpp:17-42) parse the
    reference's calibration YAML to the same CV_64FC1 values as the Python loader.  Host-only: the
    parser calls nothing in the library, so the test program needs no GPU and no link."""
    import subprocess
    from gpu_stereo_matching_amd import calib
    from conftest import ROOT
    src = tmp_path / "ldb.cpp"
    src.write_text(r'''
#include <cstdio>
#include "stereo_bm.hpp"
int main(int argc, char** argv) {
    sm::Mat m[6];
    if (!sm::LoadDataBatch(argv[1], m[0], m[1], m[2], m[3], m[4], m[5])) return 2;
    for (auto& a : m) {
        std::printf("%d %d", a.rows, a.cols);
        for (int r = 0; r < a.rows; ++r)
            for (int c = 0; c < a.cols; ++c) std::printf(" %.17g", a.ptr<double>(r)[c]);
        std::printf("\n");
    }
    sm::Mat t = sm::LoadData(argv[1], "TranslationVec");
    std::printf("%d %d %.17g\n", t.rows, t.cols, t.ptr<double>(0)[0]);
    sm::Mat none;
    return sm::LoadDataBatch(argv[1] + std::string(".missing"), none, none, none, none, none, none) ? 3 : 0;
}
''')
    exe = tmp_path / "ldb"
    subprocess.run(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    r = subprocess.run([str(exe), YML], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().splitlines()
    want = calib.load_data_batch(YML)
    for line, w in zip(lines[:6], want):
        vals = line.split()
        assert (int(vals[0]), int(vals[1])) == w.shape
        assert np.array_equal(np.array([float(v) for v in vals[2:]]).reshape(w.shape), w)
    assert lines[6].split()[:2] == ["3", "1"] and float(lines[6].split()[2]) == want[5][0, 0]
    assert "cannot open" in r.stderr
