"""The segment tree's host builder (csrc/bm_segtree_host.h: counting / radix edge sorts, Kruskal with
Felzenszwalb's threshold and the cross-segment penalty, BFS) against the C restatement of the
reference (oracle/st_oracle.c: qsort with edge::operator<), on the CPU: identical BFS order, parents
and tree distances, for colour trees (ST-1, ST-2's first pass) and colour + depth trees (ST-2)."""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def shim(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("g++ absent")
    out = str(tmp_path_factory.mktemp("st") / "libst_host_shim.so")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-shared", "-fPIC", "-o", out,
                    os.path.join(ROOT, "tests", "native", "st_host_shim.cpp")], check=True)
    L = ctypes.CDLL(out)
    u8, i32 = ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_int)
    L.st_host_tree_u8.argtypes = [u8, u8, ctypes.c_int, ctypes.c_int, ctypes.c_float, i32, i32, u8]
    L.st_host_tree_depth.argtypes = [u8, u8, u8, u8, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                     i32, i32, u8]
    L.st_host_lists_from_marks_check.argtypes = [u8, u8, u8, u8, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                 ctypes.c_int, ctypes.c_float]
    return L


def _p(a, t):
    return a.ctypes.data_as(ctypes.POINTER(t))


def colour_weights(oracle, bgr):
    """CColorWeight on the 3x3-median guide (ctmf r = 1 per channel): wr[p] = edge (p, p+1), wu[p] =
    edge (p, p-W)."""
    g = np.stack([oracle.median(np.ascontiguousarray(bgr[:, :, c]), 1) for c in range(3)], -1).astype(np.int16)
    H, W = g.shape[:2]
    wr = np.zeros((H, W), np.uint8)
    wu = np.zeros((H, W), np.uint8)
    wr[:, :-1] = np.abs(g[:, :-1] - g[:, 1:]).max(-1)
    wu[1:] = np.abs(g[1:] - g[:-1]).max(-1)
    return wr, wu


def host_tree(shim, wr, wu, disp=None, mask=None, level=60):
    H, W = wr.shape
    P = W * H
    node, parent, pdist = np.empty(P, np.int32), np.empty(P, np.int32), np.empty(P, np.uint8)
    if disp is None:
        lv = shim.st_host_tree_u8(_p(wr, ctypes.c_uint8), _p(wu, ctypes.c_uint8), W, H, 1200.0,
                                  _p(node, ctypes.c_int), _p(parent, ctypes.c_int), _p(pdist, ctypes.c_uint8))
    else:
        d, m = np.ascontiguousarray(disp, np.uint8), np.ascontiguousarray(mask, np.uint8)
        lv = shim.st_host_tree_depth(_p(wr, ctypes.c_uint8), _p(wu, ctypes.c_uint8), _p(d, ctypes.c_uint8),
                                     _p(m, ctypes.c_uint8), W, H, level, 1200.0, _p(node, ctypes.c_int),
                                     _p(parent, ctypes.c_int), _p(pdist, ctypes.c_uint8))
    return lv, node, parent, pdist


def images(seed, H, W):
    rng = np.random.default_rng(seed)
    L = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    L[H // 4: H // 2, W // 5: W // 2] = 90                      # flat: long runs of equal weights
    L[H // 2:, : W // 3] = (L[H // 2:, : W // 3] // 64) * 64    # quantised: many ties
    return L


@pytest.mark.parametrize("seed,H,W", [(1, 40, 57), (2, 1, 33), (3, 23, 2), (4, 64, 90)])
def test_colour_tree_matches_oracle(oracle, shim, seed, H, W):
    L = images(seed, H, W)
    wr, wu = colour_weights(oracle, L)
    lv, node, parent, pdist = host_tree(shim, wr, wu)
    t = oracle.st_tree(L)
    assert lv == t["levels"]
    assert np.array_equal(node, t["node"]) and np.array_equal(parent, t["parent"])
    assert np.array_equal(pdist, t["pdist"])


@pytest.mark.parametrize("seed,H,W,level", [(5, 40, 57, 60), (6, 30, 80, 16), (7, 1, 50, 9), (8, 64, 90, 128)])
def test_depth_tree_matches_oracle(oracle, shim, seed, H, W, level):
    """Float weights 0.5 |d0 - d1| / level + 0.5 c / 255 where both ends are in the mask, else c / 255:
    ordered by the 4-pass radix sort on their bits, vs the oracle's qsort on the floats."""
    rng = np.random.default_rng(seed)
    L = images(seed, H, W)
    disp = rng.integers(0, level, (H, W), dtype=np.uint8)
    disp[: H // 2] = disp[: H // 2] // 4 * 4                     # ties in |d0 - d1| as well
    mask = (rng.random((H, W)) < 0.7).astype(np.uint8)
    wr, wu = colour_weights(oracle, L)
    lv, node, parent, pdist = host_tree(shim, wr, wu, disp, mask, level)
    t = oracle.st_tree_depth(L, disp, mask, level)
    assert lv == t["levels"]
    assert np.array_equal(node, t["node"]) and np.array_equal(parent, t["parent"])
    assert np.array_equal(pdist, t["pdist"])


@pytest.mark.parametrize("seed,H,W", [(1, 40, 57), (2, 1, 33), (3, 23, 2), (4, 64, 90)])
@pytest.mark.parametrize("depth", [0, 1])
def test_lists_from_marks(oracle, shim, seed, H, W, depth):
    """The device path's neighbour lists (st_adj_kernel) restated on segment_passes' per-edge marks:
    identical to the lists segment_lists appends during the second pass, for the colour tree and the
    colour + depth tree (float weights, penalty bit, scale 255)."""
    L = images(seed, H, W)
    wr, wu = colour_weights(oracle, L)
    rng = np.random.default_rng(seed)
    d = rng.integers(0, 60, (H, W), dtype=np.uint8)
    m = (rng.random((H, W)) < 0.7).astype(np.uint8)
    bad = shim.st_host_lists_from_marks_check(_p(wr, ctypes.c_uint8), _p(wu, ctypes.c_uint8), _p(d, ctypes.c_uint8),
                                              _p(m, ctypes.c_uint8), W, H, 60, depth, 1200.0)
    assert bad == 0
