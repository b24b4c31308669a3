"""CPU tests: the oracle (oracle/bm_oracle.c) against the committed golden vectors and
against itself (two independent formulations), plus the host-side helpers."""
import numpy as np
import pytest


def _cases(bm_expected):
    for k in bm_expected.files:
        if k.startswith("lr/"):
            continue
        p, r, D = k.split("/")
        yield k, p, int(r[1:]), int(D[1:])


def test_golden_middlebury_reproduced(oracle, gray, bm_expected):
    """Stored expected maps (getDisp restatement at generation time) == oracle now, both forms."""
    for k, p, r, D in _cases(bm_expected):
        L, R = gray[f"{p}/view1"], gray[f"{p}/view5"]
        fast = oracle.box_disp(L, R, r, D)
        assert np.array_equal(fast, bm_expected[k]), k
    # the literal loop nest (slow) on the singleFrame config (Caller.cpp:19) and cfg1
    for k in ("Art_/r5/D64", "Art/r3/D64"):
        p, r, D = k.split("/")
        lit = oracle.get_disp(gray[f"{p}/view1"], gray[f"{p}/view5"], int(r[1:]), int(D[1:]))
        assert np.array_equal(lit, bm_expected[k]), k


def test_golden_synthetic_reproduced(oracle, synth_expected):
    names = sorted({f.split("/")[0] for f in synth_expected.files})
    assert len(names) >= 8
    for n in names:
        seed, W, H, r, D = (int(v) for v in synth_expected[f"{n}/meta"])
        L, R = synth_expected[f"{n}/L"], synth_expected[f"{n}/R"]
        if n != "flat":
            gL, gR = oracle.synth_pair(seed, W, H, max(D, 16))
            assert np.array_equal(gL, L) and np.array_equal(gR, R), n
        assert np.array_equal(oracle.get_disp(L, R, r, D), synth_expected[f"{n}/disp"]), n


def test_flat_images_all_zero(oracle):
    """All-equal pair: every SAD is 0, d = 0 wins everywhere (strict <, Device.cu:57)."""
    img = np.full((20, 33), 200, np.uint8)
    assert (oracle.get_disp(img, img, 2, 16) == 0).all()


def test_threshold_no_match_is_zero(oracle):
    """Maximal-difference pair: no SAD < 50*win^2 -> dm stays -256 -> (uchar)0 (Device.cu:38,63)."""
    L = np.zeros((16, 40), np.uint8)
    R = np.full((16, 40), 255, np.uint8)
    d = oracle.get_disp(L, R, 1, 8)
    # only columns x < d have zero AD; x=0 can still match d>=1 windows partially -> compare forms
    assert np.array_equal(d, oracle.box_disp(L, R, 1, 8))


@pytest.mark.parametrize("shape,r,D", [((9, 7), 0, 1), ((13, 31), 2, 40), ((25, 18), 4, 64), ((6, 70), 3, 256)])
def test_two_formulations_agree_random(oracle, shape, r, D):
    rng = np.random.default_rng(hash((shape, r, D)) & 0xFFFF)
    L = rng.integers(0, 256, shape, dtype=np.uint8)
    R = rng.integers(0, 256, shape, dtype=np.uint8)
    assert np.array_equal(oracle.get_disp(L, R, r, D), oracle.box_disp(L, R, r, D))


@pytest.mark.parametrize("W,H,D,r", [(97, 40, 64, 3), (333, 77, 100, 5), (64, 20, 200, 0), (21, 13, 30, 2),
                                     (1, 5, 8, 1), (300, 3, 256, 7)])
def test_box_lr_probe_equals_volume_form(oracle, W, H, D, r):
    """The O(P)-memory, d-chunk-parallel LR oracle (full-size cfg5 checks) equals the volume form
    (ora_box_cost -> ora_right_wta -> ora_lr_check) bit for bit: chunk merges keep the smaller d."""
    L, R = oracle.synth_pair(W * 31 + H, W, H, min(D, 64))
    for a, b in zip(oracle.box_lr(L, R, r, D), oracle.box_lr_probe(L, R, r, D)):
        assert np.array_equal(a, b)


def test_key_slices_combine_by_min(oracle, gray):
    """Multi-GPU contract: min over d-slices of the packed keys == full-range key,
    and the finalised disparity equals the single-device map."""
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    disp, keys = oracle.box_disp(L, R, 5, 64, want_keys=True)
    for cuts in ([0, 64], [0, 16, 32, 48, 64], [0, 7, 9, 40, 64], [0, 1, 2, 3, 64]):
        parts = [oracle.box_keys_slice(L, R, 5, a, b) for a, b in zip(cuts[:-1], cuts[1:])]
        k = np.minimum.reduce(parts)
        assert np.array_equal(k, keys), cuts
        T = 50 * 11 * 11
        d = np.where((k >> 8) < T, k & 0xFF, 0).astype(np.uint8)
        assert np.array_equal(d, disp)


def test_lr_golden(oracle, gray, bm_expected):
    for k in [k for k in bm_expected.files if k.startswith("lr/") and k.endswith("/checked")]:
        _, p, r, D, _ = k.split("/")
        disp, rd, chk, mask = oracle.box_lr(gray[f"{p}/view1"], gray[f"{p}/view5"], int(r[1:]), int(D[1:]))
        assert np.array_equal(rd, bm_expected[k.replace("checked", "right")])
        assert np.array_equal(chk, bm_expected[k])
        assert np.array_equal(mask, bm_expected[k.replace("checked", "mask")])
        # properties of the StereoDisparity.cpp:136-147 rule
        assert ((chk == 0) | (chk == disp)).all()
        assert (chk[mask == 1] > 0).all()


def test_lr_rule_by_hand(oracle):
    """Tiny hand case of the occlusion rule: x-d<0 -> occluded, d==0 -> occluded, |d-dR|>1 -> occluded."""
    dl = np.array([[0, 1, 2, 3, 1, 2]], np.uint8)
    dr = np.array([[1, 1, 2, 0, 0, 4]], np.uint8)
    chk, mask = oracle.lr_check(dl, dr)
    # x=0 d=0 occ; x=1 d=1 -> dR(0)=1 ok; x=2 d=2 -> dR(0)=1 ok; x=3 d=3 -> dR(0)=1 occ;
    # x=4 d=1 -> dR(3)=0 ok (|1-0|=1); x=5 d=2 -> dR(3)=0 occ
    assert mask.tolist() == [[0, 1, 1, 0, 1, 0]]
    assert chk.tolist() == [[0, 1, 2, 0, 1, 0]]


def test_right_wta_clamp_rule(oracle):
    """GetRightMatchingCostFromLeft clamp (StereoHelper.cpp:170-175): for x+d >= W the right cost
    repeats C_R(x,d-1), which can never win a strict < — so dR(x) <= W-1-x."""
    rng = np.random.default_rng(3)
    L = rng.integers(0, 256, (12, 30), dtype=np.uint8)
    R = rng.integers(0, 256, (12, 30), dtype=np.uint8)
    cost = oracle.box_cost(L, R, 2, 24)
    rd = oracle.right_wta(cost)
    x = np.arange(30)[None, :]
    assert (rd <= (29 - x)).all()


def test_guided_golden(oracle, gray, guided_expected):
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    disp, best = oracle.guided_disp(L, R, 5, 64, 1e-4 * 255 * 255)
    assert np.array_equal(disp, guided_expected["Art_/r5/D64/disp"])
    np.testing.assert_allclose(best, guided_expected["Art_/r5/D64/best"], rtol=0, atol=1e-9)


def test_guided_large_eps_tends_to_box_mean(oracle):
    """eps -> inf: a -> 0, b -> mean(p), q -> mean(mean(p)) (a box-of-box filter)."""
    rng = np.random.default_rng(5)
    L = rng.integers(0, 256, (20, 24), dtype=np.uint8)
    R = rng.integers(0, 256, (20, 24), dtype=np.uint8)
    _, q, _ = oracle.guided_disp(L, R, 2, 4, 1e12, want_q=True)
    for d in range(4):
        ad = np.zeros((20, 24))
        ad[:, d:] = np.abs(L[:, d:].astype(int) - R[:, :24 - d].astype(int))
        m1 = np.empty_like(ad)
        m2 = np.empty_like(ad)
        oracle.lib().ora_box_mean_f64(ad.ctypes.data_as(oracle._f64p), 24, 20, 2, m1.ctypes.data_as(oracle._f64p))
        oracle.lib().ora_box_mean_f64(m1.ctypes.data_as(oracle._f64p), 24, 20, 2, m2.ctypes.data_as(oracle._f64p))
        np.testing.assert_allclose(q[d], m2, atol=1e-6)


@pytest.mark.parametrize("r", [1, 2, 3])
@pytest.mark.parametrize("W,H", [(1, 1), (2, 9), (7, 7), (37, 53)])
def test_median_restatement_matches_numpy(oracle, r, W, H):
    """ora_median_u8 (ctmf restatement) == an independent numpy edge-padded window median."""
    from numpy.lib.stride_tricks import sliding_window_view
    a = np.random.default_rng(W + 10 * H + r).integers(0, 256, (H, W), dtype=np.uint8)
    p = np.pad(a, r, mode="edge")
    k = 2 * r + 1
    w = sliding_window_view(p, (k, k)).reshape(H, W, k * k)
    want = np.sort(w, axis=2)[:, :, (k * k) // 2]
    assert np.array_equal(oracle.median(a, r), want)


def test_right_wta_float_matches_int_restatement(oracle, gray):
    """The float right-view WTA used for the guided LR check (numpy) == the C restatement of
    StereoHelper.cpp:131-180 on the integer box costs of a bundled pair."""
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    _, cost = oracle.box_disp(L, R, 4, 48, want_cost=True)
    rd_f, cr, best = oracle.right_wta_float(cost.astype(np.float64))
    assert np.array_equal(rd_f, oracle.right_wta(cost))
    H, W = L.shape
    u = W - 5                                    # clamp rule: C_R(u, d) = C_R(u, d-1) for u + d >= W
    assert np.array_equal(cr[10:, :, u], np.repeat(cr[4:5, :, u], 38, axis=0))
    assert np.array_equal(best, cr.min(axis=0))


def test_guided_probe_matches_volume_oracle(oracle):
    """The O(P) probe (full-size guided checks) == the volume restatement: best, the left cost at a
    map, and the right-view costs of StereoHelper.cpp:156-180 including the u + d >= W clamp."""
    L, R = oracle.synth_pair(5, 90, 40, 32)
    eps = 1e-4 * 255 * 255
    disp, q, best = oracle.guided_disp(L, R, 3, 32, eps, want_q=True)
    rd, cr, bestr = oracle.right_wta_float(q)
    probe_r = np.random.default_rng(0).integers(0, 32, L.shape).astype(np.uint8)
    out, b2, qL, bR, qR = oracle.guided_probe(L, R, 3, 32, eps, disp, probe_r)
    ys, xs = np.mgrid[0:40, 0:90]
    assert np.array_equal(out, disp) and np.array_equal(b2, best) and np.array_equal(bR, bestr)
    assert np.array_equal(qL, q[disp.astype(int), ys, xs])
    assert np.array_equal(qR, cr[probe_r.astype(int), ys, xs])


def test_st_tree_invariants(oracle):
    """The restated segment tree (SegmentTree.cpp:38-139) is a BFS-ordered spanning tree of the pixel grid:
    a permutation of the pixels, parents before children, each node's children a contiguous BFS run whose
    parent is that node, and tree edges between 4-neighbours only."""
    rng = np.random.default_rng(7)
    H, W = 30, 40
    L = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    L[5:20, 3:25] = 120                              # a flat segment: many equal-weight edges
    t = oracle.st_tree(L)
    P = H * W
    assert t["levels"] > 1
    assert sorted(t["node"].tolist()) == list(range(P)) and t["node"][0] == 0 and t["parent"][0] == -1
    for i in range(1, P):
        p = t["parent"][i]
        assert 0 <= p < i
        a, b = t["node"][i], t["node"][p]
        assert abs(a - b) in (1, W) and (abs(a - b) == W or a // W == b // W)
    for i in range(P):
        for z in range(t["nchild"][i]):
            c = t["first"][i] + z
            assert t["parent"][c] == i and t["pdist"][c] == t["cdist"][i, z]


def test_st_recovers_shift(oracle):
    """ST-1 on a textured pair shifted by 7 pixels: the disparity (scale 1) is 7 nearly everywhere
    right of the first columns (where x < 7 has no match)."""
    rng = np.random.default_rng(3)
    H, W, s = 80, 120, 7
    base = rng.integers(0, 256, (H, W + s, 3), dtype=np.uint8)
    L, R = base[:, :W].copy(), base[:, s:].copy()    # L(x) = R(x - s)
    d, levels = oracle.st_disp(L, R, 16, 1, 0.1)
    assert levels > 0
    assert (d[:, 12:] == s).mean() > 0.97


def test_st_right_cost_closed_form(oracle):
    """GetRightMatchingCostFromLeft (StereoHelper.cpp:156-180) as restated equals the closed form the GPU
    uses: C_R(y, x, d) = C(y, min(x + d, W - 1), min(d, W - 1 - x)), including W < D."""
    rng = np.random.default_rng(5)
    for W, H, D in ((50, 12, 16), (9, 4, 20)):
        L = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        R = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        c = oracle.st_cost(L, R, D)
        x, d = np.arange(W)[:, None], np.arange(D)[None, :]
        assert np.array_equal(oracle.st_right_cost(c), c[:, np.minimum(x + d, W - 1), np.minimum(d, W - 1 - x)])


def test_st2_pipeline_pieces(oracle):
    """ST-2's first left map is ST-1 with sigma = SIGMA_ONE (0.08) and scale 1 (StereoDisparity.cpp:115-119),
    its mask is the left-right check of the two first-pass maps (:129-147), the colour + depth tree spans
    the image, and the refined map recovers a known shift."""
    rng = np.random.default_rng(4)
    H, W, s = 60, 100, 6
    base = rng.integers(0, 256, (H, W + s, 3), dtype=np.uint8)
    L, R = base[:, :W].copy(), base[:, s:].copy()
    out, levels, l1, r1, mk = oracle.st2_disp(L, R, 16, 1, 0.1)
    assert levels > 0
    st1, _ = oracle.st_disp(L, R, 16, 1, 0.08)
    assert np.array_equal(l1, st1)
    xs = np.arange(W)[None, :].repeat(H, 0)
    u = xs - l1.astype(int)
    ok = u >= 0
    dr = np.where(ok, r1[np.arange(H)[:, None], np.clip(u, 0, W - 1)], 0).astype(int)
    want = ok & (l1 != 0) & (np.abs(l1.astype(int) - dr) <= 1)
    assert np.array_equal(mk.astype(bool), want)
    t = oracle.st_tree_depth(L, l1, mk, 16)
    assert t["levels"] > 0 and sorted(t["node"].tolist()) == list(range(H * W))
    assert (out[:, 12:] == s).mean() > 0.97


@pytest.mark.parametrize("H,W,r,D", [(20, 33, 2, 16), (17, 9, 3, 12), (5, 40, 0, 40), (30, 50, 5, 8), (6, 7, 9, 10)])
def test_get_all_sad_two_restatements(oracle, H, W, r, D):
    """getAllSAD (BlockMatching.cpp:191-261): the literal loop nest (ora_get_all_sad) equals the
    separable box-sum volume (ora_box_cost) transposed to pixel-major, truncated to uchar, with 255
    where col + d > cols — including W < D and r larger than the frame."""
    rng = np.random.default_rng(H * W + r * 31 + D)
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    R = rng.integers(0, 256, (H, W), dtype=np.uint8)
    got = oracle.get_all_sad(L, R, r, D)
    low = (oracle.box_cost(L, R, r, D).transpose(1, 2, 0) & 0xFF).astype(np.uint8)
    x = np.arange(W)[None, :, None]
    d = np.arange(D)[None, None, :]
    assert np.array_equal(got, np.where(x + d > W, 255, low).astype(np.uint8))


def test_get_all_sad_golden_pair(oracle, gray):
    """On the bundled Art_ pair at singleFrame's configuration (r = 5, D = 64): every valid entry is
    the low byte of the box SAD, every entry with col + d > cols is 255."""
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    vol = oracle.get_all_sad(L, R, 5, 64)
    full = oracle.box_cost(L, R, 5, 64).transpose(1, 2, 0)
    x = np.arange(L.shape[1])[None, :, None]
    d = np.arange(64)[None, None, :]
    valid = np.broadcast_to(x + d <= L.shape[1], vol.shape)
    assert np.array_equal(vol[valid], (full[valid] & 0xFF).astype(np.uint8))
    assert (vol[~valid] == 255).all()


def test_device_cu_literal_two_restatements_and_survey_counts(oracle, gray):
    """Device.cu's literal map (launch geometry included, Device.cu:191-194, 231-233, 253): the loop nest
    over the (8, 10, D) x (32, 32) grid (ora_device_cu_literal) equals the numpy integral-image
    formulation, equals getDisp at 320x256, and differs from getDisp on exactly the pixel counts
    SURVEY §8a a1 measured independently at r = 4, D = 64: Art 85,893, Books 83,551 of 171,310."""
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    lit = oracle.device_cu_literal(L, R, 5, 64)
    assert np.array_equal(lit, oracle.get_disp(L, R, 5, 64))
    for p, n in (("Art", 85893), ("Books", 83551)):
        L, R = gray[f"{p}/view1"], gray[f"{p}/view5"]
        lit = oracle.device_cu_literal(L, R, 4, 64)
        assert np.array_equal(lit, oracle.device_cu_literal_integral(L, R, 4, 64))
        assert int((lit != oracle.box_disp(L, R, 4, 64)).sum()) == n


def test_device_cu_literal_golden_and_edges(oracle, gray):
    import os
    from conftest import GOLDEN
    exp = np.load(os.path.join(GOLDEN, "device_cu_expected.npz"))
    L, R = gray["Dolls/view1"], gray["Dolls/view5"]
    assert np.array_equal(oracle.device_cu_literal_integral(L, R, 0, 32), exp["Dolls/r0/D32"])
    A, B = oracle.synth_pair(5, 1030, 256, 32)
    assert not oracle.device_cu_literal(A, B, 2, 32).any()          # cols > 1024: the launch fails
    with pytest.raises(ValueError):
        oracle.device_cu_literal(A[:, :319], B[:, :319], 2, 32)     # below the grid's 320 x 256
    with pytest.raises(ValueError):
        oracle.device_cu_literal(A[:255], B[:255], 2, 32)
