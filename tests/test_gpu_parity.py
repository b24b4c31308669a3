"""GPU parity tests: the HIP path through the C ABI vs the oracle / golden fixtures.

Integer SAD/WTA work is compared bit-exact.  Sizes: the bundled Middlebury
pairs and the synthetic edge cases at their own size, 1080p and 4K synthetic pairs against the
fast oracle formulation (ora_box_disp, O(P*D)).
"""
import numpy as np
import pytest
from fuzz_util import fuzz_pair

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sm():
    import gpu_stereo_matching_amd as sm
    return sm


@pytest.fixture(scope="module")
def matcher(sm):
    m = sm.BlockMatcher(0, 3840, 2160, 256)
    yield m
    m.close()


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available()
    return t


def test_library_is_hip(sm):
    assert "gfx950" in sm.version()


def test_middlebury_golden_host_path(matcher, gray, bm_expected):
    for k in bm_expected.files:
        if k.startswith("lr/"):
            continue
        p, r, D = k.split("/")
        got = matcher.match(gray[f"{p}/view1"], gray[f"{p}/view5"], int(r[1:]), int(D[1:]))
        assert np.array_equal(got, bm_expected[k]), f"{k}: {int((got != bm_expected[k]).sum())} px differ"


def test_reference_entry_point(sm, gray, bm_expected):
    """blockMatching_gpu(g1, g2, 5, 64) as called at Caller.cpp:19."""
    got = sm.blockMatching_gpu(gray["Art_/view1"], gray["Art_/view5"], 5, 64)
    assert np.array_equal(got, bm_expected["Art_/r5/D64"])


def test_synthetic_edge_cases(matcher, synth_expected):
    names = sorted({f.split("/")[0] for f in synth_expected.files})
    for n in names:
        _, W, H, r, D = (int(v) for v in synth_expected[f"{n}/meta"])
        got = matcher.match(synth_expected[f"{n}/L"], synth_expected[f"{n}/R"], r, D)
        assert np.array_equal(got, synth_expected[f"{n}/disp"]), n


@pytest.mark.parametrize("r", list(range(0, 17)))
def test_every_radius(matcher, oracle, r):
    """r 0..7: packed u16 window sums; 8..15: the same kernel with u32 window halves; 16: generic."""
    rng = np.random.default_rng(100 + r)
    H, W, D = 45, 150, 40
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    R = np.roll(L, -7, axis=1) ^ rng.integers(0, 8, (H, W), dtype=np.uint8)
    assert np.array_equal(matcher.match(L, R, r, D), oracle.box_disp(L, R, r, D))


@pytest.mark.parametrize("D", [1, 2, 7, 8, 9, 15, 16, 17, 63, 64, 65, 100, 127, 128, 129, 200, 255, 256])
def test_every_disparity_count(matcher, oracle, D):
    L, R = oracle.synth_pair(D, 301, 37, max(D, 16))
    assert np.array_equal(matcher.match(L, R, 3, D), oracle.box_disp(L, R, 3, D))


@pytest.mark.parametrize("W,H", [(1, 1), (1, 50), (50, 1), (3, 3), (10, 200), (63, 31), (64, 32), (65, 33),
                                 (127, 9), (513, 67)])
def test_ragged_and_tiny_frames(matcher, oracle, W, H):
    rng = np.random.default_rng(W * 1000 + H)
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    R = rng.integers(0, 256, (H, W), dtype=np.uint8)
    for r, D in ((0, 5), (2, 64), (5, 256)):
        assert np.array_equal(matcher.match(L, R, r, D), oracle.box_disp(L, R, r, D)), (r, D)


def test_extreme_values(matcher, oracle):
    """Saturated inputs: maximal window sums (255*win^2) must not wrap the packed u16 sums."""
    H, W = 40, 120
    for r in (5, 7):
        L = np.zeros((H, W), np.uint8)
        R = np.full((H, W), 255, np.uint8)
        assert np.array_equal(matcher.match(L, R, r, 64), oracle.box_disp(L, R, r, 64))
        L = np.full((H, W), 255, np.uint8)
        R = np.zeros((H, W), np.uint8)
        R[:, ::3] = 255
        assert np.array_equal(matcher.match(L, R, r, 64), oracle.box_disp(L, R, r, 64))


def test_pitched_host_input(sm, matcher, oracle, gray):
    """Row pitch > width (a Mat ROI): the C ABI's `pitch` argument."""
    import ctypes
    L, R = gray["Art/view1"], gray["Art/view5"]
    H, W = L.shape
    P = W + 37
    Lp = np.zeros((H, P), np.uint8)
    Rp = np.zeros((H, P), np.uint8)
    Lp[:, :W] = L
    Rp[:, :W] = R
    out = np.full((H, W + 5), 7, np.uint8)
    rc = matcher._lib.sm_block_match_u8(matcher._h, Lp.ctypes.data, Rp.ctypes.data, W, H, P, 4, 64, 0,
                                        out.ctypes.data, W + 5)
    assert rc == 0
    assert np.array_equal(out[:, :W], oracle.box_disp(L, R, 4, 64))
    assert (out[:, W:] == 7).all()


def test_device_path_batched(matcher, oracle, torch):
    B, H, W, D, r = 3, 120, 333, 96, 4
    pairs = [oracle.synth_pair(50 + i, W, H, D) for i in range(B)]
    Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    out = matcher.match_device(Lt, Rt, r, D)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for i in range(B):
        assert np.array_equal(got[i], oracle.box_disp(pairs[i][0], pairs[i][1], r, D)), i


def test_1080p_d128_synthetic(matcher, oracle, torch):
    """The bench workload (cfg3 geometry) at full size."""
    L, R = oracle.synth_pair(1234, 1920, 1080, 128)
    want = oracle.box_disp(L, R, 5, 128)
    out = matcher.match_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda(), 5, 128)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), want)
    # size-independent property: on the banded synthetic pair most pixels recover ground truth
    from gpu_stereo_matching_amd.synth import ground_truth_rows
    gt = ground_truth_rows(1080, 128)[:, None]
    acc = (want[:, 200:] == gt).mean()
    assert acc > 0.95


def test_1080p_d256_and_4k_d192(matcher, oracle, torch):
    for (W, H, D, seed) in ((1920, 1080, 256, 1234), (3840, 2160, 192, 4321)):
        L, R = oracle.synth_pair(seed, W, H, D)
        want = oracle.box_disp(L, R, 5, D)
        out = matcher.match_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda(), 5, D)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), want), (W, H, D)


def test_cfg5_box_lr_full_size(matcher, oracle, torch):
    """BASELINE configs[4]'s frame size as written (3840x2160, d_max = 192, r = 5) through box + LR,
    host call and batched device call: left map, right map (STMatching's C_R rule,
    StereoHelper.cpp:131-180), checked map and mask bit-exact with the O(P) oracle."""
    W, H, D, r = 3840, 2160, 192, 5
    L, R = oracle.synth_pair(4321, W, H, D)
    disp_o, rd_o, chk_o, mask_o = oracle.box_lr_probe(L, R, r, D)
    assert np.array_equal(matcher.match(L, R, r, D), disp_o)
    chk, rd, mask = matcher.match_lr(L, R, r, D)
    assert np.array_equal(rd, rd_o), f"right: {int((rd != rd_o).sum())} pixels differ"
    assert np.array_equal(chk, chk_o) and np.array_equal(mask, mask_o)
    Lt = torch.from_numpy(np.stack([L, R])).cuda()
    Rt = torch.from_numpy(np.stack([R, L])).cuda()
    out = matcher.match_device(Lt, Rt, r, D, lr_check=True)
    torch.cuda.synchronize()
    assert np.array_equal(out[0].cpu().numpy(), chk_o)


def test_lr_golden(matcher, gray, bm_expected):
    for k in [k for k in bm_expected.files if k.startswith("lr/") and k.endswith("/checked")]:
        _, p, r, D, _ = k.split("/")
        chk, rd, mask = matcher.match_lr(gray[f"{p}/view1"], gray[f"{p}/view5"], int(r[1:]), int(D[1:]))
        assert np.array_equal(rd, bm_expected[k.replace("checked", "right")]), k
        assert np.array_equal(chk, bm_expected[k]), k
        assert np.array_equal(mask, bm_expected[k.replace("checked", "mask")]), k
        # the flag form returns the same checked map
        chk2 = matcher.match(gray[f"{p}/view1"], gray[f"{p}/view5"], int(r[1:]), int(D[1:]), lr_check=True)
        assert np.array_equal(chk2, chk)


@pytest.mark.parametrize("r,D", [(0, 8), (1, 16), (2, 1), (3, 37), (4, 64), (5, 128), (6, 256), (7, 100), (8, 48),
                                 (5, 2), (5, 129), (11, 64), (15, 256), (16, 40)])
def test_lr_random(matcher, oracle, r, D):
    """r <= 15: right view fused into the matching pass (rpart + reduce); r = 16: mirrored second pass."""
    L, R = oracle.synth_pair(r * 7 + D, 257, 61, max(D, 16))
    disp, rd, chk, mask = oracle.box_lr(L, R, r, D)
    c, rr, mm = matcher.match_lr(L, R, r, D)
    assert np.array_equal(rr, rd), (r, D)
    assert np.array_equal(c, chk) and np.array_equal(mm, mask), (r, D)


@pytest.mark.parametrize("r", [8, 11, 15])
@pytest.mark.parametrize("D", [64, 256])
def test_wide_radius_fast_path(matcher, oracle, torch, r, D):
    """Radius 8..15 (the reference's SADWindowSize is unbounded, Device.cu:46-56) on the fused kernel:
    window sums up to 31^2 * 255 need the u32 halves; bit-exact with the separable oracle, host and
    batched device path, plain and with the LR check."""
    L, R = oracle.synth_pair(1000 + 10 * r + D, 333, 150, D)
    want = oracle.box_disp(L, R, r, D)
    assert np.array_equal(matcher.match(L, R, r, D), want), (r, D)
    L2, R2 = oracle.synth_pair(2000 + r, 333, 150, D)
    Lt = torch.from_numpy(np.stack([L, L2])).cuda()
    Rt = torch.from_numpy(np.stack([R, R2])).cuda()
    out = matcher.match_device(Lt, Rt, r, D)
    torch.cuda.synchronize()
    assert np.array_equal(out[0].cpu().numpy(), want) and np.array_equal(out[1].cpu().numpy(),
                                                                          oracle.box_disp(L2, R2, r, D))
    _, rd, chk, mask = oracle.box_lr(L, R, r, D)
    c, rr, mm = matcher.match_lr(L, R, r, D)
    assert np.array_equal(rr, rd) and np.array_equal(c, chk) and np.array_equal(mm, mask), (r, D)


def test_wide_radius_saturated(matcher, oracle):
    """r = 15 on 0/255 images: window sums reach 961 * 255, the largest the u32 halves carry."""
    rng = np.random.default_rng(15)
    L = (rng.integers(0, 2, (96, 200)) * 255).astype(np.uint8)
    R = 255 - L
    for D in (16, 100):
        assert np.array_equal(matcher.match(L, R, 15, D), oracle.box_disp(L, R, 15, D))


@pytest.mark.parametrize("W,H,r,D", [(40, 30, 3, 64), (53, 7, 5, 64), (3, 5, 1, 8), (1000, 33, 5, 256), (600, 97, 7, 192)])
def test_lr_shapes(matcher, oracle, W, H, r, D):
    """Narrow (W < TW, W < D), single-tile, ragged and tall shapes through the fused right view."""
    L, R = oracle.synth_pair(W * 3 + H, W, H, max(D, 16))
    disp, rd, chk, mask = oracle.box_lr(L, R, r, D)
    c, rr, mm = matcher.match_lr(L, R, r, D)
    assert np.array_equal(rr, rd) and np.array_equal(c, chk) and np.array_equal(mm, mask), (W, H, r, D)


def test_lr_device_batch(matcher, oracle, torch):
    W, H, D, r, B = 301, 70, 64, 4, 3
    pairs = [oracle.synth_pair(900 + b, W, H, D) for b in range(B)]
    Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    out = matcher.match_device(Lt, Rt, r, D, lr_check=True)
    torch.cuda.synchronize()
    for b in range(B):
        _, _, chk, _ = oracle.box_lr(pairs[b][0], pairs[b][1], r, D)
        assert np.array_equal(out[b].cpu().numpy(), chk), b


@pytest.mark.parametrize("cuts", [[0, 128], [0, 64, 128], [0, 16, 32, 48, 64, 80, 96, 112, 128], [0, 5, 77, 128]])
def test_slice_keys_min_equals_full(matcher, oracle, torch, cuts):
    """The multi-GPU d-slice contract on one device: MIN over slice key maps == single pass."""
    L, R = oracle.synth_pair(77, 400, 90, 128)
    Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    disp, keys = oracle.box_disp(L, R, 5, 128, want_keys=True)
    parts = [matcher.slice_keys_device(Lt, Rt, 5, a, b) for a, b in zip(cuts[:-1], cuts[1:])]
    k = parts[0].clone()
    for p in parts[1:]:
        k = torch.minimum(k, p)
    torch.cuda.synchronize()
    assert np.array_equal(k.cpu().numpy().view(np.uint32), keys)
    for (a, b), p in zip(zip(cuts[:-1], cuts[1:]), parts):
        assert np.array_equal(p.cpu().numpy().view(np.uint32), oracle.box_keys_slice(L, R, 5, a, b)), (a, b)
    d = matcher.keys_to_disp_device(k, 5)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), disp)


@pytest.mark.parametrize("G,agg,lr,med", [(2, "box", False, False), (8, "box", False, False), (3, "box", True, False),
                                          (4, "guided", False, False), (5, "box", True, True), (3, "box", False, True),
                                          (3, "guided", True, True), (7, "guided", True, False)])
def test_rowband_bands_equal_full_frame(matcher, torch, G, agg, lr, med):
    """The row-band partition's per-rank compute (sharding.band_disparity), run band by band on one
    GPU on its own stream, reassembles the single-pass map bit for bit, the guided filter included:
    band inputs start on the frame's 32-row tile grid with a halo of max(2r, 16) (+3 with the
    median), the C group's rule, so every kept row sees the full frame's summation order."""
    from gpu_stereo_matching_amd import sharding
    from oracle import oracle as O
    L, R = O.synth_pair(555, 700, 203, 64)
    Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    full = matcher.match_device(Lt, Rt, 5, 64, agg=agg, lr_check=lr, median=med)
    side = torch.cuda.Stream()
    parts = []
    for k in range(G):
        y0, y1 = sharding.band_rows(203, k, G)
        if y1 > y0:
            parts.append(sharding.band_disparity(matcher, Lt, Rt, 5, 64, y0, y1, agg, lr, stream=side, median=med))
    got = torch.cat(parts)
    torch.cuda.synchronize()
    assert torch.equal(got, full)


def test_null_stream_and_stream_sync(sm, matcher, oracle, torch):
    """NULL means the default stream for sm_match_device AND for sm_stream_sync, so a C
    caller that passes NULL to both reads a finished map."""
    W, H, D, r = 640, 360, 128, 5
    L, R = oracle.synth_pair(31, W, H, D)
    want = oracle.box_disp(L, R, r, D)
    Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    out = torch.full((H, W), 7, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    for flags in (sm.SM_AGG_BOX, sm.SM_AGG_BOX | sm.SM_LR_CHECK):
        rc = matcher._lib.sm_match_device(matcher._h, Lt.data_ptr(), Rt.data_ptr(), W, H, W, 1, H * W, r, D, flags,
                                          out.data_ptr(), W, H * W, None)
        assert rc == 0
        assert matcher._lib.sm_stream_sync(matcher._h, None) == 0
        host = out.cpu().numpy()
        if flags == sm.SM_AGG_BOX:
            assert np.array_equal(host, want)
        else:
            assert np.array_equal(host, oracle.box_lr(L, R, r, D)[2])


def test_two_streams_one_handle(matcher, oracle, torch):
    """device calls on one handle from two streams share the handle's LR / median
    workspace; the second pass waits for the first, so both maps are exact."""
    W, H, D, r = 900, 400, 128, 5
    pairs = [oracle.synth_pair(61 + i, W, H, D) for i in range(2)]
    want = [oracle.box_lr(L, R, r, D)[2] for L, R in pairs]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    dev = [(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()) for L, R in pairs]
    torch.cuda.synchronize()
    for _ in range(3):
        outs = [matcher.match_device(dev[0][0], dev[0][1], r, D, lr_check=True, median=True, stream=s1),
                matcher.match_device(dev[1][0], dev[1][1], r, D, lr_check=True, median=True, stream=s2)]
        torch.cuda.synchronize()
        for o, (L, R) in zip(outs, pairs):
            ref = matcher.match_lr(L, R, r, D, median=True)[0]
            assert np.array_equal(o.cpu().numpy(), ref)
    outs = [matcher.match_device(dev[i][0], dev[i][1], r, D, lr_check=True, stream=(s1, s2)[i]) for i in range(2)]
    torch.cuda.synchronize()
    for o, w in zip(outs, want):
        assert np.array_equal(o.cpu().numpy(), w)


@pytest.mark.parametrize("r", [20, 40])
def test_two_streams_one_handle_wide(matcher, oracle, torch, r):
    """a plain box pass at r 38..127 (no LR, no median) writes the separable path's V planes into the
    handle's volume workspace and may grow it; two streams on one handle are ordered, so both maps are
    exact.  The second pair has the larger D, so its pass grows the workspace behind the first.  r = 20 runs the
    strip kernel (no workspace) under the same ordering."""
    cfg = [(700, 300, 64, 71), (900, 400, 160, 72)]
    pairs = [oracle.synth_pair(seed, W, H, D) for W, H, D, seed in cfg]
    want = [oracle.box_disp(L, R, r, D) for (L, R), (_, _, D, _) in zip(pairs, cfg)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    dev = [(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()) for L, R in pairs]
    torch.cuda.synchronize()
    for _ in range(3):
        outs = [matcher.match_device(dev[i][0], dev[i][1], r, cfg[i][2], stream=(s1, s2)[i]) for i in range(2)]
        torch.cuda.synchronize()
        for o, w in zip(outs, want):
            assert np.array_equal(o.cpu().numpy(), w)


def test_out_tensor_validation(matcher, torch):
    """a caller-supplied output of the wrong shape / dtype / device is a ValueError, never
    an out-of-bounds device write."""
    Lt = torch.zeros((64, 96), dtype=torch.uint8, device="cuda")
    for bad in (torch.empty((63, 96), dtype=torch.uint8, device="cuda"),
                torch.empty((64, 96), dtype=torch.int32, device="cuda"),
                torch.empty((64, 96), dtype=torch.uint8),
                torch.empty((96, 64), dtype=torch.uint8, device="cuda").t()):
        with pytest.raises(ValueError):
            matcher.match_device(Lt, Lt, 2, 16, out_t=bad)
    k = torch.zeros((64, 96), dtype=torch.int32, device="cuda")
    with pytest.raises(ValueError):
        matcher.keys_to_disp_device(k, 2, out_t=torch.empty((10,), dtype=torch.uint8, device="cuda"))
    with pytest.raises(ValueError):
        matcher.guided_keys_to_disp_device(k.float())


def test_error_codes(sm, matcher):
    L = np.zeros((10, 10), np.uint8)
    with pytest.raises(sm.SMError) as e:
        matcher.match(L, L, 1, 0)
    assert e.value.code == 1
    with pytest.raises(sm.SMError) as e:
        matcher.match(L, L, 1, 257)
    assert e.value.code == 1
    small = sm.BlockMatcher(0, 16, 16, 32)
    with pytest.raises(sm.SMError) as e:
        small.match(np.zeros((17, 16), np.uint8), np.zeros((17, 16), np.uint8), 1, 8)
    assert e.value.code == 5
    small.close()


def test_error_codes_side_entries(sm, torch):
    """Argument and capacity checks of the non-matching entry points, and recovery afterwards."""
    small = sm.BlockMatcher(0, 32, 16, 32)
    with pytest.raises(sm.SMError) as e:                       # capacity
        small.cvt_color(np.zeros((17, 32, 3), np.uint8))
    assert e.value.code == 5
    with pytest.raises(sm.SMError) as e:
        small.remap(np.zeros((16, 33), np.uint8), np.zeros((16, 33), np.float32), np.zeros((16, 33), np.float32))
    assert e.value.code == 5
    x = torch.zeros((8, 8), dtype=torch.uint8, device="cuda")
    for bad_r in (0, 4):
        with pytest.raises(sm.SMError) as e:
            small.median_device(x, bad_r)
        assert e.value.code == 1
    lib = small._lib
    assert lib.sm_median_u8_device(small._h, None, 8, 8, 8, 1, x.data_ptr(), 8, None) == 1
    assert lib.sm_remap_u8(small._h, None, 8, 8, 8, None, None, 8, None, 8) == 1
    assert b"remap" in lib.sm_last_error_string()
    # the handle still works after the failures
    L = np.random.default_rng(0).integers(0, 256, (16, 32), dtype=np.uint8)
    assert small.match(L, L, 1, 8).shape == (16, 32)
    small.close()


def test_stage_timings(sm, gray, oracle):
    """SM_PARAM_STAGE_TIMING: auto (default) records the upload / match / download split from the
    first sm_last_stage_ms read on (the drop-in call skips the two hipEvent markers until someone
    reads the split); 1 always; 0 never (the split reads 0).  Maps never change."""
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    with sm.BlockMatcher(0, 640, 480, 256) as m:
        want = m.match(L, R, 5, 64)
        assert m.stage_ms() == (0.0, 0.0, 0.0)      # auto: not recorded before the first read
        assert np.array_equal(m.match(L, R, 5, 64), want)
        u, c, d = m.stage_ms()                       # armed by the first read
        assert u > 0 and c > 0 and d > 0
        m.set_stage_timing(False)
        assert np.array_equal(m.match(L, R, 5, 64), want)
        assert m.stage_ms() == (0.0, 0.0, 0.0)
        m.set_stage_timing(True)
        m.match(L, R, 5, 64)
        assert min(m.stage_ms()) > 0
        m.set_stage_timing("auto")                   # back to the default: unarmed again
        m.match(L, R, 5, 64)
        assert m.stage_ms() == (0.0, 0.0, 0.0)
        m.match(L, R, 5, 64)                         # armed by that read
        assert min(m.stage_ms()) > 0
    assert np.array_equal(want, oracle.box_disp(L, R, 5, 64))


@pytest.mark.parametrize("pair,r,D", [("Art_", 5, 64), ("Art", 4, 64), ("Books", 3, 64), ("Dolls", 9, 64)])
def test_all_sad_golden_pairs(matcher, gray, oracle, pair, r, D):
    """getAllSAD (BlockMatching.cpp:191-261) bit-exact with its literal restatement ora_get_all_sad:
    pixel-major [p*D + d], uchar truncation of every window SAD, 255 where col + d > cols.  r <= 7
    runs AD volume -> u16 SAD volume -> transpose; r = 9 the direct kernel."""
    L, R = gray[f"{pair}/view1"], gray[f"{pair}/view5"]
    got = matcher.all_sad(L, R, r, D)
    assert got.shape == (*L.shape, D)
    assert np.array_equal(got, oracle.get_all_sad(L, R, r, D))


@pytest.mark.parametrize("W,H,r,D", [(1, 1, 0, 1), (5, 3, 1, 7), (40, 9, 0, 64), (65, 33, 7, 129), (33, 50, 2, 256),
                                     (200, 17, 8, 30), (31, 12, 15, 20), (4100, 3, 2, 9)])
def test_all_sad_shapes(matcher, oracle, torch, W, H, r, D):
    """getAllSAD on odd shapes: W < D (most entries 255), D = 1 / 256, r = 0 and r up to 15 (the
    direct kernel), W > 4096 (beyond the AD-volume kernel: the direct kernel); host and device forms
    equal."""
    rng = np.random.default_rng(W * 7 + H * 13 + r + D)
    L = rng.integers(0, 256, (H, W), dtype=np.uint8)
    R = rng.integers(0, 256, (H, W), dtype=np.uint8)
    want = oracle.get_all_sad(L, R, r, D)
    if W <= matcher.max_width:   # the host form stages through the handle's frames
        assert np.array_equal(matcher.all_sad(L, R, r, D), want)
    Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    out = matcher.all_sad_device(Lt, Rt, r, D)
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), want)


def test_all_sad_1080p(matcher, torch):
    """getAllSAD at 1080p D=128 r=5 (265 MB volume): the device form against the u16 SAD volume's low
    bytes (itself checked against the oracle in test_sad_volume), with the 255 rule."""
    from gpu_stereo_matching_amd import synth
    L, R = synth.synth_pair(1234, 1920, 1080, 128)
    Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    vol = matcher.sad_volume_device(Lt, Rt, 5, 128)
    allsad = matcher.all_sad_device(Lt, Rt, 5, 128)
    low = (vol.to(torch.int32) & 0xFF).permute(1, 2, 0)
    x = torch.arange(1920, device="cuda").view(1, 1920, 1)
    d = torch.arange(128, device="cuda").view(1, 1, 128)
    want = torch.where(x + d > 1920, torch.full_like(low, 255), low).to(torch.uint8)
    torch.cuda.synchronize()
    assert torch.equal(allsad, want)


def test_frame_stream_pipeline(matcher, oracle, torch):
    """FrameStream (copy/compute overlap on two streams, double-buffered pinned slots) returns every
    batch, in order, identical to the oracle."""
    from gpu_stereo_matching_amd.pipeline import FrameStream
    B, W, H, D, r = 3, 200, 64, 32, 3
    fs = FrameStream(matcher, B, W, H, r, D)
    batches, outs = [], []
    for k in range(5):
        pairs = [oracle.synth_pair(100 * k + i, W, H, D) for i in range(B)]
        Ls, Rs = np.stack([p[0] for p in pairs]), np.stack([p[1] for p in pairs])
        batches.append((Ls, Rs))
        if k % 2:
            l_view, r_view = fs.next_inputs()           # in-place producer path
            l_view[...] = Ls
            r_view[...] = Rs
            outs += fs.submit()
        else:
            outs += fs.submit(Ls, Rs)
    outs += fs.flush()
    assert len(outs) == 5
    for (Ls, Rs), got in zip(batches, outs):
        for i in range(B):
            assert np.array_equal(got[i], oracle.box_disp(Ls[i], Rs[i], r, D))


def test_frame_stream_consume_callback(matcher, oracle):
    from gpu_stereo_matching_amd.pipeline import FrameStream
    B, W, H, D, r = 2, 96, 40, 16, 2
    seen = []
    fs = FrameStream(matcher, B, W, H, r, D, consume=lambda disp: seen.append(disp.copy()))
    batches = []
    for k in range(4):
        pairs = [oracle.synth_pair(7 * k + i, W, H, D) for i in range(B)]
        Ls, Rs = np.stack([p[0] for p in pairs]), np.stack([p[1] for p in pairs])
        batches.append((Ls, Rs))
        assert fs.submit(Ls, Rs) == []
    assert fs.flush() == []
    assert len(seen) == 4
    for (Ls, Rs), got in zip(batches, seen):
        for i in range(B):
            assert np.array_equal(got[i], oracle.box_disp(Ls[i], Rs[i], r, D))


@pytest.mark.parametrize("mode", ["bgr", "rectify", "bgr+rectify"])
def test_frame_stream_camera_chain(matcher, oracle, mode):
    """FrameStream with the front end on the GPU: BGR frames -> gray (Caller.cpp:15-16) and/or the
    calibration's rectification maps (Rectify + remap, Caller.cpp:27-74) -> match; every batch
    equals the oracle chain (bgr_to_gray -> remap -> box_disp) bit for bit."""
    import os
    from gpu_stereo_matching_amd import calib
    from gpu_stereo_matching_amd.pipeline import FrameStream
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    chess = np.load(os.path.join(golden, "chess_set2_gray.npz"))
    Lg, Rg = chess["Left_320x200"], chess["Right_320x200"]
    H, W = Lg.shape
    B, r, D = 2, 4, 48
    rng = np.random.default_rng(5)
    # BGR frames whose OpenCV gray is known: random colour, then the oracle's conversion
    Lb = [rng.integers(0, 256, (H, W, 3), dtype=np.uint8) for _ in range(B)]
    Rb = [np.roll(x, -7, axis=1) for x in Lb]
    maps = None
    if "rectify" in mode:
        K1, K2, d1, d2, Rm, T = calib.load_data_batch(os.path.join(golden, "Calib_Data_OpenCV.yml"))
        R1, R2, P1, P2, _ = calib.stereo_rectify(K1, d1, K2, d2, (W, H), Rm, T)
        maps = (*oracle.init_rectify_map(K1, d1, R1, P1, W, H), *oracle.init_rectify_map(K2, d2, R2, P2, W, H))
    if "bgr" in mode:
        lefts, rights = np.stack(Lb), np.stack(Rb)
        gl = [oracle.bgr_to_gray(x) for x in Lb]
        gr = [oracle.bgr_to_gray(x) for x in Rb]
    else:
        lefts, rights = np.stack([Lg, Lg[::-1].copy()]), np.stack([Rg, Rg[::-1].copy()])
        gl, gr = list(lefts), list(rights)
    if maps is not None:
        gl = [oracle.remap(g, maps[0], maps[1]) for g in gl]
        gr = [oracle.remap(g, maps[2], maps[3]) for g in gr]
    want = [oracle.box_disp(a, b, r, D) for a, b in zip(gl, gr)]
    fs = FrameStream(matcher, B, W, H, r, D, bgr="bgr" in mode, rectify_maps=maps)
    outs = []
    for _ in range(3):
        outs += fs.submit(lefts, rights)
    outs += fs.flush()
    assert len(outs) == 3
    for got in outs:
        for i in range(B):
            assert np.array_equal(got[i], want[i])


def test_capture_loop_replay(matcher, oracle, tmp_path):
    """capture.run_loop over photo()-style saved pairs (Left_<n>/Right_<n>, Utility.cpp:217-218): PNG
    BGR frames -> GPU gray -> the calibration's rectification -> match, 2 pairs per launch over 5 pairs
    (a padded last batch); each map, delivered in pair order and written as disp_<n>.png, equals the
    oracle chain bit for bit."""
    import os
    from PIL import Image
    from gpu_stereo_matching_amd import calib
    from gpu_stereo_matching_amd.capture import PairSequence, run_loop
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    W, H, r, D = 320, 200, 4, 48
    rng = np.random.default_rng(11)
    want = {}
    K1, K2, d1, d2, Rm, T = calib.load_data_batch(os.path.join(golden, "Calib_Data_OpenCV.yml"))
    R1, R2, P1, P2, _ = calib.stereo_rectify(K1, d1, K2, d2, (W, H), Rm, T)
    maps = (*oracle.init_rectify_map(K1, d1, R1, P1, W, H), *oracle.init_rectify_map(K2, d2, R2, P2, W, H))
    for n in (1, 3, 4, 8, 12):
        Lb = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        Rb = np.roll(Lb, -5 - n, axis=1)
        Image.fromarray(Lb[:, :, ::-1]).save(tmp_path / f"Left_{n}.png")    # stored as RGB, read back as BGR
        Image.fromarray(Rb[:, :, ::-1]).save(tmp_path / f"Right_{n}.png")
        gl = oracle.remap(oracle.bgr_to_gray(Lb), maps[0], maps[1])
        gr = oracle.remap(oracle.bgr_to_gray(Rb), maps[2], maps[3])
        want[n] = oracle.box_disp(gl, gr, r, D)
    got = {}
    out = tmp_path / "maps"
    order = run_loop(PairSequence(str(tmp_path)), matcher, r, D, rectify_maps=maps, batch=2,
                     on_map=lambda n, d: got.__setitem__(n, d.copy()), out_dir=str(out))
    assert order == [1, 3, 4, 8, 12]
    for n, w in want.items():
        assert np.array_equal(got[n], w), n
        assert np.array_equal(np.asarray(Image.open(out / f"disp_{n}.png")), w), n


@pytest.mark.parametrize("W,H,D", [(64, 16, 8), (333, 77, 100), (1920, 1080, 128), (5, 3, 7), (3840, 5, 20)])
def test_ad_volume(matcher, oracle, torch, W, H, D):
    """PreCal / kernalPreCal_V2 (row a1) as a standalone HBM-bound kernel, bit-exact (bands of rows per
    block: 77 rows leave a partial last band, 3840 columns take 4 segments per thread)."""
    L, R = oracle.synth_pair(W + D, W, H, max(D, 16))
    want = oracle.precal(L, R, D)
    assert np.array_equal(matcher.ad_volume(L, R, D), want)
    got = matcher.ad_volume_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda(), D)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy(), want)


@pytest.mark.parametrize("W,H,r,D", [(320, 256, 5, 64), (333, 77, 7, 100), (1920, 1080, 5, 128), (63, 40, 0, 8),
                                     (463, 370, 3, 64)])
def test_staged_equals_fused_and_oracle(matcher, oracle, torch, W, H, r, D):
    """SM_STAGED (AD u8 -> SAD u16 -> WTA through HBM) gives the fused kernel's map, bit-exact."""
    L, R = oracle.synth_pair(W * 7 + r, W, H, max(D, 16))
    Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    staged = matcher.match_device(Lt, Rt, r, D, agg="box-staged")
    fused = matcher.match_device(Lt, Rt, r, D)
    torch.cuda.synchronize()
    assert torch.equal(staged, fused)
    if W * H <= 200_000:
        assert np.array_equal(staged.cpu().numpy(), oracle.box_disp(L, R, r, D))


def test_sad_volume(matcher, oracle, torch):
    L, R = oracle.synth_pair(31, 150, 60, 32)
    sad = matcher.sad_volume_device(torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda(), 4, 32)
    torch.cuda.synchronize()
    want = oracle.box_cost(L, R, 4, 32)
    assert np.array_equal(sad.cpu().numpy().view(np.uint16).astype(np.int32), want)


def test_staged_median_batch(matcher, oracle, torch):
    pairs = [oracle.synth_pair(60 + b, 200, 50, 32) for b in range(3)]
    Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    out = matcher.match_device(Lt, Rt, 3, 32, agg="box-staged", median=True)
    torch.cuda.synchronize()
    for b in range(3):
        assert np.array_equal(out[b].cpu().numpy(), oracle.median(oracle.box_disp(pairs[b][0], pairs[b][1], 3, 32), 3))


@pytest.mark.parametrize("median", [False, True])
def test_staged_launch_groups(matcher, oracle, torch, median):
    """11 frames = launch groups of 8 and 3 (one AD / SAD / WTA launch per group, frames from
    blockIdx.y in the WTA): every frame equals the fused kernel's map."""
    pairs = [oracle.synth_pair(500 + b, 241, 67, 48) for b in range(11)]
    Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    staged = matcher.match_device(Lt, Rt, 4, 48, agg="box-staged", median=median)
    fused = matcher.match_device(Lt, Rt, 4, 48, median=median)
    torch.cuda.synchronize()
    assert torch.equal(staged, fused)
    k = matcher.staged_kernel_ms()
    assert len(k) == 3 and all(t > 0 for t in k)


def test_staged_group_param(oracle, torch):
    """SM_PARAM_STAGED_GROUP bounds the staged workspace: groups of 1 and 3 give the same maps as 8;
    values outside 1..8 (or not integers) are rejected."""
    import gpu_stereo_matching_amd as sm
    from gpu_stereo_matching_amd import _capi
    pairs = [oracle.synth_pair(700 + b, 160, 48, 32) for b in range(5)]
    Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    with sm.BlockMatcher(0, 256, 64, 64) as m:
        want = m.match_device(Lt, Rt, 3, 32)
        for g in (1, 3, 8):
            assert m._lib.sm_set_param_f(m._h, _capi.SM_PARAM_STAGED_GROUP, float(g)) == 0
            assert torch.equal(m.match_device(Lt, Rt, 3, 32, agg="box-staged"), want)
        for bad in (0.0, 9.0, 2.5):
            assert m._lib.sm_set_param_f(m._h, _capi.SM_PARAM_STAGED_GROUP, bad) == _capi.SM_ERR_INVALID_ARG


@pytest.mark.parametrize("seed", list(range(40)))
def test_fuzz_box_lr_slices(matcher, oracle, torch, seed):
    """Seeded random shapes / radii / disparity counts / textures: box (host and batched device),
    box + LR, and the MIN over random d-slices, all bit-exact against the oracle."""
    rng = np.random.default_rng(1000 + seed)
    W, H = int(rng.integers(1, 700)), int(rng.integers(1, 120))
    r, D = int(rng.integers(0, 10)), int(rng.integers(1, 257))
    L, R = fuzz_pair(rng, W, H)
    disp, keys = oracle.box_disp(L, R, r, D, want_keys=True)
    assert np.array_equal(matcher.match(L, R, r, D), disp), (W, H, r, D)
    L2, R2 = fuzz_pair(rng, W, H)
    Lt = torch.from_numpy(np.stack([L, L2])).cuda()
    Rt = torch.from_numpy(np.stack([R, R2])).cuda()
    out = matcher.match_device(Lt, Rt, r, D).cpu().numpy()
    assert np.array_equal(out[0], disp) and np.array_equal(out[1], oracle.box_disp(L2, R2, r, D)), (W, H, r, D)
    _, rd, chk, mask = oracle.box_lr(L, R, r, D)
    c, rr, mm = matcher.match_lr(L, R, r, D)
    assert np.array_equal(rr, rd) and np.array_equal(c, chk) and np.array_equal(mm, mask), (W, H, r, D)
    if r <= 7:
        cuts = sorted({0, D, *[int(v) for v in rng.integers(1, D + 1, size=3)]})
        k = None
        for a, b in zip(cuts[:-1], cuts[1:]):
            p = matcher.slice_keys_device(Lt[0], Rt[0], r, a, b)
            k = p if k is None else torch.minimum(k, p)
        torch.cuda.synchronize()
        assert np.array_equal(k.cpu().numpy().view(np.uint32), keys), (W, H, r, D, cuts)


def test_pinned_host_buffers(sm, matcher, oracle):
    """sm_host_alloc frames and maps through the drop-in host path (DMA straight from / into the
    caller's page-locked memory) give the same maps as pageable numpy buffers."""
    W, H, D, r = 1920, 1080, 128, 5
    L, R = oracle.synth_pair(41, W, H, D)
    want = oracle.box_disp(L, R, r, D)
    Lp, Rp, Op = sm.host_empty((H, W)), sm.host_empty((H, W)), sm.host_empty((H, W))
    Lp[...] = L
    Rp[...] = R
    Op[...] = 7
    got = matcher.match(Lp, Rp, r, D, out=Op)
    assert got is Op and np.array_equal(Op, want)
    chk, rd, mask = matcher.match_lr(Lp, Rp, r, D)
    _, rd_o, chk_o, mask_o = oracle.box_lr(L, R, r, D)
    assert np.array_equal(chk, chk_o) and np.array_equal(rd, rd_o) and np.array_equal(mask, mask_o)


@pytest.mark.parametrize("W,H,D,r", [(1920, 1080, 128, 5), (463, 370, 64, 4), (97, 31, 40, 0), (333, 150, 64, 11)])
def test_pair_in_one_block(sm, matcher, oracle, W, H, D, r):
    """A pair whose right frame follows the left one in memory (one (2, H, W) block: page-locked from
    sm_host_alloc, or a pageable numpy array) goes up as one copy; maps bit-exact with the oracle for
    box, box + LR and guided, and the next call on separate frames is unaffected."""
    L, R = oracle.synth_pair(60 + r, W, H, D)
    want = oracle.box_disp(L, R, r, D)
    _, rd_o, chk_o, mask_o = oracle.box_lr(L, R, r, D)
    for pair in (sm.host_empty((2, H, W)), np.empty((2, H, W), np.uint8)):
        pair[0], pair[1] = L, R
        assert pair[1].ctypes.data == pair[0].ctypes.data + W * H
        assert np.array_equal(matcher.match(pair[0], pair[1], r, D), want)
        Op = sm.host_empty((H, W))
        assert np.array_equal(matcher.match(pair[0], pair[1], r, D, out=Op), want)
        chk, rd, mask = matcher.match_lr(pair[0], pair[1], r, D)
        assert np.array_equal(chk, chk_o) and np.array_equal(rd, rd_o) and np.array_equal(mask, mask_o)
        if r <= 7:
            g_pair = matcher.match(pair[0], pair[1], r, D, agg="guided")
            assert np.array_equal(g_pair, matcher.match(L.copy(), R.copy(), r, D, agg="guided"))
    assert np.array_equal(matcher.match(L, R, r, D), want)


@pytest.mark.parametrize("agg,med", [("box", False), ("box", True), ("guided", False), ("box-staged", False),
                                     ("box-staged", True)])
def test_zero_copy_map(sm, matcher, oracle, agg, med):
    """A map received into an sm_host_alloc block is written by the last kernel straight into it
    (zero-copy, no download): same map as a pageable output, for each kernel that can write it last;
    the block is refilled with garbage between calls so a missed write shows.  A pitched map inside a
    larger block (raw C ABI, out_pitch > width) too."""
    import ctypes
    from gpu_stereo_matching_amd import _capi
    W, H, D, r = 517, 203, 64, 4
    L, R = oracle.synth_pair(77, W, H, D)
    want = matcher.match(L, R, r, D, agg=agg, median=med)
    Op = sm.host_empty((H, W))
    for fill in (0, 255, 0x5A):
        Op[...] = fill
        assert np.array_equal(matcher.match(L, R, r, D, agg=agg, median=med, out=Op), want)
    P2 = W + 37
    big = sm.host_empty((H + 2, P2))
    big[...] = 0xEE
    view = big[1:, :]   # rows 1.. of the block, pitch P2
    rc = matcher._lib.sm_block_match_u8(matcher._h, L.ctypes.data, R.ctypes.data, W, H, W, r, D,
                                         sm._flags(agg, False, med), view.ctypes.data, P2)
    assert rc == _capi.SM_OK
    assert np.array_equal(big[1:H + 1, :W], want)
    assert (big[0] == 0xEE).all() and (big[1:H + 1, W:] == 0xEE).all()   # nothing outside the map


@pytest.mark.parametrize("W,H,D,r", [(333, 257, 64, 7), (640, 256, 96, 0), (500, 300, 128, 11),
                                     (1001, 400, 256, 15), (320, 260, 32, 3)])
def test_pinned_odd_shapes(sm, matcher, oracle, W, H, D, r):
    """Page-locked frames through the host path at odd heights, r = 0, the r > 7 kernel, with
    pageable and page-locked outputs: bit-exact with the oracle and with pageable frames."""
    L, R = oracle.synth_pair(50 + r, W, H, D)
    want = oracle.box_disp(L, R, r, D)
    Lp, Rp = sm.host_empty((H, W)), sm.host_empty((H, W))
    Lp[...] = L
    Rp[...] = R
    assert np.array_equal(matcher.match(Lp, Rp, r, D), want)           # pageable output
    Op = sm.host_empty((H, W))
    assert np.array_equal(matcher.match(Lp, Rp, r, D, out=Op), want)   # pinned output
    assert np.array_equal(matcher.match(L, R, r, D), want)             # pageable frames: one-piece path
