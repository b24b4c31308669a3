"""Guided-filter aggregation on the GPU vs the fp64 restatement (oracle/bm_oracle.c).

PARITY UNPINNED w.r.t. the reference: it has no guided filter; the build
defines the filter and checks its fp32 HIP path against its own fp64 CPU
restatement.  Tolerance (absolute, in AD units 0..255): a pixel passes when the GPU disparity
equals the oracle's, or when the oracle cost of the GPU's choice is within TOL of the oracle's
best (a near-tie), or when the oracle best is within TOL of the 50.0 threshold and the GPU
reports no match.
"""
import numpy as np
import pytest

from guided_check import tie_aware_check

pytestmark = pytest.mark.gpu
EPS = 1e-4 * 255 * 255


@pytest.fixture(scope="module")
def matcher():
    import gpu_stereo_matching_amd as sm
    m = sm.BlockMatcher(0, 1920, 1080, 256)
    m.set_guided_eps(EPS)
    yield m
    m.close()


@pytest.fixture(scope="module")
def torch():
    import torch as t
    assert t.cuda.is_available()
    return t


@pytest.mark.parametrize("r,D", [(5, 64), (3, 32), (0, 16), (7, 48)])
def test_guided_art(matcher, oracle, gray, r, D):
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    disp_o, q, best = oracle.guided_disp(L, R, r, D, EPS, want_q=True)
    got = matcher.match(L, R, r, D, agg="guided")
    ok, exact = tie_aware_check(got, q, {"disp": disp_o, "best": best}, D, L.shape[1])
    assert ok.all(), f"{int((~ok).sum())} pixels outside the tie-aware tolerance"
    assert exact.mean() > 0.995


def test_guided_golden(matcher, oracle, gray, guided_expected):
    """The committed golden map; pixels that differ from it must be fp64 near-ties (tie-aware rule)."""
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    got = matcher.match(L, R, 5, 64, agg="guided")
    want = guided_expected["Art_/r5/D64/disp"]
    assert (got == want).mean() > 0.995
    disp_o, q, best = oracle.guided_disp(L, R, 5, 64, EPS, want_q=True)
    assert np.array_equal(disp_o, want)
    ok, _ = tie_aware_check(got, q, {"disp": disp_o, "best": best}, 64, L.shape[1])
    assert ok.all(), f"{int((~ok).sum())} pixels outside the tie-aware tolerance"


@pytest.mark.parametrize("W,H,D,r", [(333, 77, 100, 4), (64, 20, 8, 1), (21, 13, 30, 2)])
def test_guided_synthetic_ragged(matcher, oracle, W, H, D, r):
    L, R = oracle.synth_pair(W + H, W, H, max(D, 16))
    disp_o, q, best = oracle.guided_disp(L, R, r, D, EPS, want_q=True)
    got = matcher.match(L, R, r, D, agg="guided")
    ok, exact = tie_aware_check(got, q, {"disp": disp_o, "best": best}, D, W)
    assert ok.all(), f"{int((~ok).sum())} pixels outside the tie-aware tolerance"


def _check_guided_lr(matcher, oracle, L, R, r, D, min_exact=0.99):
    """Guided + LR with the right view fused into the guided pass: the right map is STMatching's
    WTA of C_R(y, u, d) = C_L(y, u + d, d) (StereoHelper.cpp:131-180) on the guided left costs.
    Left and right maps are judged tie-aware against the fp64 oracle (the right keys also carry the
    2^-14 fixed-point quantisation, far inside TOL); the checked map and mask must equal the
    reference's LR rule (StereoDisparity.cpp:136-147) applied to the returned maps, bit for bit."""
    from guided_check import TOL
    H, W = L.shape
    disp_o, q, best = oracle.guided_disp(L, R, r, D, EPS, want_q=True)
    left = matcher.match(L, R, r, D, agg="guided")
    ok, _ = tie_aware_check(left, q, {"disp": disp_o, "best": best}, D, W)
    assert ok.all(), f"left: {int((~ok).sum())} pixels outside the tie-aware tolerance"
    chk, rd, mask = matcher.match_lr(L, R, r, D, agg="guided")
    rd_o, cr, best_r = oracle.right_wta_float(q)
    ys, us = np.mgrid[0:H, 0:W]
    assert (rd < D).all()
    cost_g = cr[rd.astype(np.int64), ys, us]
    ok_r = (rd == rd_o) | (cost_g <= best_r + TOL)
    assert ok_r.all(), f"right: {int((~ok_r).sum())} pixels outside the tie-aware tolerance"
    assert (rd == rd_o).mean() > min_exact
    chk_o, mask_o = oracle.lr_check(left, rd)
    assert np.array_equal(chk, chk_o) and np.array_equal(mask, mask_o)
    return mask


@pytest.mark.parametrize("r,D", [(5, 64), (3, 48), (0, 16), (7, 32), (1, 100), (4, 80), (2, 40)])
def test_guided_lr_art(matcher, oracle, gray, r, D):
    """Every right-view build: with the phase-1 wave roles (r = 0, 1, 3, 4, 5, kRolesRight) and without
    (r = 2, 7)."""
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    mask = _check_guided_lr(matcher, oracle, L, R, r, D)
    assert 0.3 < mask.mean() < 1.0


@pytest.mark.parametrize("W,H,D,r", [(333, 77, 100, 4), (64, 20, 8, 1), (21, 13, 30, 2), (97, 40, 256, 5),
                                     (130, 33, 64, 6)])
def test_guided_lr_synthetic_ragged(matcher, oracle, W, H, D, r):
    L, R = oracle.synth_pair(W * 3 + H, W, H, max(D, 16))
    _check_guided_lr(matcher, oracle, L, R, r, D)


def test_guided_lr_flat(matcher, oracle):
    """All-equal images: every cost is 0, so the first d wins everywhere in both views."""
    L = np.full((40, 90), 77, np.uint8)
    chk, rd, mask = matcher.match_lr(L, L.copy(), 5, 32, agg="guided")
    assert (rd == 0).all()
    assert (mask == 0).all() and (chk == 0).all()     # d == 0 counts as occluded (StereoDisparity.cpp:141)


def test_guided_lr_full_cfg3(matcher, oracle):
    """cfg3 exactly as BASELINE names it: 1920x1080, 11x11 (r = 5), d_max = 128, guided filter, on the
    bench's synthetic pair (seed 1234), with the LR check.  The fp64 oracle is probed at the GPU's
    left and right maps in O(P) memory (oracle.guided_probe): both maps tie-aware within TOL, the
    checked map and mask bit-exact with the reference's rule on the returned maps."""
    from guided_check import TOL
    W, H, D, r = 1920, 1080, 128, 5
    L, R = oracle.synth_pair(1234, W, H, D)
    left = matcher.match(L, R, r, D, agg="guided")
    chk, rd, mask = matcher.match_lr(L, R, r, D, agg="guided")
    disp_o, best, qL, bestR, qR = oracle.guided_probe(L, R, r, D, EPS, left, rd)
    xs = np.arange(W)[None, :]
    valid = left.astype(np.int64) <= (W - xs)
    ok_l = (left == disp_o) | (valid & (qL <= best + TOL) & (qL < 50.0 + TOL)) | ((left == 0) & (best >= 50.0 - TOL))
    assert ok_l.all(), f"left: {int((~ok_l).sum())} pixels outside the tie-aware tolerance"
    # uniform-noise texture: ~1 % of pixels have fp64 costs within TOL of another d (measured 98.9 %
    # exact on MI355X); every one of them passes the tie-aware rule above
    assert (left == disp_o).mean() > 0.98
    ok_r = qR <= bestR + TOL
    assert ok_r.all(), f"right: {int((~ok_r).sum())} pixels outside the tie-aware tolerance"
    chk_o, mask_o = oracle.lr_check(left, rd)
    assert np.array_equal(chk, chk_o) and np.array_equal(mask, mask_o)


def test_guided_lr_full_cfg5():
    """cfg5 exactly as BASELINE names it (configs[4]): 3840x2160, d_max = 192, guided filter + LR
    check, r = 5, on the bench's synthetic pair (seed 4321), host call and 2-frame batched device
    call.  Same rule as cfg3 above: both maps tie-aware within TOL against the fp64 oracle probed
    at the GPU's maps, the checked map and mask bit-exact with StereoDisparity.cpp:136-147."""
    import torch
    import gpu_stereo_matching_amd as sm
    from oracle import oracle
    from guided_check import TOL
    W, H, D, r = 3840, 2160, 192, 5
    L, R = oracle.synth_pair(4321, W, H, D)
    with sm.BlockMatcher(0, W, H, 256) as m:
        m.set_guided_eps(EPS)
        left = m.match(L, R, r, D, agg="guided")
        chk, rd, mask = m.match_lr(L, R, r, D, agg="guided")
        Lt = torch.from_numpy(np.stack([L, L])).cuda()
        Rt = torch.from_numpy(np.stack([R, R])).cuda()
        dev = m.match_device(Lt, Rt, r, D, agg="guided", lr_check=True)
        torch.cuda.synchronize()
        dev = dev.cpu().numpy()
    assert np.array_equal(dev[0], chk) and np.array_equal(dev[1], chk)
    disp_o, best, qL, bestR, qR = oracle.guided_probe(L, R, r, D, EPS, left, rd)
    xs = np.arange(W)[None, :]
    valid = left.astype(np.int64) <= (W - xs)
    ok_l = (left == disp_o) | (valid & (qL <= best + TOL) & (qL < 50.0 + TOL)) | ((left == 0) & (best >= 50.0 - TOL))
    assert ok_l.all(), f"left: {int((~ok_l).sum())} pixels outside the tie-aware tolerance"
    assert (left == disp_o).mean() > 0.98
    ok_r = qR <= bestR + TOL
    assert ok_r.all(), f"right: {int((~ok_r).sum())} pixels outside the tie-aware tolerance"
    chk_o, mask_o = oracle.lr_check(left, rd)
    assert np.array_equal(chk, chk_o) and np.array_equal(mask, mask_o)


def test_guided_lr_batched_device_and_median(matcher, oracle):
    """Batched device calls of the fused guided right view (per-frame right-key partials) give each
    frame's single-call result; with SM_MEDIAN both maps are filtered before the check."""
    import torch
    W, H, D, r = 300, 70, 64, 4
    pairs = [oracle.synth_pair(40 + i, W, H, D) for i in range(3)]
    Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
    Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
    for med in (False, True):
        out = matcher.match_device(Lt, Rt, r, D, agg="guided", lr_check=True, median=med)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        for i, (L, R) in enumerate(pairs):
            chk, rd, mask = matcher.match_lr(L, R, r, D, agg="guided", median=med)
            assert np.array_equal(got[i], chk)
        if med:
            left = matcher.match(L, R, r, D, agg="guided", median=True)
            assert np.array_equal(chk, oracle.lr_check(left, rd)[0])


@pytest.mark.parametrize("cuts", [[0, 64], [0, 32, 64], [0, 5, 17, 40, 64], [0, 8, 16, 24, 32, 40, 48, 56, 64]])
def test_guided_slice_keys_min(matcher, oracle, gray, torch, cuts):
    """Guided path sharded over d on one device (the per-rank compute of sharding.match_dslice with
    agg="guided"): each slice [a, b) scans only its own d (its keys name a d in [a, b) or are
    INT32_MAX), the signed MIN over the slices, thresholded at q < 50, is tie-aware against the fp64
    oracle and equals the single-pass guided map except at near-ties of the 2^-14-quantised costs."""
    r, D = 5, 64
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    H, W = L.shape
    Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    parts = [matcher.guided_slice_keys_device(Lt, Rt, r, a, b) for a, b in zip(cuts[:-1], cuts[1:])]
    k = parts[0].clone()
    for p in parts[1:]:
        k = torch.minimum(k, p)
    got = matcher.guided_keys_to_disp_device(k)
    full = matcher.match_device(Lt, Rt, r, D, agg="guided")
    torch.cuda.synchronize()
    xs = np.arange(W)[None, :]
    for (a, b), p in zip(zip(cuts[:-1], cuts[1:]), parts):
        pk = p.cpu().numpy()
        empty = pk == 0x7FFFFFFF
        d = pk & 0xFF
        assert ((d >= a) & (d < b) & (d <= W - xs))[~empty].all(), (a, b)
        assert (empty == (a > W - xs)).all(), (a, b)
    got = got.cpu().numpy()
    disp_o, q, best = oracle.guided_disp(L, R, r, D, EPS, want_q=True)
    ok, exact = tie_aware_check(got, q, {"disp": disp_o, "best": best}, D, W)
    assert ok.all(), f"{int((~ok).sum())} pixels outside the tie-aware tolerance"
    assert (got == full.cpu().numpy()).mean() > 0.998


def test_guided_dslice_one_rccl_rank(oracle, torch):
    """sharding.match_dslice(agg="guided") through RCCL (world 1) on a ragged frame, both collectives."""
    import torch.distributed as dist
    import gpu_stereo_matching_amd as sm
    from gpu_stereo_matching_amd import sharding
    W, H, D, r = 333, 121, 100, 4
    L, R = oracle.synth_pair(4242, W, H, D)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        with sm.BlockMatcher(0, 512, 256, 256) as m:
            m.set_guided_eps(EPS)
            Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
            full = m.match_device(Lt, Rt, r, D, agg="guided")
            disp_o, q, best = oracle.guided_disp(L, R, r, D, EPS, want_q=True)
            for coll in ("rs_ag", "allreduce"):
                got = sharding.match_dslice(m, Lt, Rt, r, D, 0, 1, collective=coll, agg="guided")
                torch.cuda.synchronize()
                got = got.cpu().numpy()
                assert (got == full.cpu().numpy()).mean() > 0.998, coll
                ok, _ = tie_aware_check(got, q, {"disp": disp_o, "best": best}, D, W)
                assert ok.all(), f"{coll}: {int((~ok).sum())} pixels outside the tie-aware tolerance"
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("W,H,D,r,cuts", [(300, 45, 256, 5, [0, 100, 256]), (61, 19, 100, 2, [0, 33, 34, 100]),
                                          (97, 40, 64, 7, [0, 31, 32, 63, 64])])
def test_guided_slice_keys_ragged(matcher, oracle, torch, W, H, D, r, cuts):
    """Slices up to d_max = 256, one-disparity slices, band-chunk edges (32) and slices wholly past
    the valid range of the right border columns, on ragged frames: same contract as above."""
    L, R = oracle.synth_pair(W * 7 + H, W, H, min(D, 64))
    Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    parts = [matcher.guided_slice_keys_device(Lt, Rt, r, a, b) for a, b in zip(cuts[:-1], cuts[1:])]
    k = parts[0].clone()
    for p in parts[1:]:
        k = torch.minimum(k, p)
    got = matcher.guided_keys_to_disp_device(k)
    torch.cuda.synchronize()
    xs = np.arange(W)[None, :]
    for (a, b), p in zip(zip(cuts[:-1], cuts[1:]), parts):
        pk = p.cpu().numpy()
        empty = pk == 0x7FFFFFFF
        d = pk & 0xFF
        assert ((d >= a) & (d < b) & (d <= W - xs))[~empty].all(), (a, b)
        assert (empty == (a > W - xs)).all(), (a, b)
    got = got.cpu().numpy()
    disp_o, q, best = oracle.guided_disp(L, R, r, D, EPS, want_q=True)
    ok, _ = tie_aware_check(got, q, {"disp": disp_o, "best": best}, D, W)
    assert ok.all(), f"{int((~ok).sum())} pixels outside the tie-aware tolerance"


def test_guided_pitched_host_input(matcher, gray):
    """Row pitch > width (a Mat ROI) on the guided path: the padding bytes (random, not zero) are never
    read, so the map is bit-identical to the contiguous call; the output pitch is honoured."""
    import gpu_stereo_matching_amd as sm
    L, R = gray["Art/view1"], gray["Art/view5"]
    H, W = L.shape
    P = W + 29
    rng = np.random.default_rng(3)
    Lp = rng.integers(0, 256, (H, P), dtype=np.uint8)
    Rp = rng.integers(0, 256, (H, P), dtype=np.uint8)
    Lp[:, :W] = L
    Rp[:, :W] = R
    out = np.full((H, W + 3), 9, np.uint8)
    rc = matcher._lib.sm_block_match_u8(matcher._h, Lp.ctypes.data, Rp.ctypes.data, W, H, P, 4, 64,
                                        sm.SM_AGG_GUIDED, out.ctypes.data, W + 3)
    assert rc == 0
    assert np.array_equal(out[:, :W], matcher.match(L, R, 4, 64, agg="guided"))
    assert (out[:, W:] == 9).all()


@pytest.mark.parametrize("eps", [1.0, 5000.0])
def test_guided_eps_parameter(oracle, gray, eps):
    """SM_PARAM_GUIDED_EPS reaches the kernel: other eps values, tie-aware against the fp64 oracle."""
    import gpu_stereo_matching_amd as sm
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    with sm.BlockMatcher(0, 640, 480, 256) as m:
        m.set_guided_eps(eps)
        got = m.match(L, R, 3, 48, agg="guided")
    disp_o, q, best = oracle.guided_disp(L, R, 3, 48, eps, want_q=True)
    ok, exact = tie_aware_check(got, q, {"disp": disp_o, "best": best}, 48, L.shape[1])
    assert ok.all(), f"{int((~ok).sum())} pixels outside the tie-aware tolerance"
    assert exact.mean() > 0.99


@pytest.mark.parametrize("seed", list(range(16)))
def test_fuzz_guided_and_lr(matcher, oracle, seed):
    """Seeded random shapes / radii (0-7) / D / textures (incl. flat halves, 0/255-only and quantised
    images: many exact ties) through guided and guided + LR, tie-aware against the fp64 oracle."""
    from fuzz_util import fuzz_pair
    rng = np.random.default_rng(5000 + seed)
    W, H = int(rng.integers(1, 400)), int(rng.integers(1, 90))
    r, D = int(rng.integers(0, 8)), int(rng.integers(1, 129))
    L, R = fuzz_pair(rng, W, H)
    disp_o, q, best = oracle.guided_disp(L, R, r, D, EPS, want_q=True)
    got = matcher.match(L, R, r, D, agg="guided")
    ok, _ = tie_aware_check(got, q, {"disp": disp_o, "best": best}, D, W)
    assert ok.all(), f"{int((~ok).sum())} pixels outside the tie-aware tolerance {(W, H, r, D)}"
    # tie-heavy textures: fp32 picks among fp64-equal costs freely, so no exact-match floor here
    _check_guided_lr(matcher, oracle, L, R, r, D, min_exact=0.0)
