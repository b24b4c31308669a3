"""d-slices with the LR check ("LR adds a second packed reduction for the right view").

Each member's one fused pass over its slice emits the left keys and the right view's keys
(C_R(y, u, d) = C_L(y, u + d, d), StereoHelper.cpp:156-180; sm_slice_keys_lr_device); both take a
MIN over the members, the right keys' d fields are dR (no threshold, :131-154) and
StereoDisparity.cpp:136-147 checks the map.  Box: bit-exact against the single-pass LR map and the
oracle's right slice keys.  Guided: the left and right maps tie-aware against the fp64 oracle, the
checked map equal to the LR rule applied to them."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

EPS = 1e-4 * 255 * 255


@pytest.fixture(scope="module")
def single():
    import gpu_stereo_matching_amd as sm
    m = sm.BlockMatcher(0, 1920, 1080, 256)
    m.set_guided_eps(EPS)
    yield m
    m.close()


def _pair(W, H, D, seed=31):
    from oracle import oracle as O
    return O.synth_pair(seed, W, H, max(D, 16))


@pytest.mark.parametrize("W,H,r,D,cuts", [(97, 31, 4, 37, (0, 10, 37)), (333, 77, 5, 128, (0, 40, 41, 128)),
                                          (64, 20, 0, 16, (0, 16)), (150, 45, 15, 64, (0, 7, 33, 64)),
                                          (41, 19, 2, 100, (0, 30, 60, 100)), (300, 64, 7, 256, (0, 128, 256))])
def test_box_slice_lr_keys_match_oracle(single, W, H, r, D, cuts):
    """The fused slice pass: left keys equal sm_slice_keys_device's, right keys equal the oracle's
    restatement (oracle.box_right_keys_slice) for slices starting past d = 0 and past the frame's
    width (W = 41 < d_lo = 60: every right key is the 0x7FFFFFFF 'none')."""
    import torch
    from oracle import oracle as O
    L, R = _pair(W, H, D)
    Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    cost = O.box_cost(L, R, r, D)
    for a, b in zip(cuts, cuts[1:]):
        lk, rk = single.slice_keys_lr_device(Lt, Rt, r, a, b)
        plain = single.slice_keys_device(Lt, Rt, r, a, b)
        torch.cuda.synchronize()
        assert np.array_equal(lk.cpu().numpy(), plain.cpu().numpy()), (a, b)
        want = O.box_right_keys_slice(L, R, r, a, b, cost)
        assert np.array_equal(rk.cpu().numpy().view(np.uint32), want), (a, b)


@pytest.mark.parametrize("members", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("W,H,r,D", [(97, 31, 4, 37), (463, 370, 4, 64), (41, 19, 2, 5), (640, 333, 5, 128),
                                     (1920, 1080, 5, 256), (120, 50, 11, 48)])
def test_dslice_rehearsal_box_lr_bit_exact(single, members, W, H, r, D):
    """The d-slice split with LR on one device: every member's fused left + right keys, the two MINs,
    the right map from the d fields and the LR check equal the single pass's checked map bit for bit
    (D = 5 with 8 members: empty slices; r = 11: the wide-radius fused right view)."""
    L, R = _pair(W, H, D, seed=members + r)
    want = single.match(L, R, r, D, lr_check=True)
    assert np.array_equal(single.dslice_rehearse(L, R, r, D, members, lr_check=True), want)


def test_dslice_lr_golden_pair(single, gray, bm_expected):
    """The bundled Art pair at the LR golden configuration, split over 4 and 7 members."""
    L, R = gray["Art/view1"], gray["Art/view5"]
    want = bm_expected["lr/Art/r4/D64/checked"]
    for n in (4, 7):
        assert np.array_equal(single.dslice_rehearse(L, R, 4, 64, n, lr_check=True), want)


@pytest.mark.parametrize("cuts", [(0, 64), (0, 21, 64), (0, 1, 32, 63, 64)])
def test_guided_slice_lr_keys(single, oracle, gray, cuts):
    """Guided d-slices with LR on one device: the signed MIN of the slices' left and right keys gives a
    left map and a right map each tie-aware against the fp64 oracle (right: STMatching's WTA of the
    oracle's C_R), and lr_check_device applies StereoDisparity.cpp:136-147 to them exactly."""
    import torch
    from guided_check import TOL, tie_aware_check
    r, D = 5, 64
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    H, W = L.shape
    Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    parts = [single.slice_keys_lr_device(Lt, Rt, r, a, b, agg="guided") for a, b in zip(cuts, cuts[1:])]
    lk, rk = parts[0][0].clone(), parts[0][1].clone()
    for a, b in parts[1:]:
        lk, rk = torch.minimum(lk, a), torch.minimum(rk, b)
    left = single.guided_keys_to_disp_device(lk)
    right = single.right_keys_to_disp_device(rk)
    chk = single.lr_check_device(left, right)
    torch.cuda.synchronize()
    left, right, chk = left.cpu().numpy(), right.cpu().numpy(), chk.cpu().numpy()
    disp_o, q, best = oracle.guided_disp(L, R, r, D, EPS, want_q=True)
    ok, _ = tie_aware_check(left, q, {"disp": disp_o, "best": best}, D, W)
    assert ok.all(), f"left: {int((~ok).sum())} pixels outside the tie-aware tolerance"
    rd_o, cr, best_r = oracle.right_wta_float(q)
    ys, us = np.mgrid[0:H, 0:W]
    ok_r = (right == rd_o) | (cr[right.astype(np.int64), ys, us] <= best_r + TOL)
    assert ok_r.all(), f"right: {int((~ok_r).sum())} pixels outside the tie-aware tolerance"
    assert (right == rd_o).mean() > 0.99
    assert np.array_equal(chk, oracle.lr_check(left, right)[0])
    # the same split through the one-call rehearsal: every pixel of its checked map is the LR rule applied
    # to some left and right disparities that each pass the tie-aware rule (no bare ratio)
    from guided_check import tie_aware_lr_check
    reh = single.dslice_rehearse(L, R, r, D, len(cuts) - 1, agg="guided", lr_check=True)
    ref = {"disp": disp_o, "best": best, "q": q, "rdisp": rd_o, "cr": cr, "best_r": best_r}
    ok = tie_aware_lr_check(reh, ref, D, W)
    assert ok.all(), f"rehearsal: {int((~ok).sum())} checked pixels without a tie-aware justification"
    assert np.array_equal(tie_aware_lr_check(chk, ref, D, W), np.ones_like(ok))


def test_dslice_lr_group_one_rccl_member(single, oracle):
    """sm_group_dslice_block_match_u8 with SM_LR_CHECK through RCCL (one member on the one GPU):
    two reduce-scatters, two all-gathers and member 0's LR check give the single pass's map (box), and a
    guided checked map every pixel of which is tie-aware-justified against the fp64 oracle."""
    import gpu_stereo_matching_amd as sm
    from guided_check import guided_reference, tie_aware_lr_check
    L, R = _pair(333, 97, 96, seed=5)
    with sm.BlockMatcherGroup([0], 512, 256, 256) as g:
        g.set_guided_eps(EPS)
        assert np.array_equal(g.match_dslice(L, R, 4, 96, lr_check=True), single.match(L, R, 4, 96, lr_check=True))
        got = g.match_dslice(L, R, 3, 48, agg="guided", lr_check=True)
    ok = tie_aware_lr_check(got, guided_reference(oracle, L, R, 3, 48, EPS), 48, L.shape[1])
    assert ok.all(), f"{int((~ok).sum())} checked pixels without a tie-aware justification"


@pytest.mark.parametrize("coll", ["rs_ag", "allreduce"])
def test_dslice_lr_torch_one_rccl_rank(coll):
    """sharding.match_dslice(lr_check=True) through torch.distributed / RCCL (world 1)."""
    import torch
    import torch.distributed as dist
    import gpu_stereo_matching_amd as sm
    from gpu_stereo_matching_amd import sharding
    W, H, D, r = 301, 67, 200, 4
    L, R = _pair(W, H, D, seed=9)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        with sm.BlockMatcher(0, 512, 256, 256) as m:
            Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
            got = sharding.match_dslice(m, Lt, Rt, r, D, 0, 1, collective=coll, lr_check=True)
            want = m.match_device(Lt, Rt, r, D, lr_check=True)
            torch.cuda.synchronize()
            assert np.array_equal(got.cpu().numpy(), want.cpu().numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("r", [16, 40, 127])
@pytest.mark.parametrize("members", [1, 2, 3, 5, 8])
def test_dslice_rehearsal_box_lr_wide_radius(single, members, r):
    """box d-slices with LR at r >= 16 take their right keys from the wide path's LDS
    atomic-min row (bm_wide.hip), sign-flipped; the split equals the single LR pass bit for bit."""
    W, H, D = 333, 97, 64
    L, R = _pair(W, H, D, seed=members * 3 + r)
    want = single.match(L, R, r, D, lr_check=True)
    assert np.array_equal(single.dslice_rehearse(L, R, r, D, members, lr_check=True), want)


def test_box_slice_lr_keys_wide_match_oracle(single):
    """Wide-path slice keys with LR (r = 21 and r = 100) against the oracle's restatement, for slices starting
    past d = 0 and past the frame's width; at r = 100 on a 255-vs-0 frame the raw right keys pass 2^31, so the
    flipped keys' signed order is exercised."""
    import torch
    from oracle import oracle as O
    for (W, H, r, D, cuts, flat) in ((150, 60, 21, 48, (0, 13, 48), False), (61, 40, 21, 100, (0, 70, 100), False),
                                     (230, 210, 100, 8, (0, 3, 8), True)):
        if flat:
            L = np.full((H, W), 255, np.uint8)
            R = np.zeros((H, W), np.uint8)
            R[:, ::5] = 17
        else:
            L, R = _pair(W, H, D)
        Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
        cost = O.box_cost(L, R, r, D)
        if flat:
            assert int(cost.max()) << 8 >= 1 << 31
        parts = []
        for a, b in zip(cuts, cuts[1:]):
            lk, rk = single.slice_keys_lr_device(Lt, Rt, r, a, b)
            torch.cuda.synchronize()
            assert np.array_equal(lk.cpu().numpy().view(np.uint32), O.box_keys_slice(L, R, r, a, b)), (r, a, b)
            want = O.box_right_keys_slice(L, R, r, a, b, cost)
            got = rk.cpu().numpy().view(np.uint32)
            assert np.array_equal(got, want), (r, a, b, int((got != want).sum()))
            parts.append(got.view(np.int32))
        rd = (np.minimum.reduce(parts) & 0xFF).astype(np.uint8)
        assert np.array_equal(rd, O.right_wta(cost)), r


@pytest.mark.parametrize("seed", list(range(12)))
def test_fuzz_dslice_lr_any_radius(single, seed):
    """Seeded fuzz of the d-slice split with LR over the whole radius range (fused right view r <= 15, the
    wide path's right row 16..127): random size, D, member count and tie-heavy textures; the rehearsal equals
    the single LR pass bit for bit, and the box right slice keys of one member equal the oracle's."""
    import torch
    from fuzz_util import fuzz_pair
    from oracle import oracle as O
    rng = np.random.default_rng(9000 + seed)
    r = int(rng.choice([int(rng.integers(0, 16)), int(rng.integers(16, 128))]))
    W = int(rng.integers(8, 400))
    H = int(rng.integers(4, 160))
    D = int(rng.integers(1, 257))
    n = int(rng.integers(1, 9))
    L, R = fuzz_pair(rng, W, H)
    want = single.match(L, R, r, D, lr_check=True)
    got = single.dslice_rehearse(L, R, r, D, n, lr_check=True)
    assert np.array_equal(got, want), (r, W, H, D, n, int((got != want).sum()))
    lo = int(rng.integers(0, D))
    hi = int(rng.integers(lo + 1, D + 1))
    Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    lk, rk = single.slice_keys_lr_device(Lt, Rt, r, lo, hi)
    torch.cuda.synchronize()
    assert np.array_equal(lk.cpu().numpy().view(np.uint32), O.box_keys_slice(L, R, r, lo, hi)), (r, lo, hi)
    assert np.array_equal(rk.cpu().numpy().view(np.uint32), O.box_right_keys_slice(L, R, r, lo, hi)), (r, lo, hi)
