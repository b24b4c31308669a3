"""The multi-GPU group handle of the C ABI (sm_create_group) on the one GPU of the test box: a
group may name a device more than once, so 2-3 members on device 0 exercise the banding, the
per-member worker threads and the batch split exactly as distinct GPUs would.  Row-banded results
must equal the single-handle pass bit for bit (every flag is row-local; guided bands start on the
full frame's tile grid), including the guided filter's float path."""
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


def _pair(W, H, D, seed=99):
    from oracle import oracle as O
    return O.synth_pair(seed, W, H, max(D, 16))


@pytest.mark.parametrize("members", [2, 3])
@pytest.mark.parametrize("agg,lr,med,r,D", [("box", False, False, 5, 128), ("box", True, False, 4, 64),
                                            ("box", True, True, 3, 64), ("guided", False, False, 5, 64),
                                            ("guided", True, False, 7, 48), ("box-staged", False, False, 5, 64)])
def test_group_row_bands_bit_exact(single, members, agg, lr, med, r, D):
    import gpu_stereo_matching_amd as sm
    W, H = 640, 333
    L, R = _pair(W, H, D)
    with sm.BlockMatcherGroup([0] * members, 1920, 1080, 256) as g:
        assert len(g) == members
        g.set_guided_eps(EPS)
        if lr:
            got = g.match_lr(L, R, r, D, agg=agg, median=med)
            want = single.match_lr(L, R, r, D, agg=agg, median=med)
            for a, b in zip(got, want):
                assert np.array_equal(a, b)
        else:
            assert np.array_equal(g.match(L, R, r, D, agg=agg, median=med), single.match(L, R, r, D, agg=agg,
                                                                                         median=med))


def test_group_more_members_than_tiles(single):
    """A frame with fewer 32-row tiles than members: the extra members stay idle."""
    import gpu_stereo_matching_amd as sm
    L, R = _pair(200, 40, 32)
    with sm.BlockMatcherGroup([0, 0, 0], 512, 256, 64) as g:
        assert np.array_equal(g.match(L, R, 2, 32), single.match(L, R, 2, 32))


def test_group_batch(single):
    import gpu_stereo_matching_amd as sm
    pairs = [_pair(320, 120, 64, seed=s) for s in range(5)]
    with sm.BlockMatcherGroup([0, 0], 512, 256, 64) as g:
        outs = g.match_batch([p[0] for p in pairs], [p[1] for p in pairs], 4, 64, lr_check=True)
    for (L, R), o in zip(pairs, outs):
        assert np.array_equal(o, single.match(L, R, 4, 64, lr_check=True))


def test_group_error_from_a_member():
    """A member's failure comes back on the calling thread with its message."""
    import gpu_stereo_matching_amd as sm
    from gpu_stereo_matching_amd import _capi
    L, R = _pair(300, 64, 16)
    with sm.BlockMatcherGroup([0, 0], 256, 64, 64) as g:          # capacity 256 wide < 300
        with pytest.raises(_capi.SMError) as e:
            g.match(L, R, 2, 16)
    assert e.value.code == _capi.SM_ERR_CAPACITY and "device 0" in str(e.value)


# ---- RCCL d-slice mode (sm_group_dslice_block_match_u8): one member per distinct device --------
@pytest.mark.parametrize("W,H,r,D", [(640, 333, 5, 128), (463, 370, 4, 64), (1920, 1080, 5, 256), (97, 31, 9, 37)])
def test_group_dslice_one_member_box(single, W, H, r, D):
    """On the one GPU of the test box the RCCL communicator has one rank: the slice is the whole
    range, the reduce-scatter and all-gather are the identity (chunk == P, no padding), and the map
    must equal the single handle bit for bit.  The n > 1 plan (slice bounds, padding, chunk order)
    runs in test_dslice_rehearsal_* below."""
    import gpu_stereo_matching_amd as sm
    L, R = _pair(W, H, D)
    with sm.BlockMatcherGroup([0], 1920, 1080, 256) as g:
        got = g.match_dslice(L, R, r, D)
        got2 = g.match_dslice(L, R, r, D)          # the communicator is reused
    want = single.match(L, R, r, D)
    assert np.array_equal(got, want) and np.array_equal(got2, want)


def test_group_dslice_one_member_guided(single):
    import gpu_stereo_matching_amd as sm
    W, H, r, D = 320, 240, 5, 64
    L, R = _pair(W, H, D, seed=7)
    with sm.BlockMatcherGroup([0], 1920, 1080, 256) as g:
        g.set_guided_eps(EPS)
        got = g.match_dslice(L, R, r, D, agg="guided")
    want = single.match(L, R, r, D, agg="guided")
    # the keys quantise q to 2^-14: equal except where two fp32 costs are that close, and every
    # pixel within the tie tolerance of the fp64 oracle (no bare ratio)
    assert (got == want).mean() >= 0.998
    from guided_check import tie_aware_check
    from oracle import oracle as O
    disp_o, q, best = O.guided_disp(L, R, r, D, EPS, want_q=True)
    ok, _ = tie_aware_check(got, q, {"disp": disp_o, "best": best}, D, W)
    assert ok.all(), f"{int((~ok).sum())} pixels outside the tie-aware tolerance"


def test_group_dslice_rejects_repeated_device_and_flags():
    import gpu_stereo_matching_amd as sm
    from gpu_stereo_matching_amd import _capi
    L, R = _pair(64, 32, 16)
    with sm.BlockMatcherGroup([0, 0], 256, 64, 64) as g:
        with pytest.raises(_capi.SMError) as e:
            g.match_dslice(L, R, 2, 16)
        assert e.value.code == _capi.SM_ERR_INVALID_ARG and "distinct devices" in str(e.value)
    out = np.empty((32, 64), np.uint8)
    with sm.BlockMatcherGroup([0], 256, 64, 64) as g:
        rc = g._lib.sm_group_dslice_block_match_u8(g._g, L.ctypes.data, R.ctypes.data, 64, 32, 64, 2, 16,
                                                   _capi.SM_MEDIAN, out.ctypes.data, 64)
    assert rc == _capi.SM_ERR_INVALID_ARG   # SM_LR_CHECK is accepted since round 5 (test_gpu_dslice_lr.py)


# ---- the d-slice plan for n > 1 members on one device (sm_dslice_rehearse_u8) ---------------------
@pytest.mark.parametrize("members", [2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("W,H,r,D", [(97, 31, 4, 37), (463, 370, 4, 64), (41, 19, 2, 5), (1920, 1080, 5, 256),
                                     (50, 3, 1, 16)])
def test_dslice_rehearsal_box_bit_exact(single, members, W, H, r, D):
    """members > 1 through the same per-member row-split upload (member k's rows into slot k of the
    gathered frames, where the in-place pair all-gather leaves them), key pass, seed padding (odd P)
    and chunk finalisation as the RCCL group call; D = 5 with 8 members gives empty slices, H = 3
    members without rows (pad slots only)."""
    L, R = _pair(W, H, D, seed=members)
    assert np.array_equal(single.dslice_rehearse(L, R, r, D, members), single.match(L, R, r, D))


@pytest.mark.parametrize("members", [2, 4, 7])
def test_dslice_rehearsal_guided(single, members):
    from oracle import oracle as O
    W, H, r, D = 160, 90, 3, 48
    L, R = _pair(W, H, D, seed=11)
    got = single.dslice_rehearse(L, R, r, D, members, agg="guided")
    want = single.match(L, R, r, D, agg="guided")
    # keys quantise q to 2^-14: equal except where two fp32 costs are that close, and
    # every pixel of the combined map is within the tie tolerance of the fp64 oracle
    assert (got == want).mean() >= 0.998
    from guided_check import tie_aware_check
    disp_o, q, best = O.guided_disp(L, R, r, D, EPS, want_q=True)
    ok, _ = tie_aware_check(got, q, {"disp": disp_o, "best": best}, D, W)
    assert ok.all(), f"{int((~ok).sum())} pixels outside the tie-aware tolerance"


@pytest.mark.parametrize("phase", ["keys", "collective"])
def test_dslice_member_failure_returns_error(single, monkeypatch, phase):
    """A member failing before the collectives (keys) or in place of them (collective) makes the call
    return its error instead of hanging the others; the next call re-creates what it must
    and is bit-exact."""
    import gpu_stereo_matching_amd as sm
    from gpu_stereo_matching_amd import _capi
    L, R = _pair(320, 97, 64, seed=5)
    want = single.match(L, R, 4, 64)
    with sm.BlockMatcherGroup([0], 512, 256, 64) as g:
        assert np.array_equal(g.match_dslice(L, R, 4, 64), want)
        monkeypatch.setenv("SM_DSLICE_FAULT", f"0:{phase}")
        with pytest.raises(_capi.SMError) as e:
            g.match_dslice(L, R, 4, 64)
        assert e.value.code == _capi.SM_ERR_LAUNCH and "injected fault" in str(e.value)
        monkeypatch.delenv("SM_DSLICE_FAULT")
        assert np.array_equal(g.match_dslice(L, R, 4, 64), want)
