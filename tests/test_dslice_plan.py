"""The d-slice plan (sm_dslice_plan), shared by the C group call (sm_group_dslice_block_match_u8), its
one-device rehearsal and the torch path (sharding.py), checked on the CPU for 2..8 members: the slices
partition [0, D) as Device.cu:43-61's independent d planes allow, and the padded reduce-scatter /
all-gather arithmetic, emulated in numpy over the oracle's per-slice keys, gives the full-range map.
Host-only: sm_dslice_plan touches no device."""
import numpy as np
import pytest

from gpu_stereo_matching_amd import sharding


@pytest.mark.parametrize("n", range(1, 9))
@pytest.mark.parametrize("P,D", [(1, 1), (37 * 23, 37), (37 * 23, 5), (1920 * 1080, 256), (97 * 31, 128)])
def test_plan_partitions(n, P, D):
    plans = [sharding.dslice_plan(P, D, k, n) for k in range(n)]
    los = [p[0] for p in plans]
    his = [p[1] for p in plans]
    assert los[0] == 0 and his[-1] == D
    assert all(his[k] == los[k + 1] for k in range(n - 1))       # contiguous, disjoint
    assert all(h >= l for l, h in zip(los, his))                # empty only when n > D
    assert sum(h - l for l, h in zip(los, his)) == D
    assert max(h - l for l, h in zip(los, his)) - min(h - l for l, h in zip(los, his)) <= 1
    chunk, padded = plans[0][2], plans[0][3]
    assert all(p[2] == chunk and p[3] == padded for p in plans)
    assert padded == n * chunk and P <= padded < P + n


def test_plan_rejects_bad_args():
    from gpu_stereo_matching_amd import _capi
    with pytest.raises(_capi.SMError):
        sharding.dslice_plan(0, 8, 0, 2)
    with pytest.raises(_capi.SMError):
        sharding.dslice_plan(10, 8, 2, 2)


@pytest.mark.parametrize("n", range(2, 9))
@pytest.mark.parametrize("W,H,r,D", [(37, 23, 3, 37), (41, 19, 2, 5), (64, 33, 5, 64)])
def test_plan_emulated_collectives_equal_full_range(n, W, H, r, D):
    """Each member's keys (oracle slice keys, or the seed for an empty slice) padded with the seed,
    elementwise MIN, chunk k finalised by member k and gathered at k*chunk == the full-range map."""
    from oracle import oracle as O
    L, R = O.synth_pair(1000 + n, W, H, max(D, 16))
    P = W * H
    seed = sharding.seed_key(r)
    bufs = []
    for k in range(n):
        lo, hi, chunk, padded = sharding.dslice_plan(P, D, k, n)
        buf = np.full(padded, seed, np.uint32)
        if hi > lo:
            buf[:P] = O.box_keys_slice(L, R, r, lo, hi).reshape(P)
        bufs.append(buf)
    red = np.minimum.reduce(bufs)
    out = np.empty(padded, np.uint8)
    for k in range(n):
        out[k * chunk:(k + 1) * chunk] = sharding.keys_to_disparity_host(red[k * chunk:(k + 1) * chunk], r)
    assert np.array_equal(out[:P].reshape(H, W), O.box_disp(L, R, r, D))


@pytest.mark.parametrize("n", range(1, 9))
@pytest.mark.parametrize("P,D", [(1, 1), (37 * 23, 37), (37 * 23, 5), (1920 * 1080, 256), (7, 300)])
def test_python_twin_equals_library(n, P, D):
    """sharding.dslice_plan_py (used where libsm_hip.so is not built) gives sm_dslice_plan's numbers."""
    for k in range(n):
        assert sharding.dslice_plan_py(P, D, k, n) == sharding.dslice_plan(P, D, k, n)
    with pytest.raises(ValueError):
        sharding.dslice_plan_py(0, 8, 0, 2)


def test_plan_without_library(monkeypatch):
    """A process without the HIP build still gets the plan (pure-Python twin), not an ImportError."""
    from gpu_stereo_matching_amd import _capi

    def missing(*a, **k):
        raise ImportError("libsm_hip.so not built")
    monkeypatch.setattr(_capi, "load", missing)
    assert sharding.dslice_plan(100, 64, 1, 4) == (16, 32, 25, 100)
    assert sharding.dslice_bounds(64, 3, 4) == (48, 64)
    assert sharding.padded_pixels(10, 10, 8) == 104
