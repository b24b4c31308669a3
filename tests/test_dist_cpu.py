"""World-size-2 gloo tests of the multi-GPU partitioning (run on CPU, no GPU needed).

The key reduction is exercised with real torch.distributed collectives; per-rank slice keys
come from the oracle (the GPU produces the same keys: tests/test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gpu_stereo_matching_amd import sharding


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, r, D, result_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    L, R = O.synth_pair(4321, W, H, max(D, 16))
    lo, hi = sharding.dslice_bounds(D, rank, world)
    if hi > lo:
        keys = O.box_keys_slice(L, R, r, lo, hi).view(np.int32)
    else:
        keys = np.full((H, W), sharding.seed_key(r), np.int32)
    for coll in ("allreduce", "rs_ag"):
        disp = sharding.match_dslice_host_keys(keys, r, world, collective=coll)
        np.save(os.path.join(result_dir, f"disp{rank}_{coll}.npy"), disp)
    # frame-parallel: every frame handled exactly once across ranks
    mine = torch.zeros(10, dtype=torch.int64)
    for f in sharding.frame_shard(10, rank, world):
        mine[f] += 1
    dist.all_reduce(mine)
    np.save(os.path.join(result_dir, f"frames{rank}.npy"), mine.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,D,W", [(2, 64, 120), (2, 7, 120), (3, 64, 121), (4, 3, 77)])
def test_dslice_min_reduction_gloo(tmp_path, world, D, W):
    """Both d-slice reductions (MIN all-reduce; MIN reduce-scatter + uint8 all-gather, with the
    pixel count padded to the world size) give the full-range disparity on every rank."""
    H, r = 40, 3
    port = _free_port()
    mp.spawn(_worker, args=(world, port, W, H, r, D, str(tmp_path)), nprocs=world, join=True)
    from oracle import oracle as O
    L, R = O.synth_pair(4321, W, H, max(D, 16))
    want = O.box_disp(L, R, r, D)
    for k in range(world):
        for coll in ("allreduce", "rs_ag"):
            assert np.array_equal(np.load(tmp_path / f"disp{k}_{coll}.npy"), want), (k, coll)
        assert (np.load(tmp_path / f"frames{k}.npy") == 1).all()


def _lr_worker(rank, world, port, W, H, r, D, result_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    L, R = O.synth_pair(77, W, H, max(D, 16))
    lo, hi = sharding.dslice_bounds(D, rank, world)
    if hi > lo:
        keys = O.box_keys_slice(L, R, r, lo, hi).view(np.int32)
        rkeys = O.box_right_keys_slice(L, R, r, lo, hi).view(np.int32)
    else:
        keys = np.full((H, W), sharding.seed_key(r), np.int32)
        rkeys = np.full((H, W), sharding.RIGHT_EMPTY_KEY, np.int32)
    for coll in ("allreduce", "rs_ag"):
        disp = sharding.match_dslice_host_keys(keys, r, world, collective=coll, right_keys=rkeys)
        np.save(os.path.join(result_dir, f"lr{rank}_{coll}.npy"), disp)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,D,W,r", [(2, 48, 90, 3), (3, 37, 61, 3), (4, 3, 50, 3), (2, 40, 90, 40),
                                         (3, 24, 70, 100)])
def test_dslice_lr_reduction_gloo(tmp_path, world, D, W, r):
    """d-slices with the LR check (a second packed reduction for the right view): the right
    view's slice keys take the same MIN collectives, their d fields form dR, and StereoDisparity.cpp:136-147
    gives the single pass's checked map (box_lr) on every rank, through both collectives, with empty slices
    (world 4 > D 3), padded pixel counts and wide windows (r = 40, 100: the wide path's radii)."""
    H = 30
    port = _free_port()
    mp.spawn(_lr_worker, args=(world, port, W, H, r, D, str(tmp_path)), nprocs=world, join=True)
    from oracle import oracle as O
    L, R = O.synth_pair(77, W, H, max(D, 16))
    want = O.box_lr(L, R, r, D)[2]
    assert want.any()
    for k in range(world):
        for coll in ("allreduce", "rs_ag"):
            assert np.array_equal(np.load(tmp_path / f"lr{k}_{coll}.npy"), want), (k, coll)


def test_right_keys_flip_orders_keys_past_2_31():
    """A 255-vs-0 frame at r = 100: window sums reach 255 * 201^2 (> 2^23), so raw right keys (SAD << 8 | d) pass
    2^31.  With the sign bit flipped a signed MIN over any partition still gives STMatching's right WTA, and
    "no d reaches u" (INT32_MAX) stays above every key."""
    from oracle import oracle as O
    W, H, r, D = 210, 205, 100, 6
    L = np.full((H, W), 255, np.uint8)
    R = np.zeros((H, W), np.uint8)
    R[:, ::7] = 9
    cost = O.box_cost(L, R, r, D)
    assert int(cost.max()) << 8 >= 1 << 31
    want = O.right_wta(cost)
    for cuts in ((0, D), (0, 2, D), (0, 1, 3, 5, D)):
        parts = [O.box_right_keys_slice(L, R, r, a, b, cost).view(np.int32) for a, b in zip(cuts, cuts[1:])]
        k = np.minimum.reduce(parts)
        assert np.array_equal((k & 0xFF).astype(np.uint8), want), cuts
        assert (k < np.iinfo(np.int32).max).all()


def test_right_keys_slice_min_is_right_wta():
    """The right view's slice keys MIN'ed over any partition of [0, D) give STMatching's right WTA
    (StereoHelper.cpp:131-180: the clamped walk, strict < from d = 0) on the oracle's cost volume."""
    from oracle import oracle as O
    L, R = O.synth_pair(5, 70, 20, 32)
    cost = O.box_cost(L, R, 2, 32)
    want = O.right_wta(cost)
    for cuts in ((0, 32), (0, 5, 32), (0, 1, 2, 17, 31, 32)):
        k = np.minimum.reduce([O.box_right_keys_slice(L, R, 2, a, b, cost).view(np.int32)
                               for a, b in zip(cuts, cuts[1:])])
        assert np.array_equal((k & 0xFF).astype(np.uint8), want), cuts


def _guided_slice_keys(q, lo, hi):
    """Host restatement of sm_guided_slice_keys_device on the oracle's fp64 q volume [D][H][W]:
    (int)(q * 2^14) << 8 | d over the valid d (d <= W - x) of [lo, hi), INT32_MAX if none."""
    _, H, W = q.shape
    xs = np.arange(W)[None, :]
    best = np.full((H, W), sharding.GUIDED_EMPTY_KEY, np.int64)
    for d in range(lo, hi):
        k = (np.trunc(np.clip(q[d] * 16384.0, -2 ** 23, 2 ** 23 - 1)).astype(np.int64) << 8) | d
        best = np.where(d <= W - xs, np.minimum(best, k), best)
    return best.astype(np.int32)


def _guided_worker(rank, world, port, W, H, r, D, result_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    q = np.load(os.path.join(result_dir, "q.npy"))
    lo, hi = sharding.dslice_bounds(D, rank, world)
    keys = _guided_slice_keys(q, lo, hi)
    for coll in ("allreduce", "rs_ag"):
        disp = sharding.match_dslice_host_keys(keys, r, world, collective=coll, agg="guided")
        np.save(os.path.join(result_dir, f"g{rank}_{coll}.npy"), disp)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,D,W", [(2, 32, 61), (3, 5, 40)])
def test_guided_dslice_reduction_gloo(tmp_path, world, D, W):
    """Guided d-slices: the signed key MIN (negative q included) through both collectives, INT32_MAX
    padding and empty slices, then q < 50, equals the full-range keys' map and the fp64 oracle's
    disparity wherever the oracle's best two costs are not within the 2^-14 key quantum."""
    from oracle import oracle as O
    H, r, eps = 23, 2, 1e-4 * 255 * 255
    L, R = O.synth_pair(99, W, H, 16)
    disp_o, q, best = O.guided_disp(L, R, r, D, eps, want_q=True)
    np.save(tmp_path / "q.npy", q)
    assert (q < 0).any()   # the guided cost can be negative: the MIN must be signed
    port = _free_port()
    mp.spawn(_guided_worker, args=(world, port, W, H, r, D, str(tmp_path)), nprocs=world, join=True)
    want = sharding.guided_keys_to_disparity_host(_guided_slice_keys(q, 0, D))
    assert (want == disp_o).mean() > 0.99
    for k in range(world):
        for coll in ("allreduce", "rs_ag"):
            assert np.array_equal(np.load(tmp_path / f"g{k}_{coll}.npy"), want), (k, coll)


def test_shard_helpers():
    assert sharding.dslice_bounds(128, 0, 8) == (0, 16)
    assert sharding.dslice_bounds(128, 7, 8) == (112, 128)
    assert sum(len(sharding.frame_shard(13, k, 4)) for k in range(4)) == 13
    assert sharding.dslice_bounds(3, 4, 8) == (1, 1)   # more ranks than disparities: empty slice
    assert sharding.padded_pixels(40, 121, 3) == 4842 and sharding.padded_pixels(40, 120, 3) == 4800


def _band_worker(rank, world, port, W, H, r, D, mode, result_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    L, R = O.synth_pair(99, W, H, max(D, 16))
    y0, y1 = sharding.band_rows(H, rank, world)
    n = -(-H // world)
    mine = torch.zeros((n, W), dtype=torch.uint8)
    if y1 > y0:
        agg = "guided" if mode == "guided" else "box"
        ys, ye = sharding.band_input_rows(H, y0, y1, sharding.band_halo(r, agg))
        if mode == "box":
            band = O.box_disp(L[ys:ye], R[ys:ye], r, D)
        elif mode == "lr":
            band = O.box_lr(L[ys:ye], R[ys:ye], r, D)[2]
        else:
            band = O.guided_disp(L[ys:ye], R[ys:ye], r, D, 1e-4 * 255 * 255)[0]
        mine[:y1 - y0] = torch.from_numpy(band[y0 - ys:y1 - ys].copy())
    full = sharding.gather_bands(mine, H, world)
    np.save(os.path.join(result_dir, f"band{rank}.npy"), full.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("world,H,mode", [(2, 40, "box"), (3, 41, "box"), (4, 9, "box"), (3, 37, "lr"),
                                          (2, 30, "guided")])
def test_rowband_allgather_gloo(tmp_path, world, H, mode):
    """Row bands with an r-row halo (2r for guided) reassemble the full-frame map."""
    W, r, D = 96, 3, 32
    port = _free_port()
    mp.spawn(_band_worker, args=(world, port, W, H, r, D, mode, str(tmp_path)), nprocs=world, join=True)
    from oracle import oracle as O
    L, R = O.synth_pair(99, W, H, max(D, 16))
    if mode == "box":
        want = O.box_disp(L, R, r, D)
    elif mode == "lr":
        want = O.box_lr(L, R, r, D)[2]
    else:
        want = O.guided_disp(L, R, r, D, 1e-4 * 255 * 255)[0]
    for k in range(world):
        got = np.load(tmp_path / f"band{k}.npy")
        if mode == "guided":   # fp64 sums in another order: equal up to near-ties
            assert (got == want).mean() > 0.999
        else:
            assert np.array_equal(got, want)


def test_box_keys_fit_signed_int32_at_every_radius():
    """The torch d-slice collectives take a signed int32 MIN of the box keys: every key is min'ed with the
    seed (50 win^2) << 8 (Device.cu:37), which stays below 2^31 up to the largest radius (127)."""
    assert all(sharding.seed_key(r) < (1 << 31) for r in range(128))
    assert sharding.seed_key(127) == (50 * 255 * 255) << 8
