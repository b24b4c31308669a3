"""Multi-GPU partitioning of the matching path, one process per GPU.

Two ways to spread the work over ranks:
  * frames (independent rectified pairs): each rank matches its own frames; no collective in the
    data path — the path's natural partition, used for the headline maps/s ("scaling": "weak");
  * disparity slices of ONE frame: rank k scans d in [k*D/G, (k+1)*D/G) and emits per-pixel
    packed keys (SAD << 8 | d); an elementwise MIN all-reduce (RCCL over xGMI on GPUs, gloo on
    CPU) gives the global argmin with the reference's smallest-d tie break (strict <,
    Device.cu:57); the threshold / no-match rule is applied after the reduction.
"""
from __future__ import annotations

from typing import List, Tuple


def frame_shard(n_frames: int, rank: int, world: int) -> List[int]:
    """Contiguous, balanced split of frame indices [0, n_frames) over ranks."""
    lo = rank * n_frames // world
    hi = (rank + 1) * n_frames // world
    return list(range(lo, hi))


def dslice_bounds(num_disp: int, rank: int, world: int) -> Tuple[int, int]:
    """Disparity slice [lo, hi) of `rank`; empty slices are allowed when world > num_disp."""
    return rank * num_disp // world, (rank + 1) * num_disp // world


def seed_key(radius: int) -> int:
    """(50*win^2) << 8: the reference's start value (Device.cu:37) as a packed key."""
    win = 2 * radius + 1
    return (50 * win * win) << 8


def reduce_slice_keys(keys, group=None):
    """In-place MIN all-reduce of an int32 key map (keys < 2^31 by construction)."""
    import torch.distributed as dist
    dist.all_reduce(keys, op=dist.ReduceOp.MIN, group=group)
    return keys


def keys_to_disparity_host(keys, radius: int):
    """numpy helper: key map -> uint8 disparity (d if SAD < 50*win^2, else 0)."""
    import numpy as np
    k = keys.astype(np.uint32)
    return np.where((k >> 8) < (seed_key(radius) >> 8), k & 0xFF, 0).astype(np.uint8)


def match_dslice(matcher, left_t, right_t, radius: int, num_disp: int, rank: int, world: int,
                 keys_t=None, out_t=None, stream=None, group=None):
    """One frame, d-sharded over the process group: slice keys -> MIN all-reduce -> disparity."""
    import torch
    lo, hi = dslice_bounds(num_disp, rank, world)
    H, W = left_t.shape[-2:]
    if keys_t is None:
        keys_t = torch.empty((H, W), dtype=torch.int32, device=left_t.device)
    if hi > lo:
        matcher.slice_keys_device(left_t, right_t, radius, lo, hi, keys_t=keys_t, stream=stream)
    else:
        keys_t.fill_(seed_key(radius))
    reduce_slice_keys(keys_t, group)
    return matcher.keys_to_disp_device(keys_t, radius, out_t=out_t, stream=stream)
