"""Multi-GPU partitioning of the matching path, one process per GPU.

Three ways to spread the work over ranks:
  * frames (independent rectified pairs): each rank matches its own frames; no collective in the
    data path — the path's natural partition, used for the headline maps/s ("scaling": "weak");
  * disparity slices of ONE frame: rank k scans d in [k*D/G, (k+1)*D/G) and emits per-pixel
    packed keys (SAD << 8 | d); an elementwise MIN all-reduce (RCCL over xGMI on GPUs, gloo on
    CPU) gives the global argmin with the reference's smallest-d tie break (strict <,
    Device.cu:57); the threshold / no-match rule is applied after the reduction;
  * row bands of ONE frame: rank k owns output rows [k*ceil(H/G), ...) and matches them from its
    rows plus a halo (r rows for box windows, 2r for the guided filter's two nested windows, +3
    with the 7x7 median post-filter);
    a window never reaches past the halo, so each band equals the same rows of the full-frame
    result, and one all-gather of uint8 bands (H*W bytes in total) assembles the map.
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


def band_rows(height: int, rank: int, world: int) -> Tuple[int, int]:
    """Output rows [y0, y1) of `rank`: equal bands of ceil(H/G) rows (the last may be short or empty)."""
    n = -(-height // world)
    y0 = min(height, rank * n)
    return y0, min(height, y0 + n)


MEDIAN_RADIUS = 3   # SM_MEDIAN: 7x7 post-filter (StereoDisparity.cpp:85)


def band_halo(radius: int, agg: str = "box", median: bool = False) -> int:
    """Input rows needed on each side of an output band: the aggregation window (2r for the
    guided filter's two nested windows) plus the median's 3 rows when the post-filter is on."""
    return (2 * radius if agg == "guided" else radius) + (MEDIAN_RADIUS if median else 0)


def band_input_rows(height: int, y0: int, y1: int, halo: int) -> Tuple[int, int]:
    return max(0, y0 - halo), min(height, y1 + halo)


def gather_bands(mine, height: int, world: int, group=None):
    """All-gather equal [ceil(H/G), W] bands (rows past a rank's band are padding) -> [H, W]."""
    import torch
    import torch.distributed as dist
    parts = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine, group=group)
    return torch.cat(parts)[:height]


def band_disparity(matcher, left_t, right_t, radius: int, num_disp: int, y0: int, y1: int, agg: str = "box",
                   lr_check: bool = False, stream=None, median: bool = False):
    """Disparity rows [y0, y1) of an [H, W] device frame, matched from those rows plus the halo."""
    import torch
    H = left_t.shape[-2]
    ys, ye = band_input_rows(H, y0, y1, band_halo(radius, agg, median))
    band = matcher.match_device(left_t[ys:ye], right_t[ys:ye], radius, num_disp, agg=agg, lr_check=lr_check,
                                stream=stream, median=median)
    if stream is not None:
        torch.cuda.current_stream(left_t.device).wait_stream(stream)
    return band[y0 - ys:y1 - ys]


def match_rowband(matcher, left_t, right_t, radius: int, num_disp: int, rank: int, world: int, agg: str = "box",
                  lr_check: bool = False, out_t=None, stream=None, group=None, median: bool = False):
    """One [H, W] frame, row-sharded: this rank's band (with halo) -> all-gather -> full map on every rank."""
    import torch
    H, W = left_t.shape[-2:]
    n = -(-H // world)
    y0, y1 = band_rows(H, rank, world)
    mine = torch.zeros((n, W), dtype=torch.uint8, device=left_t.device)
    if y1 > y0:
        mine[:y1 - y0].copy_(band_disparity(matcher, left_t, right_t, radius, num_disp, y0, y1, agg, lr_check, stream,
                                            median))
    res = gather_bands(mine, H, world, group)
    if out_t is not None:
        out_t.copy_(res)
        return out_t
    return res
