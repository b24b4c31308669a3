"""Multi-GPU partitioning of the matching path, one process per GPU.

Three ways to spread the work over ranks:
  * frames (independent rectified pairs): each rank matches its own frames; no collective in the
    data path — the path's natural partition, used for the headline maps/s ("scaling": "weak");
  * disparity slices of ONE frame: rank k scans d in [k*D/G, (k+1)*D/G) and emits per-pixel
    packed keys (SAD << 8 | d); an elementwise MIN gives the global argmin with the reference's
    smallest-d tie break (strict <, Device.cu:57); the threshold / no-match rule is applied after
    the reduction.  Default collective: MIN reduce-scatter of the 4-byte keys, each rank turns
    its 1/G of the pixels into uint8 disparities, all-gather of those bytes — 5P(G-1)/G bytes
    through each rank's links instead of the 8P(G-1)/G of a MIN all-reduce of the keys (xGMI
    is point-to-point, so the ring collectives are per-link bound: SURVEY §8e).  RCCL over xGMI
    on GPUs, gloo on CPU;
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


def dslice_plan_py(pixels: int, num_disp: int, rank: int, world: int) -> Tuple[int, int, int, int]:
    """The same plan as sm_dslice_plan in pure Python (host arithmetic, no device): used where the
    HIP library is not built (CPU-only gloo ranks); tests/test_dslice_plan.py checks that both agree
    whenever the library is present."""
    if pixels <= 0 or num_disp < 1 or world < 1 or not 0 <= rank < world:
        raise ValueError(f"d-slice plan: pixels {pixels}, num_disp {num_disp}, member {rank} of {world}")
    chunk = (pixels + world - 1) // world
    return rank * num_disp // world, (rank + 1) * num_disp // world, chunk, chunk * world


def dslice_plan(pixels: int, num_disp: int, rank: int, world: int) -> Tuple[int, int, int, int]:
    """(d_lo, d_hi, chunk, padded_pixels) of `rank`: the library's own plan (sm_dslice_plan), the
    one sm_group_dslice_block_match_u8 uses, so the torch and C paths cannot drift apart.  Rank k
    scans d in [k*D/G, (k+1)*D/G) (empty when G > D); the keys are padded to G*chunk pixels and the
    reduce-scatter hands rank k pixels [k*chunk, (k+1)*chunk).  Without the HIP library (a CPU-only
    process) the pure-Python twin dslice_plan_py gives the same numbers."""
    import ctypes
    from . import _capi
    try:
        lib = _capi.load()
    except ImportError:
        return dslice_plan_py(pixels, num_disp, rank, world)
    lo, hi = ctypes.c_int(), ctypes.c_int()
    chunk, padded = ctypes.c_int64(), ctypes.c_int64()
    _capi.check(lib.sm_dslice_plan(pixels, num_disp, world, rank, ctypes.byref(lo), ctypes.byref(hi),
                                   ctypes.byref(chunk), ctypes.byref(padded)))
    return lo.value, hi.value, chunk.value, padded.value


def dslice_bounds(num_disp: int, rank: int, world: int) -> Tuple[int, int]:
    """Disparity slice [lo, hi) of `rank`; empty slices are allowed when world > num_disp."""
    lo, hi, _, _ = dslice_plan(1, num_disp, rank, world)
    return lo, hi


def seed_key(radius: int) -> int:
    """(50*win^2) << 8: the reference's start value (Device.cu:37) as a packed key."""
    win = 2 * radius + 1
    return (50 * win * win) << 8


def _host_staged(group) -> bool:
    """gloo takes CPU tensors only for some collectives: device tensors are staged through host
    copies there (the rehearsal mode of bench.py, several ranks on one GPU).  RCCL works in place."""
    import torch.distributed as dist
    return dist.get_backend(group) == "gloo"


def reduce_slice_keys(keys, group=None):
    """In-place signed MIN all-reduce of an int32 key map (box keys are < 2^31 by construction: every
    key is min'ed with the seed (50 win^2) << 8, at most 832,320,000 at r = 127; guided keys carry a
    signed cost)."""
    import torch.distributed as dist
    if keys.is_cuda and _host_staged(group):
        h = keys.cpu()
        dist.all_reduce(h, op=dist.ReduceOp.MIN, group=group)
        keys.copy_(h)
        return keys
    dist.all_reduce(keys, op=dist.ReduceOp.MIN, group=group)
    return keys


def keys_to_disparity_host(keys, radius: int):
    """numpy helper: key map -> uint8 disparity (d if SAD < 50*win^2, else 0)."""
    import numpy as np
    k = keys.astype(np.uint32)
    return np.where((k >> 8) < (seed_key(radius) >> 8), k & 0xFF, 0).astype(np.uint8)


def padded_pixels(height: int, width: int, world: int) -> int:
    """Pixels rounded up to a multiple of the world size (the reduce-scatter chunking)."""
    return dslice_plan(height * width, 1, 0, world)[3]


def dslice_buffers(height: int, width: int, world: int, device):
    """(flat int32 keys, flat uint8 disparity) of padded_pixels(...) elements for match_dslice."""
    import torch
    n = padded_pixels(height, width, world)
    return (torch.empty(n, dtype=torch.int32, device=device), torch.empty(n, dtype=torch.uint8, device=device))


def reduce_scatter_keys(keys_flat, world: int, group=None):
    """MIN reduce-scatter of a flat padded key map: this rank's 1/world chunk of the global minimum."""
    import torch
    import torch.distributed as dist
    chunk = torch.empty(keys_flat.numel() // world, dtype=keys_flat.dtype, device=keys_flat.device)
    if keys_flat.is_cuda and _host_staged(group):
        h = chunk.cpu()
        dist.reduce_scatter_tensor(h, keys_flat.cpu(), op=dist.ReduceOp.MIN, group=group)
        return chunk.copy_(h)
    dist.reduce_scatter_tensor(chunk, keys_flat, op=dist.ReduceOp.MIN, group=group)
    return chunk


def gather_disparity(chunk_u8, out_flat, group=None):
    """All-gather of the per-rank uint8 disparity chunks into the flat padded map."""
    import torch.distributed as dist
    if out_flat.is_cuda and _host_staged(group):
        h = out_flat.cpu()
        dist.all_gather_into_tensor(h, chunk_u8.cpu(), group=group)
        return out_flat.copy_(h)
    dist.all_gather_into_tensor(out_flat, chunk_u8, group=group)
    return out_flat


GUIDED_EMPTY_KEY = 0x7FFFFFFF   # guided slice key of a pixel with no valid d (INT32_MAX)
RIGHT_EMPTY_KEY = 0x7FFFFFFF    # right-view slice key of a pixel no d of the slice reaches (box and guided)


def lr_check_host(left_disp, right_disp):
    """numpy twin of sm_lr_check_device (StereoDisparity.cpp:136-147): d = dL(x); occluded when x - d < 0,
    d == 0 or |d - dR(x - d)| > 1; returns (checked map, valid mask)."""
    import numpy as np
    dl = np.asarray(left_disp, np.int64)
    dr = np.asarray(right_disp, np.int64)
    H, W = dl.shape
    x = np.arange(W)[None, :]
    src = x - dl
    inb = src >= 0
    got = np.take_along_axis(dr, np.clip(src, 0, W - 1), axis=1)
    occ = ~inb | (dl == 0) | (np.abs(dl - got) > 1)
    return np.where(occ, 0, dl).astype(np.uint8), (~occ).astype(np.uint8)


def match_dslice(matcher, left_t, right_t, radius: int, num_disp: int, rank: int, world: int,
                 keys_t=None, out_t=None, stream=None, group=None, collective: str = "rs_ag", agg: str = "box",
                 lr_check: bool = False, right_bufs=None):
    """One frame, d-sharded over the process group: slice keys -> MIN reduce -> disparity.

    collective "rs_ag" (default): reduce-scatter the keys, convert this rank's chunk, all-gather
    uint8; "allreduce": MIN all-reduce of the whole key map, then convert.  keys_t / out_t: the
    flat buffers of dslice_buffers() (allocated when None).  agg "guided": the keys are the guided
    path's signed (q * 2^14) << 8 | d (the same MIN collectives; padding / empty slices hold
    INT32_MAX, the threshold q < 50 is applied after the reduction).  lr_check: the slice pass also
    emits the right view's keys (C_R(u, d) = C_L(u + d, d), StereoHelper.cpp:156-180, one fused pass:
    sm_slice_keys_lr_device), which take the same MIN collective ("LR adds a second packed reduction
    for the right view"); their d fields form dR and StereoDisparity.cpp:136-147 checks the
    map.  right_bufs: a second dslice_buffers() pair for the right view (allocated when None).
    Returns the [H, W] disparity."""
    import torch
    if collective not in ("rs_ag", "allreduce"):
        raise ValueError("collective must be 'rs_ag' or 'allreduce'")
    if lr_check:
        return _match_dslice_lr(matcher, left_t, right_t, radius, num_disp, rank, world, keys_t, out_t, stream,
                                group, collective, agg, right_bufs)
    if agg == "box":
        fill = seed_key(radius)
        slice_keys = lambda lo, hi, k: matcher.slice_keys_device(left_t, right_t, radius, lo, hi,  # noqa: E731
                                                                 keys_t=k, stream=stream)
        to_disp = lambda k, o=None: matcher.keys_to_disp_device(k, radius, out_t=o)  # noqa: E731
    elif agg == "guided":
        fill = GUIDED_EMPTY_KEY
        slice_keys = lambda lo, hi, k: matcher.guided_slice_keys_device(left_t, right_t, radius, lo, hi,  # noqa: E731
                                                                        keys_t=k, stream=stream)
        to_disp = lambda k, o=None: matcher.guided_keys_to_disp_device(k, out_t=o)  # noqa: E731
    else:
        raise ValueError("agg must be 'box' or 'guided'")
    lo, hi = dslice_bounds(num_disp, rank, world)
    H, W = left_t.shape[-2:]
    P = H * W
    if keys_t is None or out_t is None:
        keys_t, out_t = dslice_buffers(H, W, world, left_t.device)
    if keys_t.numel() != padded_pixels(H, W, world) or out_t.numel() != keys_t.numel():
        raise ValueError("keys_t / out_t must be dslice_buffers(H, W, world)")
    keys_img = keys_t[:P].view(H, W)
    if stream is not None:   # frames and keys_t (last read by the previous collective) belong to the current stream
        stream.wait_stream(torch.cuda.current_stream(left_t.device))
    if hi > lo:
        slice_keys(lo, hi, keys_img)
    else:
        keys_img.fill_(fill)
    keys_t[P:].fill_(fill)
    if stream is not None:
        torch.cuda.current_stream(left_t.device).wait_stream(stream)
    if collective == "allreduce":
        reduce_slice_keys(keys_t, group)
        to_disp(keys_t.view(1, -1), out_t.view(1, -1))
        return out_t[:P].view(H, W)
    chunk = reduce_scatter_keys(keys_t, world, group)
    n = chunk.numel()
    mine = to_disp(chunk.view(1, n))
    gather_disparity(mine.view(n), out_t, group)
    return out_t[:P].view(H, W)


def _match_dslice_lr(matcher, left_t, right_t, radius, num_disp, rank, world, keys_t, out_t, stream, group,
                     collective, agg, right_bufs):
    import torch
    if agg not in ("box", "guided"):
        raise ValueError("agg must be 'box' or 'guided'")
    fill = GUIDED_EMPTY_KEY if agg == "guided" else seed_key(radius)
    to_disp = ((lambda k, o=None: matcher.guided_keys_to_disp_device(k, out_t=o)) if agg == "guided"  # noqa: E731
               else (lambda k, o=None: matcher.keys_to_disp_device(k, radius, out_t=o)))
    lo, hi = dslice_bounds(num_disp, rank, world)
    H, W = left_t.shape[-2:]
    P = H * W
    if keys_t is None or out_t is None:
        keys_t, out_t = dslice_buffers(H, W, world, left_t.device)
    rkeys_t, rout_t = right_bufs if right_bufs is not None else dslice_buffers(H, W, world, left_t.device)
    n_pad = padded_pixels(H, W, world)
    for t in (keys_t, out_t, rkeys_t, rout_t):
        if t.numel() != n_pad:
            raise ValueError("keys_t / out_t / right_bufs must be dslice_buffers(H, W, world)")
    keys_img, rkeys_img = keys_t[:P].view(H, W), rkeys_t[:P].view(H, W)
    if stream is not None:
        stream.wait_stream(torch.cuda.current_stream(left_t.device))
    if hi > lo:
        matcher.slice_keys_lr_device(left_t, right_t, radius, lo, hi, agg=agg, keys_t=keys_img,
                                     right_keys_t=rkeys_img, stream=stream)
    else:
        keys_img.fill_(fill)
        rkeys_img.fill_(RIGHT_EMPTY_KEY)
    keys_t[P:].fill_(fill)
    rkeys_t[P:].fill_(RIGHT_EMPTY_KEY)
    if stream is not None:
        torch.cuda.current_stream(left_t.device).wait_stream(stream)
    if collective == "allreduce":
        reduce_slice_keys(keys_t, group)
        reduce_slice_keys(rkeys_t, group)
        to_disp(keys_t.view(1, -1), out_t.view(1, -1))
        matcher.right_keys_to_disp_device(rkeys_t, out_t=rout_t)
    else:
        chunk = reduce_scatter_keys(keys_t, world, group)
        rchunk = reduce_scatter_keys(rkeys_t, world, group)
        n = chunk.numel()
        gather_disparity(to_disp(chunk.view(1, n)).view(n), out_t, group)
        gather_disparity(matcher.right_keys_to_disp_device(rchunk), rout_t, group)
    img = out_t[:P].view(H, W)
    return matcher.lr_check_device(img, rout_t[:P].view(H, W), out_t=img)


GUIDED_SEED_Q = 50 * 16384   # q < 50 in the guided keys' 2^-14 fixed point (Device.cu:37 seed)


def guided_keys_to_disparity_host(keys):
    """numpy twin of sm_guided_keys_to_disp_device: signed key map -> d where q < 50, else 0."""
    import numpy as np
    k = np.asarray(keys, np.int32)
    return np.where((k >> 8) < GUIDED_SEED_Q, k & 0xFF, 0).astype(np.uint8)


def match_dslice_host_keys(keys, radius: int, world: int, collective: str = "rs_ag", group=None, agg: str = "box",
                           right_keys=None):
    """CPU (gloo) form of match_dslice's reduction for tests: this rank's [H, W] slice keys (int32
    numpy) -> the [H, W] uint8 disparity of the global minimum, through the same collectives.
    agg "guided": signed guided keys, INT32_MAX padding, threshold q < 50.  right_keys: this rank's
    right-view slice keys; they take the same reduction, their d fields form dR, and the map is
    LR-checked (lr_check_host) — match_dslice(lr_check=True)'s data flow."""
    import numpy as np
    import torch
    H, W = keys.shape
    P = H * W
    if right_keys is not None:
        left = match_dslice_host_keys(keys, radius, world, collective, group, agg)
        flat = torch.full((padded_pixels(H, W, world),), RIGHT_EMPTY_KEY, dtype=torch.int32)
        flat[:P] = torch.from_numpy(np.ascontiguousarray(right_keys, np.int32).reshape(P))
        if collective == "allreduce":
            reduce_slice_keys(flat, group)
            right = (flat.numpy()[:P] & 0xFF).astype(np.uint8)
        else:
            chunk = reduce_scatter_keys(flat, world, group)
            out = torch.empty(flat.numel(), dtype=torch.uint8)
            gather_disparity(torch.from_numpy((chunk.numpy() & 0xFF).astype(np.uint8)), out, group)
            right = out.numpy()[:P]
        return lr_check_host(left, right.reshape(H, W))[0]
    if agg == "guided":
        fill = GUIDED_EMPTY_KEY
        finish = lambda k: guided_keys_to_disparity_host(k)   # noqa: E731
    else:
        fill = seed_key(radius)
        finish = lambda k: keys_to_disparity_host(k.view(np.uint32), radius)   # noqa: E731
    flat = torch.full((padded_pixels(H, W, world),), fill, dtype=torch.int32)
    flat[:P] = torch.from_numpy(np.ascontiguousarray(keys, np.int32).reshape(P))
    if collective == "allreduce":
        reduce_slice_keys(flat, group)
        return finish(flat.numpy()[:P]).reshape(H, W)
    chunk = reduce_scatter_keys(flat, world, group)
    mine = torch.from_numpy(finish(chunk.numpy()))
    out = torch.empty(flat.numel(), dtype=torch.uint8)
    gather_disparity(mine, out, group)
    return out.numpy()[:P].reshape(H, W)


def band_rows(height: int, rank: int, world: int) -> Tuple[int, int]:
    """Output rows [y0, y1) of `rank`: equal bands of ceil(H/G) rows (the last may be short or empty)."""
    n = -(-height // world)
    y0 = min(height, rank * n)
    return y0, min(height, y0 + n)


MEDIAN_RADIUS = 3   # SM_MEDIAN: 7x7 post-filter (StereoDisparity.cpp:85)


BAND_ALIGN = 32   # band inputs start on the frame's 32-row tile grid (sm_capi.hip group_bands)


def band_halo(radius: int, agg: str = "box", median: bool = False) -> int:
    """Input rows needed on each side of an output band: the aggregation window (for the guided
    filter's two nested windows 2r, at least 16 so that its 8-row float running sums of the kept
    rows start on rows the band holds) plus the median's 3 rows when the post-filter is on."""
    return (max(2 * radius, 16) if agg == "guided" else radius) + (MEDIAN_RADIUS if median else 0)


def band_input_rows(height: int, y0: int, y1: int, halo: int) -> Tuple[int, int]:
    """Input rows [ys, ye) of output band [y0, y1): ys floored to the 32-row tile grid."""
    ys = 0 if y0 - halo <= 0 else ((y0 - halo) // BAND_ALIGN) * BAND_ALIGN
    return ys, min(height, y1 + halo)


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
    if stream is not None:   # the frames were written on the current stream
        stream.wait_stream(torch.cuda.current_stream(left_t.device))
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
