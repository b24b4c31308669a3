"""Host frame streams with copies overlapped with matching (cfg5's "pair stream", batched frames).

`FrameStream` keeps a ring of slots (3 by default) of pinned host and device buffers. While batch k is matched on the
compute stream, batch k+1 is uploaded and the disparities of batch k-1 are downloaded, each on its
own stream. One batch is one `sm_match_device` launch over `batch` frames, so the kernel work is
exactly the device-resident path's. The overlap removes the PCIe time from the critical path
whenever a batch's upload + download take less time than its matching.

    fs = FrameStream(matcher, batch=8, width=1920, height=1080, radius=5, num_disp=128)
    for lefts, rights in source:                 # numpy uint8 [batch, H, W] each
        for disp in fs.submit(lefts, rights):    # batches that completed meanwhile, in order
            consume(disp)
    for disp in fs.flush():                      # the batches still in flight
        consume(disp)

With ``bgr=True`` the inputs are the cameras' BGR frames ([batch, H, W, 3]) and with
``rectify_maps=(mapX1, mapY1, mapX2, mapY2)`` (CV_32FC1, e.g. from calib.rectify) each view is
rectified before matching: the reference's capture chain imread/cvtColor (Caller.cpp:12-16) ->
Rectify + remap (Caller.cpp:27-74) -> blockMatching_gpu (Caller.cpp:19), every step on the GPU
on the compute stream, in front of the same batched match.
"""
from __future__ import annotations

from typing import Callable, List, Optional

import numpy as np


class FrameStream:
    def __init__(self, matcher, batch: int, width: int, height: int, radius: int, num_disp: int,
                 agg: str = "box", lr_check: bool = False, device: Optional[int] = None,
                 consume: Optional[Callable[[np.ndarray], None]] = None, slots: int = 3, bgr: bool = False,
                 rectify_maps=None):
        """consume: optional callback given each completed batch as a view of its pinned buffer
        (no host copy; the view is only valid during the call).  Without it, submit()/flush()
        return copies.  bgr: inputs are [batch, H, W, 3] BGR frames, converted on the GPU.
        rectify_maps: (mapX1, mapY1, mapX2, mapY2) float32 [H, W] maps, applied on the GPU."""
        import torch
        self.consume = consume
        self.NS = slots
        self.torch = torch
        self.m = matcher
        self.B, self.W, self.H = batch, width, height
        self.r, self.D, self.agg, self.lr = radius, num_disp, agg, lr_check
        dev = torch.device("cuda", matcher.device if device is None else device)
        self.dev = dev
        shape = (batch, height, width)
        self.bgr = bgr
        in_shape = (batch, height, width, 3) if bgr else shape
        self.in_shape = in_shape
        self.h_in = [(torch.empty(in_shape, dtype=torch.uint8).pin_memory(),
                      torch.empty(in_shape, dtype=torch.uint8).pin_memory()) for _ in range(slots)]
        self.h_out = [torch.empty(shape, dtype=torch.uint8).pin_memory() for _ in range(slots)]
        self.d_in = [(torch.empty(in_shape, dtype=torch.uint8, device=dev),
                      torch.empty(in_shape, dtype=torch.uint8, device=dev)) for _ in range(slots)]
        # front-end stages (compute stream, in front of the match): gray planes, rectified planes
        self.maps = None
        if rectify_maps is not None:
            if len(rectify_maps) != 4 or any(np.shape(mp) != (height, width) for mp in rectify_maps):
                raise ValueError("rectify_maps: four float32 [H, W] maps (mapX1, mapY1, mapX2, mapY2)")
            self.maps = [torch.from_numpy(np.ascontiguousarray(mp, np.float32)).to(dev) for mp in rectify_maps]
        self.d_gray = ((torch.empty(shape, dtype=torch.uint8, device=dev),
                        torch.empty(shape, dtype=torch.uint8, device=dev)) if bgr and self.maps is not None else None)
        self.d_front = ((torch.empty(shape, dtype=torch.uint8, device=dev),
                         torch.empty(shape, dtype=torch.uint8, device=dev)) if (bgr or self.maps is not None) else None)
        self.d_out = [torch.empty(shape, dtype=torch.uint8, device=dev) for _ in range(slots)]
        # uploads, matching and downloads on three streams: upload k+1 and download k-1 run while
        # batch k is matched
        self.s_up = torch.cuda.Stream(dev)
        self.s_comp = torch.cuda.Stream(dev)
        self.s_down = torch.cuda.Stream(dev)
        self.ev_up = [torch.cuda.Event() for _ in range(slots)]
        self.ev_done = [torch.cuda.Event() for _ in range(slots)]
        self.ev_down = [torch.cuda.Event() for _ in range(slots)]
        self.pending: List[int] = []        # slots with a download in flight, oldest first
        self.ready: List[np.ndarray] = []   # completed batches not yet returned
        self.k = 0

    def _collect(self, slot: int) -> Optional[np.ndarray]:
        self.ev_down[slot].synchronize()
        if self.consume is not None:
            self.consume(self.h_out[slot].numpy())
            return None
        return self.h_out[slot].numpy().copy()

    def _free_slot(self) -> int:
        """The slot of the next batch, after collecting the batch that last used it."""
        if len(self.pending) == self.NS:
            r = self._collect(self.pending.pop(0))
            if r is not None:
                self.ready.append(r)
        return self.k % self.NS

    def next_inputs(self):
        """Pinned (left, right) numpy views [batch, H, W] of the next batch: a producer that fills
        them in place (e.g. a capture thread) saves the host copy that submit(lefts, rights) does."""
        slot = self._free_slot()
        hl, hr = self.h_in[slot]
        return hl.numpy(), hr.numpy()

    def submit(self, lefts: Optional[np.ndarray] = None, rights: Optional[np.ndarray] = None) -> List[np.ndarray]:
        """Queue one batch (copied into the pinned slot, or already written through next_inputs());
        returns the disparity batches that completed meanwhile, oldest first (a batch completes
        when its slot comes round again, `slots` submits later)."""
        torch = self.torch
        slot = self._free_slot()
        hl, hr = self.h_in[slot]
        if lefts is not None or rights is not None:
            if lefts.shape != self.in_shape or rights.shape != lefts.shape:
                raise ValueError(f"expected two uint8 arrays of shape {self.in_shape}")
            hl.numpy()[...] = lefts
            hr.numpy()[...] = rights
        dl, dr = self.d_in[slot]
        with torch.cuda.stream(self.s_up):
            dl.copy_(hl, non_blocking=True)
            dr.copy_(hr, non_blocking=True)
            self.ev_up[slot].record(self.s_up)
        self.s_comp.wait_event(self.ev_up[slot])
        ml, mr = self._front(dl, dr)
        self.m.match_device(ml, mr, self.r, self.D, out_t=self.d_out[slot], agg=self.agg, lr_check=self.lr,
                            stream=self.s_comp)
        self.ev_done[slot].record(self.s_comp)
        with torch.cuda.stream(self.s_down):
            self.s_down.wait_event(self.ev_done[slot])
            self.h_out[slot].copy_(self.d_out[slot], non_blocking=True)
            self.ev_down[slot].record(self.s_down)
        self.pending.append(slot)
        self.k += 1
        out, self.ready = self.ready, []
        return out

    def _front(self, dl, dr):
        """BGR -> gray and rectification of one uploaded batch on the compute stream; returns the
        [batch, H, W] planes to match (the front buffers are reused: the compute stream orders the
        next batch's front end after this batch's match)."""
        if self.d_front is None:
            return dl, dr
        fl, fr = self.d_front
        for k, (src, dst) in enumerate(((dl, fl), (dr, fr))):
            for f in range(self.B):
                if self.bgr and self.maps is not None:
                    g = self.d_gray[k][f]
                    self.m.bgr_to_gray_device(src[f], out_t=g, stream=self.s_comp)
                    self.m.remap_device(g, self.maps[2 * k], self.maps[2 * k + 1], out_t=dst[f], stream=self.s_comp)
                elif self.bgr:
                    self.m.bgr_to_gray_device(src[f], out_t=dst[f], stream=self.s_comp)
                else:
                    self.m.remap_device(src[f], self.maps[2 * k], self.maps[2 * k + 1], out_t=dst[f],
                                        stream=self.s_comp)
        return fl, fr

    def flush(self) -> List[np.ndarray]:
        outs = self.ready + [r for r in (self._collect(s) for s in self.pending) if r is not None]
        self.pending, self.ready = [], []
        return outs
