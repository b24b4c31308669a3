"""Streaming-write ceiling of this MI355X, for the staged AD kernel's roofline: time
hipMemsetAsync (torch zero_ on a byte tensor), torch fill_ and a device-to-device copy over buffers the
size of the AD kernel's 8-frame launch (2.16 GB), with HIP events.  Prints GB/s and the fraction of 8 TB/s.
    python tools/write_ceiling.py"""
import json
import torch

N = 2_156_544_000            # AD volume bytes of 8 x 1080p D=128 frames
dev = torch.device("cuda:0")
buf = torch.empty(N, dtype=torch.uint8, device=dev)
src = torch.empty(N // 2, dtype=torch.uint8, device=dev)
dst = torch.empty(N // 2, dtype=torch.uint8, device=dev)
res = {}


def timed(name, fn, nbytes, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    res[name] = {"ms": round(ms, 4), "GBs": round(nbytes / ms / 1e6, 1), "frac_of_8TBs": round(nbytes / ms / 1e6 / 8000, 3)}
    print(name, res[name], flush=True)


timed("memset (zero_ on u8)", lambda: buf.zero_(), N)
timed("fill_ u8 (value 7)", lambda: buf.fill_(7), N)
timed("copy d2d (read + write bytes)", lambda: dst.copy_(src), N)
print(json.dumps(res))
