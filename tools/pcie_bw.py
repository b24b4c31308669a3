"""Pinned host<->device copy bandwidth on one GPU, each direction alone and both at once (for
pipeline.FrameStream's PCIe ceiling)."""
import time
import torch

dev = torch.device("cuda", 0)
n = 64 << 20
h = torch.empty(n, dtype=torch.uint8).pin_memory()
h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
d = torch.empty(n, dtype=torch.uint8, device=dev)
d2 = torch.empty(n, dtype=torch.uint8, device=dev)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def run(fn, reps=10):
    fn()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / reps


def h2d():
    with torch.cuda.stream(s1):
        d.copy_(h, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        h2.copy_(d2, non_blocking=True)


def both():
    h2d()
    d2h()


for name, fn, nbytes in (("H2D", h2d, n), ("D2H", d2h, n), ("H2D+D2H concurrent", both, 2 * n)):
    t = run(fn)
    print(f"{name:20s} {nbytes / t / 1e9:7.1f} GB/s")
