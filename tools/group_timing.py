"""Host round trip (pageable host frame in, disparity out) of one 1080p D=128 r=5 frame: one handle
vs sm_create_group over the same GPU repeated (row bands on parallel host threads) and, when more
GPUs are visible, over distinct GPUs.  Prints ms per frame (median of 5 runs of 20)."""
import os, statistics, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gpu_stereo_matching_amd as sm
from gpu_stereo_matching_amd import _capi
import ctypes

W, H, D, r = 1920, 1080, 128, 5
L, R = sm.synth_pair(1234, W, H, D)


def timed(fn, n=20, reps=5):
    for _ in range(3):
        fn()
    res = []
    for _ in range(reps):
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        res.append((time.perf_counter() - t0) * 1000 / n)
    return round(statistics.median(res), 4)


m = sm.BlockMatcher(0, W, H, 256)
want = m.match(L, R, r, D)
print("single handle", timed(lambda: m.match(L, R, r, D)), "ms/frame")
n = ctypes.c_int()
_capi.load().sm_device_count(ctypes.byref(n))
configs = [[0, 0], [0, 0, 0, 0]] + ([list(range(n.value))] if n.value > 1 else [])
for devs in configs:
    with sm.BlockMatcherGroup(devs, W, H, 256) as g:
        assert (g.match(L, R, r, D) == want).all()
        print("group", devs, timed(lambda: g.match(L, R, r, D)), "ms/frame")
m.close()
