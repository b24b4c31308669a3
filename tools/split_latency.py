"""Batch-1 latency experiment: one 1080p D=128 frame as one launch vs the d-range split into S slices
launched concurrently on S streams (slice keys), MIN-combined and thresholded."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
import gpu_stereo_matching_amd as sm

W, H, D, r = 1920, 1080, 128, 5
m = sm.BlockMatcher(0, W, H, 256)
L, R = sm.synth_pair(1234, W, H, D)
Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
main = torch.cuda.current_stream()
ref = m.match_device(Lt, Rt, r, D, stream=main)
torch.cuda.synchronize()


def timeit(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    for _ in range(n):
        fn()
    e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000


o1 = torch.empty_like(Lt)
print(f"single launch           {timeit(lambda: m.match_device(Lt, Rt, r, D, out_t=o1, stream=main)):7.1f} us")
for S in (2, 3, 4):
    streams = [torch.cuda.Stream() for _ in range(S)]
    keys = [torch.empty((H, W), dtype=torch.int32, device="cuda") for _ in range(S)]
    cuts = [k * D // S for k in range(S + 1)]
    cuts = [c - c % 8 if 0 < c < D else c for c in cuts]

    def split():
        ev = torch.cuda.Event()
        ev.record(main)
        for k in range(S):
            streams[k].wait_event(ev)
            m.slice_keys_device(Lt, Rt, r, cuts[k], cuts[k + 1], keys_t=keys[k], stream=streams[k])
        for k in range(S):
            e = torch.cuda.Event()
            e.record(streams[k])
            main.wait_event(e)
        kk = keys[0]
        for k in range(1, S):
            kk = torch.minimum(kk, keys[k])
        return m.keys_to_disp_device(kk, r, out_t=o1, stream=main)

    t = timeit(split)
    got = split()
    torch.cuda.synchronize()
    print(f"split x{S} on {S} streams  {t:7.1f} us  equal={bool((got == ref).all())}  cuts={cuts}")
