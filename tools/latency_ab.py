"""Batch-1 latency of the plain box matcher under build/env switches, one process per setting (the
switches are read at the first launch): 1080p, 960x540, 640x480, 463x370 and 320x240 frames, device resident,
50 back-to-back calls, HIP events; each map is checked against the first setting's.
usage: python tools/latency_ab.py "SM_WIDE_TILES=0" "SM_WIDE_TILES=1" ..."""
import os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r"""
import sys; sys.path.insert(0, %r)
import numpy as np, torch, gpu_stereo_matching_amd as sm
m = sm.BlockMatcher(0, 1920, 1080, 256)
for (W, H, D, r) in ((1920, 1080, 128, 5), (463, 370, 64, 4), (640, 480, 64, 5), (960, 540, 128, 5), (320, 240, 32, 2)):
    L, R = sm.synth_pair(1234, W, H, D)
    Lt, Rt = torch.from_numpy(L).cuda(), torch.from_numpy(R).cuda()
    o = torch.empty_like(Lt)
    got = m.match_device(Lt, Rt, r, D).cpu().numpy()
    np.save(%r + f"/lat_{W}_{D}_{r}_%s.npy", got)
    for _ in range(5): m.match_device(Lt, Rt, r, D, out_t=o)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50): m.match_device(Lt, Rt, r, D, out_t=o)
    e1.record(); torch.cuda.synchronize()
    print(f"%s {W}x{H} D={D} r={r}: {e0.elapsed_time(e1) / 50 * 1000:.1f} us/call", flush=True)
"""
import tempfile
import numpy as np
td = tempfile.mkdtemp()
settings = sys.argv[1:] or ["SM_WIDE_TILES=0", "SM_WIDE_TILES=1"]
for i, st in enumerate(settings):
    env = dict(os.environ)
    for kv in st.split():
        k, v = kv.split("=")
        env[k] = v
    subprocess.run([sys.executable, "-c", CODE % (ROOT, td, i, st)], env=env, check=True)
for f in sorted(os.listdir(td)):
    if f.endswith("_0.npy"):
        a = np.load(os.path.join(td, f))
        for i in range(1, len(settings)):
            b = np.load(os.path.join(td, f.replace("_0.npy", f"_{i}.npy")))
            print(f"{f[:-6]} setting {i} identical to setting 0: {np.array_equal(a, b)}")
