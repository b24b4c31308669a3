"""Same-box A/B of the staged kernels' HIP-event times (sm_last_staged_kernel_ms) for several
libsm_hip.so builds, 1080p D=128 r=5 frames, rounds alternated, one process per library and round.
usage: python tools/ab_staged_kernels.py lib1.so lib2.so ... [--rounds N] [--frames F]
(F frames per call, default 8 = one launch group; the kernel times are per frame)"""
import os, statistics, subprocess, sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
libs = [a for a in sys.argv[1:] if a.endswith(".so")]
rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 3
frames = int(sys.argv[sys.argv.index("--frames") + 1]) if "--frames" in sys.argv else 8
CODE = """
import sys; sys.path.insert(0, {root!r})
import numpy as np, torch, gpu_stereo_matching_amd._capi as C
C.load({lib!r})
import gpu_stereo_matching_amd as sm
m = sm.BlockMatcher(0, 1920, 1080, 256)
F = {frames}
pairs = [sm.synth_pair(1234 + i, 1920, 1080, 128) for i in range(F)]
Lt = torch.from_numpy(np.stack([p[0] for p in pairs])).cuda()
Rt = torch.from_numpy(np.stack([p[1] for p in pairs])).cuda()
out = torch.empty_like(Lt)
ref = m.match_device(Lt, Rt, 5, 128, agg='box').cpu().numpy()
acc = []
for i in range(12):
    m.match_device(Lt, Rt, 5, 128, out_t=out, agg='box-staged'); torch.cuda.synchronize()
    if i >= 2: acc.append(m.staged_kernel_ms())
import os
if not os.environ.get('SM_AB_NOCHECK'): assert np.array_equal(out.cpu().numpy(), ref), 'staged map differs from the fused one'
a = np.median(np.array(acc), axis=0)
print('KMS', *a)
"""
P, D = 1920 * 1080, 128
alg = [P * (D + 2), 3 * P * D, 2 * P * D + P]
res = {l: [] for l in libs}
for r in range(rounds):
    for l in libs:
        o = subprocess.run([sys.executable, "-c", CODE.format(root=ROOT, lib=os.path.abspath(l), frames=frames)], capture_output=True,
                           text=True, timeout=300)
        line = [x for x in o.stdout.splitlines() if x.startswith("KMS")]
        if not line:
            print(o.stdout, o.stderr)
            sys.exit(1)
        res[l].append([float(v) for v in line[0].split()[1:]])
for l in libs:
    med = [statistics.median(v[i] for v in res[l]) for i in range(3)]
    fr = [alg[i] / (med[i] * 1e-3) / 8e12 for i in range(3)]
    print(f"{os.path.basename(l):12s} ad {med[0]*1e3:6.1f} us ({fr[0]:.3f})  sad {med[1]*1e3:6.1f} us ({fr[1]:.3f})  "
          f"wta {med[2]*1e3:6.1f} us ({fr[2]:.3f})  of 8 TB/s")
