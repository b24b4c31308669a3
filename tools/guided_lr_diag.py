import sys, os
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import gpu_stereo_matching_amd as sm
from oracle import oracle as O
from guided_check import TOL
EPS = 1e-4 * 255 * 255
W, H, D, r = 1920, 1080, 128, 5
L, R = O.synth_pair(1234, W, H, D)
m = sm.BlockMatcher(0, 3840, 2160, 256)
rds, lefts = [], []
for i in range(4):
    chk, rd, mask = m.match_lr(L, R, r, D, agg="guided")
    rds.append(rd)
    lefts.append(m.match(L, R, r, D, agg="guided"))
print("right maps identical across runs:", [int((rds[0] != x).sum()) for x in rds[1:]])
print("left maps identical across runs:", [int((lefts[0] != x).sum()) for x in lefts[1:]], flush=True)
left, rd = lefts[0], rds[0]
disp_o, best, qL, bestR, qR = O.guided_probe(L, R, r, D, EPS, left, rd)
bad = ~(qR <= bestR + TOL)
ys, xs = np.nonzero(bad)
print("bad right pixels:", len(ys))
for y, x in zip(ys[:5], xs[:5]):
    print(f"  y={y} x={x} gpu dR={rd[y,x]} q(gpu)={qR[y,x]:.6f} best={bestR[y,x]:.6f} diff={qR[y,x]-bestR[y,x]:.6f}")
for k, rr in enumerate(rds[1:]):
    _, _, _, bR2, qR2 = O.guided_probe(L, R, r, D, EPS, left, rr)
    print(f"run {k+1}: bad right pixels {int((~(qR2 <= bR2 + TOL)).sum())}")
