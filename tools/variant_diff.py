"""Bit-compare guided (and box) maps of libsm_hip.so builds: python tools/variant_diff.py base.so other.so ...
Each library runs in its own process (one HIP library per process); outputs are compared with the first."""
import os, subprocess, sys, tempfile
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_one(lib, out):
    code = f"""
import sys; sys.path.insert(0, {ROOT!r})
import numpy as np, gpu_stereo_matching_amd._capi as C
C.load({lib!r})
import gpu_stereo_matching_amd as sm
g = np.load({os.path.join(ROOT, 'tests', 'golden', 'middlebury_gray.npz')!r})
res = {{}}
L, R = g['Art_/view1'], g['Art_/view5']
sL, sR = sm.synth_pair(7, 1920, 1080, 128)
with sm.BlockMatcher(0, 1920, 1080, 256) as m:
    for r in (1, 3, 5):
        res[f'art_g{{r}}'] = m.match(L, R, r, 64, agg='guided')
        chk, rd, mask = m.match_lr(L, R, r, 64, agg='guided')
        res[f'art_glr{{r}}'] = np.stack([chk, rd, mask])
    res['syn_g5'] = m.match(sL, sR, 5, 128, agg='guided')
    import os as _os
    # box + LR (the fused right view), d_max 128 and 192, several radii
    if _os.environ.get('SM_DIFF_BOXLR'):
        for r in (1, 4, 5, 6):
            res[f'syn_blr{{r}}'] = np.stack(m.match_lr(sL, sR, r, 128))
            res[f'syn_blr{{r}}_d192'] = np.stack(m.match_lr(sL, sR, r, 192))
        res['art_blr5'] = np.stack(m.match_lr(L, R, 5, 64))
        res['syn_blr5_d100'] = np.stack(m.match_lr(sL[:300, :777], sR[:300, :777], 5, 100))
    if _os.environ.get('SM_DIFF_BOX'):
        for r in (0, 1, 2, 3, 4, 5, 6, 7, 9, 15):
            res[f'syn_b{{r}}'] = m.match(sL, sR, r, 128)
        res['syn_b5_d256'] = m.match(sL, sR, 5, 256)
        res['syn_b5_odd'] = m.match(sL[:301, :777], sR[:301, :777], 5, 100)
        for k in ('Art', 'Books', 'Dolls'):
            res[f'mb_{{k}}_b4'] = m.match(g[f'{{k}}/view1'], g[f'{{k}}/view5'], 4, 64)
    if _os.environ.get('SM_DIFF_WIDE'):
        res['syn_w20'] = m.match(sL, sR, 20, 128)
        res['syn_w127lr'] = np.stack(m.match_lr(sL, sR, 127, 128))
        res['syn_w40_odd'] = m.match(sL[:77, :333], sR[:77, :333], 40, 100)
        res['syn_w16_lr'] = np.stack(m.match_lr(sL[:500, :1001], sR[:500, :1001], 16, 64))
        res['syn_w16_d256'] = m.match(sL, sR, 16, 256)
        res['syn_w31_odd'] = m.match(sL[:301, :1003], sR[:301, :1003], 31, 70)
np.savez({out!r}, **res)
"""
    subprocess.run([sys.executable, "-c", code], check=True, timeout=300)


libs = sys.argv[1:]
tmp = tempfile.mkdtemp()
outs = []
for i, lib in enumerate(libs):
    o = os.path.join(tmp, f"{i}.npz")
    run_one(os.path.abspath(lib), o)
    outs.append(np.load(o))
for lib, o in zip(libs[1:], outs[1:]):
    for k in outs[0].files:
        a, b = outs[0][k], o[k]
        print(f"{os.path.basename(lib):14s} {k:10s} differing pixels: {int((a != b).sum())} of {a.size}")
