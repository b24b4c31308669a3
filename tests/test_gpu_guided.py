"""Guided-filter aggregation on the GPU vs the fp64 restatement (oracle/bm_oracle.c).

PARITY UNPINNED w.r.t. the reference: it has no guided filter; the build
defines the filter and checks its fp32 HIP path against its own fp64 CPU
restatement.  Tolerance (absolute, in AD units 0..255): a pixel passes when the GPU disparity
equals the oracle's, or when the oracle cost of the GPU's choice is within TOL of the oracle's
best (a near-tie), or when the oracle best is within TOL of the 50.0 threshold and the GPU
reports no match.
"""
import numpy as np
import pytest

from guided_check import tie_aware_check

pytestmark = pytest.mark.gpu
EPS = 1e-4 * 255 * 255


@pytest.fixture(scope="module")
def matcher():
    import gpu_stereo_matching_amd as sm
    m = sm.BlockMatcher(0, 1024, 512, 256)
    m.set_guided_eps(EPS)
    yield m
    m.close()


@pytest.mark.parametrize("r,D", [(5, 64), (3, 32), (0, 16), (7, 48)])
def test_guided_art(matcher, oracle, gray, r, D):
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    disp_o, q, best = oracle.guided_disp(L, R, r, D, EPS, want_q=True)
    got = matcher.match(L, R, r, D, agg="guided")
    ok, exact = tie_aware_check(got, q, {"disp": disp_o, "best": best}, D, L.shape[1])
    assert ok.all(), f"{int((~ok).sum())} pixels outside the tie-aware tolerance"
    assert exact.mean() > 0.995


def test_guided_golden(matcher, gray, guided_expected):
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    got = matcher.match(L, R, 5, 64, agg="guided")
    want = guided_expected["Art_/r5/D64/disp"]
    assert (got == want).mean() > 0.995


@pytest.mark.parametrize("W,H,D,r", [(333, 77, 100, 4), (64, 20, 8, 1), (21, 13, 30, 2)])
def test_guided_synthetic_ragged(matcher, oracle, W, H, D, r):
    L, R = oracle.synth_pair(W + H, W, H, max(D, 16))
    disp_o, q, best = oracle.guided_disp(L, R, r, D, EPS, want_q=True)
    got = matcher.match(L, R, r, D, agg="guided")
    ok, exact = tie_aware_check(got, q, {"disp": disp_o, "best": best}, D, W)
    assert ok.all(), f"{int((~ok).sum())} pixels outside the tie-aware tolerance"


def test_guided_lr(matcher, gray):
    """Guided + LR: the occlusion rule applied to guided left/right maps (checked map is a
    subset of the left map, occluded pixels 0)."""
    L, R = gray["Art_/view1"], gray["Art_/view5"]
    left = matcher.match(L, R, 5, 64, agg="guided")
    chk, rd, mask = matcher.match_lr(L, R, 5, 64, agg="guided")
    assert ((chk == 0) | (chk == left)).all()
    assert (chk[mask == 1] == left[mask == 1]).all()
    assert 0.3 < mask.mean() < 1.0
