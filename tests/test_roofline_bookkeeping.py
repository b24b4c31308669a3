"""The bench's VALU roofline reads counters from profiles/ (valu_counts.json, isa_mix_box.json); each entry carries the
sha256 of the machine code it was measured on (tools/codeobj.py).  This CPU test fails when a
kernel those files describe was edited without a re-count, instead of the bench line silently reporting stale
numbers (bench.py reports frac null in that case)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "gpu_stereo_matching_amd", "libsm_hip.so")
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.fixture(scope="module")
def codeobj():
    if not os.path.exists(LIB):
        pytest.skip("libsm_hip.so not built")
    import codeobj as c
    return c


def test_valu_counts_match_the_built_kernels(codeobj):
    counts = json.load(open(os.path.join(ROOT, "profiles", "valu_counts.json")))["kernels"]
    assert counts
    for name, entry in counts.items():
        assert entry.get("code_symbol") and entry.get("code_sha256"), name
        assert codeobj.kernel_sha256(LIB, entry["code_symbol"]) == entry["code_sha256"], (
            f"{name}: {entry['code_symbol']} changed since its counters were taken; re-run tools/valu_counts.py")


def test_isa_mix_matches_the_built_kernel(codeobj):
    mix = json.load(open(os.path.join(ROOT, "profiles", "isa_mix_box.json")))
    assert codeobj.kernel_sha256(LIB, mix["code_symbol"]) == mix["code_sha256"]


def test_hash_is_of_one_kernel(codeobj):
    """A symbol part matching several kernels is an error, not a hash of the first one."""
    with pytest.raises(ValueError):
        codeobj.kernel_code(LIB, "right_reduce_lr_vec_kernel")
    code = codeobj.kernel_code(LIB, "box_match_kernelILi5ELi128ELb0ELi4E")
    assert len(code) > 1000 and len(code) % 4 == 0
