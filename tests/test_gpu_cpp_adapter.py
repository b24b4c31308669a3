"""The C++ drop-in path: examples/Main.cpp -> singleFrame() -> blockMatching_gpu(Mat&...) ->
C ABI -> HIP, compared with the golden map of Caller.cpp:19's configuration."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "build", "single_frame")


def _write_pgm(path, a):
    with open(path, "wb") as f:
        f.write(b"P5\n%d %d\n255\n" % (a.shape[1], a.shape[0]))
        f.write(np.ascontiguousarray(a).tobytes())


def _read_pgm(path):
    with open(path, "rb") as f:
        data = f.read()
    parts = data.split(b"\n", 3)
    w, h = (int(v) for v in parts[1].split())
    return np.frombuffer(parts[3], np.uint8).reshape(h, w)


def test_example_builds():
    assert os.path.exists(EXE), "examples/build/single_frame missing: run __graft_entry__.build()"


CVMAT_SRC = os.path.join(ROOT, "tests", "native", "cvmat_single_frame.cpp")
CVMAT_EXE = os.path.join(ROOT, "examples", "build", "cvmat_single_frame")


def test_cvmat_branch_compiles(tmp_path):
    """stereo_bm.hpp's SM_WITH_OPENCV branch (blockMatching_gpu / testBM on cv::Mat, whose step is a
    cv::MatStep) instantiates and links against libsm_hip.so.  OpenCV is absent: the test's own
    minimal cv::Mat declares only the members the adapter touches (tests/native/cvmat_single_frame.cpp)."""
    r = subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                        CVMAT_SRC, "-o", str(tmp_path / "cvm"), "-L" + os.path.join(ROOT, "gpu_stereo_matching_amd"),
                        "-lsm_hip"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_cvmat_single_frame_cpp(tmp_path, gray, bm_expected):
    """singleFrame() (Caller.cpp:9-25) on the cv::Mat-shaped type, rows padded to 64 bytes: the golden
    map of Caller.cpp:19's configuration, and testBM agrees with blockMatching_gpu."""
    _write_pgm(tmp_path / "l.pgm", gray["Art_/view1"])
    _write_pgm(tmp_path / "r.pgm", gray["Art_/view5"])
    r = subprocess.run([CVMAT_EXE, str(tmp_path / "l.pgm"), str(tmp_path / "r.pgm"), str(tmp_path / "d.pgm"), "5",
                        "64"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(_read_pgm(tmp_path / "d.pgm"), bm_expected["Art_/r5/D64"])


@pytest.mark.gpu
@pytest.mark.parametrize("pair,sad,rng", [("Art_", 5, 64), ("Books", 4, 64)])
def test_single_frame_cpp(tmp_path, gray, bm_expected, pair, sad, rng):
    _write_pgm(tmp_path / "l.pgm", gray[f"{pair}/view1"])
    _write_pgm(tmp_path / "r.pgm", gray[f"{pair}/view5"])
    env = dict(os.environ, SM_LEFT=str(tmp_path / "l.pgm"), SM_RIGHT=str(tmp_path / "r.pgm"),
               SM_OUT=str(tmp_path / "d.pgm"), SM_SAD=str(sad), SM_RANGE=str(rng))
    env.pop("SM_QUIET", None)
    r = subprocess.run([EXE], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    # Device.cu:218,238,257,292: the four stage lines, in order, always printed (ms; the upload, match
    # and download times are the recorded hipEvent split, "pre calculation" is fused and reads 0)
    lines = r.stdout.splitlines()
    labels = [ln.split(" : ")[0] for ln in lines if " : " in ln]
    assert labels[:4] == ["upload data", "pre calculation", "find corr", "download data"], r.stdout
    vals = {ln.split(" : ")[0]: float(ln.split(" : ")[1]) for ln in lines[:4]}
    assert vals["upload data"] > 0 and vals["find corr"] > 0 and vals["download data"] > 0
    assert vals["pre calculation"] == 0
    assert "GPU : " in r.stdout
    env["SM_QUIET"] = "1"
    r = subprocess.run([EXE], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "find corr" not in r.stdout
    got = _read_pgm(tmp_path / "d.pgm")
    assert np.array_equal(got, bm_expected[f"{pair}/r{sad}/D{rng}"])


@pytest.mark.gpu
def test_single_frame_cpp_wide_window(tmp_path, gray, oracle):
    """An unchanged singleFrame() caller with SADWindowSize 20 (41 x 41, Device.cu's unbounded window):
    blockMatching_gpu runs the separable wide-window path (bm_wide.hip) and writes the oracle's map."""
    L, R = gray["Art/view1"], gray["Art/view5"]
    _write_pgm(tmp_path / "l.pgm", L)
    _write_pgm(tmp_path / "r.pgm", R)
    env = dict(os.environ, SM_LEFT=str(tmp_path / "l.pgm"), SM_RIGHT=str(tmp_path / "r.pgm"),
               SM_OUT=str(tmp_path / "d.pgm"), SM_SAD="20", SM_RANGE="64", SM_QUIET="1")
    r = subprocess.run([EXE], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(_read_pgm(tmp_path / "d.pgm"), oracle.box_disp(L, R, 20, 64))


@pytest.mark.gpu
def test_single_frame_cpp_device_group(tmp_path, gray, bm_expected):
    """SM_DEVICES=0,0,0: the unchanged singleFrame() caller runs through a 3-member group handle
    (row bands, one per member) and still writes the golden map."""
    _write_pgm(tmp_path / "l.pgm", gray["Books/view1"])
    _write_pgm(tmp_path / "r.pgm", gray["Books/view5"])
    env = dict(os.environ, SM_LEFT=str(tmp_path / "l.pgm"), SM_RIGHT=str(tmp_path / "r.pgm"),
               SM_OUT=str(tmp_path / "d.pgm"), SM_SAD="4", SM_RANGE="64", SM_DEVICES="0,0,0")
    r = subprocess.run([EXE], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(_read_pgm(tmp_path / "d.pgm"), bm_expected["Books/r4/D64"])


@pytest.mark.gpu
def test_single_frame_cpp_dslice_group(tmp_path, gray, bm_expected):
    """SM_GROUP_MODE=dslice: the unchanged singleFrame() caller (Caller.cpp:19 -> blockMatching_gpu)
    runs through the RCCL d-slice group mode (a one-rank communicator on the test box's one GPU:
    slice keys, MIN reduce-scatter, finalise, all-gather) and still writes the golden map."""
    _write_pgm(tmp_path / "l.pgm", gray["Books/view1"])
    _write_pgm(tmp_path / "r.pgm", gray["Books/view5"])
    env = dict(os.environ, SM_LEFT=str(tmp_path / "l.pgm"), SM_RIGHT=str(tmp_path / "r.pgm"),
               SM_OUT=str(tmp_path / "d.pgm"), SM_SAD="4", SM_RANGE="64", SM_GROUP_MODE="dslice")
    env.pop("SM_DEVICES", None)
    r = subprocess.run([EXE], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(_read_pgm(tmp_path / "d.pgm"), bm_expected["Books/r4/D64"])


@pytest.mark.gpu
def test_remap_test_cpp(tmp_path, oracle):
    """remapTest() (Caller.cpp:27-74) end to end through stereo_bm.hpp: LoadDataBatch of the reference's
    calibration YAML -> Rectify (stereoRectify + GPU maps) -> remap_gpu on the Chess/Set2 pair at
    320x200.  Maps bit-exact with the oracle's initUndistortRectifyMap on the same R/P, and both
    rectified views bit-exact with the CPU_Remap restatement."""
    from gpu_stereo_matching_amd import calib
    chess = np.load(os.path.join(ROOT, "tests", "golden", "chess_set2_gray.npz"))
    L, R = chess["Left_320x200"], chess["Right_320x200"]
    H, W = L.shape
    yml = os.path.join(ROOT, "tests", "golden", "Calib_Data_OpenCV.yml")
    _write_pgm(tmp_path / "l.pgm", L)
    _write_pgm(tmp_path / "r.pgm", R)
    env = dict(os.environ, SM_DEMO="remapTest", SM_LEFT=str(tmp_path / "l.pgm"), SM_RIGHT=str(tmp_path / "r.pgm"),
               SM_CALIB=yml, SM_OUT=str(tmp_path / "o.pgm"), SM_OUT2=str(tmp_path / "o2.pgm"),
               SM_MAPS=str(tmp_path / "maps.f32"))
    r = subprocess.run([EXE], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "GPU Remap : " in r.stdout
    K1, K2, d1, d2, Rm, T = calib.load_data_batch(yml)
    R1, R2, P1, P2, _ = calib.stereo_rectify(K1, d1, K2, d2, (W, H), Rm, T)
    mx1, my1 = oracle.init_rectify_map(K1, d1, R1, P1, W, H)
    mx2, my2 = oracle.init_rectify_map(K2, d2, R2, P2, W, H)
    maps = np.fromfile(tmp_path / "maps.f32", np.float32).reshape(4, H, W)
    for got, want in zip(maps, (mx1, my1, mx2, my2)):
        assert np.array_equal(got, want)
    assert np.array_equal(_read_pgm(tmp_path / "o.pgm"), oracle.remap(L, mx1, my1))
    assert np.array_equal(_read_pgm(tmp_path / "o2.pgm"), oracle.remap(R, mx2, my2))


@pytest.mark.gpu
def test_cvtcolor_test_cpp(tmp_path, gray, oracle):
    """cvtColorTest() -> cvtColor_gpu(uchar3*...) (Device.cuh:52): OpenCV 2.4 BGR2GRAY, bit-exact."""
    bgr = gray["Art_/view1_bgr"]
    with open(tmp_path / "c.ppm", "wb") as f:
        f.write(b"P6\n%d %d\n255\n" % (bgr.shape[1], bgr.shape[0]))
        f.write(np.ascontiguousarray(bgr[..., ::-1]).tobytes())        # RGB on disk
    env = dict(os.environ, SM_DEMO="cvtColorTest", SM_BGR=str(tmp_path / "c.ppm"), SM_OUT=str(tmp_path / "g.pgm"))
    r = subprocess.run([EXE], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    got = _read_pgm(tmp_path / "g.pgm")
    assert np.array_equal(got, oracle.bgr_to_gray(bgr))
    assert np.array_equal(got, gray["Art_/view1"])


def _sections(stdout: str):
    """stdout of blockMatchingApiTest split at its "== name" markers -> {name: [lines]}"""
    out, cur = {}, None
    for ln in stdout.splitlines():
        if ln.startswith("== "):
            cur = ln[3:]
            out[cur] = []
        elif cur is not None and ln:
            out[cur].append(ln)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("pair,sad", [("Art", 3), ("Books", 9)])
def test_blockmatching_h_api_cpp(tmp_path, gray, bm_expected, oracle, pair, sad):
    """All seven BlockMatching.h functions (BlockMatching.h:8-15) through stereo_bm.hpp, in one C++
    caller: testBM / getDisp maps and the PreCal volume against the oracle, getAllSAD's pixel-major
    uchar volume bit-exact against ora_get_all_sad (BlockMatching.cpp:191-261; r = 9 takes the direct
    kernel, r = 3 the volume + transpose path), and compareDiff / compareDisp / compareSAD printing
    the reference's format (BlockMatching.cpp:263-308): nothing but "-1" on the computed results, and
    exactly the planted index on a corrupted copy."""
    L, R = gray[f"{pair}/view1"], gray[f"{pair}/view5"]
    H, W = L.shape
    _write_pgm(tmp_path / "l.pgm", L)
    _write_pgm(tmp_path / "r.pgm", R)
    env = dict(os.environ, SM_DEMO="blockMatchingApiTest", SM_LEFT=str(tmp_path / "l.pgm"),
               SM_RIGHT=str(tmp_path / "r.pgm"), SM_SAD=str(sad), SM_RANGE="64", SM_OUT=str(tmp_path / "a.pgm"),
               SM_OUT2=str(tmp_path / "b.pgm"), SM_VOL=str(tmp_path / "v.u8"), SM_SADVOL=str(tmp_path / "s.u8"))
    env.pop("SM_QUIET", None)
    r = subprocess.run([EXE], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    want = bm_expected[f"{pair}/r{sad}/D64"] if f"{pair}/r{sad}/D64" in bm_expected else oracle.box_disp(L, R, sad, 64)
    assert np.array_equal(_read_pgm(tmp_path / "a.pgm"), want)
    assert np.array_equal(_read_pgm(tmp_path / "b.pgm"), want)
    vol = np.fromfile(tmp_path / "v.u8", np.uint8).reshape(64, H, W)
    assert np.array_equal(vol, oracle.precal(L, R, 64))
    allsad = np.fromfile(tmp_path / "s.u8", np.uint8).reshape(H, W, 64)
    assert np.array_equal(allsad, oracle.get_all_sad(L, R, sad, 64))
    sec = _sections(r.stdout)
    # BlockMatching.cpp's step lines around each call (getDisp inside compareDisp prints them too)
    assert "main loop" in r.stdout and "precalculate diff" in r.stdout and "prep location" in r.stdout
    assert sec["compareDiff clean"] == ["-1"]
    assert [ln for ln in sec["compareDisp clean"] if ln.startswith(("[", "CPU"))] == []
    assert [ln for ln in sec["compareSAD clean"] if not ln.startswith(("prep", "precalculate"))] == ["-1"]
    assert sec["compareDiff planted"] == ["7", "-1"]
    d = int(want[1, 2])
    assert [ln for ln in sec["compareDisp planted"] if ln.startswith(("[", "CPU"))] == \
        ["[1:2]", f"CPU = {d}, GPU = {d ^ 1}"]
    assert [ln for ln in sec["compareSAD planted"] if not ln.startswith(("prep", "precalculate"))] == ["5", "-1"]


@pytest.mark.gpu
def test_single_frame_cpp_device_cu_grid(tmp_path, gray):
    """SM_DEVICE_CU_GRID=1: an unchanged blockMatching_gpu caller gets Device.cu's literal map (its fixed
    launch grid covers rows < 256, cols < 320 only, Device.cu:231-233) on a 463x370 bundled pair."""
    exp = np.load(os.path.join(ROOT, "tests", "golden", "device_cu_expected.npz"))
    _write_pgm(tmp_path / "l.pgm", gray["Books/view1"])
    _write_pgm(tmp_path / "r.pgm", gray["Books/view5"])
    env = dict(os.environ, SM_LEFT=str(tmp_path / "l.pgm"), SM_RIGHT=str(tmp_path / "r.pgm"),
               SM_OUT=str(tmp_path / "d.pgm"), SM_SAD="4", SM_RANGE="64", SM_QUIET="1", SM_DEVICE_CU_GRID="1")
    r = subprocess.run([EXE], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert np.array_equal(_read_pgm(tmp_path / "d.pgm"), exp["Books/r4/D64"])
