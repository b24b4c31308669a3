"""Drop-in host round trip (sm_block_match_u8, 1080p D=128 r=5) on sm_host_alloc frames and map: DMA upload +
download (SM_ZERO_COPY=0) against DMA upload + zero-copy map (the default).  Each setting runs in its own process,
alternated 3 times; prints the median wall ms per call of each run and the last call's stage split."""
import os, subprocess, sys, statistics
if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import time
    import numpy as np
    import gpu_stereo_matching_amd as sm
    W, H, D, r = 1920, 1080, 128, 5
    L, R = sm.synth_pair(1234, W, H, D)
    with sm.BlockMatcher(0, W, H, 256) as m:
        Op = sm.host_empty((H, W))
        if os.environ.get("SM_AB_NOTIMING") == "1":   # no stage-split events (SM_PARAM_STAGE_TIMING 0)
            m.set_stage_timing(False)
        if os.environ.get("SM_AB_PAIR") == "1":   # the pair in one page-locked block
            pair = sm.host_empty((2, H, W))
            Lp, Rp = pair[0], pair[1]
        else:
            Lp, Rp = sm.host_empty((H, W)), sm.host_empty((H, W))
        Lp[...] = L
        Rp[...] = R
        for _ in range(20):
            m.match(Lp, Rp, r, D, out=Op)
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            m.match(Lp, Rp, r, D, out=Op)
            ts.append(time.perf_counter() - t0)
        print("RESULT", statistics.median(ts) * 1e3, *m.stage_ms())
    sys.exit(0)
SETTINGS = {"dma": {"SM_ZERO_COPY": "0"}, "zc": {"SM_ZERO_COPY": "1"},
            # round 3: the pair in one block, uploaded as one copy (default) or as two (SM_PAIR_COPY=0)
            "zc_pair": {"SM_ZERO_COPY": "1", "SM_AB_PAIR": "1"},
            "zc_pair_2copies": {"SM_ZERO_COPY": "1", "SM_AB_PAIR": "1", "SM_PAIR_COPY": "0"},
            "zc_pair_noev": {"SM_ZERO_COPY": "1", "SM_AB_PAIR": "1", "SM_AB_NOTIMING": "1"},
            # round 4: the start event recorded in every call (round 3) against only with the stage split
            "zc_pair_startev": {"SM_ZERO_COPY": "1", "SM_AB_PAIR": "1", "SM_START_EVENT": "1"},
            "zc_pair_scratchev": {"SM_ZERO_COPY": "1", "SM_AB_PAIR": "1", "SM_SCRATCH_EVENT": "1"}}
res = {k: [] for k in SETTINGS}
for _ in range(3):
    for zc, env in SETTINGS.items():
        out = subprocess.run([sys.executable, __file__, "child"], env=dict(os.environ, **env),
                             capture_output=True, text=True, timeout=200)
        line = [l for l in out.stdout.splitlines() if l.startswith("RESULT")]
        if not line:
            print(out.stdout, out.stderr)
            sys.exit(1)
        res[zc].append([float(v) for v in line[0].split()[1:]])
for zc, name in (("dma", "DMA up + download"), ("zc", "DMA up + zero-copy map"),
                 ("zc_pair", "pair block, one copy + zc map"), ("zc_pair_2copies", "pair block, two copies + zc"),
                 ("zc_pair_noev", "pair block, one copy, no stage events"),
                 ("zc_pair_startev", "pair block, start event every call"),
                 ("zc_pair_scratchev", "pair block, scratch event every pass")):
    walls = [v[0] for v in res[zc]]
    print(f"{name:28s} wall ms/call median {statistics.median(walls):.4f} all {[round(w, 4) for w in walls]} "
          f"last stages upload/match/download {[round(x, 4) for x in res[zc][-1][1:]]}")
