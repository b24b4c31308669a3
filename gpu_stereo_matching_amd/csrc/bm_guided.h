// bm_guided.h — guided-filter cost aggregation (absent from the reference).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sm {

// Per-handle scratch for the guided path (grown on demand, freed in sm_destroy).
struct GuidedWorkspace {
    static constexpr int kChunk = 16;   // disparities per a/b hand-off (a, b planes live in HBM/MALL)
    float* stats = nullptr;             // [3][P] guide stats, [P] best q, [P] best d, [2*kChunk][P] a/b
    size_t stats_bytes = 0;
};

void guided_workspace_free(GuidedWorkspace& ws);

// Guided-filter aggregation + WTA over d in [0, D).  valid_mode as MatchArgs (0: left view,
// threshold 50 and d <= W - x;  1: mirrored right view, d <= x, no threshold).
hipError_t launch_guided_match(GuidedWorkspace& ws, const uint8_t* L, const uint8_t* R, int W, int H, int pitch,
                               int batch, int64_t frame_stride, int radius, int D, float eps, int valid_mode,
                               uint8_t* disp, int out_pitch, int64_t out_frame_stride, hipStream_t s);

}  // namespace sm
