// bm_segtree.h — segment-tree aggregation (STMatching ST-1) on the GPU: internal interface.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

namespace sm {

// Device workspace of segment_tree_match, owned by a handle, grown on demand.
struct StWorkspace {
    uint8_t* w8 = nullptr;     // 3P: edge weights (2P), then the unfiltered map
    float* grad = nullptr;     // 2P: gradients of both views
    float* vol = nullptr;      // 2PD: cost / leaf-to-root sums, filtered cost ([D][P], BFS order)
    int* tree_i = nullptr;     // 5P + 2: rank, parent, first, child, level offsets
    uint8_t* tree_b = nullptr; // P: distance to the parent
    float* table = nullptr;    // 256: exp(-i / (255 sigma))
    size_t w8_n = 0, grad_n = 0, vol_n = 0, tree_i_n = 0, tree_b_n = 0, table_n = 0;
    ~StWorkspace();
    void release();
};

struct StStats {
    int levels = 0;        // BFS levels of the tree
    float tree_ms = 0.f;   // host time of the tree build
};

// stereo_disparity_normal (StereoDisparity.cpp:57-89) on device BGR frames (3 bytes per pixel, row
// pitch `pitch`): D = max_dis_level, tau = TAU (Toolkit.h:34); d_out [H][W] uint8, pitch W.
// Synchronous on stream s (the tree is built on the host from the GPU's edge weights).
hipError_t segment_tree_match(StWorkspace& ws, const uint8_t* dL, const uint8_t* dR, int W, int H, int pitch, int D,
                              int scale, float sigma, float tau, uint8_t* d_out, hipStream_t s, StStats* st);

}  // namespace sm
