// bm_segtree.h — segment-tree aggregation (STMatching ST-1 and ST-2) on the GPU: internal interface.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

namespace sm {

// Device workspace of segment_tree_match, owned by a handle, grown on demand.
struct StWorkspace {
    uint8_t* w8 = nullptr;     // ST-1 3P: edge weights (2P), then the unfiltered map; ST-2 10P: both views'
                               // weights (4P), then the pass maps, the checked map and the mask
    float* grad = nullptr;     // 2P: gradients of both views
    float* vol = nullptr;      // ST-1 2PD, ST-2 4PD: cost / leaf-to-root sums, filtered cost ([D][P], BFS order)
    int* tree_i = nullptr;     // (5P + 2) per tree: rank, parent, first, child, level offsets
    uint8_t* tree_b = nullptr; // P per tree: distance to the parent
    float* table = nullptr;    // 256 per tree: exp(-i / (255 sigma))
    int* task = nullptr;       // per tree: the wave filter's level tasks (int4 each), up to 2 * (P + levels)
    int* bfs[2] = {nullptr, nullptr};   // the device BFS's scratch per tree slot (round 4, bm_segtree.hip: bfs_scratch)
    hipStream_t side = nullptr;         // ST-2: the right view's BFS runs on it beside the left's
    hipEvent_t side_ev = nullptr;       // recorded on `side` after that BFS
    int* node = nullptr;       // P per tree: BFS index -> pixel (the WTA's output order)
    size_t node_n = 0;
    int* h_hdr = nullptr;      // page-locked: per tree slot {levels, widest level, up tasks, down tasks}
    hipEvent_t bfs_ev = nullptr;   // recorded after the device BFS's header copies
    int last_P = 0, last_nlev = 0; // tree slot 0 of the last call (sm_last_segment_tree_arrays)
    uint32_t* sortbuf = nullptr;   // edge sort: keys and values (2 x 2 nE), digit counts, sorted edges (3 nE)
    void* h_edges[2] = {nullptr, nullptr};   // page-locked host copies of sorted edges (12 B each), 2 trees
    // round 4, per edge slot: the sorted edges on the device (12 B each) and each grid edge's sorted
    // position (2P); the host passes' per-edge marks, page-locked (nE bytes)
    uint32_t* dedge[2] = {nullptr, nullptr};
    int* sidx[2] = {nullptr, nullptr};
    void* h_marks[2] = {nullptr, nullptr};
    size_t dedge_n[2] = {0, 0}, sidx_n[2] = {0, 0}, h_marks_n[2] = {0, 0};
    // page-locked host trees (round 4), one per tree slot: ints in the device slot's layout (rank, parent,
    // first, child: 4P; level offsets: P + 2), then pdist (P bytes): one DMA copy per tree
    void* h_tree[2] = {nullptr, nullptr};
    void* host_tree[2] = {nullptr, nullptr};   // st_host::HostTree per slot, reused across calls (bm_segtree.hip)
    // the sorted edges come down in kEdgeChunks copies, each followed by its event (the host tree starts
    // on the first chunk)
    static constexpr int kEdgeChunks = 4;
    hipEvent_t edge_ev[2][kEdgeChunks] = {};
    int edge_chunk[2] = {0, 0};   // edges per chunk of each slot's last download
    size_t w8_n = 0, grad_n = 0, vol_n = 0, tree_i_n = 0, tree_b_n = 0, table_n = 0, task_n = 0, sortbuf_n = 0,
           bfs_n[2] = {0, 0};
    size_t h_edges_n[2] = {0, 0}, h_tree_n[2] = {0, 0};
    ~StWorkspace();
    void release();
};

struct StStats {
    int levels = 0;        // BFS levels of the (last) tree
    float tree_ms = 0.f;   // time of the tree builds (host lists + the BFS, until its level count is back)
};

// stereo_disparity_normal (StereoDisparity.cpp:57-89) on device BGR frames (3 bytes per pixel, row
// pitch `pitch`): D = max_dis_level, tau = TAU (Toolkit.h:34); d_out [H][W] uint8, pitch W.
// Synchronous on stream s (the tree is built on the host from the GPU's edge weights).
hipError_t segment_tree_match(StWorkspace& ws, const uint8_t* dL, const uint8_t* dR, int W, int H, int pitch, int D,
                              int scale, float sigma, float tau, uint8_t* d_out, hipStream_t s, StStats* st);

// stereo_disparity_iteration, ST-2 (StereoDisparity.cpp:91-160), same arguments: first-pass left and
// right maps on colour trees of each view (sigma SIGMA_ONE = 0.08, Toolkit.h:35), the left-right check,
// then a colour + depth tree (CColorDepthWeight) on the left view with `sigma`.
hipError_t segment_tree_refined_match(StWorkspace& ws, const uint8_t* dL, const uint8_t* dR, int W, int H, int pitch,
                                      int D, int scale, float sigma, float tau, uint8_t* d_out, hipStream_t s,
                                      StStats* st);

}  // namespace sm
