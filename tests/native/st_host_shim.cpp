// Test-only C shim over the segment tree's host builder (gpu_stereo_matching_amd/csrc/bm_segtree_host.h),
// compiled by tests/test_st_host.py with g++ so the CPU suite can compare its trees with the C
// restatement (oracle/st_oracle.c).  Not part of the product library.
#include <cstring>

#include "../../gpu_stereo_matching_amd/csrc/bm_segtree_host.h"

using namespace sm::st_host;

static int export_tree(const HostTree& t, int P, int* node, int* parent, uint8_t* pdist) {
    std::memcpy(node, t.node.data(), sizeof(int) * P);
    std::memcpy(parent, t.parent, sizeof(int) * P);
    std::memcpy(pdist, t.pdist, (size_t)P);
    return (int)t.lev.size() - 1;
}

// CColorWeight tree from the colour weights wr (edge p -> p+1) and wu (edge p -> p-W); returns the BFS
// level count, -1 if the tree does not span the image
extern "C" int st_host_tree_u8(const uint8_t* wr, const uint8_t* wu, int W, int H, float tau, int* node, int* parent,
                               uint8_t* pdist) {
    HostTree t;
    if (!build_tree(wr, wu, W, H, tau, t)) return -1;
    return export_tree(t, W * H, node, parent, pdist);
}

// CColorDepthWeight tree (float weights, GetScale 255) from the same colour weights, a map and a mask
extern "C" int st_host_tree_depth(const uint8_t* wr, const uint8_t* wu, const uint8_t* disp, const uint8_t* mask,
                                  int W, int H, int level, float tau, int* node, int* parent, uint8_t* pdist) {
    const int P = W * H;
    std::vector<float> fw((size_t)P * 2);
    depth_weights(wr, wu, disp, mask, W, H, (float)level, fw.data(), fw.data() + P);
    std::vector<Edge> e = sorted_edges_f(fw.data(), fw.data() + P, W, P);
    HostTree t;
    if (!tree_from_edges(e.data(), (int)e.size(), P, W, tau, 255.0f, t)) return -1;
    return export_tree(t, P, node, parent, pdist);
}
