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

// The device path's neighbour lists (bm_segtree.hip st_adj_kernel: per pixel, its marked grid edges at
// their sorted positions, in position order, distances from the marks' penalty bit) restated here on
// the marks of segment_passes, against segment_lists' lists built during the second pass.  depth != 0:
// the colour + depth weights of st_host_tree_depth (disp, mask, level), scale 255.  Returns the number of
// pixels whose lists differ.
extern "C" int st_host_lists_from_marks_check(const uint8_t* wr, const uint8_t* wu, const uint8_t* disp,
                                              const uint8_t* mask, int W, int H, int level, int depth, float tau) {
    const int P = W * H;
    std::vector<Edge> e;
    float wscale = 1.0f;
    if (depth) {
        std::vector<float> fw((size_t)P * 2);
        depth_weights(wr, wu, disp, mask, W, H, (float)level, fw.data(), fw.data() + P);
        e = sorted_edges_f(fw.data(), fw.data() + P, W, P);
        wscale = 255.0f;
    } else {
        e = sorted_edges_u8(wr, wu, W, P);
    }
    const int nE = (int)e.size();
    HostTree t1, t2;
    std::vector<AdjRec> want(P);
    segment_lists(e.data(), nE, P, tau, wscale, t1, nE, [](int) {}, want.data());
    std::vector<uint8_t> marks(nE);
    segment_passes(e.data(), nE, P, tau, t2, nE, [](int) {}, marks.data(), [](int) {});
    std::vector<int> sidx((size_t)2 * P, -1);
    for (int q = 0; q < nE; ++q) sidx[2 * e[q].b + (e[q].a == e[q].b + W ? 1 : 0)] = q;
    int bad = 0;
    for (int p = 0; p < P; ++p) {
        const int x = p % W;
        int pos[4];
        uint32_t cd[4];
        for (int c = 0; c < 4; ++c) {
            const bool ex = c == 0 ? x >= 1 : c == 1 ? x + 1 < W : c == 2 ? p >= W : p + W < P;
            const int v = c == 0 ? 2 * p : c == 1 ? 2 * (p + 1) : c == 2 ? 2 * (p - W) + 1 : 2 * p + 1;
            pos[c] = 0x7FFFFFFF;
            cd[c] = 0;
            if (ex && (marks[sidx[v]] & 1)) {
                pos[c] = sidx[v];
                cd[c] = (uint32_t)c | ((uint32_t)tree_dist(e[sidx[v]].w, marks[sidx[v]], wscale) << 8);
            }
        }
        for (int i = 1; i < 4; ++i)
            for (int j = i; j > 0 && pos[j] < pos[j - 1]; --j) {
                std::swap(pos[j], pos[j - 1]);
                std::swap(cd[j], cd[j - 1]);
            }
        uint32_t d = 0, dir = 0, n = 0;
        for (int k = 0; k < 4; ++k)
            if (pos[k] != 0x7FFFFFFF) {
                d |= (cd[k] >> 8) << (8 * k);
                dir |= (cd[k] & 3u) << (2 * k);
                ++n;
            }
        if (d != want[p].d || dir != want[p].dir || n != want[p].n) ++bad;
    }
    return bad;
}
