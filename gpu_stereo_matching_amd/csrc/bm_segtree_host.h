// bm_segtree_host.h — the segment tree's host side (STMatching BuildSegmentTree, SegmentTree.cpp:38-139;
// segment_graph, segment-graph.h:48-101; disjoint-set.h:30-82; CColorDepthWeight, SegmentTree.cpp:196-219).
// Plain C++17, no HIP: bm_segtree.hip builds its trees with it, and tests/native/st_host_shim.cpp
// exposes it to the CPU test suite, which compares its trees with the C restatement (oracle/st_oracle.c).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

// the float steps (thresholds, tree distances, depth weights) are rounded one operation at a time
#if defined(__clang__)
#define SM_ST_NO_CONTRACT _Pragma("clang fp contract(off)")
#else
#define SM_ST_NO_CONTRACT
#endif

namespace sm {
namespace st_host {

// ---- host: the tree (sequential, as the reference's) ----
// disjoint-set.h's forest as separate arrays: find walks only the parent array (a packed 16-B record
// per element measured 25 % slower on the Art tree)
struct Dsu {
    std::vector<int> p, rank, size;
    explicit Dsu(int n) : p(n), rank(n, 0), size(n, 1) {
        for (int i = 0; i < n; ++i) p[i] = i;
    }
    // disjoint-set.h:58-64 walks to the root and points x at it.  Path halving here: compression moves
    // only non-root parent pointers, so every root, rank and size (all that join and segment_graph
    // read) is the reference's; the walks are shorter.
    int find(int x) {
        while (x != p[x]) {
            p[x] = p[p[x]];
            x = p[x];
        }
        return x;
    }
    void join(int x, int y) {   // disjoint-set.h:66-82
        if (x != p[x]) x = find(x);
        if (y != p[y]) y = find(y);
        if (x == y) return;
        if (rank[x] > rank[y]) {
            p[y] = x;
            size[x] += size[y];
        } else {
            p[x] = y;
            size[y] += size[x];
            if (rank[x] == rank[y]) rank[y]++;
        }
    }
};

struct HostTree {
    std::vector<int> node, rank, parent, first, lev;
    std::vector<uint8_t> pdist;
    std::vector<uint32_t> child;
};

struct Edge {
    int a, b;
    float w;
};

// Every edge of SegmentTree.cpp:44-62 in increasing b, and for one b in increasing a: (b-1, b) is the
// right edge of b-1 (weight wr[b-1]) and (b+W, b) the upper edge of b+W (weight wu[b+W]).
template <class F>
void each_edge(int W, int P, F&& f) {
    for (int y0 = 0; y0 < P; y0 += W) {
        const int ye = std::min(y0 + W, P), up = P - W;   // b + W < P  <=>  b < up
        if (y0 < up) f(y0 + W, y0, 1);
        for (int b = y0 + 1; b < ye; ++b) {
            f(b - 1, b, 0);
            if (b < up) f(b + W, b, 1);
        }
    }
}

// CColorWeight edges (integer weights) in edge::operator< order (SegmentTree.h:103-111): a counting sort
// by weight filled in (b, a) order is that order exactly.
std::vector<Edge> sorted_edges_u8(const uint8_t* wr, const uint8_t* wu, int W, int P) {
    std::vector<int> cnt(257, 0);
    each_edge(W, P, [&](int a, int, int up) { cnt[(up ? wu[a] : wr[a]) + 1]++; });
    for (int k = 0; k < 256; ++k) cnt[k + 1] += cnt[k];
    std::vector<Edge> e(cnt[256]);
    each_edge(W, P, [&](int a, int b, int up) {
        const uint8_t w = up ? wu[a] : wr[a];
        e[cnt[w]++] = Edge{a, b, (float)w};
    });
    return e;
}

// Float-weighted edges (CColorDepthWeight) in edge::operator< order: generated in (b, a) order, then a
// stable LSD radix sort on the weights' bit patterns (non-negative floats order as their bits).
std::vector<Edge> sorted_edges_f(const float* wr, const float* wu, int W, int P) {
    std::vector<Edge> e, tmp;
    e.reserve((size_t)2 * P);
    each_edge(W, P, [&](int a, int b, int up) { e.push_back(Edge{a, b, up ? wu[a] : wr[a]}); });
    tmp.resize(e.size());
    for (int shift = 0; shift < 32; shift += 8) {
        size_t cnt[257] = {0};
        for (const Edge& x : e) cnt[((__builtin_bit_cast(uint32_t, x.w) >> shift) & 0xFFu) + 1]++;
        if (cnt[1] == e.size() && shift > 0) continue;   // every key has a zero digit here
        for (int k = 0; k < 256; ++k) cnt[k + 1] += cnt[k];
        for (const Edge& x : e) tmp[cnt[(__builtin_bit_cast(uint32_t, x.w) >> shift) & 0xFFu]++] = x;
        e.swap(tmp);
    }
    return e;
}

// BuildSegmentTree (SegmentTree.cpp:38-139) from the nE sorted edges e (consumed: the cross-segment
// penalty is added in place): segment_graph, the neighbour
// lists with dist = min(int(w * wscale + 0.5), 255) (wscale = GetScale(): 1 colour, 255 colour + depth),
// BFS from pixel 0, level by level.
bool tree_from_edges(Edge* e, int nE, int P, float tau, float wscale, HostTree& t) {
SM_ST_NO_CONTRACT
    // segment_graph (segment-graph.h:48-101)
    Dsu u(P);
    std::vector<float> thr(P, tau / 1);
    std::vector<uint8_t> mask(nE, 0);
    for (int i = 0; i < nE; ++i) {
        int a = u.find(e[i].a), b = u.find(e[i].b);
        if (a != b && e[i].w <= thr[a] && e[i].w <= thr[b]) {
            mask[i] = 1;
            u.join(a, b);
            a = u.find(a);
            thr[a] = e[i].w + tau / u.size[a];
        }
    }
    for (int i = 0; i < nE; ++i) {
        const int a = u.find(e[i].a), b = u.find(e[i].b);
        if (a != b) {
            const int size_min = std::min(u.size[a], u.size[b]);
            u.join(a, b);
            mask[i] = 1;
            if (size_min > 50) e[i].w += 5;   // MIN_SIZE_SEG, PENALTY_CROSS_SEG
        }
    }
    // neighbour lists in sorted-edge order (SegmentTree.cpp:74-95), one 24-B record per pixel
    struct Adj {
        int q[4];
        uint8_t d[4];
        int n;
    };
    std::vector<Adj> adj(P);
    for (int p = 0; p < P; ++p) adj[p].n = 0;
    for (int i = 0; i < nE; ++i) {
        if (!mask[i]) continue;
        const int pa = e[i].a, pb = e[i].b;
        const float sw = e[i].w * wscale;
        const uint8_t dis = (uint8_t)std::min((int)(sw + 0.5f), 255);
        Adj& A = adj[pa];
        A.q[A.n] = pb;
        A.d[A.n++] = dis;
        Adj& B = adj[pb];
        B.q[B.n] = pa;
        B.d[B.n++] = dis;
    }
    // BFS from pixel 0 (SegmentTree.cpp:97-130), level by level
    t.node.assign(P, 0);
    t.rank.assign(P, 0);
    t.parent.assign(P, -1);
    t.first.assign(P, 0);
    t.pdist.assign(P, 0);
    t.child.assign(P, 0);
    t.lev.assign(1, 0);
    // the marked edges form a forest, so a node's neighbours other than its parent are exactly the ones
    // BFS has not visited yet (SegmentTree.cpp:116's visited test): compare with the parent's pixel
    std::vector<int> ppix(P);
    ppix[0] = -1;
    int end = 1;
    for (int lo = 0, hi = 1; lo < hi; lo = hi, hi = end) {
        t.lev.push_back(hi);
        for (int i = lo; i < hi; ++i) {
            const int p = t.node[i], pp = ppix[i];
            t.rank[p] = i;
            t.first[i] = end;
            uint32_t ch = 0, n = 0;
            const Adj& A = adj[p];
            for (int k = 0; k < A.n; ++k) {
                const int q = A.q[k];
                if (q == pp) continue;
                ppix[end] = p;
                const uint8_t dis = A.d[k];
                ch |= (uint32_t)dis << (8 * (n + 1));
                ++n;
                t.node[end] = q;
                t.parent[end] = i;
                t.pdist[end] = dis;
                ++end;
            }
            t.child[i] = ch | n;
        }
    }
    return end == P;
}

bool build_tree(const uint8_t* wr, const uint8_t* wu, int W, int H, float tau, HostTree& t) {
    std::vector<Edge> e = sorted_edges_u8(wr, wu, W, W * H);
    return tree_from_edges(e.data(), (int)e.size(), W * H, tau, 1.0f, t);
}

// CColorDepthWeight::GetWeight (SegmentTree.cpp:204-219) from the colour weights (max channel |diff| on
// the 3x3-median guide), the first left map and the mask, in the reference's float operations
void depth_weights(const uint8_t* wr, const uint8_t* wu, const uint8_t* disp, const uint8_t* mask, int W, int H,
                   float level, float* fr, float* fu) {
SM_ST_NO_CONTRACT
    auto weight = [&](int p, int q, uint8_t c) -> float {
        if (mask[p] && mask[q]) {
            const float dispValue = (float)std::abs(disp[p] - disp[q]) / level;
            const float colorValue = (float)c / 255.0f;
            return 0.5f * dispValue + (1.0f - 0.5f) * colorValue;
        }
        return (float)c / 255.0f;
    };
    const int P = W * H;
    for (int p = 0; p < P; ++p) {
        fr[p] = (p % W + 1 < W) ? weight(p, p + 1, wr[p]) : 0.f;
        fu[p] = (p >= W) ? weight(p, p - W, wu[p]) : 0.f;
    }
}

}  // namespace st_host
}  // namespace sm
