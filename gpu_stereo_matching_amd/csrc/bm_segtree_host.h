// bm_segtree_host.h — the segment tree's host side (STMatching BuildSegmentTree, SegmentTree.cpp:38-139;
// segment_graph, segment-graph.h:48-101; disjoint-set.h:30-82; CColorDepthWeight, SegmentTree.cpp:196-219).
// Plain C++17, no HIP: bm_segtree.hip builds its trees with it, and tests/native/st_host_shim.cpp
// exposes it to the CPU test suite, which compares its trees with the C restatement (oracle/st_oracle.c).
#pragma once
#include <stdint.h>

#include <algorithm>
#include <cstdlib>
#include <vector>

// phase marks for tools/microbench/st_host_bench.cpp (0: first pass, 1: second pass + lists, 2: BFS done)
#ifndef SM_ST_PHASE
#define SM_ST_PHASE(k)
#endif

// the float steps (thresholds, tree distances, depth weights) are rounded one operation at a time
#if defined(__clang__)
#define SM_ST_NO_CONTRACT _Pragma("clang fp contract(off)")
#else
#define SM_ST_NO_CONTRACT
#endif

namespace sm {
namespace st_host {

// ---- host: the tree (sequential, as the reference's) ----
// rank | parent | first | child (P ints each) sit in one block laid out as the device's tree slot (round 4),
// in the tree's own vector or, after bind(), in caller storage (the GPU path binds page-locked memory, so
// the tree goes up as one DMA copy without a staging memcpy); pdist likewise.  node and lev stay vectors.
// a root's threshold (segment-graph.h:63, tau / 1 at the start), size and rank in one record
struct RootRec {
    float thr;
    int size, rank;
};
// neighbour list of a pixel: direction k is (dir >> 2k) & 3 -> offset -1, +1, -W, +W, distance byte k of d
struct AdjRec {
    uint32_t d;
    uint16_t dir, n;
};

struct HostTree {
    std::vector<int> node, lev;
    // the builder's scratch (round 4): kept with the tree, so a tree object reused from call to call (the
    // GPU path keeps one per slot) touches memory that is already mapped instead of ~5 MB of fresh pages
    std::vector<int> par, ppix;
    std::vector<RootRec> roots;
    std::vector<AdjRec> adj;
    std::vector<uint8_t> mask;
    int* rank = nullptr;
    int* parent = nullptr;
    int* first = nullptr;
    uint32_t* child = nullptr;
    uint8_t* pdist = nullptr;
    std::vector<int> own_i;
    std::vector<uint8_t> own_b;
    // ints: 4P (+ the caller's room after them); bytes: P.  Null storage: the tree's own vectors.
    void bind(int P, int* ints = nullptr, uint8_t* bytes = nullptr) {
        if (!ints) {
            own_i.resize((size_t)4 * P);
            ints = own_i.data();
        }
        if (!bytes) {
            own_b.resize((size_t)P);
            bytes = own_b.data();
        }
        rank = ints;
        parent = ints + P;
        first = ints + 2 * (size_t)P;
        child = reinterpret_cast<uint32_t*>(ints + 3 * (size_t)P);
        pdist = bytes;
    }
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
inline std::vector<Edge> sorted_edges_u8(const uint8_t* wr, const uint8_t* wu, int W, int P) {
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
inline std::vector<Edge> sorted_edges_f(const float* wr, const float* wu, int W, int P) {
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

// BuildSegmentTree (SegmentTree.cpp:38-139) from the nE sorted edges e of a W-wide image: segment_graph,
// the neighbour lists with dist = min(int(w * wscale + 0.5), 255) (wscale = GetScale(): 1 colour, 255
// colour + depth; w + PENALTY_CROSS_SEG for the penalised edges), BFS from pixel 0, level by level.
// Round 4 (same trees bit for bit, tests/test_st_host.py): a root's size, rank and threshold in one
// record (they are read together at every join); the second segment_graph pass skips the edges the
// first one joined (their ends already share a root) and hands each tree edge over as it goes, in the
// sorted-edge order of SegmentTree.cpp:74-95, without a third pass; the lists are 8 B per pixel (four
// distances, four 2-bit directions, the count) instead of 24.
// `arrived(i)` (round 4) returns once edges [0, i) are readable: the GPU path downloads the sorted edges in
// chunks and the first pass starts on the first chunk while the rest is still in flight.  It is called
// with increasing i at most every `step` edges, and with nE before the second pass.
// In parts (round 4): segment_passes (segment_graph's two passes: per-edge marks), segment_lists (the
// passes + the neighbour lists, P records) and bfs_tree (the BFS from the lists).  The GPU path runs
// only segment_passes here; the lists and the BFS are built on the device from the marks
// (bm_segtree.hip: st_adj_kernel, st_arc_kernel ..), into the same arrays.
// segment_graph's two passes over the sorted edges.  marks (nE bytes, written): bit 0 = edge i is a tree
// edge (joined in either pass), bit 1 = the second pass joined it across two segments both larger than
// MIN_SIZE_SEG (the PENALTY_CROSS_SEG of +5 on its weight).  on_tree(i) is called for every tree edge in
// sorted order during the second pass, after its marks are set.
template <class Arrived, class OnTree>
void segment_passes(const Edge* e, int nE, int P, float tau, HostTree& t, int step, Arrived&& arrived,
                    uint8_t* marks, OnTree&& on_tree) {
SM_ST_NO_CONTRACT
    // segment_graph (segment-graph.h:48-101) on disjoint-set.h's forest (Dsu's rules, roots packed)
    std::vector<int>& par = t.par;
    par.resize(P);
    for (int i = 0; i < P; ++i) par[i] = i;
    std::vector<RootRec>& R = t.roots;
    R.assign(P, RootRec{tau / 1, 1, 0});
    auto find = [&](int x) {   // path halving, as Dsu::find
        while (x != par[x]) {
            par[x] = par[par[x]];
            x = par[x];
        }
        return x;
    };
    auto join = [&](int x, int y) {   // disjoint-set.h:66-82 on roots x != y; returns the new root
        if (R[x].rank > R[y].rank) {
            par[y] = x;
            R[x].size += R[y].size;
            return x;
        }
        par[x] = y;
        R[y].size += R[x].size;
        if (R[x].rank == R[y].rank) R[y].rank++;
        return y;
    };
    std::fill(marks, marks + nE, (uint8_t)0);
    int avail = 0;
    for (int i = 0; i < nE; ++i) {
        if (i == avail) {
            avail = std::min(nE, avail + std::max(step, 1));
            arrived(avail);
        }
        const int a = find(e[i].a), b = find(e[i].b);
        if (a != b && e[i].w <= R[a].thr && e[i].w <= R[b].thr) {
            marks[i] = 1;
            const int r = join(a, b);
            R[r].thr = e[i].w + tau / R[r].size;
        }
    }
    SM_ST_PHASE(0);
    for (int i = 0; i < nE; ++i) {
        if (!marks[i]) {   // segment-graph.h:88-99: join the remaining components
            const int a = find(e[i].a), b = find(e[i].b);
            if (a == b) continue;
            const int size_min = std::min(R[a].size, R[b].size);
            join(a, b);
            marks[i] = size_min > 50 ? 3 : 1;   // MIN_SIZE_SEG, PENALTY_CROSS_SEG
        }
        on_tree(i);
    }
}

// the tree distance of a marked edge: dist = min(int(w * wscale + 0.5), 255) on its (penalised) weight
inline uint8_t tree_dist(float w, uint8_t mark, float wscale) {
SM_ST_NO_CONTRACT
    if (mark & 2) w += 5;
    const float sw = w * wscale;
    return (uint8_t)std::min((int)(sw + 0.5f), 255);
}

// The passes with the neighbour lists built as they go (the host BFS path); `adj` (P records) receives
// the lists.
template <class Arrived>
void segment_lists(const Edge* e, int nE, int P, float tau, float wscale, HostTree& t, int step, Arrived&& arrived,
                   AdjRec* adj) {
    std::fill(adj, adj + P, AdjRec{0u, 0, 0});
    auto link = [&](int pa, int pb, uint8_t dis) {
        const int diff = pb - pa;
        const uint32_t da = diff == -1 ? 0u : diff == 1 ? 1u : diff < 0 ? 2u : 3u;
        AdjRec& A = adj[pa];
        A.d |= (uint32_t)dis << (8 * A.n);
        A.dir |= (uint16_t)(da << (2 * A.n));
        A.n++;
        AdjRec& B = adj[pb];
        B.d |= (uint32_t)dis << (8 * B.n);
        B.dir |= (uint16_t)((da ^ 1u) << (2 * B.n));
        B.n++;
    };
    t.mask.resize(nE);
    uint8_t* marks = t.mask.data();
    segment_passes(e, nE, P, tau, t, step, arrived, marks,
                   [&](int i) { link(e[i].a, e[i].b, tree_dist(e[i].w, marks[i], wscale)); });
    SM_ST_PHASE(1);
}

// BFS from pixel 0 (SegmentTree.cpp:97-130) over the neighbour lists, level by level; every entry is
// written once the tree spans the image (end == P), so the arrays need no clearing beyond the root's.
// The tree's arrays must be bound (HostTree::bind) unless it owns none yet.
inline bool bfs_tree(const AdjRec* adj, int P, int W, HostTree& t) {
    const int off[4] = {-1, 1, -W, W};
    if (!t.rank) t.bind(P);
    t.node.resize(P);
    t.lev.assign(1, 0);
    t.node[0] = 0;
    t.parent[0] = -1;
    t.pdist[0] = 0;
    // the marked edges form a forest, so a node's neighbours other than its parent are exactly the ones
    // BFS has not visited yet (SegmentTree.cpp:116's visited test): compare with the parent's pixel
    std::vector<int>& ppix = t.ppix;
    ppix.resize(P);
    ppix[0] = -1;
    int end = 1;
    for (int lo = 0, hi = 1; lo < hi; lo = hi, hi = end) {
        t.lev.push_back(hi);
        for (int i = lo; i < hi; ++i) {
            // the neighbour list and rank slot of the node 8 places on (already queued: BFS order):
            // BFS 1.58 -> 1.45 ms on the GPU box's host for Art (profiles/microbench/r04_st_host_phases.txt;
            // the same prefetch in the two edge passes made them slower)
            if (i + 8 < end) {
                __builtin_prefetch(&adj[t.node[i + 8]]);
                __builtin_prefetch(&t.rank[t.node[i + 8]]);
            }
            const int p = t.node[i], pp = ppix[i];
            t.rank[p] = i;
            t.first[i] = end;
            uint32_t ch = 0, n = 0;
            const AdjRec A = adj[p];
            for (int k = 0; k < A.n; ++k) {
                const int q = p + off[(A.dir >> (2 * k)) & 3];
                if (q == pp) continue;
                ppix[end] = p;
                const uint8_t dis = (uint8_t)(A.d >> (8 * k));
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
    SM_ST_PHASE(2);
    return end == P;
}

template <class Arrived>
bool tree_from_edges(const Edge* e, int nE, int P, int W, float tau, float wscale, HostTree& t, int step,
                     Arrived&& arrived) {
    t.adj.resize(P);
    segment_lists(e, nE, P, tau, wscale, t, step, arrived, t.adj.data());
    return bfs_tree(t.adj.data(), P, W, t);
}

// every edge already in memory
inline bool tree_from_edges(const Edge* e, int nE, int P, int W, float tau, float wscale, HostTree& t) {
    return tree_from_edges(e, nE, P, W, tau, wscale, t, nE, [](int) {});
}

inline bool build_tree(const uint8_t* wr, const uint8_t* wu, int W, int H, float tau, HostTree& t) {
    std::vector<Edge> e = sorted_edges_u8(wr, wu, W, W * H);
    return tree_from_edges(e.data(), (int)e.size(), W * H, W, tau, 1.0f, t);
}

// CColorDepthWeight::GetWeight (SegmentTree.cpp:204-219) from the colour weights (max channel |diff| on
// the 3x3-median guide), the first left map and the mask, in the reference's float operations
inline void depth_weights(const uint8_t* wr, const uint8_t* wu, const uint8_t* disp, const uint8_t* mask, int W, int H,
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
