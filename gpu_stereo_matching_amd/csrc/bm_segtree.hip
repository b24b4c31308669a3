// bm_segtree.hip — segment-tree cost aggregation: the reference's STMatching ST-1
// pipeline (stereo_disparity_normal, StereoDisparity.cpp:57-89) with its O(P*D) parts on the GPU.
//
//   guide + edge weights  GPU: 3x3 median of each BGR channel of the left view (MeanFilter(img, 1)
//                         = ctmf, SegmentTree.cpp:185), max channel |diff| to the right / upper
//                         neighbour (CColorWeight::GetWeight, :189-194)
//   tree                  host: the reference builds it sequentially and so does this file.  Edges in
//                         (weight, b, a) order (edge::operator<, SegmentTree.h:103-111) by a counting sort
//                         over the 256 integer weights, filled in b order, which is that order exactly;
//                         Kruskal with Felzenszwalb's size threshold, then the rest of the spanning tree
//                         with the cross-segment penalty (segment-graph.h:48-101; disjoint-set.h:30-82);
//                         neighbour lists in that edge order, BFS from pixel 0 (SegmentTree.cpp:71-130)
//   cost volume           GPU: truncated colour + gradient cost (StereoHelper.cpp:37-129), written
//                         channel-major in BFS order, C[d][i], so a tree level is a contiguous run
//   filter                GPU: one workgroup per disparity d walks the BFS levels: leaf-to-root sums,
//                         then root-to-leaf (SegmentTree.cpp:148-181), one barrier per level; each node
//                         sums its children in the reference's order with separate multiplies and adds
//   WTA, x scale, median  GPU: first d with the smallest cost (StereoHelper.cpp:131-154), times scale
//                         (saturated; a non-decreasing map commutes with the median), then the 7x7
//                         median (MeanFilter(disparity, 3), bm_post.hip)
// The map is bit-exact with the restated oracle (oracle/st_oracle.c).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <vector>

#include "bm_common.h"
#include "bm_segtree.h"

namespace sm {
namespace {

constexpr int kST = 256;

// median of 9 (the classic 19-exchange network)
__device__ __forceinline__ uint8_t med9(uint8_t* v) {
    auto s = [&](int i, int j) {
        const uint8_t a = min(v[i], v[j]), b = max(v[i], v[j]);
        v[i] = a;
        v[j] = b;
    };
    s(1, 2); s(4, 5); s(7, 8); s(0, 1); s(3, 4); s(6, 7); s(1, 2); s(4, 5); s(7, 8);
    s(0, 3); s(5, 8); s(4, 7); s(3, 6); s(1, 4); s(2, 5); s(4, 7); s(4, 2); s(6, 4); s(4, 2);
    return v[4];
}

// per pixel p: wr[p] = weight of edge (p, p+1), wu[p] = weight of edge (p, p-W), on the 3x3-median
// guide (replicate borders, as ctmf)
__global__ __launch_bounds__(kST) void st_weights_kernel(const uint8_t* __restrict__ bgr, int W, int H, int pitch,
                                                         uint8_t* __restrict__ wr, uint8_t* __restrict__ wu) {
    const int x = blockIdx.x * kST + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    auto guide = [&](int gx, int gy, uint8_t out[3]) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            uint8_t v[9];
#pragma unroll
            for (int i = -1; i <= 1; ++i)
#pragma unroll
                for (int j = -1; j <= 1; ++j) {
                    const int yy = min(max(gy + i, 0), H - 1), xx = min(max(gx + j, 0), W - 1);
                    v[(i + 1) * 3 + (j + 1)] = bgr[(int64_t)yy * pitch + 3 * xx + c];
                }
            out[c] = med9(v);
        }
    };
    uint8_t g[3], n[3];
    guide(x, y, g);
    uint8_t r = 0, u = 0;
    if (x + 1 < W) {
        guide(x + 1, y, n);
        r = max(max((uint8_t)abs(g[0] - n[0]), (uint8_t)abs(g[1] - n[1])), (uint8_t)abs(g[2] - n[2]));
    }
    if (y >= 1) {
        guide(x, y - 1, n);
        u = max(max((uint8_t)abs(g[0] - n[0]), (uint8_t)abs(g[1] - n[1])), (uint8_t)abs(g[2] - n[2]));
    }
    wr[(int64_t)y * W + x] = r;
    wu[(int64_t)y * W + x] = u;
}

// GetGradient (StereoHelper.cpp:39-73) of one view: gray (rgb_2_gray, :37, in double) and the
// central / one-sided difference + 127.5 in float
__global__ __launch_bounds__(kST) void st_gradient_kernel(const uint8_t* __restrict__ bgr, int W, int H, int pitch,
                                                          float* __restrict__ grad) {
#pragma clang fp contract(off)
    const int x = blockIdx.x * kST + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    auto gray = [&](int xx) -> float {
        const uint8_t* in = bgr + (int64_t)y * pitch + 3 * xx;
        return (float)(uint8_t)(0.299 * in[2] + 0.587 * in[1] + 0.114 * in[0] + 0.5);
    };
    float g;
    if (x == 0) g = gray(1) - gray(0) + 127.5f;
    else if (x == W - 1) g = gray(W - 1) - gray(W - 2) + 127.5f;
    else g = 0.5f * (gray(x + 1) - gray(x - 1)) + 127.5f;
    grad[(int64_t)y * W + x] = g;
}

// GetMatchingCost (StereoHelper.cpp:75-129) into C[d][rank[p]]; right pixels left of column 0 repeat
// column 0 (:107-110); double arithmetic as the reference's, rounded to float once
__global__ __launch_bounds__(kST) void st_cost_kernel(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R,
                                                      int W, int H, int pitch, const float* __restrict__ gL,
                                                      const float* __restrict__ gR, const int* __restrict__ rank, int D,
                                                      float* __restrict__ C) {
#pragma clang fp contract(off)
    const int x = blockIdx.x * kST + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const int64_t P = (int64_t)W * H, p = (int64_t)y * W + x;
    const uint8_t* l = L + (int64_t)y * pitch + 3 * x;
    const int lb = l[0], lg = l[1], lr = l[2];
    const float gl = gL[p];
    const int i = rank[p];
    const double wc = 0.11, wg = 1.0 - wc;
    for (int d = 0; d < D; ++d) {
        const int xs = x >= d ? x - d : 0;
        const uint8_t* r = R + (int64_t)y * pitch + 3 * xs;
        double cc = (double)(abs(lb - r[0]) + abs(lg - r[1]) + abs(lr - r[2]));
        cc = cc / 3 < 7.0 ? cc / 3 : 7.0;
        double cg = fabsf(gl - gR[(int64_t)y * W + xs]);
        cg = cg < 2.0 ? cg : 2.0;
        C[(int64_t)d * P + i] = (float)(wc * cc + wg * cg);
    }
}

// Filter (SegmentTree.cpp:148-181) of disparity d = blockIdx.x.  C (in: cost, out: the leaf-to-root
// sums, the reference's costBuffer) and F (out: the filtered cost) are [D][P] in BFS order; levels
// are the BFS position ranges [lev[l], lev[l + 1]).
__global__ __launch_bounds__(1024) void st_filter_kernel(float* __restrict__ C, float* __restrict__ F,
                                                         const int* __restrict__ parent,
                                                         const uint8_t* __restrict__ pdist,
                                                         const int* __restrict__ first,
                                                         const uint32_t* __restrict__ child, const int* __restrict__ lev,
                                                         int nlev, int P, const float* __restrict__ table_g) {
#pragma clang fp contract(off)
    __shared__ float table[256];
    for (int k = threadIdx.x; k < 256; k += blockDim.x) table[k] = table_g[k];
    __syncthreads();
    float* U = C + (int64_t)blockIdx.x * P;
    float* Fd = F + (int64_t)blockIdx.x * P;
    // leaf to root: a node adds its children in order, each term multiplied then added
    for (int l = nlev - 1; l >= 0; --l) {
        const int lo = lev[l], hi = lev[l + 1];
        for (int i = lo + (int)threadIdx.x; i < hi; i += blockDim.x) {
            const uint32_t ch = child[i];                    // count | dist0 << 8 | dist1 << 16 | dist2 << 24
            const int n = (int)(ch & 0xFFu);
            if (n == 0) continue;
            float u = U[i];
            const int f = first[i];
            for (int z = 0; z < n; ++z) {
                const float t = U[f + z] * table[(ch >> (8 * (z + 1))) & 0xFFu];
                u = u + t;
            }
            U[i] = u;
        }
        __syncthreads();
    }
    // root to leaf
    if (threadIdx.x == 0) Fd[0] = U[0];
    __syncthreads();
    for (int l = 1; l < nlev; ++l) {
        const int lo = lev[l], hi = lev[l + 1];
        for (int i = lo + (int)threadIdx.x; i < hi; i += blockDim.x) {
            const float w = table[pdist[i]], cur = U[i];
            const float t = w * cur;
            Fd[i] = w * (Fd[parent[i]] - t) + cur;
        }
        __syncthreads();
    }
}

// GetDisparity_WTA (StereoHelper.cpp:131-154): strict < from d = 0; times scale, saturated
__global__ __launch_bounds__(kST) void st_wta_kernel(const float* __restrict__ F, const int* __restrict__ rank, int P,
                                                     int D, int scale, uint8_t* __restrict__ out) {
    const int p = blockIdx.x * kST + threadIdx.x;
    if (p >= P) return;
    const int i = rank[p];
    float v = F[i];
    int m = 0;
    for (int d = 1; d < D; ++d) {
        const float c = F[(int64_t)d * P + i];
        if (c < v) {
            v = c;
            m = d;
        }
    }
    out[p] = (uint8_t)min(m * scale, 255);
}

// ---- host: the tree (sequential, as the reference's) ----
struct Dsu {
    std::vector<int> p, rank, size;
    explicit Dsu(int n) : p(n), rank(n, 0), size(n, 1) {
        for (int i = 0; i < n; ++i) p[i] = i;
    }
    int find(int x) {   // disjoint-set.h:58-64: walk to the root, then point x at it
        int y = x;
        while (y != p[y]) y = p[y];
        p[x] = y;
        return y;
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

bool build_tree(const uint8_t* wr, const uint8_t* wu, int W, int H, float tau, HostTree& t) {
    const int P = W * H;
    // edges sorted by (weight, b, a): for a given b the candidates are (a = b-1, right edge of b-1)
    // and (a = b+W, upper edge of b+W), in that a order; a counting sort by weight filled in b order
    // is therefore the reference's std::sort order exactly
    struct E {
        int a, b;
        float w;
    };
    std::vector<int> cnt(257, 0);
    auto each_edge = [&](auto&& f) {
        for (int b = 0; b < P; ++b) {
            const int x = b % W;
            if (x >= 1) f(b - 1, b, wr[b - 1]);           // (b-1, b): right neighbour of b-1
            if (b + W < P) f(b + W, b, wu[b + W]);        // (b+W, b): upper neighbour of b+W
        }
    };
    each_edge([&](int, int, uint8_t w) { cnt[w + 1]++; });
    for (int k = 0; k < 256; ++k) cnt[k + 1] += cnt[k];
    const int nE = cnt[256];
    std::vector<E> e(nE);
    each_edge([&](int a, int b, uint8_t w) { e[cnt[w]++] = E{a, b, (float)w}; });
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
    // neighbour lists in sorted-edge order, dist = min(int(w * 1 + 0.5), 255) (SegmentTree.cpp:74-95)
    std::vector<int> adj((size_t)P * 4);
    std::vector<uint8_t> adjd((size_t)P * 4), na(P, 0);
    for (int i = 0; i < nE; ++i) {
        if (!mask[i]) continue;
        const int pa = e[i].a, pb = e[i].b;
        const uint8_t dis = (uint8_t)std::min((int)(e[i].w * 1.0f + 0.5f), 255);
        adj[(size_t)pa * 4 + na[pa]] = pb;
        adjd[(size_t)pa * 4 + na[pa]++] = dis;
        adj[(size_t)pb * 4 + na[pb]] = pa;
        adjd[(size_t)pb * 4 + na[pb]++] = dis;
    }
    // BFS from pixel 0 (SegmentTree.cpp:97-130), level by level
    t.node.assign(P, 0);
    t.rank.assign(P, 0);
    t.parent.assign(P, -1);
    t.first.assign(P, 0);
    t.pdist.assign(P, 0);
    t.child.assign(P, 0);
    t.lev.assign(1, 0);
    std::vector<uint8_t> vis(P, 0);
    vis[0] = 1;
    int end = 1;
    for (int lo = 0, hi = 1; lo < hi; lo = hi, hi = end) {
        t.lev.push_back(hi);
        for (int i = lo; i < hi; ++i) {
            const int p = t.node[i];
            t.rank[p] = i;
            t.first[i] = end;
            uint32_t ch = 0, n = 0;
            for (int k = 0; k < na[p]; ++k) {
                const int q = adj[(size_t)p * 4 + k];
                if (vis[q]) continue;
                vis[q] = 1;
                const uint8_t dis = adjd[(size_t)p * 4 + k];
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

template <class T>
hipError_t grow(T*& p, size_t& have, size_t n) {
    if (have >= n) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    have = 0;
    hipError_t e = hipMalloc(&p, n * sizeof(T));
    if (e == hipSuccess) have = n;
    return e;
}

}  // namespace

StWorkspace::~StWorkspace() { release(); }

void StWorkspace::release() {
    (void)hipFree(w8);
    (void)hipFree(grad);
    (void)hipFree(vol);
    (void)hipFree(tree_i);
    (void)hipFree(tree_b);
    (void)hipFree(table);
    w8 = nullptr;
    grad = nullptr;
    vol = nullptr;
    tree_i = nullptr;
    tree_b = nullptr;
    table = nullptr;
    w8_n = grad_n = vol_n = tree_i_n = tree_b_n = table_n = 0;
}

hipError_t segment_tree_match(StWorkspace& ws, const uint8_t* dL, const uint8_t* dR, int W, int H, int pitch, int D,
                              int scale, float sigma, float tau, uint8_t* d_out, hipStream_t s, StStats* st) {
    if (W < 2 || H < 1 || D < 1 || D > kMaxDisp || scale < 0) return hipErrorInvalidValue;
    const int64_t P = (int64_t)W * H;
    if (P > (1 << 28)) return hipErrorInvalidValue;
    hipError_t e;
#define ST_CHK(x)          \
    do {                   \
        e = (x);           \
        if (e != hipSuccess) return e; \
    } while (0)
    ST_CHK(grow(ws.w8, ws.w8_n, (size_t)P * 3));
    ST_CHK(grow(ws.grad, ws.grad_n, (size_t)P * 2));
    ST_CHK(grow(ws.vol, ws.vol_n, (size_t)P * D * 2));
    ST_CHK(grow(ws.tree_i, ws.tree_i_n, (size_t)P * 5 + 2));
    ST_CHK(grow(ws.tree_b, ws.tree_b_n, (size_t)P));
    ST_CHK(grow(ws.table, ws.table_n, (size_t)256));
    const dim3 rows((unsigned)((W + kST - 1) / kST), (unsigned)H);
    // guide weights -> host
    uint8_t* wr = ws.w8;
    uint8_t* wu = ws.w8 + P;
    hipLaunchKernelGGL(st_weights_kernel, rows, dim3(kST), 0, s, dL, W, H, pitch, wr, wu);
    ST_CHK(hipGetLastError());
    std::vector<uint8_t> hw((size_t)P * 2);
    ST_CHK(hipMemcpyAsync(hw.data(), ws.w8, (size_t)P * 2, hipMemcpyDeviceToHost, s));
    // gradients of both views meanwhile (same stream, after the download in order)
    hipLaunchKernelGGL(st_gradient_kernel, rows, dim3(kST), 0, s, dL, W, H, pitch, ws.grad);
    hipLaunchKernelGGL(st_gradient_kernel, rows, dim3(kST), 0, s, dR, W, H, pitch, ws.grad + P);
    ST_CHK(hipGetLastError());
    ST_CHK(hipStreamSynchronize(s));
    // tree on the host
    const auto t0 = std::chrono::steady_clock::now();
    HostTree t;
    if (!build_tree(hw.data(), hw.data() + P, W, H, tau, t)) return hipErrorInvalidValue;
    const int nlev = (int)t.lev.size() - 1;
    if ((size_t)nlev + 1 > (size_t)P + 2) return hipErrorInvalidValue;
    float table[256];
    const float sg = std::max(0.01f, sigma);
    for (int i = 0; i <= 255; ++i) table[i] = std::exp(-float(i) / (255 * sg));   // UpdateTable, :141-146
    const auto t1 = std::chrono::steady_clock::now();
    // tree arrays: int [rank | parent | first | child | lev], uint8 pdist
    int* d_rank = ws.tree_i;
    int* d_parent = d_rank + P;
    int* d_first = d_parent + P;
    uint32_t* d_child = reinterpret_cast<uint32_t*>(d_first + P);
    int* d_lev = reinterpret_cast<int*>(d_child + P);
    ST_CHK(hipMemcpyAsync(d_rank, t.rank.data(), (size_t)P * 4, hipMemcpyHostToDevice, s));
    ST_CHK(hipMemcpyAsync(d_parent, t.parent.data(), (size_t)P * 4, hipMemcpyHostToDevice, s));
    ST_CHK(hipMemcpyAsync(d_first, t.first.data(), (size_t)P * 4, hipMemcpyHostToDevice, s));
    ST_CHK(hipMemcpyAsync(d_child, t.child.data(), (size_t)P * 4, hipMemcpyHostToDevice, s));
    ST_CHK(hipMemcpyAsync(d_lev, t.lev.data(), t.lev.size() * 4, hipMemcpyHostToDevice, s));
    ST_CHK(hipMemcpyAsync(ws.tree_b, t.pdist.data(), (size_t)P, hipMemcpyHostToDevice, s));
    ST_CHK(hipMemcpyAsync(ws.table, table, sizeof(table), hipMemcpyHostToDevice, s));
    float* C = ws.vol;
    float* F = ws.vol + (size_t)P * D;
    hipLaunchKernelGGL(st_cost_kernel, rows, dim3(kST), 0, s, dL, dR, W, H, pitch, ws.grad, ws.grad + P, d_rank, D, C);
    ST_CHK(hipGetLastError());
    hipLaunchKernelGGL(st_filter_kernel, dim3((unsigned)D), dim3(1024), 0, s, C, F, d_parent, ws.tree_b, d_first,
                       d_child, d_lev, nlev, (int)P, ws.table);
    ST_CHK(hipGetLastError());
    uint8_t* raw = ws.w8;   // the weights are consumed: reuse for the unfiltered map
    hipLaunchKernelGGL(st_wta_kernel, dim3((unsigned)((P + kST - 1) / kST)), dim3(kST), 0, s, F, d_rank, (int)P, D,
                       scale, raw);
    ST_CHK(hipGetLastError());
    ST_CHK(launch_median(raw, W, H, W, P, 1, 3, d_out, W, P, s));   // MeanFilter(disparity, disparity, 3)
    if (st) {
        st->levels = nlev;
        st->tree_ms = std::chrono::duration<float, std::milli>(t1 - t0).count();
    }
#undef ST_CHK
    // keep the host tree alive until its uploads have been consumed
    return hipStreamSynchronize(s);
}

}  // namespace sm
