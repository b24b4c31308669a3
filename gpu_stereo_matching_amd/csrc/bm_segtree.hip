// bm_segtree.hip — segment-tree cost aggregation: the reference's STMatching ST-1
// pipeline (stereo_disparity_normal, StereoDisparity.cpp:57-89) and ST-2 (stereo_disparity_iteration,
// :91-160) with their O(P*D) parts on the GPU.
//
//   guide + edge weights  GPU: 3x3 median of each BGR channel of the left view (MeanFilter(img, 1)
//                         = ctmf, SegmentTree.cpp:185), max channel |diff| to the right / upper
//                         neighbour (CColorWeight::GetWeight, :189-194)
//   edge order            GPU: the edges in (b, a) order, stably radix-sorted by weight, which is
//                         edge::operator<'s (weight, b, a) order (SegmentTree.h:103-111); the sorted
//                         edges come back to the host page-locked
//   tree                  host: segment_graph's two passes, sequential as the reference's: Kruskal with
//                         Felzenszwalb's size threshold, then the rest of the spanning tree with the
//                         cross-segment penalty (segment-graph.h:48-101; disjoint-set.h:30-82), as per-edge
//                         marks.  GPU (round 4): the neighbour lists in the sorted edge order and the BFS
//                         from pixel 0 (SegmentTree.cpp:71-130), by an Euler tour ranked with pointer
//                         jumping and a depth sort (st_adj_kernel .. st_task_kernel, gpu_bfs)
//   cost volume           GPU: truncated colour + gradient cost (StereoHelper.cpp:37-129), written
//                         channel-major in BFS order, C[d][i], so a tree level is a contiguous run
//   filter                GPU: one wave per disparity walks the BFS levels (st_filter_wave_kernel; one
//                         workgroup per disparity for trees wider than its LDS): leaf-to-root sums, then
//                         root-to-leaf (SegmentTree.cpp:148-181); each node sums its children in the
//                         reference's order with separate multiplies and adds
//   WTA, x scale, median  GPU: first d with the smallest cost (StereoHelper.cpp:131-154), times scale
//                         (saturated; a non-decreasing map commutes with the median), then the 7x7
//                         median (MeanFilter(disparity, 3), bm_post.hip)
// ST-2 adds: the right view's cost taken from the left's (GetRightMatchingCostFromLeft,
// StereoHelper.cpp:156-180: C_R(y, x, d) = C(y, min(x + d, W - 1), min(d, W - 1 - x)), computed directly),
// a colour tree of each view filtered in one launch, the left-right check (bm_aux.hip), and a colour +
// depth tree (CColorDepthWeight, SegmentTree.cpp:196-219) whose float weights the GPU forms from the
// colour weights, the first left map and the mask, and orders by a stable radix sort of their bits.
// The maps are bit-exact with the restated oracle (oracle/st_oracle.c).
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <thread>
#include <vector>

#include "bm_common.h"
#include "bm_segtree.h"
#include "bm_segtree_host.h"

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
// column 0 (:107-110); double arithmetic as the reference's, rounded to float once.  RIGHT: the right
// view's cost at pixel p = (y, x), GetRightMatchingCostFromLeft (StereoHelper.cpp:156-180): the left
// cost at (y, min(x + d, W - 1)) and disparity min(d, W - 1 - x), whose right pixel is (y, x) itself.
// One thread per BFS index i (pixel node[i]), so the D stores of a wave are coalesced (round 4: one thread
// per pixel scattered them through rank; Art D = 60: 81 -> 51 us, rocprof); the image and gradient reads
// gather from L2-resident rows instead.
template <bool RIGHT>
__global__ __launch_bounds__(kST) void st_cost_kernel(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R,
                                                      int W, int H, int pitch, const float* __restrict__ gL,
                                                      const float* __restrict__ gR, const int* __restrict__ node, int D,
                                                      float* __restrict__ C) {
#pragma clang fp contract(off)
    const int64_t P = (int64_t)W * H;
    const int i = blockIdx.x * kST + threadIdx.x;
    if (i >= P) return;
    const int p = node[i];
    if ((unsigned)p >= (unsigned)P) return;
    const int y = p / W, x = p - y * W;
    const double wc = 0.11, wg = 1.0 - wc;
    auto cost = [&](int xl, int xr) -> float {
        const uint8_t* l = L + (int64_t)y * pitch + 3 * xl;
        const uint8_t* r = R + (int64_t)y * pitch + 3 * xr;
        double cc = (double)(abs(l[0] - r[0]) + abs(l[1] - r[1]) + abs(l[2] - r[2]));
        cc = cc / 3 < 7.0 ? cc / 3 : 7.0;
        double cg = fabsf(gL[(int64_t)y * W + xl] - gR[(int64_t)y * W + xr]);
        cg = cg < 2.0 ? cg : 2.0;
        return (float)(wc * cc + wg * cg);
    };
    for (int d = 0; d < D; ++d) {
        const float c = RIGHT ? cost(min(x + d, W - 1), x) : cost(x, x >= d ? x - d : 0);
        C[(int64_t)d * P + i] = c;
    }
}

// One tree's filter input: C (in: cost, out: the leaf-to-root sums, the reference's costBuffer) and F
// (out: the filtered cost) are [D][P] in that tree's BFS order; levels are the BFS position ranges
// [lev[l], lev[l + 1]).
struct FilterJob {
    float* C;
    float* F;
    const int* parent;
    const uint8_t* pdist;
    const int* first;
    const uint32_t* child;
    const int* lev;
    int nlev;
    const float* table;
};
struct FilterJobs {
    FilterJob j[2];
};

// Filter (SegmentTree.cpp:148-181) of disparity d = blockIdx.x of job blockIdx.y (ST-2 filters the left
// and right views' volumes in one launch: each job has only D workgroups).
#ifndef SM_ST_FILTER_THREADS
#define SM_ST_FILTER_THREADS 1024
#endif
constexpr int kFT = SM_ST_FILTER_THREADS;
__global__ __launch_bounds__(kFT) void st_filter_kernel(FilterJobs jobs, int P) {
#pragma clang fp contract(off)
    const FilterJob& jb = jobs.j[blockIdx.y];
    const int* __restrict__ parent = jb.parent;
    const uint8_t* __restrict__ pdist = jb.pdist;
    const int* __restrict__ first = jb.first;
    const uint32_t* __restrict__ child = jb.child;
    const int* __restrict__ lev = jb.lev;
    const int nlev = jb.nlev;
    __shared__ float table[256];
    for (int k = threadIdx.x; k < 256; k += blockDim.x) table[k] = jb.table[k];
    __syncthreads();
    float* __restrict__ U = jb.C + (int64_t)blockIdx.x * P;
    float* __restrict__ Fd = jb.F + (int64_t)blockIdx.x * P;
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

// ---- the same filter, one wave per disparity (st_filter_wave_kernel) ----
// A tree level's values depend only on the next (leaf to root) or the previous (root to leaf) level,
// and in BFS order the children of one level are exactly the next level, contiguous.  So one wave per
// disparity walks the levels with the two live levels in LDS (ping-pong buffers of the widest
// level), wave-synchronous: no workgroup barrier and no global store -> load round trip per level,
// which bound st_filter_kernel (~0.7 us per level).  The host cuts every level into tasks of <= 64
// nodes (one node per lane), each an int4 {x = first node, count - 1, LDS byte offset of the task's
// first node in its level buffer, LDS byte offset that the node index of a child (up) / parent (down)
// is added to}.
//
// The tasks run in blocks of kStBlk.  While block b runs, the wave's global loads for block b + 1 (its
// lanes' node operands) and the records of block b + 2 are in flight; they land in LDS at the end of
// the block (a wait that is long satisfied by then), where block b + 1 reads them.  Staging through LDS
// keeps every load and its wait in one loop iteration: a register ring carried across the loop's back
// edge made the compiler drain all loads (vmcnt(0)) once per trip.  Global memory goes through buffer
// descriptors (32-bit offsets).
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));   // 16 B in memory (a 3-vector is padded)
typedef int i32x4 __attribute__((ext_vector_type(4)));
constexpr int kStBlk = 16;                              // tasks per block: the 64 lanes load 16 int4 records
constexpr int kStNodeOff = 1024;                        // LDS: [0, 1024) the weight table
constexpr int kStRecOff = kStNodeOff + kStBlk * 64 * (int)sizeof(u32x3);   // [kStBlk][64 lanes] node operands
constexpr int kStZeroOff = kStRecOff + 2 * kStBlk * 16;  // [2 blocks][kStBlk] records, then a float 0
constexpr int kStLvlOff = kStZeroOff + 16;               // then the level buffers

struct WaveJob {
    float* C;                  // in: cost, out: leaf-to-root sums (read again by the root-to-leaf pass)
    float* F;                  // out: filtered cost
    const int* parent;
    const uint8_t* pdist;
    const int* first;
    const uint32_t* child;
    const int4* task;          // [n_up tasks, leaf to root][n_dn tasks, root to leaf]
    int n_up, n_dn;            // the task records carry the LDS offsets
    const float* table;
};
struct WaveJobs {
    WaveJob j[2];
};

using BufRsrc = __amdgpu_buffer_rsrc_t;
__device__ __forceinline__ BufRsrc buf_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)bytes, 0x00020000);
}
constexpr int kAuxSc1 = 16;   // sc1: the load misses the (non-coherent) L1, as an agent-scope atomic load
template <int AUX = 0>
__device__ __forceinline__ uint32_t buf_ld(BufRsrc r, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, AUX);
}
// one wave per CU at most (D or 2 D waves on 256 CUs): the compiler may schedule for latency, not occupancy
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1))) void st_filter_wave_kernel(WaveJobs jobs,
                                                                                                       int P) {
#pragma clang fp contract(off)
    const WaveJob& jb = jobs.j[blockIdx.y];
    extern __shared__ float sbuf[];          // layout: kSt*Off above
    const int lane = threadIdx.x;
    for (int k = lane; k < 256; k += 64) sbuf[k] = jb.table[k];
    if (lane == 0) sbuf[kStZeroOff / 4] = 0.0f;
    const uint32_t Pb = (uint32_t)P * 4u;
    const BufRsrc rU = buf_rsrc(jb.C + (int64_t)blockIdx.x * P, Pb);
    const BufRsrc rF = buf_rsrc(jb.F + (int64_t)blockIdx.x * P, Pb);
    char* lds = reinterpret_cast<char*>(sbuf);
    auto lds_f = [&](int off) -> float& { return *reinterpret_cast<float*>(lds + off); };
    u32x3* node_area = reinterpret_cast<u32x3*>(lds + kStNodeOff);   // [k][lane]
    i32x4* rec_area = reinterpret_cast<i32x4*>(lds + kStRecOff);     // [block parity][k]
    __syncthreads();

    // node_load(record) -> u32x3 of this lane's node; body(record, node operands)
    auto pass = [&](const int4* tk0, int nt, auto node_load, auto body) {
        if (nt <= 0) return;
        const BufRsrc rT = buf_rsrc(tk0, (uint32_t)nt * 16u);
        // lane l loads dword l & 3 of record (block start + l / 4), clamped to the last task
        auto rec_block = [&](int blk) {
            const int t = min(blk * kStBlk + (lane >> 2), nt - 1);
            return (int)buf_ld(rT, (uint32_t)t * 16u + (uint32_t)(lane & 3) * 4u);
        };
        auto rec_put = [&](int parity, int v) { reinterpret_cast<int*>(rec_area + parity * kStBlk)[lane] = v; };
        // the node loads of a block need each record's first node and count - 1: one LDS dword per lane
        // (lane l: dword l & 3 of record l / 4) read out with v_readlane, rather than 16 128-bit reads
        // whose registers the compiler overlaps (and then serialises)
        auto gather = [&](int parity, u32x3* g) {
            const int rv = reinterpret_cast<const int*>(rec_area + parity * kStBlk)[lane];
#pragma unroll
            for (int k = 0; k < kStBlk; ++k) {
                i32x4 rr;
                rr.x = __builtin_amdgcn_readlane(rv, 4 * k);
                rr.y = __builtin_amdgcn_readlane(rv, 4 * k + 1);
                rr.z = rr.w = 0;
                g[k] = node_load(rr);
            }
        };
        const int nb = (nt + kStBlk - 1) / kStBlk;
        // prologue: records of blocks 0 and 1, node operands of block 0
        rec_put(0, rec_block(0));
        const int r1 = rec_block(1);
        {
            u32x3 g[kStBlk];
            gather(0, g);
#pragma unroll
            for (int k = 0; k < kStBlk; ++k) node_area[k * 64 + lane] = g[k];
        }
        rec_put(1, r1);
        for (int b = 0; b < nb; ++b) {
            const int cur = b & 1;
            // loads for later blocks: the records of block b + 2, the node operands of block b + 1
            const int rn = rec_block(b + 2);
            u32x3 g[kStBlk];
            gather(cur ^ 1, g);
            // block b: its records and node operands all read before the first level write
            i32x4 rc[kStBlk];
            u32x3 nd[kStBlk];
#pragma unroll
            for (int k = 0; k < kStBlk; ++k) {
                rc[k] = rec_area[cur * kStBlk + k];
                nd[k] = node_area[k * 64 + lane];
            }
            // no branches: a block past the last task repeats the last task (records clamped), which
            // rewrites the same values
#pragma unroll
            for (int k = 0; k < kStBlk; ++k) body(rc[k], nd[k]);
            // stage block b + 1's operands and block b + 2's records
#pragma unroll
            for (int k = 0; k < kStBlk; ++k) node_area[k * 64 + lane] = g[k];
            rec_put(cur, rn);
        }
    };
    // byte offset of this lane's node (lanes past the task's count repeat its last node); the store
    // offset of those lanes lies past the buffer's end, where the hardware drops the store
    auto node_off = [&](const i32x4& r) { return (uint32_t)(r.x + min(lane, r.y)) * 4u; };
    auto store_off = [&](const i32x4& r) { return lane <= r.y ? (uint32_t)(r.x + lane) * 4u : 0x80000000u; };

    // ---- leaf to root: u = C[i] + sum_z table[dist_z] * u(child z), children in order ----
    const BufRsrc rChild = buf_rsrc(jb.child, Pb), rFirst = buf_rsrc(jb.first, Pb);
    pass(jb.task, jb.n_up,
         [&](const i32x4& r) {
             const uint32_t o = node_off(r);
             return u32x3{buf_ld(rU, o), buf_ld(rChild, o), buf_ld(rFirst, o)};
         },
         [&](const i32x4& r, const u32x3& n0) {
             // every lane computes (those past the count into the level buffer's 64-float pad)
             {
                 const uint32_t ch = n0.y;
                 const int n = (int)(ch & 0xFFu);
                 const int rd = r.w + (int)n0.z * 4;
                 float u = __builtin_bit_cast(float, n0.x);
                 // at most 3 children (a grid node has 4 neighbours, one of them its parent; the root is
                 // the corner pixel 0): all six LDS reads issued together.  An absent child reads the
                 // float 0 (its distance byte is 0, weight 1): its term is +0, and u + 0 = u exactly for the
                 // non-negative sums here, so the chain after the reads is one multiply and three adds.
                 float cv[3], wv[3];
#pragma unroll
                 for (int z = 0; z < 3; ++z) {
                     cv[z] = lds_f(z < n ? rd + 4 * z : kStZeroOff);
                     wv[z] = sbuf[(ch >> (8 * (z + 1))) & 0xFFu];
                 }
#pragma unroll
                 for (int z = 0; z < 3; ++z) {
                     const float tt = cv[z] * wv[z];
                     u = u + tt;
                 }
                 lds_f(r.z + lane * 4) = u;
                 // a leaf's u is its C: rewritten unchanged
                 __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, u), rU, store_off(r), 0, 0);
             }
         });
    __syncthreads();   // the U stores have completed (vmcnt) before the root-to-leaf pass reads them back

    // ---- root to leaf: F[i] = w (F[parent] - w U[i]) + U[i] ----
    if (lane == 0) {
        const float u0 = __builtin_bit_cast(float, buf_ld<kAuxSc1>(rU, 0));
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, u0), rF, 0, 0, 0);
        lds_f(kStLvlOff) = u0;   // level 0 (the root) has parity 0
    }
    __builtin_amdgcn_wave_barrier();
    const BufRsrc rParent = buf_rsrc(jb.parent, Pb), rDist = buf_rsrc(jb.pdist, (uint32_t)P);
    pass(jb.task + jb.n_up, jb.n_dn,
         [&](const i32x4& r) {
             const uint32_t o = node_off(r);
             // U was written by this wave's leaf-to-root pass: read past the (non-coherent) L1
             return u32x3{buf_ld<kAuxSc1>(rU, o), buf_ld(rParent, o),
                          (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rDist, o >> 2, 0, 0)};
         },
         [&](const i32x4& r, const u32x3& n0) {
             {
                 const float w = sbuf[n0.z], u = __builtin_bit_cast(float, n0.x);
                 const float tt = w * u;
                 const float fv = w * (lds_f(r.w + (int)n0.y * 4) - tt) + u;
                 lds_f(r.z + lane * 4) = fv;
                 __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, fv), rF, store_off(r), 0, 0);
             }
         });
}

// node[i] = the pixel at BFS index i (the inverse of rank)
__global__ __launch_bounds__(kST) void st_node_kernel(const int* __restrict__ rank, int P, int* __restrict__ node) {
    const int p = blockIdx.x * kST + threadIdx.x;
    if (p >= P) return;
    const int i = rank[p];
    if ((unsigned)i < (unsigned)P) node[i] = p;
}

// GetDisparity_WTA (StereoHelper.cpp:131-154): strict < from d = 0; times scale, saturated.  One thread
// per BFS index, so the D cost reads of a wave are coalesced (round 4: per pixel, they were gathers
// through rank, 62 -> 9 us for Art at D = 60); the result goes to its pixel.
__global__ __launch_bounds__(kST) void st_wta_kernel(const float* __restrict__ F, const int* __restrict__ node, int P,
                                                     int D, int scale, uint8_t* __restrict__ out) {
    const int i = blockIdx.x * kST + threadIdx.x;
    if (i >= P) return;
    float v = F[i];
    int m = 0;
    for (int d = 1; d < D; ++d) {
        const float c = F[(int64_t)d * P + i];
        if (c < v) {
            v = c;
            m = d;
        }
    }
    const int p = node[i];
    if ((unsigned)p < (unsigned)P) out[p] = (uint8_t)min(m * scale, 255);
}

// ---- the edge order on the GPU: SegmentTree.cpp:44-69's edges sorted by edge::operator< (weight, then
// b, then a; SegmentTree.h:103-111) ----
// Edges are generated in (b, a) order and sorted stably by weight (LSD radix, 8-bit digits: one pass for
// the integer colour weights, four for the colour + depth floats, whose non-negative values order as
// their bits), which is that order.  Edge index of pixel b = (y, x): in a row y < H - 1 the edges of b
// are (b - 1, b) for x >= 1 then (b + W, b), so row y starts at y (2W - 1); the last row has (b - 1, b)
// only.  Value = 2 b + (edge is (b + W, b)).
__host__ __device__ inline int64_t st_edge_count(int W, int H) { return (int64_t)(H - 1) * (2 * W - 1) + (W - 1); }

// DEPTH = false: key = colour weight (u8); DEPTH = true: CColorDepthWeight::GetWeight (SegmentTree.cpp:
// 204-219) from the colour weight, the first left map and its mask, in the reference's float steps
// (as st_host::depth_weights), key = the float's bits.
template <bool DEPTH>
__global__ __launch_bounds__(kST) void st_edge_keys_kernel(const uint8_t* __restrict__ wr, const uint8_t* __restrict__ wu,
                                                           const uint8_t* __restrict__ disp,
                                                           const uint8_t* __restrict__ mask, float level, int W, int H,
                                                           uint32_t* __restrict__ keys, uint32_t* __restrict__ vals) {
#pragma clang fp contract(off)
    const int x = blockIdx.x * kST + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const int b = y * W + x;
    auto key = [&](int a, int q, uint8_t c) -> uint32_t {
        if constexpr (DEPTH) {
            float w;
            if (mask[a] && mask[q]) {
                const float dispValue = (float)abs((int)disp[a] - (int)disp[q]) / level;
                const float colorValue = (float)c / 255.0f;
                w = 0.5f * dispValue + (1.0f - 0.5f) * colorValue;
            } else {
                w = (float)c / 255.0f;
            }
            return __builtin_bit_cast(uint32_t, w);
        } else {
            return c;
        }
    };
    const int64_t base = (int64_t)y * (2 * W - 1);
    if (y < H - 1) {
        if (x >= 1) {
            keys[base + 2 * x - 1] = key(b - 1, b, wr[b - 1]);   // (b - 1, b): right edge of b - 1
            vals[base + 2 * x - 1] = 2u * (uint32_t)b;
        }
        const int64_t iu = x >= 1 ? base + 2 * x : base;
        keys[iu] = key(b + W, b, wu[b + W]);                     // (b + W, b): upper edge of b + W
        vals[iu] = 2u * (uint32_t)b + 1u;
    } else if (x >= 1) {
        keys[base + x - 1] = key(b - 1, b, wr[b - 1]);
        vals[base + x - 1] = 2u * (uint32_t)b;
    }
}

// one radix pass: single-wave blocks of R * 64 consecutive items, 64 per round (the edge sort: kRxRounds;
// the device BFS's scans and depth sort: kScRounds, 4x the waves for its P-item passes)
constexpr int kRxRounds = 32;
constexpr int kRxIPB = 64 * kRxRounds;
constexpr int kScRounds = 8;
constexpr int kScIPB = 64 * kScRounds;

// gate (the device BFS's sort of depths, bm_segtree.hip st_radix_passes_run): a pass with shift > 0 whose
// digit is 0 for every key (gate[4] = the largest key) does nothing; null for the edge sort
__device__ __forceinline__ bool st_rx_skip(const int* gate, int shift) {
    return gate && shift > 0 && (gate[4] >> shift) == 0;
}

template <int R>
__global__ __launch_bounds__(64) void st_rx_hist_kernel(const uint32_t* __restrict__ keys, int n, int shift,
                                                        uint32_t* __restrict__ hist, int nb, const int* gate) {
    if (st_rx_skip(gate, shift)) return;
    __shared__ uint32_t h[256];
    const int lane = threadIdx.x, blk = blockIdx.x;
    for (int k = lane; k < 256; k += 64) h[k] = 0;
    __syncthreads();
    for (int r = 0; r < R; ++r) {
        const int i = blk * R * 64 + r * 64 + lane;
        if (i < n) atomicAdd(&h[(keys[i] >> shift) & 0xFFu], 1u);
    }
    __syncthreads();
    for (int k = lane; k < 256; k += 64) hist[(size_t)k * nb + blk] = h[k];
}

// exclusive scan of the digit-major counts [256][nb]: each digit's row scanned over the blocks by one
// wave (st_rx_scan_rows_kernel, also writing the row total), then the 256 totals by one wave into the
// digits' bases (st_rx_scan_bases_kernel), which the scatter adds
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t u = __shfl_up(v, off, 64);
        if (lane >= off) v += u;
    }
    return v;
}
__global__ __launch_bounds__(64) void st_rx_scan_rows_kernel(uint32_t* __restrict__ hist, int nb,
                                                             uint32_t* __restrict__ total, const int* gate, int shift) {
    if (st_rx_skip(gate, shift)) return;
    const int lane = threadIdx.x, dg = blockIdx.x;
    uint32_t* row = hist + (size_t)dg * nb;
    uint32_t run = 0;
    for (int b0 = 0; b0 < nb; b0 += 64) {
        const int b = b0 + lane;
        const uint32_t c = b < nb ? row[b] : 0u;
        const uint32_t inc = wave_incl_scan(c, lane);
        if (b < nb) row[b] = run + inc - c;
        run += __shfl(inc, 63, 64);
    }
    if (lane == 0) total[dg] = run;
}
__global__ __launch_bounds__(64) void st_rx_scan_bases_kernel(uint32_t* __restrict__ total, const int* gate, int shift) {
    if (st_rx_skip(gate, shift)) return;
    const int lane = threadIdx.x;
    uint32_t run = 0;
    for (int d0 = 0; d0 < 256; d0 += 64) {
        const uint32_t c = total[d0 + lane];
        const uint32_t inc = wave_incl_scan(c, lane);
        total[d0 + lane] = run + inc - c;
        run += __shfl(inc, 63, 64);
    }
}

// stable scatter of one pass: an item's position = its digit's offset for the block + the items of the
// same digit before it in the block (earlier rounds: the running counts cnt; this round: the lanes below
// it whose 8 digit bits all agree, from 8 ballots).  FINAL: write the edge records {a, b, w} instead of
// keys and values.
template <bool FINAL, bool DEPTH, int R = kRxRounds>
__global__ __launch_bounds__(64) void st_rx_scatter_kernel(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                           int n, int shift, const uint32_t* __restrict__ hist,
                                                           const uint32_t* __restrict__ bases, int nb,
                                                           uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                           st_host::Edge* __restrict__ eout, int W, const int* gate,
                                                           int* __restrict__ sidx = nullptr) {
    if (st_rx_skip(gate, shift)) return;
    __shared__ uint32_t cnt[256];
    const int lane = threadIdx.x, blk = blockIdx.x;
    for (int k = lane; k < 256; k += 64) cnt[k] = bases[k] + hist[(size_t)k * nb + blk];
    __syncthreads();
    const uint64_t lt = (1ull << lane) - 1ull;
    for (int r = 0; r < R; ++r) {
        const int i = blk * R * 64 + r * 64 + lane;
        const bool valid = i < n;
        const uint32_t k = valid ? kin[i] : 0u, v = valid ? vin[i] : 0u;
        const uint32_t dg = (k >> shift) & 0xFFu;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int bit = 0; bit < 8; ++bit) {
            const bool on = (dg >> bit) & 1u;
            const uint64_t bb = __ballot(on);
            peers &= on ? bb : ~bb;
        }
        const uint32_t base = cnt[dg];
        __builtin_amdgcn_wave_barrier();
        // the lowest lane of each digit group advances the digit's count (after every lane has read it)
        if (valid && (peers & lt) == 0) cnt[dg] = base + (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        if (valid) {
            const uint32_t pos = base + (uint32_t)__popcll(peers & lt);
            if constexpr (FINAL) {
                const int b = (int)(v >> 1);
                eout[pos] = st_host::Edge{(v & 1u) ? b + W : b - 1, b,
                                          DEPTH ? __builtin_bit_cast(float, k) : (float)k};
                sidx[v] = (int)pos;   // grid edge v's sorted position (st_adj_kernel)
            } else {
                kout[pos] = k;
                vout[pos] = v;
            }
        }
    }
}

// ---- the BFS order on the GPU (round 4) ----
// The host keeps segment_graph's two passes (sequential: every join's threshold depends on the joins
// before it) and hands over the neighbour lists (st_host::AdjRec, 8 B per pixel: four distance bytes,
// four 2-bit directions, the count).  The BFS of SegmentTree.cpp:97-130 (FIFO from pixel 0, a node's
// children in list order) follows from them without walking the levels one by one:
//  1. an Euler tour of the tree (arc p -> q continues from q to the neighbour after p in q's list,
//     cyclically), ranked by pointer jumping (Wyllie), roots the tree: u is v's parent iff arc u -> v
//     comes before v -> u, and v's subtree has (dist(u -> v) - dist(v -> u) + 1) / 2 nodes, dist being
//     the number of arcs after an arc;
//  2. a node's children in list order (the parent skipped) get the preorder offsets 1 + the sizes of
//     their earlier siblings.  A prefix sum along the tour of {+1, +offset(v)} on each arc into v and
//     {-1, -offset(v)} on each arc out of v's subtree leaves, at the arc into v, exactly the terms of v's
//     ancestors and v (a finished subtree cancels, whatever the tour's order): v's depth and preorder
//     number;
//  3. in a FIFO BFS the nodes of one level come in preorder (by induction over the levels: nodes with
//     different parents follow their parents' order, whose subtrees are disjoint preorder intervals in
//     that order; siblings follow the list order), so the BFS order is the preorder stably sorted by
//     depth (the edge sort's radix passes, those above the deepest level's top bit skipped);
//  4. rank, child words and level offsets from that order; first = 1 + the exclusive scan of the child
//     counts (the BFS appends a node's children at the running end), and each node writes its children's
//     parent index and distance byte there; the wave filter's tasks (wave_tasks' layout) from a scan of
//     the per-level task counts.
// The same arrays as st_host::bfs_tree, bit for bit (tests/test_gpu_segtree.py compares both).
static_assert(sizeof(st_host::AdjRec) == 8, "AdjRec is read as a uint2 {d, dir | n << 16}");

__device__ __forceinline__ int st_nb(int p, uint32_t dir, int k, int W) {
    const uint32_t c = (dir >> (2 * k)) & 3u;
    return c == 0 ? p - 1 : c == 1 ? p + 1 : c == 2 ? p - W : p + W;
}

// The neighbour lists from the host passes' marks (segment_passes): pixel p's tree edges in sorted-edge
// order, as segment_lists appends them (SegmentTree.cpp:74-95), each with its direction code (0: p - 1,
// 1: p + 1, 2: p - W, 3: p + W) and distance min(int(w' * wscale + 0.5), 255), w' = w (+ 5 when
// penalised, st_host::tree_dist).  Grid edge v = 2 b + (edge is (b + W, b)) sits at sorted position
// sidx[v].  Out: AdjRec bits {d, dir | n << 16}.
__global__ __launch_bounds__(kST) void st_adj_kernel(const st_host::Edge* __restrict__ edges, const int* __restrict__ sidx,
                                                     const uint8_t* __restrict__ marks, int W, int P, float wscale,
                                                     uint2* __restrict__ adj) {
#pragma clang fp contract(off)
    const int p = blockIdx.x * kST + threadIdx.x;
    if (p >= P) return;
    const int x = p % W;
    int pos[4];
    uint32_t cd[4];   // direction code | distance << 8
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const bool ex = c == 0 ? x >= 1 : c == 1 ? x + 1 < W : c == 2 ? p >= W : p + W < P;
        const int v = c == 0 ? 2 * p : c == 1 ? 2 * (p + 1) : c == 2 ? 2 * (p - W) + 1 : 2 * p + 1;
        pos[c] = INT_MAX;
        cd[c] = 0;
        if (ex) {
            const int q = sidx[v];
            const uint8_t m = marks[q];
            if (m & 1u) {
                float w = edges[q].w;
                if (m & 2u) w += 5;
                const float sw = w * wscale;
                pos[c] = q;
                cd[c] = (uint32_t)c | ((uint32_t)min((int)(sw + 0.5f), 255) << 8);
            }
        }
    }
    // sort the (at most 4) tree edges by sorted position
#pragma unroll
    for (int i = 1; i < 4; ++i)
#pragma unroll
        for (int j = i; j > 0; --j)
            if (pos[j] < pos[j - 1]) {
                const int tp = pos[j];
                pos[j] = pos[j - 1];
                pos[j - 1] = tp;
                const uint32_t tc = cd[j];
                cd[j] = cd[j - 1];
                cd[j - 1] = tc;
            }
    uint32_t d = 0, dir = 0, n = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (pos[k] != INT_MAX) {
            d |= (cd[k] >> 8) << (8 * k);
            dir |= (cd[k] & 3u) << (2 * k);
            ++n;
        }
    adj[p] = make_uint2(d, dir | (n << 16));
}

// arcs: slot k of pixel p is arc 4 p + k {next arc of the tour, 1}; the arc into arc 0 (pixel 0 to its
// first neighbour, where the tour starts) ends it {-1, 0}, and so do the unused slots; rev = the reverse
// arc (an unused slot: itself)
__global__ __launch_bounds__(kST) void st_arc_kernel(const uint2* __restrict__ adj, int P, int W,
                                                     int2* __restrict__ arc, int* __restrict__ rev) {
    const int p = blockIdx.x * kST + threadIdx.x;
    if (p >= P) return;
    const uint2 a = adj[p];
    const int n = (int)(a.y >> 16);
    const uint32_t dir = a.y & 0xFFFFu;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int2 r = make_int2(-1, 0);
        int rv = 4 * p + k;
        if (k < n) {
            const int q = st_nb(p, dir, k, W);
            const uint2 b = adj[q];
            const int nq = (int)(b.y >> 16);
            const uint32_t back = ((dir >> (2 * k)) & 3u) ^ 1u, dq = b.y & 0xFFFFu;
            int j = -1;
#pragma unroll
            for (int z = 0; z < 4; ++z)
                if (z < nq && ((dq >> (2 * z)) & 3u) == back) j = z;
            if (j >= 0) {
                rv = 4 * q + j;
                const int nx = 4 * q + (j + 1 == nq ? 0 : j + 1);
                if (nx != 0) r = make_int2(nx, 1);
            }
        }
        arc[4 * p + k] = r;
        rev[4 * p + k] = rv;
    }
}

// one pointer-jumping step: {next, count} -> {next of next, count + its count}
__global__ __launch_bounds__(kST) void st_list_rank_kernel(const int2* __restrict__ in, int2* __restrict__ out, int n) {
    const int a = blockIdx.x * kST + threadIdx.x;
    if (a >= n) return;
    int2 v = in[a];
    if (v.x >= 0) {
        const int2 w = in[v.x];
        v = make_int2(w.x, v.y + w.y);
    }
    out[a] = v;
}

// parent slot (4: the root) and subtree size of every pixel from the ranked tour
__global__ __launch_bounds__(kST) void st_root_kernel(const uint2* __restrict__ adj, const int2* __restrict__ rk,
                                                      const int* __restrict__ rev, int P, int* __restrict__ psl,
                                                      int* __restrict__ size) {
    const int p = blockIdx.x * kST + threadIdx.x;
    if (p >= P) return;
    int slot = 4, sz = P;
    if (p != 0) {
        const int n = (int)(adj[p].y >> 16);
        for (int k = 0; k < n; ++k) {
            const int da = rk[4 * p + k].y, db = rk[rev[4 * p + k]].y;
            if (db > da) {   // the arc into p comes first: its other end is the parent
                slot = k;
                sz = (db - da + 1) >> 1;
            }
        }
    }
    psl[p] = slot;
    size[p] = sz;
}

// every node writes its children's preorder offsets and its child word (count | distance bytes in list
// order, as bfs_tree's)
__global__ __launch_bounds__(kST) void st_child_kernel(const uint2* __restrict__ adj, const int* __restrict__ psl,
                                                       const int* __restrict__ size, int P, int W,
                                                       int* __restrict__ offs, uint32_t* __restrict__ chw) {
    const int p = blockIdx.x * kST + threadIdx.x;
    if (p >= P) return;
    const uint2 a = adj[p];
    const int n = (int)(a.y >> 16), ps = psl[p];
    int run = 1;
    uint32_t ch = 0, m = 0;
    for (int k = 0; k < n; ++k) {
        if (k == ps) continue;
        const int c = st_nb(p, a.y & 0xFFFFu, k, W);
        const uint32_t dis = (a.x >> (8 * k)) & 0xFFu;
        offs[c] = run;
        run += size[c];
        ch |= dis << (8 * (m + 1));
        ++m;
    }
    chw[p] = ch | m;
    if (p == 0) offs[0] = 0;
}

// {depth, preorder} weights of the arcs in tour order (position = L - 1 - dist, L = 2 (P - 1) arcs):
// into a child {+1, +offset}, to the parent {-1, -offset}; tv = the child an arc enters, else -1
struct U2 {
    uint32_t a, b;
};
__device__ __forceinline__ U2 operator+(U2 x, U2 y) { return U2{x.a + y.a, x.b + y.b}; }
__device__ __forceinline__ U2 operator-(U2 x, U2 y) { return U2{x.a - y.a, x.b - y.b}; }
__global__ __launch_bounds__(kST) void st_tour_kernel(const uint2* __restrict__ adj, const int2* __restrict__ rk,
                                                      const int* __restrict__ psl, const int* __restrict__ offs, int P,
                                                      int W, U2* __restrict__ tw, int* __restrict__ tv) {
    const int p = blockIdx.x * kST + threadIdx.x;
    if (p >= P) return;
    const uint2 a = adj[p];
    const int n = (int)(a.y >> 16), ps = psl[p], L = 2 * (P - 1);
    for (int k = 0; k < n; ++k) {
        const int pos = L - 1 - rk[4 * p + k].y;
        if ((unsigned)pos >= (unsigned)L) continue;
        if (k == ps) {
            tw[pos] = U2{~0u, (uint32_t)(-offs[p])};
            tv[pos] = -1;
        } else {
            const int q = st_nb(p, a.y & 0xFFFFu, k, W);
            tw[pos] = U2{1u, (uint32_t)offs[q]};
            tv[pos] = q;
        }
    }
}

// wave-wide inclusive scans of uint32_t / U2 (the U2 halves wrap independently: partial sums of the
// tour's weights go negative)
__device__ __forceinline__ uint32_t shfl_up_v(uint32_t v, int off) { return __shfl_up(v, off, 64); }
__device__ __forceinline__ U2 shfl_up_v(U2 v, int off) { return U2{__shfl_up(v.a, off, 64), __shfl_up(v.b, off, 64)}; }
__device__ __forceinline__ uint32_t shfl_v(uint32_t v, int l) { return __shfl(v, l, 64); }
__device__ __forceinline__ U2 shfl_v(U2 v, int l) { return U2{__shfl(v.a, l, 64), __shfl(v.b, l, 64)}; }
template <class V>
__device__ __forceinline__ V wave_scan_v(V v, int lane) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const V u = shfl_up_v(v, off);
        if (lane >= off) v = v + u;
    }
    return v;
}

// exclusive scan in blocks of kScIPB items, one wave each: the blocks' totals (st_scan_sums_kernel), one
// wave over the totals (st_scan_rows_kernel, also writing the grand total), then the items with their
// block's base (st_scan_apply_kernel: dst(i, exclusive prefix, item))
template <class V, class Src>
__global__ __launch_bounds__(64) void st_scan_sums_kernel(Src src, int n, V* __restrict__ sums) {
    const int lane = threadIdx.x, blk = blockIdx.x;
    V t{};
    for (int r = 0; r < kScRounds; ++r) {
        const int i = blk * kScIPB + r * 64 + lane;
        if (i < n) t = t + src(i);
    }
    t = wave_scan_v(t, lane);
    if (lane == 63) sums[blk] = t;
}
template <class V>
__global__ __launch_bounds__(64) void st_scan_rows_kernel(V* __restrict__ sums, int nb, V* __restrict__ total) {
    const int lane = threadIdx.x;
    V run{};
    for (int b0 = 0; b0 < nb; b0 += 64) {
        const int b = b0 + lane;
        const V c = b < nb ? sums[b] : V{};
        const V inc = wave_scan_v(c, lane);
        if (b < nb) sums[b] = run + inc - c;
        run = run + shfl_v(inc, 63);
    }
    if (lane == 0 && total) *total = run;
}
template <class V, class Src, class Dst>
__global__ __launch_bounds__(64) void st_scan_apply_kernel(Src src, int n, const V* __restrict__ sums, Dst dst) {
    const int lane = threadIdx.x, blk = blockIdx.x;
    V run = sums[blk];
    for (int r = 0; r < kScRounds; ++r) {
        const int i = blk * kScIPB + r * 64 + lane;
        const V c = i < n ? src(i) : V{};
        const V inc = wave_scan_v(c, lane);
        if (i < n) dst(i, run + inc - c, c);
        run = run + shfl_v(inc, 63);
    }
}

// the tour's prefix sums -> the nodes in preorder (key = depth, value = pixel); hdr[4] = the largest depth
struct StTourW {
    const U2* tw;
    __device__ U2 operator()(int i) const { return tw[i]; }
};
__global__ __launch_bounds__(64) void st_tour_apply_kernel(const U2* __restrict__ tw, const int* __restrict__ tv, int L,
                                                           const U2* __restrict__ sums, uint32_t* __restrict__ keys,
                                                           uint32_t* __restrict__ vals, int P, int* __restrict__ hdr) {
    const int lane = threadIdx.x, blk = blockIdx.x;
    U2 run = sums[blk];
    uint32_t dmax = 0;
    for (int r = 0; r < kScRounds; ++r) {
        const int i = blk * kScIPB + r * 64 + lane;
        const U2 c = i < L ? tw[i] : U2{0u, 0u};
        const U2 inc = wave_scan_v(c, lane);
        if (i < L) {
            const int v = tv[i];
            const U2 at = run + inc;   // inclusive: the arc into v counts v itself
            if (v >= 0 && at.b < (uint32_t)P) {
                keys[at.b] = at.a;
                vals[at.b] = (uint32_t)v;
                dmax = max(dmax, at.a);
            }
        }
        run = run + shfl_v(inc, 63);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) dmax = max(dmax, (uint32_t)__shfl_xor(dmax, off, 64));
    if (lane == 0) {
        atomicMax(&hdr[4], (int)dmax);
        if (blk == 0) {   // the root: depth 0, preorder 0
            keys[0] = 0;
            vals[0] = 0;
        }
    }
}

// radix passes above the deepest level's top bit are skipped (gate = hdr, gate[4] the largest depth):
// the pass results alternate A -> B -> A.., so the sorted order is in B after an odd number of passes
__device__ __forceinline__ int st_radix_passes_run(const int* hdr, int launched) {
    int e = 0;
    for (int k = 0; k < launched; ++k)
        if (k == 0 || (hdr[4] >> (8 * k)) != 0) ++e;
    return e;
}

// BFS-order arrays from the sorted nodes: rank, child words; lev[d] = the first node of depth d,
// lev[levels] = P; hdr {levels, widest level = 1 (st_level_sums_kernel raises it)}
__global__ __launch_bounds__(kST) void st_bfs_arrays_kernel(const uint32_t* __restrict__ kA, const uint32_t* __restrict__ vA,
                                                            const uint32_t* __restrict__ kB, const uint32_t* __restrict__ vB,
                                                            int launched, const uint32_t* __restrict__ chw, int P,
                                                            int* __restrict__ rank, uint32_t* __restrict__ child,
                                                            int* __restrict__ lev, int* __restrict__ hdr) {
    const int i = blockIdx.x * kST + threadIdx.x;
    if (i >= P) return;
    const bool inB = st_radix_passes_run(hdr, launched) & 1;
    const uint32_t* node = inB ? vB : vA;
    const uint32_t* dep = inB ? kB : kA;
    const uint32_t p = min(node[i], (uint32_t)P - 1u);
    rank[p] = i;
    child[i] = chw[p];
    const int d = (int)min(dep[i], (uint32_t)P - 1u);
    if (i == 0 || dep[i - 1] != dep[i]) lev[d] = i;
    if (i == P - 1) {
        lev[d + 1] = P;
        hdr[0] = d + 1;
        hdr[1] = 1;
    }
}

// first = 1 + the exclusive scan of the child counts; node i writes its children's parent index and
// distance byte (the root's: -1, 0)
struct StChildCount {
    const uint32_t* child;
    __device__ uint32_t operator()(int i) const { return child[i] & 0xFFu; }
};
struct StFirstOut {
    const uint32_t* child;
    int* first;
    int* parent;
    uint8_t* pdist;
    int P;
    __device__ void operator()(int i, uint32_t e, uint32_t n) const {
        const int f = 1 + (int)e;
        first[i] = f;
        const uint32_t ch = child[i];
        for (int z = 0; z < (int)n; ++z) {
            if (f + z < P) {
                parent[f + z] = i;
                pdist[f + z] = (uint8_t)(ch >> (8 * (z + 1)));
            }
        }
        if (i == 0) {
            parent[0] = -1;
            pdist[0] = 0;
        }
    }
};

// tasks of <= 64 nodes per level; the sums pass also raises hdr[1] to the widest level
struct StLevelTasks {
    const int* lev;
    const int* hdr;
    __device__ uint32_t operator()(int l) const { return l < hdr[0] ? (uint32_t)(lev[l + 1] - lev[l] + 63) / 64u : 0u; }
};
struct StIntOut {
    int* out;
    __device__ void operator()(int i, uint32_t e, uint32_t) const { out[i] = (int)e; }
};
__global__ __launch_bounds__(64) void st_level_sums_kernel(const int* __restrict__ lev, int* __restrict__ hdr, int n,
                                                           uint32_t* __restrict__ sums) {
    const int lane = threadIdx.x, blk = blockIdx.x, nlev = hdr[0];
    uint32_t t = 0;
    int wmax = 1;
    for (int r = 0; r < kScRounds; ++r) {
        const int l = blk * kScIPB + r * 64 + lane;
        if (l < n && l < nlev) {
            const int w = lev[l + 1] - lev[l];
            t += (uint32_t)(w + 63) / 64u;
            wmax = max(wmax, w);
        }
    }
    t = wave_scan_v(t, lane);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) wmax = max(wmax, __shfl_xor(wmax, off, 64));
    if (lane == 63) sums[blk] = t;
    if (lane == 0 && blk * kScIPB < nlev) atomicMax(&hdr[1], wmax);
}

// wave_tasks on the device: level l's up tasks after those of the levels below it in the up order
// (levels - 1 .. 0), its down tasks (levels 1 .. levels - 1) after the up list; E = the exclusive scan of
// the per-level task counts, hdr[2] its total (= the up tasks); writes hdr[3] = the down tasks
__global__ __launch_bounds__(kST) void st_task_kernel(const int* __restrict__ lev, const int* __restrict__ E,
                                                      int* __restrict__ hdr, int P, int4* __restrict__ task) {
    const int l = blockIdx.x * kST + threadIdx.x;
    const int nlev = hdr[0];
    if (l >= P || l >= nlev) return;
    const int stride = hdr[1] + 64, total = hdr[2];
    const int lo = lev[l], hi = lev[l + 1], q = l & 1, nt = (hi - lo + 63) / 64;
    auto cut = [&](int4* dst, int other) {
        const int rb = kStLvlOff + ((q ^ 1) * stride - other) * 4;
        for (int t = 0; t < nt; ++t) {
            const int s0 = lo + 64 * t;
            dst[t] = make_int4(s0, min(64, hi - s0) - 1, kStLvlOff + (q * stride + s0 - lo) * 4, rb);
        }
    };
    cut(task + (total - E[l] - nt), l + 1 < nlev ? lev[l + 1] : lo);
    if (l >= 1) cut(task + total + E[l] - 1, lev[l - 1]);   // level 0 has one task
    if (l == 0) hdr[3] = total - 1;
}

// The sorted edges of one tree into page-locked host slot `slot` of the workspace (asynchronous on s).
// DEPTH: colour + depth weights from the left map `disp` and its mask.
hipError_t gpu_sorted_edges(StWorkspace& ws, const uint8_t* wr, const uint8_t* wu, const uint8_t* disp,
                            const uint8_t* mask, float level, int W, int H, bool depth, int slot, hipStream_t s,
                            int& nE);

// ---- host: the tree, sequential as the reference's (bm_segtree_host.h) ----
using namespace st_host;

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

hipError_t gpu_sorted_edges(StWorkspace& ws, const uint8_t* wr, const uint8_t* wu, const uint8_t* disp,
                            const uint8_t* mask, float level, int W, int H, bool depth, int slot, hipStream_t s,
                            int& nE) {
    const int64_t n64 = st_edge_count(W, H);
    if (n64 <= 0 || n64 > (1 << 30)) return hipErrorInvalidValue;
    const int n = (int)n64, nb = (n + kRxIPB - 1) / kRxIPB;
    // keys / values x 2, digit counts; the edge records (3 dwords each) and sorted positions per slot
    const size_t need = (size_t)4 * n + (size_t)256 * (nb + 1);
    hipError_t e;
    if ((e = grow(ws.sortbuf, ws.sortbuf_n, need)) != hipSuccess) return e;
    if ((e = grow(ws.dedge[slot], ws.dedge_n[slot], (size_t)3 * n)) != hipSuccess) return e;
    if ((e = grow(ws.sidx[slot], ws.sidx_n[slot], (size_t)2 * W * H)) != hipSuccess) return e;
    const size_t hbytes = (size_t)n * sizeof(st_host::Edge);
    if (ws.h_edges_n[slot] < hbytes) {
        if (ws.h_edges[slot]) (void)hipHostFree(ws.h_edges[slot]);
        ws.h_edges[slot] = nullptr;
        ws.h_edges_n[slot] = 0;
        if ((e = hipHostMalloc(&ws.h_edges[slot], hbytes, hipHostMallocDefault)) != hipSuccess) return e;
        ws.h_edges_n[slot] = hbytes;
    }
    uint32_t* k0 = ws.sortbuf;
    uint32_t* v0 = k0 + n;
    uint32_t* k1 = v0 + n;
    uint32_t* v1 = k1 + n;
    uint32_t* hist = v1 + n;
    uint32_t* bases = hist + (size_t)256 * nb;
    auto* edges = reinterpret_cast<st_host::Edge*>(ws.dedge[slot]);
    int* sidx = ws.sidx[slot];
    const dim3 rows((unsigned)((W + kST - 1) / kST), (unsigned)H);
    if (depth)
        hipLaunchKernelGGL(st_edge_keys_kernel<true>, rows, dim3(kST), 0, s, wr, wu, disp, mask, level, W, H, k0, v0);
    else
        hipLaunchKernelGGL(st_edge_keys_kernel<false>, rows, dim3(kST), 0, s, wr, wu, disp, mask, level, W, H, k0, v0);
    const int passes = depth ? 4 : 1;
    for (int ps = 0; ps < passes; ++ps) {
        const int shift = 8 * ps;
        hipLaunchKernelGGL(st_rx_hist_kernel<kRxRounds>, dim3((unsigned)nb), dim3(64), 0, s, k0, n, shift, hist, nb, nullptr);
        hipLaunchKernelGGL(st_rx_scan_rows_kernel, dim3(256), dim3(64), 0, s, hist, nb, bases, nullptr, shift);
        hipLaunchKernelGGL(st_rx_scan_bases_kernel, dim3(1), dim3(64), 0, s, bases, nullptr, shift);
        if (ps + 1 < passes) {
            hipLaunchKernelGGL((st_rx_scatter_kernel<false, false>), dim3((unsigned)nb), dim3(64), 0, s, k0, v0, n, shift,
                               hist, bases, nb, k1, v1, edges, W, nullptr);
            std::swap(k0, k1);
            std::swap(v0, v1);
        } else if (depth) {
            hipLaunchKernelGGL((st_rx_scatter_kernel<true, true>), dim3((unsigned)nb), dim3(64), 0, s, k0, v0, n, shift,
                               hist, bases, nb, k1, v1, edges, W, nullptr, sidx);
        } else {
            hipLaunchKernelGGL((st_rx_scatter_kernel<true, false>), dim3((unsigned)nb), dim3(64), 0, s, k0, v0, n, shift,
                               hist, bases, nb, k1, v1, edges, W, nullptr, sidx);
        }
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    nE = n;
    // down in kEdgeChunks copies, each followed by its event: the host tree's first pass starts on the
    // first chunk (wait_edges) while the rest is still in flight
    constexpr int K = StWorkspace::kEdgeChunks;
    const int chunk = (n + K - 1) / K;
    ws.edge_chunk[slot] = chunk;
    for (int k = 0; k < K; ++k) {
        if (!ws.edge_ev[slot][k] &&
            (e = hipEventCreateWithFlags(&ws.edge_ev[slot][k], hipEventDisableTiming)) != hipSuccess)
            return e;
        const int lo = std::min(n, k * chunk), hi = std::min(n, lo + chunk);
        if (hi > lo && (e = hipMemcpyAsync(static_cast<st_host::Edge*>(ws.h_edges[slot]) + lo, edges + lo,
                                           (size_t)(hi - lo) * sizeof(st_host::Edge), hipMemcpyDeviceToHost, s)) !=
                           hipSuccess)
            return e;
        if ((e = hipEventRecord(ws.edge_ev[slot][k], s)) != hipSuccess) return e;
    }
    return hipSuccess;
}

// Blocks until the sorted edges [0, upto) of `slot` have landed on the host (the chunk events of
// gpu_sorted_edges); false if an event reports an error.
bool wait_edges(StWorkspace& ws, int slot, int upto) {
    const int chunk = std::max(ws.edge_chunk[slot], 1);
    const int last = std::min(StWorkspace::kEdgeChunks, (upto + chunk - 1) / chunk);
    for (int k = 0; k < last; ++k)
        if (hipEventSynchronize(ws.edge_ev[slot][k]) != hipSuccess) return false;
    return true;
}

// One tree on the device: workspace slot k holds int [rank | parent | first | child | lev] (5P + 2),
// uint8 pdist (P) and the 256-entry weight table.
struct DevTree {
    int* rank;
    int* parent;
    int* first;
    uint32_t* child;
    int* lev;
    uint8_t* pdist;
    float* table;
    int nlev;
};

DevTree tree_slot(StWorkspace& ws, int64_t P, int k) {
    DevTree d{};
    d.rank = ws.tree_i + (size_t)k * (5 * P + 2);
    d.parent = d.rank + P;
    d.first = d.parent + P;
    d.child = reinterpret_cast<uint32_t*>(d.first + P);
    d.lev = reinterpret_cast<int*>(d.child + P);
    d.pdist = ws.tree_b + (size_t)k * P;
    d.table = ws.table + (size_t)k * 256;
    return d;
}

// UpdateTable (SegmentTree.cpp:141-146)
void weight_table(float sigma, float* table) {
    const float sg = std::max(0.01f, sigma);
    for (int i = 0; i <= 255; ++i) table[i] = std::exp(-float(i) / (255 * sg));
}

// Page-locked host tree of slot k (StWorkspace::h_tree): ints (5P + 2) in the device slot's layout, then
// pdist (P bytes); the slot's previous upload must have completed before a new tree is bound to it.
hipError_t host_tree_slot(StWorkspace& ws, int64_t P, int k, HostTree*& tp, bool hbfs = true) {
    if (!ws.host_tree[k]) ws.host_tree[k] = new HostTree();
    tp = static_cast<HostTree*>(ws.host_tree[k]);
    if (!hbfs) return hipSuccess;   // the device BFS: the host keeps only the passes' forest
    HostTree& t = *tp;
    const size_t need = (size_t)(5 * P + 2) * 4 + (size_t)P;
    if (ws.h_tree_n[k] < need) {
        if (ws.h_tree[k]) (void)hipHostFree(ws.h_tree[k]);
        ws.h_tree[k] = nullptr;
        ws.h_tree_n[k] = 0;
        const hipError_t e = hipHostMalloc(&ws.h_tree[k], need, hipHostMallocDefault);
        if (e != hipSuccess) return e;
        ws.h_tree_n[k] = need;
    }
    int* ints = static_cast<int*>(ws.h_tree[k]);
    t.bind((int)P, ints, reinterpret_cast<uint8_t*>(ints + 5 * P + 2));
    return hipSuccess;
}

// ---- the device BFS (st_arc_kernel ..): scratch and launch sequence ----
// SM_ST_HOST_BFS=1 builds the BFS on the host instead (st_host::bfs_tree, round 3's path), read at every
// call: the A/B baseline and the reference the GPU test compares the device arrays with
bool host_bfs_requested() {
    const char* e = std::getenv("SM_ST_HOST_BFS");
    return e && e[0] == '1';
}

struct BfsScratch {
    int2* arcA;        // 4P {next arc, arcs counted}, ping-pong
    int2* arcB;
    U2* tw;            // L = 2 (P - 1) tour weights
    uint2* adj;        // P neighbour lists
    U2* usums;         // tour scan block sums
    int* rev;          // 4P reverse arcs
    int* tv;           // L
    int* psl;          // P parent slots
    int* size;         // P subtree sizes
    int* offs;         // P preorder offsets
    uint32_t* chw;     // P child words per pixel
    uint32_t *kA, *vA, *kB, *vB;   // P each: depth keys and pixels of the radix passes
    uint32_t* hist;    // 256 (nb + 1)
    uint32_t* sums;    // nb + 2
    int* E;            // P + 2
    int* hdr;          // 8: {levels, widest level, up tasks, down tasks, largest depth}
    uint8_t* marks;    // nE: the host passes' marks
};

int64_t rx_blocks(int64_t n) { return (n + kScIPB - 1) / kScIPB; }

// ints of the scratch, carved in this order (8- and 16-B arrays first, at even offsets)
size_t bfs_scratch_ints(int64_t P, int64_t nE) {
    const int64_t L = 2 * (P - 1), nb = rx_blocks(P), nbL = rx_blocks(L);
    return (size_t)(8 * P * 2 + 2 * L + 2 * P + 2 * (nbL + 2) + 4 * P + L + 4 * P + 4 * P + 256 * (nb + 1) + (nb + 2) +
                    (P + 2) + 8 + (nE + 3) / 4);
}

BfsScratch bfs_scratch(int* base, int64_t P, int64_t nE) {
    const int64_t L = 2 * (P - 1), nb = rx_blocks(P), nbL = rx_blocks(L);
    BfsScratch b{};
    int* q = base;
    auto take = [&](int64_t n) {
        int* r = q;
        q += n;
        return r;
    };
    b.arcA = reinterpret_cast<int2*>(take(8 * P));
    b.arcB = reinterpret_cast<int2*>(take(8 * P));
    b.tw = reinterpret_cast<U2*>(take(2 * L));
    b.adj = reinterpret_cast<uint2*>(take(2 * P));
    b.usums = reinterpret_cast<U2*>(take(2 * (nbL + 2)));
    b.rev = take(4 * P);
    b.tv = take(L);
    b.psl = take(P);
    b.size = take(P);
    b.offs = take(P);
    b.chw = reinterpret_cast<uint32_t*>(take(P));
    b.kA = reinterpret_cast<uint32_t*>(take(P));
    b.vA = reinterpret_cast<uint32_t*>(take(P));
    b.kB = reinterpret_cast<uint32_t*>(take(P));
    b.vB = reinterpret_cast<uint32_t*>(take(P));
    b.hist = reinterpret_cast<uint32_t*>(take(256 * (nb + 1)));
    b.sums = reinterpret_cast<uint32_t*>(take(nb + 2));
    b.E = take(P + 2);
    b.hdr = take(8);
    b.marks = reinterpret_cast<uint8_t*>(take((nE + 3) / 4));
    return b;
}

// tasks per tree slot: up and down each <= P / 64 + levels, levels <= P
size_t task_slot_cap(int64_t P) { return (size_t)(2 * (P + P / 64 + 2)); }

int ceil_log2(int64_t n) {
    int r = 0;
    while (((int64_t)1 << r) < n) ++r;
    return r;
}

// The neighbour lists and their BFS from edge slot scr's marks (ws.h_marks[scr], page-locked, nE bytes,
// consumed once the copy has run) and sorted edges (ws.dedge / ws.sidx[scr], from gpu_sorted_edges) into
// device tree slot d and the wave filter's tasks into `task` (task_slot_cap(P) int4), all on stream s;
// the header {levels, widest level, up tasks, down tasks} lands in page-locked h_hdr once the stream has
// passed the copy this enqueues last.
hipError_t gpu_bfs(StWorkspace& ws, int scr, int P, int W, int nE, float wscale, const DevTree& d, int4* task,
                   int* h_hdr, hipStream_t s) {
    hipError_t e;
    if ((e = grow(ws.bfs[scr], ws.bfs_n[scr], bfs_scratch_ints(P, nE))) != hipSuccess) return e;
    const BfsScratch b = bfs_scratch(ws.bfs[scr], P, nE);
    const int L = 2 * (P - 1), nb = (int)rx_blocks(P), nbL = (int)rx_blocks(L);
    if ((e = hipMemsetAsync(b.hdr, 0, 8 * sizeof(int), s)) != hipSuccess) return e;
    if ((e = hipMemcpyAsync(b.marks, ws.h_marks[scr], (size_t)nE, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    const dim3 gP((unsigned)((P + kST - 1) / kST)), g4P((unsigned)((4 * (int64_t)P + kST - 1) / kST));
    // 0. the neighbour lists from the marks and the edge slot's sorted edges
    hipLaunchKernelGGL(st_adj_kernel, gP, dim3(kST), 0, s, reinterpret_cast<const st_host::Edge*>(ws.dedge[scr]),
                       ws.sidx[scr], b.marks, W, P, wscale, b.adj);
    // 1. rank the tour: jumps of 2^r cover its L arcs after ceil(log2 L) steps; root it
    hipLaunchKernelGGL(st_arc_kernel, gP, dim3(kST), 0, s, b.adj, P, W, b.arcA, b.rev);
    int2 *ain = b.arcA, *aout = b.arcB;
    for (int r = ceil_log2(L); r > 0; --r) {
        hipLaunchKernelGGL(st_list_rank_kernel, g4P, dim3(kST), 0, s, ain, aout, 4 * P);
        std::swap(ain, aout);
    }
    hipLaunchKernelGGL(st_root_kernel, gP, dim3(kST), 0, s, b.adj, ain, b.rev, P, b.psl, b.size);
    // 2. preorder offsets, the tour's prefix sums -> depth and preorder of every node
    hipLaunchKernelGGL(st_child_kernel, gP, dim3(kST), 0, s, b.adj, b.psl, b.size, P, W, b.offs, b.chw);
    hipLaunchKernelGGL(st_tour_kernel, gP, dim3(kST), 0, s, b.adj, ain, b.psl, b.offs, P, W, b.tw, b.tv);
    hipLaunchKernelGGL((st_scan_sums_kernel<U2, StTourW>), dim3((unsigned)nbL), dim3(64), 0, s, StTourW{b.tw}, L, b.usums);
    hipLaunchKernelGGL(st_scan_rows_kernel<U2>, dim3(1), dim3(64), 0, s, b.usums, nbL, nullptr);
    hipLaunchKernelGGL(st_tour_apply_kernel, dim3((unsigned)nbL), dim3(64), 0, s, b.tw, b.tv, L, b.usums, b.kA, b.vA, P,
                       b.hdr);
    // 3. stable sort by depth (< P): 8-bit digits up to P - 1's top bit, passes above the deepest level's
    // top bit skipped on the device
    uint32_t *k0 = b.kA, *v0 = b.vA, *k1 = b.kB, *v1 = b.vB;
    uint32_t* bases = b.hist + (size_t)256 * nb;
    int launched = 0;
    for (int shift = 0; shift < std::max(1, ceil_log2(P)); shift += 8, ++launched) {
        hipLaunchKernelGGL(st_rx_hist_kernel<kScRounds>, dim3((unsigned)nb), dim3(64), 0, s, k0, P, shift, b.hist, nb, b.hdr);
        hipLaunchKernelGGL(st_rx_scan_rows_kernel, dim3(256), dim3(64), 0, s, b.hist, nb, bases, b.hdr, shift);
        hipLaunchKernelGGL(st_rx_scan_bases_kernel, dim3(1), dim3(64), 0, s, bases, b.hdr, shift);
        hipLaunchKernelGGL((st_rx_scatter_kernel<false, false, kScRounds>), dim3((unsigned)nb), dim3(64), 0, s, k0, v0, P,
                           shift, b.hist, bases, nb, k1, v1, nullptr, W, b.hdr);
        std::swap(k0, k1);
        std::swap(v0, v1);
    }
    // 4. the BFS-order arrays, first / parent / pdist, the wave filter's tasks
    hipLaunchKernelGGL(st_bfs_arrays_kernel, gP, dim3(kST), 0, s, b.kA, b.vA, b.kB, b.vB, launched, b.chw, P, d.rank,
                       d.child, d.lev, b.hdr);
    const StChildCount cc{d.child};
    hipLaunchKernelGGL((st_scan_sums_kernel<uint32_t, StChildCount>), dim3((unsigned)nb), dim3(64), 0, s, cc, P, b.sums);
    hipLaunchKernelGGL(st_scan_rows_kernel<uint32_t>, dim3(1), dim3(64), 0, s, b.sums, nb, nullptr);
    hipLaunchKernelGGL((st_scan_apply_kernel<uint32_t, StChildCount, StFirstOut>), dim3((unsigned)nb), dim3(64), 0, s, cc,
                       P, b.sums, StFirstOut{d.child, d.first, d.parent, d.pdist, P});
    hipLaunchKernelGGL(st_level_sums_kernel, dim3((unsigned)nb), dim3(64), 0, s, d.lev, b.hdr, P, b.sums);
    hipLaunchKernelGGL(st_scan_rows_kernel<uint32_t>, dim3(1), dim3(64), 0, s, b.sums, nb,
                       reinterpret_cast<uint32_t*>(b.hdr + 2));
    hipLaunchKernelGGL((st_scan_apply_kernel<uint32_t, StLevelTasks, StIntOut>), dim3((unsigned)nb), dim3(64), 0, s,
                       StLevelTasks{d.lev, b.hdr}, P, b.sums, StIntOut{b.E});
    hipLaunchKernelGGL(st_task_kernel, gP, dim3(kST), 0, s, d.lev, b.E, b.hdr, P, task);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return hipMemcpyAsync(h_hdr, b.hdr, 4 * sizeof(int), hipMemcpyDeviceToHost, s);
}

// A tree bound by host_tree_slot: its level offsets join the ints, which go up as one copy (rank .. lev),
// then pdist and the weight table.  `t`'s slot and `table` must stay alive until the stream has consumed
// the copies.
hipError_t upload_tree(const HostTree& t, const float* table, int64_t P, DevTree& d, hipStream_t s) {
    d.nlev = (int)t.lev.size() - 1;
    if ((size_t)d.nlev + 1 > (size_t)P + 2) return hipErrorInvalidValue;
    int* ints = t.rank;
    std::copy(t.lev.begin(), t.lev.end(), ints + 4 * P);
    hipError_t e;
    if ((e = hipMemcpyAsync(d.rank, ints, ((size_t)4 * P + t.lev.size()) * 4, hipMemcpyHostToDevice, s)) != hipSuccess)
        return e;
    if ((e = hipMemcpyAsync(d.pdist, t.pdist, (size_t)P, hipMemcpyHostToDevice, s)) != hipSuccess) return e;
    return hipMemcpyAsync(d.table, table, 256 * sizeof(float), hipMemcpyHostToDevice, s);
}

// node[i] of tree d (the inverse of its rank) into `node` (P ints), for the cost volume and the WTA
hipError_t launch_node(const DevTree& d, int* node, int P, hipStream_t s) {
    hipLaunchKernelGGL(st_node_kernel, dim3((unsigned)((P + kST - 1) / kST)), dim3(kST), 0, s, d.rank, P, node);
    return hipGetLastError();
}

// the cost volume in tree d's BFS order (node: launch_node's), RIGHT: the right view's
template <bool RIGHT>
hipError_t launch_cost(const uint8_t* dL, const uint8_t* dR, int W, int H, int pitch, const float* grad, const int* node,
                       int D, float* C, hipStream_t s) {
    const int64_t P = (int64_t)W * H;
    hipLaunchKernelGGL(st_cost_kernel<RIGHT>, dim3((unsigned)((P + kST - 1) / kST)), dim3(kST), 0, s, dL, dR, W, H,
                       pitch, grad, grad + P, node, D, C);
    return hipGetLastError();
}

// WTA of the filtered cost F (BFS order) into the map `out` (pixel order); node: launch_node's
hipError_t launch_wta(const float* F, const int* node, int P, int D, int scale, uint8_t* out, hipStream_t s) {
    hipLaunchKernelGGL(st_wta_kernel, dim3((unsigned)((P + kST - 1) / kST)), dim3(kST), 0, s, F, node, P, D, scale, out);
    return hipGetLastError();
}

FilterJob filter_job(float* C, float* F, const DevTree& d) {
    return FilterJob{C, F, d.parent, d.pdist, d.first, d.child, d.lev, d.nlev, d.table};
}

// a level buffer holds the widest level and 64 floats of pad for the lanes past a task's count
int wave_level_stride(int maxw) { return maxw + 64; }

// The wave filter's tasks of one tree (st_filter_wave_kernel): every level cut into runs of <= 64 nodes,
// leaf to root, then root to leaf from level 1; each task {first node, count - 1, LDS byte offset of its
// first node in the level buffer of its level's parity, LDS byte offset that the index of a node of the
// level it reads (children up, parents down; the other parity's buffer) is added to}.  Returns the
// widest level, which sizes the buffers.
int wave_tasks(const HostTree& t, std::vector<int4>& out, int& n_up, int& n_dn) {
    const int nlev = (int)t.lev.size() - 1;
    out.clear();
    int maxw = 1;
    for (int l = 0; l < nlev; ++l) maxw = std::max(maxw, t.lev[l + 1] - t.lev[l]);
    const int stride = wave_level_stride(maxw);
    auto cut = [&](int l, int other) {
        const int lo = t.lev[l], hi = t.lev[l + 1], q = l & 1;
        const int rb = kStLvlOff + ((q ^ 1) * stride - other) * 4;
        for (int s0 = lo; s0 < hi; s0 += 64)
            out.push_back(make_int4(s0, std::min(64, hi - s0) - 1, kStLvlOff + (q * stride + s0 - lo) * 4, rb));
    };
    for (int l = nlev - 1; l >= 0; --l) cut(l, l + 1 < nlev ? t.lev[l + 1] : t.lev[l]);
    n_up = (int)out.size();
    for (int l = 1; l < nlev; ++l) cut(l, t.lev[l - 1]);
    n_dn = (int)out.size() - n_up;
    return maxw;
}

constexpr int kWaveMaxLevel = (65536 - kStLvlOff) / 8 - 64;   // 64 KB of LDS; wider trees keep st_filter_kernel

// One filter launch over 1 or 2 jobs: the wave filter when every level fits its LDS buffers, else the
// workgroup-per-disparity filter.
// SM_ST_WAVE_FILTER=0 forces the workgroup filter (the path of trees wider than the wave filter's LDS,
// which no bundled image reaches; tests/test_gpu_segtree.py runs it this way)
bool wave_filter_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("SM_ST_WAVE_FILTER");
        return !(e && e[0] == '0');
    }();
    return on;
}

hipError_t launch_filter(const FilterJobs& fj, const WaveJobs& wj, int njobs, int maxw, int D, int P, hipStream_t s) {
    if (maxw <= kWaveMaxLevel && wave_filter_enabled()) {
        hipLaunchKernelGGL(st_filter_wave_kernel, dim3((unsigned)D, (unsigned)njobs), dim3(64),
                           (size_t)kStLvlOff + (size_t)(2 * wave_level_stride(maxw)) * sizeof(float), s, wj, P);
    } else {
        hipLaunchKernelGGL(st_filter_kernel, dim3((unsigned)D, (unsigned)njobs), dim3(kFT), 0, s, fj, P);
    }
    return hipGetLastError();
}

// A built tree's filter inputs: its device slot, its tasks and their counts
struct TreeJob {
    DevTree d;
    int4* task;
    int maxw, n_up, n_dn;
};

// Neighbour-list storage of the host BFS path (the tree's own vector; its arrays take the page-locked
// slot); the device path builds the lists on the GPU (null)
AdjRec* list_storage(HostTree& t, bool hbfs, int64_t P) {
    if (!hbfs) return nullptr;
    t.adj.resize((size_t)P);
    return t.adj.data();
}

// The host part of one tree from the sorted edges of edge slot `slot`: segment_graph's passes, starting
// on the first downloaded chunk, into the slot's page-locked marks; with hbfs the neighbour lists and
// the BFS on the host instead.  False on a failed build.
bool host_tree_part(StWorkspace& ws, int slot, HostTree& t, AdjRec* adj, bool hbfs, int nE, int64_t P, int W, float tau,
                    float wscale) {
    bool arrived = true;
    auto hook = [&](int upto) { arrived = arrived && wait_edges(ws, slot, upto); };
    const Edge* e = static_cast<const Edge*>(ws.h_edges[slot]);
    if (hbfs) {
        segment_lists(e, nE, (int)P, tau, wscale, t, ws.edge_chunk[slot], hook, adj);
        return arrived && bfs_tree(adj, (int)P, W, t);
    }
    segment_passes(e, nE, (int)P, tau, t, ws.edge_chunk[slot], hook, static_cast<uint8_t*>(ws.h_marks[slot]),
                   [](int) {});
    return arrived;
}

// Enqueue tree slot k's device part: the weight table and the device BFS (header to h_hdr + 4 k, scratch
// ws.bfs[k]), or with hbfs the host tree's upload and its host tasks (`tv` must stay alive until the stream
// has run the copy).  The caller grows ws.task to task_slot_cap(P) per slot first.
hipError_t enqueue_tree(StWorkspace& ws, HostTree& t, bool hbfs, int64_t P, int W, int nE, float wscale,
                        const float* table, int k, hipStream_t s, std::vector<int4>& tv, TreeJob& j) {
    j.d = tree_slot(ws, P, k);
    j.task = reinterpret_cast<int4*>(ws.task) + task_slot_cap(P) * (size_t)k;
    hipError_t e;
    if (!ws.h_hdr) return hipErrorNotInitialized;   // tree_resources
    if (!hbfs) {
        if ((e = hipMemcpyAsync(j.d.table, table, 256 * sizeof(float), hipMemcpyHostToDevice, s)) != hipSuccess)
            return e;
        return gpu_bfs(ws, k, (int)P, W, nE, wscale, j.d, j.task, ws.h_hdr + 4 * k, s);
    }
    if ((e = upload_tree(t, table, P, j.d, s)) != hipSuccess) return e;
    j.maxw = wave_tasks(t, tv, j.n_up, j.n_dn);
    if (tv.size() > task_slot_cap(P)) return hipErrorInvalidValue;
    return hipMemcpyAsync(j.task, tv.data(), tv.size() * sizeof(int4), hipMemcpyHostToDevice, s);
}

// Per-call resources of the tree builds, allocated before any build thread starts: task slots for `trees`
// trees, the page-locked headers, the events and (two trees) the side stream
hipError_t tree_resources(StWorkspace& ws, int64_t P, int nE, int trees) {
    hipError_t e;
    if ((e = grow(ws.task, ws.task_n, task_slot_cap(P) * 4 * (size_t)trees)) != hipSuccess) return e;
    for (int k = 0; k < trees; ++k) {
        if (ws.h_marks_n[k] >= (size_t)nE) continue;
        if (ws.h_marks[k]) (void)hipHostFree(ws.h_marks[k]);
        ws.h_marks[k] = nullptr;
        ws.h_marks_n[k] = 0;
        if ((e = hipHostMalloc(&ws.h_marks[k], (size_t)nE, hipHostMallocDefault)) != hipSuccess) return e;
        ws.h_marks_n[k] = (size_t)nE;
    }
    if (!ws.h_hdr && (e = hipHostMalloc(&ws.h_hdr, 8 * sizeof(int), hipHostMallocDefault)) != hipSuccess) return e;
    if (!ws.bfs_ev && (e = hipEventCreateWithFlags(&ws.bfs_ev, hipEventDisableTiming)) != hipSuccess) return e;
    if (trees > 1) {
        if (!ws.side_ev && (e = hipEventCreateWithFlags(&ws.side_ev, hipEventDisableTiming)) != hipSuccess) return e;
        if (!ws.side && (e = hipStreamCreateWithFlags(&ws.side, hipStreamNonBlocking)) != hipSuccess) return e;
    }
    return hipSuccess;
}

// After the enqueue_tree calls: an event behind the device BFS's header copies (work enqueued after it,
// e.g. the cost volume, runs while read_trees waits)
hipError_t mark_trees(StWorkspace& ws, hipStream_t s) { return hipEventRecord(ws.bfs_ev, s); }

// The device BFS's headers of tree slots [0, n) once mark_trees' event has passed (host BFS: known already)
hipError_t read_trees(StWorkspace& ws, bool hbfs, TreeJob* j, int n, int64_t P) {
    if (hbfs) return hipSuccess;
    const hipError_t e = hipEventSynchronize(ws.bfs_ev);
    if (e != hipSuccess) return e;
    for (int k = 0; k < n; ++k) {
        const int* h = ws.h_hdr + 4 * k;
        if (h[0] < 1 || h[0] > P || h[1] < 1 || h[1] > P || h[2] < 1 || h[3] != h[2] - 1) return hipErrorUnknown;
        j[k].d.nlev = h[0];
        j[k].maxw = h[1];
        j[k].n_up = h[2];
        j[k].n_dn = h[3];
    }
    return hipSuccess;
}

WaveJob wave_job(float* C, float* F, const TreeJob& t) {
    return WaveJob{C, F, t.d.parent, t.d.pdist, t.d.first, t.d.child, t.task, t.n_up, t.n_dn, t.d.table};
}

float ms_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
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
    (void)hipFree(task);
    task = nullptr;
    (void)hipFree(node);
    node = nullptr;
    node_n = 0;
    (void)hipFree(sortbuf);
    sortbuf = nullptr;
    sortbuf_n = 0;
    for (int k = 0; k < 2; ++k) {
        (void)hipFree(bfs[k]);
        bfs[k] = nullptr;
        bfs_n[k] = 0;
    }
    if (side) (void)hipStreamDestroy(side);
    side = nullptr;
    if (side_ev) (void)hipEventDestroy(side_ev);
    side_ev = nullptr;
    if (h_hdr) (void)hipHostFree(h_hdr);
    h_hdr = nullptr;
    if (bfs_ev) (void)hipEventDestroy(bfs_ev);
    bfs_ev = nullptr;
    last_P = last_nlev = 0;
    for (int k = 0; k < 2; ++k) {
        if (h_edges[k]) (void)hipHostFree(h_edges[k]);
        h_edges[k] = nullptr;
        h_edges_n[k] = 0;
        if (h_tree[k]) (void)hipHostFree(h_tree[k]);
        h_tree[k] = nullptr;
        h_tree_n[k] = 0;
        if (h_marks[k]) (void)hipHostFree(h_marks[k]);
        h_marks[k] = nullptr;
        h_marks_n[k] = 0;
        (void)hipFree(dedge[k]);
        dedge[k] = nullptr;
        dedge_n[k] = 0;
        (void)hipFree(sidx[k]);
        sidx[k] = nullptr;
        sidx_n[k] = 0;
        delete static_cast<st_host::HostTree*>(host_tree[k]);
        host_tree[k] = nullptr;
        for (auto& ev : edge_ev[k]) {
            if (ev) (void)hipEventDestroy(ev);
            ev = nullptr;
        }
    }
    w8 = nullptr;
    grad = nullptr;
    vol = nullptr;
    tree_i = nullptr;
    tree_b = nullptr;
    table = nullptr;
    w8_n = grad_n = vol_n = tree_i_n = tree_b_n = table_n = task_n = 0;
}

#define ST_CHK(x)                          \
    do {                                   \
        const hipError_t e_ = (x);         \
        if (e_ != hipSuccess) return e_;   \
    } while (0)

hipError_t segment_tree_match(StWorkspace& ws, const uint8_t* dL, const uint8_t* dR, int W, int H, int pitch, int D,
                              int scale, float sigma, float tau, uint8_t* d_out, hipStream_t s, StStats* st) {
    if (W < 2 || H < 1 || D < 1 || D > kMaxDisp || scale < 0) return hipErrorInvalidValue;
    const int64_t P = (int64_t)W * H;
    if (P > (1 << 28)) return hipErrorInvalidValue;
    ST_CHK(grow(ws.w8, ws.w8_n, (size_t)P * 3));
    ST_CHK(grow(ws.grad, ws.grad_n, (size_t)P * 2));
    ST_CHK(grow(ws.vol, ws.vol_n, (size_t)P * D * 2));
    ST_CHK(grow(ws.tree_i, ws.tree_i_n, (size_t)P * 5 + 2));
    ST_CHK(grow(ws.tree_b, ws.tree_b_n, (size_t)P));
    ST_CHK(grow(ws.table, ws.table_n, (size_t)256));
    ST_CHK(grow(ws.node, ws.node_n, (size_t)P));
    const dim3 rows((unsigned)((W + kST - 1) / kST), (unsigned)H);
    // guide weights -> host
    uint8_t* wr = ws.w8;
    uint8_t* wu = ws.w8 + P;
    hipLaunchKernelGGL(st_weights_kernel, rows, dim3(kST), 0, s, dL, W, H, pitch, wr, wu);
    ST_CHK(hipGetLastError());
    // the edges in the reference's order, sorted on the GPU, -> host
    int nE = 0;
    ST_CHK(gpu_sorted_edges(ws, wr, wu, nullptr, nullptr, 0.f, W, H, false, 0, s, nE));
    // gradients of both views meanwhile (same stream, after the download in order)
    hipLaunchKernelGGL(st_gradient_kernel, rows, dim3(kST), 0, s, dL, W, H, pitch, ws.grad);
    hipLaunchKernelGGL(st_gradient_kernel, rows, dim3(kST), 0, s, dR, W, H, pitch, ws.grad + P);
    ST_CHK(hipGetLastError());
    // segment_graph's passes on the host, starting on the first edge chunk (no stream sync: the gradients
    // run meanwhile), into page-locked lists; the BFS on the device
    const auto t0 = std::chrono::steady_clock::now();
    const bool hbfs = host_bfs_requested();
    ST_CHK(tree_resources(ws, P, nE, 1));
    HostTree* tp = nullptr;
    ST_CHK(host_tree_slot(ws, P, 0, tp, hbfs));
    HostTree& t = *tp;
    AdjRec* adj = list_storage(t, hbfs, P);
    if (!host_tree_part(ws, 0, t, adj, hbfs, nE, P, W, tau, 1.0f)) {
        (void)hipStreamSynchronize(s);   // no copy into the page-locked buffers may outlive the call
        return hipErrorInvalidValue;
    }
    float table[256];
    weight_table(sigma, table);
    std::vector<int4> tv;
    TreeJob tj{};
    ST_CHK(enqueue_tree(ws, t, hbfs, P, W, nE, 1.0f, table, 0, s, tv, tj));
    ST_CHK(mark_trees(ws, s));
    const DevTree& dt = tj.d;
    float* C = ws.vol;
    float* F = ws.vol + (size_t)P * D;
    ST_CHK(launch_node(dt, ws.node, (int)P, s));
    ST_CHK(launch_cost<false>(dL, dR, W, H, pitch, ws.grad, ws.node, D, C, s));
    ST_CHK(read_trees(ws, hbfs, &tj, 1, P));
    const float tree_ms = ms_since(t0);
    FilterJobs jobs{};
    jobs.j[0] = filter_job(C, F, tj.d);
    WaveJobs wj{};
    wj.j[0] = wave_job(C, F, tj);
    ST_CHK(launch_filter(jobs, wj, 1, tj.maxw, D, (int)P, s));
    uint8_t* raw = ws.w8;   // the weights are consumed: reuse for the unfiltered map
    ST_CHK(launch_wta(F, ws.node, (int)P, D, scale, raw, s));
    ST_CHK(launch_median(raw, W, H, W, P, 1, 3, d_out, W, P, s));   // MeanFilter(disparity, disparity, 3)
    if (st) {
        st->levels = tj.d.nlev;
        st->tree_ms = tree_ms;
    }
    ws.last_P = (int)P;
    ws.last_nlev = tj.d.nlev;
    // keep the host tree alive until its uploads have been consumed
    return hipStreamSynchronize(s);
}

hipError_t segment_tree_refined_match(StWorkspace& ws, const uint8_t* dL, const uint8_t* dR, int W, int H, int pitch,
                                      int D, int scale, float sigma, float tau, uint8_t* d_out, hipStream_t s,
                                      StStats* st) {
    if (W < 2 || H < 1 || D < 1 || D > kMaxDisp || scale < 0) return hipErrorInvalidValue;
    const int64_t P = (int64_t)W * H;
    if (P > (1 << 28)) return hipErrorInvalidValue;
    constexpr float kSigmaOne = 0.08f;   // SIGMA_ONE, Toolkit.h:35
    ST_CHK(grow(ws.w8, ws.w8_n, (size_t)P * 10));
    ST_CHK(grow(ws.grad, ws.grad_n, (size_t)P * 2));
    ST_CHK(grow(ws.vol, ws.vol_n, (size_t)P * D * 4));
    ST_CHK(grow(ws.tree_i, ws.tree_i_n, ((size_t)P * 5 + 2) * 2));
    ST_CHK(grow(ws.tree_b, ws.tree_b_n, (size_t)P * 2));
    ST_CHK(grow(ws.table, ws.table_n, (size_t)512));
    ST_CHK(grow(ws.node, ws.node_n, (size_t)P * 2));
    const dim3 rows((unsigned)((W + kST - 1) / kST), (unsigned)H);
    uint8_t* wrL = ws.w8;
    uint8_t* wrR = ws.w8 + 2 * P;
    uint8_t* raw0 = ws.w8 + 4 * P;
    uint8_t* raw1 = ws.w8 + 5 * P;
    uint8_t* mapL = ws.w8 + 6 * P;   // first-pass maps after the 7x7 median
    uint8_t* mapR = ws.w8 + 7 * P;
    uint8_t* chk = ws.w8 + 8 * P;
    uint8_t* mask = ws.w8 + 9 * P;
    // colour weights of both views (wr, wu planes each) -> host; gradients
    hipLaunchKernelGGL(st_weights_kernel, rows, dim3(kST), 0, s, dL, W, H, pitch, wrL, wrL + P);
    hipLaunchKernelGGL(st_weights_kernel, rows, dim3(kST), 0, s, dR, W, H, pitch, wrR, wrR + P);
    ST_CHK(hipGetLastError());
    // both views' edges in the reference's order, sorted on the GPU, -> host
    int nE = 0;
    ST_CHK(gpu_sorted_edges(ws, wrL, wrL + P, nullptr, nullptr, 0.f, W, H, false, 0, s, nE));
    ST_CHK(gpu_sorted_edges(ws, wrR, wrR + P, nullptr, nullptr, 0.f, W, H, false, 1, s, nE));
    hipLaunchKernelGGL(st_gradient_kernel, rows, dim3(kST), 0, s, dL, W, H, pitch, ws.grad);
    hipLaunchKernelGGL(st_gradient_kernel, rows, dim3(kST), 0, s, dR, W, H, pitch, ws.grad + P);
    ST_CHK(hipGetLastError());
    // first run: colour trees of the left and the right view, segment_graph's passes side by side
    // (StereoDisparity.cpp:112-123) into page-locked lists 0 and 1, each starting on the first chunk of its
    // edges; each build enqueues its BFS as soon as its lists are done, the left on s, the right on the
    // side stream (the two BFSs are chains of small latency-bound kernels: side by side they overlap)
    auto t0 = std::chrono::steady_clock::now();
    const bool hbfs = host_bfs_requested();
    ST_CHK(tree_resources(ws, P, nE, 2));
    HostTree *tlp = nullptr, *trp = nullptr;
    ST_CHK(host_tree_slot(ws, P, 0, tlp, hbfs));
    ST_CHK(host_tree_slot(ws, P, 1, trp, hbfs));
    HostTree &tl = *tlp, &tr = *trp;
    AdjRec* adjL = list_storage(tl, hbfs, P);
    AdjRec* adjR = list_storage(tr, hbfs, P);
    float tab1[256];
    weight_table(kSigmaOne, tab1);
    std::vector<int4> tv[2];
    TreeJob tj[2] = {};
    hipStream_t bs[2] = {s, ws.side};
    // neither build may leave its exception behind the other's thread (a joinable std::thread must not
    // be destroyed): a failed build reports false, a failed enqueue its error
    auto build = [&](int slot, HostTree& t, AdjRec* adj, hipError_t& err) {
        try {
            if (!host_tree_part(ws, slot, t, adj, hbfs, nE, P, W, tau, 1.0f)) return false;
            if (!hbfs) {
                err = enqueue_tree(ws, t, false, P, W, nE, 1.0f, tab1, slot, bs[slot], tv[slot], tj[slot]);
                if (err == hipSuccess && slot == 1) err = hipEventRecord(ws.side_ev, ws.side);
            }
            return true;
        } catch (...) {
            return false;
        }
    };
    bool okR = false;
    hipError_t errL = hipSuccess, errR = hipSuccess;
    int dev = 0;
    ST_CHK(hipGetDevice(&dev));
    std::thread th([&] {
        errR = hipSetDevice(dev);   // the current device is per thread (the scratch allocation, the launches)
        if (errR == hipSuccess) okR = build(1, tr, adjR, errR);
    });
    const bool okL = build(0, tl, adjL, errL);
    th.join();
    if (!okL || !okR || errL != hipSuccess || errR != hipSuccess) {
        // no copy into the page-locked buffers may outlive the call
        (void)hipStreamSynchronize(ws.side);
        (void)hipStreamSynchronize(s);
        return errL != hipSuccess ? errL : errR != hipSuccess ? errR : hipErrorInvalidValue;
    }
    if (hbfs) {
        ST_CHK(enqueue_tree(ws, tl, true, P, W, nE, 1.0f, tab1, 0, s, tv[0], tj[0]));
        ST_CHK(enqueue_tree(ws, tr, true, P, W, nE, 1.0f, tab1, 1, s, tv[1], tj[1]));
    } else {
        ST_CHK(hipStreamWaitEvent(s, ws.side_ev, 0));
    }
    ST_CHK(mark_trees(ws, s));
    const DevTree &d0 = tj[0].d, &d1 = tj[1].d;
    float* C0 = ws.vol;
    float* F0 = ws.vol + (size_t)P * D;
    float* C1 = ws.vol + (size_t)P * D * 2;
    float* F1 = ws.vol + (size_t)P * D * 3;
    ST_CHK(launch_node(d0, ws.node, (int)P, s));
    ST_CHK(launch_node(d1, ws.node + P, (int)P, s));
    ST_CHK(launch_cost<false>(dL, dR, W, H, pitch, ws.grad, ws.node, D, C0, s));
    ST_CHK(launch_cost<true>(dL, dR, W, H, pitch, ws.grad, ws.node + P, D, C1, s));
    ST_CHK(read_trees(ws, hbfs, tj, 2, P));
    float tree_ms = ms_since(t0);
    FilterJobs jobs{};
    jobs.j[0] = filter_job(C0, F0, d0);
    jobs.j[1] = filter_job(C1, F1, d1);
    WaveJobs wj{};
    wj.j[0] = wave_job(C0, F0, tj[0]);
    wj.j[1] = wave_job(C1, F1, tj[1]);
    ST_CHK(launch_filter(jobs, wj, 2, std::max(tj[0].maxw, tj[1].maxw), D, (int)P, s));
    ST_CHK(launch_wta(F0, ws.node, (int)P, D, 1, raw0, s));
    ST_CHK(launch_wta(F1, ws.node + P, (int)P, D, 1, raw1, s));
    ST_CHK(launch_median(raw0, W, H, W, P, 1, 3, mapL, W, P, s));   // MeanFilter(disparityLeft, ..., 3)
    ST_CHK(launch_median(raw1, W, H, W, P, 1, 3, mapR, W, P, s));
    // left-right check (StereoDisparity.cpp:129-147): mask = !occluded
    ST_CHK(launch_lr_check(mapL, W, P, mapR, W, P, 0, W, H, 1, chk, W, P, nullptr, mask, W, P, s));
    // re-segmentation: colour + depth tree on the left view (StereoDisparity.cpp:150-152), its weights
    // from the first left map and mask, sorted on the GPU
    ST_CHK(gpu_sorted_edges(ws, wrL, wrL + P, mapL, mask, (float)D, W, H, true, 0, s, nE));
    // the first run's uploads from page-locked slot 0 were enqueued before this download: once its first
    // chunk has landed, slot 0 is free for the depth tree
    if (!wait_edges(ws, 0, 1)) {
        (void)hipStreamSynchronize(s);
        return hipErrorUnknown;
    }
    t0 = std::chrono::steady_clock::now();
    HostTree* tdp = nullptr;   // slot 0's tree object again
    ST_CHK(host_tree_slot(ws, P, 0, tdp, hbfs));
    HostTree& td = *tdp;
    AdjRec* adjD = list_storage(td, hbfs, P);
    if (!host_tree_part(ws, 0, td, adjD, hbfs, nE, P, W, tau, 255.0f)) {
        (void)hipStreamSynchronize(s);   // no copy into the page-locked buffers may outlive the call
        return hipErrorInvalidValue;
    }
    float tab2[256];
    weight_table(sigma, tab2);
    std::vector<int4> tv2;
    TreeJob t2{};
    ST_CHK(enqueue_tree(ws, td, hbfs, P, W, nE, 255.0f, tab2, 0, s, tv2, t2));
    ST_CHK(mark_trees(ws, s));
    // second run on the same cost (the reference recomputes it, :150)
    ST_CHK(launch_node(t2.d, ws.node, (int)P, s));
    ST_CHK(launch_cost<false>(dL, dR, W, H, pitch, ws.grad, ws.node, D, C0, s));
    ST_CHK(read_trees(ws, hbfs, &t2, 1, P));
    tree_ms += ms_since(t0);
    FilterJobs job2{};
    job2.j[0] = filter_job(C0, F0, t2.d);
    WaveJobs wj2{};
    wj2.j[0] = wave_job(C0, F0, t2);
    ST_CHK(launch_filter(job2, wj2, 1, t2.maxw, D, (int)P, s));
    ST_CHK(launch_wta(F0, ws.node, (int)P, D, scale, raw0, s));
    ST_CHK(launch_median(raw0, W, H, W, P, 1, 3, d_out, W, P, s));
    if (st) {
        st->levels = t2.d.nlev;
        st->tree_ms = tree_ms;
    }
    ws.last_P = (int)P;
    ws.last_nlev = t2.d.nlev;
    return hipStreamSynchronize(s);
}

#undef ST_CHK

}  // namespace sm
