// bm_wide.hip — box matching at wide windows (radius 16..127), the reference's unbounded SADWindowSize
// (Device.cu:46-56 / BlockMatching.cpp:168-177).  The fused tile kernel (bm_box.hip) covers r <= 15: its
// 64-column tile keeps TW = 64 - 2r output columns, which vanishes as r grows.  Here the window sum is
// separable through HBM, so a (pixel, d) costs the same at any radius:
//   wide_vsum_kernel : V_d(y, c) = sum of AD_d over rows y-r..y+r (clipped), AD_d(y, c) = |L(y,c) - R(y,c-d)|
//                      for c >= d else 0 (Device.cu:27-31); one lane per 4 columns walks a chunk of rows with
//                      packed-u16 running sums (V <= 255 * 255 = 65025), 8 rows' dword loads in flight at a
//                      time (buffer loads, row offset in the SGPR soffset), one d per block row; u16 planes
//                      written nontemporally, 8 B per lane per row.
//   wide_hwta_kernel : one 256-lane block per image row: per d the row of V (prefetched one d ahead) is
//                      prefix-summed across the block (local prefix + DPP wave scan + 4-wave offsets) into LDS,
//                      each output's window sum is two prefix reads, and the key (S << 8 | d) is min-folded in
//                      registers with the validity d <= W - x (Device.cu:44) and the 50 win^2 seed (:37).  The
//                      right view's candidate for u = x - d (C_R(u, d) = C_L(u + d, d), StereoHelper.cpp:
//                      156-180) is folded into an LDS row by atomic min, so LR needs no second pass.
// Frames go through in groups of up to 8 per vsum / hwta pair (wide_group: ~32 row blocks per CU, at most
// 4.5 GB of V planes), the group's planes in the handle's workspace.  HBM per (pixel, d): 2 B written + 2 B read (the V planes); L and R
// come from L2.
// Exact integer arithmetic throughout: S <= 255 * 255^2 < 2^24, prefix sums < 4096 * 65025 < 2^32.
#include <algorithm>
#include <type_traits>

#include "bm_common.h"

namespace sm {
namespace {

using u16x2 = unsigned short __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

// |L - R| of 4 bytes as two packed-u16 pairs: even bytes (columns 0, 2) and odd bytes (1, 3)
__device__ __forceinline__ void ad4(uint32_t l, uint32_t r, u16x2& e, u16x2& o) {
    const u16x2 le = as_u16x2(__builtin_amdgcn_perm(0u, l, 0x0c020c00u)), lo = as_u16x2(__builtin_amdgcn_perm(0u, l, 0x0c030c01u));
    const u16x2 re = as_u16x2(__builtin_amdgcn_perm(0u, r, 0x0c020c00u)), ro = as_u16x2(__builtin_amdgcn_perm(0u, r, 0x0c030c01u));
    e = __builtin_elementwise_max(le, re) - __builtin_elementwise_min(le, re);
    o = __builtin_elementwise_max(lo, ro) - __builtin_elementwise_min(lo, ro);
}

// Inclusive prefix sum over the 64 lanes with DPP moves (no LDS round trip): row_shr 1/2/4/8 scans each
// 16-lane row, row_bcast:15 and :31 carry the rows' totals (disabled lanes read 0 through `old`).
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);   // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);   // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return v;
}

constexpr int kVT = 64;   // one wave per block: 256 columns

// Columns c4..c4+3 of one d plane, rows [y0, y1).  L and R are read as one (possibly unaligned) dword per row
// at a column clamped into [0, W - 4] and shifted back to c4 (resp. c4 - d) by a per-lane byte shift; the
// keep-masks then zero the columns < d (Device.cu:27-31 + the memset) and >= W, whatever bytes the clamp read.
// No lane takes a byte-load path (a wave straddling c = d costs what any other wave costs).
__device__ __forceinline__ void vsum_walk(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R, int W, int H,
                                          int pitch, int radius, int d, int c4, int y0, int y1,
                                          uint16_t* __restrict__ Vd) {
    // the columns kept, in output order (columns c4, c4 + 1 | c4 + 2, c4 + 3): the running sums of a
    // column < d or >= W carry garbage (wrapping u16 arithmetic) and are zeroed at the store
    uint32_t keep01 = 0, keep23 = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t m = (c4 + j >= d && c4 + j < W) ? 0xFFFFu << (16 * (j & 1)) : 0u;
        if (j < 2) keep01 |= m; else keep23 |= m;
    }
    const int xl = min(c4, W - 4), xr = min(max(c4 - d, 0), W - 4);
    const uint32_t shl = 8u * (uint32_t)(c4 - xl);                         // 0..3 bytes right
    const int dr = c4 - d - xr;                                           // > 0: right edge, < 0: left of R's column 0
    const uint32_t shr_r = 8u * (uint32_t)max(dr, 0), shl_r = 8u * (uint32_t)min(max(-dr, 0), 3);
    // buffer loads: the row offset is wave-uniform (SGPR soffset), the column a 32-bit lane offset, so a
    // load needs no per-lane 64-bit address math (global loads spent a v_mad_i64_i32 per load); the frame
    // bounds check of the descriptor returns 0 past the last row (never reached: rows are clamped)
    const int nrec = pitch * H;
    const __amdgpu_buffer_rsrc_t rsl = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(L), 0, nrec, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(R), 0, nrec, 0x00020000);
    auto row4 = [&](int y, uint32_t& l, uint32_t& r) {
        const int ro = y * pitch;
        l = __builtin_amdgcn_raw_buffer_load_b32(rsl, xl, ro, 0);
        r = __builtin_amdgcn_raw_buffer_load_b32(rsr, xr, ro, 0);
        l >>= shl;
        r = (r >> shr_r) << shl_r;
    };
    u16x2 se = {0, 0}, so = {0, 0};
    const int ps = max(y0 - radius, 0), pe = min(y0 + radius, H - 1);   // the window of row y0
    for (int y = ps; y <= pe; y += 8) {
        uint32_t l8[8], r8[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) row4(min(y + k, pe), l8[k], r8[k]);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            u16x2 e, o;
            ad4(l8[k], r8[k], e, o);
            const u16x2 z = {0, 0};
            se += y + k <= pe ? e : z;
            so += y + k <= pe ? o : z;
        }
    }
    // 8-B vector store only where the row start keeps it 8-B aligned (W % 4 == 0), else per column
    const bool full = c4 + 4 <= W && (W & 3) == 0;
    constexpr int kU = 8;   // 4 and 16 measured the same (profiles/microbench/r05_wide_path.txt)
    // one batch of kU rows: the kU entering and kU leaving rows, clamped into the frame, loaded together
    // (4 kU loads in flight), then the sums; EDGE batches (a row entering past H or leaving above 0,
    // wave-uniform) mask those rows' AD
    auto batch = [&](int y, auto edge) {
        constexpr bool EDGE = decltype(edge)::value;
        uint32_t la[kU], ra[kU], lb[kU], rb[kU];
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            row4(EDGE ? min(y + k + radius + 1, H - 1) : y + k + radius + 1, la[k], ra[k]);
            row4(EDGE ? max(y + k - radius, 0) : y + k - radius, lb[k], rb[k]);
        }
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            if (!EDGE || y + k < y1) {
                // output columns c4..c4+3 = se.x, so.x, se.y, so.y
                const uint32_t v01 = __builtin_amdgcn_perm(as_u32(so), as_u32(se), 0x05040100u) & keep01;
                const uint32_t v23 = __builtin_amdgcn_perm(as_u32(so), as_u32(se), 0x07060302u) & keep23;
                uint16_t* dst = Vd + (int64_t)(y + k) * W + c4;
                if (full) {
                    // nontemporal: the planes are streamed once each way (plain stores and loads measured
                    // 8-13 % slower over both kernels)
                    const u32x2 v = {v01, v23};
                    __builtin_nontemporal_store(v, reinterpret_cast<u32x2*>(dst));
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (c4 + j < W) dst[j] = (uint16_t)((j < 2 ? v01 : v23) >> (16 * (j & 1)));
                }
            }
            u16x2 ei, oi, eo, oo;
            ad4(la[k], ra[k], ei, oi);
            ad4(lb[k], rb[k], eo, oo);
            if (EDGE) {
                const uint32_t mi = y + k + radius + 1 < H ? 0xFFFFFFFFu : 0u;
                const uint32_t mo = y + k - radius >= 0 ? 0xFFFFFFFFu : 0u;
                ei = as_u16x2(as_u32(ei) & mi);
                oi = as_u16x2(as_u32(oi) & mi);
                eo = as_u16x2(as_u32(eo) & mo);
                oo = as_u16x2(as_u32(oo) & mo);
            }
            se = se + ei - eo;
            so = so + oi - oo;
        }
    };
    for (int y = y0; y < y1; y += kU) {
        if (y - radius >= 0 && y + kU + radius < H && y + kU <= y1)
            batch(y, std::false_type{});
        else
            batch(y, std::true_type{});
    }
}

// grid (ceil(W / 256), d_hi - d_lo, row chunks x frames of the group), one wave per block; V <= 255 * 255 so
// the packed u16 running sums are exact (wrap-around in the intermediate add/sub cancels).
__global__ __launch_bounds__(kVT) void wide_vsum_kernel(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R,
                                                        int64_t fstride, int W, int H, int pitch, int radius, int d_lo,
                                                        int d_hi, int chunk, int nch, uint16_t* __restrict__ V) {
    const int c4 = (blockIdx.x * kVT + threadIdx.x) * 4;
    const int d = d_lo + blockIdx.y;
    const int g = blockIdx.z / nch;
    const int y0 = (blockIdx.z - g * nch) * chunk, y1 = min(y0 + chunk, H);
    if (c4 >= W || d >= d_hi || y0 >= H) return;
    L += g * fstride;
    R += g * fstride;
    uint16_t* Vd = V + ((int64_t)g * (d_hi - d_lo) + (d - d_lo)) * H * W;
    vsum_walk(L, R, W, H, pitch, radius, d, c4, y0, y1, Vd);
}

struct WideOut {
    uint8_t* disp;    // left map (or null), out_pitch / out_frame_stride
    int opitch;
    int64_t ofs;
    uint32_t* keys;   // raw keys [frame][H][W] (or null)
    uint8_t* right;   // right view (or null)
    int rpitch;
    int64_t rfs;
    uint32_t* rkeys;  // d-slice right keys [frame][H][W], sign bit flipped (or null)
};

// One block per image row, grid (H, frames of the group).
// NPT outputs per thread (W <= 256 * NPT), contiguous: x in [8t, 8t + 8) for NPT 8.  The prefix row lives in LDS
// with one pad dword after every 8 (index i -> i + i / 8), so the 64 lanes' segment stores and their window
// reads (lanes 9 dwords apart) fall on distinct banks.  Dynamic LDS: pref[2][NPAD] u32 (double-buffered over
// d: two barriers per d), then rmin[NPAD] u32 (same padding) when the right view is requested.  (Two d per
// barrier pair, DP = 2, measured 7-20 % slower: profiles/microbench/r05_wide_path.txt.)
template <int NPT, int NT>
__global__ __launch_bounds__(NT) void wide_hwta_kernel(const uint16_t* __restrict__ V, int W, int H, int radius,
                                                        int d_lo, int d_hi, uint32_t seed, uint32_t thresh,
                                                        WideOut out) {
    extern __shared__ __attribute__((aligned(16))) uint32_t wl[];
    constexpr int NX = NT * NPT + 1;                  // prefix entries 0..NT NPT
    constexpr int NPAD = NX + NX / 8 + 1;
    __shared__ uint32_t wsum[2][NT / 64];
    uint32_t* rmin = wl + 2 * NPAD;
    auto pad = [](int i) { return i + (i >> 3); };
    const int y = blockIdx.x, g = blockIdx.y;
    V += (int64_t)g * (d_hi - d_lo) * H * W;
    uint8_t* __restrict__ disp = out.disp ? out.disp + g * out.ofs : nullptr;
    uint32_t* __restrict__ keys = out.keys ? out.keys + (int64_t)g * W * H : nullptr;
    uint8_t* __restrict__ right = out.right ? out.right + g * out.rfs : nullptr;
    uint32_t* __restrict__ rkeys = out.rkeys ? out.rkeys + (int64_t)g * W * H : nullptr;
    const int opitch = out.opitch, rpitch = out.rpitch;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int x0 = t * NPT;
    const bool want_right = right != nullptr || rkeys != nullptr;
    if (want_right)
        for (int i = t; i < NPAD; i += NT) rmin[i] = 0xFFFFFFFFu;   // indexed pad(u), as pref
    uint32_t best[NPT];
    int lo[NPT], hi[NPT];
    bool xin[NPT];
    const int p0 = pad(x0);
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        best[k] = seed;
        const int x = x0 + k;
        xin[k] = x < W;
        lo[k] = pad(max(x - radius, 0));              // window columns [lo, hi) of the prefix (Device.cu:51)
        hi[k] = pad(min(x + radius, W - 1) + 1);
    }
    // a row of V as NPT / 2 packed u16 pairs: 16-B loads (8-B at NPT 4) when W is a multiple of the chunk
    constexpr int CH = NPT < 8 ? NPT : 8;
    const bool vec = (W % CH) == 0;
    auto load_row = [&](int d, uint32_t* raw) {
        const uint16_t* row = V + ((int64_t)(d - d_lo) * H + y) * W;
        if (vec) {
#pragma unroll
            for (int k = 0; k < NPT; k += CH) {
                if constexpr (CH == 8) {
                    u32x4 q = {0u, 0u, 0u, 0u};
                    if (x0 + k < W) q = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(row + x0 + k));
                    raw[k / 2] = q.x; raw[k / 2 + 1] = q.y; raw[k / 2 + 2] = q.z; raw[k / 2 + 3] = q.w;
                } else {
                    uint2 q = make_uint2(0, 0);
                    if (x0 + k < W) q = *reinterpret_cast<const uint2*>(row + x0 + k);
                    raw[k / 2] = q.x; raw[k / 2 + 1] = q.y;
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < NPT; k += 2) {
                const uint32_t v0 = x0 + k < W ? (uint32_t)row[x0 + k] : 0u;
                const uint32_t v1 = x0 + k + 1 < W ? (uint32_t)row[x0 + k + 1] : 0u;
                raw[k / 2] = v0 | v1 << 16;
            }
        }
    };
    // the next d's row is loaded while this d's is scanned and folded: its HBM latency off the d loop's path
    // (two d ahead measured the same: profiles/microbench/r05_wide_path.txt)
    uint32_t nxt[NPT / 2];
    load_row(d_lo, nxt);
    for (int d = d_lo; d < d_hi; ++d) {
        const int b = (d - d_lo) & 1;
        uint32_t* pref = wl + b * NPAD;
        uint32_t raw[NPT / 2];
#pragma unroll
        for (int k = 0; k < NPT / 2; ++k) raw[k] = nxt[k];
        if (d + 1 < d_hi) load_row(d + 1, nxt);
        uint32_t p[NPT];
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < NPT / 2; ++k) {
            acc += raw[k] & 0xFFFFu;
            p[2 * k] = acc;
            acc += raw[k] >> 16;
            p[2 * k + 1] = acc;
        }
        // inclusive scan of the per-thread totals across the wave, then the waves' offsets
        const uint32_t inc = wave_inclusive_scan(acc);
        if (lane == 63) wsum[b][wv] = inc;
        __syncthreads();
        uint32_t base = inc - acc;
#pragma unroll
        for (int w = 0; w < NT / 64; ++w) base += w < wv ? wsum[b][w] : 0u;
        if (t == 0) pref[0] = 0u;
#pragma unroll
        for (int k = 0; k < NPT; ++k) pref[pad(x0 + k + 1)] = base + p[k];
        __syncthreads();
        const uint32_t dd = (uint32_t)(d & 0xFF);
        // branch-free: columns x >= W fold garbage into best (never stored); the right view's fold is an LDS
        // atomic min (no read-back), neutral 0xFFFFFFFF on the lane's own slot when x < d or x >= W
        uint32_t key[NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) key[k] = ((pref[hi[k]] - pref[lo[k]]) << 8) | dd;
        if (x0 + NPT - 1 <= W - d) {   // every column of the thread valid at d (all but one wave)
#pragma unroll
            for (int k = 0; k < NPT; ++k) best[k] = min(best[k], key[k]);
        } else {
#pragma unroll
            for (int k = 0; k < NPT; ++k) best[k] = d <= W - x0 - k ? min(best[k], key[k]) : best[k];   // Device.cu:44
        }
        if (want_right) {
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                const bool ok = x0 + k >= d && xin[k];
                if constexpr (NPT % 8 == 0) {
                    // x0 a multiple of 8: pad(x - d) = pad(x0) + (k - d) + ((k - d) >> 3), one lane constant
                    // plus a wave-uniform part
                    const int off = ok ? (k - d) + ((k - d) >> 3) : k + (k >> 3);
                    atomicMin(&rmin[p0 + off], ok ? key[k] : 0xFFFFFFFFu);
                } else {
                    atomicMin(&rmin[pad(ok ? x0 + k - d : x0 + k)], ok ? key[k] : 0xFFFFFFFFu);
                }
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const int x = x0 + k;
        if (x < W) {
            if (disp) disp[(int64_t)y * opitch + x] = best[k] < thresh ? (uint8_t)(best[k] & 0xFFu) : (uint8_t)0;
            if (keys) keys[(int64_t)y * W + x] = best[k];
            if (right) right[(int64_t)y * rpitch + x] = (uint8_t)(rmin[pad(x)] & 0xFFu);   // no threshold
            // slice keys: (cost << 8 | d) of the slice's best d for u = x (0xFFFFFFFF where no d of the slice has
            // x + d < W), sign bit flipped
            if (rkeys) rkeys[(int64_t)y * W + x] = rmin[pad(x)] ^ kRightKeyFlip;
        }
    }
}

template <int NPT, int NT>
hipError_t launch_h(const uint16_t* V, int W, int H, int radius, int d_lo, int d_hi, uint32_t seed, uint32_t thresh,
                    const WideOut& out, int frames, hipStream_t s) {
    constexpr int NX = NT * NPT + 1;
    const size_t lds = (size_t)((out.right || out.rkeys ? 3 : 2) * (NX + NX / 8 + 1)) * 4;
    hipLaunchKernelGGL((wide_hwta_kernel<NPT, NT>), dim3((unsigned)H, (unsigned)frames), dim3(NT), lds, s, V, W, H,
                       radius, d_lo, d_hi, seed, thresh, out);
    return hipGetLastError();
}

// 256 threads per row block, NPT = span / 256 outputs each (512- and 1024-thread blocks measured 20 % / 65 %
// slower, 128-thread blocks 13 %: profiles/microbench/r05_wide_path.txt)
template <int SPAN>
hipError_t launch_span(const uint16_t* V, int W, int H, int radius, int d_lo, int d_hi, uint32_t seed, uint32_t thresh,
                       const WideOut& out, int frames, hipStream_t s) {
    constexpr int NPT = SPAN / 256;
    return launch_h<NPT, 256>(V, W, H, radius, d_lo, d_hi, seed, thresh, out, frames, s);
}

// frames per vsum / hwta launch pair: enough row blocks for ~32 per CU (1080 rows of one 1080p frame give 4),
// at most 8 frames and 4.5 GB of V planes (1080p D=128: 8 frames, 4.2 GB).  Same box, 1080p D=128, 8 frames per
// call (profiles/microbench/r05_wide_path.txt): 2 / 4 / 8 frames per pair 0.280 / 0.268 / 0.265 ms at r = 16,
// 0.280 / 0.251 / 0.239 at r = 127
int wide_group(int W, int H, int D, int batch) {
    const int64_t plane = (int64_t)W * H * D * (int64_t)sizeof(uint16_t);
    const int by_mem = (int)std::max<int64_t>(1, ((int64_t)4608 << 20) / std::max<int64_t>(plane, 1));
    const int want = (8192 + H - 1) / H;
    return std::max(1, std::min({want, batch, 8, by_mem}));
}

}  // namespace

size_t wide_workspace_bytes(int W, int H, int D, int batch) {
    return (size_t)wide_group(W, H, D, batch) * D * W * H * sizeof(uint16_t);
}

hipError_t launch_box_match_wide(const MatchArgs& a, int batch, uint16_t* ws, uint8_t* right, int rpitch,
                                 int64_t rstride, hipStream_t s, uint32_t* rkeys) {
    if (!wide_path(kMaxBoxRadius + 1, a.W, a.H, a.pitch) || a.valid_mode != 0 || a.d_hi <= a.d_lo || batch <= 0)
        return hipErrorInvalidValue;
    const int nd = a.d_hi - a.d_lo;
    const int G = wide_group(a.W, a.H, nd, batch);
    // row chunks: enough waves to fill the chip (~32 per CU), each chunk at least a window tall (its prologue
    // re-reads the 2r + 1 rows above it, from L2)
    const unsigned gx = (unsigned)((a.W + 4 * kVT - 1) / (4 * kVT));
    const int64_t waves = (int64_t)gx * nd * G;
    const int want = (int)std::max<int64_t>(1, (8192 + waves - 1) / waves);
    int chunk = std::max({(a.H + want - 1) / want, 2 * a.radius + 1, 32});
    int nch = (a.H + chunk - 1) / chunk;
    if ((int64_t)nch * G > 65535) {   // grid.z limit (very tall frames): longer chunks
        const int nmax = 65535 / G;
        chunk = (a.H + nmax - 1) / nmax;
        nch = (a.H + chunk - 1) / chunk;
    }
    for (int f = 0; f < batch; f += G) {
        const int n = std::min(G, batch - f);
        hipLaunchKernelGGL(wide_vsum_kernel, dim3(gx, (unsigned)nd, (unsigned)(nch * n)), dim3(kVT), 0, s,
                           a.left + (int64_t)f * a.frame_stride, a.right + (int64_t)f * a.frame_stride, a.frame_stride,
                           a.W, a.H, a.pitch, a.radius, a.d_lo, a.d_hi, chunk, nch, ws);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        WideOut out;
        out.disp = a.disp ? a.disp + (int64_t)f * a.out_frame_stride : nullptr;
        out.opitch = a.out_pitch;
        out.ofs = a.out_frame_stride;
        out.keys = a.keys ? a.keys + (int64_t)f * a.W * a.H : nullptr;
        out.right = right ? right + (int64_t)f * rstride : nullptr;
        out.rpitch = rpitch;
        out.rfs = rstride;
        out.rkeys = rkeys ? rkeys + (int64_t)f * a.W * a.H : nullptr;
        if (a.W <= 1024)
            e = launch_span<1024>(ws, a.W, a.H, a.radius, a.d_lo, a.d_hi, a.seed_key, a.thresh_key, out, n, s);
        else if (a.W <= 2048)
            e = launch_span<2048>(ws, a.W, a.H, a.radius, a.d_lo, a.d_hi, a.seed_key, a.thresh_key, out, n, s);
        else
            e = launch_span<4096>(ws, a.W, a.H, a.radius, a.d_lo, a.d_hi, a.seed_key, a.thresh_key, out, n, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace sm
