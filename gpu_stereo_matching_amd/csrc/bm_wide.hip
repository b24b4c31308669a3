// bm_wide.hip — box matching at wide windows (radius 16..127), the reference's unbounded SADWindowSize
// (Device.cu:46-56 / BlockMatching.cpp:168-177).  The fused tile kernel (bm_box.hip) covers r <= 15: its
// 64-column tile keeps TW = 64 - 2r output columns, which vanishes as r grows.  Here the window sum is
// separable through HBM, so a (pixel, d) costs the same at any radius:
//   wide_vsum_kernel : V_d(y, c) = sum of AD_d over rows y-r..y+r (clipped), AD_d(y, c) = |L(y,c) - R(y,c-d)|
//                      for c >= d else 0 (Device.cu:27-31); one thread per column walks the rows with a
//                      running sum, one d per block column, u16 planes (V <= 255 * 255 = 65025).
//   wide_hwta_kernel : one block per image row: per d the row of V is prefix-summed across the block (local
//                      prefix + wave scan + 4-wave offsets), each output's window sum is two prefix reads,
//                      and the key (S << 8 | d) is min-folded in registers with the validity d <= W - x
//                      (Device.cu:44) and the 50 win^2 seed (:37).  The right view's candidate for u = x - d
//                      (C_R(u, d) = C_L(u + d, d), StereoHelper.cpp:156-180) is min-folded into an LDS row
//                      as well, so LR needs no second pass: the row is complete when the d loop ends.
// Exact integer arithmetic throughout: S <= 255 * 255^2 < 2^24, prefix sums < 4096 * 65025 < 2^32.
#include <algorithm>

#include "bm_common.h"

namespace sm {
namespace {

constexpr int kWT = 256;

__global__ __launch_bounds__(kWT) void wide_vsum_kernel(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R,
                                                        int W, int H, int pitch, int radius, int d_lo, int d_hi,
                                                        uint16_t* __restrict__ V) {
    const int c = blockIdx.x * kWT + threadIdx.x;
    const int d = d_lo + blockIdx.y;
    if (c >= W || d >= d_hi) return;
    uint16_t* Vd = V + (int64_t)(d - d_lo) * H * W + c;
    if (c < d) {   // every AD of this column is 0 (Device.cu:27-31 + the memset)
        for (int y = 0; y < H; ++y) Vd[(int64_t)y * W] = 0;
        return;
    }
    const uint8_t* lc = L + c;
    const uint8_t* rc = R + c - d;
    auto ad = [&](int y) -> uint32_t {
        const int v = (int)lc[(int64_t)y * pitch] - (int)rc[(int64_t)y * pitch];
        return (uint32_t)(v < 0 ? -v : v);
    };
    uint32_t s = 0;
    const int y0e = min(radius, H - 1);
    for (int y = 0; y <= y0e; ++y) s += ad(y);
    // rows in blocks of kU: the kU entering and kU leaving rows of a block are loaded before the running sum
    // consumes them (the loads of one row are independent of s), so their latencies overlap
    constexpr int kU = 8;
    int y = 0;
    for (; y + kU <= H; y += kU) {
        uint32_t ain[kU], aout[kU];
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            const int ya = y + k + radius + 1, yb = y + k - radius;
            ain[k] = ya < H ? ad(ya) : 0u;
            aout[k] = yb >= 0 ? ad(yb) : 0u;
        }
#pragma unroll
        for (int k = 0; k < kU; ++k) {
            Vd[(int64_t)(y + k) * W] = (uint16_t)s;
            s += ain[k];
            s -= aout[k];
        }
    }
    for (; y < H; ++y) {
        Vd[(int64_t)y * W] = (uint16_t)s;
        const int ya = y + radius + 1, yb = y - radius;
        if (ya < H) s += ad(ya);
        if (yb >= 0) s -= ad(yb);
    }
}

// NPT outputs per thread (W <= 256 * NPT), contiguous: x in [8t, 8t + 8) for NPT 8.  The prefix row lives in LDS
// with one pad dword after every 8 (index i -> i + i / 8), so the 64 lanes' segment stores and their window
// reads (lanes 9 dwords apart) fall on distinct banks.  Dynamic LDS: pref[2][NPAD] u32 (double-buffered over
// d: two barriers per d), then rmin[NPAD] u32 (same padding) when the right view is requested.
template <int NPT>
__global__ __launch_bounds__(kWT) void wide_hwta_kernel(const uint16_t* __restrict__ V, int W, int H, int radius,
                                                        int d_lo, int d_hi, uint32_t seed, uint32_t thresh,
                                                        uint8_t* __restrict__ disp, int opitch,
                                                        uint32_t* __restrict__ keys, uint8_t* __restrict__ right,
                                                        int rpitch) {
    extern __shared__ __attribute__((aligned(16))) uint32_t wl[];
    constexpr int NX = kWT * NPT + 1;                 // prefix entries 0..256 NPT
    constexpr int NPAD = NX + NX / 8 + 1;
    __shared__ uint32_t wsum[2][kWT / 64];
    uint32_t* rmin = wl + 2 * NPAD;
    auto pad = [](int i) { return i + (i >> 3); };
    const int y = blockIdx.x;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int x0 = t * NPT;
    const bool want_right = right != nullptr;
    if (want_right)
        for (int i = t; i < NPAD; i += kWT) rmin[i] = 0xFFFFFFFFu;   // indexed pad(u), as pref
    uint32_t best[NPT];
    int lo[NPT], hi[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        best[k] = seed;
        const int x = x0 + k;
        lo[k] = pad(max(x - radius, 0));              // window columns [lo, hi) of the prefix (Device.cu:51)
        hi[k] = pad(min(x + radius, W - 1) + 1);
    }
    const bool vec = (W % 8) == 0 && (NPT % 8) == 0;   // 16-B rows: 8 u16 per load
    for (int d = d_lo; d < d_hi; ++d) {
        const int b = (d - d_lo) & 1;
        uint32_t* pref = wl + b * NPAD;
        const uint16_t* row = V + ((int64_t)(d - d_lo) * H + y) * W;
        uint32_t p[NPT];
        uint32_t acc = 0;
        if (vec) {
#pragma unroll
            for (int k = 0; k < NPT; k += 8) {
                uint4 q = make_uint4(0, 0, 0, 0);
                if (x0 + k < W) q = *reinterpret_cast<const uint4*>(row + x0 + k);
                const uint32_t w4[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    acc += w4[j] & 0xFFFFu;
                    p[k + 2 * j] = acc;
                    acc += w4[j] >> 16;
                    p[k + 2 * j + 1] = acc;
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < NPT; ++k) {
                acc += x0 + k < W ? (uint32_t)row[x0 + k] : 0u;
                p[k] = acc;
            }
        }
        // inclusive scan of the per-thread totals across the wave, then the waves' offsets
        uint32_t inc = acc;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const uint32_t n = __shfl_up(inc, off, 64);
            if (lane >= off) inc += n;
        }
        if (lane == 63) wsum[b][wv] = inc;
        __syncthreads();
        uint32_t base = inc - acc;
#pragma unroll
        for (int w = 0; w < kWT / 64; ++w) base += w < wv ? wsum[b][w] : 0u;
        if (t == 0) pref[0] = 0u;
#pragma unroll
        for (int k = 0; k < NPT; ++k) pref[pad(x0 + k + 1)] = base + p[k];
        __syncthreads();
        const uint32_t dd = (uint32_t)(d & 0xFF);
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const int x = x0 + k;
            if (x < W) {
                const uint32_t key = ((pref[hi[k]] - pref[lo[k]]) << 8) | dd;
                if (d <= W - x) best[k] = min(best[k], key);       // Device.cu:44
                if (want_right && x >= d) rmin[pad(x - d)] = min(rmin[pad(x - d)], key);
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
            if (want_right) right[(int64_t)y * rpitch + x] = (uint8_t)(rmin[pad(x)] & 0xFFu);   // no threshold
        }
    }
}

template <int NPT>
hipError_t launch_h(const uint16_t* V, int W, int H, int radius, int d_lo, int d_hi, uint32_t seed, uint32_t thresh,
                    uint8_t* disp, int opitch, uint32_t* keys, uint8_t* right, int rpitch, hipStream_t s) {
    constexpr int NX = kWT * NPT + 1;
    const size_t lds = (size_t)((right ? 3 : 2) * (NX + NX / 8 + 1)) * 4;
    hipLaunchKernelGGL(wide_hwta_kernel<NPT>, dim3((unsigned)H), dim3(kWT), lds, s, V, W, H, radius, d_lo, d_hi, seed,
                       thresh, disp, opitch, keys, right, rpitch);
    return hipGetLastError();
}

}  // namespace

size_t wide_workspace_bytes(int W, int H, int D) { return (size_t)D * W * H * sizeof(uint16_t); }

hipError_t launch_box_match_wide(const MatchArgs& a, int batch, uint16_t* ws, uint8_t* right, int rpitch,
                                 int64_t rstride, hipStream_t s) {
    if (a.W <= 0 || a.H <= 0 || a.W > 4096 || a.valid_mode != 0 || a.d_hi <= a.d_lo || batch <= 0)
        return hipErrorInvalidValue;
    const int nd = a.d_hi - a.d_lo;
    for (int f = 0; f < batch; ++f) {
        const uint8_t* Lf = a.left + (int64_t)f * a.frame_stride;
        const uint8_t* Rf = a.right + (int64_t)f * a.frame_stride;
        hipLaunchKernelGGL(wide_vsum_kernel, dim3((unsigned)((a.W + kWT - 1) / kWT), (unsigned)nd), dim3(kWT), 0, s, Lf,
                           Rf, a.W, a.H, a.pitch, a.radius, a.d_lo, a.d_hi, ws);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        uint8_t* disp = a.disp ? a.disp + (int64_t)f * a.out_frame_stride : nullptr;
        uint32_t* keys = a.keys ? a.keys + (int64_t)f * a.W * a.H : nullptr;
        uint8_t* rf = right ? right + (int64_t)f * rstride : nullptr;
        if (a.W <= 4 * kWT)
            e = launch_h<4>(ws, a.W, a.H, a.radius, a.d_lo, a.d_hi, a.seed_key, a.thresh_key, disp, a.out_pitch, keys, rf,
                            rpitch, s);
        else if (a.W <= 8 * kWT)
            e = launch_h<8>(ws, a.W, a.H, a.radius, a.d_lo, a.d_hi, a.seed_key, a.thresh_key, disp, a.out_pitch, keys, rf,
                            rpitch, s);
        else
            e = launch_h<16>(ws, a.W, a.H, a.radius, a.d_lo, a.d_hi, a.seed_key, a.thresh_key, disp, a.out_pitch, keys,
                             rf, rpitch, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace sm
