// bm_post.hip — disparity post-filter: the (2r+1)^2 median that the
// reference's STMatching pipeline applies to its WTA maps, MeanFilter(disp, disp, 3)
// (Toolkit.cpp:33-48 -> ctmf(), STMatching/ctmf.c:378-433; used at StereoDisparity.cpp:85,
// 119, 126, 156).  ctmf clamps its row/column histograms to the image (replicate padding) and
// returns the (t+1)-th smallest value, t = 2r^2 + 2r (ctmf.c:230-329).
//
// median_kernel<R>: a 64 x 32 output tile per workgroup; the (32 + 2R) x (64 + 2R) input tile is
// staged in LDS with clamped coordinates.  Each thread owns one column and 8 consecutive rows.
// Each input row's 2R+1 window bytes are packed once into R+1 u32 words of two u16 lanes,
// v | 0x100 (plus one dummy lane of 255).  A radix select over the 8 bits then counts the values
// >= cand for all lanes at once:
//   lane = 0x100 + v - cand  (never borrows: 1 <= lane <= 511), bit 8 set <=> v >= cand.
// That is one v_sub, v_and and v_bcnt per word and bit.  Integer throughout, so bit-exact.
#include "bm_common.h"

namespace sm {
namespace {

constexpr int kMTW = 64, kMTH = 32, kMRows = 8;   // tile, rows per thread

template <int R>
__global__ __launch_bounds__(256) void median_kernel(const uint8_t* __restrict__ src, int W, int H, int pitch,
                                                     int64_t stride, uint8_t* __restrict__ dst, int dpitch,
                                                     int64_t dstride, int tiles_x, int tiles) {
    constexpr int SW = kMTW + 2 * R, SH = kMTH + 2 * R;
    constexpr int SEGW = R + 1;                         // packed words per window row
    constexpr int NIN = kMRows + 2 * R;                 // input rows per thread
    constexpr int T = 2 * R * R + 2 * R;                // rank of the median (0-based)
    constexpr int LANES = 2 * SEGW * (2 * R + 1);       // lanes per window incl. one dummy per row
    __shared__ uint8_t tile[SH][SW + 1];

    const int frame = blockIdx.x / tiles;
    const int t = blockIdx.x - frame * tiles;
    const int ty = t / tiles_x, tx = t - ty * tiles_x;
    const int x0 = tx * kMTW, y0 = ty * kMTH;
    const uint8_t* S = src + (int64_t)frame * stride;
    for (int e = threadIdx.x; e < SH * SW; e += 256) {
        const int i = e / SW, j = e - (e / SW) * SW;
        int y = y0 - R + i, x = x0 - R + j;
        y = y < 0 ? 0 : (y > H - 1 ? H - 1 : y);
        x = x < 0 ? 0 : (x > W - 1 ? W - 1 : x);
        tile[i][j] = S[(int64_t)y * pitch + x];
    }
    __syncthreads();

    const int c = threadIdx.x & 63;                     // output column in the tile
    const int r0 = (threadIdx.x >> 6) * kMRows;         // first output row in the tile
    uint32_t wds[NIN][SEGW];
#pragma unroll
    for (int i = 0; i < NIN; ++i) {
#pragma unroll
        for (int k = 0; k < SEGW; ++k) {
            const uint32_t a = tile[r0 + i][c + 2 * k];
            const uint32_t b = (2 * k + 1 <= 2 * R) ? (uint32_t)tile[r0 + i][c + 2 * k + 1] : 255u;
            wds[i][k] = a | (b << 16) | 0x01000100u;
        }
    }
    uint8_t* D = dst + (int64_t)frame * dstride;
#pragma unroll
    for (int o = 0; o < kMRows; ++o) {
        uint32_t ans = 0;
#pragma unroll
        for (int bit = 7; bit >= 0; --bit) {
            const uint32_t cand = ans | (1u << bit);
            const uint32_t c2 = cand * 0x00010001u;
            uint32_t ge = 0;
#pragma unroll
            for (int i = 0; i <= 2 * R; ++i)
#pragma unroll
                for (int k = 0; k < SEGW; ++k) ge += (uint32_t)__builtin_popcount((wds[o + i][k] - c2) & 0x01000100u);
            // values < cand among the real ones = LANES - ge (every dummy 255 >= cand)
            ans = (LANES - (int)ge <= T) ? cand : ans;
        }
        const int y = y0 + r0 + o, x = x0 + c;
        if (y < H && x < W) D[(int64_t)y * dpitch + x] = (uint8_t)ans;
    }
}

}  // namespace

hipError_t launch_median(const uint8_t* src, int W, int H, int pitch, int64_t stride, int batch, int radius,
                         uint8_t* dst, int dpitch, int64_t dstride, hipStream_t s) {
    const int tiles_x = (W + kMTW - 1) / kMTW, tiles_y = (H + kMTH - 1) / kMTH;
    const int64_t blocks = (int64_t)tiles_x * tiles_y * batch;
    if (blocks <= 0 || blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    const dim3 g((unsigned)blocks), b(256);
    switch (radius) {
        case 1: hipLaunchKernelGGL(median_kernel<1>, g, b, 0, s, src, W, H, pitch, stride, dst, dpitch, dstride, tiles_x, tiles_x * tiles_y); break;
        case 2: hipLaunchKernelGGL(median_kernel<2>, g, b, 0, s, src, W, H, pitch, stride, dst, dpitch, dstride, tiles_x, tiles_x * tiles_y); break;
        case 3: hipLaunchKernelGGL(median_kernel<3>, g, b, 0, s, src, W, H, pitch, stride, dst, dpitch, dstride, tiles_x, tiles_x * tiles_y); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace sm
