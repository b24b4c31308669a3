// bm_staged.hip — the staged (cost-volume) formulation of the box path:
//   K1 ad_volume_kernel (bm_volume.hip): AD volume, u8 [D][H][W]               P*D bytes written
//   K2 box_sad_kernel:  SAD volume, u16 [D][H][W]: the (2r+1)^2 window sum of each AD plane,
//                       zero-padded at the borders (= the clipped window, Device.cu:46-56)
//                                                                               P*D read, 2*P*D written
//   K3 volume_wta_kernel: first d with the smallest SAD below 50*win^2, valid d <= W-x
//                       (Device.cu:37-63); 0 where none                          2*P*D read, P written
// The fused box_match_kernel computes the same map without the volumes; this chain streams them
// through HBM, so each kernel is bandwidth-bound and its rocprof HBM rate is the meaningful
// figure (SURVEY §7 hard part (b)).  The u16 SAD volume is also the cost volume for callers who
// aggregate or post-process themselves: the reference's getAllSAD / kernalFindAllSAD
// (BlockMatching.cpp:191-261, Device.cu:67-125) stored it as uint8, truncating mod 256.
#include "bm_common.h"

namespace sm {
namespace {

constexpr int kST = 256;
constexpr int kSW = 64, kSH = 32;   // K2 output tile

// K2: one (64 x 32) tile of one d plane per block.  The input tile is staged with dword loads;
// vertical running sums (lane = column, the 32 rows in 3 chunks so ~all threads work) go to LDS,
// then horizontal running sums, 8 outputs per thread written as one 16-B store.
__device__ __forceinline__ uint32_t ld4z(const uint8_t* plane, int y, int x, int W, int H) {
    if (y < 0 || y >= H) return 0u;
    const uint8_t* row = plane + (int64_t)y * W;
    if (x >= 0 && x + 3 < W) {
        uint32_t v;
        __builtin_memcpy(&v, row + x, 4);
        return v;
    }
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b)
        if (x + b >= 0 && x + b < W) v |= (uint32_t)row[x + b] << (8 * b);
    return v;
}

template <int R>
__global__ __launch_bounds__(kST) void box_sad_kernel(const uint8_t* __restrict__ ad, int W, int H, int tiles_x,
                                                      uint16_t* __restrict__ sad) {
    constexpr int IW = kSW + 2 * R, IH = kSH + 2 * R;
    constexpr int IWD = (IW + 3) / 4;                 // dwords per staged row
    constexpr int CH = 3, CR = (kSH + CH - 1) / CH;   // vertical pass: 3 chunks of <= 11 output rows
    __shared__ __attribute__((aligned(16))) uint8_t tin[IH][IWD * 4 + 4];
    __shared__ uint16_t vs[kSH][IW + 2];
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x, d = blockIdx.y;
    const int x0 = tx * kSW, y0 = ty * kSH;
    const int64_t P = (int64_t)W * H;
    const uint8_t* plane = ad + (int64_t)d * P;
    for (int e = threadIdx.x; e < IH * IWD; e += kST) {
        const int i = e / IWD, j = e - (e / IWD) * IWD;
        *reinterpret_cast<uint32_t*>(&tin[i][4 * j]) = ld4z(plane, y0 - R + i, x0 - R + 4 * j, W, H);
    }
    __syncthreads();
    if (threadIdx.x < CH * IW) {
        const int j = threadIdx.x % IW, c = threadIdx.x / IW;
        const int r0 = c * CR, r1 = r0 + CR < kSH ? r0 + CR : kSH;
        uint32_t sv = 0;
#pragma unroll
        for (int i = 0; i < 2 * R; ++i) sv += tin[r0 + i][j];
        for (int rr = r0; rr < r1; ++rr) {
            sv += tin[rr + 2 * R][j];
            vs[rr][j] = (uint16_t)sv;        // <= (2r+1) * 255, fits u16
            sv -= tin[rr][j];
        }
    }
    __syncthreads();
    const int r = threadIdx.x >> 3, c0 = (threadIdx.x & 7) * 8;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 2 * R; ++k) s += vs[r][c0 + k];
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        s += vs[r][c0 + k + 2 * R];
        const uint32_t v = s;                // <= (2r+1)^2 * 255 < 2^16 for r <= 7
        if (k & 1) o[k >> 1] |= v << 16; else o[k >> 1] = v;
        s -= vs[r][c0 + k];
    }
    const int y = y0 + r, x = x0 + c0;
    if (y >= H) return;
    uint16_t* dst = sad + (int64_t)d * P + (int64_t)y * W + x;
    if (x + 8 <= W && ((reinterpret_cast<uintptr_t>(dst) & 15) == 0)) {
        *reinterpret_cast<uint4*>(dst) = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
        for (int k = 0; k < 8 && x + k < W; ++k) dst[k] = (uint16_t)(o[k >> 1] >> (16 * (k & 1)));
    }
}

// K3: 4 pixels per thread, 8-B loads of the u16 SAD planes.
__global__ __launch_bounds__(kST) void volume_wta_kernel(const uint16_t* __restrict__ sad, int W, int H, int D,
                                                         uint32_t seed_key, uint8_t* __restrict__ disp,
                                                         int out_pitch) {
    const int64_t P = (int64_t)W * H;
    const int64_t p0 = ((int64_t)blockIdx.x * kST + threadIdx.x) * 4;
    if (p0 >= P) return;
    const int n = P - p0 < 4 ? (int)(P - p0) : 4;
    int xs[4];
    uint32_t best[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        xs[k] = (int)((p0 + k) % W);
        best[k] = seed_key;
    }
    const bool vec = n == 4 && ((p0 & 3) == 0) && ((reinterpret_cast<uintptr_t>(sad) & 7) == 0) && ((P & 3) == 0);
    for (int d = 0; d < D; ++d) {
        const uint16_t* pl = sad + (int64_t)d * P + p0;
        uint32_t s[4];
        if (vec) {
            const uint2 v = *reinterpret_cast<const uint2*>(pl);
            s[0] = v.x & 0xFFFFu; s[1] = v.x >> 16; s[2] = v.y & 0xFFFFu; s[3] = v.y >> 16;
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) s[k] = k < n ? pl[k] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t key = (s[k] << 8) | (uint32_t)d;
            // validity: d <= W - x (the `col + d > cols` break, Device.cu:44)
            best[k] = (d <= W - xs[k] && key < best[k]) ? key : best[k];
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (k >= n) break;
        const int64_t p = p0 + k;
        const int y = (int)(p / W);
        disp[(int64_t)y * out_pitch + xs[k]] = best[k] < seed_key ? (uint8_t)(best[k] & 0xFFu) : (uint8_t)0;
    }
}

template <int R>
hipError_t launch_box_sad_r(const uint8_t* ad, int W, int H, int D, uint16_t* sad, hipStream_t s) {
    const int tiles_x = (W + kSW - 1) / kSW, tiles_y = (H + kSH - 1) / kSH;
    hipLaunchKernelGGL(box_sad_kernel<R>, dim3(tiles_x * tiles_y, D), dim3(kST), 0, s, ad, W, H, tiles_x, sad);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_box_sad_volume(const uint8_t* ad, int W, int H, int radius, int D, uint16_t* sad, hipStream_t s) {
#define SM_BOX_SAD_CASE(r) \
    case r: return launch_box_sad_r<r>(ad, W, H, D, sad, s)
    switch (radius) {
        SM_BOX_SAD_CASE(0);
        SM_BOX_SAD_CASE(1);
        SM_BOX_SAD_CASE(2);
        SM_BOX_SAD_CASE(3);
        SM_BOX_SAD_CASE(4);
        SM_BOX_SAD_CASE(5);
        SM_BOX_SAD_CASE(6);
        SM_BOX_SAD_CASE(7);
        default: return hipErrorInvalidValue;
    }
#undef SM_BOX_SAD_CASE
}

hipError_t launch_volume_wta(const uint16_t* sad, int W, int H, int D, uint32_t seed_key, uint8_t* disp,
                             int out_pitch, hipStream_t s) {
    const int64_t P = (int64_t)W * H;
    const int64_t blocks = (P + 4 * kST - 1) / (4 * kST);
    if (blocks <= 0 || blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    hipLaunchKernelGGL(volume_wta_kernel, dim3((unsigned)blocks), dim3(kST), 0, s, sad, W, H, D, seed_key, disp,
                       out_pitch);
    return hipGetLastError();
}

}  // namespace sm
