// bm_pre.hip — the steps in front of the matching path (SURVEY §8f "next", ranks 1-2).
//
// bgr_to_gray: the caller's cvtColor(src, gray, CV_BGR2GRAY) (Caller.cpp:15-16) with OpenCV 2.4's
//   8-bit fixed-point weights, Y = (1868 B + 9617 G + 4899 R + 8192) >> 14 — NOT the reference's
//   own kernalCvtColor (Device.cu:136-143), which applies the luma weights to B,G,R in the wrong
//   order with float rounding.  Integer, bit-exact.  HBM-bound: 4 pixels per thread.
// remap_bilinear: kernalRemap + BilinearInterpolation + float2uchar (Device.cu:127-167), i.e.
//   rectification with CV_32FC1 maps.  Out-of-range taps -> 0 (Device.cu:155-157), round half to
//   even and saturate (cvt.rni.sat, Device.cu:148).  Float expressions are evaluated exactly as
//   written, without FMA contraction, so results match the CPU twin CPU_Remap (Utility.cpp:239-264).
#include "bm_common.h"

namespace sm {
namespace {

__global__ __launch_bounds__(256) void bgr_to_gray_kernel(const uint8_t* __restrict__ src, int W, int H, int pitch,
                                                          int channels, uint8_t* __restrict__ dst, int dpitch) {
    const int x4 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const int y = blockIdx.y;
    if (x4 >= W) return;
    const uint8_t* row = src + (int64_t)y * pitch;
    uint32_t out = 0;
    const int n = W - x4 < 4 ? W - x4 : 4;
    for (int k = 0; k < n; ++k) {
        const uint8_t* px = row + (int64_t)(x4 + k) * channels;
        const uint32_t v = 1868u * px[0] + 9617u * px[1] + 4899u * px[2] + 8192u;
        out |= (v >> 14) << (8 * k);
    }
    uint8_t* o = dst + (int64_t)y * dpitch + x4;
    if (n == 4 && ((reinterpret_cast<uintptr_t>(o) & 3) == 0)) {
        *reinterpret_cast<uint32_t*>(o) = out;
    } else {
        for (int k = 0; k < n; ++k) o[k] = (uint8_t)(out >> (8 * k));
    }
}

#pragma clang fp contract(off)
__device__ __forceinline__ float bilinear(const uint8_t* __restrict__ src, int rows, int cols, int pitch, float x,
                                          float y) {
    // x = row coordinate (map_y), y = column coordinate (map_x), as Device.cu:152-167
    const int x1 = (int)floorf(x), y1 = (int)floorf(y), x2 = x1 + 1, y2 = y1 + 1;
    if (x1 < 0 || x2 >= rows || y1 < 0 || y2 >= cols) return 0.f;
    const uint8_t* r1 = src + (int64_t)x1 * pitch;
    const uint8_t* r2 = r1 + pitch;
    const float q11 = r1[y1], q12 = r1[y2], q21 = r2[y1], q22 = r2[y2];
    const float left = (float)(x2 - x) * q11 + (x - (float)x1) * q21;
    const float right = (float)(x2 - x) * q12 + (x - (float)x1) * q22;
    return ((float)y2 - y) * left + (y - (float)y1) * right;
}

__global__ __launch_bounds__(256) void remap_kernel(const uint8_t* __restrict__ src, int W, int H, int pitch,
                                                    const float* __restrict__ mapx, const float* __restrict__ mapy,
                                                    int mpitch, uint8_t* __restrict__ dst, int dpitch) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const float xcoo = mapx[(int64_t)y * mpitch + x];
    const float ycoo = mapy[(int64_t)y * mpitch + x];
    const float v = bilinear(src, H, W, pitch, ycoo, xcoo);
    // cvt.rni.sat.u8.f32: round half to even, saturate to [0, 255] (NaN -> 0)
    const float r = __builtin_rintf(v);
    const float c = r > 255.f ? 255.f : (r > 0.f ? r : 0.f);
    dst[(int64_t)y * dpitch + x] = (uint8_t)c;
}
#pragma clang fp contract(on)

}  // namespace

hipError_t launch_bgr_to_gray(const uint8_t* src, int W, int H, int pitch, int channels, uint8_t* dst, int dpitch,
                              hipStream_t s) {
    dim3 grid((W + 1023) / 1024, H);
    hipLaunchKernelGGL(bgr_to_gray_kernel, grid, dim3(256), 0, s, src, W, H, pitch, channels, dst, dpitch);
    return hipGetLastError();
}

hipError_t launch_remap(const uint8_t* src, int W, int H, int pitch, const float* mapx, const float* mapy, int mpitch,
                        uint8_t* dst, int dpitch, hipStream_t s) {
    dim3 grid((W + 255) / 256, H);
    hipLaunchKernelGGL(remap_kernel, grid, dim3(256), 0, s, src, W, H, pitch, mapx, mapy, mpitch, dst, dpitch);
    return hipGetLastError();
}

}  // namespace sm
