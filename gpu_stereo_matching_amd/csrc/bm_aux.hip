// bm_aux.hip — byte-streaming kernels around the matcher: key finalisation (multi-GPU
// d-slice reduction), horizontal mirror (right view), left-right consistency check.
// All are HBM-bound elementwise passes (the LR check: one row per block, 4 pixels per thread).
#include "bm_common.h"

namespace sm {
namespace {

// key -> disparity (Device.cu:37-38,57,63: d when the best SAD is below 50*win^2, else 0)
__global__ __launch_bounds__(256) void keys_to_disp_kernel(const uint32_t* __restrict__ keys, int W, int H,
                                                           uint32_t thresh_key, uint8_t* __restrict__ disp,
                                                           int out_pitch) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= W) return;
    const uint32_t k = keys[(int64_t)y * W + x];
    disp[(int64_t)y * out_pitch + x] = k < thresh_key ? (uint8_t)(k & 0xFFu) : (uint8_t)0;
}

// dst(y, x) = src(y, W-1-x) for each frame
__global__ __launch_bounds__(256) void mirror_kernel(const uint8_t* __restrict__ src, int W, int H, int pitch,
                                                     int64_t stride, uint8_t* __restrict__ dst, int dpitch,
                                                     int64_t dstride) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int f = blockIdx.z;
    if (x >= W) return;
    dst[(int64_t)f * dstride + (int64_t)y * dpitch + x] = src[(int64_t)f * stride + (int64_t)y * pitch + (W - 1 - x)];
}

// StereoDisparity.cpp:136-147; the right map is stored plain or mirrored (index W-1-u holds dR(u)):
//   d = dL(y,x); occ = x-d < 0 || d == 0 || |d - dR(y, x-d)| > 1;  out = occ ? 0 : d
// `out` may alias `ld` (each thread reads its own pixel before writing it).
__global__ __launch_bounds__(256) void lr_check_kernel(const uint8_t* ld, int lpitch, int64_t lstride,
                                                       const uint8_t* __restrict__ rd, int rpitch, int64_t rstride,
                                                       int mirrored, int W, uint8_t* out, int opitch, int64_t ostride,
                                                       uint8_t* __restrict__ right_out, uint8_t* __restrict__ mask_out,
                                                       int apitch, int64_t astride) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    const int f = blockIdx.z;
    if (x >= W) return;
    const uint8_t* lrow = ld + (int64_t)f * lstride + (int64_t)y * lpitch;
    const uint8_t* rrow = rd + (int64_t)f * rstride + (int64_t)y * rpitch;
    const int d = lrow[x];
    int occ = 1;
    if (x - d >= 0) {
        const int u = x - d;
        const int dr = rrow[mirrored ? W - 1 - u : u];
        const int diff = d - dr;
        occ = (d == 0) || diff > 1 || diff < -1;
    }
    out[(int64_t)f * ostride + (int64_t)y * opitch + x] = occ ? (uint8_t)0 : (uint8_t)d;
    if (mask_out) mask_out[(int64_t)f * astride + (int64_t)y * apitch + x] = (uint8_t)!occ;
    if (right_out) right_out[(int64_t)f * astride + (int64_t)y * apitch + x] = rrow[mirrored ? W - 1 - x : x];
}

// The same check with one block per (row, frame) (round 4): the right row is staged in LDS, so its
// gathers dR(x - d) stay on chip, and each thread takes 4 pixels with dword loads and stores when the
// rows are 4-byte aligned (bytes otherwise, and for a row's last W mod 4 pixels).  The byte-per-thread
// kernel above took 6.2 us per 1080p frame for ~8 MB of traffic (guided + LR, 32-frame launches).
__global__ __launch_bounds__(256) void lr_check_row_kernel(const uint8_t* ld, int lpitch, int64_t lstride,
                                                           const uint8_t* __restrict__ rd, int rpitch, int64_t rstride,
                                                           int mirrored, int W, uint8_t* out, int opitch,
                                                           int64_t ostride, uint8_t* __restrict__ right_out,
                                                           uint8_t* __restrict__ mask_out, int apitch,
                                                           int64_t astride) {
    extern __shared__ uint8_t rs[];   // the right row, W bytes (+3 pad)
    const int y = blockIdx.x, f = blockIdx.y;
    const uint8_t* lrow = ld + (int64_t)f * lstride + (int64_t)y * lpitch;
    const uint8_t* rrow = rd + (int64_t)f * rstride + (int64_t)y * rpitch;
    uint8_t* orow = out + (int64_t)f * ostride + (int64_t)y * opitch;
    uint8_t* mrow = mask_out ? mask_out + (int64_t)f * astride + (int64_t)y * apitch : nullptr;
    uint8_t* rorow = right_out ? right_out + (int64_t)f * astride + (int64_t)y * apitch : nullptr;
    const bool vec = ((reinterpret_cast<uintptr_t>(lrow) | reinterpret_cast<uintptr_t>(rrow) |
                       reinterpret_cast<uintptr_t>(orow) | reinterpret_cast<uintptr_t>(mrow) |
                       reinterpret_cast<uintptr_t>(rorow)) & 3) == 0;
    const int W4 = vec ? (W & ~3) : 0;   // pixels taken 4 at a time
    for (int i = threadIdx.x * 4; i < W4; i += blockDim.x * 4)
        *reinterpret_cast<uint32_t*>(rs + i) = *reinterpret_cast<const uint32_t*>(rrow + i);
    for (int i = W4 + threadIdx.x; i < W; i += blockDim.x) rs[i] = rrow[i];
    __syncthreads();
    auto one = [&](int x, int d) -> uint32_t {   // checked d (low byte) | mask << 8 | dR(x) << 16
        int occ = 1;
        if (x - d >= 0) {
            const int u = x - d;
            const int diff = d - (int)rs[mirrored ? W - 1 - u : u];
            occ = (d == 0) || diff > 1 || diff < -1;
        }
        return (occ ? 0u : (uint32_t)d) | ((uint32_t)!occ << 8) | ((uint32_t)rs[mirrored ? W - 1 - x : x] << 16);
    };
    for (int x = threadIdx.x * 4; x < W4; x += blockDim.x * 4) {
        const uint32_t dl = *reinterpret_cast<const uint32_t*>(lrow + x);
        uint32_t o = 0, m = 0, r = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t v = one(x + b, (int)((dl >> (8 * b)) & 0xFFu));
            o |= (v & 0xFFu) << (8 * b);
            m |= ((v >> 8) & 0xFFu) << (8 * b);
            r |= (v >> 16) << (8 * b);
        }
        *reinterpret_cast<uint32_t*>(orow + x) = o;
        if (mrow) *reinterpret_cast<uint32_t*>(mrow + x) = m;
        if (rorow) *reinterpret_cast<uint32_t*>(rorow + x) = r;
    }
    for (int x = W4 + threadIdx.x; x < W; x += blockDim.x) {
        const uint32_t v = one(x, lrow[x]);
        orow[x] = (uint8_t)(v & 0xFFu);
        if (mrow) mrow[x] = (uint8_t)(v >> 8);
        if (rorow) rorow[x] = (uint8_t)(v >> 16);
    }
}

// acc[i] = min(acc[i], src[i]), signed (box keys are < 2^31, guided keys carry a signed cost): the
// MIN of an RCCL reduce-scatter, for the d-slice split rehearsed on one device (sm_dslice_rehearse_u8)
__global__ __launch_bounds__(256) void min_keys_kernel(int* __restrict__ acc, const int* __restrict__ src, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) acc[i] = min(acc[i], src[i]);
}

__global__ __launch_bounds__(256) void min_keys_u32_kernel(uint32_t* __restrict__ acc, const uint32_t* __restrict__ src,
                                                           int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) acc[i] = min(acc[i], src[i]);
}

__global__ __launch_bounds__(256) void keys_low_byte_kernel(const uint32_t* __restrict__ keys, int64_t n,
                                                            uint8_t* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint8_t)(keys[i] & 0xFFu);
}

}  // namespace

hipError_t launch_min_keys_u32(uint32_t* acc, const uint32_t* src, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(min_keys_u32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, acc, src, n);
    return hipGetLastError();
}

hipError_t launch_keys_low_byte(const uint32_t* keys, int64_t n, uint8_t* out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(keys_low_byte_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, keys, n, out);
    return hipGetLastError();
}

hipError_t launch_min_keys(int* acc, const int* src, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(min_keys_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, acc, src, n);
    return hipGetLastError();
}

hipError_t launch_keys_to_disp(const uint32_t* keys, int W, int H, uint32_t thresh_key, uint8_t* disp,
                               int out_pitch, hipStream_t s) {
    dim3 grid((W + 255) / 256, H, 1);
    hipLaunchKernelGGL(keys_to_disp_kernel, grid, dim3(256), 0, s, keys, W, H, thresh_key, disp, out_pitch);
    return hipGetLastError();
}

hipError_t launch_mirror(const uint8_t* src, int W, int H, int pitch, int64_t stride, int batch, uint8_t* dst,
                         int dst_pitch, int64_t dst_stride, hipStream_t s) {
    dim3 grid((W + 255) / 256, H, batch);
    hipLaunchKernelGGL(mirror_kernel, grid, dim3(256), 0, s, src, W, H, pitch, stride, dst, dst_pitch, dst_stride);
    return hipGetLastError();
}

hipError_t launch_lr_check(const uint8_t* left_disp, int lpitch, int64_t lstride, const uint8_t* right_disp,
                           int rpitch, int64_t rstride, int right_mirrored, int W, int H, int batch, uint8_t* out,
                           int opitch, int64_t ostride, uint8_t* right_out, uint8_t* mask_out, int aux_pitch,
                           int64_t aux_stride, hipStream_t s) {
    if (W <= 0 || H <= 0 || batch <= 0) return hipSuccess;
    if (W <= 16384) {   // the right row in LDS
        hipLaunchKernelGGL(lr_check_row_kernel, dim3((unsigned)H, (unsigned)batch), dim3(256), (size_t)((W + 3) & ~3), s,
                           left_disp, lpitch, lstride, right_disp, rpitch, rstride, right_mirrored, W, out, opitch,
                           ostride, right_out, mask_out, aux_pitch, aux_stride);
        return hipGetLastError();
    }
    dim3 grid((W + 255) / 256, H, batch);
    hipLaunchKernelGGL(lr_check_kernel, grid, dim3(256), 0, s, left_disp, lpitch, lstride, right_disp, rpitch, rstride,
                       right_mirrored, W, out, opitch, ostride, right_out, mask_out, aux_pitch, aux_stride);
    return hipGetLastError();
}

}  // namespace sm
