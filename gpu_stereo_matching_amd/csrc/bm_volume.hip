// bm_volume.hip — the absolute-difference cost volume itself, for callers of the
// reference's PreCal (BlockMatching.cpp:89-109) / kernalPreCal_V2 (Device.cu:19-32):
//   dif[d][y][x] = |L(y,x) - R(y,x-d)|  for x >= d,  0 otherwise (the memset, Device.cu:194),
// d-major planes [D][H][W] exactly as Device.cu:193 lays them out.  The matching path never
// builds this volume (it is fused into box_match_kernel); this kernel exists for drop-in callers
// and is HBM-write-bound (P*D bytes out, 2*P in).
//
// One block per (image row, d-chunk); the R row sits in LDS behind 16 zero bytes.  A thread owns a 16-byte
// segment of the row (its 16 L bytes stay in registers) and walks d: the R bytes x-d .. x-d+15
// come from 5 aligned dword LDS reads and 4 v_alignbyte_b32, |L - R| is formed 2 bytes per
// packed 16-bit lane (v_pk_sub_i16 / v_pk_max_i16), and the 16 result bytes go out as one 16-B
// store (byte stores when the plane layout is not 16-B aligned).
#include "bm_common.h"

namespace sm {
namespace {

constexpr int kVT = 256;
#ifndef SM_ADV_BLOCKS
#define SM_ADV_BLOCKS 16384   // 8-frame staged launches: 52.6 us per frame vs 55.6 at 4096
#endif
#ifndef SM_ADV_MAXSPLIT
#define SM_ADV_MAXSPLIT 16
#endif
#ifndef SM_ADV_NT
#define SM_ADV_NT 1
#endif

typedef short v2i16 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// bytewise |a - b| of two packed u32 words
__device__ __forceinline__ uint32_t absdiff_u8x4(uint32_t a, uint32_t b) {
    const uint32_t ae = a & 0x00FF00FFu, ao = (a >> 8) & 0x00FF00FFu;
    const uint32_t be = b & 0x00FF00FFu, bo = (b >> 8) & 0x00FF00FFu;
    v2i16 de = __builtin_bit_cast(v2i16, ae) - __builtin_bit_cast(v2i16, be);
    v2i16 dO = __builtin_bit_cast(v2i16, ao) - __builtin_bit_cast(v2i16, bo);
    de = __builtin_elementwise_max(de, -de);
    dO = __builtin_elementwise_max(dO, -dO);
    return __builtin_bit_cast(uint32_t, de) | (__builtin_bit_cast(uint32_t, dO) << 8);
}


// SEG output bytes per thread and d (16 or 64).  With 64 each lane stores its 64-B piece of the plane row
// as four 16-B stores (lane l at 64 l + 16 k in store k): the pattern that measured 6.0 TB/s of pure
// writes on this part against 5.5-5.8 for one lane-consecutive 16-B store per lane
// (profiles/microbench/r02_hbm_vendor_ceilings.txt, "chunk 4/lane").
#ifndef SM_ADV_SEG
#define SM_ADV_SEG 16
#endif
template <int SEG>
__global__ __launch_bounds__(kVT) void ad_volume_kernel(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R,
                                                        int W, int H, int pitch, int64_t fstride, int D,
                                                        uint8_t* __restrict__ dif, int64_t dstride) {
    constexpr int NQ = SEG / 4;                                      // dwords per thread and d
    constexpr int kVPad = SEG;   // zero bytes in front of the staged R row (x - d down to -SEG)
    extern __shared__ __attribute__((aligned(16))) uint8_t rrow[];   // [kVPad + nseg * SEG + 4]
    const int y = blockIdx.x, f = blockIdx.y;
    const int dc = (D + gridDim.z - 1) / gridDim.z;               // disparities of this block
    const int d_begin = blockIdx.z * dc, d_end = d_begin + dc < D ? d_begin + dc : D;
    const uint8_t* lr = L + (int64_t)f * fstride + (int64_t)y * pitch;
    const uint8_t* rr = R + (int64_t)f * fstride + (int64_t)y * pitch;
    const int nseg = (W + SEG - 1) / SEG;
    // stage the R row as dwords: rrow dword j = R bytes 4j - kVPad .. 4j - kVPad + 3 (0 outside the row)
    for (int j = threadIdx.x; j < (kVPad + nseg * SEG + 4) / 4; j += kVT) {
        const int c = 4 * j - kVPad;
        uint32_t v = 0;
        if (c >= 0 && c + 3 < W) {
            __builtin_memcpy(&v, rr + c, 4);
        } else {
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (c + b >= 0 && c + b < W) v |= (uint32_t)rr[c + b] << (8 * b);
        }
        // SEG = 64: one pad dword after every 16 (64 B), so the 64-B-strided windows of consecutive
        // lanes start on banks 17 apart instead of 16 (16-way conflicts without it)
        reinterpret_cast<uint32_t*>(rrow)[SEG == 64 ? j + (j >> 4) : j] = v;
    }
    __syncthreads();
    const int64_t P = (int64_t)W * H;
    uint8_t* out = dif + (int64_t)f * dstride + (int64_t)y * W;
    const bool vec = ((W & 15) == 0) && ((P & 15) == 0) && ((reinterpret_cast<uintptr_t>(dif) & 15) == 0) &&
                     ((dstride & 15) == 0);
    // thread -> (segment, d phase): consecutive lanes take consecutive segments of one plane row
    const int groups = kVT / nseg > 0 ? kVT / nseg : 1;
    const int seg = threadIdx.x % nseg, g = threadIdx.x / nseg;
    if (g >= groups) return;
    const int x0 = seg * SEG;
    uint32_t l[NQ];
    if (x0 + SEG <= W) {
        __builtin_memcpy(l, lr + x0, SEG);
    } else {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int x = x0 + 4 * q + b;
                v |= (x < W ? (uint32_t)lr[x] : 0u) << (8 * b);
            }
            l[q] = v;
        }
    }
#pragma unroll 2
    for (int d = d_begin + g; d < d_end; d += groups) {
        // R bytes at x0-d .. x0-d+SEG-1, from the padded row (index kVPad + x0 - d >= 0 while d <= x0 + SEG; a
        // larger d leaves every byte of the segment at x < d)
        uint32_t r[NQ];
        const int start = kVPad + x0 - d;
        if (start >= 0) {
            const int base = start & ~3, sh = start & 3;
            uint32_t wv[NQ + 1];
            if constexpr (SEG == 64) {
                // logical dword j0 + q lives at j0 + q + (j0 + q) / 16; with x0 a multiple of 64 the
                // window's first dword j0 = 16 * seg + s (s uniform), so the pad before dword q is
                // crossed at the same q in every lane
                const int j0 = base >> 2, s16 = j0 & 15;
                const uint32_t* w = reinterpret_cast<const uint32_t*>(rrow) + j0 + (j0 >> 4);
#pragma unroll
                for (int q = 0; q <= NQ; ++q) wv[q] = w[q + (q + s16 >= 16 ? 1 : 0) + (q + s16 >= 32 ? 1 : 0)];
            } else {
                const uint32_t* w = reinterpret_cast<const uint32_t*>(rrow + base);
#pragma unroll
                for (int q = 0; q <= NQ; ++q) wv[q] = w[q];
            }
#pragma unroll
            for (int q = 0; q < NQ; ++q) r[q] = __builtin_amdgcn_alignbyte(wv[q + 1], wv[q], sh);
        } else {
#pragma unroll
            for (int q = 0; q < NQ; ++q) r[q] = 0u;   // every byte of this segment has x < d: masked below
        }
        uint32_t o[NQ];
#pragma unroll
        for (int q = 0; q < NQ; ++q) o[q] = absdiff_u8x4(l[q], r[q]);
        if (x0 < d + SEG) {   // bytes with x < d are 0 (Device.cu:27-31 + the memset)
            // dword q drops its low n = clamp(d - x0 - 4q, 0, 4) bytes: one 64-bit shift per dword (a
            // per-byte compare + select here cost 8 VALU per dword plus hazard nops, in every wave
            // holding the row's first segment)
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                const int n = min(max(d - x0 - 4 * q, 0), 4);
                o[q] &= (uint32_t)(~0ull << (8 * n));
            }
        }
        uint8_t* dst = out + (int64_t)d * P + x0;
        if (vec && x0 + SEG <= W) {
            // streaming output (P*D bytes, larger than the MALL): nontemporal 16-B stores
#pragma unroll
            for (int k = 0; k < NQ / 4; ++k) {
                const u32x4 v = {o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]};
                if (SM_ADV_NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst) + k);
                else reinterpret_cast<u32x4*>(dst)[k] = v;
            }
        } else {
            const int n = W - x0 < SEG ? W - x0 : SEG;
            for (int b = 0; b < n; ++b) dst[b] = (uint8_t)(o[b >> 2] >> (8 * (b & 3)));
        }
    }
}

}  // namespace

hipError_t launch_ad_volume(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int64_t fstride, int batch,
                            int D, uint8_t* dif, int64_t dstride, hipStream_t s) {
    constexpr int SEG = SM_ADV_SEG;
    const int nseg = (W + SEG - 1) / SEG;
    if (W <= 0 || H <= 0 || D <= 0 || batch <= 0 || nseg > kVT) return hipErrorInvalidValue;
    const size_t lds = ((size_t)(SEG + nseg * SEG + 4) * (SEG == 64 ? 17 : 16) / 16 + 4 + 15) & ~(size_t)15;
    // enough blocks in flight (>= ~4 per CU of 256) to keep the stores streaming
    int dsplit = (SM_ADV_BLOCKS + H * batch - 1) / (H * batch);
    dsplit = dsplit < 1 ? 1 : (dsplit > D ? D : (dsplit > SM_ADV_MAXSPLIT ? SM_ADV_MAXSPLIT : dsplit));
    hipLaunchKernelGGL(ad_volume_kernel<SEG>, dim3(H, batch, dsplit), dim3(kVT), lds, s, L, R, W, H, pitch, fstride,
                       D, dif, dstride);
    return hipGetLastError();
}

}  // namespace sm
