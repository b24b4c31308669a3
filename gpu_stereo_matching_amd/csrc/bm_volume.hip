// bm_volume.hip — the absolute-difference cost volume itself, for callers of the
// reference's PreCal (BlockMatching.cpp:89-109) / kernalPreCal_V2 (Device.cu:19-32):
//   dif[d][y][x] = |L(y,x) - R(y,x-d)|  for x >= d,  0 otherwise (the memset, Device.cu:194),
// d-major planes [D][H][W] exactly as Device.cu:193 lays them out.  The matching path never
// builds this volume (it is fused into box_match_kernel); this kernel exists for drop-in callers
// and is HBM-write-bound (P*D bytes out, 2*P in).
//
// One block per (band of rows, d-chunk); the band's R rows sit in LDS behind 16 zero bytes.  A thread owns
// 16-byte segments of the band (their L bytes stay in registers) and walks d: the R bytes x-d .. x-d+15
// come from 5 aligned dword LDS reads and 4 v_alignbyte_b32, |L - R| is formed 2 bytes per packed
// 16-bit lane (v_pk_sub_i16 / v_pk_max_i16), and the 16 result bytes go out as one 16-B store (byte
// stores when the plane layout is not 16-B aligned).
#include <algorithm>

#include "bm_common.h"

namespace sm {
namespace {

constexpr int kVT = 256;
// Round 4 (profiles/microbench/r04_ad_order_ab.txt): 2 d chunks of 2-row bands.  Each
// chunk re-reads its band, so the fabric traffic is ~(1 + chunks * 2 / (D + 2)) x the algorithmic bytes:
// rocprof 1.013x at 2 chunks (0.408 ms per 8-frame launch, 0.661 of 8 TB/s), against 1.166x at the round-3
// 16 chunks of 4 rows (0.40-0.44 ms) and 1.083x at 8 (0.400 ms).
#ifndef SM_ADV_MAXSPLIT
#define SM_ADV_MAXSPLIT 2    // d chunks per (band, frame): 64 d per block at D = 128
#endif
#ifndef SM_ADV_NT
#define SM_ADV_NT 1
#endif
#ifndef SM_ADV_ROWS
#define SM_ADV_ROWS 2      // image rows per block
#endif
// Block order (round 4; profiles/microbench/r04_ad_order_ab.txt): the grid (band, frame,
// chunk) in blockIdx (x, y, z), so the blocks in flight write the planes of one chunk for ~8 frames.  Measured
// and removed in round 5 (git history): a flat d-fastest XCD-contiguous order (63 us per 1080p frame against
// 48: every plane written at once), chunk groups (54-59 us) and (band, chunk, frame).

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


// A block owns RB consecutive image rows and a d range; per d it writes those rows of the plane, one
// contiguous RB * W-byte run (16 B per lane, a wave's store 1 KiB contiguous).  With RB * nseg segments
// per d: <= 256 -> 256 / (RB * nseg) d phases of one segment per thread; else KF segments per thread.
// (Writing one image row per block and d, the planes' 1.9-KB pieces from ~2000 resident blocks landed
// in 64 planes at once: 0.64 of 8 TB/s against 0.72-0.76 for streamed pure writes.)
template <int KF>
__global__ __launch_bounds__(kVT) void ad_volume_kernel(const uint8_t* __restrict__ L, const uint8_t* __restrict__ R,
                                                        int W, int H, int pitch, int64_t fstride, int D, int RB,
                                                        int dsp, uint8_t* __restrict__ dif, int64_t dstride) {
    constexpr int SEG = 16, NQ = 4;
    constexpr int kVPad = SEG;   // zero bytes in front of each staged R row (x - d down to -SEG)
    extern __shared__ __attribute__((aligned(16))) uint8_t rrow[];   // [RB][rstride]
    const int y0 = blockIdx.x * RB, f = blockIdx.y;
    const int dz = blockIdx.z;
    const int dc = (D + dsp - 1) / dsp;                           // disparities of this block
    const int d_begin = dz * dc, d_end = d_begin + dc < D ? d_begin + dc : D;
    const int nseg = (W + SEG - 1) / SEG;
    const int rdw = (kVPad + nseg * SEG + 4) / 4;                 // staged dwords per R row
    const int rows = min(RB, H - y0);
    // stage the R rows as dwords: dword j of row i = R bytes 4j - kVPad .. 4j - kVPad + 3 (0 outside the row)
    for (int e = threadIdx.x; e < rows * rdw; e += kVT) {
        const int i = e / rdw, j = e - i * rdw;
        const uint8_t* rr = R + (int64_t)f * fstride + (int64_t)(y0 + i) * pitch;
        const int c = 4 * j - kVPad;
        uint32_t v = 0;
        if (c >= 0 && c + 3 < W) {
            __builtin_memcpy(&v, rr + c, 4);
        } else {
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (c + b >= 0 && c + b < W) v |= (uint32_t)rr[c + b] << (8 * b);
        }
        reinterpret_cast<uint32_t*>(rrow)[e] = v;
    }
    __syncthreads();
    const int64_t P = (int64_t)W * H;
    uint8_t* out = dif + (int64_t)f * dstride + (int64_t)y0 * W;   // + d * P + row * W + x
    const bool vec = ((W & 15) == 0) && ((P & 15) == 0) && ((reinterpret_cast<uintptr_t>(dif) & 15) == 0) &&
                     ((dstride & 15) == 0);
    const int nflat = rows * nseg;
    const int groups = KF == 1 && kVT / nflat > 0 ? kVT / nflat : 1;
    const int g = KF == 1 ? threadIdx.x / nflat : 0;
    if (g >= groups) return;
    // this thread's segments: flat index fl = row * nseg + seg
    int fl[KF], x0[KF];
    uint32_t l[KF][NQ];
#pragma unroll
    for (int k = 0; k < KF; ++k) {
        fl[k] = KF == 1 ? (int)threadIdx.x % nflat : (int)threadIdx.x + k * kVT;
        const int i = fl[k] < nflat ? fl[k] / nseg : 0;
        x0[k] = (fl[k] - i * nseg) * SEG;
        const uint8_t* lr = L + (int64_t)f * fstride + (int64_t)(y0 + i) * pitch;
        if (fl[k] < nflat && x0[k] + SEG <= W) {
            __builtin_memcpy(l[k], lr + x0[k], SEG);
        } else {
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                uint32_t v = 0;
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int x = x0[k] + 4 * q + b;
                    v |= (fl[k] < nflat && x < W ? (uint32_t)lr[x] : 0u) << (8 * b);
                }
                l[k][q] = v;
            }
        }
    }
#pragma unroll 2
    for (int d = d_begin + g; d < d_end; d += groups) {
#pragma unroll
        for (int k = 0; k < KF; ++k) {
            if (fl[k] >= nflat) continue;
            const int i = fl[k] / nseg;
            // R bytes at x0-d .. x0-d+15 from the padded row (index kVPad + x0 - d >= 0 while d <= x0 + 16;
            // a larger d leaves every byte of the segment at x < d)
            uint32_t r[NQ];
            const int start = kVPad + x0[k] - d;
            if (start >= 0) {
                const int base = start & ~3, sh = start & 3;
                const uint32_t* w = reinterpret_cast<const uint32_t*>(rrow + (size_t)i * rdw * 4 + base);
                uint32_t wv[NQ + 1];
#pragma unroll
                for (int q = 0; q <= NQ; ++q) wv[q] = w[q];
#pragma unroll
                for (int q = 0; q < NQ; ++q) r[q] = __builtin_amdgcn_alignbyte(wv[q + 1], wv[q], sh);
            } else {
#pragma unroll
                for (int q = 0; q < NQ; ++q) r[q] = 0u;   // every byte of this segment has x < d: masked below
            }
            uint32_t o[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q) o[q] = absdiff_u8x4(l[k][q], r[q]);
            if (x0[k] < d + SEG) {   // bytes with x < d are 0 (Device.cu:27-31 + the memset)
                // dword q drops its low n = clamp(d - x0 - 4q, 0, 4) bytes: one 64-bit shift per dword
#pragma unroll
                for (int q = 0; q < NQ; ++q) {
                    const int n = min(max(d - x0[k] - 4 * q, 0), 4);
                    o[q] &= (uint32_t)(~0ull << (8 * n));
                }
            }
            uint8_t* dst = out + (int64_t)d * P + (int64_t)i * W + x0[k];
            if (vec && x0[k] + SEG <= W) {
                // streaming output (P*D bytes, larger than the MALL): nontemporal 16-B stores
                const u32x4 v = {o[0], o[1], o[2], o[3]};
                if (SM_ADV_NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst));
                else *reinterpret_cast<u32x4*>(dst) = v;
            } else {
                const int n = W - x0[k] < SEG ? W - x0[k] : SEG;
                for (int b = 0; b < n; ++b) dst[b] = (uint8_t)(o[b >> 2] >> (8 * (b & 3)));
            }
        }
    }
}

}  // namespace

hipError_t launch_ad_volume(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int64_t fstride, int batch,
                            int D, uint8_t* dif, int64_t dstride, hipStream_t s) {
    constexpr int SEG = 16;
    const int nseg = (W + SEG - 1) / SEG;
    if (W <= 0 || H <= 0 || D <= 0 || batch <= 0 || nseg > 4 * kVT) return hipErrorInvalidValue;
    // rows per block: up to SM_ADV_ROWS, at most 4 segments per thread
    int rb = SM_ADV_ROWS;
    while (rb > 1 && rb * nseg > 4 * kVT) --rb;
    if (rb > H) rb = H;
    const int kf = (rb * nseg + kVT - 1) / kVT;
    const size_t lds = (size_t)rb * ((SEG + nseg * SEG + 4) / 4) * 4;
    const int bands = (H + rb - 1) / rb;
    // Same-box A/B, 8 x 1080p D = 128 frames per launch (tools/ab_staged_kernels.py, HIP events), rows per
    // block x d chunks, round 3: 1 x 2 52.3 us per frame; 4 x 16 48.0; 1 x 8 49.2; 8 x 16 50.6; 4 x 32
    // 59.6; plain instead of nontemporal stores 49.2.  Round 4 (one box): 4 x 16 50.2; 4 x 8 50.7;
    // 2 x 4 50.7; 4 x 2 53.7; 2 x 2 52.1 (kept: the fewest re-reads of the band, see SM_ADV_MAXSPLIT)
    const int dsplit = std::max(1, std::min(D, SM_ADV_MAXSPLIT));
    const dim3 grid((unsigned)bands, (unsigned)batch, (unsigned)dsplit);
    if (kf <= 1)
        hipLaunchKernelGGL(ad_volume_kernel<1>, grid, dim3(kVT), lds, s, L, R, W, H, pitch, fstride, D, rb, dsplit, dif,
                           dstride);
    else if (kf == 2)
        hipLaunchKernelGGL(ad_volume_kernel<2>, grid, dim3(kVT), lds, s, L, R, W, H, pitch, fstride, D, rb, dsplit, dif,
                           dstride);
    else
        hipLaunchKernelGGL(ad_volume_kernel<4>, grid, dim3(kVT), lds, s, L, R, W, H, pitch, fstride, D, rb, dsplit, dif,
                           dstride);
    return hipGetLastError();
}

}  // namespace sm
