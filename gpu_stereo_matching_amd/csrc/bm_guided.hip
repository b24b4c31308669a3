// bm_guided.hip — guided-filter cost aggregation + WTA, one fused kernel.
//
// The reference has no guided filter; this build defines it and
// the fp64 restatement oracle/bm_oracle.c:ora_guided_disp is its checker:
//   guide I = L, cost p_d = AD_d (0 for x < d, as Device.cu:27-31), f = clipped-window mean,
//   a = (f(Ip) - f(I) f(p)) / (f(II) - f(I)^2 + eps),  b = f(p) - a f(I),  q = f(a) I + f(b),
//   WTA: first d with the smallest q below 50 (= 50*win^2 / win^2, Device.cu:37), valid d <= W-x.
// In window sums (N = clipped window count, S* = sums):
//   a = (N*SIp - SI*Sp) / (N*SII - SI^2 + eps*N^2)   numerator exact in u32 (|N^2 cov| < 2^31)
//   b = (Sp - a*SI) / N
//
// guided_fused_kernel: the whole pipeline for one output tile and every d, inside LDS.
//   P region (cost sums)   : 64 columns (one per lane) x (TH + 4R) rows from image (x0-2R, y0-2R)
//   A region (a, b)        : (TW + 2R) x (TH + 2R) from image (x0-R, y0-R)
//   output tile            : TW = 64 - 4R  x  TH = 32
// Stages per d:
//   S1V  lane = P column; waves split the A rows: prefix T += AD*(1 + 4096 L) -> packed CS rows
//   S1H  thread = (A row, segment): running Sp / SIp -> a, b
//   S2V  thread = (A column, 8-row group): running float sums of a, b over 2R+1 rows
//   S2H  thread = (output row, segment): running sums -> N*q = sum(a) I + sum(b) -> WTA in registers
// The stages of consecutive disparities are software-pipelined with separate LDS buffers, so one
// iteration runs {S1V(d), S2V(d-1)} | barrier | {S1H(d), S2H(d-1)} | barrier: two workgroup
// barriers per d instead of four.  The guide statistics (SI = sum L, SII = sum L^2, N) come from
// S1V/S1H on AD := L (R band read as 0), once per tile.
#include "bm_common.h"
#include "bm_guided.h"

namespace sm {
namespace {

constexpr int kT = 256;   // threads per workgroup

__device__ __forceinline__ int win_count(int x, int r, int n) {
    const int lo = x - r < 0 ? 0 : x - r;
    const int hi = x + r > n - 1 ? n - 1 : x + r;
    return hi - lo + 1;
}

// 4 bytes of row y from column x (little-endian), outside the image = 0
__device__ __forceinline__ uint32_t ld4(const uint8_t* p, int y, int x, int W, int H, int pitch) {
    if (y < 0 || y >= H) return 0u;
    const uint8_t* row = p + (int64_t)y * pitch;
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

constexpr int kBandChunk = 64;   // disparities per staged right band

template <int R>
struct GeoF {
    static constexpr int TW = 64 - 4 * R;
    static constexpr int TH = 32;
    static constexpr int AW = TW + 2 * R;
    static constexpr int AH = TH + 2 * R;
    static constexpr int PH = TH + 4 * R;
    static constexpr int RPW = (AH + 3) / 4;                 // A rows per wave in S1V
    static constexpr int NV = RPW + 2 * R;                   // P rows walked per wave
    static constexpr int NSEG1 = kT / AH;                    // S1H segments per A row
    static constexpr int SW1 = (AW + NSEG1 - 1) / NSEG1;
    static constexpr int SW2 = (TW + 7) / 8;                 // S2H outputs per thread
    static constexpr int CSS0 = (NSEG1 * SW1 + 2 * R) > 64 ? (NSEG1 * SW1 + 2 * R) : 64;
    // strides kept minimal so that r <= 5 fits 3 workgroups per CU (<= 52 KB): an odd CS stride
    // spreads the S1H rows over the banks (padding mm / a/b rows for banks measured slower).
    // S2H threads whose last outputs fall past TW read beyond their mm row (the next row, or abp
    // after the last one) into values that only reach those discarded outputs.
    static constexpr int CSS = CSS0 + 1;                     // u32 per CS row
    static constexpr int MS = AW;                            // float2 per mm row
    static constexpr int ABS = AW;                           // float2 per a/b row
    static constexpr int RBW = 64 + kBandChunk;              // right band bytes per P row (one d-chunk)
    static constexpr int CS_BYTES = ((AH * CSS * 4 > PH * 64 ? AH * CSS * 4 : PH * 64) + 15) & ~15;  // lt aliases cs
    static constexpr int MM_BYTES = TH * MS * 8;
    static constexpr int AB_BYTES = AH * ABS * 8;
    static constexpr int RB_BYTES = (PH * RBW + 15) & ~15;
    static constexpr int LDS = CS_BYTES + MM_BYTES + AB_BYTES + RB_BYTES;
};

// r >= 6 needs > 168 VGPRs without spilling: 2 waves/SIMD there, 3 elsewhere
template <int R>
constexpr int kGuidedWavesPerEU = (R >= 6) ? 2 : 3;

template <int R>
__global__ __launch_bounds__(kT, (kGuidedWavesPerEU<R>)) void guided_fused_kernel(
    const uint8_t* __restrict__ Limg, const uint8_t* __restrict__ Rimg, int W, int H, int pitch, int64_t fstride,
    int D, float eps, int valid_mode, uint8_t* __restrict__ disp, int out_pitch, int64_t ostride, int tiles_x,
    int tiles) {
    using G = GeoF<R>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* cs = reinterpret_cast<uint32_t*>(smem);                                  // [AH][CSS] packed sums
    uint8_t* lt = smem;                                                                 // [PH][64] (aliases cs)
    float2* mm = reinterpret_cast<float2*>(smem + G::CS_BYTES);                        // [TH][MS]
    float2* abp = reinterpret_cast<float2*>(smem + G::CS_BYTES + G::MM_BYTES);         // [AH][ABS]
    uint8_t* rb = smem + G::CS_BYTES + G::MM_BYTES + G::AB_BYTES;                      // [PH][RBW]

    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int tile_id = xcd_tile(blockIdx.x, gridDim.x);
    const int frame = tile_id / tiles;
    const int t = tile_id - frame * tiles;
    const int ty = t / tiles_x, tx = t - ty * tiles_x;
    const int x0 = tx * G::TW, y0 = ty * G::TH;
    const int px0 = x0 - 2 * R, py0 = y0 - 2 * R;      // P region origin (image coords)
    const uint8_t* L = Limg + (int64_t)frame * fstride;
    const uint8_t* Rf = Rimg + (int64_t)frame * fstride;

    // ---- right band of d-chunk k: rb[i][j] = R(py0 + i, px0 - 64k - 64 + j), so P column c at
    //      disparity d (in chunk k) reads rb[i][c + 64 - (d & 63)] ----
    auto stage_band = [&](int k) {
        const int rbase = px0 - kBandChunk * k - kBandChunk;
        for (int e = tid; e < G::PH * (G::RBW / 4); e += kT) {
            const int i = e / (G::RBW / 4), j = e - (e / (G::RBW / 4)) * (G::RBW / 4);
            *reinterpret_cast<uint32_t*>(rb + i * G::RBW + 4 * j) = ld4(Rf, py0 + i, rbase + 4 * j, W, H, pitch);
        }
    };
    stage_band(0);
    for (int e = tid; e < G::PH * 16; e += kT) {
        const int i = e >> 4, j = e & 15;
        *reinterpret_cast<uint32_t*>(lt + i * 64 + 4 * j) = ld4(L, py0 + i, px0 + 4 * j, W, H, pitch);
    }
    __syncthreads();
    // S1V state: this wave walks P rows [a0, a0 + NV); lane = P column c
    const int a0 = wave * G::RPW;
    const int c = lane;
    const int xc = px0 + c;
    const bool col_in = xc >= 0 && xc < W;
    uint32_t lzm[G::NV];   // (L << 12) | 1: the S1V multiplier; L itself is lzm >> 12
#pragma unroll
    for (int k = 0; k < G::NV; ++k) lzm[k] = (((a0 + k < G::PH) ? (uint32_t)lt[(a0 + k) * 64 + c] : 0u) << 12) | 1u;
    __syncthreads();   // lt (aliased with cs) is consumed

    // S1H ownership: A row h1i, segment h1s (threads >= AH*NSEG1 idle in S1H)
    const bool h1_on = tid < G::AH * G::NSEG1;
    const int h1i = h1_on ? tid / G::NSEG1 : 0, h1s = h1_on ? tid % G::NSEG1 : 0;
    const int h1y = y0 - R + h1i;
    // S2V ownership: A column v2j, output rows [8*v2g, 8*v2g + 8)
    const bool v2_on = tid < 4 * G::AW;
    const int v2g = v2_on ? tid / G::AW : 0, v2j = v2_on ? tid % G::AW : 0;
    // S2H ownership: output row h2r, outputs [h2s*SW2, h2s*SW2 + SW2); rows run across lanes
    // (measured 2 % faster than segments across lanes)
    const int h2r = tid & 31, h2s = tid >> 5;
    const int oy = y0 + h2r;

    // per-A-pixel constants (filled by the stats pass) and per-output WTA state.
    // WTA runs on N*q = sum(a)*I + sum(b): N (output window count) is a positive per-pixel
    // constant, so the argmin is that of q; the Device.cu:37 seed 50 becomes 50*N (exact in fp32).
    uint32_t nN[G::SW1], nSI[G::SW1];
    float invden[G::SW1], invN[G::SW1];
    float oI[G::SW2], bq[G::SW2];
    int bdd[G::SW2];
#pragma unroll
    for (int o = 0; o < G::SW2; ++o) {
        const int x = x0 + h2s * G::SW2 + o;
        const bool ok = oy < H && x < W && h2s * G::SW2 + o < G::TW;
        oI[o] = ok ? (float)L[(int64_t)oy * pitch + x] : 0.f;
        bq[o] = valid_mode == 0 ? 50.0f * (float)(win_count(x, R, W) * win_count(oy, R, H)) : __builtin_huge_valf();
        bdd[o] = -256;
    }

    // ================= S1V: d < 0 is the guide-statistics pass (AD := L) =================
    auto s1v = [&](int d) {
        const bool m = d < 0 ? true : (col_in && xc >= d);
        const uint8_t* rc = rb + (c + kBandChunk - (d < 0 ? 0 : (d & (kBandChunk - 1))));
        uint32_t T = 0u, Tp[2 * R + 1];
#pragma unroll
        for (int k = 0; k < G::NV; ++k) {
            const int i = a0 + k;                                   // P row
            const uint32_t rv = (d < 0 || i >= G::PH) ? 0u : (uint32_t)rc[i * G::RBW];
            uint32_t ad = __builtin_amdgcn_sad_u8(lzm[k] >> 12, rv, 0u);
            ad = m ? ad : 0u;
            T = __umul24(ad, lzm[k]) + T;
            if (k >= 2 * R) {
                const uint32_t old = (k == 2 * R) ? 0u : Tp[(k - 2 * R - 1) % (2 * R + 1)];
                const int j = i - 2 * R;                            // A row
                if (j < a0 + G::RPW && j < G::AH) cs[j * G::CSS + c] = T - old;
            }
            Tp[k % (2 * R + 1)] = T;
        }
    };
    // ================= S1H =================
    auto s1h = [&](int d) {
        if (!h1_on) return;
        const uint32_t* row = cs + h1i * G::CSS + h1s * G::SW1;
        uint32_t sp = 0, sip = 0;
#pragma unroll
        for (int k = 0; k < 2 * R; ++k) {
            const uint32_t v = row[k];
            sp += v & 0xFFFu;
            sip += v >> 12;
        }
#pragma unroll
        for (int o = 0; o < G::SW1; ++o) {
            const uint32_t vin = row[o + 2 * R];
            sp += vin & 0xFFFu;
            sip += vin >> 12;
            const int j = h1s * G::SW1 + o;                         // A column
            const int x = x0 - R + j;
            const bool inimg = h1y >= 0 && h1y < H && x >= 0 && x < W && j < G::AW;
            if (d < 0) {
                // guide statistics: sp = SI, sip = SII
                const uint32_t N = inimg ? (uint32_t)(win_count(x, R, W) * win_count(h1y, R, H)) : 1u;
                const int32_t nvar = (int32_t)(N * sip - sp * sp);
                nN[o] = N;
                nSI[o] = sp;
                invden[o] = 1.0f / ((float)nvar + eps * (float)N * (float)N);
                invN[o] = inimg ? 1.0f / (float)N : 0.f;
            } else if (j < G::AW) {
                const int32_t num = (int32_t)(nN[o] * sip - nSI[o] * sp);
                const float a = (float)num * invden[o];
                const float b = ((float)sp - a * (float)nSI[o]) * invN[o];
                abp[h1i * G::ABS + j] = inimg ? make_float2(a, b) : make_float2(0.f, 0.f);
            }
            const uint32_t vout = row[o];
            sp -= vout & 0xFFFu;
            sip -= vout >> 12;
        }
    };
    // ================= S2V =================
    auto s2v = [&]() {
        if (!v2_on) return;
        const float2* col = abp + v2j;
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int k = 0; k < 2 * R; ++k) {
            const float2 v = col[(8 * v2g + k) * G::ABS];
            sa += v.x;
            sb += v.y;
        }
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const float2 vin = col[(8 * v2g + r + 2 * R) * G::ABS];
            sa += vin.x;
            sb += vin.y;
            mm[(8 * v2g + r) * G::MS + v2j] = make_float2(sa, sb);
            const float2 vout = col[(8 * v2g + r) * G::ABS];
            sa -= vout.x;
            sb -= vout.y;
        }
    };
    // ================= S2H + WTA =================
    auto s2h = [&](int d) {
        const float2* row = mm + h2r * G::MS + h2s * G::SW2;
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int k = 0; k < 2 * R; ++k) {
            const float2 v = row[k];
            sa += v.x;
            sb += v.y;
        }
#pragma unroll
        for (int o = 0; o < G::SW2; ++o) {
            const float2 vin = row[o + 2 * R];
            sa += vin.x;
            sb += vin.y;
            const float q = sa * oI[o] + sb;
            const int x = x0 + h2s * G::SW2 + o;
            const int lim = valid_mode == 0 ? (W - x) : x;
            if (d <= lim && q < bq[o]) {
                bq[o] = q;
                bdd[o] = d;
            }
            const float2 vout = row[o];
            sa -= vout.x;
            sb -= vout.y;
        }
    };

    s1v(-1);
    __syncthreads();
    s1h(-1);
    __syncthreads();
    // buffers: cs (S1V -> S1H), abp (S1H -> S2V), mm (S2V -> S2H); each producer of iteration d+1
    // runs after the barrier that ends the consumer of iteration d.  The right band (read only by
    // S1V) is restaged for the next d-chunk in the second phase of the chunk's last iteration.
    for (int d = 0; d <= D; ++d) {
        if (d < D) s1v(d);
        if (d > 0) s2v();
        __syncthreads();
        if (d + 1 < D && ((d + 1) & (kBandChunk - 1)) == 0) stage_band((d + 1) / kBandChunk);
        if (d < D) s1h(d);
        if (d > 0) s2h(d - 1);
        __syncthreads();
    }
    uint8_t* Df = disp + (int64_t)frame * ostride;
#pragma unroll
    for (int o = 0; o < G::SW2; ++o) {
        const int x = x0 + h2s * G::SW2 + o;
        if (oy < H && x < W && h2s * G::SW2 + o < G::TW)
            Df[(int64_t)oy * out_pitch + x] = (uint8_t)(bdd[o] & 0xFF);   // (uchar)dm, Device.cu:63
    }
}

template <int R>
hipError_t run_fused(const uint8_t* L, const uint8_t* Rimg, int W, int H, int pitch, int64_t fstride, int batch,
                     int D, float eps, int valid_mode, uint8_t* disp, int out_pitch, int64_t ostride, hipStream_t s) {
    using G = GeoF<R>;
    const int tiles_x = (W + G::TW - 1) / G::TW, tiles_y = (H + G::TH - 1) / G::TH;
    const int64_t blocks = (int64_t)tiles_x * tiles_y * batch;
    if (blocks <= 0 || blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    hipLaunchKernelGGL((guided_fused_kernel<R>), dim3((unsigned)blocks), dim3(kT), (size_t)G::LDS, s, L, Rimg, W,
                       H, pitch, fstride, D, eps, valid_mode, disp, out_pitch, ostride, tiles_x, tiles_x * tiles_y);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_guided_match(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int batch,
                               int64_t frame_stride, int radius, int D, float eps, int valid_mode, uint8_t* disp,
                               int out_pitch, int64_t out_frame_stride, hipStream_t s) {
    if (D < 1 || D > kMaxDisp) return hipErrorInvalidValue;
#define SM_GUIDED_CASE(r) \
    case r: return run_fused<r>(L, R, W, H, pitch, frame_stride, batch, D, eps, valid_mode, disp, out_pitch, out_frame_stride, s)
    switch (radius) {
        SM_GUIDED_CASE(0);
        SM_GUIDED_CASE(1);
        SM_GUIDED_CASE(2);
        SM_GUIDED_CASE(3);
        SM_GUIDED_CASE(4);
        SM_GUIDED_CASE(5);
        SM_GUIDED_CASE(6);
        SM_GUIDED_CASE(7);
        default: return hipErrorInvalidValue;
    }
#undef SM_GUIDED_CASE
}

}  // namespace sm
