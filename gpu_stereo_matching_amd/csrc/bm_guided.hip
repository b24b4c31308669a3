// bm_guided.hip — guided-filter cost aggregation + WTA.
//
// The reference has no guided filter; this build defines it and
// the fp64 restatement oracle/bm_oracle.c:ora_guided_disp is its checker:
//   guide I = L, cost p_d = AD_d (0 for x < d, as Device.cu:27-31), f = clipped-window mean,
//   a = (f(Ip) - f(I) f(p)) / (f(II) - f(I)^2 + eps),  b = f(p) - a f(I),  q = f(a) I + f(b),
//   WTA: first d with the smallest q below 50 (= 50*win^2 / win^2, Device.cu:37), valid d <= W-x.
//
// Three kernels per frame:
//   guided_stats  (once):        per pixel SI = sum L, N = window count, invden = 1/(N*SII - SI^2 + eps N^2)
//   guided_ab     (per d-chunk): exact integer window sums Sp = sum AD, SIp = sum L*AD (packed into one
//                                u32 column sum, Vp + VIp*4096), then
//                                a = (N*SIp - SI*Sp) * invden   (numerator exact: u32 wrap, |N^2 cov| < 2^31)
//                                b = (Sp - a*SI) / N
//   guided_wta    (per d-chunk): q = f(a)*I + f(b) with direct window sums, running best per pixel.
#include <cstdlib>

#include "bm_common.h"
#include "bm_guided.h"

namespace sm {
namespace {

constexpr int kT = 256;        // threads per workgroup
constexpr int kGTW = 64;       // stats / wta tile width (columns)
constexpr int kGTH = 16;       // stats / wta tile height (rows)

__device__ __forceinline__ int win_count(int x, int r, int n) {
    const int lo = x - r < 0 ? 0 : x - r;
    const int hi = x + r > n - 1 ? n - 1 : x + r;
    return hi - lo + 1;
}

// ----------------------------------------------------------------------------------------
// guided_stats: st[0][p] = SI (as float bits of int), st[1][p] = invden, st[2][p] = 1/N
// Direct window sums from an LDS tile (once per frame; cheap).
// ----------------------------------------------------------------------------------------
template <int R>
__global__ __launch_bounds__(kT) void guided_stats_kernel(const uint8_t* __restrict__ L, int W, int H, int pitch,
                                                          float eps, float* __restrict__ st) {
    __shared__ uint32_t tile[kGTH + 2 * R][kGTW + 2 * R];
    __shared__ uint32_t vs[kGTH][kGTW + 2 * R];
    __shared__ uint32_t vss[kGTH][kGTW + 2 * R];
    const int x0 = blockIdx.x * kGTW, y0 = blockIdx.y * kGTH;
    for (int e = threadIdx.x; e < (kGTH + 2 * R) * (kGTW + 2 * R); e += kT) {
        const int i = e / (kGTW + 2 * R), j = e % (kGTW + 2 * R);
        const int y = y0 - R + i, x = x0 - R + j;
        tile[i][j] = (y >= 0 && y < H && x >= 0 && x < W) ? L[(int64_t)y * pitch + x] : 0u;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < kGTH * (kGTW + 2 * R); e += kT) {
        const int i = e / (kGTW + 2 * R), j = e % (kGTW + 2 * R);
        uint32_t s = 0, ss = 0;
#pragma unroll
        for (int k = 0; k <= 2 * R; ++k) {
            const uint32_t v = tile[i + k][j];
            s += v;
            ss += v * v;
        }
        vs[i][j] = s;
        vss[i][j] = ss;
    }
    __syncthreads();
    const int64_t P = (int64_t)W * H;
    for (int e = threadIdx.x; e < kGTH * kGTW; e += kT) {
        const int i = e / kGTW, j = e % kGTW;
        const int y = y0 + i, x = x0 + j;
        if (y >= H || x >= W) continue;
        uint32_t s = 0, ss = 0;
#pragma unroll
        for (int k = 0; k <= 2 * R; ++k) {
            s += vs[i][j + k];
            ss += vss[i][j + k];
        }
        const uint32_t N = (uint32_t)(win_count(x, R, W) * win_count(y, R, H));
        const int32_t nvar = (int32_t)(N * ss - s * s);            // N^2 var, exact (wraps cancel)
        const float den = (float)nvar + eps * (float)N * (float)N;
        const int64_t p = (int64_t)y * W + x;
        st[p] = __int_as_float((int)s);
        st[P + p] = 1.0f / den;
        st[2 * P + p] = 1.0f / (float)N;
    }
}

// ----------------------------------------------------------------------------------------
// guided_ab: a, b for d in [d0, d0 + nd) over the whole frame.  Tile: 64 CS columns (lanes)
// x 32 rows, TW = 64 - 2R outputs; wave w handles d = d0 + w, d0 + w + 4, ...
// ----------------------------------------------------------------------------------------
constexpr int kABRows = 32;

template <int R>
struct GeoAB {
    static constexpr int TW = 64 - 2 * R;
    static constexpr int ROWS = kABRows + 2 * R;
    static constexpr int NOUT = (TW + 1) / 2;                   // outputs per phase-H thread
    static constexpr int CSS = 68 > (NOUT * 2 + 2 * R + 1) ? 68 : ((NOUT * 2 + 2 * R + 1 + 7) & ~7) + 4;
    static constexpr int RBW = 64 + 64 + 8;                     // right band bytes per row (d chunk <= 64)
};

// a/b planes are stored tile-blocked so that each phase-H lane's run of outputs is contiguous
// and 16-B aligned: plane[d][tile][row(32)][half(2)][32 floats]  (8 KB per tile per plane).
constexpr int kABTile = kABRows * 64;

template <int R>
__device__ __forceinline__ int64_t ab_index(int y, int x, int tiles_x) {
    using G = GeoAB<R>;
    const int ty = y / kABRows, tx = x / G::TW;
    const int xi = x - tx * G::TW;
    const int half = xi / G::NOUT, xo = xi - half * G::NOUT;
    return ((int64_t)(ty * tiles_x + tx) * kABTile) + (y - ty * kABRows) * 64 + half * 32 + xo;
}

template <int R>
__global__ __launch_bounds__(kT, 2) void guided_ab_kernel(const uint8_t* __restrict__ L, const uint8_t* __restrict__ Rimg,
                                                          int W, int H, int pitch, int d0, int nd,
                                                          const float* __restrict__ st, float* __restrict__ ab,
                                                          int tiles_x, int tiles_y) {
    using G = GeoAB<R>;
    __shared__ uint8_t rband[G::ROWS][G::RBW];
    __shared__ uint32_t csp[4][kABRows][G::CSS];
    __shared__ uint4 pix[kABRows][G::TW];

    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int x0 = tx * G::TW, y0 = ty * kABRows;
    const int64_t P = (int64_t)W * H;
    // right band: columns [x0 - R - d0 - 63, x0 - R + 64)  (nd <= 64)
    const int rbase = x0 - R - d0 - 64;
    for (int e = tid; e < G::ROWS * G::RBW; e += kT) {
        const int i = e / G::RBW, k = e % G::RBW;
        const int y = y0 - R + i, x = rbase + k;
        rband[i][k] = (y >= 0 && y < H && x >= 0 && x < W) ? Rimg[(int64_t)y * pitch + x] : (uint8_t)0;
    }
    const int c = x0 - R + lane;
    const bool col_in = c >= 0 && c < W;
    uint32_t lz[G::ROWS];
#pragma unroll
    for (int i = 0; i < G::ROWS; ++i) {
        const int y = y0 - R + i;
        lz[i] = (col_in && y >= 0 && y < H) ? L[(int64_t)y * pitch + c] : 0u;
    }
    // phase-H ownership: row hj, half hh -> outputs [hh*NOUT, hh*NOUT + NOUT)
    const int hj = lane & 31, hh = lane >> 5, obase = hh * G::NOUT;
    // per-pixel d-independent constants in LDS: {N, SI, 1/(N^2 var + eps N^2), 1/N}
    for (int e = tid; e < kABRows * G::TW; e += kT) {
        const int i = e / G::TW, j = e % G::TW;
        const int y = y0 + i, x = x0 + j;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (y < H && x < W) {
            const int64_t p = (int64_t)y * W + x;
            const uint32_t si = (uint32_t)__float_as_int(st[p]);
            const float in = st[2 * P + p];
            v = make_uint4((uint32_t)(win_count(x, R, W) * win_count(y, R, H)), si, __float_as_uint(st[P + p]),
                           __float_as_uint(in));
        }
        pix[i][j] = v;
    }
    __syncthreads();

    for (int dd = wave; dd < nd; dd += 4) {
        const int d = d0 + dd;
        // ---- phase V: packed prefix of AD * (1 + 4096 L) ----
        const bool m = col_in && (c >= d);
        const uint8_t* rc = &rband[0][0] + (c - d - rbase);
        uint32_t T = 0u, Tp[2 * R + 1];
#pragma unroll
        for (int i = 0; i < G::ROWS; ++i) {
            const uint32_t rv = rc[i * G::RBW];
            uint32_t ad = __builtin_amdgcn_sad_u8(lz[i], rv, 0u);
            ad = m ? ad : 0u;
            T += __umul24(ad, (lz[i] << 12) | 1u);
            if (i >= 2 * R) {
                const uint32_t old = (i == 2 * R) ? 0u : Tp[(i - 2 * R - 1) % (2 * R + 1)];
                csp[wave][i - 2 * R][lane] = T - old;
            }
            Tp[i % (2 * R + 1)] = T;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // ---- phase H: running sums of Vp (12 bits) and VIp (>> 12) along the row ----
        {
            const uint32_t* row = &csp[wave][hj][obase];
            uint32_t sp = 0, sip = 0;
#pragma unroll
            for (int k = 0; k < 2 * R; ++k) {
                const uint32_t v = row[k];
                sp += v & 0xFFFu;
                sip += v >> 12;
            }
            const int64_t plane = (int64_t)tiles_x * tiles_y * kABTile;
            float* ap = ab + (int64_t)(2 * dd) * plane + (int64_t)blockIdx.x * kABTile + hj * 64 + hh * 32;
            float* bp = ab + (int64_t)(2 * dd + 1) * plane + (int64_t)blockIdx.x * kABTile + hj * 64 + hh * 32;
            float av[(G::NOUT + 3) & ~3], bv[(G::NOUT + 3) & ~3];
#pragma unroll
            for (int o = 0; o < G::NOUT; ++o) {
                const uint32_t vin = row[o + 2 * R];
                sp += vin & 0xFFFu;
                sip += vin >> 12;
                // a = (N*SIp - SI*Sp) / (N*SII - SI^2 + eps N^2): numerator exact mod 2^32, |.| < 2^31
                const uint4 pc = pix[hj][obase + o < G::TW ? obase + o : 0];
                const int32_t num = (int32_t)(pc.x * sip - pc.y * sp);
                const float a = (float)num * __uint_as_float(pc.z);
                av[o] = a;
                bv[o] = ((float)sp - a * (float)pc.y) * __uint_as_float(pc.w);   // (Sp - a SI) / N
                const uint32_t vout = row[o];
                sp -= vout & 0xFFFu;
                sip -= vout >> 12;
            }
#pragma unroll
            for (int o = G::NOUT; o < ((G::NOUT + 3) & ~3); ++o) av[o] = bv[o] = 0.f;
#pragma unroll
            for (int q = 0; q < ((G::NOUT + 3) & ~3) / 4; ++q) {
                *reinterpret_cast<float4*>(ap + 4 * q) = make_float4(av[4 * q], av[4 * q + 1], av[4 * q + 2], av[4 * q + 3]);
                *reinterpret_cast<float4*>(bp + 4 * q) = make_float4(bv[4 * q], bv[4 * q + 1], bv[4 * q + 2], bv[4 * q + 3]);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// ----------------------------------------------------------------------------------------
// guided_wta: q = f(a) I + f(b) for d in [d0, d0+nd); update best (float) and bd (int) per pixel.
// Tile 64 x 16; separable direct window sums (exact order, no running-sum drift).
// ----------------------------------------------------------------------------------------
template <int R>
__global__ __launch_bounds__(kT) void guided_wta_kernel(const uint8_t* __restrict__ L, int W, int H, int pitch,
                                                        int d0, int nd, const float* __restrict__ ab,
                                                        const float* __restrict__ st, int valid_mode,
                                                        float* __restrict__ best, int* __restrict__ bd,
                                                        int ab_tiles_x, int ab_tiles_y) {
    __shared__ float ta[kGTH + 2 * R][kGTW + 2 * R + 1];
    __shared__ float tb[kGTH + 2 * R][kGTW + 2 * R + 1];
    __shared__ float va[kGTH][kGTW + 2 * R + 1];
    __shared__ float vb[kGTH][kGTW + 2 * R + 1];
    const int x0 = blockIdx.x * kGTW, y0 = blockIdx.y * kGTH;
    const int64_t P = (int64_t)W * H;
    constexpr int NPT = kGTH * kGTW / kT;   // pixels per thread (4)
    float bq[NPT];
    int bdd[NPT];
    float lI[NPT], iN[NPT];
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const int e = threadIdx.x + k * kT;
        const int i = e / kGTW, j = e % kGTW;
        const int y = y0 + i, x = x0 + j;
        const bool ok = y < H && x < W;
        const int64_t p = ok ? (int64_t)y * W + x : 0;
        bq[k] = ok ? best[p] : 0.f;
        bdd[k] = ok ? bd[p] : 0;
        lI[k] = ok ? (float)L[(int64_t)y * pitch + x] : 0.f;
        iN[k] = ok ? st[2 * P + p] : 0.f;
    }
    for (int dd = 0; dd < nd; ++dd) {
        const int d = d0 + dd;
        const int64_t plane = (int64_t)ab_tiles_x * ab_tiles_y * kABTile;
        const float* ap = ab + (int64_t)(2 * dd) * plane;
        const float* bp = ab + (int64_t)(2 * dd + 1) * plane;
        __syncthreads();
        for (int e = threadIdx.x; e < (kGTH + 2 * R) * (kGTW + 2 * R); e += kT) {
            const int i = e / (kGTW + 2 * R), j = e % (kGTW + 2 * R);
            const int y = y0 - R + i, x = x0 - R + j;
            const bool ok = y >= 0 && y < H && x >= 0 && x < W;
            const int64_t p = ok ? ab_index<R>(y, x, ab_tiles_x) : 0;
            ta[i][j] = ok ? ap[p] : 0.f;
            tb[i][j] = ok ? bp[p] : 0.f;
        }
        __syncthreads();
        for (int e = threadIdx.x; e < kGTH * (kGTW + 2 * R); e += kT) {
            const int i = e / (kGTW + 2 * R), j = e % (kGTW + 2 * R);
            float sa = 0.f, sb = 0.f;
#pragma unroll
            for (int k = 0; k <= 2 * R; ++k) {
                sa += ta[i + k][j];
                sb += tb[i + k][j];
            }
            va[i][j] = sa;
            vb[i][j] = sb;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
            const int e = threadIdx.x + k * kT;
            const int i = e / kGTW, j = e % kGTW;
            const int x = x0 + j;
            float sa = 0.f, sb = 0.f;
#pragma unroll
            for (int t = 0; t <= 2 * R; ++t) {
                sa += va[i][j + t];
                sb += vb[i][j + t];
            }
            const float q = (sa * iN[k]) * lI[k] + sb * iN[k];
            const int lim = valid_mode == 0 ? (W - x) : x;
            if (d <= lim && q < bq[k]) {
                bq[k] = q;
                bdd[k] = d;
            }
        }
    }
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
        const int e = threadIdx.x + k * kT;
        const int i = e / kGTW, j = e % kGTW;
        const int y = y0 + i, x = x0 + j;
        if (y < H && x < W) {
            const int64_t p = (int64_t)y * W + x;
            best[p] = bq[k];
            bd[p] = bdd[k];
        }
    }
}

// ----------------------------------------------------------------------------------------
// guided_fused: the whole guided pipeline for one output tile, every d, inside LDS.
//   P region (cost sums)   : 64 columns (one per lane) x (TH + 4R) rows, image cols x0-2R ..
//   A region (a, b)        : (TW + 2R) x (TH + 2R), image (x0-R, y0-R) ..
//   output tile            : TW = 64 - 4R  x  TH = 32
// Per d (4 block barriers):
//   S1V  lane = P column; waves split the A rows: packed prefix T += AD*(1 + 4096 L) -> CS rows
//   S1H  thread = (A row, segment): running Sp / SIp -> a, b  (exact integer numerators)
//   S2V  thread = (A column, 8-row group): running float sums of a, b over 2R+1 rows
//   S2H  thread = (output row, segment): running sums -> q = f(a) I + f(b) -> WTA in registers
// The guide statistics (SI = sum L, SII = sum L^2) come from the same S1V/S1H with R := 0
// (AD = L, L*AD = L^2), once per tile.
// ----------------------------------------------------------------------------------------
template <int R>
struct GeoF {
    static constexpr int TW = 64 - 4 * R;
    static constexpr int TH = 32;
    static constexpr int AW = TW + 2 * R;
    static constexpr int AH = TH + 2 * R;
    static constexpr int PH = TH + 4 * R;
    static constexpr int RPW = (AH + 3) / 4;                 // A rows per wave in S1V
    static constexpr int NV = RPW + 2 * R;                   // P rows walked per wave
    static constexpr int NSEG1 = 256 / AH;                   // S1H segments per A row
    static constexpr int SW1 = (AW + NSEG1 - 1) / NSEG1;
    static constexpr int SW2 = (TW + 7) / 8;                 // S2H outputs per thread
    static constexpr int CSS = ((NSEG1 * SW1 + 2 * R) > 64 ? (NSEG1 * SW1 + 2 * R) : 64) + 4;
    static constexpr int MS = ((8 * SW2 + 2 * R) > AW ? (8 * SW2 + 2 * R) : AW) + 1;
    static constexpr int ABS = AW + 1;
    static constexpr int RBW = 64 + 256 + 8;                 // right band bytes per P row (D <= 256)
    static constexpr int CSM = (AH * CSS * 4 > TH * MS * 8 ? AH * CSS * 4 : TH * MS * 8);
    static constexpr int LT = PH * 64;                       // staged left tile bytes (aliases CSM)
    static constexpr int CSM_BYTES = ((CSM > LT ? CSM : LT) + 15) & ~15;
    static constexpr int AB_BYTES = AH * ABS * 8;
    static constexpr int RB_BYTES = (PH * RBW + 15) & ~15;
    static constexpr int LDS = CSM_BYTES + AB_BYTES + RB_BYTES;
};

template <int R>
__global__ __launch_bounds__(kT, ((R == 3 || R == 7) ? 2 : 3)) void guided_fused_kernel(const uint8_t* __restrict__ L, const uint8_t* __restrict__ Rimg,
                                                             int W, int H, int pitch, int D, float eps, int valid_mode,
                                                             uint8_t* __restrict__ disp, int out_pitch, int tiles_x) {
    using G = GeoF<R>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* cs = reinterpret_cast<uint32_t*>(smem);                           // [AH][CSS] packed sums
    float2* mm = reinterpret_cast<float2*>(smem);                               // [TH][MS]  (aliases cs)
    uint8_t* lt = smem;                                                          // [PH][64]  (aliases cs)
    float2* abp = reinterpret_cast<float2*>(smem + G::CSM_BYTES);               // [AH][ABS]
    uint8_t* rb = smem + G::CSM_BYTES + G::AB_BYTES;                             // [PH][RBW]

    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int x0 = tx * G::TW, y0 = ty * G::TH;
    const int px0 = x0 - 2 * R, py0 = y0 - 2 * R;      // P region origin (image coords)
    const int rbase = px0 - 256;                      // image column of rb[.][0]

    // ---- stage right band (all d) and left P tile ----
    for (int e = tid; e < G::PH * (G::RBW / 4); e += kT) {
        const int i = e / (G::RBW / 4), j = e % (G::RBW / 4);
        const int y = py0 + i;
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int x = rbase + 4 * j + b;
            if (y >= 0 && y < H && x >= 0 && x < W) v |= (uint32_t)Rimg[(int64_t)y * pitch + x] << (8 * b);
        }
        *reinterpret_cast<uint32_t*>(rb + i * G::RBW + 4 * j) = v;
    }
    for (int e = tid; e < G::PH * 16; e += kT) {
        const int i = e / 16, j = e % 16;
        const int y = py0 + i;
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int x = px0 + 4 * j + b;
            if (y >= 0 && y < H && x >= 0 && x < W) v |= (uint32_t)L[(int64_t)y * pitch + x] << (8 * b);
        }
        *reinterpret_cast<uint32_t*>(lt + i * 64 + 4 * j) = v;
    }
    __syncthreads();
    // S1V state: this wave walks P rows [a0, a0 + NV); lane = P column c
    const int a0 = wave * G::RPW;
    const int c = lane;
    const int xc = px0 + c;
    const bool col_in = xc >= 0 && xc < W;
    uint32_t lzm[G::NV];   // (L << 12) | 1: the S1V multiplier; L itself is lzm >> 12
#pragma unroll
    for (int t = 0; t < G::NV; ++t) lzm[t] = (((a0 + t < G::PH) ? (uint32_t)lt[(a0 + t) * 64 + c] : 0u) << 12) | 1u;
    __syncthreads();   // lt (aliased with cs) is consumed

    // S1H ownership: A row h1i, segment h1s (threads >= AH*NSEG1 idle in S1H)
    const bool h1_on = tid < G::AH * G::NSEG1;
    const int h1i = h1_on ? tid / G::NSEG1 : 0, h1s = h1_on ? tid % G::NSEG1 : 0;
    const int h1y = y0 - R + h1i;
    // S2V ownership: A column v2j, output rows [8*v2g, 8*v2g + 8)
    const bool v2_on = tid < 4 * G::AW;
    const int v2g = v2_on ? tid / G::AW : 0, v2j = v2_on ? tid % G::AW : 0;
    // S2H ownership: output row h2r, outputs [h2s*SW2, h2s*SW2 + SW2)
    const int h2r = tid >> 3, h2s = tid & 7;
    const int oy = y0 + h2r;

    // per-A-pixel constants (filled by the stats pass) and per-output WTA state
    uint32_t nN[G::SW1], nSI[G::SW1];
    float invden[G::SW1], invN[G::SW1];
    // WTA on N*q = sum(a)*I + sum(b) (N = output window count > 0 is constant per pixel, so the
    // argmin is that of q); the Device.cu:37 seed 50 becomes 50*N (exact in fp32)
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

    for (int d = -1; d < D; ++d) {              // d = -1: guide statistics pass
        // ================= S1V =================
        {
            const bool m = d < 0 ? true : (col_in && xc >= d);
            const uint8_t* rc = rb + (c - (d < 0 ? 0 : d) + 256);
            uint32_t T = 0u, Tp[2 * R + 1];
#pragma unroll
            for (int t = 0; t < G::NV; ++t) {
                const int i = a0 + t;                                   // P row
                const uint32_t rv = (d < 0 || i >= G::PH) ? 0u : (uint32_t)rc[i * G::RBW];
                uint32_t ad = __builtin_amdgcn_sad_u8(lzm[t] >> 12, rv, 0u);
                ad = m ? ad : 0u;
                T = __umul24(ad, lzm[t]) + T;
                if (t >= 2 * R) {
                    const uint32_t old = (t == 2 * R) ? 0u : Tp[(t - 2 * R - 1) % (2 * R + 1)];
                    const int j = i - 2 * R;                            // A row
                    if (j < a0 + G::RPW && j < G::AH) cs[j * G::CSS + c] = T - old;
                }
                Tp[t % (2 * R + 1)] = T;
            }
        }
        __syncthreads();
        // ================= S1H =================
        if (h1_on) {
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
        }
        if (d < 0) {
            __syncthreads();
            continue;
        }
        __syncthreads();
        // ================= S2V =================
        if (v2_on) {
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
        }
        __syncthreads();
        // ================= S2H + WTA =================
        {
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
        }
        __syncthreads();
    }
#pragma unroll
    for (int o = 0; o < G::SW2; ++o) {
        const int x = x0 + h2s * G::SW2 + o;
        if (oy < H && x < W && h2s * G::SW2 + o < G::TW)
            disp[(int64_t)oy * out_pitch + x] = (uint8_t)(bdd[o] & 0xFF);   // (uchar)dm, Device.cu:63
    }
}

__global__ __launch_bounds__(256) void guided_init_kernel(float* best, int* bd, int64_t P, float seed) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < P) {
        best[i] = seed;
        bd[i] = -256;
    }
}

__global__ __launch_bounds__(256) void guided_final_kernel(const int* bd, int W, int H, uint8_t* disp, int out_pitch) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
    if (x < W) disp[(int64_t)y * out_pitch + x] = (uint8_t)(bd[(int64_t)y * W + x] & 0xFF);  // (uchar)dm, Device.cu:63
}

template <int R>
hipError_t run_r(GuidedWorkspace& ws, const uint8_t* L, const uint8_t* Rimg, int W, int H, int pitch, int D,
                 float eps, int valid_mode, uint8_t* disp, int out_pitch, hipStream_t s) {
    const int64_t P = (int64_t)W * H;
    float* st = ws.stats;
    float* best = ws.stats + 3 * P;
    int* bd = reinterpret_cast<int*>(ws.stats + 4 * P);
    float* ab = ws.stats + 5 * P;
    hipLaunchKernelGGL((guided_stats_kernel<R>), dim3((W + kGTW - 1) / kGTW, (H + kGTH - 1) / kGTH), dim3(kT), 0, s,
                       L, W, H, pitch, eps, st);
    hipLaunchKernelGGL(guided_init_kernel, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, s, best, bd, P,
                       valid_mode == 0 ? 50.0f : __builtin_huge_valf());
    using G = GeoAB<R>;
    const int tiles_x = (W + G::TW - 1) / G::TW, tiles_y = (H + kABRows - 1) / kABRows;
    for (int d0 = 0; d0 < D; d0 += GuidedWorkspace::kChunk) {
        const int nd = D - d0 < GuidedWorkspace::kChunk ? D - d0 : GuidedWorkspace::kChunk;
        hipLaunchKernelGGL((guided_ab_kernel<R>), dim3(tiles_x * tiles_y), dim3(kT), 0, s, L, Rimg, W, H, pitch, d0,
                           nd, st, ab, tiles_x, tiles_y);
        hipLaunchKernelGGL((guided_wta_kernel<R>), dim3((W + kGTW - 1) / kGTW, (H + kGTH - 1) / kGTH), dim3(kT), 0,
                           s, L, W, H, pitch, d0, nd, ab, st, valid_mode, best, bd, tiles_x, tiles_y);
    }
    hipLaunchKernelGGL(guided_final_kernel, dim3((W + 255) / 256, H), dim3(256), 0, s, bd, W, H, disp, out_pitch);
    return hipGetLastError();
}

template <int R>
hipError_t run_fused(const uint8_t* L, const uint8_t* Rimg, int W, int H, int pitch, int D, float eps, int valid_mode,
                     uint8_t* disp, int out_pitch, hipStream_t s) {
    using G = GeoF<R>;
    const int tiles_x = (W + G::TW - 1) / G::TW, tiles_y = (H + G::TH - 1) / G::TH;
    hipLaunchKernelGGL((guided_fused_kernel<R>), dim3(tiles_x * tiles_y), dim3(kT), (size_t)G::LDS, s, L, Rimg, W, H,
                       pitch, D, eps, valid_mode, disp, out_pitch, tiles_x);
    return hipGetLastError();
}

}  // namespace

void guided_workspace_free(GuidedWorkspace& ws) {
    if (ws.stats) (void)hipFree(ws.stats);
    ws.stats = nullptr;
    ws.stats_bytes = 0;
}

hipError_t launch_guided_match(GuidedWorkspace& ws, const uint8_t* L, const uint8_t* R, int W, int H, int pitch,
                               int batch, int64_t frame_stride, int radius, int D, float eps, int valid_mode,
                               uint8_t* disp, int out_pitch, int64_t out_frame_stride, hipStream_t s) {
    if (radius < 0 || radius > kMaxFastRadius) return hipErrorInvalidValue;
    if (D > 256) return hipErrorInvalidValue;
    const int64_t P = (int64_t)W * H;
    const int64_t tiles = (int64_t)((W + 64 - 2 * radius - 1) / (64 - 2 * radius)) * ((H + kABRows - 1) / kABRows);
    const int64_t plane = tiles * kABTile;
    const size_t need = (size_t)(5 * P + 2 * GuidedWorkspace::kChunk * plane) * sizeof(float);
    if (ws.stats_bytes < need) {
        guided_workspace_free(ws);
        hipError_t e = hipMalloc(&ws.stats, need);
        if (e != hipSuccess) return e;
        ws.stats_bytes = need;
    }
    static const bool use_fused = [] { const char* e = std::getenv("SM_GUIDED_UNFUSED"); return !(e && e[0] == '1'); }();
    for (int f = 0; f < batch; ++f) {
        const uint8_t* Lf = L + (int64_t)f * frame_stride;
        const uint8_t* Rf = R + (int64_t)f * frame_stride;
        uint8_t* Df = disp + (int64_t)f * out_frame_stride;
        hipError_t e;
        if (use_fused) {
            switch (radius) {
                case 0: e = run_fused<0>(Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
                case 1: e = run_fused<1>(Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
                case 2: e = run_fused<2>(Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
                case 3: e = run_fused<3>(Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
                case 4: e = run_fused<4>(Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
                case 5: e = run_fused<5>(Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
                case 6: e = run_fused<6>(Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
                default: e = run_fused<7>(Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
            }
            if (e != hipSuccess) return e;
            continue;
        }
        switch (radius) {
            case 0: e = run_r<0>(ws, Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
            case 1: e = run_r<1>(ws, Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
            case 2: e = run_r<2>(ws, Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
            case 3: e = run_r<3>(ws, Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
            case 4: e = run_r<4>(ws, Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
            case 5: e = run_r<5>(ws, Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
            case 6: e = run_r<6>(ws, Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
            default: e = run_r<7>(ws, Lf, Rf, W, H, pitch, D, eps, valid_mode, Df, out_pitch, s); break;
        }
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace sm
