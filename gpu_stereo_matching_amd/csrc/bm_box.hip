// bm_box.hip — fused AD + box-window SAD + winner-take-all for gfx950 (CDNA4).
//
// Replaces the reference's two-kernel pipeline
//   kernalPreCal_V2  (BlockMatching/Device.cu:19-32)   AD volume, P*D bytes to HBM
//   kernalFindCorr   (BlockMatching/Device.cu:34-64)   win^2 byte loads per (pixel, d) + WTA
// with one kernel that never materialises the AD or SAD volume: per tile the right-image
// scanline band (block + d_max wide) sits in LDS, vertical window sums run down each column
// in registers, horizontal window sums run along rows from an LDS hand-off, and the
// (SAD << 8 | d) argmin is kept per pixel in VGPRs.  Semantics (bit-exact with getDisp,
// BlockMatching.cpp:111-189):
//   AD_d(y,c)  = |L(y,c) - R(y,c-d)| for c >= d, else 0            (Device.cu:27-31, :194)
//   S_d(y,x)   = sum of AD_d over the (2r+1)^2 window clipped to the image (Device.cu:46-56)
//   valid      = d <= W - x   (the `col + d > cols` break, Device.cu:44)
//   WTA        = first d with the smallest S_d below 50*win^2, else 0  (Device.cu:37-38,57,63)
//
// Tile geometry (R = radius, compile-time for R <= 7):
//   64 CS columns (one per lane) -> TW = 64 - 2R output columns, TH = 32 output rows.
//   A chunk of 8 disparities = 4 pairs; wave w owns pair w in both phases.
//   Phase V (lane = column): T += |L - R_d| in the low u16 and |L - R_{d+1}| in the high u16
//     (v_sad_u8 / v_sad_hi_u8); CS = T_i - T_{i-2R-1} (column window sums, two d per dword).
//   Phase H (lane = row x half-row): running window sum along x over the packed pairs, keys
//     (S << 8 | d) built with v_perm_b32, folded with v_min3_u32.
#include "bm_common.h"

namespace sm {
namespace {

constexpr int kThreads = 256;
constexpr int kTileH = 32;
constexpr int kPairs = 4;
constexpr int kChunk = 2 * kPairs;
constexpr int kCols = 64;

template <int R, int DMAX>
struct Geo {
    static constexpr int TW = kCols - 2 * R;                  // output columns per tile
    static constexpr int ROWS = kTileH + 2 * R;                 // input rows per tile
    static constexpr int HALF = kTileH / 2;                     // rows per CS hand-off
    static constexpr int NLQ = (ROWS + 3) / 4;                  // packed-L dwords per lane
    static constexpr int NQ = (((TW + 3) / 4) + 1) & ~1;        // outputs per phase-H thread (even: b64 reads)
    static constexpr int NCS2 = (NQ + 2 * R + 1) / 2;           // 8-B CS reads per phase-H thread
    static constexpr int NEED = 3 * NQ + 2 * NCS2;              // last CS column read + 1
    // row stride in dwords == 4 (mod 64): the 32 lanes of a ds_read_b64 group (16 rows x 2
    // quarters, quarter offsets NQ apart with NQ == 2 mod 4) start on 32 distinct even banks
    static constexpr int CSS = ((NEED - 4 + 63) / 64) * 64 + 4;
    static constexpr int CS_BYTES = 4 * HALF * CSS * 4;         // 4 waves x one half-tile plane
    static constexpr int RW = kCols + DMAX + 4;                 // u16 entries per right-band row (x4-aligned base)
    static constexpr int NDW = RW / 4;                          // dwords staged per right-band row
    static constexpr int LSTR = kCols + 4;                      // bytes per staged left row
    static constexpr int RS_BYTES = ((ROWS * RW * 2) + 15) & ~15;
    static constexpr int FOLD_BYTES = kTileH * TW * 4;          // final cross-wave fold plane
    static constexpr int L_BYTES = ROWS * LSTR;                 // staged left tile
    static constexpr int FRONT0 = CS_BYTES > FOLD_BYTES ? CS_BYTES : FOLD_BYTES;
    static constexpr int FRONT = ((FRONT0 > L_BYTES ? FRONT0 : L_BYTES) + 15) & ~15;  // CS / fold / L alias
    static constexpr int LDS_BYTES = FRONT + RS_BYTES;
    static_assert(NQ % 4 == 2 || NQ % 4 == 0, "NQ even");
};

__device__ __forceinline__ uint32_t ld_u8(const uint8_t* p, int y, int x, int W, int H, int pitch) {
    return (y >= 0 && y < H && x >= 0 && x < W) ? (uint32_t)p[(int64_t)y * pitch + x] : 0u;
}

// 4 image bytes of row y from column x (little-endian), bytes outside the image read as 0.
// Interior dwords are one (possibly unaligned) global_load_dword; border dwords go byte-wise.
__device__ __forceinline__ uint32_t ld_u32(const uint8_t* p, int y, int x, int W, int H, int pitch) {
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

// v_perm_b32 selectors building the v_sad operands from w = R(c-d) | R(c-d-1) << 8 and the packed
// left column word lq (L of rows 4q..4q+3 in bytes 0..3); pool byte 0-3 = lq, 4-7 = w:
//   A = [L, R(c-d-1), 0, 0]  -> sad_u8(A, w)    = |L - R(c-d)|
//   B = [R(c-d), L, 0, 0]    -> sad_hi_u8(B, w) = |L - R(c-d-1)| << 16
// A masked lane (AD forced to 0: column outside the image or c < d) uses A = B = w.
__host__ __device__ constexpr uint32_t sel_a(int k) { return 0x0C0C0500u | (uint32_t)k; }
__host__ __device__ constexpr uint32_t sel_b(int k) { return 0x0C0C0004u | ((uint32_t)k << 8); }
constexpr uint32_t kSelW = 0x0C0C0504u;

template <int R, int DMAX>
__global__ __launch_bounds__(kThreads, 4) void box_match_kernel(MatchArgs a, int tiles_x, int tiles_y) {
    using G = Geo<R, DMAX>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* cs = reinterpret_cast<uint32_t*>(smem);                     // [kPairs][kTileH][CSS]
    uint16_t* rs = reinterpret_cast<uint16_t*>(smem + G::FRONT);          // [ROWS][RW]
    uint8_t* rsb = smem + G::FRONT;                                       // byte view of rs

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int lane = tid & 63;

    const int tiles = tiles_x * tiles_y;
    const int frame = blockIdx.x / tiles;
    const int t = blockIdx.x - frame * tiles;
    const int ty = t / tiles_x;
    const int tx = t - ty * tiles_x;
    const int x0 = tx * G::TW;
    const int y0 = ty * kTileH;
    const int W = a.W, H = a.H;

    const uint8_t* Lf = a.left + (int64_t)frame * a.frame_stride;
    const uint8_t* Rf = a.right + (int64_t)frame * a.frame_stride;

    const int d_lo = a.d_lo, d_hi = a.d_hi;
    const int dspan = (d_hi - d_lo + kChunk - 1) & ~(kChunk - 1);
    const int base = (x0 - R - d_lo - dspan) & ~3;   // image column of rs[.][0] (floor to x4)
    const int off0 = x0 - R - base;                  // rs index of (column c = x0-R+lane) at d = 0, minus lane

    // ---- stage the right band: rs[i][k] = R(y, base+k) | R(y, base+k-1) << 8, from dword loads
    //      (all issued before any LDS write; image borders read as 0) ----
#if SM_ABLATE & 8
    if (false)
#endif
    {
        constexpr int N = G::ROWS * G::NDW;
#pragma unroll 4
        for (int e = tid; e < N; e += kThreads) {
            const int i = e / G::NDW, j = e - (e / G::NDW) * G::NDW;
            const int y = y0 - R + i, col = base + 4 * j;
            const uint32_t cur = ld_u32(Rf, y, col, W, H, a.pitch);
            const uint32_t prv = ld_u32(Rf, y, col - 4, W, H, a.pitch);
            uint2 v;
            v.x = __builtin_amdgcn_perm(cur, prv, 0x04050304u);   // [b0, p3, b1, b0]
            v.y = __builtin_amdgcn_perm(cur, cur, 0x06070506u);   // [b2, b1, b3, b2]
            *reinterpret_cast<uint2*>(rs + i * G::RW + 4 * j) = v;
        }
    }
    // ---- stage the left tile (64 columns from x0-R) into the CS area, then pack this lane's
    //      column 4 rows per dword ----
    const int c = x0 - R + lane;                   // image column of CS column `lane`
    const int lbase = (x0 - R) & ~3;
    {
        uint8_t* ls = smem;                        // [ROWS][LSTR] bytes, aliases cs (unused yet)
        constexpr int NL = G::ROWS * (G::LSTR / 4);
        for (int e = tid; e < NL; e += kThreads) {
            const int i = e / (G::LSTR / 4), j = e - (e / (G::LSTR / 4)) * (G::LSTR / 4);
            *reinterpret_cast<uint32_t*>(ls + i * G::LSTR + 4 * j) = ld_u32(Lf, y0 - R + i, lbase + 4 * j, W, H, a.pitch);
        }
    }
    __syncthreads();
    uint32_t lq[G::NLQ];
    {
        const uint8_t* lcol = smem + (c - lbase);
#pragma unroll
        for (int q = 0; q < G::NLQ; ++q) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                const int i = 4 * q + b;
                if (i < G::ROWS) v |= (uint32_t)lcol[i * G::LSTR] << (8 * b);
            }
            lq[q] = v;
        }
    }

    // ---- per-thread phase-H state: (row j of the half, quarter q); the wave owns pairs [p_lo, p_hi) ----
    const int hj = lane & 15;
    const int hq = lane >> 4;
    const int obase = hq * G::NQ;                  // first tile output column of this thread
    uint32_t best[2][G::NQ];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int o = 0; o < G::NQ; ++o) best[h][o] = a.seed_key;

    const int xmax_tile = min(x0 + G::TW, W) - 1;
    const bool d_edge = a.valid_mode == 0 ? (xmax_tile + d_hi - 1 > W) : (d_hi - 1 > x0);
    const bool col_in = (c >= 0) && (c < W);
    const int npairs = dspan >> 1;                 // multiple of 4
    const int p_lo = (wave * npairs) / 4;
    const int p_hi = ((wave + 1) * npairs) / 4;
    uint32_t* csw = cs + wave * (G::HALF * G::CSS);   // this wave's private half-tile CS plane

    __syncthreads();   // lq reads of the aliased staging area are done before any CS write

    for (int p = p_lo; p < p_hi; ++p) {
        const int d = d_lo + 2 * p;                // pair (d, d+1)
        const uint16_t* rcol = rs + (lane + off0 - d);               // + i*RW: R(c-d) | R(c-d-1)<<8
        uint32_t* col = csw + lane;
        const bool m0 = col_in && (c >= d);
        const bool m1 = col_in && (c >= d + 1);
        uint32_t sa[4], sb[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            sa[k] = m0 ? sel_a(k) : kSelW;
            sb[k] = m1 ? sel_b(k) : kSelW;
        }
        const uint32_t dsel = (uint32_t)(d & 0xFF) | ((uint32_t)((d + 1) & 0xFF) << 8);
        const bool dm = d_edge || (d + 1 >= d_hi);
        uint32_t T = 0u, Tprev[2 * R + 1];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            // ====== phase V (lane = CS column): input rows of this half, CS rows h*HALF.. ======
#pragma unroll
            for (int i = (h == 0 ? 0 : 2 * R + G::HALF); i < (h == 0 ? 2 * R + G::HALF : G::ROWS); ++i) {
                const uint32_t w = rcol[i * G::RW];
                const uint32_t A = __builtin_amdgcn_perm(w, lq[i >> 2], sa[i & 3]);
                const uint32_t B = __builtin_amdgcn_perm(w, lq[i >> 2], sb[i & 3]);
                T = __builtin_amdgcn_sad_u8(A, w, T);
                T = __builtin_amdgcn_sad_hi_u8(B, w, T);
                if (i >= 2 * R) {
                    const uint32_t old = (i == 2 * R) ? 0u : Tprev[(i - 2 * R - 1) % (2 * R + 1)];
                    col[(i - 2 * R - h * G::HALF) * G::CSS] = T - old;
                }
                Tprev[i % (2 * R + 1)] = T;
            }
            // the plane is private to this wave and one wave's LDS ops complete in order: only the
            // compiler must keep phase-H reads below phase-V writes (and the next writes below them)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // ====== phase H (lane = half-row j x quarter q) ======
            {
                const uint32_t* row = csw + hj * G::CSS + obase;
                uint32_t v[2 * G::NCS2];
#pragma unroll
                for (int q = 0; q < G::NCS2; ++q) {
                    const uint2 x2 = *reinterpret_cast<const uint2*>(row + 2 * q);
                    v[2 * q + 0] = x2.x;
                    v[2 * q + 1] = x2.y;
                }
                uint32_t S = 0u;
#pragma unroll
                for (int k = 0; k < 2 * R; ++k) S += v[k];
                if (!dm) {
#pragma unroll
                    for (int o = 0; o < G::NQ; ++o) {
                        S += v[o + 2 * R];
                        const uint32_t klo = __builtin_amdgcn_perm(S, dsel, 0x0C050400u);
                        const uint32_t khi = __builtin_amdgcn_perm(S, dsel, 0x0C070601u);
                        best[h][o] = min(best[h][o], min(klo, khi));
                        S -= v[o];
                    }
                } else {
#pragma unroll
                    for (int o = 0; o < G::NQ; ++o) {
                        S += v[o + 2 * R];
                        const int x = x0 + obase + o;
                        const int lim = a.valid_mode == 0 ? (W - x) : x;
                        uint32_t klo = __builtin_amdgcn_perm(S, dsel, 0x0C050400u);
                        uint32_t khi = __builtin_amdgcn_perm(S, dsel, 0x0C070601u);
                        klo = (d <= lim && d < d_hi) ? klo : 0xFFFFFFFFu;
                        khi = (d + 1 <= lim && d + 1 < d_hi) ? khi : 0xFFFFFFFFu;
                        best[h][o] = min(best[h][o], min(klo, khi));
                        S -= v[o];
                    }
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    __syncthreads();

#if SM_ABLATE & 4
    if (a.W > 0) { if (tid == 0) a.disp[0] = (uint8_t)(best[0][0] ^ best[1][G::NQ - 1]); return; }
#endif
    // ---- fold the 4 waves (same lane = same pixels in every wave) through one LDS plane ----
    uint32_t* fold = cs;                                   // [kTileH][TW] keys
    if (wave == 0) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int o = 0; o < G::NQ; ++o)
                if (obase + o < G::TW) fold[(h * G::HALF + hj) * G::TW + obase + o] = best[h][o];
    }
    __syncthreads();
    if (wave != 0) {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int o = 0; o < G::NQ; ++o)
                if (obase + o < G::TW) atomicMin(&fold[(h * G::HALF + hj) * G::TW + obase + o], best[h][o]);
    }
    __syncthreads();
    uint8_t* Df = a.disp ? a.disp + (int64_t)frame * a.out_frame_stride : nullptr;
    uint32_t* Kf = a.keys ? a.keys + (int64_t)frame * W * H : nullptr;
    for (int e = tid; e < kTileH * G::TW; e += kThreads) {
        const int j = e / G::TW, o = e - j * G::TW;
        const int y = y0 + j, x = x0 + o;
        if (y >= H || x >= W) continue;
        const uint32_t k = fold[e];
        if (Df) Df[(int64_t)y * a.out_pitch + x] = k < a.thresh_key ? (uint8_t)(k & 0xFFu) : (uint8_t)0;
        if (Kf) Kf[(int64_t)y * W + x] = k;
    }
}

template <int R, int DMAX>
hipError_t launch_rd(const MatchArgs& a, int batch, hipStream_t s) {
    using G = Geo<R, DMAX>;
    const int tiles_x = (a.W + G::TW - 1) / G::TW;
    const int tiles_y = (a.H + kTileH - 1) / kTileH;
    const int64_t blocks = (int64_t)tiles_x * tiles_y * batch;
    if (blocks <= 0 || blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    hipLaunchKernelGGL((box_match_kernel<R, DMAX>), dim3((unsigned)blocks), dim3(kThreads), (size_t)G::LDS_BYTES, s,
                       a, tiles_x, tiles_y);
    return hipGetLastError();
}

template <int R>
hipError_t launch_r(const MatchArgs& a, int batch, hipStream_t s) {
    const int dspan = (a.d_hi - a.d_lo + kChunk - 1) & ~(kChunk - 1);
    if (dspan <= 64) return launch_rd<R, 64>(a, batch, s);
    if (dspan <= 128) return launch_rd<R, 128>(a, batch, s);
    return launch_rd<R, 256>(a, batch, s);
}

// ---------------------------------------------------------------------------------------
// Generic path for radius > 7 (u16 packing would overflow): direct window sum per (pixel, d)
// straight from the reference formulation.  Correct for any radius; not a performance path.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void box_match_generic_kernel(MatchArgs a, int64_t total) {
    const int64_t P = (int64_t)a.W * a.H;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= total) return;
    const int frame = (int)(gid / P);
    const int64_t p = gid - (int64_t)frame * P;
    const int y = (int)(p / a.W), x = (int)(p - (int64_t)y * a.W);
    const uint8_t* Lf = a.left + (int64_t)frame * a.frame_stride;
    const uint8_t* Rf = a.right + (int64_t)frame * a.frame_stride;
    const int r = a.radius;
    uint32_t best = a.seed_key;
    for (int d = a.d_lo; d < a.d_hi; ++d) {
        const int lim = a.valid_mode == 0 ? (a.W - x) : x;
        if (d > lim) continue;
        uint32_t sad = 0;
        for (int i = -r; i <= r; ++i) {
            const int yy = y + i;
            if (yy < 0 || yy >= a.H) continue;
            const uint8_t* lr = Lf + (int64_t)yy * a.pitch;
            const uint8_t* rr = Rf + (int64_t)yy * a.pitch;
            for (int j = -r; j <= r; ++j) {
                const int cc = x + j;
                if (cc < 0 || cc >= a.W || cc < d) continue;
                const int v = (int)lr[cc] - (int)rr[cc - d];
                sad += (uint32_t)(v < 0 ? -v : v);
            }
        }
        const uint32_t k = (sad << 8) | (uint32_t)(d & 0xFF);
        best = k < best ? k : best;
    }
    if (a.disp) a.disp[(int64_t)frame * a.out_frame_stride + (int64_t)y * a.out_pitch + x] =
        best < a.thresh_key ? (uint8_t)(best & 0xFFu) : (uint8_t)0;
    if (a.keys) a.keys[(int64_t)frame * P + p] = best;
}

}  // namespace

hipError_t launch_box_match(const MatchArgs& a, int batch, hipStream_t s) {
    switch (a.radius) {
        case 0: return launch_r<0>(a, batch, s);
        case 1: return launch_r<1>(a, batch, s);
        case 2: return launch_r<2>(a, batch, s);
        case 3: return launch_r<3>(a, batch, s);
        case 4: return launch_r<4>(a, batch, s);
        case 5: return launch_r<5>(a, batch, s);
        case 6: return launch_r<6>(a, batch, s);
        case 7: return launch_r<7>(a, batch, s);
        default: return launch_box_match_generic(a, batch, s);
    }
}

hipError_t launch_box_match_generic(const MatchArgs& a, int batch, hipStream_t s) {
    const int64_t total = (int64_t)a.W * a.H * batch;
    const int64_t blocks = (total + 255) / 256;
    if (blocks <= 0 || blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    hipLaunchKernelGGL(box_match_generic_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, total);
    return hipGetLastError();
}

}  // namespace sm
