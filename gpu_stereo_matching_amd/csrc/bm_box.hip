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
// Tile geometry (R = radius, compile-time for R <= 15; the generic kernel beyond):
//   64 CS columns (one per lane) -> TW = 64 - 2R output columns, TH = 32 output rows.
//   Disparities are processed in pairs; wave w of NW owns the contiguous pair range
//   [w*npairs/NW, (w+1)*npairs/NW) end to end (phase V -> its private CS plane -> phase H), so
//   the main loop has no workgroup barrier; the NW partial argmins are folded once at the end.
//   Phase V (lane = column): T += |L - R_d| in the low u16 and |L - R_{d+1}| in the high u16
//     (v_sad_u8 / v_sad_hi_u8); CS = T_i - T_{i-2R-1} (column window sums, two d per dword).
//   Phase H (lane = row x half-row): running window sum along x over the packed pairs, keys
//     (S << 8 | d) built with v_perm_b32, folded with v_min3_u32.
#include <cstdlib>

#include "bm_common.h"

namespace sm {
namespace {

// waves per workgroup: 4 for the plain matcher (34 KB LDS, 4 WGs/CU); 8 for the fused right view,
// whose extra 25 KB right-key rows are then shared by 8 waves (2 WGs/CU = the same 16 waves/CU)
// (r = 0 and r = 7 keep 4 waves: their fused loops need > 128 VGPRs, so they run at 2 waves/SIMD
// without spills)
template <bool RIGHT, int R>
constexpr bool kWideRight = RIGHT && R >= 1 && R <= 6;
template <bool RIGHT, int R>
constexpr int kWaves = kWideRight<RIGHT, R> ? 8 : 4;
// d_max 192 with the right view: 8 waves need 90 KB of LDS (one workgroup per CU, 8 waves); 6 waves
// need 81.6 KB, so two workgroups fit the 160 KB (12 waves per CU, 3 per SIMD: 168 VGPRs)
template <bool RIGHT, int R, int DMAX>
constexpr int kWavesD = (kWideRight<RIGHT, R> && DMAX == 192) ? 6 : kWaves<RIGHT, R>;
// right-view scatter: pair the two candidates of one u in registers (one ds_min per u) except where
// the extra live values push the fused loop past 128 VGPRs (r = 3: NQ = 16)
// (round 5, same box: unpaired, two ds_min_u32 per output and pair, ran box + LR 86.1 against 79.2 us per
// 1080p frame and 591 against 551 at 4K D=192: the scatter is LDS-atomic-bound; profiles/microbench/
// r05_box_lr_paired_scatter_ab.txt)
template <int R>
constexpr bool kPairedScatter = (R != 3);
// (round 6, VERDICT r5 item 4, not kept: a register window over two disparity pairs, whose NQ + 1 held values per
// half-row are min'ed into the next pair's before one ds_min_u32 per u, NQ + 3 atomics per two pairs instead of
// 2 NQ + 2.  Bit-exact, but the window needs ~179 VGPRs: at the 6-wave kernel's 168 it spilled 48 B per lane, and
// box + LR ran 552 -> 757 us per 4K D=192 frame, 79.0 -> 138.0 us per 1080p frame with d_max 128 moved to 6 waves;
// profiles/microbench/r06_box_lr_rwin_ab.txt)
// radius 8..15 (WIDE): the packed u16 column sums still fit (<= (32 + 2r) * 255), the window sums do
// not, so phase H keeps the two halves in separate u32 sums; the longer CS rows and the 2r+1-row
// ring need more than 128 VGPRs (2 waves/SIMD)
template <int R>
constexpr bool kWideR = R > 7;
template <bool RIGHT, int R>
constexpr int kMinWavesPerEU = ((RIGHT && !kWideRight<RIGHT, R>) || kWideR<R>) ? 2 : 4;
constexpr int kTileH = 32;        // output rows per tile (48: 4 % slower, 3 waves/SIMD)
constexpr int kNB = kTileH / 16;   // 16-row CS hand-off blocks per tile
constexpr int kPairs = 4;
constexpr int kChunk = 2 * kPairs;
constexpr int kCols = 64;
// right-key partial rows: 16-B aligned groups of 4 u, reduced with 16-B loads (round 3; one 4-B load per u
// and tile before), rows skewed against the scatter's bank conflicts (round 4, Geo::RB_SKEW)

// pad slots in front of tile tx's partial row: lead + (u - tx*TW + dmax + 1) == 0 (mod 4) for u == 0 (mod 4)
__host__ __device__ constexpr int rr_lead(int tx, int TW, int dmax) {
    return 1 + ((((tx * TW - dmax - 1) - 1) % 4 + 4) % 4);
}

template <int R, int DMAX, int NW = 4>
struct Geo {
    static constexpr int TW = kCols - 2 * R;                  // output columns per tile
    static constexpr int ROWS = kTileH + 2 * R;                 // input rows per tile
    static constexpr int HALF = 16;                             // rows per CS hand-off
    static constexpr int NLQ = (ROWS + 3) / 4;                  // packed-L dwords per lane
    static constexpr int NQ = (((TW + 3) / 4) + 1) & ~1;        // outputs per phase-H thread (even: b64 reads)
    static constexpr int NCS2 = (NQ + 2 * R + 1) / 2;           // 8-B CS reads per phase-H thread
    static constexpr int NEED = 3 * NQ + 2 * NCS2;              // last CS column read + 1
    // row stride in dwords, chosen by measurement on MI355X (32 x 1080p frames, D = 128):
    //   NQ = 14 (r >= 4): the smallest >= NEED with stride == 2 (mod 4); at r = 5, 66 / 70 run
    //     56.1 us/frame against 58.7 for 68 / 76 / 84, 76.5 for 72 and 124.3 for 80 (r = 4, 6, 7
    //     gain 3.5-6 % over the old == 4 (mod 8) rule);
    //   NQ = 16 (r <= 3): the smallest even stride that is not a multiple of 32.
    static constexpr int CSS_EVEN = (NEED + 1) & ~1;
    static constexpr int CSS = (NQ % 4 == 2) ? NEED + ((6 - NEED % 4) % 4)
                                             : (CSS_EVEN % 32 == 0 ? CSS_EVEN + 2 : CSS_EVEN);
    static constexpr int CS_BYTES = NW * HALF * CSS * 4;        // NW waves x one half-tile plane
    static constexpr int RW = kCols + DMAX + 4;                 // u16 entries per right-band row (x4-aligned base)
    static constexpr int NDW = RW / 4;                          // dwords staged per right-band row
    static constexpr int LSTR = kCols + 4;                      // bytes per staged left row
    static constexpr int RS_BYTES = ((ROWS * RW * 2) + 15) & ~15;
    static constexpr int FOLD_BYTES = kTileH * TW * 4;          // final cross-wave fold plane
    static constexpr int L_BYTES = ROWS * LSTR;                 // staged left tile
    static constexpr int FRONT0 = CS_BYTES > FOLD_BYTES ? CS_BYTES : FOLD_BYTES;
    static constexpr int FRONT = ((FRONT0 > L_BYTES ? FRONT0 : L_BYTES) + 15) & ~15;  // CS / fold / L alias
    static constexpr int LDS_BYTES = FRONT + RS_BYTES;
    // fused right view (RIGHT kernels): per-tile right-key rows indexed by u - (x0 - DMAX - 1);
    // row stride == 1 (mod 64) keeps the 64 lanes of a scatter on distinct banks (2-way for NQ 14)
    static constexpr int PW = TW + DMAX + 1;                    // right-key entries per partial row
    // partial row in HBM: the PW entries behind lead(tx) in 1..4 pad slots, so that the
    // entry of every u = 0 (mod 4) is 16-B aligned in every tile's row; pads are neutral (0xFFFFFFFF)
    static constexpr int PWP = (PW + 7 + 3) & ~3;
    static constexpr int RBW = ((PW + 63) / 64) * 64 + 1;       // >= PW + 1
    // row j starts at rb_row(j) = j * RBW + skew(j): a scatter's 32-lane group is rows hj = 0..15 of two
    // quarter-rows 14 columns apart (NQ = 14), so the row starts must cover the banks = 0, 1 (mod 4)
    // (their +14 the banks = 2, 3): skew 2 * (hj >> 1), plus 16 for the second 16-row half so that the
    // skew never decreases from one row to the next (a row keeps its full RBW entries; rows 15 and 16
    // overlapped by 4 entries when the skew restarted at 0).  With RBW = 1 (mod 32) alone, rows 14, 15 of
    // one quarter met rows 0, 1 of the next: every ds_min_u32 2-way conflicted (rocprof: 17 % of the
    // kernel's LDS cycles were bank conflicts; 1.5 % with the skew)
    static constexpr int RB_SKEW = 2;
    static constexpr int RB_BYTES = ((kTileH * RBW + 15 * RB_SKEW) * 4 + 15) & ~15;
    static constexpr int LDS_BYTES_R = LDS_BYTES + RB_BYTES;
    static_assert(NQ % 4 == 2 || NQ % 4 == 0, "NQ even");
    __host__ __device__ static constexpr int rb_row(int j) {
        return j * RBW + RB_SKEW * (((j & 15) >> 1) + 8 * (j >> 4));
    }
    static_assert(kTileH == 32, "rb_row's skew covers two 16-row halves");
};

// two right-view workgroups per CU at d_max 128 (8 waves) and 192 (6 waves), skewed rows included
static_assert(Geo<1, 128, 8>::LDS_BYTES_R <= 81920 && Geo<5, 128, 8>::LDS_BYTES_R <= 81920 &&
                  Geo<6, 128, 8>::LDS_BYTES_R <= 81920, "right view d_max 128: 2 workgroups per CU");
static_assert(Geo<1, 192, 6>::LDS_BYTES_R <= 81920 && Geo<5, 192, 6>::LDS_BYTES_R <= 81920,
              "right view d_max 192: 2 workgroups per CU (r = 6 needs 82.7 KB, one)");

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

// RIGHT = true additionally produces the right view (StereoHelper.cpp:156-180): its cost is
// C_R(u, d) = C_L(u + d, d), so every key (S << 8 | d) formed for left pixel x is also a candidate
// for right pixel u = x - d.  Phase H scatter-mins them into a per-tile LDS row (ds_min_u32) that
// is written to `a.rpart`; right_reduce_lr_kernel folds the ~(TW + D) / TW tiles covering each u.
// This replaces a second matching pass over the mirrored pair.
// NW = kWideTile (16 waves, one workgroup per CU) for launches of few tiles: the d range of a tile is
// split over 4x the waves, so a launch of ~1 round of workgroups runs in ~4 short rounds instead.
constexpr int kWideTile = 16;
template <int R, int DMAX, bool RIGHT, int NW = kWavesD<RIGHT, R, DMAX>>
__global__ __launch_bounds__((64 * NW), (NW == kWideTile ? 4 : NW == 6 ? 3 : kMinWavesPerEU<RIGHT, R>))
void box_match_kernel(MatchArgs a, int tiles_x, int tiles_y) {
    constexpr int kThreads = 64 * NW;
    using G = Geo<R, DMAX, NW>;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* cs = reinterpret_cast<uint32_t*>(smem);                     // [NW][HALF][CSS]
    uint16_t* rs = reinterpret_cast<uint16_t*>(smem + G::FRONT);          // [ROWS][RW]
    uint32_t* rb = reinterpret_cast<uint32_t*>(smem + G::FRONT + G::RS_BYTES);  // RIGHT: [kTileH][RBW]

    const int tid = threadIdx.x;
    const int wave = tid >> 6;
    const int lane = tid & 63;

    const int tiles = tiles_x * tiles_y;
    const int tile_id = xcd_tile(blockIdx.x, gridDim.x);   // [frame][ty][tx]
    const int frame = tile_id / tiles;
    const int t = tile_id - frame * tiles;
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

    // ---- stage the right band: rs[i][k] = R(y, base+k) | R(y, base+k-1) << 8, from dword loads,
    //      and the left tile (64 columns from x0-R) into the CS area.  Interior tiles (every row
    //      and column of both bands inside the image: the common case) take a branch-free path so
    //      all loads issue before the first wait; border tiles read outside bytes as 0 ----
    const int c = x0 - R + lane;                   // image column of CS column `lane`
    const int lbase = (x0 - R) & ~3;
    uint8_t* ls = smem;                            // [ROWS][LSTR] bytes, aliases cs (unused yet)
    constexpr int NR = G::ROWS * G::NDW;
    constexpr int NL = G::ROWS * (G::LSTR / 4);
    const bool interior = (y0 - R >= 0) && (y0 + kTileH + R <= H) && (base - 4 >= 0) &&
                          (base + 4 * G::NDW <= W) && (lbase >= 0) && (lbase + G::LSTR <= W);
    if (interior) {
        const uint8_t* r0 = Rf + (int64_t)(y0 - R) * a.pitch + base;
        const uint8_t* l0 = Lf + (int64_t)(y0 - R) * a.pitch + lbase;
#pragma unroll 4
        for (int e = tid; e < NR; e += kThreads) {
            const int i = e / G::NDW, j = e - (e / G::NDW) * G::NDW;
            const uint8_t* p = r0 + (int64_t)i * a.pitch + 4 * j;
            uint32_t cur, prv;
            __builtin_memcpy(&cur, p, 4);
            __builtin_memcpy(&prv, p - 4, 4);
            uint2 v;
            v.x = __builtin_amdgcn_perm(cur, prv, 0x04050304u);   // [b0, p3, b1, b0]
            v.y = __builtin_amdgcn_perm(cur, cur, 0x06070506u);   // [b2, b1, b3, b2]
            *reinterpret_cast<uint2*>(rs + i * G::RW + 4 * j) = v;
        }
#pragma unroll 4
        for (int e = tid; e < NL; e += kThreads) {
            const int i = e / (G::LSTR / 4), j = e - (e / (G::LSTR / 4)) * (G::LSTR / 4);
            uint32_t v;
            __builtin_memcpy(&v, l0 + (int64_t)i * a.pitch + 4 * j, 4);
            *reinterpret_cast<uint32_t*>(ls + i * G::LSTR + 4 * j) = v;
        }
    } else {
        for (int e = tid; e < NR; e += kThreads) {
            const int i = e / G::NDW, j = e - (e / G::NDW) * G::NDW;
            const int y = y0 - R + i, col = base + 4 * j;
            const uint32_t cur = ld_u32(Rf, y, col, W, H, a.pitch);
            const uint32_t prv = ld_u32(Rf, y, col - 4, W, H, a.pitch);
            uint2 v;
            v.x = __builtin_amdgcn_perm(cur, prv, 0x04050304u);
            v.y = __builtin_amdgcn_perm(cur, cur, 0x06070506u);
            *reinterpret_cast<uint2*>(rs + i * G::RW + 4 * j) = v;
        }
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
    uint32_t best[kNB][G::NQ];
#pragma unroll
    for (int h = 0; h < kNB; ++h)
#pragma unroll
        for (int o = 0; o < G::NQ; ++o) best[h][o] = a.seed_key;

    const int xmax_tile = min(x0 + G::TW, W) - 1;
    // the masked phase H (the validity d <= W - x of Device.cu:44, or d <= x mirrored; a partial final
    // pair; the right view's outputs past W) runs only for the pairs that need it.  d_free is the largest
    // d valid for every output of the tile, so a pair (d, d + 1) masks nothing while d + 1 <= d_free
    // (round 4: an edge tile's small-d pairs take the unmasked path; until then every pair of an edge tile
    // was masked)
    const int d_free = a.valid_mode == 0 ? W - xmax_tile : x0;
    const bool r_out = RIGHT && x0 + G::TW > W;
    const bool col_in = (c >= 0) && (c < W);
    int npairs = dspan >> 1;                       // multiple of 4
    if constexpr (!RIGHT) {
        // pairs whose d exceeds the largest d valid for ANY output of the tile (W - x0 for the left view,
        // Device.cu:44's break; x_max mirrored) leave every key of the tile unchanged: the tile's waves split
        // only the pairs below (round 5: the right-edge tiles skip their all-invalid pairs instead of running
        // them through the masked phase H; the right view (RIGHT) still needs their raw keys)
        const int dv = a.valid_mode == 0 ? W - x0 : xmax_tile;
        const int pe = dv < d_lo ? 0 : ((dv - d_lo) >> 1) + 1;
        npairs = pe < npairs ? pe : npairs;
    }
    const int p_lo = (wave * npairs) / NW;
    const int p_hi = ((wave + 1) * npairs) / NW;
    uint32_t* csw = cs + wave * (G::HALF * G::CSS);   // this wave's private half-tile CS plane
    if constexpr (RIGHT) {
        for (int e = tid; e < G::RB_BYTES / 4; e += kThreads) rb[e] = 0xFFFFFFFFu;
    }

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
        const bool dm = r_out || (d + 1 > d_free) || (d + 1 >= d_hi);
        uint32_t T = 0u, Tprev[2 * R + 1];
#pragma unroll
        for (int h = 0; h < kNB; ++h) {
            // ====== phase V (lane = CS column): input rows of this half, CS rows h*HALF.. ======
#pragma unroll
            for (int i = (h == 0 ? 0 : 2 * R + h * G::HALF); i < 2 * R + (h + 1) * G::HALF; ++i) {
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
                // WIDE: the two u16 halves of each CS word summed separately (window sums need 18 bits)
                uint32_t S = 0u, Sh = 0u;
#pragma unroll
                for (int k = 0; k < 2 * R; ++k) {
                    if constexpr (kWideR<R>) {
                        S += v[k] & 0xFFFFu;
                        Sh += v[k] >> 16;
                    } else {
                        S += v[k];
                    }
                }
                // keys (S << 8 | d): packed halves by v_perm; WIDE halves by v_lshl_or
                auto add_in = [&](uint32_t x) {
                    if constexpr (kWideR<R>) {
                        S += x & 0xFFFFu;
                        Sh += x >> 16;
                    } else {
                        S += x;
                    }
                };
                auto sub_out = [&](uint32_t x) {
                    if constexpr (kWideR<R>) {
                        S -= x & 0xFFFFu;
                        Sh -= x >> 16;
                    } else {
                        S -= x;
                    }
                };
                auto key_lo = [&]() -> uint32_t {
                    if constexpr (kWideR<R>) return (S << 8) | (dsel & 0xFFu);
                    else return __builtin_amdgcn_perm(S, dsel, 0x0C050400u);
                };
                auto key_hi = [&]() -> uint32_t {
                    if constexpr (kWideR<R>) return (Sh << 8) | (dsel >> 8);
                    else return __builtin_amdgcn_perm(S, dsel, 0x0C070601u);
                };
                // RIGHT: klo of output o goes to u_o = x_o - d, khi to u_o - 1 = u_{o-1}; the two
                // candidates of one u are min'ed in registers, one ds_min_u32 per u
                // (in slice mode, d_lo > 0, the rows hold u' = u + d_lo: the d_lo = 0 layout of d - d_lo)
                uint32_t* rrow = rb + G::rb_row(h * G::HALF + hj) + (obase - (d - d_lo) + DMAX + 1);   // + o: u_o
                uint32_t plo = 0xFFFFFFFFu;
                if (!dm) {
#pragma unroll
                    for (int o = 0; o < G::NQ; ++o) {
                        add_in(v[o + 2 * R]);
                        const uint32_t klo = key_lo();
                        const uint32_t khi = key_hi();
                        best[h][o] = min(best[h][o], min(klo, khi));
                        if constexpr (RIGHT) {
                            // outputs past TW (last quarter only) read CS columns outside the tile
                            const bool ov = (o >= G::TW - 3 * G::NQ) && (obase + o >= G::TW);
                            if constexpr (kPairedScatter<R>) {
                                const uint32_t rhi = ov ? 0xFFFFFFFFu : khi;
                                atomicMin(rrow + o - 1, min(plo, rhi));
                                plo = ov ? 0xFFFFFFFFu : klo;
                            } else if (!ov) {
                                atomicMin(rrow + o - 1, khi);
                                atomicMin(rrow + o, klo);
                            }
                        }
                        sub_out(v[o]);
                    }
                } else {
#pragma unroll
                    for (int o = 0; o < G::NQ; ++o) {
                        add_in(v[o + 2 * R]);
                        const int x = x0 + obase + o;
                        const int lim = a.valid_mode == 0 ? (W - x) : x;
                        const uint32_t klo = key_lo();
                        const uint32_t khi = key_hi();
                        const uint32_t mlo = (d <= lim && d < d_hi) ? klo : 0xFFFFFFFFu;
                        const uint32_t mhi = (d + 1 <= lim && d + 1 < d_hi) ? khi : 0xFFFFFFFFu;
                        best[h][o] = min(best[h][o], min(mlo, mhi));
                        if constexpr (RIGHT) {
                            const bool okx = (obase + o < G::TW) && (x < W);
                            const uint32_t rhi = (okx && d + 1 < d_hi) ? khi : 0xFFFFFFFFu;
                            const uint32_t rlo = (okx && d < d_hi) ? klo : 0xFFFFFFFFu;
                            if constexpr (kPairedScatter<R>) {
                                atomicMin(rrow + o - 1, min(plo, rhi));
                                plo = rlo;
                            } else {
                                atomicMin(rrow + o - 1, rhi);
                                atomicMin(rrow + o, rlo);
                            }
                        }
                        sub_out(v[o]);
                    }
                }
                if constexpr (RIGHT && kPairedScatter<R>) atomicMin(rrow + G::NQ - 1, plo);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
    }
    __syncthreads();

    // ---- fold the NW waves (same lane = same pixels in every wave) through one LDS plane ----
    uint32_t* fold = cs;                                   // [kTileH][TW] keys
    if (wave == 0) {
#pragma unroll
        for (int h = 0; h < kNB; ++h)
#pragma unroll
            for (int o = 0; o < G::NQ; ++o)
                if (obase + o < G::TW) fold[(h * G::HALF + hj) * G::TW + obase + o] = best[h][o];
    }
    __syncthreads();
    if (wave != 0) {
#pragma unroll
        for (int h = 0; h < kNB; ++h)
#pragma unroll
            for (int o = 0; o < G::NQ; ++o)
                if (obase + o < G::TW) atomicMin(&fold[(h * G::HALF + hj) * G::TW + obase + o], best[h][o]);
    }
    __syncthreads();
    uint8_t* Df = a.disp ? a.disp + (int64_t)frame * a.out_frame_stride : nullptr;
    uint32_t* Kf = a.keys ? a.keys + (int64_t)frame * W * H : nullptr;
    // lane = output column (TW <= 64), rows over the waves: no per-element division, wave-uniform row bases
    if (lane < G::TW && x0 + lane < W) {
        const int ylim = min(kTileH, H - y0);
        uint8_t* drow = Df ? Df + (int64_t)y0 * a.out_pitch + x0 + lane : nullptr;
        uint32_t* krow = Kf ? Kf + (int64_t)y0 * W + x0 + lane : nullptr;
#pragma unroll
        for (int j = wave; j < kTileH; j += NW) {
            if (j >= ylim) break;
            const uint32_t k = fold[j * G::TW + lane];
            if (drow) drow[(int64_t)j * a.out_pitch] = k < a.thresh_key ? (uint8_t)(k & 0xFFu) : (uint8_t)0;
            if (krow) krow[(int64_t)j * W] = k;
        }
    }
    if constexpr (RIGHT) {
        // rb is untouched by the fold (which aliases the CS area); rows past H are never read
        uint32_t* P = a.rpart + (int64_t)tile_id * (kTileH * G::PWP);   // [frame][ty][tx][kTileH][PWP]
        const int lead = rr_lead(tx, G::TW, DMAX);
        // rows over the waves, entries over the lanes (no per-element division)
        for (int j = wave; j < kTileH; j += NW) {
            uint32_t* prow = P + j * G::PWP;
            const uint32_t* rrow = rb + G::rb_row(j) - lead;
#pragma unroll
            for (int e = lane; e < G::PWP; e += 64) {
                const int k = e - lead;
                prow[e] = (k >= 0 && k < G::PW) ? rrow[e] : 0xFFFFFFFFu;
            }
        }
    }
}

// Right view (+ LR check when `check`) for one image row per block.  Right key of u = min over the tiles whose
// partial rows cover u (x0 - DMAX - 1 <= u < x0 + TW, x0 <= u + d_hi - 1); dR = key & 0xFF with no
// threshold (StereoHelper.cpp:131-154).  Then StereoDisparity.cpp:136-147 on the row:
//   d = dL(x); occ = x-d < 0 || d == 0 || |d - dR(x-d)| > 1;  out = occ ? 0 : d.
// The partial rows are padded (Geo::PWP): a thread takes u = 4m..4m+3 and reads each covering
// tile's four entries with one 16-B load.  The tile range is that of the group (a tile covering only some
// of the four u holds 0xFFFFFFFF or a valid candidate of the others: every entry a tile writes is
// C_L(u + d, d) of one of its pixels, so a min over a superset of the covering tiles is the same key).
// The LR check then runs on 4 pixels per thread with dword loads and stores where the rows allow.
// Slice mode (rkeys != nullptr, multi-GPU d-slices with LR): the partial rows of a pass over d in
// [d_lo, d_hi) hold u' = u + d_lo (box_match_kernel's right rows), `d_hi` is then the span d_hi - d_lo, and
// the kernel writes the minimum key of every right pixel u to rkeys[f][y][u], sign bit flipped (kRightKeyFlip;
// 0x7FFFFFFF where no d of the slice has u + d < W), instead of dR: keys of disjoint slices combine with a
// signed MIN.
template <int MAXT>
__global__ __launch_bounds__(256) void right_reduce_lr_vec_kernel(const uint32_t* __restrict__ rpart, int tiles_x,
                                                                  int tiles_y, int TW, int PWP, int dmax, int d_hi,
                                                                  int W, int H, int check, uint8_t* disp, int opitch,
                                                                  int64_t ostride, uint8_t* __restrict__ right_out,
                                                                  uint8_t* __restrict__ mask_out, int apitch,
                                                                  int64_t astride, uint32_t* __restrict__ rkeys,
                                                                  int d_lo) {
    extern __shared__ __attribute__((aligned(16))) uint8_t dr_row[];   // W rounded up to 4
    const int y = blockIdx.x, f = blockIdx.y;
    uint32_t* krow = rkeys ? rkeys + ((int64_t)f * H + y) * W : nullptr;
    if (krow)   // right pixels past every slice disparity's reach: u + d_lo >= W
        for (int u = max(W - d_lo, 0) + (int)threadIdx.x; u < W; u += blockDim.x) krow[u] = 0x7FFFFFFFu;
    const int ty = y / kTileH, j = y - ty * kTileH;
    const uint32_t* base = rpart + (((int64_t)f * tiles_y + ty) * tiles_x * kTileH + j) * PWP;
    const int64_t tstride = (int64_t)kTileH * PWP;
    uint8_t* rrow = right_out ? right_out + (int64_t)f * astride + (int64_t)y * apitch : nullptr;
    const bool rvec = rrow && ((reinterpret_cast<uintptr_t>(rrow) & 3) == 0);
    const int groups = (W + 3) >> 2;
    for (int m = threadIdx.x; m < groups; m += blockDim.x) {
        const int u = 4 * m;
        const int tlo = u / TW;
        const int thi = min(tiles_x - 1, (u + 3 + d_hi - 1) / TW);
        uint4 v[MAXT];
#pragma unroll
        for (int k = 0; k < MAXT; ++k) {
            const int tx = min(tlo + k, thi);   // repeated last tile: same keys, fixed trip count
            const int idx = rr_lead(tx, TW, dmax) + u - tx * TW + dmax + 1;
            v[k] = *reinterpret_cast<const uint4*>(base + tx * tstride + idx);
        }
        uint32_t k0 = v[0].x, k1 = v[0].y, k2 = v[0].z, k3 = v[0].w;
#pragma unroll
        for (int k = 1; k < MAXT; ++k) {
            k0 = min(k0, v[k].x);
            k1 = min(k1, v[k].y);
            k2 = min(k2, v[k].z);
            k3 = min(k3, v[k].w);
        }
        if (krow) {
            const uint32_t kk[4] = {k0, k1, k2, k3};
#pragma unroll
            for (int b = 0; b < 4; ++b)
                if (u + b < W && u + b >= d_lo) krow[u + b - d_lo] = kk[b] ^ kRightKeyFlip;
            continue;
        }
        const uint32_t dr4 = __builtin_amdgcn_perm(__builtin_amdgcn_perm(k3, k2, 0x0C0C0400u),
                                                   __builtin_amdgcn_perm(k1, k0, 0x0C0C0400u), 0x05040100u);
        *reinterpret_cast<uint32_t*>(dr_row + u) = dr4;
        if (rrow) {
            if (rvec && u + 3 < W) {
                *reinterpret_cast<uint32_t*>(rrow + u) = dr4;
            } else {
                for (int b = 0; b < 4 && u + b < W; ++b) rrow[u + b] = (uint8_t)(dr4 >> (8 * b));
            }
        }
    }
    if (!check) return;
    __syncthreads();
    uint8_t* drow = disp + (int64_t)f * ostride + (int64_t)y * opitch;
    uint8_t* mrow = mask_out ? mask_out + (int64_t)f * astride + (int64_t)y * apitch : nullptr;
    const bool dvec = ((reinterpret_cast<uintptr_t>(drow) & 3) == 0) &&
                      (!mrow || ((reinterpret_cast<uintptr_t>(mrow) & 3) == 0));
    for (int m = threadIdx.x; m < groups; m += blockDim.x) {
        const int x0 = 4 * m;
        const bool vec = dvec && x0 + 3 < W;
        uint32_t dw = 0;
        if (vec) {
            dw = *reinterpret_cast<const uint32_t*>(drow + x0);
        } else {
            for (int b = 0; b < 4 && x0 + b < W; ++b) dw |= (uint32_t)drow[x0 + b] << (8 * b);
        }
        uint32_t ow = 0, mw = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int x = x0 + b;
            const int d = (dw >> (8 * b)) & 0xFF;
            int occ = 1;
            if (x - d >= 0) {
                const int diff = d - (int)dr_row[x - d];
                occ = (d == 0) || diff > 1 || diff < -1;
            }
            ow |= (uint32_t)(occ ? 0 : d) << (8 * b);
            mw |= (uint32_t)(!occ) << (8 * b);
        }
        if (vec) {
            *reinterpret_cast<uint32_t*>(drow + x0) = ow;
            if (mrow) *reinterpret_cast<uint32_t*>(mrow + x0) = mw;
        } else {
            for (int b = 0; b < 4 && x0 + b < W; ++b) {
                drow[x0 + b] = (uint8_t)(ow >> (8 * b));
                if (mrow) mrow[x0 + b] = (uint8_t)(mw >> (8 * b));
            }
        }
    }
}

// Output buffers of the fused right view (launch_box_match_lr).
struct RightOut {
    int check;        // 1: apply the LR check to a.disp; 0: only produce dR
    uint8_t* right;   // dR (optional when check)
    uint8_t* mask;    // optional valid mask
    int pitch;
    int64_t stride;
    uint32_t* rkeys;  // slice mode: raw right keys [batch][H][W] instead of dR (check 0, right null)
};

int compute_units() {
    static const int n = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return cus;
    }();
    return n;
}

// SM_WIDE_TILES=0 keeps the 4-wave kernel for every launch (A/B timing)
bool wide_tiles_enabled() {
    static const bool on = [] {
        const char* e = std::getenv("SM_WIDE_TILES");
        return !(e && e[0] == '0');
    }();
    return on;
}

// Launches of more tiles than CUs but at most SM_BOX_MID_MAX (default 8) tiles per CU (batch 1 of a
// mid-size frame) take 8-wave tiles, the d pairs split over twice the waves: the last round of tiles
// ends sooner.  Same box, device resident, batch 1 (profiles/microbench/r04_box_mid_tiles_latency.txt):
// 960x540 D=128 47.5 -> 39.7 us, 320x240 D=32 16.7 -> 13.6, 1080p D=128 88.5 -> 86.3; maps identical.
// SM_BOX_MID=0 (read once) keeps the 4-wave tiles (A/B).
int mid_tiles_max() {
    static const int v = [] {
        const char* e = std::getenv("SM_BOX_MID");
        if (e && e[0] == '0') return 0;
        const char* m = std::getenv("SM_BOX_MID_MAX");
        return m ? std::atoi(m) : 8;
    }();
    return v;
}

template <int R, int DMAX, bool RIGHT>
hipError_t launch_rd(const MatchArgs& a, int batch, const RightOut* ro, hipStream_t s) {
    using G = Geo<R, DMAX, kWavesD<RIGHT, R, DMAX>>;
    const int tiles_x = (a.W + G::TW - 1) / G::TW;
    const int tiles_y = (a.H + kTileH - 1) / kTileH;
    const int64_t blocks = (int64_t)tiles_x * tiles_y * batch;
    if (blocks <= 0 || blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    if constexpr (RIGHT) {
        hipLaunchKernelGGL((box_match_kernel<R, DMAX, true>), dim3((unsigned)blocks), dim3(64 * kWavesD<true, R, DMAX>),
                           (size_t)G::LDS_BYTES_R, s, a, tiles_x, tiles_y);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        // tiles covering one of u .. u + 3: ceil((d_hi + 2) / TW) + 1 at most
        constexpr int kMaxT4 = (DMAX + 2 + G::TW - 1) / G::TW + 1;
        hipLaunchKernelGGL((right_reduce_lr_vec_kernel<kMaxT4>), dim3(a.H, batch), dim3(256),
                           (size_t)((a.W + 3) & ~3), s, a.rpart, tiles_x, tiles_y, G::TW, G::PWP, DMAX,
                           a.d_hi - a.d_lo, a.W, a.H, ro->check, a.disp, a.out_pitch, a.out_frame_stride, ro->right,
                           ro->mask, ro->pitch, ro->stride, ro->rkeys, a.d_lo);
    } else {
        // no more tiles than CUs (a small frame, batch 1): 16 waves per tile, >= 2 d-pairs each, so every
        // CU runs 16 waves instead of <= 4 (R <= 7: the wide-radius kernels need > 128 VGPRs).  Beyond
        // one tile per CU the 4-wave kernel wins: with one 16-wave workgroup per CU a tile's staging
        // overlaps no other tile's compute (1080p batch 1: 102.8 vs 87.8 us).
        const int npairs = ((a.d_hi - a.d_lo + kChunk - 1) & ~(kChunk - 1)) / 2;
        if constexpr (!kWideR<R>) {
            if (wide_tiles_enabled() && blocks <= compute_units() && npairs >= 2 * kWideTile) {
                using GW = Geo<R, DMAX, kWideTile>;
                hipLaunchKernelGGL((box_match_kernel<R, DMAX, false, kWideTile>), dim3((unsigned)blocks),
                                   dim3(64 * kWideTile), (size_t)GW::LDS_BYTES, s, a, tiles_x, tiles_y);
                return hipGetLastError();
            }
        }
        if constexpr (!kWideR<R>) {
            if (mid_tiles_max() > 0 && blocks <= (int64_t)mid_tiles_max() * compute_units() && npairs >= 16) {
                using GM = Geo<R, DMAX, 8>;
                hipLaunchKernelGGL((box_match_kernel<R, DMAX, false, 8>), dim3((unsigned)blocks), dim3(64 * 8),
                                   (size_t)GM::LDS_BYTES, s, a, tiles_x, tiles_y);
                return hipGetLastError();
            }
        }
        hipLaunchKernelGGL((box_match_kernel<R, DMAX, false>), dim3((unsigned)blocks), dim3(64 * kWaves<false, R>),
                           (size_t)G::LDS_BYTES, s, a, tiles_x, tiles_y);
    }
    return hipGetLastError();
}

template <int R, bool RIGHT>
hipError_t launch_r(const MatchArgs& a, int batch, const RightOut* ro, hipStream_t s) {
    const int dspan = (a.d_hi - a.d_lo + kChunk - 1) & ~(kChunk - 1);
    if (dspan <= 64) return launch_rd<R, 64, RIGHT>(a, batch, ro, s);
    if (dspan <= 128) return launch_rd<R, 128, RIGHT>(a, batch, ro, s);
    // 192 (cfg5): the right band and the right-key rows sized for 192, not 256, keep the plain kernel
    // at 4 workgroups/CU and the right-view kernel at 2
    if (dspan <= 192) return launch_rd<R, 192, RIGHT>(a, batch, ro, s);
    return launch_rd<R, 256, RIGHT>(a, batch, ro, s);
}

template <int R>
size_t partial_bytes_r(int W, int H, int D, int batch) {
    const int dspan = (D + kChunk - 1) & ~(kChunk - 1);
    const int dmax = dspan <= 64 ? 64 : (dspan <= 128 ? 128 : (dspan <= 192 ? 192 : 256));
    const int TW = kCols - 2 * R;
    const int PW = TW + dmax + 1;
    const int PWP = (PW + 7 + 3) & ~3;   // Geo::PWP
    const size_t tiles = (size_t)((W + TW - 1) / TW) * ((H + kTileH - 1) / kTileH);
    return tiles * (size_t)batch * kTileH * PWP * 4;
}

// ---------------------------------------------------------------------------------------
// Generic path for radius > 15 (the u16 column prefix would overflow): direct window sum per (pixel, d)
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
        case 0: return launch_r<0, false>(a, batch, nullptr, s);
        case 1: return launch_r<1, false>(a, batch, nullptr, s);
        case 2: return launch_r<2, false>(a, batch, nullptr, s);
        case 3: return launch_r<3, false>(a, batch, nullptr, s);
        case 4: return launch_r<4, false>(a, batch, nullptr, s);
        case 5: return launch_r<5, false>(a, batch, nullptr, s);
        case 6: return launch_r<6, false>(a, batch, nullptr, s);
        case 7: return launch_r<7, false>(a, batch, nullptr, s);
        case 8: return launch_r<8, false>(a, batch, nullptr, s);
        case 9: return launch_r<9, false>(a, batch, nullptr, s);
        case 10: return launch_r<10, false>(a, batch, nullptr, s);
        case 11: return launch_r<11, false>(a, batch, nullptr, s);
        case 12: return launch_r<12, false>(a, batch, nullptr, s);
        case 13: return launch_r<13, false>(a, batch, nullptr, s);
        case 14: return launch_r<14, false>(a, batch, nullptr, s);
        case 15: return launch_r<15, false>(a, batch, nullptr, s);
        default: return launch_box_match_generic(a, batch, s);
    }
}

size_t box_right_partial_bytes(int W, int H, int radius, int D, int batch) {
    switch (radius) {
        case 0: return partial_bytes_r<0>(W, H, D, batch);
        case 1: return partial_bytes_r<1>(W, H, D, batch);
        case 2: return partial_bytes_r<2>(W, H, D, batch);
        case 3: return partial_bytes_r<3>(W, H, D, batch);
        case 4: return partial_bytes_r<4>(W, H, D, batch);
        case 5: return partial_bytes_r<5>(W, H, D, batch);
        case 6: return partial_bytes_r<6>(W, H, D, batch);
        case 7: return partial_bytes_r<7>(W, H, D, batch);
        case 8: return partial_bytes_r<8>(W, H, D, batch);
        case 9: return partial_bytes_r<9>(W, H, D, batch);
        case 10: return partial_bytes_r<10>(W, H, D, batch);
        case 11: return partial_bytes_r<11>(W, H, D, batch);
        case 12: return partial_bytes_r<12>(W, H, D, batch);
        case 13: return partial_bytes_r<13>(W, H, D, batch);
        case 14: return partial_bytes_r<14>(W, H, D, batch);
        case 15: return partial_bytes_r<15>(W, H, D, batch);
        default: return 0;
    }
}

static hipError_t launch_box_right(const MatchArgs& a, int batch, const RightOut* rop, hipStream_t s) {
    const RightOut& ro = *rop;
    switch (a.radius) {
        case 0: return launch_r<0, true>(a, batch, &ro, s);
        case 1: return launch_r<1, true>(a, batch, &ro, s);
        case 2: return launch_r<2, true>(a, batch, &ro, s);
        case 3: return launch_r<3, true>(a, batch, &ro, s);
        case 4: return launch_r<4, true>(a, batch, &ro, s);
        case 5: return launch_r<5, true>(a, batch, &ro, s);
        case 6: return launch_r<6, true>(a, batch, &ro, s);
        case 7: return launch_r<7, true>(a, batch, &ro, s);
        case 8: return launch_r<8, true>(a, batch, &ro, s);
        case 9: return launch_r<9, true>(a, batch, &ro, s);
        case 10: return launch_r<10, true>(a, batch, &ro, s);
        case 11: return launch_r<11, true>(a, batch, &ro, s);
        case 12: return launch_r<12, true>(a, batch, &ro, s);
        case 13: return launch_r<13, true>(a, batch, &ro, s);
        case 14: return launch_r<14, true>(a, batch, &ro, s);
        case 15: return launch_r<15, true>(a, batch, &ro, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_box_match_lr(const MatchArgs& a, int batch, int check, uint8_t* right_out, uint8_t* mask_out,
                               int aux_pitch, int64_t aux_stride, hipStream_t s) {
    if (a.d_lo != 0 || a.valid_mode != 0 || !a.disp || !a.rpart || (!check && !right_out)) return hipErrorInvalidValue;
    const RightOut ro{check, right_out, mask_out, aux_pitch, aux_stride, nullptr};
    return launch_box_right(a, batch, &ro, s);
}

hipError_t launch_box_slice_lr_keys(const MatchArgs& a, int batch, uint32_t* right_keys, hipStream_t s) {
    if (a.valid_mode != 0 || !a.keys || !a.rpart || !right_keys || a.d_lo < 0 || a.d_hi <= a.d_lo ||
        a.d_hi > kMaxDisp)
        return hipErrorInvalidValue;
    const RightOut ro{0, nullptr, nullptr, 0, 0, right_keys};
    return launch_box_right(a, batch, &ro, s);
}

hipError_t launch_box_match_generic(const MatchArgs& a, int batch, hipStream_t s) {
    const int64_t total = (int64_t)a.W * a.H * batch;
    const int64_t blocks = (total + 255) / 256;
    if (blocks <= 0 || blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    hipLaunchKernelGGL(box_match_generic_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, total);
    return hipGetLastError();
}

}  // namespace sm
