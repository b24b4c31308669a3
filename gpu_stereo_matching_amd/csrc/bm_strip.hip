// bm_strip.hip — box matching at radius 16..37 with the disparities across the lanes (round 6).
//
// The fused tile kernel (bm_box.hip) keeps TW = 64 - 2r output columns per 64-lane tile and stops at r = 15; the
// separable path (bm_wide.hip) streams a u16 plane of vertical sums per d through HBM (2 B written + 2 B read per
// (pixel, d)) at any r.  This kernel keeps the vertical sums on chip instead, for the radii just past the tile
// kernel: one workgroup walks a band of rows of a 128-column strip, lane = disparity (d_lo + 64 * wave + lane), and
// each lane holds V_d(c) = sum of AD_d over the rows y-r..y+r for all 128 columns of the strip in 64 registers (u16
// pairs of adjacent columns, V <= 75 * 255).  Per row step, for its d:
//   V_d(c) += AD_d(y + r, c) - AD_d(y - r - 1, c)      (Device.cu:27-31; rows outside the frame are 0)
//   S_d(x) = sum of V_d over c = x-r..x+r              (running sum along the strip, SDWA adds, Device.cu:46-56)
//   key = S << 8 | d, min over the 64 lanes by a transpose-reduce butterfly (permlane32 / permlane16 swaps, a DPP
//   half-row exchange, three DPP steps within 8 lanes: 18 VALU per 8 outputs, no LDS), then over the waves through
//   LDS, with the 50 win^2 seed (Device.cu:37) and the validity d <= W - x (:44): the WTA of getDisp, bit for bit.
// The step's L and R rows (the row entering V and the row leaving it) are staged in LDS as u16 pairs: L once, R in
// two copies one column apart so that every lane reads aligned words whatever the parity of its offset DP - d
// (copy stride = 16 mod 32 words: conflict-free).  Their global loads are issued two steps ahead into registers,
// written to LDS one step ahead (double buffer), so no step waits on memory.  Nothing but the pair and the map
// touches HBM.  Interior strips run an unmasked body; the strips at the frame's edges (columns below d or past W,
// outputs past W or with d > W - x) a masked copy.
// Output columns per strip: 128 - 2r (r = 16: 96, r = 37: 54); a band's first 2r row steps only build V.  Bands:
// as many as the resident workgroups allow in one round (4 waves per SIMD: <= 128 VGPRs).
// 1080p, D = 128, 8 frames per call (us per frame, MI355X, same box, against the separable path's 234-237):
// r = 16 141.9, r = 20 150.7, r = 25 180.2, r = 31 203.9, r = 37 223.4.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "bm_common.h"

namespace sm {
namespace {

constexpr int kSC = 128;      // input columns per strip
constexpr int kSP = kSC / 2;  // u16 column pairs per strip row
constexpr int kSQ = kSC / 4;  // 4-column groups per strip
constexpr int kNT = 256;      // max threads per workgroup (4 waves: d spans up to 256)
#ifndef SM_STRIP_WPE
#define SM_STRIP_WPE 4        // waves per SIMD the register budget is sized for
#endif
#ifndef SM_STRIP_LA
#define SM_STRIP_LA 1         // 4-column groups whose LDS reads are in flight ahead of the one being summed
#endif
#ifndef SM_STRIP_ADOR
#define SM_STRIP_ADOR 1       // |a - b| as (a -sat b) | (b -sat a) (2 % faster than max - min at r = 20)
#endif
#ifndef SM_STRIP_CH2
#define SM_STRIP_CH2 0        // 1: the row's window sums as two independent chains (first / second half of the groups)
#endif
#ifndef SM_STRIP_VMASK
#define SM_STRIP_VMASK 1
#endif
#ifndef SM_STRIP_ONELOOP
#define SM_STRIP_ONELOOP 0
#endif
// every lambda of the kernel inlined: one left out of line takes V (captured by reference) to scratch
#define SM_INL __attribute__((always_inline))

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as16(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

// 4 bytes of row y from column x (little-endian), 0 outside the frame.  One dword load clamped into the row
// (W >= 4), shifted so that the bytes of in-frame columns land in place: a group straddling an edge keeps its
// in-frame bytes, a group wholly outside reads 0
__device__ __forceinline__ uint32_t ld4(const uint8_t* p, int y, int x, int W, int H, int pitch) {
    if (y < 0 || y >= H) return 0u;
    const int xc = min(max(x, 0), W - 4);
    uint32_t v;
    __builtin_memcpy(&v, p + (int64_t)y * pitch + xc, 4);
    const int sh = x - xc;   // > 0: past the right edge by sh columns, < 0: before the left edge
    if (sh != 0) v = (sh >= 4 || sh <= -4) ? 0u : sh > 0 ? v >> (8 * sh) : v << (-8 * sh);
    return v;
}

// min of `keep` and lane `partner`'s `send` (DPP control `CTRL`, every row and bank)
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_min(uint32_t keep, uint32_t send) {
    return min(keep, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)send, CTRL, 0xF, 0xF, false));
}

// R staged words per copy of a row: columns rb0 .. rb0 + DP - d_lo + kSC + 3 (d_lo rounded down to 4; the lanes
// read staged columns DP - d .. DP - d + 127) as u16 pairs; copies r_stride words apart, = 16 mod 32, so that the
// lanes reading copy 0 (even DP - d) and copy 1 (odd) fall on disjoint halves of the banks
constexpr int r_words(int DP, int d_lo) { return (DP - (d_lo & ~3) + kSC + 4) / 2; }
constexpr int r_stride(int RW) { return ((RW + 15) & ~31) + 16; }
constexpr int stage_bytes(int RS) { return 2 * kSP * 4 + 2 * 2 * RS * 4; }

// RIGHT: the right view too, folded per output row into an LDS row by atomic min (C_R(u, d) = C_L(u + d, d) for
// u = x - d >= 0, StereoHelper.cpp:156-180, as the separable path's hwta kernel) and flushed into rk, the frame's
// right keys [batch][H][W] (filled with ~0 by the caller), by global atomic min (strips overlap in u)
template <int R, bool RIGHT>
__global__ __launch_bounds__(kNT, SM_STRIP_WPE) void strip_kernel(const uint8_t* __restrict__ Limg, const uint8_t* __restrict__ Rimg,
                                                    int64_t fstride, int W, int H, int pitch, int d_lo, int d_hi, int EL,
                                                    int NI, int nb, int nbe, int vm,
                                                    int DP, int RW, int RS, int nw, uint32_t seed, uint32_t thresh,
                                                    uint8_t* __restrict__ disp, int opitch, int64_t ostride,
                                                    uint32_t* __restrict__ keys, uint32_t* __restrict__ rk) {
    constexpr int SW = kSC - 2 * R;            // output columns of the strip
    constexpr int NG = (SW + 7) / 8;           // groups of 8 outputs
    extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
    const int BUF = stage_bytes(RS);           // one step: L in/out as u16 column pairs, R in/out as two copies
    const int nt = 64 * nw;                    // threads (blockDim.x, kept in an SGPR)
    uint32_t* wmin = reinterpret_cast<uint32_t*>(lds + 2 * BUF);   // [2][nw][NG * 8]
    const int RN = SW + DP;                    // right row: u = x0 - DP + i, i < RN
    uint32_t* rrow = wmin + 2 * nw * NG * 8;   // [2][RN] (RIGHT)

    // blockIdx.x runs over the (strip, band) pairs of a frame: the EL left edge strips in nbe bands each, the NI
    // interior strips in nb bands, the remaining (right edge) strips in nbe bands.  The edge strips' masked body
    // costs more per row, so their bands are shorter: every workgroup of the one round finishes at about the same time
    const int f = blockIdx.z;
    int strip, band, bands;
    {
        const int b = blockIdx.x, e0 = EL * nbe, i0 = e0 + NI * nb;
        if (b < e0) {
            strip = b / nbe;
            band = b - strip * nbe;
            bands = nbe;
        } else if (b < i0) {
            const int k = (b - e0) / nb;
            strip = EL + k;
            band = b - e0 - k * nb;
            bands = nb;
        } else {
            const int k = (b - i0) / nbe;
            strip = EL + NI + k;
            band = b - i0 - k * nbe;
            bands = nbe;
        }
    }
    const int BH = (H + bands - 1) / bands;
    const int x0 = strip * SW, cs0 = x0 - R, rb0 = cs0 - DP;
    const int y0 = band * BH, y1 = min(y0 + BH, H);
    const uint8_t* Lf = Limg + (int64_t)f * fstride;
    const uint8_t* Rf = Rimg + (int64_t)f * fstride;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int d = d_lo + wave * 64 + lane;
    const uint32_t dd = (uint32_t)(d & 0xFF);
    // lanes past the slice: their window sums start at 2^23, so every key they form is >= 2^31, above every real key
    // (< 2^28) and the seed; where an output may have no real key (the masked path) they are forced to ~0 as well
    const bool live = d < d_hi;
    const uint32_t dmask = live ? 0u : 0xFFFFFFFFu;
    const uint32_t s0 = live ? 0u : (1u << 23);

    // strip-uniform: every column of the strip >= every d and inside the frame (no AD masks), and every output
    // inside the frame with every d valid (no key masks)
    const bool col_ok = cs0 >= d_hi - 1 && cs0 + kSC <= W;
    // (vm = valid_mode: 0 d <= W - x, Device.cu:44; 1 the mirrored right view's d <= x)
    const bool out_ok = x0 + SW <= W && (vm == 0 ? (d_hi - 1) <= W - (x0 + SW - 1) : (d_hi - 1) <= x0);

    // L: [2][kSP] words (L(2p), L(2p + 1)); R: [2 rows][2 copies][RS] words, copy 0 word i = (R(rb0 + 2i),
    // R(rb0 + 2i + 1)), copy 1 one column back (R(rb0 + 2i - 1), R(rb0 + 2i)), so that every lane reads aligned words whatever d's parity
    // item e of a step: e < nL one 4-column group of the L rows (in, out), else one of the R rows.  The loads of
    // step s + 2 are issued in step s into registers (kPF items per thread) and written to LDS in step s + 1, so
    // no step waits on a global load
    const int ng = RW / 2;                      // 4-column groups per R row
    const int nL = 2 * kSQ, nItems = nL + 2 * ng;
    constexpr int kPF = 3;                      // items per thread: 64 + 2 ceil((nd + 135) / 4) <= 3 * 64 nw
    uint32_t pw[kPF], pw2[kPF];
    auto fetch = [&](int yin, int yout) SM_INL {
#pragma unroll
        for (int i = 0; i < kPF; ++i) {
            int e = tid + i * nt;
            asm volatile("" : "+v"(e));   // item compares inside the loop (hoisted, their masks pin SGPR pairs)
            pw[i] = pw2[i] = 0u;
            if (e < nL) {
                const bool io = e >= kSQ;
                pw[i] = ld4(Lf, io ? yout : yin, cs0 + 4 * (e & (kSQ - 1)), W, H, pitch);
            } else if (e < nItems) {
                const int e2 = e - nL;
                const bool io = e2 >= ng;
                const int j = io ? e2 - ng : e2;
                const int y = io ? yout : yin;
                pw[i] = ld4(Rf, y, rb0 + 4 * j, W, H, pitch);
                pw2[i] = ld4(Rf, y, rb0 + 4 * j - 4, W, H, pitch);
            }
        }
    };
    auto store = [&](int buf) SM_INL {
        uint8_t* B = lds + buf * BUF;
        uint2* Ls = reinterpret_cast<uint2*>(B);                   // [2][kSQ]
        uint32_t* Rs = reinterpret_cast<uint32_t*>(B + 2 * kSP * 4);   // [2][2][RS]
#pragma unroll
        for (int i = 0; i < kPF; ++i) {
            int e = tid + i * nt;
            asm volatile("" : "+v"(e));
            const uint32_t w = pw[i], w2 = pw2[i];
            if (e < nL) {
                Ls[e] = make_uint2(__builtin_amdgcn_perm(0u, w, 0x0c010c00u), __builtin_amdgcn_perm(0u, w, 0x0c030c02u));
            } else if (e < nItems) {
                const int e2 = e - nL;
                const bool io = e2 >= ng;
                const int j = io ? e2 - ng : e2;
                uint32_t* row = Rs + (io ? 2 * RS : 0) + 2 * j;
                *reinterpret_cast<uint2*>(row) =
                    make_uint2(__builtin_amdgcn_perm(0u, w, 0x0c010c00u), __builtin_amdgcn_perm(0u, w, 0x0c030c02u));
                *reinterpret_cast<uint2*>(row + RS) =
                    make_uint2(__builtin_amdgcn_perm(w, w2, 0x0c040c03u), __builtin_amdgcn_perm(0u, w, 0x0c020c01u));
            }
        }
    };

    // this lane's R window: strip column c reads R(cs0 + c - d) = staged column DP - d + c of copy 0
    const int ro = DP - d;                      // >= 0 (DP >= d_hi - 1 >= d for the lanes that count)
    const int roc = ro < 0 ? 0 : ro;            // lanes past the slice read in range
    // (odd: copy 1 word (roc + 1) / 2; with RS = 16 mod 32 the 32 lanes of a read half hit 32 distinct banks)
    const int rword = (roc >> 1) + (roc & 1) * (RS + 1);
    // AD masks for the edge strips: column c = cs0 + k counts when d <= c < W (Device.cu:27-31 and the frame)
    const int clo = d - cs0, chi = W - cs0;     // strip column index range [clo, chi)

    uint32_t V[kSP];                            // V(2p), V(2p + 1), u16 each (V <= 63 * 255)
#pragma unroll
    for (int p = 0; p < kSP; ++p) V[p] = 0u;

    // one step's rows: AD of the in row into V and (OUT) of the out row out of it, from buffer buf.  The LDS reads of
    // 4-column group q + SM_STRIP_LA are issued before group q's arithmetic
    auto update = [&](int buf, auto edge, auto with_out) SM_INL {
        constexpr bool EDGE = decltype(edge)::value;
        constexpr bool OUT = decltype(with_out)::value;
        const uint8_t* B = lds + buf * BUF;
        const uint2* Ls = reinterpret_cast<const uint2*>(B);       // [2][kSQ]
        const uint32_t* Rr = reinterpret_cast<const uint32_t*>(B + 2 * kSP * 4) + rword;   // row io at + io * 2 * RS
#if SM_STRIP_VMASK
        // edge strips: the AD is summed unmasked and V is cleared afterwards at the columns outside [clo, chi) (what
        // they hold is never read before the next clear): 4 VALU per register and step instead of a select per
        // column and row.  mw[i]: bit c of the 32 columns 32 i .. 32 i + 31 set where the column counts
        uint32_t mw[4];
        if constexpr (EDGE) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                int a0 = clo - 32 * i, a1 = chi - 32 * i;
                asm volatile("" : "+v"(a0), "+v"(a1));   // per step, not hoisted into live registers
                a0 = min(max(a0, 0), 32);
                a1 = min(max(a1, 0), 32);
                const uint32_t lo = a0 >= 32 ? 0u : ~0u << a0;
                const uint32_t hi = a1 >= 32 ? ~0u : (1u << a1) - 1u;
                mw[i] = lo & hi;
            }
        }
        int mlo = 0, mhi = 0;
#else
        // opaque copies of the mask bounds: otherwise the column compares, loop-invariant, are hoisted out of the
        // row loop into 128 SGPR pairs and spilled
        int mlo = clo, mhi = chi;
        if constexpr (EDGE) asm volatile("" : "+v"(mlo), "+v"(mhi));
#endif
        struct G { uint2 li, lo; uint32_t ri0, ri1, ro0, ro1; };
        auto load = [&](int q) SM_INL {
            G g;
            g.li = Ls[q];
            g.ri0 = Rr[2 * q];
            g.ri1 = Rr[2 * q + 1];
            if constexpr (OUT) {
                g.lo = Ls[kSQ + q];
                g.ro0 = Rr[2 * RS + 2 * q];
                g.ro1 = Rr[2 * RS + 2 * q + 1];
            }
            return g;
        };
        auto ad = [&](uint32_t l, uint32_t r, int c) SM_INL {
            const u16x2 a = as16(l), b = as16(r);
#if SM_STRIP_ADOR
            // |a - b| = (a -sat b) | (b -sat a): two packed clamped subtracts and a VOP2 or
            u16x2 e = as16(as32(__builtin_elementwise_sub_sat(a, b)) | as32(__builtin_elementwise_sub_sat(b, a)));
#else
            u16x2 e = __builtin_elementwise_max(a, b) - __builtin_elementwise_min(a, b);
#endif
            if constexpr (EDGE && !SM_STRIP_VMASK) {
                e.x = (c >= mlo && c < mhi) ? e.x : (unsigned short)0;
                e.y = (c + 1 >= mlo && c + 1 < mhi) ? e.y : (unsigned short)0;
            }
            return e;
        };
        G g[kSQ];
#pragma unroll
        for (int q = 0; q < SM_STRIP_LA && q < kSQ; ++q) g[q] = load(q);
#pragma unroll
        for (int q = 0; q < kSQ; ++q) {
            if (q + SM_STRIP_LA < kSQ) g[q + SM_STRIP_LA] = load(q + SM_STRIP_LA);
            const G& cur = g[q];
            u16x2 v0 = as16(V[2 * q]) + ad(cur.li.x, cur.ri0, 4 * q);
            u16x2 v1 = as16(V[2 * q + 1]) + ad(cur.li.y, cur.ri1, 4 * q + 2);
            if constexpr (OUT) {
                v0 = v0 - ad(cur.lo.x, cur.ro0, 4 * q);
                v1 = v1 - ad(cur.lo.y, cur.ro1, 4 * q + 2);
            }
            V[2 * q] = as32(v0);
            V[2 * q + 1] = as32(v1);
#if SM_STRIP_VMASK
            if constexpr (EDGE) {
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    // columns 4q + 2k, 4q + 2k + 1: bit (4q + 2k) % 32 of word q / 8, each bit to a u16 half
                    const uint32_t w = mw[q >> 3];
                    const int b = (4 * q + 2 * k) & 31;
                    const uint32_t m0 = (uint32_t)__builtin_amdgcn_sbfe((int)w, b, 1);
                    const uint32_t m1 = (uint32_t)__builtin_amdgcn_sbfe((int)w, b + 1, 1);
                    V[2 * q + k] &= (m0 & 0xFFFFu) | (m1 & 0xFFFF0000u);
                }
            }
#endif
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    // S +/- V(c), c static: one SDWA add / sub reading the u16 half in place (an extracted copy of every V(c) would
    // stay live across the 2R + 1 columns between its two uses)
    auto sacc = [&](uint32_t S, int c, auto add) SM_INL -> uint32_t {
        const uint32_t w = V[c >> 1];
        uint32_t o;
        if constexpr (decltype(add)::value) {
            if (c & 1)
                asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
                    : "=v"(o) : "v"(S), "v"(w));
            else
                asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
                    : "=v"(o) : "v"(S), "v"(w));
        } else {
            if (c & 1)
                asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
                    : "=v"(o) : "v"(S), "v"(w));
            else
                asm("v_sub_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
                    : "=v"(o) : "v"(S), "v"(w));
        }
        return o;
    };

    // the row's S, keys and the wave minimum of each output; lane 8i of group g stores output 8g + i's minimum
    auto row_wta = [&](int wb, auto omask) SM_INL {
        constexpr bool OMASK = decltype(omask)::value;
        // output j counts when x0 + j < W and jl <= j <= jd: d <= W - x0 - j (vm 0) or d <= x0 + j (vm 1); opaque
        // for the same reason as update's bounds
        int jw = W - x0, jd = vm == 0 ? W - x0 - d : (1 << 30), jl = vm == 0 ? -(1 << 30) : d - x0, jr = d - x0;
        if constexpr (OMASK) asm volatile("" : "+v"(jw), "+v"(jd), "+v"(jl), "+v"(jr));
        // RIGHT: LDS byte address of this lane's slot for output 0 of the row buffer wb
        [[maybe_unused]] const uint32_t rbase =
            (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t*)(rrow + wb * RN + roc);
        // the groups' minima, stored after the last group: a store per group would end the basic block (the
        // 8-lane mask), serialising each group's butterfly behind the next group's window sums
        uint32_t res[NG];
        auto grp = [&](uint32_t S, int g) SM_INL -> uint32_t {
            uint32_t k[8];
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const int j = 8 * g + m;          // output x0 + j, window columns j .. j + 2R
                if (j < SW) {
                    S = sacc(S, j + 2 * R, std::true_type{});
                    uint32_t key = (S << 8) | dd;
                    if constexpr (RIGHT) {
                        // right candidate u = x - d: valid for x >= d and x < W (lanes past the slice: ~0).  An
                        // inline ds_min_u32 with an immediate offset: the C++ atomic under a select became a
                        // divergent branch per output (and 230 VGPRs); LDS ops complete in order, so the compiler's
                        // own waitcnts stay conservative, and the step ends with an explicit lgkmcnt(0)
                        uint32_t kr = key | dmask;
                        if constexpr (OMASK) kr = (j < jw && j >= jr) ? kr : 0xFFFFFFFFu;
                        asm volatile("ds_min_u32 %0, %1 offset:%2" : : "v"(rbase), "v"(kr), "i"(4 * j) : "memory");
                    }
                    if constexpr (OMASK) key = (j < jw && j <= jd && j >= jl) ? key | dmask : 0xFFFFFFFFu;   // Device.cu:44
                    k[m] = key;
                    S = sacc(S, j, std::false_type{});
                } else {
                    k[m] = 0xFFFFFFFFu;
                }
            }
            // 8 outputs x 64 lanes -> every lane of the 8-lane block i holds output i's minimum over the wave:
            // lanes 32 apart (permlane32 swap: outputs m | m + 4 in the two halves), 16 apart (permlane16 swap:
            // rows hold outputs m, m + 2, m + 4, m + 6), 8 apart (a row_shr / row_shl:8 exchange of the two
            // registers' half rows), then within the 8 lanes (DPP row_half_mirror, quad xor 1, quad xor 2)
            uint32_t m4[4], m2[2];
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const auto t = __builtin_amdgcn_permlane32_swap(k[m], k[m + 4], false, false);
                m4[m] = min((uint32_t)t[0], (uint32_t)t[1]);
            }
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                const auto t = __builtin_amdgcn_permlane16_swap(m4[m], m4[m + 2], false, false);
                m2[m] = min((uint32_t)t[0], (uint32_t)t[1]);
            }
            // row r of m2[0] holds output 2r, of m2[1] output 2r + 1
            const uint32_t a = (uint32_t)__builtin_amdgcn_update_dpp((int)m2[0], (int)m2[1], 0x118, 0xF, 0xC, false);
            const uint32_t b = (uint32_t)__builtin_amdgcn_update_dpp((int)m2[1], (int)m2[0], 0x108, 0xF, 0x3, false);
            uint32_t n = min(a, b);               // lanes 0-7 of row r: output 2r, lanes 8-15: 2r + 1
            n = dpp_min<0x141>(n, n);
            n = dpp_min<0xB1>(n, n);
            res[g] = dpp_min<0x4E>(n, n);
            return S;
        };
        // window sum of output 8 g0 - 1's successor: columns 8 g0 .. 8 g0 + 2R - 1
        auto init = [&](int g0) SM_INL -> uint32_t {
            uint32_t S = s0;
#pragma unroll
            for (int c = 8 * g0; c < 8 * g0 + 2 * R; ++c) S = sacc(S, c, std::true_type{});
            return S;
        };
        if constexpr (SM_STRIP_CH2 != 0 && NG >= 2) {
            constexpr int NGA = (NG + 1) / 2;
            uint32_t SA = init(0), SB = init(NGA);
#pragma unroll
            for (int i = 0; i < NGA; ++i) {
                SA = grp(SA, i);
                if (NGA + i < NG) SB = grp(SB, NGA + i);
            }
        } else {
            uint32_t S = init(0);
#pragma unroll
            for (int g = 0; g < NG; ++g) S = grp(S, g);
        }
        if ((lane & 7) == 0) {
            uint32_t* wm = wmin + (wb * nw + wave) * (NG * 8) + (lane >> 3);
#pragma unroll
            for (int g = 0; g < NG; ++g) wm[8 * g] = res[g];
        }
    };
    // the previous row's map: the minimum over the waves and the seed (Device.cu:37-38, 63)
    auto emit = [&](int wb, int y) SM_INL {
        if constexpr (RIGHT) {   // the row's right candidates into the frame's right keys, the LDS row cleared
            uint32_t* rr = rrow + wb * RN;
            uint32_t* dst = rk + ((int64_t)f * H + y) * W + (x0 - DP);
            for (int i = tid; i < RN; i += nt) {
                const uint32_t v = rr[i];
                if (v != 0xFFFFFFFFu) atomicMin(dst + i, v);   // valid keys only: 0 <= u < W
                rr[i] = 0xFFFFFFFFu;
            }
        }
        for (int j = tid; j < SW; j += nt) {
            const int x = x0 + j;
            if (x >= W) continue;
            uint32_t best = seed;
            for (int w = 0; w < nw; ++w) best = min(best, wmin[(wb * nw + w) * (NG * 8) + j]);
            if (disp) disp[(int64_t)f * ostride + (int64_t)y * opitch + x] = best < thresh ? (uint8_t)(best & 0xFFu) : (uint8_t)0;
            if (keys) keys[((int64_t)f * H + y) * W + x] = best;
        }
    };

    // step s: row t_in = y0 - R + s enters V; from s = 2R + 1 row t_in - 2R - 1 leaves; from s = 2R output row
    // y0 + s - 2R is complete
    const int nsteps = 2 * R + (y1 - y0);
    if (nsteps <= 2 * R) return;
#ifndef SM_STRIP_SKIP
#define SM_STRIP_SKIP 0   // timing only (wrong maps): 1 no staging, 2 no V update, 4 no row WTA
#endif
    // step s reads rows y0 - R + s (in) and y0 - 3R - 1 + s (out; staged as zeros before step 2R + 1, where nothing
    // leaves V: the steps from 2R on then run one uniform body)
    auto rows_of = [&](int st, int& yin, int& yout) SM_INL {
        yin = y0 - R + st;
        yout = st >= 2 * R + 1 ? y0 - 3 * R - 1 + st : -1;
    };
    int yi, yo;
    rows_of(0, yi, yo);
    fetch(yi, yo);
    store(0);
    if constexpr (RIGHT)
        for (int i = tid; i < 2 * RN; i += nt) rrow[i] = 0xFFFFFFFFu;
    if (nsteps > 1) {
        rows_of(1, yi, yo);
        fetch(yi, yo);
    }
    __syncthreads();
#ifdef SM_STRIP_PROF
    // timing-only instrumentation: shader-clock cycles per phase over all steps, summed per wave; block
    // (SM_STRIP_PROF_X, 0, 0)'s wave 0 writes them over the first map bytes of frame 0 at the end
    uint64_t prof[5] = {0, 0, 0, 0, 0};
#define SM_STAMP(v) do { __builtin_amdgcn_sched_barrier(0); v = __builtin_amdgcn_s_memtime(); __builtin_amdgcn_sched_barrier(0); } while (0)
#else
#define SM_STAMP(v) do { } while (0)
#endif
    auto step = [&](int st, auto edge, auto with_out) SM_INL {
        const int buf = st & 1;
        [[maybe_unused]] uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
        SM_STAMP(t0);
        if (!(SM_STRIP_SKIP & 1) && st + 1 < nsteps) {
            store(buf ^ 1);
            if (st + 2 < nsteps) {
                int a, b;
                rows_of(st + 2, a, b);
                fetch(a, b);
            }
        }
        SM_STAMP(t1);
        if (!(SM_STRIP_SKIP & 2)) update(buf, edge, with_out);
        SM_STAMP(t2);
        if (decltype(with_out)::value && (SM_STRIP_ONELOOP == 0 || st >= 2 * R)) {
            if (!(SM_STRIP_SKIP & 4)) {
                const int wb = (st - 2 * R) & 1;
                row_wta(wb, edge);                                // the masked keys go with the masked columns
                SM_STAMP(t3);
                if (st > 2 * R) emit(wb ^ 1, y0 + st - 2 * R - 1);   // written in the step before, behind its barrier
            }
        }
        SM_STAMP(t4);
        if constexpr (RIGHT) asm volatile("s_waitcnt lgkmcnt(0)" : : : "memory");   // the inline ds_min_u32s
        __syncthreads();
#ifdef SM_STRIP_PROF
        uint64_t t5;
        SM_STAMP(t5);
        {
            prof[0] += t1 - t0;
            prof[1] += t2 - t1;
            prof[2] += t3 - t2;
            prof[3] += t4 - t3;
            prof[4] += t5 - t4;
        }
#endif
    };
    // the edge strips (columns outside the frame or below d, outputs past W or with invalid d) take the masked body
    // SM_STRIP_ONELOOP: one loop body for every step (the first 2R subtract staged zero rows: a third less code, but
    // 8 % slower at r = 20), else a separate add-only loop for them
    auto run = [&](auto edge) SM_INL {
        int st = 0;
        if constexpr (SM_STRIP_ONELOOP == 0)
            for (; st < 2 * R; ++st) step(st, edge, std::false_type{});
        for (; st < nsteps; ++st) step(st, edge, std::true_type{});
    };
    if (col_ok && out_ok) run(std::false_type{});
    else run(std::true_type{});
    emit((nsteps - 1 - 2 * R) & 1, y1 - 1);
#ifdef SM_STRIP_PROF
#ifndef SM_STRIP_PROF_X
#define SM_STRIP_PROF_X 0
#endif
    if (disp && blockIdx.x == SM_STRIP_PROF_X && blockIdx.y == 0 && blockIdx.z == 0 && tid == 0) {
        __syncthreads();
        for (int i = 0; i < 5; ++i) __builtin_memcpy(disp + 8 * i, &prof[i], 8);
    }
#endif
    if constexpr ((SM_STRIP_SKIP & 4) != 0) {   // keep the V update live in the timing-only build
        uint32_t t = 0;
#pragma unroll
        for (int p = 0; p < kSP; ++p) t ^= V[p];
        if (t == 0x12345u && keys) keys[0] = t;
    }
}

int device_cus() {
    static const int n = [] {
        int dev = 0, cus = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
        return cus;
    }();
    return n;
}

// Row bands, one round of workgroups (a second, partial round would leave most of the chip idle while it runs):
// interior strips in nb bands, edge strips in nbe, chosen to minimise the longer of the two band walks, a band of
// height h costing (h + 2r) row steps (its first 2r steps only build V), an edge step SM_STRIP_EDGE_COST % of an
// interior one (the masked body), over the (nb, nbe) whose workgroups all fit at once.
#ifndef SM_STRIP_EDGE_COST
#define SM_STRIP_EDGE_COST 150
#endif
#ifndef SM_STRIP_FILL
#define SM_STRIP_FILL 100   // percent of the resident workgroups the bands aim at
#endif
struct StripGrid {
    int EL, NI, ER;   // left edge, interior and right edge strips
    int nb, nbe;      // bands per interior / edge strip
};

StripGrid strip_grid(const MatchArgs& a, int R, int SW, int frames, int resident) {
    StripGrid g{0, 0, 0, 1, 1};
    const int strips = (a.W + SW - 1) / SW;
    // the kernel's col_ok && out_ok, per strip: the interior strips are one contiguous run
    auto interior = [&](int st) {
        const int x0 = st * SW, cs0 = x0 - R;
        return cs0 >= a.d_hi - 1 && cs0 + kSC <= a.W && x0 + SW <= a.W &&
               (a.valid_mode == 0 ? (a.d_hi - 1) <= a.W - (x0 + SW - 1) : (a.d_hi - 1) <= x0);
    };
    while (g.EL < strips && !interior(g.EL)) ++g.EL;
    g.NI = 0;
    while (g.EL + g.NI < strips && interior(g.EL + g.NI)) ++g.NI;
    g.ER = strips - g.EL - g.NI;
    const int ne = g.EL + g.ER;
    const int nb_max = std::max(1, a.H / (4 * R)), nbe_max = std::max(1, a.H / (2 * R));
    int64_t best = -1;
    for (int nb = 1; nb <= (g.NI ? nb_max : 1); ++nb)
        for (int nbe = 1; nbe <= (ne ? nbe_max : 1); ++nbe) {
            const int64_t blocks = ((int64_t)ne * nbe + (int64_t)g.NI * nb) * frames;
            if (blocks > resident && !(nb == 1 && nbe == 1)) continue;
            const int64_t ti = g.NI ? (int64_t)((a.H + nb - 1) / nb + 2 * R) * 100 : 0;
            const int64_t te = ne ? (int64_t)((a.H + nbe - 1) / nbe + 2 * R) * SM_STRIP_EDGE_COST : 0;
            const int64_t t = std::max(ti, te);
            if (best < 0 || t < best) {
                best = t;
                g.nb = nb;
                g.nbe = nbe;
            }
        }
    return g;
}

template <int R, bool RIGHT>
hipError_t launch_strip_r(const MatchArgs& a, int batch, hipStream_t s, uint32_t* rk) {
    constexpr int SW = kSC - 2 * R;
    const int nd = a.d_hi - a.d_lo;
    const int nw = (nd + 63) / 64;
    const int DP = ((a.d_hi - 1) + 3) & ~3;
    const int RW = r_words(DP, a.d_lo), RS = r_stride(RW);
    const size_t lds = (size_t)2 * stage_bytes(RS) + (size_t)2 * nw * ((SW + 7) / 8) * 8 * 4 +
                       (RIGHT ? (size_t)2 * (SW + DP) * 4 : 0);
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, strip_kernel<R, RIGHT>, 64 * nw, lds) != hipSuccess ||
        per_cu <= 0)
        per_cu = 1;
    const StripGrid g = strip_grid(a, R, SW, batch, per_cu * device_cus() * SM_STRIP_FILL / 100);
    const int64_t nblk = (int64_t)(g.EL + g.ER) * g.nbe + (int64_t)g.NI * g.nb;
    if (nblk > 0x7FFFFFFF || batch > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL((strip_kernel<R, RIGHT>), dim3((unsigned)nblk, 1u, (unsigned)batch), dim3(64 * nw), lds, s,
                       a.left, a.right, a.frame_stride, a.W, a.H, a.pitch, a.d_lo, a.d_hi, g.EL, g.NI, g.nb, g.nbe,
                       a.valid_mode, DP, RW, RS, nw, a.seed_key, a.thresh_key, a.disp, a.out_pitch, a.out_frame_stride,
                       a.keys, rk);
    return hipGetLastError();
}

template <int R, bool RIGHT>
hipError_t dispatch_strip(const MatchArgs& a, int batch, hipStream_t s, uint32_t* rk) {
    if constexpr (R > kStripMaxRadius) {
        return hipErrorInvalidValue;
    } else {
        if (a.radius == R) return launch_strip_r<R, RIGHT>(a, batch, s, rk);
        return dispatch_strip<R + 1, RIGHT>(a, batch, s, rk);
    }
}

}  // namespace

#ifndef SM_STRIP_RIGHT_TU
bool strip_path(const MatchArgs& a) {
    static const bool on = [] {
#ifdef SM_STRIP_OFF
        return false;   // A/B builds
#endif
        const char* e = getenv("SM_WIDE_STRIP");
        return !(e && e[0] == '0');
    }();
    return on && a.radius >= kStripMinRadius && a.radius <= kStripMaxRadius && (a.valid_mode == 0 || a.valid_mode == 1) &&
           a.d_hi > a.d_lo && a.d_hi <= kMaxDisp && a.W >= 4 && a.H >= 1;
}

hipError_t launch_box_match_strip(const MatchArgs& a, int batch, hipStream_t s) {
    if (!strip_path(a) || batch <= 0) return hipErrorInvalidValue;
    return dispatch_strip<kStripMinRadius, false>(a, batch, s, nullptr);
}
#else
// bm_strip_lr.hip: the instantiations with the right view, compiled in their own translation unit
hipError_t launch_box_match_strip_lr(const MatchArgs& a, int batch, uint32_t* right_keys, hipStream_t s) {
    if (!strip_path(a) || a.valid_mode != 0 || a.d_lo != 0 || !right_keys || batch <= 0) return hipErrorInvalidValue;
    return dispatch_strip<kStripMinRadius, true>(a, batch, s, right_keys);
}
#endif

}  // namespace sm
