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
//   S1V  lane = P column; waves split the A rows: prefix T += AD*(L + 2^20) -> packed CS rows
//   S1H  thread = (A row, segment): running Sp / SIp -> a, b
//   S2V  thread = (A column, 8-row group): running float sums of a, b over 2R+1 rows
//   S2H  thread = (output row, segment): running sums -> N*q = sum(a) I + sum(b) -> WTA in registers
// The stages of consecutive disparities are software-pipelined with separate LDS buffers, so one
// iteration runs {S1V(d), S2V(d-1)} | barrier | {S1H(d), S2H(d-1)} | barrier: two workgroup
// barriers per d instead of four.  The guide statistics (SI = sum L, SII = sum L^2, N) come from
// S1V/S1H on AD := L (R band read as 0), once per tile.
//
// Fused right view (RIGHT = true, the LR check): STMatching derives the right-view cost from the
// left one, C_R(y, u, d) = C_L(y, u + d, d) (GetRightMatchingCostFromLeft, StereoHelper.cpp:156-180),
// and takes its WTA with strict < from d = 0 and no threshold (StereoHelper.cpp:131-154).  S2H makes
// every output's q (= N*q / N) at disparity d a candidate for the right pixel u = x - d:
//   key = (int)(q * 2^14) << 8 | position      (q clamped to [-512, 512), truncated: error < 6.2e-5)
// and keeps, per thread, one key slot per output; slot j holds u = xs + j - d at step d.  After each
// step the top slot can gain nothing more from this segment: it is passed to the next segment of
// the row (the lane to its right, DPP row_shr:1) whose new bottom slot is that same u.  The last
// segment of the row writes it to HBM (gpart), and guided_right_reduce_kernel takes the minimum
// over the ~(D + 8 SW2) / TW tiles covering each u.  The position field is the output column within
// the tile, kept relative to the current segment (+ SW2 * (7 - s)) so that keys created in this
// segment need no per-lane constant; each hop subtracts SW2.  Ties (equal keys) resolve to the
// smaller column, i.e. the smaller d, as the reference's strict < does.
#include <climits>
#include <type_traits>

#include "bm_common.h"
#include "bm_guided.h"

// Every addtid store sets M0 inside its own asm statement and names it clobbered (a
// separate M0 write could be separated from its stores by a compiler-generated M0 use);
// tools/check_lds_barriers.py --m0 checks the ISA for it.  Clang's reserved-register warning about
// the clobber is noise here.
#pragma clang diagnostic ignored "-Winline-asm"

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

// disparities per staged right band: 32 keeps LDS <= 52.3 KB at r = 5 with the bank-spread CS stride
// (3 workgroups/CU; measured occupancy drops to 2 at 54 KB)
constexpr int kBandChunk = 32;
constexpr uint32_t kPOne = 1u << 20;   // S1V multiplier L | 2^20: low 20 bits sum I*p, high 12 bits sum p
constexpr uint32_t kPLow = kPOne - 1;

// Phase-1 wave roles (round 3): S1V on 2 waves over half the A rows each and S2V on the other 2 over
// 16 output rows each, instead of both stages on all 4 waves over a quarter: S1V's integer running sums
// re-walk their 2R-row warm-up once per wave, so two taller strips walk 62 P rows instead of 84, and
// S2V reads each a/b row once per 16-row strip (52 reads instead of 72; its float sums still restart
// every 8 rows, so the maps do not change).  Roles rotate with the workgroup index, so the
// co-resident workgroups of a CU put their S1V waves on different SIMDs.
#ifndef SM_G_ROLES
#define SM_G_ROLES 1
#endif
constexpr bool kGuidedRoles = SM_G_ROLES != 0;

// SM_G_ACC (round 6, default 1): S1H's window sums of the packed columns without unpacking SIp per column (s1h
// below): 152 -> 142 VALU per wave and d, 459.9 -> 452.9 us per 1080p guided frame, guided + LR 511.1 -> 505.0,
// maps bit-identical (profiles/microbench/r06_guided_acc_pk_ab.txt).  0 keeps the unpacking form for A/B.
// Not kept (same file): S2V's (a, b) running sums as v_pk_add_f32 pairs, 100 -> 50 VALU but 462.1 us (+0.5 %):
// a packed f32 add costs the SIMD about what the two adds it replaces do.
#ifndef SM_G_ACC
#define SM_G_ACC 1
#endif

// SM_G_MARK=1 (analysis builds only, tools/isa_stage_mix.py): an assembly comment at each stage's entry and exit,
// so the per-stage VALU mix can be read from the ISA.  The empty asm statements also act as scheduling
// barriers, so the marked build is for counting, not for timing.
#ifndef SM_G_MARK
#define SM_G_MARK 0
#endif
#if SM_G_MARK
#define G_MARK(tag) asm volatile(";@stage " tag ::: "memory")
#else
#define G_MARK(tag) ((void)0)
#endif

// Taller tiles (round 4: 48 rows on 6 waves, 96 rows on one 12-wave workgroup per CU) cut the halo but
// lost occupancy and ran 1.9x / 1.3x slower; the variants were removed in round 5
// (git history: SM_G_TALL / SM_G_TALL_RIGHT before commit "guided: drop the measured tall-tile variants").
template <int R, bool ROLES = kGuidedRoles>
struct GeoF {
    static constexpr int NT = kT;                            // threads per workgroup
    static constexpr int NWV = NT / 64;                      // waves per workgroup
    static constexpr int TW = 64 - 4 * R;
    static constexpr int TH = 32;
    static constexpr int AW = TW + 2 * R;
    static constexpr int AH = TH + 2 * R;
    static constexpr int PH = TH + 4 * R;
    // phase 1 runs S1V on SV waves and S2V on the other NWV - SV (kGuidedRoles), else both on all NWV
    static constexpr int SV = ROLES ? NWV / 2 : NWV;
    static constexpr int RPS = TH / (ROLES ? NWV - SV : NWV);   // output rows per S2V wave
    static constexpr int RPW = (AH + SV - 1) / SV;           // A rows per wave in S1V
    static constexpr int NV = RPW + 2 * R;                   // P rows walked per wave
    static constexpr int AHP = SV * RPW;                     // cs rows incl. the last wave's pad rows
    static constexpr int PHP = SV * RPW + 2 * R;             // staged P rows incl. pad rows (>= PH)
    // S1H segments per A row
    static constexpr int NSEG1 = NT / AH;
    static constexpr int SW1 = (AW + NSEG1 - 1) / NSEG1;
    static constexpr int SW2 = (TW + 7) / 8;                 // S2H outputs per thread
    static constexpr int CSS0 = (NSEG1 * SW1 + 2 * R) > 64 ? (NSEG1 * SW1 + 2 * R) : 64;
    // strides kept minimal so that r <= 5 fits 3 workgroups per CU (<= 52 KB): an odd CS stride
    // spreads the S1H rows over the banks (padding mm / a/b rows for banks measured slower).
    // S2H threads whose last outputs fall past TW read beyond their mm row (the next row, or abp
    // after the last one) into values that only reach those discarded outputs.  S1H writes every
    // one of its NSEG1*SW1 columns (those past AW are never read), so a/b rows are that wide.
    // S1H thread tid reads CS dword h1i*CSS + h1s*SW1 + k (h1i = tid / NSEG1, h1s = tid % NSEG1):
    // with SW1 odd and CSS == NSEG1*SW1 (mod 32) that is SW1*tid + k (mod 32), a distinct bank for
    // each lane of a 32-lane group (the odd CS stride left 2-way conflicts, 25 % of LDS cycles)
    static constexpr int CSS_B = CSS0 + ((NSEG1 * SW1 - CSS0) % 32 + 32) % 32;
    static constexpr int CSS_OLD = CSS0 + 1;
    static constexpr int MSA_ = AW % 4 == 2 ? AW : AW + ((6 - AW % 4) % 4);
    static constexpr int lds_for(int css) {
        return ((((AHP * css * 4 > PHP * 64 ? AHP * css * 4 : PHP * 64) + 15) & ~15)) + 2 * TH * MSA_ * 4 +
               AH * (NSEG1 * SW1 > AW ? NSEG1 * SW1 : AW) * 8 + ((PHP * (64 + kBandChunk) + 15) & ~15);
    }
    static constexpr int CSS =
        (SW1 % 2 == 1 && lds_for(CSS_B) <= (R >= 6 ? 81920 : 53248)) ? CSS_B
                                                                                                       : CSS_OLD;
    // mm is two float planes (sum a, sum b), rows of MSA floats.  S2V stores them lane-consecutively
    // (ds_write_addtid_b32, 2 LDS cycles per 64 lanes against 6 for a float2 ds_write_b64); S2H reads
    // its segment as ds_read_b64 pairs.  MSA = 2 (mod 4): the b64 reads of 32 lanes (32 rows, one
    // segment; or, with the fused right view, rows {G, G+8, G+16, G+24} x 8 segments) fall on
    // distinct bank pairs.
    static constexpr int MSA = AW % 4 == 2 ? AW : AW + ((6 - AW % 4) % 4);
    static constexpr int ABS = NSEG1 * SW1 > AW ? NSEG1 * SW1 : AW;   // float2 per a/b row
    static constexpr int RBW = 64 + kBandChunk;              // right band bytes per P row (one d-chunk)
    static constexpr int CS_BYTES = ((AHP * CSS * 4 > PHP * 64 ? AHP * CSS * 4 : PHP * 64) + 15) & ~15;  // lt aliases cs
    static constexpr int MM_PLANE = TH * MSA * 4;            // bytes per mm plane
    static constexpr int MM_BYTES = 2 * MM_PLANE;
    static constexpr int AB_BYTES = AH * ABS * 8;
    static constexpr int RB_BYTES = (PHP * RBW + 15) & ~15;
    static constexpr int LDS = CS_BYTES + MM_BYTES + AB_BYTES + RB_BYTES;
};

typedef float vf2 __attribute__((ext_vector_type(2)));   // a VGPR pair for asm operands

// S2H's mm loads: N ds_read_b64 from plane A at `addr` and N from plane B at addr + PLANE, all in
// flight before one s_waitcnt, written out in asm because the compiler pairs neighbouring b64 loads
// into ds_read2_b64 (8 LDS cycles per pair against 2 per ds_read_b64, MI355X_MICROARCH.md LDS table).
// The block waits for its own loads, so its outputs are ready when it ends.

template <int N, int PLANE>
__device__ __forceinline__ typename std::enable_if<N == 4>::type s2h_load_impl(uint32_t addr, vf2 (&a)[N], vf2 (&b)[N]) {
    asm volatile("ds_read_b64 %0, %8 offset:0\n\t"
                 "ds_read_b64 %1, %8 offset:8\n\t"
                 "ds_read_b64 %2, %8 offset:16\n\t"
                 "ds_read_b64 %3, %8 offset:24\n\t"
                 "ds_read_b64 %4, %8 offset:%9\n\t"
                 "ds_read_b64 %5, %8 offset:%10\n\t"
                 "ds_read_b64 %6, %8 offset:%11\n\t"
                 "ds_read_b64 %7, %8 offset:%12\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3]), "=&v"(b[0]), "=&v"(b[1]), "=&v"(b[2]), "=&v"(b[3])
                 : "v"(addr), "i"(PLANE + 0), "i"(PLANE + 8), "i"(PLANE + 16), "i"(PLANE + 24)
                 : "memory");
}

template <int N, int PLANE>
__device__ __forceinline__ typename std::enable_if<N == 5>::type s2h_load_impl(uint32_t addr, vf2 (&a)[N], vf2 (&b)[N]) {
    asm volatile("ds_read_b64 %0, %10 offset:0\n\t"
                 "ds_read_b64 %1, %10 offset:8\n\t"
                 "ds_read_b64 %2, %10 offset:16\n\t"
                 "ds_read_b64 %3, %10 offset:24\n\t"
                 "ds_read_b64 %4, %10 offset:32\n\t"
                 "ds_read_b64 %5, %10 offset:%11\n\t"
                 "ds_read_b64 %6, %10 offset:%12\n\t"
                 "ds_read_b64 %7, %10 offset:%13\n\t"
                 "ds_read_b64 %8, %10 offset:%14\n\t"
                 "ds_read_b64 %9, %10 offset:%15\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3]), "=&v"(a[4]), "=&v"(b[0]), "=&v"(b[1]), "=&v"(b[2]), "=&v"(b[3]), "=&v"(b[4])
                 : "v"(addr), "i"(PLANE + 0), "i"(PLANE + 8), "i"(PLANE + 16), "i"(PLANE + 24), "i"(PLANE + 32)
                 : "memory");
}

template <int N, int PLANE>
__device__ __forceinline__ typename std::enable_if<N == 6>::type s2h_load_impl(uint32_t addr, vf2 (&a)[N], vf2 (&b)[N]) {
    asm volatile("ds_read_b64 %0, %12 offset:0\n\t"
                 "ds_read_b64 %1, %12 offset:8\n\t"
                 "ds_read_b64 %2, %12 offset:16\n\t"
                 "ds_read_b64 %3, %12 offset:24\n\t"
                 "ds_read_b64 %4, %12 offset:32\n\t"
                 "ds_read_b64 %5, %12 offset:40\n\t"
                 "ds_read_b64 %6, %12 offset:%13\n\t"
                 "ds_read_b64 %7, %12 offset:%14\n\t"
                 "ds_read_b64 %8, %12 offset:%15\n\t"
                 "ds_read_b64 %9, %12 offset:%16\n\t"
                 "ds_read_b64 %10, %12 offset:%17\n\t"
                 "ds_read_b64 %11, %12 offset:%18\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3]), "=&v"(a[4]), "=&v"(a[5]), "=&v"(b[0]), "=&v"(b[1]), "=&v"(b[2]), "=&v"(b[3]), "=&v"(b[4]), "=&v"(b[5])
                 : "v"(addr), "i"(PLANE + 0), "i"(PLANE + 8), "i"(PLANE + 16), "i"(PLANE + 24), "i"(PLANE + 32), "i"(PLANE + 40)
                 : "memory");
}

template <int N, int PLANE>
__device__ __forceinline__ typename std::enable_if<N == 7>::type s2h_load_impl(uint32_t addr, vf2 (&a)[N], vf2 (&b)[N]) {
    asm volatile("ds_read_b64 %0, %14 offset:0\n\t"
                 "ds_read_b64 %1, %14 offset:8\n\t"
                 "ds_read_b64 %2, %14 offset:16\n\t"
                 "ds_read_b64 %3, %14 offset:24\n\t"
                 "ds_read_b64 %4, %14 offset:32\n\t"
                 "ds_read_b64 %5, %14 offset:40\n\t"
                 "ds_read_b64 %6, %14 offset:48\n\t"
                 "ds_read_b64 %7, %14 offset:%15\n\t"
                 "ds_read_b64 %8, %14 offset:%16\n\t"
                 "ds_read_b64 %9, %14 offset:%17\n\t"
                 "ds_read_b64 %10, %14 offset:%18\n\t"
                 "ds_read_b64 %11, %14 offset:%19\n\t"
                 "ds_read_b64 %12, %14 offset:%20\n\t"
                 "ds_read_b64 %13, %14 offset:%21\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3]), "=&v"(a[4]), "=&v"(a[5]), "=&v"(a[6]), "=&v"(b[0]), "=&v"(b[1]), "=&v"(b[2]), "=&v"(b[3]), "=&v"(b[4]), "=&v"(b[5]), "=&v"(b[6])
                 : "v"(addr), "i"(PLANE + 0), "i"(PLANE + 8), "i"(PLANE + 16), "i"(PLANE + 24), "i"(PLANE + 32), "i"(PLANE + 40), "i"(PLANE + 48)
                 : "memory");
}

template <int N, int PLANE>
__device__ __forceinline__ typename std::enable_if<N == 8>::type s2h_load_impl(uint32_t addr, vf2 (&a)[N], vf2 (&b)[N]) {
    asm volatile("ds_read_b64 %0, %16 offset:0\n\t"
                 "ds_read_b64 %1, %16 offset:8\n\t"
                 "ds_read_b64 %2, %16 offset:16\n\t"
                 "ds_read_b64 %3, %16 offset:24\n\t"
                 "ds_read_b64 %4, %16 offset:32\n\t"
                 "ds_read_b64 %5, %16 offset:40\n\t"
                 "ds_read_b64 %6, %16 offset:48\n\t"
                 "ds_read_b64 %7, %16 offset:56\n\t"
                 "ds_read_b64 %8, %16 offset:%17\n\t"
                 "ds_read_b64 %9, %16 offset:%18\n\t"
                 "ds_read_b64 %10, %16 offset:%19\n\t"
                 "ds_read_b64 %11, %16 offset:%20\n\t"
                 "ds_read_b64 %12, %16 offset:%21\n\t"
                 "ds_read_b64 %13, %16 offset:%22\n\t"
                 "ds_read_b64 %14, %16 offset:%23\n\t"
                 "ds_read_b64 %15, %16 offset:%24\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3]), "=&v"(a[4]), "=&v"(a[5]), "=&v"(a[6]), "=&v"(a[7]), "=&v"(b[0]), "=&v"(b[1]), "=&v"(b[2]), "=&v"(b[3]), "=&v"(b[4]), "=&v"(b[5]), "=&v"(b[6]), "=&v"(b[7])
                 : "v"(addr), "i"(PLANE + 0), "i"(PLANE + 8), "i"(PLANE + 16), "i"(PLANE + 24), "i"(PLANE + 32), "i"(PLANE + 40), "i"(PLANE + 48), "i"(PLANE + 56)
                 : "memory");
}

template <int N, int PLANE>
__device__ __forceinline__ void s2h_load(uint32_t addr, float (&va)[2 * N], float (&vb)[2 * N]) {
    vf2 a[N], b[N];
    s2h_load_impl<N, PLANE>(addr, a, b);
#pragma unroll
    for (int i = 0; i < N; ++i) {
        va[2 * i] = a[i].x;
        va[2 * i + 1] = a[i].y;
        vb[2 * i] = b[i].x;
        vb[2 * i + 1] = b[i].y;
    }
}

// r >= 6 needs > 168 VGPRs without spilling: 2 waves/SIMD there, 3 elsewhere; with the fused right
// view r = 3 (7 outputs per S2H thread) spills at 168 and also runs at 2
// SM_G_ROLES_RIGHT: the phase-1 wave roles in the right-view kernel too.  2 (default): at r = 0, 1, 4, 5,
// where the kernel keeps 3 waves/SIMD with them (<= 168 VGPRs: the output guide values packed as f16
// pairs and one validity register, LEAN below), and at r = 3, whose right view runs 2 waves/SIMD either
// way (598.4 vs 618.8 us per 1080p frame); not at r = 2 (spills at 3 waves/SIMD); 1 (A/B only): every
// radius, at 2 waves/SIMD; 0: never.
// Same box, guided + LR, 1080p D=128 32 frames per call, us per frame: r = 5 549.1 -> 523.0, r = 4
// 532.7 -> 518.9, r = 1 373.0 -> 368.4; 4K D=192 8 frames, r = 5: 3238 -> 3083; maps bit-identical.
// 1 ran 552 -> 650 (round 3, 2 waves/SIMD)
#ifndef SM_G_ROLES_RIGHT
#define SM_G_ROLES_RIGHT 2
#endif
template <int R>
constexpr bool kRolesRight = SM_G_ROLES_RIGHT == 1 || (SM_G_ROLES_RIGHT == 2 && R <= 5 && R != 2);
template <int R, bool RIGHT>
constexpr int kGuidedWavesPerEU = (R >= 6 || (RIGHT && (R == 3 || SM_G_ROLES_RIGHT == 1))) ? 2 : 3;

static_assert(GeoF<5, true>::LDS <= 53248 && GeoF<5, false>::LDS <= 53248, "r = 5: three workgroups per CU");

// right-key scale: q * 2^14 in a signed 24-bit field above the 8-bit position field
constexpr float kRightScale = 16384.0f;
constexpr float kRightMax = 8388607.0f;    // 2^23 - 1
constexpr float kRightMin = -8388608.0f;   // -2^23
// Fused right view's keys (round 4): v_cvt_i32_f32(q * 2^22) with its low 8 bits replaced by the position,
// i.e. floor(q * 2^14) above the position field.  The conversion saturates at |q| >= 512, so a key costs a
// multiply, one v_min_f32 (a NaN scale, outputs outside the tile or the image, becomes 4e9 and so the
// largest key), the convert and one v_and_or_b32 (the round-3 clamped (int)(q * 2^14) << 8 | position took
// v_min_f32 + v_max_f32 + multiply + convert + v_lshl_or_b32: 527.8 -> 515.4 us per 1080p frame).
constexpr float kRightScaleSat = 4194304.0f;   // 2^22

template <int R, bool RIGHT>
__global__ __launch_bounds__(kT, (kGuidedWavesPerEU<R, RIGHT>)) void guided_fused_kernel(
    const uint8_t* __restrict__ Limg, const uint8_t* __restrict__ Rimg, int W, int H, int pitch, int64_t fstride,
    int d_lo, int D, float eps, int valid_mode, uint8_t* __restrict__ disp, int out_pitch, int64_t ostride,
    int tiles_x, int tiles, int* __restrict__ gpart, int K, int* __restrict__ keys) {
    // wave roles with the fused right view only where its key chain leaves registers for the taller
    // strips (kRolesRight: r = 0, 1, 4, 5 at 3 waves/SIMD with the LEAN state below, r = 3 at 2)
    constexpr bool ROLES = kGuidedRoles && (!RIGHT || kRolesRight<R>);
    // the right view with the roles needs S2H's per-output state in fewer registers: I as f16 pairs read
    // by v_fma_mix_f32 (the same single-rounding fma, so the same maps; issued as VOP3P it costs more than
    // the v_fmac the f32 form gets: +0.8 % on the left-only kernel, which keeps that form; at r = 2 the
    // right view measured 409.6 -> 417.5 us/frame with it instead of its 5 spilled VGPRs, not kept)
    constexpr bool LEAN = RIGHT && ROLES;
    using G = GeoF<R, ROLES>;
    constexpr int NT = G::NT;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* cs = reinterpret_cast<uint32_t*>(smem);                                  // [AHP][CSS] packed sums
    uint8_t* lt = smem;                                                                 // [PHP][64] (aliases cs)
    const float* mmA = reinterpret_cast<const float*>(smem + G::CS_BYTES);             // [TH][MSA] sum a
    const float* mmB = reinterpret_cast<const float*>(smem + G::CS_BYTES + G::MM_PLANE); // [TH][MSA] sum b
    float2* abp = reinterpret_cast<float2*>(smem + G::CS_BYTES + G::MM_BYTES);         // [AH][ABS]
    uint8_t* rb = smem + G::CS_BYTES + G::MM_BYTES + G::AB_BYTES;                      // [PHP][RBW]

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: S1V's row range
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
        for (int e = tid; e < G::PHP * (G::RBW / 4); e += NT) {
            const int i = e / (G::RBW / 4), j = e - (e / (G::RBW / 4)) * (G::RBW / 4);
            *reinterpret_cast<uint32_t*>(rb + i * G::RBW + 4 * j) = ld4(Rf, py0 + i, rbase + 4 * j, W, H, pitch);
        }
    };
    stage_band(d_lo / kBandChunk);
    for (int e = tid; e < G::PHP * 16; e += NT) {
        const int i = e >> 4, j = e & 15;
        *reinterpret_cast<uint32_t*>(lt + i * 64 + 4 * j) = ld4(L, py0 + i, px0 + 4 * j, W, H, pitch);
    }
    __syncthreads();
    // phase-1 role of this wave: S1V strip `role` (role < SV) or S2V strip role - SV
    const int role = ROLES ? __builtin_amdgcn_readfirstlane((wave + (int)blockIdx.x) % G::NWV) : wave;
    const bool is_s1v = !ROLES || role < G::SV;
    // S1V state: this wave walks P rows [a0, a0 + NV) (rows past PH are pad rows that only reach
    // the pad rows of cs); lane = P column c
    const int a0 = (is_s1v ? role : 0) * G::RPW;
    const uint32_t m0_cs = __builtin_amdgcn_readfirstlane((uint32_t)(a0 * G::CSS * 4));   // cs is the first LDS block
    const int c = lane;
    const int xc = px0 + c;
    const bool col_in = xc >= 0 && xc < W;
    // m = L | 2^20: T += AD * m accumulates sum(I*p) in the low 20 bits (<= 15 * 255^2 < 2^20) and
    // sum(p) above them; v_sad_u8(m, R, -16) = |L - R| + |0x10 - 0| - 16 = AD exactly
    uint32_t mul[G::NV];
#pragma unroll
    for (int k = 0; k < G::NV; ++k) mul[k] = (uint32_t)lt[(a0 + k) * 64 + c] | kPOne;
    __syncthreads();   // lt (aliased with cs) is consumed

    // S1H's constants as SGPR operands: the compiler would fold them into literal operands, whose 64-bit
    // encodings issue slower than the 32-bit VOP2 form with an SGPR source (38 ands, 9 ors and 9 adds
    // per wave and d)
    uint32_t k_plow = kPLow, k_magic = 0x4B000000u, k_m2p20 = (uint32_t)-(int)kPOne;
    float k_magicf = -8388608.0f;
    asm volatile("" : "+s"(k_plow), "+s"(k_magic), "+s"(k_magicf), "+s"(k_m2p20));
    // S1H ownership: A row h1i, segment h1s (threads >= AH*NSEG1 idle in S1H)
    const bool h1_on = tid < G::AH * G::NSEG1;
    const int h1i = h1_on ? tid / G::NSEG1 : 0, h1s = h1_on ? tid % G::NSEG1 : 0;
    const int h1y = y0 - R + h1i;
    // S1H's a/b row segment as an LDS byte address (the kernel has no static LDS, so the dynamic
    // block starts at 0).  The stores are written as ds_write_b64 with immediate offsets: 8-B
    // aligned, serviced in 16-lane groups, where thread tid writes bank pair 9 tid + c (mod 16) at
    // r = 5 (distinct within each group).  The compiler's ds_write2_b32 for a float2 store was 2-way
    // conflicted on the (a/4) mod 32 write banks.
    uint32_t h1off = (uint32_t)(reinterpret_cast<uint8_t*>(abp + h1i * G::ABS + h1s * G::SW1) - smem);
    // S2V ownership: A column v2j = lane, output rows [8*v2g, 8*v2g + 8) with v2g = wave (one row
    // group per wave: its lanes read one contiguous a/b row span, no bank conflicts at a wrap)
    const bool v2_on = lane < G::AW;
    const int v2g = ROLES ? (is_s1v ? 0 : role - G::SV) : wave, v2j = v2_on ? lane : 0;
    const float2* v2col[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        uint32_t off = (uint32_t)(((G::RPS * v2g + k) * G::ABS + v2j) * 8);
        asm volatile("" : "+v"(off));
        v2col[k] = reinterpret_cast<const float2*>(reinterpret_cast<const uint8_t*>(abp) + off);
    }
    // S2H ownership: output row h2r, outputs [h2s*SW2, h2s*SW2 + SW2).  Rows run across lanes
    // (measured 2 % faster than segments across lanes), except with the fused right view, whose
    // key chain runs from each segment to the next lane: lane = segment + 8 * row.
    // With the right view, the 32-lane half-wave G = tid >> 5 holds rows {G, G + TH/4, G + TH/2, G + 3TH/4}
    // (8 segments each) so that its b64 reads of the mm planes fall on distinct bank pairs.
    const int h2r = RIGHT ? (((tid >> 3) & 3) * (G::TH / 4) + (tid >> 5)) : (tid % G::TH);
    const int h2s = RIGHT ? (tid & 7) : (tid / G::TH);
    // S2H's mm row segment (plane A) as an LDS byte address; plane B is MM_PLANE bytes further
    const uint32_t h2off = (uint32_t)(G::CS_BYTES + (h2r * G::MSA + h2s * G::SW2) * 4);
    // S2V's first mm row of this wave (plane A), for the add-TID stores
    const uint32_t m0_mm = __builtin_amdgcn_readfirstlane((uint32_t)(G::CS_BYTES + G::RPS * v2g * G::MSA * 4));
    const int oy = y0 + h2r;

    // per-A-pixel constants (filled by the stats pass) and per-output WTA state.
    // WTA runs on N*q = sum(a)*I + sum(b): N (output window count) is a positive per-pixel
    // constant, so the argmin is that of q; the Device.cu:37 seed 50 becomes 50*N (exact in fp32).
    // A pixels outside the image get invden = invN = 0, so their a and b come out 0.
    uint32_t nN[G::SW1];
    uint32_t nSI[G::SW1];
    float fSI[G::SW1], invden[G::SW1], invN[G::SW1];
    // output guide values I: f32, or (LEAN) f16 pairs, exact for 0..255
    float oI[LEAN ? 1 : G::SW2];
    uint32_t oIh[LEAN ? (G::SW2 + 1) / 2 : 1];
    float bq[G::SW2];
    int bdd[G::SW2], dlim[LEAN ? 1 : G::SW2];
    // LEAN: the validity d <= W - x (Device.cu:44; mirrored pass: d <= x) as d - dsgn * o <= dl0 for
    // output o, one VGPR instead of one per output (the left-hand side is wave-uniform)
    const int dsgn = valid_mode != 1 ? -1 : 1;
    const int dl0 = valid_mode != 1 ? W - (x0 + h2s * G::SW2) : x0 + h2s * G::SW2;
    // fused right view: 2^14 / N per output (NaN for outputs outside the image or the tile, whose
    // keys then clamp to the maximum), and the key slots
    float rinv[RIGHT ? G::SW2 : 1];
    int rk[RIGHT ? G::SW2 : 1];
#pragma unroll
    for (int o = 0; o < G::SW2; ++o) {
        const int x = x0 + h2s * G::SW2 + o;
        const bool ok = oy < H && x < W && h2s * G::SW2 + o < G::TW;
        const float iv = ok ? (float)L[(int64_t)oy * pitch + x] : 0.f;
        if constexpr (LEAN) {
            const uint32_t ih = __builtin_bit_cast(uint16_t, (_Float16)iv);
            oIh[o / 2] = (o % 2 == 0) ? ih : (oIh[o / 2] | (ih << 16));
        } else {
            oI[o] = iv;
            dlim[o] = valid_mode != 1 ? (W - x) : x;   // d <= W - x (Device.cu:44); mirrored pass: d <= x
        }
        bq[o] = valid_mode == 0 ? 50.0f * (float)(win_count(x, R, W) * win_count(oy, R, H)) : __builtin_huge_valf();
        bdd[o] = -256;
        if constexpr (RIGHT) {
            rinv[o] = ok ? kRightScaleSat / (float)(win_count(x, R, W) * win_count(oy, R, H))
                         : __builtin_nanf("");
            rk[o] = INT_MAX;
        }
    }

    // right-key chain: first / last segment of the row, this row's partial-key column in gpart
    const bool seg_first = h2s == 0, seg_last = h2s == 7;
    int* gdst = RIGHT ? gpart + ((int64_t)frame * tiles + t) * K * G::TH + h2r : nullptr;
    auto chain_step = [&](int k) {
        if constexpr (RIGHT) {
            const int leaving = rk[G::SW2 - 1];
#pragma unroll
            for (int j = G::SW2 - 1; j > 0; --j) rk[j] = rk[j - 1];
            // row_shr:1 = lane - 1, i.e. the previous segment of the same row (lane 8r + s)
            const int in = __builtin_amdgcn_update_dpp(INT_MAX, leaving, 0x111, 0xF, 0xF, false) - G::SW2;
            rk[0] = seg_first ? INT_MAX : in;
            // step k - d_lo: a slice pass (d_lo > 0) lays its chain out as the d_lo = 0 pass of d - d_lo does
            if (seg_last) gdst[(int64_t)(k - d_lo) * G::TH] = leaving;
        }
    };

    // ================= S1V =================
    // STATS: the guide statistics pass, AD := L (the R band read as 0)
    // NOMASK: every P column of the tile is inside the image and >= every d (tile-uniform)
    auto s1v = [&](int d, auto stats, auto nomask) {
        constexpr bool STATS = decltype(stats)::value;
        constexpr bool NOMASK = decltype(nomask)::value;
        G_MARK("S1V");
        const bool m = STATS || NOMASK || (col_in && xc >= d);
        const uint8_t* rc = rb + (c + kBandChunk - (d & (kBandChunk - 1)));
        uint32_t rv[G::NV];
#pragma unroll
        for (int k = 0; k < G::NV; ++k) rv[k] = STATS ? 0u : (uint32_t)rc[(a0 + k) * G::RBW];
        uint32_t T = 0u, Tp[2 * R + 1];
#pragma unroll
        for (int k = 0; k < G::NV; ++k) {
            const uint32_t ad = __builtin_amdgcn_sad_u8(mul[k], rv[k], 0xFFFFFFF0u);
            T = __umul24(ad, mul[k]) + T;
            if (k >= 2 * R) {
                const uint32_t old = (k == 2 * R) ? 0u : Tp[(k - 2 * R - 1) % (2 * R + 1)];
                const uint32_t val = m ? T - old : 0u;
                // cs[(a0 + k - 2R) * CSS + lane]: lane-consecutive dwords, so ds_write_addtid_b32
                // (2 LDS cycles per store instead of 4).  M0 (this wave's first cs row) is written in the
                // same asm statement as the store that reads it, so no compiler-generated M0 use can
                // fall between them; the SALU write needs one wait state before the add-TID LDS read
                // of M0 (a hazard the compiler does not see inside asm): s_nop 0.
                asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tds_write_addtid_b32 %0 offset:%2"
                             : : "v"(val), "s"(m0_cs), "i"((k - 2 * R) * G::CSS * 4) : "memory", "m0");
            }
            Tp[k % (2 * R + 1)] = T;
        }
        G_MARK("end");
    };
    // ================= S1H =================
    auto s1h_stats = [&]() {
        if (!h1_on) return;
        const uint32_t* row = cs + h1i * G::CSS + h1s * G::SW1;
        uint32_t sp = 0, sip = 0;
#pragma unroll
        for (int k = 0; k < 2 * R; ++k) {
            const uint32_t v = row[k];
            sp += v >> 20;
            sip += v & k_plow;
        }
#pragma unroll
        for (int o = 0; o < G::SW1; ++o) {
            const uint32_t vin = row[o + 2 * R];
            sp += vin >> 20;
            sip += vin & k_plow;
            // guide statistics: sp = SI, sip = SII
            const int j = h1s * G::SW1 + o;                         // A column
            const int x = x0 - R + j;
            const bool inimg = h1y >= 0 && h1y < H && x >= 0 && x < W && j < G::AW;
            const uint32_t N = inimg ? (uint32_t)(win_count(x, R, W) * win_count(h1y, R, H)) : 1u;
            const int32_t nvar = (int32_t)(N * sip - sp * sp);
            nN[o] = N;
            nSI[o] = 0u - sp;   // -SI, for the signed 24-bit products in S1H
            fSI[o] = (float)sp;
            invden[o] = inimg ? 1.0f / ((float)nvar + eps * (float)N * (float)N) : 0.f;
            invN[o] = inimg ? 1.0f / (float)N : 0.f;
            const uint32_t vout = row[o];
            sp -= vout >> 20;
            sip -= vout & k_plow;
        }
    };
    auto s1h = [&]() {
        if (!h1_on) return;
        G_MARK("S1H");
        const uint32_t* row = cs + h1i * G::CSS + h1s * G::SW1;
        // the whole segment is loaded before the first a/b store (the compiler cannot tell abp
        // from cs, so interleaved loads would each wait for the stores before them)
        uint32_t v[G::SW1 + 2 * R];
#pragma unroll
        for (int k = 0; k < G::SW1 + 2 * R; ++k) v[k] = row[k];
#if SM_G_ACC
        // SM_G_ACC: the packed column sums are summed as they are (acc, wrapping u32) beside the exact Sp; the
        // window's SIp < 2^23 is then acc - Sp * 2^20 (mod 2^32, exact), one v_mad_i32_i24 per output instead of
        // an and + add per column
        uint32_t sp = 0, acc = 0;
#pragma unroll
        for (int k = 0; k < 2 * R; ++k) {
            sp += v[k] >> 20;
            acc += v[k];
        }
#else
        uint32_t sp = 0, sip = 0;
#pragma unroll
        for (int k = 0; k < 2 * R; ++k) {
            sp += v[k] >> 20;
            sip += v[k] & k_plow;
        }
#endif
#pragma unroll
        for (int o = 0; o < G::SW1; ++o) {
#if SM_G_ACC
            sp += v[o + 2 * R] >> 20;
            acc += v[o + 2 * R];
            uint32_t sip;
            asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(sip) : "v"(sp), "s"(k_m2p20), "v"(acc));
#else
            sp += v[o + 2 * R] >> 20;
            sip += v[o + 2 * R] & k_plow;
#endif
            // N*SIp - SI*Sp = N^2 cov(I, p), |.| < 2^30, exactly: every factor fits a signed 24-bit
            // operand (SIp <= 121 * 255^2 < 2^23), so v_mul_i32_i24 + v_mad_i32_i24 (written out: the
            // compiler otherwise turns one product into a quarter-rate v_mul_lo_u32)
            int32_t num;
            asm("v_mul_i32_i24 %0, %1, %2" : "=v"(num) : "v"(nSI[o]), "v"(sp));
            asm("v_mad_i32_i24 %0, %1, %2, %0" : "+v"(num) : "v"(nN[o]), "v"(sip));
            const float a = (float)num * invden[o];
            // float(Sp) without v_cvt (a quarter-rate op here): Sp < 2^22, float(2^23 + Sp) is exact
            const float fsp = __builtin_bit_cast(float, k_magic | sp) + k_magicf;
            const float b = __builtin_fmaf(-a, fSI[o], fsp) * invN[o];
            // one ds_write_b64 (the compiler emits ds_write2_b32 for a float2 store here)
            asm volatile("ds_write_b64 %0, %1 offset:%2"
                         :
                         : "v"(h1off), "v"(__builtin_bit_cast(double, make_float2(a, b))), "i"(8 * o)
                         : "memory");
            sp -= v[o] >> 20;
#if SM_G_ACC
            acc -= v[o];
#else
            sip -= v[o] & k_plow;
#endif
        }
        G_MARK("end");
    };
    // ================= S2V =================
    auto s2v = [&]() {
        if (!v2_on) return;
        G_MARK("S2V");
        // one ds_read_b64 per row (2 LDS cycles) instead of a merged ds_read2_b64 (8 cycles for the
        // same two rows, MI355X_MICROARCH.md LDS table): rows k and k + 5 share a base whose value the
        // compiler cannot relate to the others, and 5 rows (2160 B) exceed ds_read2's offset range
        // RPS output rows in groups of 8: the rows a group adds are loaded at its start (the first group
        // also loads the 2R warm-up rows), before its mm stores, as in S1H; a row's registers are
        // free once no later group reads it.  Each group restarts its running sums from its own 2R
        // warm-up rows, as an 8-row strip does without the roles: the float sums, and so the maps, are
        // the same bit for bit in every configuration (the right-view kernel runs without the roles at
        // r = 2, 6, 7, and the LR check pairs its left map with the left-only kernel's)
        // (round 6, not kept: one running sum over the wave's whole 16-row strip, 100 -> 82 VALU per wave and d, ran
        // 451.3 -> 457.2 us per 1080p guided frame, guided + LR 504.7 -> 528.6 and 2968 -> 3110 at 4K: fewer
        // instructions, longer dependent chains; profiles/microbench/r06_guided_s2v_run_ab.txt)
        constexpr int GS = 8;
        constexpr int NRW = G::RPS + 2 * R;
        float2 v[NRW];
#pragma unroll
        for (int k = 0; k < GS + 2 * R; ++k) v[k] = v2col[k % 5][(k / 5) * 5 * G::ABS];
#pragma unroll
        for (int g = 0; g < G::RPS / GS; ++g) {
            if (g > 0) {
#pragma unroll
                for (int k = GS * g + 2 * R; k < GS * g + GS + 2 * R; ++k) v[k] = v2col[k % 5][(k / 5) * 5 * G::ABS];
            }
            float sa = 0.f, sb = 0.f;
#pragma unroll
            for (int k = GS * g; k < GS * g + 2 * R; ++k) {
                sa += v[k].x;
                sb += v[k].y;
            }
#pragma unroll
            for (int r = GS * g; r < GS * g + GS; ++r) {
                sa += v[r + 2 * R].x;
                sb += v[r + 2 * R].y;
                // mmA / mmB [(RPS v2g + r) * MSA + lane]: lane-consecutive, so ds_write_addtid_b32, with
                // M0 (this wave's first mm row, plane A) set inside the same asm statement as in S1V
                asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\t"
                             "ds_write_addtid_b32 %0 offset:%3\n\tds_write_addtid_b32 %1 offset:%4"
                             :
                             : "v"(sa), "v"(sb), "s"(m0_mm), "i"(r * G::MSA * 4), "i"(r * G::MSA * 4 + G::MM_PLANE)
                             : "memory", "m0");
                sa -= v[r].x;
                sb -= v[r].y;
            }
        }
        G_MARK("end");
    };
    // ================= S2H + WTA =================
    // LIM: some output of the tile can have d past its validity limit (tile-uniform; interior tiles skip the test)
    auto s2h = [&](int d, auto lim) {
        constexpr bool LIM = decltype(lim)::value;
        G_MARK("S2H");
        constexpr int NR = G::SW2 + 2 * R;   // mm values read per plane
        float va[NR], vb[NR];
        if constexpr (G::SW2 % 2 == 0) {
            s2h_load<NR / 2, G::MM_PLANE>(h2off, va, vb);
        } else {   // odd segment starts: 4-byte reads
            const float* ra = mmA + h2r * G::MSA + h2s * G::SW2;
            const float* rbb = mmB + h2r * G::MSA + h2s * G::SW2;
#pragma unroll
            for (int k = 0; k < NR; ++k) {
                va[k] = ra[k];
                vb[k] = rbb[k];
            }
        }
        float sa = 0.f, sb = 0.f;
#pragma unroll
        for (int k = 0; k < 2 * R; ++k) {
            sa += va[k];
            sb += vb[k];
        }
#pragma unroll
        for (int o = 0; o < G::SW2; ++o) {
            sa += va[o + 2 * R];
            sb += vb[o + 2 * R];
            float q;   // sa * I + sb, one rounding
            bool valid;
            if constexpr (LEAN) {
                if (o % 2 == 0)
                    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[0,1,0]" : "=v"(q) : "v"(sa), "v"(oIh[o / 2]), "v"(sb));
                else
                    asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,1,0] op_sel_hi:[0,1,0]"
                        : "=v"(q) : "v"(sa), "v"(oIh[o / 2]), "v"(sb));
                valid = d - dsgn * o <= dl0;
            } else {
                q = sa * oI[o] + sb;
                valid = d <= dlim[o];
            }
            const bool take = (!LIM || valid) && q < bq[o];
            bq[o] = take ? q : bq[o];
            bdd[o] = take ? d : bdd[o];
            if constexpr (RIGHT) {
                // candidate for right pixel u = x - d (slot o): q = (N q) / N, fixed point, position
                // 7 SW2 + o (the output column relative to this segment, see the file header).
                // NaN (outputs outside) -> 4e9 -> INT_MAX; the conversion saturates both ways
                const float qs = __builtin_fminf(q * rinv[o], 4.0e9f);
                int kq;
                asm("v_cvt_i32_f32 %0, %1" : "=v"(kq) : "v"(qs));
                const int key = (kq & ~0xFF) | (7 * G::SW2 + o);
                rk[o] = key < rk[o] ? key : rk[o];
            }
            sa -= va[o];
            sb -= vb[o];
        }
        chain_step(d);
        G_MARK("end");
    };

    // S1V's cs stores and S1H's a/b stores are inline asm, which the compiler's wait-count pass does
    // not see: where no compiler-visible LDS op is pending (the stats pass, the first d) it issues the
    // barrier without waiting for them, and another wave can read the rows before they land.  Every
    // barrier that hands those rows over waits for the LDS queue explicitly.
    auto lds_barrier = [] {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __syncthreads();
    };
    if (is_s1v) s1v(0, std::true_type{}, std::false_type{});
    // (round 5: stopping the left-only kernel at the tile's last valid d, W - x0, measured +0.7 % slower on the
    // 1080p guided launch (453.5 -> 456.9 us per frame, profiles/microbench/r05_skip_invalid_pairs_ab.txt): not kept)
    const int Dk = D;
    const bool s1_nomask = px0 >= Dk - 1 && px0 >= 0 && px0 + 63 < W;
    const bool s2_lim = valid_mode != 1 ? (Dk - 1 > W - (x0 + G::TW - 1)) : (Dk - 1 > x0);
    lds_barrier();
    s1h_stats();
    __syncthreads();
    // buffers: cs (S1V -> S1H), abp (S1H -> S2V), mm (S2V -> S2H); each producer of iteration d+1
    // runs after the barrier that ends the consumer of iteration d.  The right band (read only by
    // S1V) is restaged for the next d-chunk in the second phase of the chunk's last iteration.
    for (int d = d_lo; d <= Dk; ++d) {
        if (is_s1v && d < Dk) {
            if (s1_nomask) s1v(d, std::false_type{}, std::true_type{});
            else s1v(d, std::false_type{}, std::false_type{});
        }
        if ((!ROLES || !is_s1v) && d > d_lo) s2v();
        lds_barrier();
        if (d + 1 < Dk && ((d + 1) & (kBandChunk - 1)) == 0) stage_band((d + 1) / kBandChunk);
        if (d < Dk) s1h();
        if (d > d_lo) {
            if (s2_lim) s2h(d - 1, std::true_type{});
            else s2h(d - 1, std::false_type{});
        }
        lds_barrier();
    }
    // drain the right-key chain: 8 SW2 - 1 more steps move every slot out through the last segment
    if constexpr (RIGHT) {
        for (int k = D; k < d_lo + K; ++k) chain_step(k);
    }
    if (valid_mode == 2) {
        // d-slice keys: (q * 2^14 << 8) | d, INT_MAX where no d of the slice is valid
        int* Kf = keys + (int64_t)frame * H * W;
#pragma unroll
        for (int o = 0; o < G::SW2; ++o) {
            const int x = x0 + h2s * G::SW2 + o;
            if (oy < H && x < W && h2s * G::SW2 + o < G::TW) {
                const float s = kRightScale / (float)(win_count(x, R, W) * win_count(oy, R, H));
                const float qs = __builtin_fmaxf(__builtin_fminf(bq[o] * s, kRightMax), kRightMin);
                Kf[(int64_t)oy * W + x] = bdd[o] < 0 ? INT_MAX : (((int)qs << 8) | bdd[o]);
            }
        }
        return;
    }
    uint8_t* Df = disp + (int64_t)frame * ostride;
#pragma unroll
    for (int o = 0; o < G::SW2; ++o) {
        const int x = x0 + h2s * G::SW2 + o;
        if (oy < H && x < W && h2s * G::SW2 + o < G::TW)
            Df[(int64_t)oy * out_pitch + x] = (uint8_t)(bdd[o] & 0xFF);   // (uchar)dm, Device.cu:63
    }
}

// Guided d-slice keys -> disparity: d where q < 50 (the Device.cu:37 seed, strict), else 0.
// 50 * 2^14 is exact and the keys truncate q * 2^14, so (key >> 8) < 819200 iff q < 50.
__global__ __launch_bounds__(256) void guided_keys_to_disp_kernel(const int* __restrict__ keys, int W, int H,
                                                                  uint8_t* __restrict__ disp, int out_pitch) {
    const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= W) return;
    const int k = keys[(int64_t)y * W + x];
    disp[(int64_t)y * out_pitch + x] = (k >> 8) < (int)(50.0f * kRightScale) ? (uint8_t)(k & 0xFF) : (uint8_t)0;
}

// Right view of the fused pass: for each right pixel u of a tile row band, the minimum key over the
// tiles whose chain emitted u (k = x0 + SPAN - 1 - u in [0, K)), decoded to d = x0 + position - u.
// Block = 64 columns x the 32 rows of one tile band; reads are 128-B rows of gpart ([k][row]).
// MAXT >= the most tiles covering one u, (K + TW - 1) / TW + 1: a fixed trip count, so every key load of
// an entry issues before the first compare (round 4; the loop over the covering tiles had each load wait
// for the compare before it)
// Slice mode (rkeys != nullptr, multi-GPU d-slices with LR): the chains of a pass over d in [d_lo, d_hi)
// index u' = u + d_lo (the layout of the d_lo = 0 pass of d - d_lo), and the kernel writes the right key
// of every pixel u, (its cost field) | d, to rkeys[f][y][u] (INT_MAX where no d of the slice has u + d < W):
// keys of disjoint slices combine with a signed MIN (smaller cost, then smaller d).
template <int TH, int MAXT>
__global__ __launch_bounds__(256) void guided_right_reduce_kernel(const int* __restrict__ gpart, int tiles_x, int tiles,
                                                                  int TW, int SPAN, int K, int W, int H,
                                                                  uint8_t* __restrict__ right, int rpitch,
                                                                  int64_t rstride, int* __restrict__ rkeys, int d_lo) {
    constexpr int UC = 64;
    __shared__ uint8_t band[TH][UC];
    const int u0 = blockIdx.x * UC, ty = blockIdx.y, f = blockIdx.z;
    const int* base = gpart + ((int64_t)f * tiles + (int64_t)ty * tiles_x) * K * TH;
    int* kf = rkeys ? rkeys + (int64_t)f * H * W : nullptr;
    for (int e = threadIdx.x; e < TH * UC; e += blockDim.x) {
        const int j = e % TH, ul = e / TH, u = u0 + ul;
        int dr = 0;
        if (u < W) {
            const int n = u - SPAN + 1;
            const int tlo = n <= 0 ? 0 : (n + TW - 1) / TW;
            const int thi = min(tiles_x - 1, (u - SPAN + K) / TW);
            int key[MAXT];
#pragma unroll
            for (int m = 0; m < MAXT; ++m) {
                const int tx = tlo + m;
                key[m] = tx <= thi ? base[((int64_t)tx * K + (tx * TW + SPAN - 1 - u)) * TH + j] : INT_MAX;
            }
            // keys order (cost, column) within a tile only: across tiles compare the cost field,
            // strict <, in ascending tile order, so equal costs keep the smaller column = smaller d
            int best = key[0], bm = 0;
#pragma unroll
            for (int m = 1; m < MAXT; ++m) {
                if ((key[m] >> 8) < (best >> 8)) {
                    best = key[m];
                    bm = m;
                }
            }
            dr = (tlo + bm) * TW + (best & 0xFF) - u;
            const int y = ty * TH + j;
            if (kf && y < H && u >= d_lo) kf[(int64_t)y * W + u - d_lo] = (best & ~0xFF) | (dr + d_lo);
        }
        if (kf) {   // right pixels with u + d_lo >= W: no d of the slice reaches them
            const int y = ty * TH + j;
            if (y < H && u < W && u >= W - d_lo) kf[(int64_t)y * W + u] = INT_MAX;
            continue;
        }
        band[j][ul] = (uint8_t)dr;
    }
    if (kf) return;
    __syncthreads();
    uint8_t* Rf = right + (int64_t)f * rstride;
    for (int e = threadIdx.x; e < TH * UC; e += blockDim.x) {
        const int j = e / UC, ul = e % UC;
        const int y = ty * TH + j, u = u0 + ul;
        if (y < H && u < W) Rf[(int64_t)y * rpitch + u] = band[j][ul];
    }
}

// the reduce with the smallest instantiated MAXT >= (K + TW - 1) / TW + 1 (D <= 256, TW >= 36: <= 10)
template <int TH>
hipError_t launch_right_reduce(const int* gpart, int tiles_x, int tiles_y, int batch, int TW, int span, int K, int W,
                               int H, uint8_t* right, int rpitch, int64_t rstride, int* rkeys, int d_lo,
                               hipStream_t s) {
    const int need = (K + TW - 1) / TW + 1;
    const dim3 grid((unsigned)((W + 63) / 64), (unsigned)tiles_y, (unsigned)batch);
    const int tiles = tiles_x * tiles_y;
#define SM_RIGHT_REDUCE(M)                                                                                      \
    hipLaunchKernelGGL((guided_right_reduce_kernel<TH, M>), grid, dim3(256), 0, s, gpart, tiles_x, tiles, TW, span, K, \
                       W, H, right, rpitch, rstride, rkeys, d_lo)
    if (need <= 4) SM_RIGHT_REDUCE(4);
    else if (need <= 6) SM_RIGHT_REDUCE(6);
    else if (need <= 8) SM_RIGHT_REDUCE(8);
    else if (need <= 10) SM_RIGHT_REDUCE(10);
    else return hipErrorInvalidValue;
#undef SM_RIGHT_REDUCE
    return hipGetLastError();
}

template <int R>
hipError_t run_fused(const uint8_t* L, const uint8_t* Rimg, int W, int H, int pitch, int64_t fstride, int batch,
                     int d_lo, int D, float eps, int valid_mode, uint8_t* disp, int out_pitch, int64_t ostride,
                     int* gpart, uint8_t* right, int rpitch, int64_t rstride, int* keys, hipStream_t s,
                     int* rkeys = nullptr) {
    using G = GeoF<R, false>;   // tile geometry (TW, TH, SW2) is the same with or without the roles
    const int tiles_x = (W + G::TW - 1) / G::TW, tiles_y = (H + G::TH - 1) / G::TH;
    const int64_t blocks = (int64_t)tiles_x * tiles_y * batch;
    if (blocks <= 0 || blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    // the left-only kernel may run the phase-1 wave roles: its LDS plan is GeoF<R, kGuidedRoles>'s
    constexpr size_t lds_left = (size_t)GeoF<R, kGuidedRoles>::LDS;
    constexpr size_t lds_right = (size_t)GeoF<R, kGuidedRoles && kRolesRight<R>>::LDS;
    if (!gpart) {
        hipLaunchKernelGGL((guided_fused_kernel<R, false>), dim3((unsigned)blocks), dim3(kT), lds_left, s, L,
                           Rimg, W, H, pitch, fstride, d_lo, D, eps, valid_mode, disp, out_pitch, ostride, tiles_x,
                           tiles_x * tiles_y, nullptr, 0, keys);
        return hipGetLastError();
    }
    // with the right view: valid_mode 0 (d_lo 0, the left map + dR) or 2 (a d slice: left keys + right keys in
    // rkeys, the chains laid out for d - d_lo)
    const int span = 8 * G::SW2;
    const int K = (D - d_lo) + span - 1;
    hipLaunchKernelGGL((guided_fused_kernel<R, true>), dim3((unsigned)blocks), dim3(kT), lds_right, s, L, Rimg,
                       W, H, pitch, fstride, d_lo, D, eps, valid_mode, disp, out_pitch, ostride, tiles_x,
                       tiles_x * tiles_y, gpart, K, keys);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_right_reduce<G::TH>(gpart, tiles_x, tiles_y, batch, G::TW, span, K, W, H, right, rpitch, rstride,
                                      rkeys, d_lo, s);
}

template <int R>
size_t partial_bytes(int W, int H, int D, int batch) {   // D: the pass's span d_hi - d_lo
    using G = GeoF<R, false>;
    const int64_t tiles = (int64_t)((W + G::TW - 1) / G::TW) * ((H + G::TH - 1) / G::TH);
    return (size_t)(tiles * batch * (D + 8 * G::SW2 - 1) * G::TH * 4);
}

}  // namespace

hipError_t launch_guided_match(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int batch,
                               int64_t frame_stride, int radius, int D, float eps, int valid_mode, uint8_t* disp,
                               int out_pitch, int64_t out_frame_stride, hipStream_t s) {
    return launch_guided_match_lr(L, R, W, H, pitch, batch, frame_stride, radius, D, eps, valid_mode, disp, out_pitch,
                                  out_frame_stride, nullptr, nullptr, 0, 0, s);
}

size_t guided_right_partial_bytes(int W, int H, int radius, int D, int batch) {
#define SM_GUIDED_BYTES(r) \
    case r: return partial_bytes<r>(W, H, D, batch)
    switch (radius) {
        SM_GUIDED_BYTES(0);
        SM_GUIDED_BYTES(1);
        SM_GUIDED_BYTES(2);
        SM_GUIDED_BYTES(3);
        SM_GUIDED_BYTES(4);
        SM_GUIDED_BYTES(5);
        SM_GUIDED_BYTES(6);
        SM_GUIDED_BYTES(7);
        default: return 0;
    }
#undef SM_GUIDED_BYTES
}

hipError_t launch_guided_match_lr(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int batch,
                                  int64_t frame_stride, int radius, int D, float eps, int valid_mode, uint8_t* disp,
                                  int out_pitch, int64_t out_frame_stride, int* gpart, uint8_t* right, int rpitch,
                                  int64_t rstride, hipStream_t s) {
    if (D < 1 || D > kMaxDisp) return hipErrorInvalidValue;
    if (gpart && (!right || valid_mode != 0)) return hipErrorInvalidValue;
#define SM_GUIDED_CASE(r) \
    case r: return run_fused<r>(L, R, W, H, pitch, frame_stride, batch, 0, D, eps, valid_mode, disp, out_pitch, out_frame_stride, gpart, right, rpitch, rstride, nullptr, s)
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

hipError_t launch_guided_slice_keys(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int batch,
                                    int64_t frame_stride, int radius, int d_lo, int d_hi, float eps, int* keys,
                                    hipStream_t s) {
    if (d_lo < 0 || d_hi <= d_lo || d_hi > kMaxDisp || !keys) return hipErrorInvalidValue;
#define SM_GUIDED_SLICE(r) \
    case r: return run_fused<r>(L, R, W, H, pitch, frame_stride, batch, d_lo, d_hi, eps, 2, nullptr, 0, 0, nullptr, nullptr, 0, 0, keys, s)
    switch (radius) {
        SM_GUIDED_SLICE(0);
        SM_GUIDED_SLICE(1);
        SM_GUIDED_SLICE(2);
        SM_GUIDED_SLICE(3);
        SM_GUIDED_SLICE(4);
        SM_GUIDED_SLICE(5);
        SM_GUIDED_SLICE(6);
        SM_GUIDED_SLICE(7);
        default: return hipErrorInvalidValue;
    }
#undef SM_GUIDED_SLICE
}

hipError_t launch_guided_slice_lr_keys(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int batch,
                                       int64_t frame_stride, int radius, int d_lo, int d_hi, float eps, int* keys,
                                       int* right_keys, int* gpart, hipStream_t s) {
    if (d_lo < 0 || d_hi <= d_lo || d_hi > kMaxDisp || !keys || !right_keys || !gpart) return hipErrorInvalidValue;
#define SM_GUIDED_SLICE_LR(r) \
    case r: return run_fused<r>(L, R, W, H, pitch, frame_stride, batch, d_lo, d_hi, eps, 2, nullptr, 0, 0, gpart, nullptr, 0, 0, keys, s, right_keys)
    switch (radius) {
        SM_GUIDED_SLICE_LR(0);
        SM_GUIDED_SLICE_LR(1);
        SM_GUIDED_SLICE_LR(2);
        SM_GUIDED_SLICE_LR(3);
        SM_GUIDED_SLICE_LR(4);
        SM_GUIDED_SLICE_LR(5);
        SM_GUIDED_SLICE_LR(6);
        SM_GUIDED_SLICE_LR(7);
        default: return hipErrorInvalidValue;
    }
#undef SM_GUIDED_SLICE_LR
}

hipError_t launch_guided_keys_to_disp(const int* keys, int W, int H, uint8_t* disp, int out_pitch, hipStream_t s) {
    if (W <= 0 || H <= 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(guided_keys_to_disp_kernel, dim3((unsigned)((W + 255) / 256), (unsigned)H), dim3(256), 0, s,
                       keys, W, H, disp, out_pitch);
    return hipGetLastError();
}

}  // namespace sm
