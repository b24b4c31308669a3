// bm_staged.hip — the staged (cost-volume) formulation of the box path:
//   K1 ad_volume_kernel (bm_volume.hip): AD volume, u8 [D][H][W]               P*D bytes written
//   K2 box_sad_kernel:  SAD volume, u16 [D][H][W]: the (2r+1)^2 window sum of each AD plane,
//                       zero-padded at the borders (= the clipped window, Device.cu:46-56);
//                       column strips walked top to bottom    P*D read (+2r rows per band), 2*P*D written
//   K3 volume_wta_kernel: first d with the smallest SAD below 50*win^2, valid d <= W-x
//                       (Device.cu:37-63); 0 where none                          2*P*D read, P written
// The fused box_match_kernel computes the same map without the volumes; this chain streams them
// through HBM, so each kernel is bandwidth-bound and its rocprof HBM rate is the meaningful
// figure (SURVEY §7 hard part (b)).  The u16 SAD volume is also the cost volume for callers who
// aggregate or post-process themselves: the reference's getAllSAD / kernalFindAllSAD
// (BlockMatching.cpp:191-261, Device.cu:67-125) stored it as uint8, truncating mod 256.
#include "bm_common.h"

namespace sm {
namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kST = 256;
// K2 build switches (same-box A/B, 8 x 1080p D=128 frames per launch, tools/ab_staged_kernels.py):
//   SM_SAD_CPT 8 vs 4 columns per thread (16-B vs 8-B stores): 162 vs 188 us per frame;
//   SM_SAD_NT nontemporal SAD stores: the WTA that reads them back runs 81 vs 93 us;
//   SM_SAD_BLOCKS 16384 vs 2048 / 4096 / 8192: 156 vs 169 / 163 / 164 us.
#ifndef SM_SAD_CPT
#define SM_SAD_CPT 8
#endif
#ifndef SM_SAD_NT
#define SM_SAD_NT 1
#endif
constexpr int kCPT = SM_SAD_CPT;    // K2: input (and output) columns per thread, 4 or 8
constexpr int kSC = kCPT * kST;     // K2: input columns per strip
constexpr int kSO = kSC - 16;      // K2: output columns per strip (the strip starts 8 columns early)
#ifndef SM_SAD_BLOCKS
#define SM_SAD_BLOCKS 16384
#endif
constexpr int kSadBlocks = SM_SAD_BLOCKS;  // K2 blocks per launch (>= 32-row bands)
// K2 walking direction (round 4): odd bands walk their rows bottom-up, so the 2r halo
// rows two neighbouring bands share are read by both at the same phase of their walks (both at the
// start, or both at the end) while they run side by side on one XCD: the second read hits that XCD's
// L2.  With every band walking down, band b read its top halo at its start and band b - 1 the same
// rows at its end, ~12 MB of XCD traffic later (4 MB L2): rocprof counted 1.046x the algorithmic bytes
// (1.004x with the zigzag, at ~3 % of this kernel's time).
static_assert(kCPT == 4 || kCPT == 8, "K2 columns per thread");

// K2: one column strip x one row band of one d plane per block.  A thread owns kCPT input columns
// and walks the band's rows once: vertical window sums run in registers (packed u16 pairs, the
// rows leaving the window kept in a register ring of 2r+1 words), each output row's vertical sums
// go to LDS, and each thread forms kCPT horizontal window sums from its neighbours' columns.
// Every AD byte is read once per band (the 2r halo rows of a band are re-read; >= ~64-row bands),
// every SAD value written once as part of a 2*kCPT-byte store.
template <int N>
struct Words {
    uint32_t w[N];
};

template <int R>
__global__ __launch_bounds__(kST) void box_sad_kernel(const uint8_t* __restrict__ ad, int W, int H, int rows_per_band,
                                                      int bands, int strips, uint16_t* __restrict__ sad) {
    constexpr int K = 2 * R + 1;
    constexpr int NG = kCPT / 4;                        // 4-column groups per thread
    __shared__ __attribute__((aligned(16))) uint16_t vs[2][kSC + 16];
    const int t = threadIdx.x;
    // XCD-aware order: each XCD walks a contiguous run of (plane, strip, band) ids, band fastest,
    // so the 2r halo rows a band shares with the band above are still in that XCD's L2
    const int id = xcd_tile(blockIdx.x, gridDim.x);
    const int band = id % bands, sx = (id / bands) % strips, d = id / (bands * strips);
    const int yo0 = band * rows_per_band;
    const int yo1 = min(H, yo0 + rows_per_band);
    if (yo0 >= H) return;                               // block-uniform
    // the walk runs over virtual rows v; image row phys(v) reflects the band's input range
    // [yo0 - R, yo1 + R) (and its output rows [yo0, yo1)) onto itself for a bottom-up band
    const bool up = (band & 1) != 0;
    auto phys = [&](int v) { return up ? yo0 + yo1 - 1 - v : v; };
    const int64_t P = (int64_t)W * H;
    const uint8_t* plane = ad + (int64_t)d * P;
    uint16_t* outp = sad + (int64_t)d * P;
    const int xs = sx * kSO;                            // first output column of the strip
    const int xin = xs - 8 + kCPT * t;                  // this thread's kCPT input columns
    const bool vec_out = (W % kCPT == 0) && ((reinterpret_cast<uintptr_t>(sad) & (2 * kCPT - 1)) == 0);
    const int x = xs + kCPT * t;
    const bool out_on = kCPT * t < kSO && x < W;
    // vertical sums of group g: E = (col0, col2), O = (col1, col3) as u16 pairs (<= (2r+1) * 255)
    uint32_t E[NG], O[NG], ring[K][NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        E[g] = O[g] = 0u;
#pragma unroll
        for (int j = 0; j < K; ++j) ring[j][g] = 0u;
    }
    const int yi_end = yo1 + R;                         // input rows [yo0 - R, yo1 + R)
    int buf = 0;
    // horizontal sums of output row y, staged in vs[buf], behind one barrier
    auto flush = [&](int y) {
        // an LDS-only barrier: __syncthreads' workgroup fence would also wait for every global load and
        // store in flight (s_waitcnt vmcnt(0) before each row), draining the prefetched rows
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        const uint16_t* row = vs[buf];
        // outputs xs + kCPT t + k (k < kCPT): window of vs indices [kCPT t + 8 + k - R, kCPT t + 8 + k + R]
        constexpr int NW2 = (kCPT + 16) / 4;            // 8-B reads covering kCPT + 16 u16
        uint32_t w[2 * NW2];
#pragma unroll
        for (int u = 0; u < NW2; ++u) {
            const uint2 x2 = *reinterpret_cast<const uint2*>(row + kCPT * t + 4 * u);
            w[2 * u] = x2.x;
            w[2 * u + 1] = x2.y;
        }
        auto val = [&](int i) -> uint32_t { return (i & 1) ? (w[i >> 1] >> 16) : (w[i >> 1] & 0xFFFFu); };
        uint32_t sum = 0;
#pragma unroll
        for (int i = 8 - R; i <= 8 + R; ++i) sum += val(i);
        uint32_t res[kCPT];
        res[0] = sum;
#pragma unroll
        for (int k = 1; k < kCPT; ++k) {
            sum += val(8 + R + k) - val(8 - R + k - 1);
            res[k] = sum;                               // <= (2r+1)^2 * 255 < 2^16 for r <= 7
        }
        if (out_on) {
            uint16_t* dst = outp + (int64_t)phys(y) * W + x;
            if (vec_out && x + kCPT <= W) {
                if constexpr (kCPT == 8) {
                    const u32x4 v = {res[0] | (res[1] << 16), res[2] | (res[3] << 16), res[4] | (res[5] << 16),
                                     res[6] | (res[7] << 16)};
                    if (SM_SAD_NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst));
                    else *reinterpret_cast<u32x4*>(dst) = v;
                } else {
                    const uint2 v = make_uint2(res[0] | (res[1] << 16), res[2] | (res[3] << 16));
                    if (SM_SAD_NT) {
                        __builtin_nontemporal_store(v.x, reinterpret_cast<uint32_t*>(dst));
                        __builtin_nontemporal_store(v.y, reinterpret_cast<uint32_t*>(dst) + 1);
                    } else {
                        *reinterpret_cast<uint2*>(dst) = v;
                    }
                }
            } else {
                for (int k = 0; k < kCPT && x + k < W; ++k) dst[k] = (uint16_t)res[k];
            }
        }
        buf ^= 1;                                       // the next row goes to the other buffer
    };
    // one buffer load of kCPT bytes per row and thread, whatever the row: rows outside the plane (and
    // past the band) read at an offset past the descriptor's end, which returns 0; a word reaching past
    // column W - 1 keeps only its bytes inside.  A fixed number of loads per group lets the compiler's
    // wait counts follow the prefetched group (the byte-wise border loads made them all vmcnt(0)).
    // the hardware range-checks each dword of the (unaligned) word as a whole, so the range reaches 8
    // bytes past the plane: the next plane's or the allocation's pad (ensure_vol), dropped by the
    // column mask
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(plane), 0, (int)(P + 8), 0x00020000);
    const bool col_in = xin >= 0 && xin < W;
    const int col_bytes = col_in ? min(kCPT, W - xin) : 0;
    auto load_group = [&](int base, Words<NG>* nw) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const int y = phys(base + j);
            const bool ok = col_in && y >= 0 && y < H && base + j < yi_end;
            const uint32_t off = ok ? (uint32_t)(y * W + xin) : 0x80000000u;
            if constexpr (kCPT == 8) {
                uint64_t v = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(prs, off, 0, 0));
                if (col_bytes < 8) v &= col_bytes <= 0 ? 0ull : (~0ull >> (64 - 8 * col_bytes));
                nw[j].w[0] = (uint32_t)v;
                nw[j].w[1] = (uint32_t)(v >> 32);
            } else {
                uint32_t v = __builtin_amdgcn_raw_buffer_load_b32(prs, off, 0, 0);
                if (col_bytes < 4) v &= col_bytes <= 0 ? 0u : (~0u >> (32 - 8 * col_bytes));
                nw[j].w[0] = v;
            }
        }
    };
    // ring slot j holds row base + j - K (this group's row base + j replaces it)
    auto run_group = [&](int base, const Words<NG>* nw) {
#pragma unroll
        for (int j = 0; j < K; ++j) {
            const int yi = base + j;
            if (yi >= yi_end) break;                    // block-uniform
#pragma unroll
            for (int g = 0; g < NG; ++g) {
                const uint32_t v = nw[j].w[g], o = ring[j][g];
                ring[j][g] = v;
                E[g] += (v & 0x00FF00FFu) - (o & 0x00FF00FFu);
                O[g] += ((v >> 8) & 0x00FF00FFu) - ((o >> 8) & 0x00FF00FFu);
            }
            if (yi - R < yo0) continue;                 // warm-up rows of the band (window centred on yi - R)
#pragma unroll
            for (int g = 0; g < NG; ++g)
                *reinterpret_cast<uint2*>(&vs[buf][kCPT * t + 4 * g]) =
                    make_uint2(__builtin_amdgcn_perm(O[g], E[g], 0x05040100u), __builtin_amdgcn_perm(O[g], E[g], 0x07060302u));
            flush(yi - R);
        }
    };
    // two row groups in flight: group g + 1 loads while group g runs (A / B buffers, no copies; one group at a
    // time measured 156.8 against 154.6 us per frame, same box, 5 rounds)
    Words<NG> na[K], nb[K];
    load_group(yo0 - R, na);
    for (int base = yo0 - R; base < yi_end; base += 2 * K) {
        load_group(base + K, nb);
        run_group(base, na);
        if (base + K >= yi_end) break;
        load_group(base + 2 * K, na);
        run_group(base + K, nb);
    }
}

// K3: 8 pixels per thread, one 16-B nontemporal load per d plane (the volume is streamed once and
// is larger than the MALL).  The loads of kWtaUnroll consecutive planes are issued before any of
// them is used, so each wave keeps kWtaUnroll KB in flight (one plane at a time measured 4.4 TB/s:
// a read stream needs ~20 KB in flight per CU at HBM latency).  The d range is split over SPLIT
// thread groups of one workgroup (same pixels, consecutive d ranges), merged through LDS in d order:
// SPLIT times the workgroups of a one-group-per-pixel-block grid, for the same bytes per thread.
#ifndef SM_WTA_UNROLL
#define SM_WTA_UNROLL 16   // 8-frame launches: 81.4 us per frame vs 93.5 for 8 (with nontemporal SAD stores)
#endif
#ifndef SM_WTA_SPLIT
#define SM_WTA_SPLIT 4   // 1080p D=128 same-box A/B: 102.6 us (1 group), 99.2 (4 groups)
#endif
constexpr int kWtaUnroll = SM_WTA_UNROLL;
// nontemporal: plain loads measured 135 us against 103 (one group)
__device__ __forceinline__ u32x4 ld_plane(const u32x4* p) { return __builtin_nontemporal_load(p); }
constexpr int kWtaSplit = SM_WTA_SPLIT;

__global__ __launch_bounds__(kST) void volume_wta_kernel(const uint16_t* __restrict__ sad, int W, int H, int D,
                                                         uint32_t seed_key, uint8_t* __restrict__ disp,
                                                         int out_pitch, int64_t out_stride) {
    constexpr int NPX = 8;
    // frame blockIdx.y of the launch group: its D planes follow the previous frame's
    sad += (int64_t)blockIdx.y * D * ((int64_t)W * H);
    disp += (int64_t)blockIdx.y * out_stride;
    constexpr int TPG = kST / kWtaSplit;             // threads per d group
    __shared__ uint32_t part[kWtaSplit > 1 ? kWtaSplit - 1 : 1][TPG][NPX + 1];
    const int64_t P = (int64_t)W * H;
    const int grp = threadIdx.x / TPG, gt = threadIdx.x - grp * TPG;
    const int64_t p0 = ((int64_t)blockIdx.x * TPG + gt) * NPX;
    const int n = p0 >= P ? 0 : (P - p0 < NPX ? (int)(P - p0) : NPX);
    // this group's planes: [d_lo, d_hi), whole unroll blocks except the last group
    const int dper = ((D + kWtaSplit - 1) / kWtaSplit + kWtaUnroll - 1) / kWtaUnroll * kWtaUnroll;
    const int d_lo = min(D, grp * dper), d_hi = min(D, d_lo + dper);
    int lim[NPX];
    uint32_t best[NPX];
#pragma unroll
    for (int k = 0; k < NPX; ++k) {
        lim[k] = W - (int)((p0 + k) % W);            // validity: d <= W - x (Device.cu:44)
        best[k] = seed_key;
    }
    auto take = [&](uint32_t word, int k, int d) {
        const uint32_t key = (word << 8) | (uint32_t)d;
        best[k] = (d <= lim[k] && key < best[k]) ? key : best[k];
    };
    const bool vec = n == NPX && ((reinterpret_cast<uintptr_t>(sad) & 15) == 0) && ((P & 7) == 0);
    if (vec) {
        const u32x4* base = reinterpret_cast<const u32x4*>(sad + p0);
        const int64_t pstride = P / 8;                // one plane in u32x4 units
        int d = d_lo;
        for (; d + kWtaUnroll <= d_hi; d += kWtaUnroll) {
            u32x4 v[kWtaUnroll];
#pragma unroll
            for (int u = 0; u < kWtaUnroll; ++u) v[u] = ld_plane(base + (int64_t)(d + u) * pstride);
#pragma unroll
            for (int u = 0; u < kWtaUnroll; ++u)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    take(v[u][q] & 0xFFFFu, 2 * q, d + u);
                    take(v[u][q] >> 16, 2 * q + 1, d + u);
                }
        }
        for (; d < d_hi; ++d) {
            const u32x4 v = ld_plane(base + (int64_t)d * pstride);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                take(v[q] & 0xFFFFu, 2 * q, d);
                take(v[q] >> 16, 2 * q + 1, d);
            }
        }
    } else if (n > 0) {
        for (int d = d_lo; d < d_hi; ++d) {
            const uint16_t* pl = sad + (int64_t)d * P + p0;
#pragma unroll
            for (int k = 0; k < NPX; ++k)
                if (k < n) take(pl[k], k, d);
        }
    }
    if constexpr (kWtaSplit > 1) {
        // keys (SAD << 8 | d) order by cost, then d: a plain min over the groups is the first-d argmin
        if (grp > 0)
#pragma unroll
            for (int k = 0; k < NPX; ++k) part[grp - 1][gt][k] = best[k];
        __syncthreads();
        if (grp > 0) return;
#pragma unroll
        for (int g = 0; g < kWtaSplit - 1; ++g)
#pragma unroll
            for (int k = 0; k < NPX; ++k) best[k] = min(best[k], part[g][gt][k]);
    }
#pragma unroll
    for (int k = 0; k < NPX; ++k) {
        if (k >= n) break;
        const int64_t p = p0 + k;
        const int y = (int)(p / W), x = (int)(p - (int64_t)y * W);
        disp[(int64_t)y * out_pitch + x] = best[k] < seed_key ? (uint8_t)(best[k] & 0xFFu) : (uint8_t)0;
    }
}

// getAllSAD (BlockMatching.cpp:191-261): the SAD volume pixel-major, data_dm[p * D + d], each sum stored
// as uchar (truncated mod 256, :258) and 255 where x + d > W (:245-249).  The d-major u16 volume of
// box_sad_kernel is transposed through LDS, 64 pixels per block: the loads read 128 B of one plane per
// wave and d, and the block's 64 * D output bytes are one contiguous run written as dwords.  The low 8
// bits of a u16 sum are the low 8 bits of the true sum, so uchar truncation of either is the same.
constexpr int kAsPx = 64;
__global__ __launch_bounds__(kST) void all_sad_transpose_kernel(const uint16_t* __restrict__ sad, int W, int64_t P,
                                                                int D, int Dp, uint8_t* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t tile[];   // [kAsPx][Dp]
    const int64_t p0 = (int64_t)blockIdx.x * kAsPx;
    const int npx = P - p0 < kAsPx ? (int)(P - p0) : kAsPx;
    // a thread always handles pixel px = tid mod 64 (its e advances by 256 = 4 * 64): one x per thread
    const int px = threadIdx.x & (kAsPx - 1);
    const int x = (int)((p0 + px) % W);
    if (px < npx) {
        for (int d = threadIdx.x >> 6; d < D; d += kST / kAsPx) {
            const uint16_t v = sad[(int64_t)d * P + p0 + px];
            tile[px * Dp + d] = x + d > W ? (uint8_t)255 : (uint8_t)v;
        }
    }
    __syncthreads();
    uint8_t* o = out + p0 * D;
    const int n = npx * D;
    if ((D & 3) == 0 && (reinterpret_cast<uintptr_t>(o) & 3) == 0) {
        for (int e = 4 * threadIdx.x; e < n; e += 4 * kST) {
            const int q = e / D, d = e - q * D;
            *reinterpret_cast<uint32_t*>(o + e) = *reinterpret_cast<const uint32_t*>(tile + q * Dp + d);
        }
    } else {
        for (int e = threadIdx.x; e < n; e += kST) {
            const int q = e / D;
            o[e] = tile[q * Dp + (e - q * D)];
        }
    }
}

// getAllSAD at any radius (the u16 volume's box_sad_kernel covers r <= 7): one thread per (row, d),
// lanes over d, walking the row with a running sum of column sums; each column sum is its (clipped)
// 2r + 1 taps of |L - R(x - d)|, zero where x < d (Device.cu:27-31).  The stores of one wave and column
// are 64 consecutive bytes of the pixel-major volume.  Not a performance path: the reference's
// getAllSAD is a CPU debugging aid (BlockMatching.h:11, Device.cu:265-268).
__global__ __launch_bounds__(kST) void all_sad_generic_kernel(const uint8_t* __restrict__ L,
                                                              const uint8_t* __restrict__ R, int W, int H, int pitch,
                                                              int radius, int D, uint8_t* __restrict__ out) {
    const int d = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * (kST / 64) + (threadIdx.x >> 6);
    if (d >= D || y >= H) return;
    const int y0 = max(0, y - radius), y1 = min(H - 1, y + radius);
    auto colsum = [&](int xc) -> uint32_t {
        if (xc < 0 || xc >= W || xc < d) return 0u;
        uint32_t s = 0;
        for (int yy = y0; yy <= y1; ++yy) {
            const int a = L[(int64_t)yy * pitch + xc], b = R[(int64_t)yy * pitch + xc - d];
            s += (uint32_t)(a > b ? a - b : b - a);
        }
        return s;
    };
    uint32_t S = 0;
    for (int j = -radius; j <= radius; ++j) S += colsum(j);
    uint8_t* o = out + (int64_t)y * W * D + d;
    for (int x = 0; x < W; ++x) {
        o[(int64_t)x * D] = x + d > W ? (uint8_t)255 : (uint8_t)S;
        S += colsum(x + radius + 1) - colsum(x - radius);
    }
}

template <int R>
hipError_t launch_box_sad_r(const uint8_t* ad, int W, int H, int D, uint16_t* sad, hipStream_t s) {
    const int strips = (W + kSO - 1) / kSO;
    // ~kSadBlocks blocks, bands of >= 32 rows (the 2r halo rows of a band are read twice)
    int bands = (kSadBlocks + strips * D - 1) / (strips * D);
    const int max_bands = (H + 31) / 32;
    bands = bands < 1 ? 1 : (bands > max_bands ? max_bands : bands);
    const int rows = (H + bands - 1) / bands;
    bands = (H + rows - 1) / rows;
    const int64_t blocks = (int64_t)strips * bands * D;
    if (blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    hipLaunchKernelGGL(box_sad_kernel<R>, dim3((unsigned)blocks), dim3(kST), 0, s, ad, W, H, rows, bands, strips, sad);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_box_sad_volume(const uint8_t* ad, int W, int H, int radius, int D, uint16_t* sad, hipStream_t s) {
#define SM_BOX_SAD_CASE(r) \
    case r: return launch_box_sad_r<r>(ad, W, H, D, sad, s)
    switch (radius) {
        SM_BOX_SAD_CASE(0);
        SM_BOX_SAD_CASE(1);
        SM_BOX_SAD_CASE(2);
        SM_BOX_SAD_CASE(3);
        SM_BOX_SAD_CASE(4);
        SM_BOX_SAD_CASE(5);
        SM_BOX_SAD_CASE(6);
        SM_BOX_SAD_CASE(7);
        default: return hipErrorInvalidValue;
    }
#undef SM_BOX_SAD_CASE
}

hipError_t launch_all_sad_transpose(const uint16_t* sad, int W, int H, int D, uint8_t* out, hipStream_t s) {
    const int64_t P = (int64_t)W * H;
    const int64_t blocks = (P + kAsPx - 1) / kAsPx;
    if (W <= 0 || H <= 0 || D < 1 || D > kMaxDisp || blocks > 0x7FFFFFFF) return hipErrorInvalidValue;
    const int Dp = ((D + 3) & ~3) + 4;   // dword-aligned tile rows, offset by one bank per pixel
    hipLaunchKernelGGL(all_sad_transpose_kernel, dim3((unsigned)blocks), dim3(kST), (size_t)(kAsPx * Dp), s, sad, W, P,
                       D, Dp, out);
    return hipGetLastError();
}

hipError_t launch_all_sad_generic(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int radius, int D,
                                  uint8_t* out, hipStream_t s) {
    if (W <= 0 || H <= 0 || D < 1 || D > kMaxDisp || radius < 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(all_sad_generic_kernel, dim3((unsigned)((D + 63) / 64), (unsigned)((H + 3) / 4)), dim3(kST), 0,
                       s, L, R, W, H, pitch, radius, D, out);
    return hipGetLastError();
}

hipError_t launch_volume_wta(const uint16_t* sad, int W, int H, int D, int frames, uint32_t seed_key, uint8_t* disp,
                             int out_pitch, int64_t out_stride, hipStream_t s) {
    const int64_t P = (int64_t)W * H;
    const int64_t blocks = (P + 8 * (kST / kWtaSplit) - 1) / (8 * (kST / kWtaSplit));
    if (blocks <= 0 || blocks > 0x7FFFFFFF || frames <= 0 || frames > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(volume_wta_kernel, dim3((unsigned)blocks, (unsigned)frames), dim3(kST), 0, s, sad, W, H, D,
                       seed_key, disp, out_pitch, out_stride);
    return hipGetLastError();
}

}  // namespace sm
