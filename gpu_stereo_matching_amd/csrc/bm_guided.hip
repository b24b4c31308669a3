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
    const int yo = y0 + hj;
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
    for (int f = 0; f < batch; ++f) {
        const uint8_t* Lf = L + (int64_t)f * frame_stride;
        const uint8_t* Rf = R + (int64_t)f * frame_stride;
        uint8_t* Df = disp + (int64_t)f * out_frame_stride;
        hipError_t e;
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
