/*
 * bm_oracle.c — CPU restatement of the reference block-matching path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (gpu_stereo_matching_amd/,
 * include/) links, loads or calls this file.  It is imported exclusively by
 * tests/, by __graft_entry__.smoke() as the checker, and by bench.py's
 * cpu_baseline leg (timed, never used to produce the measured GPU result).
 *
 * Reference: ningw42/GPU_Stereo_Matching (read-only at /root/reference).
 * The reference's own CPU file BlockMatching/BlockMatching.cpp needs OpenCV
 * headers that this image does not have, so it is unbuildable here (see
 * DESIGN.md §Oracle).  Every function below restates the algorithm of the
 * cited reference lines in plain C; the comments say which line each rule
 * comes from.
 *
 * Layouts: images are uint8 row-major, width W, height H, row pitch == W.
 *          cost volumes are d-major planes [D][H][W] (as Device.cu:193).
 */
#include <stdint.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <stdlib.h>
#include <string.h>
#include <math.h>

#define ORA_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------- */
/* a9: gray conversion used by the caller before the path                    */
/* Caller.cpp:15-16 cvtColor(..., CV_BGR2GRAY) on an imread() BGR image.     */
/* OpenCV 2.4 8-bit fixed point: Y = (1868 B + 9617 G + 4899 R + 8192) >> 14  */
/* ------------------------------------------------------------------------- */
ORA_API void ora_bgr_to_gray(const uint8_t *bgr, int64_t npix, int channels, uint8_t *gray)
{
    for (int64_t i = 0; i < npix; ++i) {
        const uint8_t *px = bgr + i * channels;
        uint32_t y = 1868u * px[0] + 9617u * px[1] + 4899u * px[2] + 8192u;
        gray[i] = (uint8_t)(y >> 14);
    }
}

/* ------------------------------------------------------------------------- */
/* next: rectification remap, the reference's CPU twin   */
/* CPU_Remap + CPU_BilinearInterpolation (Utility.cpp:239-264), identical    */
/* to kernalRemap/BilinearInterpolation (Device.cu:127-167):                 */
/*   x = map_y (row), y = map_x (col); taps outside [0,rows-1]x[0,cols-1]     */
/*   -> 0; value = bilinear blend evaluated in float exactly as written       */
/*   (no FMA contraction: built with -ffp-contract=off); saturate_cast<uchar> */
/*   = round half to even + clamp.                                            */
/* ------------------------------------------------------------------------- */
static float ora_bilinear(const uint8_t *src, int rows, int cols, float x, float y)
{
    int x1 = (int)floorf(x), y1 = (int)floorf(y), x2 = x1 + 1, y2 = y1 + 1;
    if (x1 < 0 || x2 >= rows || y1 < 0 || y2 >= cols) return 0.0f;
    float q11 = src[x1 * cols + y1], q12 = src[x1 * cols + y2], q21 = src[x2 * cols + y1], q22 = src[x2 * cols + y2];
    float left = (x2 - x) * q11 + (x - x1) * q21;
    float right = (x2 - x) * q12 + (x - x1) * q22;
    return (y2 - y) * left + (y - y1) * right;
}

ORA_API void ora_remap(const uint8_t *src, int W, int H, const float *mapx, const float *mapy, uint8_t *dst)
{
    for (int row = 0; row < H; ++row)
        for (int col = 0; col < W; ++col) {
            float v = ora_bilinear(src, H, W, mapy[row * W + col], mapx[row * W + col]);
            float r = rintf(v);
            if (!(r > 0.0f)) r = 0.0f;
            if (r > 255.0f) r = 255.0f;
            dst[row * W + col] = (uint8_t)r;
        }
}

/* ------------------------------------------------------------------------- */
/* Rectification maps in front of the remap: Rectify (Utility.cpp:228-234)     */
/* calls initUndistortRectifyMap(K, dist, R1, P1, size, CV_32FC1, mapX, mapY).  */
/* OpenCV 2.4.12 is a third-party dependency absent from the reference tree;   */
/* this restates its published imgproc/src/undistort.cpp algorithm:            */
/*   iR = (P[:, :3] * R)^-1, the 3x3 inverse by OpenCV's adjugate formula       */
/*        (cv::invert DECOMP_LU for n == 3: det3, d = 1/det, cofactors * d);    */
/*   per row i: _x = i*ir[1] + ir[2], _y = i*ir[4] + ir[5], _w = i*ir[7] + ir[8],*/
/*   then per column j (accumulated: _x += ir[0], _y += ir[3], _w += ir[6]):    */
/*   w = 1/_w, x = _x*w, y = _y*w, r2 = x^2 + y^2,                               */
/*   kr = (1 + ((k3 r2 + k2) r2 + k1) r2) / (1 + ((k6 r2 + k5) r2 + k4) r2),     */
/*   u = fx (x kr + p1 2xy + p2 (r2 + 2x^2)) + u0,                              */
/*   v = fy (y kr + p1 (r2 + 2y^2) + p2 2xy) + v0,   map = ((float)u, (float)v). */
/* dist holds ndist (0, 4, 5 or 8) coefficients k1 k2 p1 p2 [k3 [k4 k5 k6]].   */
/* Compiled with -ffp-contract=off, so every product / sum rounds as written.  */
/* Parity with OpenCV itself is unpinned (no OpenCV here).                     */
/* ------------------------------------------------------------------------- */
static void ora_inv3(const double *m, double *t)
{
    double d = (m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6])) +
               m[2] * (m[3] * m[7] - m[4] * m[6]);
    d = 1. / d;
    t[0] = (m[4] * m[8] - m[5] * m[7]) * d;
    t[1] = (m[2] * m[7] - m[1] * m[8]) * d;
    t[2] = (m[1] * m[5] - m[2] * m[4]) * d;
    t[3] = (m[5] * m[6] - m[3] * m[8]) * d;
    t[4] = (m[0] * m[8] - m[2] * m[6]) * d;
    t[5] = (m[2] * m[3] - m[0] * m[5]) * d;
    t[6] = (m[3] * m[7] - m[4] * m[6]) * d;
    t[7] = (m[1] * m[6] - m[0] * m[7]) * d;
    t[8] = (m[0] * m[4] - m[1] * m[3]) * d;
}

ORA_API void ora_init_rectify_map(const double *K, const double *dist, int ndist, const double *R,
                                  const double *P, int W, int H, float *mapx, float *mapy)
{
    double k[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ar[9], iR[9];
    for (int i = 0; i < ndist && i < 8; ++i) k[i] = dist[i];
    for (int i = 0; i < 3; ++i)          /* Ar = P(:, 0:3) (3x4 row-major), Ar * R */
        for (int j = 0; j < 3; ++j)
            ar[i * 3 + j] = ((P[i * 4 + 0] * R[0 * 3 + j]) + P[i * 4 + 1] * R[1 * 3 + j]) + P[i * 4 + 2] * R[2 * 3 + j];
    ora_inv3(ar, iR);
    const double u0 = K[2], v0 = K[5], fx = K[0], fy = K[4];
    const double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3], k3 = k[4], k4 = k[5], k5 = k[6], k6 = k[7];
    for (int i = 0; i < H; ++i) {
        double _x = i * iR[1] + iR[2], _y = i * iR[4] + iR[5], _w = i * iR[7] + iR[8];
        for (int j = 0; j < W; ++j, _x += iR[0], _y += iR[3], _w += iR[6]) {
            double w = 1. / _w, x = _x * w, y = _y * w;
            double x2 = x * x, y2 = y * y;
            double r2 = x2 + y2, _2xy = 2 * x * y;
            double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2);
            double u = fx * (x * kr + p1 * _2xy + p2 * (r2 + 2 * x2)) + u0;
            double v = fy * (y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy) + v0;
            mapx[(int64_t)i * W + j] = (float)u;
            mapy[(int64_t)i * W + j] = (float)v;
        }
    }
}

/* ------------------------------------------------------------------------- */
/* a1: absolute-difference volume.                                           */
/* PreCal BlockMatching.cpp:89-109 / kernalPreCal_V2 Device.cu:19-32:        */
/*   dif[d][p] = |L[p] - R[p-d]| when (p mod W) >= d, else left at the       */
/*   memset value 0 (BlockMatching.cpp:143, Device.cu:194).                  */
/* ------------------------------------------------------------------------- */
ORA_API void ora_precal(const uint8_t *L, const uint8_t *R, int W, int H, int D, uint8_t *dif)
{
    const int64_t P = (int64_t)W * H;
    memset(dif, 0, (size_t)(P * D));
    for (int d = 0; d < D; ++d) {
        uint8_t *plane = dif + (int64_t)d * P;
        for (int y = 0; y < H; ++y) {
            const uint8_t *l = L + (int64_t)y * W;
            const uint8_t *r = R + (int64_t)y * W;
            uint8_t *o = plane + (int64_t)y * W;
            for (int x = d; x < W; ++x) {
                int v = (int)l[x] - (int)r[x - d];
                o[x] = (uint8_t)(v < 0 ? -v : v);
            }
        }
    }
}

/* ------------------------------------------------------------------------- */
/* a2/a4: literal restatement of getDisp (BlockMatching.cpp:111-189), the    */
/* CPU twin of kernalFindCorr (Device.cu:34-64).  Same loop nest, same       */
/* early exit (:174-176), same start value 50*win^2 (:157), same -256 seed   */
/* (:158) truncated to uchar on store (:184).  Used as the CPU baseline      */
/* ("port") and as the slow-path checker.                                     */
/*   dif: caller-provided scratch of P*D bytes, or NULL to allocate.          */
/* ------------------------------------------------------------------------- */
ORA_API int ora_get_disp(const uint8_t *L, const uint8_t *R, int W, int H, int radius, int D,
                         uint8_t *out, uint8_t *dif)
{
    const int64_t P = (int64_t)W * H;
    const int win = 2 * radius + 1;
    const int taps = win * win;
    uint8_t *own = NULL;
    if (!dif) {
        own = (uint8_t *)malloc((size_t)(P * D));
        if (!own) return -1;
        dif = own;
    }
    /* tap table: (dx, dy, linear offset) in raster order of the window
       (BlockMatching.cpp:130-133: i%win - r, i/win - r, dx + dy*W) */
    int *tdx = (int *)malloc(sizeof(int) * taps);
    int *tdy = (int *)malloc(sizeof(int) * taps);
    int64_t *toff = (int64_t *)malloc(sizeof(int64_t) * taps);
    for (int t = 0; t < taps; ++t) {
        tdx[t] = t % win - radius;
        tdy[t] = t / win - radius;
        toff[t] = tdx[t] + (int64_t)tdy[t] * W;
    }
    ora_precal(L, R, W, H, D, dif);

    for (int64_t p = 0; p < P; ++p) {
        const int col = (int)(p % W), row = (int)(p / W);
        int best = 50 * taps;
        int dm = -256;
        for (int d = 0; d < D; ++d) {
            if (col + d > W) break;                         /* :166 */
            const uint8_t *plane = dif + (int64_t)d * P;
            int acc = 0;
            for (int t = 0; t < taps; ++t) {
                int c = col + tdx[t];
                if (c >= W || c < 0) continue;              /* :170 */
                int rr = row + tdy[t];
                if (rr >= H || rr < 0) continue;            /* :172 */
                acc += plane[p + toff[t]];
                if (acc > best) break;                      /* :174-176 */
            }
            if (acc < best) { best = acc; dm = d; }         /* :178-181 */
        }
        out[p] = (uint8_t)dm;                               /* :184 */
    }
    free(tdx); free(tdy); free(toff); free(own);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* a6: literal restatement of getAllSAD (BlockMatching.cpp:191-261), the CPU  */
/* twin of the dead kernalFindAllSAD (Device.cu:67-103): every window SAD,    */
/* pixel-major out[p*D + d], stored into uchar (truncated mod 256, :258), and */
/* 255 where col + d > W (:245-249).  No early exit in this loop nest.  The   */
/* memset of the first P bytes (:201) is overwritten by the loop, which       */
/* writes every one of the P*D entries.                                        */
/*   dif: caller-provided scratch of P*D bytes, or NULL to allocate.          */
/* ------------------------------------------------------------------------- */
ORA_API int ora_get_all_sad(const uint8_t *L, const uint8_t *R, int W, int H, int radius, int D,
                            uint8_t *out, uint8_t *dif)
{
    const int64_t P = (int64_t)W * H;
    const int win = 2 * radius + 1;
    const int taps = win * win;
    uint8_t *own = NULL;
    if (!dif) {
        own = (uint8_t *)malloc((size_t)(P * D));
        if (!own) return -1;
        dif = own;
    }
    int *tdx = (int *)malloc(sizeof(int) * taps);
    int *tdy = (int *)malloc(sizeof(int) * taps);
    int64_t *toff = (int64_t *)malloc(sizeof(int64_t) * taps);
    for (int t = 0; t < taps; ++t) {                        /* :209-212 */
        tdx[t] = t % win - radius;
        tdy[t] = t / win - radius;
        toff[t] = tdx[t] + (int64_t)tdy[t] * W;
    }
    ora_precal(L, R, W, H, D, dif);                         /* :221-230 */
    memset(out, 0, (size_t)P);                              /* :201 */
    for (int64_t p = 0; p < P; ++p) {
        const int col = (int)(p % W), row = (int)(p / W);
        for (int d = 0; d < D; ++d) {
            if (col + d > W) {                              /* :245-249 */
                out[p * D + d] = 255;
                continue;
            }
            const uint8_t *plane = dif + (int64_t)d * P;
            int acc = 0;
            for (int t = 0; t < taps; ++t) {
                int c = col + tdx[t];
                if (c >= W || c < 0) continue;              /* :253 */
                int rr = row + tdy[t];
                if (rr >= H || rr < 0) continue;            /* :255 */
                acc += plane[p + toff[t]];
            }
            out[p * D + d] = (uint8_t)acc;                  /* :258, uchar store */
        }
    }
    free(tdx); free(tdy); free(toff); free(own);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* a1+a2 as Device.cu actually launches them (blockMatching_gpu, :173-301),  */
/* launch geometry included:                                                  */
/*  - d_disparity and d_difference are memset to 0 (:191-194);                */
/*  - kernalPreCal_V2 runs on grid (8, 10, D) x block (32, 32) (:231-233):    */
/*    rowIndex = blockIdx.x*32 + threadIdx.x < 256, colIndex = blockIdx.y*32  */
/*    + threadIdx.y < 320 (:21-22), so only rows < 256, cols < 320 get an AD  */
/*    value (:27-31); the rest of every plane keeps the memset 0;             */
/*  - kernalFindCorr runs <<<rows, cols>>> (:253): one thread per pixel, the  */
/*    getDisp rule without the early exit (:36-63).  A block of more than     */
/*    1024 threads does not launch, so for cols > 1024 the map stays the      */
/*    memset 0 (the reference checks no error).                               */
/* rows < 256 or cols < 320 make the fixed grid read and write outside the    */
/* frame (frameBias up to 255*cols + 319 >= rows*cols): undefined in the      */
/* reference, rejected here (returns -2).  At exactly 320x256 the grid covers */
/* every (row, col, d) and this equals ora_get_disp.                          */
/* ------------------------------------------------------------------------- */
ORA_API int ora_device_cu_literal(const uint8_t *L, const uint8_t *R, int W, int H, int radius, int D,
                                  uint8_t *out)
{
    const int64_t total = (int64_t)W * H;
    if (W < 320 || H < 256) return -2;
    memset(out, 0, (size_t)total);                          /* :191-192 */
    if (W > 1024) return 0;                                 /* :253 launch failure */
    uint8_t *dif = (uint8_t *)calloc((size_t)(total * D), 1); /* :193-194 */
    if (!dif) return -1;
    for (int z = 0; z < D; ++z)                             /* grid.z = frameIndex */
        for (int bx = 0; bx < 8; ++bx)
            for (int by = 0; by < 10; ++by)
                for (int tx = 0; tx < 32; ++tx)
                    for (int ty = 0; ty < 32; ++ty) {
                        const int colIndex = by * 32 + ty;  /* :21 */
                        const int rowIndex = bx * 32 + tx;  /* :22 */
                        const int64_t frameBias = (int64_t)rowIndex * W + colIndex; /* :23 */
                        const int64_t index = (int64_t)z * total + frameBias;       /* :25 */
                        if (colIndex - z >= 0) {            /* :27-28 */
                            int v = (int)L[frameBias] - (int)R[frameBias - z];
                            dif[index] = (uint8_t)(v < 0 ? -v : v);             /* :30 */
                        }
                    }
    const int windowArea = (2 * radius + 1) * (2 * radius + 1);
    for (int64_t t = 0; t < total; ++t) {                   /* threadIndex, :36 */
        int best = 50 * windowArea;                         /* :37 */
        int dm = -256;                                      /* :38 */
        const int col = (int)(t % W), row = (int)(t / W);   /* :39-40 */
        int64_t th = 0;
        for (int s = 0; s < D; ++s, th += total) {          /* :43 */
            if (col + s > W) break;                         /* :44 */
            int sad = 0;
            for (int i = -radius; i <= radius; ++i)
                for (int j = -radius; j <= radius; ++j) {
                    const int c = col + j;
                    if (c >= W || c < 0) continue;          /* :51 */
                    const int rr = row + i;
                    if (rr >= H || rr < 0) continue;        /* :53 */
                    sad += dif[th + t + (int64_t)W * i + j]; /* :54 */
                }
            if (sad < best) { dm = s; best = sad; }         /* :57-60 */
        }
        out[t] = (uint8_t)dm;                               /* :63 */
    }
    free(dif);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* a3: independent restatement of the same map as                            */
/*   zero-padded (2r+1)^2 box sum of each AD plane                           */
/*   + validity d <= W - x (the break at BlockMatching.cpp:166/Device.cu:44) */
/*   + strict-< WTA seeded with 50*win^2, no match -> 0.                     */
/* Separable running sums, O(P*D); fast enough for 1080p parity tests.       */
/* Optional outputs: cost volume [D][H][W] int32 (box SAD, no validity), and */
/* the winning packed key per pixel ((cost << 8) | d, or T << 8 for none).   */
/* ------------------------------------------------------------------------- */
static void box_plane(const uint8_t *L, const uint8_t *R, int W, int H, int r, int d,
                      int32_t *colsum /* W */, int32_t *out /* H*W */)
{
    /* running vertical window sums per column (rows outside the image add
       nothing), then a running horizontal window sum per row */
    memset(colsum, 0, sizeof(int32_t) * W);
    for (int yy = 0; yy < r && yy < H; ++yy) {
        const uint8_t *l = L + (int64_t)yy * W, *rr = R + (int64_t)yy * W;
        for (int x = d; x < W; ++x) { int v = (int)l[x] - (int)rr[x - d]; colsum[x] += v < 0 ? -v : v; }
    }
    for (int y = 0; y < H; ++y) {
        if (y + r < H) {
            const uint8_t *l = L + (int64_t)(y + r) * W, *rr = R + (int64_t)(y + r) * W;
            for (int x = d; x < W; ++x) { int v = (int)l[x] - (int)rr[x - d]; colsum[x] += v < 0 ? -v : v; }
        }
        if (y - r - 1 >= 0) {
            const uint8_t *l = L + (int64_t)(y - r - 1) * W, *rr = R + (int64_t)(y - r - 1) * W;
            for (int x = d; x < W; ++x) { int v = (int)l[x] - (int)rr[x - d]; colsum[x] -= v < 0 ? -v : v; }
        }
        int32_t *o = out + (int64_t)y * W;
        int32_t run = 0;
        for (int x = 0; x < r && x < W; ++x) run += colsum[x];
        for (int x = 0; x < W; ++x) {
            if (x + r < W) run += colsum[x + r];
            if (x - r - 1 >= 0) run -= colsum[x - r - 1];
            o[x] = run;
        }
    }
}

ORA_API int ora_box_disp(const uint8_t *L, const uint8_t *R, int W, int H, int radius, int D,
                         uint8_t *out, int32_t *cost_out, uint32_t *key_out)
{
    const int64_t P = (int64_t)W * H;
    const int win = 2 * radius + 1;
    const int32_t T = 50 * win * win;
    int32_t *colsum = (int32_t *)malloc(sizeof(int32_t) * W);
    int32_t *plane = (int32_t *)malloc(sizeof(int32_t) * P);
    int32_t *best = (int32_t *)malloc(sizeof(int32_t) * P);
    int32_t *bd = (int32_t *)malloc(sizeof(int32_t) * P);
    if (!colsum || !plane || !best || !bd) { free(colsum); free(plane); free(best); free(bd); return -1; }
    for (int64_t p = 0; p < P; ++p) { best[p] = T; bd[p] = -256; }
    for (int d = 0; d < D; ++d) {
        box_plane(L, R, W, H, radius, d, colsum, plane);
        if (cost_out) memcpy(cost_out + (int64_t)d * P, plane, sizeof(int32_t) * P);
        for (int y = 0; y < H; ++y) {
            for (int x = 0; x < W; ++x) {
                if (x + d > W) continue;
                int64_t p = (int64_t)y * W + x;
                if (plane[p] < best[p]) { best[p] = plane[p]; bd[p] = d; }
            }
        }
    }
    for (int64_t p = 0; p < P; ++p) {
        out[p] = (uint8_t)bd[p];
        if (key_out) key_out[p] = bd[p] < 0 ? ((uint32_t)T << 8) : (((uint32_t)best[p] << 8) | (uint32_t)(bd[p] & 0xFF));
    }
    free(colsum); free(plane); free(best); free(bd);
    return 0;
}

/* Box SAD cost volume only ([D][H][W] int32), for LR / key tests. */
ORA_API int ora_box_cost(const uint8_t *L, const uint8_t *R, int W, int H, int radius, int D, int32_t *cost)
{
    int32_t *colsum = (int32_t *)malloc(sizeof(int32_t) * W);
    if (!colsum) return -1;
    for (int d = 0; d < D; ++d)
        box_plane(L, R, W, H, radius, d, colsum, cost + (int64_t)d * W * H);
    free(colsum);
    return 0;
}

/* Partial-range key map for one d-slice [d_lo, d_hi): per pixel the minimum of
   (cost << 8 | d) over valid d in the slice, seeded with T << 8.  The min over
   slices equals ora_box_disp's key (the multi-GPU reduction contract). */
ORA_API int ora_box_keys_slice(const uint8_t *L, const uint8_t *R, int W, int H, int radius,
                               int d_lo, int d_hi, uint32_t *keys)
{
    const int64_t P = (int64_t)W * H;
    const int win = 2 * radius + 1;
    const uint32_t seed = (uint32_t)(50 * win * win) << 8;
    int32_t *colsum = (int32_t *)malloc(sizeof(int32_t) * W);
    int32_t *plane = (int32_t *)malloc(sizeof(int32_t) * P);
    if (!colsum || !plane) { free(colsum); free(plane); return -1; }
    for (int64_t p = 0; p < P; ++p) keys[p] = seed;
    for (int d = d_lo; d < d_hi; ++d) {
        box_plane(L, R, W, H, radius, d, colsum, plane);
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                if (x + d > W) continue;
                int64_t p = (int64_t)y * W + x;
                uint32_t k = ((uint32_t)plane[p] << 8) | (uint32_t)(d & 0xFF);
                if (k < keys[p]) keys[p] = k;
            }
    }
    free(colsum); free(plane);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* a7: left-right consistency.                                               */
/* Right cost from the left volume, GetRightMatchingCostFromLeft             */
/*   (STMatching/StereoHelper.cpp:156-180): C_R(y,x,d) = C_L(y,x+d,d) when   */
/*   x+d < W, else C_R(y,x,d-1).                                             */
/* Right WTA, GetDisparity_WTA (StereoHelper.cpp:131-154): argmin from d=0,  */
/*   strict <, no threshold.                                                 */
/* Check, StereoDisparity.cpp:136-147: d = dL(y,x); occluded when x-d < 0,   */
/*   d == 0, or |d - dR(y,x-d)| > 1.  Output: checked map (occluded -> 0)    */
/*   and the valid mask (!occ).                                              */
/* cost: [D][H][W] int32 (ora_box_cost).                                     */
/* ------------------------------------------------------------------------- */
ORA_API void ora_right_wta(const int32_t *cost, int W, int H, int D, uint8_t *right_disp)
{
    const int64_t P = (int64_t)W * H;
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            int64_t rowbase = (int64_t)y * W;
            /* walk d keeping the clamped value like StereoHelper.cpp:170-175 */
            int32_t cur = cost[rowbase + x];              /* d = 0: x+0 < W */
            int32_t minv = cur;
            int minpos = 0;
            for (int d = 1; d < D; ++d) {
                if (x + d < W) cur = cost[(int64_t)d * P + rowbase + x + d];
                /* else cur stays = C_R(y,x,d-1) */
                if (cur < minv) { minv = cur; minpos = d; }
            }
            right_disp[rowbase + x] = (uint8_t)minpos;
        }
    }
}

/* Box left + right WTA in O(P) memory per thread (full-size LR checks, cfg5 at
   3840x2160 D=192, without the D x P volume).  Left: ora_box_disp's rule.
   Right: STMatching's C_R(y,u,d) = C_L(y,u+d,d) for u+d < W, else C_R(y,u,d-1)
   (StereoHelper.cpp:156-180); the repeated value never wins a strict < again,
   so the right WTA is the first argmin over d with u+d < W (:131-154).
   OpenMP over contiguous d chunks; chunks merge in d order with strict <, so
   ties keep the smaller d exactly as the sequential scan does. */
ORA_API int ora_box_lr_probe(const uint8_t *L, const uint8_t *R, int W, int H, int radius, int D,
                             uint8_t *left_out, uint8_t *right_out)
{
    const int64_t P = (int64_t)W * H;
    const int win = 2 * radius + 1;
    const int32_t T = 50 * win * win;
    int nt = 1;
#ifdef _OPENMP
    nt = omp_get_max_threads();
#endif
    if (nt > D) nt = D;
    if (nt < 1) nt = 1;
    int32_t *bl = (int32_t *)malloc(sizeof(int32_t) * P * nt), *dl = (int32_t *)malloc(sizeof(int32_t) * P * nt);
    int32_t *br = (int32_t *)malloc(sizeof(int32_t) * P * nt), *dr = (int32_t *)malloc(sizeof(int32_t) * P * nt);
    int fail = !bl || !dl || !br || !dr;
    if (!fail) {
#pragma omp parallel num_threads(nt)
        {
            int t = 0;
#ifdef _OPENMP
            t = omp_get_thread_num();
#endif
            int d0 = (int)((int64_t)D * t / nt), d1 = (int)((int64_t)D * (t + 1) / nt);
            int32_t *colsum = (int32_t *)malloc(sizeof(int32_t) * W);
            int32_t *plane = (int32_t *)malloc(sizeof(int32_t) * P);
            int32_t *b_l = bl + P * t, *d_l = dl + P * t, *b_r = br + P * t, *d_r = dr + P * t;
            if (!colsum || !plane) {
#pragma omp atomic write
                fail = 1;
            } else {
                for (int64_t p = 0; p < P; ++p) { b_l[p] = T; d_l[p] = -256; b_r[p] = INT32_MAX; d_r[p] = 0; }
                for (int d = d0; d < d1; ++d) {
                    box_plane(L, R, W, H, radius, d, colsum, plane);
                    for (int y = 0; y < H; ++y) {
                        const int64_t row = (int64_t)y * W;
                        for (int x = 0; x < W; ++x) {
                            int32_t c = plane[row + x];
                            if (x + d <= W && c < b_l[row + x]) { b_l[row + x] = c; d_l[row + x] = d; }
                            int u = x - d;                  /* C_R(y, u, d) = C_L(y, x, d), u + d < W */
                            if (u >= 0 && c < b_r[row + u]) { b_r[row + u] = c; d_r[row + u] = d; }
                        }
                    }
                }
            }
            free(colsum); free(plane);
        }
    }
    if (!fail) {
        for (int64_t p = 0; p < P; ++p) {
            int32_t bestl = bl[p], bdl = dl[p], bestr = br[p], bdr = dr[p];
            for (int t = 1; t < nt; ++t) {
                if (bl[P * t + p] < bestl) { bestl = bl[P * t + p]; bdl = dl[P * t + p]; }
                if (br[P * t + p] < bestr) { bestr = br[P * t + p]; bdr = dr[P * t + p]; }
            }
            left_out[p] = (uint8_t)bdl;
            right_out[p] = (uint8_t)bdr;
        }
    }
    free(bl); free(dl); free(br); free(dr);
    return fail ? -1 : 0;
}

ORA_API void ora_lr_check(const uint8_t *left_disp, const uint8_t *right_disp, int W, int H,
                          uint8_t *checked, uint8_t *valid_mask)
{
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            int64_t p = (int64_t)y * W + x;
            int d = left_disp[p];
            int occ;
            if (x - d >= 0) {
                int dr = right_disp[p - d];
                int diff = d - dr;
                occ = (d == 0) || (diff > 1 || diff < -1);
            } else {
                occ = 1;
            }
            if (checked) checked[p] = occ ? 0 : (uint8_t)d;
            if (valid_mask) valid_mask[p] = (uint8_t)!occ;
        }
    }
}

/* ------------------------------------------------------------------------- */
/* a8: guided-filter cost aggregation (absent from the reference; this       */
/* build's definition, see DESIGN.md §Guided.  PARITY UNPINNED vs the        */
/* reference, pinned only against this fp64 restatement.)                    */
/*   guide I = L (0..255), cost p_d = AD_d (0..255, AD_d = 0 for x < d as a1),*/
/*   f(.) = mean over the clipped (2r+1)^2 window (divide by in-image count), */
/*   a = (f(I p) - f(I) f(p)) / (f(I I) - f(I)^2 + eps), b = f(p) - a f(I),   */
/*   q = f(a) I + f(b);  WTA: seed 50.0 (= 50*win^2 / win^2), strict <,       */
/*   validity d <= W - x, no match -> 0 (same rules as a2).                   */
/* q_out (optional): [D][H][W] doubles.                                       */
/* ------------------------------------------------------------------------- */
static void box_mean_d(const double *src, int W, int H, int r, double *tmp, double *dst)
{
    /* vertical sums (OpenMP over columns / rows: same per-pixel order of operations) */
#pragma omp parallel for schedule(static)
    for (int x = 0; x < W; ++x) {
        double run = 0.0;
        for (int y = 0; y < r && y < H; ++y) run += src[(int64_t)y * W + x];
        for (int y = 0; y < H; ++y) {
            if (y + r < H) run += src[(int64_t)(y + r) * W + x];
            if (y - r - 1 >= 0) run -= src[(int64_t)(y - r - 1) * W + x];
            tmp[(int64_t)y * W + x] = run;
        }
    }
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y) {
        int ny = (y + r < H ? y + r : H - 1) - (y - r > 0 ? y - r : 0) + 1;
        double run = 0.0;
        const double *t = tmp + (int64_t)y * W;
        for (int x = 0; x < r && x < W; ++x) run += t[x];
        for (int x = 0; x < W; ++x) {
            if (x + r < W) run += t[x + r];
            if (x - r - 1 >= 0) run -= t[x - r - 1];
            int nx = (x + r < W ? x + r : W - 1) - (x - r > 0 ? x - r : 0) + 1;
            dst[(int64_t)y * W + x] = run / (double)(nx * ny);
        }
    }
}

/* Exact box sum of an integer plane, then divided by count: avoids running-sum
   drift so the restatement is exact up to the final division. */
static void box_mean_i(const int64_t *src, int W, int H, int r, int64_t *tmp, double *dst)
{
#pragma omp parallel for schedule(static)
    for (int x = 0; x < W; ++x) {
        int64_t run = 0;
        for (int y = 0; y < r && y < H; ++y) run += src[(int64_t)y * W + x];
        for (int y = 0; y < H; ++y) {
            if (y + r < H) run += src[(int64_t)(y + r) * W + x];
            if (y - r - 1 >= 0) run -= src[(int64_t)(y - r - 1) * W + x];
            tmp[(int64_t)y * W + x] = run;
        }
    }
#pragma omp parallel for schedule(static)
    for (int y = 0; y < H; ++y) {
        int ny = (y + r < H ? y + r : H - 1) - (y - r > 0 ? y - r : 0) + 1;
        int64_t run = 0;
        const int64_t *t = tmp + (int64_t)y * W;
        for (int x = 0; x < r && x < W; ++x) run += t[x];
        for (int x = 0; x < W; ++x) {
            if (x + r < W) run += t[x + r];
            if (x - r - 1 >= 0) run -= t[x - r - 1];
            int nx = (x + r < W ? x + r : W - 1) - (x - r > 0 ? x - r : 0) + 1;
            dst[(int64_t)y * W + x] = (double)run / (double)(nx * ny);
        }
    }
}

/* Box-mean helper shared with the tests: exact mean over the clipped window.
   Double version of the f(.) above (vertical-then-horizontal order). */
ORA_API void ora_box_mean_f64(const double *src, int W, int H, int r, double *dst)
{
    double *tmp = (double *)malloc(sizeof(double) * (size_t)W * H);
    box_mean_d(src, W, H, r, tmp, dst);
    free(tmp);
}

ORA_API int ora_guided_disp(const uint8_t *L, const uint8_t *R, int W, int H, int radius, int D,
                            double eps, uint8_t *out, double *q_out, double *best_out)
{
    const int64_t P = (int64_t)W * H;
    int64_t *isrc = (int64_t *)malloc(sizeof(int64_t) * P);
    int64_t *itmp = (int64_t *)malloc(sizeof(int64_t) * P);
    double *mI = (double *)malloc(sizeof(double) * P);
    double *mII = (double *)malloc(sizeof(double) * P);
    double *mp = (double *)malloc(sizeof(double) * P);
    double *mIp = (double *)malloc(sizeof(double) * P);
    double *a = (double *)malloc(sizeof(double) * P);
    double *b = (double *)malloc(sizeof(double) * P);
    double *ma = (double *)malloc(sizeof(double) * P);
    double *mb = (double *)malloc(sizeof(double) * P);
    double *dtmp = (double *)malloc(sizeof(double) * P);
    double *best = (double *)malloc(sizeof(double) * P);
    int *bd = (int *)malloc(sizeof(int) * P);
    int rc = 0;
    if (!isrc || !itmp || !mI || !mII || !mp || !mIp || !a || !b || !ma || !mb || !dtmp || !best || !bd) {
        rc = -1;
        goto done;
    }

    for (int64_t p = 0; p < P; ++p) isrc[p] = L[p];
    box_mean_i(isrc, W, H, radius, itmp, mI);
    for (int64_t p = 0; p < P; ++p) isrc[p] = (int64_t)L[p] * L[p];
    box_mean_i(isrc, W, H, radius, itmp, mII);
    for (int64_t p = 0; p < P; ++p) { best[p] = 50.0; bd[p] = -256; }

    for (int d = 0; d < D; ++d) {
        /* p_d = AD_d, with the a1 zero for x < d */
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                int64_t p = (int64_t)y * W + x;
                int v = 0;
                if (x >= d) { v = (int)L[p] - (int)R[p - d]; if (v < 0) v = -v; }
                isrc[p] = v;
            }
        box_mean_i(isrc, W, H, radius, itmp, mp);
        for (int64_t p = 0; p < P; ++p) isrc[p] *= L[p];
        box_mean_i(isrc, W, H, radius, itmp, mIp);
        for (int64_t p = 0; p < P; ++p) {
            double var = mII[p] - mI[p] * mI[p];
            double cov = mIp[p] - mI[p] * mp[p];
            a[p] = cov / (var + eps);
            b[p] = mp[p] - a[p] * mI[p];
        }
        box_mean_d(a, W, H, radius, dtmp, ma);
        box_mean_d(b, W, H, radius, dtmp, mb);
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                int64_t p = (int64_t)y * W + x;
                double q = ma[p] * (double)L[p] + mb[p];
                if (q_out) q_out[(int64_t)d * P + p] = q;
                if (x + d > W) continue;
                if (q < best[p]) { best[p] = q; bd[p] = d; }
            }
    }
    for (int64_t p = 0; p < P; ++p) {
        out[p] = (uint8_t)bd[p];
        if (best_out) best_out[p] = best[p];
    }
done:
    free(isrc); free(itmp); free(mI); free(mII); free(mp); free(mIp); free(a); free(b);
    free(ma); free(mb); free(dtmp); free(best); free(bd);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* The same fp64 guided filter, probed at given disparities in O(P) memory    */
/* (full-size checks, cfg3 at 1920x1080 D=128, without the D x P volume):     */
/*   left : best[p] / bd[p] as ora_guided_disp; qL[p] = q(p, dL[p]) (x+d<=W   */
/*          or not: the raw cost);                                           */
/*   right: STMatching's C_R(y,u,d) = q(y,u+d,d) if u+d < W, else C_R(u,d-1) */
/*          (StereoHelper.cpp:156-180); bestR[u] = min_d C_R, qR[u] =        */
/*          C_R(u, dR[u]).  dR / the right outputs may be NULL.              */
/* ------------------------------------------------------------------------- */
ORA_API int ora_guided_probe(const uint8_t *L, const uint8_t *R, int W, int H, int radius, int D, double eps,
                             const uint8_t *dL, const uint8_t *dR, uint8_t *out, double *best_out, double *qL,
                             double *bestR, double *qR)
{
    const int64_t P = (int64_t)W * H;
    int64_t *isrc = (int64_t *)malloc(sizeof(int64_t) * P);
    int64_t *itmp = (int64_t *)malloc(sizeof(int64_t) * P);
    double *mI = (double *)malloc(sizeof(double) * P);
    double *mII = (double *)malloc(sizeof(double) * P);
    double *mp = (double *)malloc(sizeof(double) * P);
    double *mIp = (double *)malloc(sizeof(double) * P);
    double *a = (double *)malloc(sizeof(double) * P);
    double *b = (double *)malloc(sizeof(double) * P);
    double *ma = (double *)malloc(sizeof(double) * P);
    double *mb = (double *)malloc(sizeof(double) * P);
    double *dtmp = (double *)malloc(sizeof(double) * P);
    double *best = (double *)malloc(sizeof(double) * P);
    int *bd = (int *)malloc(sizeof(int) * P);
    int rc = 0;
    if (!isrc || !itmp || !mI || !mII || !mp || !mIp || !a || !b || !ma || !mb || !dtmp || !best || !bd) {
        rc = -1;
        goto done;
    }
    for (int64_t p = 0; p < P; ++p) isrc[p] = L[p];
    box_mean_i(isrc, W, H, radius, itmp, mI);
    for (int64_t p = 0; p < P; ++p) isrc[p] = (int64_t)L[p] * L[p];
    box_mean_i(isrc, W, H, radius, itmp, mII);
    for (int64_t p = 0; p < P; ++p) {
        best[p] = 50.0;
        bd[p] = -256;
        if (bestR) bestR[p] = 1e300;
    }
    for (int d = 0; d < D; ++d) {
#pragma omp parallel for schedule(static)
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                int64_t p = (int64_t)y * W + x;
                int v = 0;
                if (x >= d) { v = (int)L[p] - (int)R[p - d]; if (v < 0) v = -v; }
                isrc[p] = v;
            }
        box_mean_i(isrc, W, H, radius, itmp, mp);
#pragma omp parallel for schedule(static)
        for (int64_t p = 0; p < P; ++p) isrc[p] *= L[p];
        box_mean_i(isrc, W, H, radius, itmp, mIp);
#pragma omp parallel for schedule(static)
        for (int64_t p = 0; p < P; ++p) {
            double var = mII[p] - mI[p] * mI[p];
            double cov = mIp[p] - mI[p] * mp[p];
            a[p] = cov / (var + eps);
            b[p] = mp[p] - a[p] * mI[p];
        }
        box_mean_d(a, W, H, radius, dtmp, ma);
        box_mean_d(b, W, H, radius, dtmp, mb);
        /* rows are independent: the right pixel u = x - d stays in row y */
#pragma omp parallel for schedule(static)
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                int64_t p = (int64_t)y * W + x;
                double q = ma[p] * (double)L[p] + mb[p];
                if (qL && dL && dL[p] == d) qL[p] = q;
                /* right pixel u = x - d sees q as C_R(u, d); u + d < W holds (x < W) */
                int u = x - d;
                if (u >= 0 && bestR) {
                    int64_t pu = (int64_t)y * W + u;
                    if (q < bestR[pu]) bestR[pu] = q;
                    if (qR && dR) {
                        int dr = dR[pu], lim = W - 1 - u;   /* C_R(u, dr) = C_R(u, min(dr, lim)) */
                        if ((dr <= lim ? dr : lim) == d) qR[pu] = q;
                    }
                }
                if (x + d > W) continue;
                if (q < best[p]) { best[p] = q; bd[p] = d; }
            }
    }
    for (int64_t p = 0; p < P; ++p) {
        if (out) out[p] = (uint8_t)bd[p];
        if (best_out) best_out[p] = best[p];
    }
done:
    free(isrc); free(itmp); free(mI); free(mII); free(mp); free(mIp); free(a); free(b);
    free(ma); free(mb); free(dtmp); free(best); free(bd);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* Synthetic rectified pair: SplitMix64(seed) texture T of      */
/* H x (W + 2D); L[y][x] = T[y][x + D], R[y][x] = T[y][x + D + gt(y)],       */
/* gt(y) = 8 + floor(8y/H) * floor((D-16)/7) (clamped at >= 0 bands).         */
/* Byte-for-byte the same as gpu_stereo_matching_amd.synth (numpy), which     */
/* the tests check; kept here so the CPU baseline needs no numpy.             */
/* ------------------------------------------------------------------------- */
static uint64_t splitmix64_at(uint64_t seed, uint64_t i)
{
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

ORA_API void ora_synth_pair(uint64_t seed, int W, int H, int D, uint8_t *L, uint8_t *R)
{
    const int TW = W + 2 * D;
    int step = (D - 16) / 7;
    if (step < 0) step = 0;
    for (int y = 0; y < H; ++y) {
        int gt = 8 + (8 * y / H) * step;
        if (gt > D - 1) gt = D - 1;
        if (gt < 0) gt = 0;
        for (int x = 0; x < W; ++x) {
            uint64_t iL = (uint64_t)y * TW + (uint64_t)(x + D);
            uint64_t iR = (uint64_t)y * TW + (uint64_t)(x + D + gt);
            L[(int64_t)y * W + x] = (uint8_t)(splitmix64_at(seed, iL) >> 56);
            R[(int64_t)y * W + x] = (uint8_t)(splitmix64_at(seed, iR) >> 56);
        }
    }
}

/* ------------------------------------------------------------------------- */
/* §8f rank 4: the disparity median post-filter of the reference's STMatching */
/* pipeline, MeanFilter(disp, disp, 3) (Toolkit.cpp:33-48, used at            */
/* StereoDisparity.cpp:85,119,126,156) = ctmf() (STMatching/ctmf.c:378-433,    */
/* Perreault & Hebert's constant-time median).  Restated from its source:      */
/* the column histograms are seeded with row 0 r+1 times and re-read row      */
/* MIN(m-1, i+r) (ctmf.c:230-257), the row histograms do the same with columns */
/* (:263-315), so the window is replicate-padded; the output is the first      */
/* value whose cumulative count exceeds t = 2r^2 + 2r (:284, :322-329), i.e.   */
/* the (t+1)-th smallest of the (2r+1)^2 values.  The stripe split (:421-431)  */
/* overlaps stripes by 2r and does not change the result.  Parity unpinned:    */
/* the reference ships no median vectors and building ctmf.c here was refused. */
/* ------------------------------------------------------------------------- */
ORA_API void ora_median_u8(const uint8_t *src, int W, int H, int r, uint8_t *dst)
{
    const int t = 2 * r * r + 2 * r;
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) {
            int hist[256];
            memset(hist, 0, sizeof(hist));
            for (int i = -r; i <= r; ++i) {
                int yy = y + i;
                yy = yy < 0 ? 0 : (yy > H - 1 ? H - 1 : yy);
                for (int j = -r; j <= r; ++j) {
                    int xx = x + j;
                    xx = xx < 0 ? 0 : (xx > W - 1 ? W - 1 : xx);
                    hist[src[(int64_t)yy * W + xx]]++;
                }
            }
            int sum = 0, v = 0;
            for (; v < 256; ++v) {
                sum += hist[v];
                if (sum > t) break;
            }
            dst[(int64_t)y * W + x] = (uint8_t)v;
        }
    }
}
