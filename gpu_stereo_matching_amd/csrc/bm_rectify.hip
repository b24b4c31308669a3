// bm_rectify.hip — the rectification maps in front of the remap.
//
// The reference's remapTest (Caller.cpp:27-74) loads the stereo calibration (LoadDataBatch,
// Utility.cpp:25-42), builds the maps with Rectify (Utility.cpp:228-234) and remaps both views
// (remap_gpu, Device.cu:303-342).  Rectify is OpenCV 2.4.12:
//   stereoRectify(K1, D1, K2, D2, size, R, T, R1, R2, P1, P2, Q, CV_CALIB_ZERO_DISPARITY)
//     with the C++ defaults alpha = -1, newImageSize = size;
//   initUndistortRectifyMap(Kk, Dk, Rk, Pk, size, CV_32FC1, mapXk, mapYk) for k = 1, 2.
// OpenCV is a third-party dependency absent from the reference tree and from this image; this
// file restates its published algorithms (calib3d/src/calibration.cpp cvStereoRectify,
// cvRodrigues2, cvUndistortPoints, cvProjectPoints2; imgproc/src/undistort.cpp
// initUndistortRectifyMap):
//   * stereo_rectify: host fp64, 3x3 matrices (microseconds, once per calibration);
//   * rectify_map_kernel: the per-pixel map on the GPU, fp64 in OpenCV's operation order
//     (incremental _x/_y/_w along each row, no FMA contraction), rounded to float once.
// Checked against the oracle's independent numpy / C restatements (tests/test_rectify.py,
// tests/test_gpu_rectify.py); parity with OpenCV itself is unpinned.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>

#include "bm_common.h"

#pragma clang fp contract(off)

namespace sm {
namespace {

void mul3(const double* a, const double* b, double* c) {   // c = a * b (row-major 3x3)
    double t[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) t[i * 3 + j] = (a[i * 3] * b[j] + a[i * 3 + 1] * b[3 + j]) + a[i * 3 + 2] * b[6 + j];
    for (int i = 0; i < 9; ++i) c[i] = t[i];
}

void mul3t(const double* a, const double* b, double* c) {  // c = a * b^T
    double t[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            t[i * 3 + j] = (a[i * 3] * b[j * 3] + a[i * 3 + 1] * b[j * 3 + 1]) + a[i * 3 + 2] * b[j * 3 + 2];
    for (int i = 0; i < 9; ++i) c[i] = t[i];
}

void mulv3(const double* a, const double* v, double* o) {
    double t[3];
    for (int i = 0; i < 3; ++i) t[i] = (a[i * 3] * v[0] + a[i * 3 + 1] * v[1]) + a[i * 3 + 2] * v[2];
    o[0] = t[0], o[1] = t[1], o[2] = t[2];
}

// cv::invert(DECOMP_LU) for n == 3: the adjugate over det3 (OpenCV lapack.cpp)
bool inv3(const double* m, double* t) {
    double d = (m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6])) +
               m[2] * (m[3] * m[7] - m[4] * m[6]);
    if (d == 0.) return false;
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
    return true;
}

// Rodrigues, vector -> matrix: R = cos I + (1 - cos) n n^T + sin [n]x (cvRodrigues2)
void rodrigues_mat(const double* r, double* R) {
    const double theta = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (theta < 2.220446049250313e-16) {
        for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0) ? 1. : 0.;
        return;
    }
    const double c = std::cos(theta), s = std::sin(theta), c1 = 1. - c, it = 1. / theta;
    const double x = r[0] * it, y = r[1] * it, z = r[2] * it;
    const double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
    const double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
    for (int i = 0; i < 9; ++i) R[i] = ((i % 4 == 0) ? c : 0.) + c1 * rrt[i] + s * rx[i];
}

// Rodrigues, matrix -> vector.  cvRodrigues2 first replaces R by the nearest rotation U V^T (its
// SVD); here the same orthogonal polar factor comes from the Newton iteration
// X <- (X + X^-T) / 2, which converges quadratically to U V^T for a matrix with det > 0.
bool rodrigues_vec(const double* Rin, double* r) {
    double X[9], inv[9];
    for (int i = 0; i < 9; ++i) X[i] = Rin[i];
    for (int it = 0; it < 50; ++it) {
        if (!inv3(X, inv)) return false;
        double delta = 0.;
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                const double nv = 0.5 * (X[i * 3 + j] + inv[j * 3 + i]);
                delta = std::fmax(delta, std::fabs(nv - X[i * 3 + j]));
                X[i * 3 + j] = nv;
            }
        if (delta < 1e-16) break;
    }
    const double* R = X;
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    const double s = std::sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1.) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    const double theta = std::acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            r[0] = r[1] = r[2] = 0.;
            return true;
        }
        // theta ~ pi: axis from the diagonal of (R + I) / 2, signs as cvRodrigues2
        rx = std::sqrt(std::fmax((R[0] + 1.) * 0.5, 0.));
        ry = std::sqrt(std::fmax((R[4] + 1.) * 0.5, 0.)) * (R[1] < 0 ? -1. : 1.);
        rz = std::sqrt(std::fmax((R[8] + 1.) * 0.5, 0.)) * (R[2] < 0 ? -1. : 1.);
        if (std::fabs(rx) < std::fabs(ry) && std::fabs(rx) < std::fabs(rz) && (R[5] > 0) != (ry * rz > 0)) rz = -rz;
        const double th = theta / std::sqrt(rx * rx + ry * ry + rz * rz);
        r[0] = rx * th, r[1] = ry * th, r[2] = rz * th;
        return true;
    }
    double vth = 1. / (2. * s);
    vth *= theta;
    r[0] = rx * vth, r[1] = ry * vth, r[2] = rz * vth;
    return true;
}

// cvUndistortPoints with R = P = none: 5 fixed-point iterations, normalised coordinates
void undistort_point(double u, double v, const double* K, const double* k, bool has_dist, double* x_out,
                     double* y_out) {
    const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
    const double ifx = 1. / fx, ify = 1. / fy;
    double x = (u - cx) * ifx, y = (v - cy) * ify;
    const double x0 = x, y0 = y;
    for (int j = 0; j < (has_dist ? 5 : 0); ++j) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        const double dx = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
        const double dy = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
        x = (x0 - dx) * icdist;
        y = (y0 - dy) * icdist;
    }
    *x_out = x, *y_out = y;
}

// initUndistortRectifyMap, CV_32FC1.  One thread per image row, walking the row in 64-column
// chunks so that _x/_y/_w accumulate exactly as OpenCV's loop does (`_x += ir[0]` per column);
// a chunk goes through LDS so the float stores are coalesced (lane = column).
constexpr int kMapRows = 64;
struct MapParams {
    double ir[9];
    double fx, fy, u0, v0;
    double k[8];
};

__global__ __launch_bounds__(kMapRows) void rectify_map_kernel(MapParams p, int W, int H, float* __restrict__ mapx,
                                                               float* __restrict__ mapy, int map_pitch) {
    __shared__ float tx[kMapRows][kMapRows + 1];
    __shared__ float ty[kMapRows][kMapRows + 1];
    const int t = threadIdx.x;
    const int row0 = blockIdx.x * kMapRows;
    const int i = row0 + t;
    const double* ir = p.ir;
    double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
    const double k1 = p.k[0], k2 = p.k[1], p1 = p.k[2], p2 = p.k[3], k3 = p.k[4], k4 = p.k[5], k5 = p.k[6],
                 k6 = p.k[7];
    const int nrows = min(kMapRows, H - row0);
    for (int c0 = 0; c0 < W; c0 += kMapRows) {
        const int nc = min(kMapRows, W - c0);
        for (int j = 0; j < nc; ++j, _x += ir[0], _y += ir[3], _w += ir[6]) {
            const double w = 1. / _w, x = _x * w, y = _y * w;
            const double x2 = x * x, y2 = y * y;
            const double r2 = x2 + y2, _2xy = 2 * x * y;
            const double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2);
            const double u = p.fx * (x * kr + p1 * _2xy + p2 * (r2 + 2 * x2)) + p.u0;
            const double v = p.fy * (y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy) + p.v0;
            tx[t][j] = (float)u;
            ty[t][j] = (float)v;
        }
        __syncthreads();
        for (int r = 0; r < nrows; ++r) {
            if (t < nc) {
                mapx[(int64_t)(row0 + r) * map_pitch + c0 + t] = tx[r][t];
                mapy[(int64_t)(row0 + r) * map_pitch + c0 + t] = ty[r][t];
            }
        }
        __syncthreads();
    }
}

}  // namespace

bool stereo_rectify(const double* K1, const double* dist1, int ndist1, const double* K2, const double* dist2,
                    int ndist2, int width, int height, const double* R, int r_len, const double* T, double* R1,
                    double* R2, double* P1, double* P2, double* Q) {
    const double nx = width, ny = height;
    double om[3], r_r[9], t[3], uu[3] = {0, 0, 0}, ww[3], wR[9];
    if (r_len == 9) {
        if (!rodrigues_vec(R, om)) return false;
    } else {
        om[0] = R[0], om[1] = R[1], om[2] = R[2];
    }
    for (double& v : om) v *= -0.5;                          // average rotation
    rodrigues_mat(om, r_r);
    mulv3(r_r, T, t);
    const int idx = std::fabs(t[0]) > std::fabs(t[1]) ? 0 : 1;
    const double c = t[idx], nt = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
    uu[idx] = c > 0 ? 1 : -1;
    ww[0] = t[1] * uu[2] - t[2] * uu[1];                     // global Z rotation: t x uu
    ww[1] = t[2] * uu[0] - t[0] * uu[2];
    ww[2] = t[0] * uu[1] - t[1] * uu[0];
    const double nw = std::sqrt(ww[0] * ww[0] + ww[1] * ww[1] + ww[2] * ww[2]);
    if (nw > 0.0)
        for (double& v : ww) v *= std::acos(std::fabs(c) / nt) / nw;
    rodrigues_mat(ww, wR);
    mul3t(wR, r_r, R1);                                      // R1 = wR * r_r^T
    mul3(wR, r_r, R2);                                       // R2 = wR * r_r
    mulv3(R2, T, t);

    double k[2][8] = {{0}, {0}};
    for (int i = 0; i < ndist1 && i < 8; ++i) k[0][i] = dist1[i];
    for (int i = 0; i < ndist2 && i < 8; ++i) k[1][i] = dist2[i];
    const double* Ks[2] = {K1, K2};
    const double* Rs[2] = {R1, R2};
    const bool has[2] = {ndist1 > 0, ndist2 > 0};
    double fc_new = 1.7976931348623157e308;
    for (int kk = 0; kk < 2; ++kk) {
        const double dk1 = k[kk][0];
        double fc = Ks[kk][(idx ^ 1) * 3 + (idx ^ 1)];
        if (dk1 < 0) fc *= 1 + dk1 * (nx * nx + ny * ny) / (4 * fc * fc);
        fc_new = fc < fc_new ? fc : fc_new;
    }
    double cc[2][2];
    for (int kk = 0; kk < 2; ++kk) {
        double sx = 0., sy = 0.;
        for (int i = 0; i < 4; ++i) {
            // image corners as CV_32FC2 points, undistorted into the same float buffer
            const float pu = (float)((i % 2) * (nx - 1)), pv = (float)((i < 2 ? 0 : 1) * (ny - 1));
            double xn, yn;
            undistort_point(pu, pv, Ks[kk], k[kk], has[kk], &xn, &yn);
            const double X = (float)xn, Y = (float)yn, Z = 1.;
            const double* Rk = Rs[kk];
            // cvProjectPoints2 with rotation Rk, t = 0, fx = fy = fc_new, c = 0, no distortion
            const double px = (Rk[0] * X + Rk[1] * Y) + Rk[2] * Z;
            const double py = (Rk[3] * X + Rk[4] * Y) + Rk[5] * Z;
            const double pz = 1. / ((Rk[6] * X + Rk[7] * Y) + Rk[8] * Z);
            sx += (double)(float)(px * pz * fc_new);
            sy += (double)(float)(py * pz * fc_new);
        }
        cc[kk][0] = (nx - 1) / 2 - sx / 4;
        cc[kk][1] = (ny - 1) / 2 - sy / 4;
    }
    double cx = (cc[0][0] + cc[1][0]) * 0.5, cy = (cc[0][1] + cc[1][1]) * 0.5;         // ZERO_DISPARITY
    // newImgSize == imageSize: cx1 = newImgSize.width * cx1_0 / imageSize.width (rounds twice)
    cx = nx * cx / nx;
    cy = ny * cy / ny;
    for (int i = 0; i < 12; ++i) P1[i] = P2[i] = 0.;
    P1[0] = P1[5] = P2[0] = P2[5] = fc_new;
    P1[2] = P2[2] = cx;
    P1[6] = P2[6] = cy;
    P1[10] = P2[10] = 1.;
    P2[idx * 4 + 3] = t[idx] * fc_new;                       // baseline * focal length
    const double q[16] = {1, 0, 0, -cx, 0, 1, 0, -cy, 0, 0, 0, fc_new, 0, 0, -1. / t[idx], (cx - cx) / t[idx]};
    for (int i = 0; i < 16; ++i) Q[i] = q[i];
    return true;
}

hipError_t launch_rectify_map(const double* K, const double* dist, int ndist, const double* R, const double* P,
                              int W, int H, float* mapx, float* mapy, int map_pitch, hipStream_t s) {
    MapParams p{};
    double ar[9];
    for (int i = 0; i < 3; ++i)   // Ar = P(:, 0:3), Ar * R
        for (int j = 0; j < 3; ++j)
            ar[i * 3 + j] = (P[i * 4] * R[j] + P[i * 4 + 1] * R[3 + j]) + P[i * 4 + 2] * R[6 + j];
    if (!inv3(ar, p.ir)) return hipErrorInvalidValue;
    p.fx = K[0], p.fy = K[4], p.u0 = K[2], p.v0 = K[5];
    for (int i = 0; i < 8; ++i) p.k[i] = i < ndist ? dist[i] : 0.;
    hipLaunchKernelGGL(rectify_map_kernel, dim3((unsigned)((H + kMapRows - 1) / kMapRows)), dim3(kMapRows), 0, s, p, W,
                       H, mapx, mapy, map_pitch);
    return hipGetLastError();
}

}  // namespace sm
