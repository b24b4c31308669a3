// bm_common.h — shared definitions for the gfx950 block-matching kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sm {

// Launch parameters of one block-matching pass over a batch of frames.
struct MatchArgs {
    const uint8_t* left;    // [batch][H][pitch]
    const uint8_t* right;
    int W, H, pitch;
    int64_t frame_stride;   // bytes between frames (inputs)
    int radius;             // window = (2r+1)^2 (SADWindowSize, Device.cu:181)
    int d_lo, d_hi;         // disparities handled by this launch: [d_lo, d_hi)
    int valid_mode;         // 0: d <= W - x (Device.cu:44);  1: d <= x (right view, mirrored)
    uint32_t seed_key;      // starting best key: (50*win^2) << 8 (Device.cu:37) or ~0u (no threshold)
    uint32_t thresh_key;    // disparity = key < thresh_key ? key & 0xFF : 0   (Device.cu:38,63)
    uint8_t* disp;          // optional: uint8 disparity [batch][H][out_pitch]
    int out_pitch;
    int64_t out_frame_stride;
    uint32_t* keys;         // optional: packed keys [batch][H][W] (multi-GPU slice reduction)
    uint32_t* rpart;        // fused right view: per-tile right-key partials (box_right_partial_bytes)
};

constexpr int kMaxDisp = 256;      // uint8 output / 8-bit d field of the packed key
constexpr int kNumXcd = 8;         // MI355X: 8 XCDs, each with its own L2

// Workgroups are dispatched round-robin over the XCDs (blockIdx % 8).  Remapping so that XCD k
// works through a contiguous run of tile indices keeps neighbouring tiles, whose right bands
// overlap by (D + 64 - TW) / (D + 64), in one L2.
__device__ __forceinline__ int xcd_tile(int b, int nb) {
    const int per = nb / kNumXcd, rem = nb - per * kNumXcd;
    const int x = b % kNumXcd, i = b / kNumXcd;
    return x < rem ? x * (per + 1) + i : rem * (per + 1) + (x - rem) * per + i;
}
constexpr int kMaxFastRadius = 7;  // u16 packed sums stay < 2^16 up to r = 7 (15*15*255 = 57375)
// fused box matcher (bm_box.hip): u16 packed column prefixes stay < 2^16 up to r = 15
// ((32 + 30) * 255 = 15810); r 8..15 sum the window's two halves in u32
constexpr int kMaxBoxRadius = 15;

// Host-side launchers (bm_box.hip, bm_aux.hip).
hipError_t launch_box_match(const MatchArgs& a, int batch, hipStream_t s);
hipError_t launch_box_match_generic(const MatchArgs& a, int batch, hipStream_t s);
// Box matching + right view (+ LR check) in two launches (radius <= kMaxBoxRadius, d_lo == 0).
// check = 1: a.disp receives the checked left disparity, right_out/mask_out (optional) dR and the
// valid mask.  check = 0: a.disp the unchecked left map and right_out (required) dR.
hipError_t launch_box_match_lr(const MatchArgs& a, int batch, int check, uint8_t* right_out, uint8_t* mask_out,
                               int aux_pitch, int64_t aux_stride, hipStream_t s);
size_t box_right_partial_bytes(int W, int H, int radius, int D, int batch);
// d-slice with LR (multi-GPU): one fused pass over d in [a.d_lo, a.d_hi) (radius <= kMaxBoxRadius)
// writing the left slice keys to a.keys (as launch_box_match) and the right view's slice keys
// min over d in the slice with u + d < W of (C_L(u + d, d) << 8 | d) to right_keys [batch][H][W]
// (0x7FFFFFFF where none; every key < 2^31 at these radii): keys of disjoint slices combine with a MIN.  a.rpart:
// box_right_partial_bytes(W, H, radius, d_hi - d_lo, batch) bytes.
hipError_t launch_box_slice_lr_keys(const MatchArgs& a, int batch, uint32_t* right_keys, hipStream_t s);
// acc = min(acc, src) elementwise over n unsigned keys
hipError_t launch_min_keys_u32(uint32_t* acc, const uint32_t* src, int64_t n, hipStream_t s);
// right-view key map -> dR: the d field (low byte) of each key, no threshold (StereoHelper.cpp:131-154)
hipError_t launch_keys_low_byte(const uint32_t* keys, int64_t n, uint8_t* out, hipStream_t s);
hipError_t launch_keys_to_disp(const uint32_t* keys, int W, int H, uint32_t thresh_key,
                               uint8_t* disp, int out_pitch, hipStream_t s);
// acc = min(acc, src) elementwise over n signed keys (the d-slice MIN, rehearsed on one device)
hipError_t launch_min_keys(int* acc, const int* src, int64_t n, hipStream_t s);
hipError_t launch_mirror(const uint8_t* src, int W, int H, int pitch, int64_t stride, int batch,
                         uint8_t* dst, int dst_pitch, int64_t dst_stride, hipStream_t s);
// right_mirrored: 1 if the right map is stored mirrored (index W-1-u holds dR(u)), 0 if plain
hipError_t launch_lr_check(const uint8_t* left_disp, int lpitch, int64_t lstride,
                           const uint8_t* right_disp, int rpitch, int64_t rstride, int right_mirrored,
                           int W, int H, int batch, uint8_t* out, int opitch, int64_t ostride,
                           uint8_t* right_out, uint8_t* mask_out, int aux_pitch, int64_t aux_stride,
                           hipStream_t s);
// AD volume dif[d][y][x] (PreCal / kernalPreCal_V2), d-major planes per frame (bm_volume.hip)
hipError_t launch_ad_volume(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int64_t fstride, int batch,
                            int D, uint8_t* dif, int64_t dstride, hipStream_t s);
// staged box path (bm_staged.hip): u16 SAD volume from the AD volume, and WTA over the SAD volume
// `ad` must have 8 readable bytes past its last plane (ensure_vol pads the handle's volume)
hipError_t launch_box_sad_volume(const uint8_t* ad, int W, int H, int radius, int D, uint16_t* sad, hipStream_t s);
// getAllSAD's pixel-major uchar volume out[p * D + d] (255 where x + d > W): from the u16 SAD volume
// (radius <= 7), or computed directly at any radius
hipError_t launch_all_sad_transpose(const uint16_t* sad, int W, int H, int D, uint8_t* out, hipStream_t s);
hipError_t launch_all_sad_generic(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int radius, int D,
                                  uint8_t* out, hipStream_t s);
// (`frames` consecutive frames of D planes each; frame f's map at disp + f * out_stride)
hipError_t launch_volume_wta(const uint16_t* sad, int W, int H, int D, int frames, uint32_t seed_key, uint8_t* disp,
                             int out_pitch, int64_t out_stride, hipStream_t s);
// radius 16..127 (bm_wide.hip): V planes (u16, (d_hi - d_lo) * W * H per frame of a launch group, in `ws`,
// wide_workspace_bytes) then one block per image row; a.valid_mode 0, 4 <= W <= 4096.  right (optional): the right view's dR [batch][H][rpitch]
size_t wide_workspace_bytes(int W, int H, int D, int batch);
// rkeys (d-slices with LR): the right view's raw keys [batch][H][W] of the slice [a.d_lo, a.d_hi), sign bit flipped
// (kRightKeyFlip), instead of / beside `right`
hipError_t launch_box_match_wide(const MatchArgs& a, int batch, uint16_t* ws, uint8_t* right, int rpitch,
                                 int64_t rstride, hipStream_t s, uint32_t* rkeys = nullptr);
// Box right-view slice keys carry the sign bit flipped: (cost << 8 | d) ^ 2^31, so that a signed MIN orders them
// like the unsigned keys at every radius (a wide window's key reaches 255 * 255^2 << 8 > 2^31 from r = 91), and
// "no d of the slice reaches u" (0xFFFFFFFF before the flip) is INT32_MAX, as for the guided keys.
constexpr uint32_t kRightKeyFlip = 0x80000000u;
// radius 16..37 without the right view (bm_strip.hip; valid_mode 0 or 1, the mirrored right-view pass of frames
// wider than the separable path takes): disparities across the lanes, vertical sums in registers,
// no workspace; strip_path says whether a pass takes it (SM_WIDE_STRIP=0, read once, turns it off for A/B).  Past
// r = 37 the strip's 128 - 2r outputs per 128 summed columns make it slower than the separable path (1080p D=128,
// us per frame: r = 37 223.4 vs 236.3, r = 40 256.6 vs 236.6)
constexpr int kStripMinRadius = 16;
#ifndef SM_STRIP_MAX_R
#define SM_STRIP_MAX_R 37
#endif
constexpr int kStripMaxRadius = SM_STRIP_MAX_R;
bool strip_path(const MatchArgs& a);
hipError_t launch_box_match_strip(const MatchArgs& a, int batch, hipStream_t s);
// the same with the right view (a.valid_mode 0, a.d_lo 0; bm_strip_lr.hip): right_keys [batch][H][W], filled with
// ~0 by the caller, receives the MIN over d of (C_L(u + d, d) << 8 | d) over d <= u + d < W: the separable path's
// right-view keys, whose low byte is dR
hipError_t launch_box_match_strip_lr(const MatchArgs& a, int batch, uint32_t* right_keys, hipStream_t s);
constexpr int kMaxWideWidth = 4096;
// radius 16..127, 4 <= W <= 4096 and frames below 2^31 bytes (its buffer loads address a frame with 32-bit
// offsets) take the separable wide-window path (bm_wide.hip); the rest the generic kernel
inline bool wide_path(int radius, int W, int H, int pitch) {
    return radius > kMaxBoxRadius && W >= 4 && W <= kMaxWideWidth && (int64_t)pitch * H < ((int64_t)1 << 31);
}
// SM_DEVICE_CU_GRID (bm_literal.hip): Device.cu's literal map, AD only for rows < 256 and cols < 320, all zero
// for W > 1024; needs W >= 320, H >= 256 and literal_workspace_bytes(D) of device scratch in `ws`
size_t literal_workspace_bytes(int D);
hipError_t launch_device_cu_literal(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int radius, int D,
                                    uint32_t* ws, uint8_t* out, int opitch, hipStream_t s);
// (2r+1)^2 median with replicate borders, radius 1..3 (bm_post.hip)
hipError_t launch_median(const uint8_t* src, int W, int H, int pitch, int64_t stride, int batch, int radius,
                         uint8_t* dst, int dpitch, int64_t dstride, hipStream_t s);

hipError_t launch_bgr_to_gray(const uint8_t* src, int W, int H, int pitch, int channels, uint8_t* dst, int dpitch,
                              hipStream_t s);
hipError_t launch_remap(const uint8_t* src, int W, int H, int pitch, const float* mapx, const float* mapy, int mpitch,
                        uint8_t* dst, int dpitch, hipStream_t s);

// rectification (bm_rectify.hip): OpenCV 2.4 stereoRectify (CV_CALIB_ZERO_DISPARITY, alpha = -1) on the
// host, and initUndistortRectifyMap (CV_32FC1) on the GPU.  r_len: 9 (3x3 matrix) or 3 (rotation vector).
bool stereo_rectify(const double* K1, const double* dist1, int ndist1, const double* K2, const double* dist2,
                    int ndist2, int width, int height, const double* R, int r_len, const double* T, double* R1,
                    double* R2, double* P1, double* P2, double* Q);
hipError_t launch_rectify_map(const double* K, const double* dist, int ndist, const double* R, const double* P,
                              int W, int H, float* mapx, float* mapy, int map_pitch, hipStream_t s);

}  // namespace sm
