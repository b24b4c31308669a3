/*
 * sm_hip.h — C ABI of the MI355X stereo block-matching engine (libsm_hip.so).
 *
 * Drop-in boundary for the reference's GPU proxy
 *     void blockMatching_gpu(cv::Mat &h_left, cv::Mat &h_right, cv::Mat &h_disparity,
 *                            int SADWindowSize, int searchRange);
 * declared at BlockMatching/Device.cuh:50 and defined at BlockMatching/Device.cu:173-301.
 * The reference's argument meaning is kept exactly:
 *   SADWindowSize  -> `radius`    (window is (2*radius+1)^2; Device.cu:181, BlockMatching.cpp:119)
 *   searchRange    -> `num_disp`  (disparities d = 0 .. num_disp-1; Device.cu:43)
 * and so is the output convention: uint8 disparity, 0 where no window SAD falls
 * below 50*win^2 (Device.cu:37-38,63).
 *
 * Everything is plain C: pointers, sizes, int status codes.  No OpenCV or torch
 * types cross this boundary.  include/stereo_bm.hpp maps the reference's Mat API
 * onto it; gpu_stereo_matching_amd/_capi.py binds it with ctypes.
 *
 * Threading: one handle per host thread.  A handle owns its device buffers and a
 * HIP stream; calls on one handle are serialised.
 */
#ifndef SM_HIP_H
#define SM_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SM_API __attribute__((visibility("default")))

/* ---- status codes (the reference has none: Device.cu never checks errors) ---- */
enum {
    SM_OK = 0,
    SM_ERR_INVALID_ARG = 1,   /* bad size / pointer / radius / num_disp */
    SM_ERR_OUT_OF_MEMORY = 2, /* hipMalloc / hipHostMalloc failed */
    SM_ERR_DEVICE = 3,        /* no usable gfx950 device */
    SM_ERR_LAUNCH = 4,        /* kernel launch or runtime error */
    SM_ERR_CAPACITY = 5       /* frame larger than the handle was created for */
};

/* ---- aggregation / post-processing flags ---- */
enum {
    SM_AGG_BOX = 0u,        /* (2r+1)^2 zero-padded SAD window: the reference's kernalFindCorr */
    SM_AGG_GUIDED = 1u,     /* guided-filter aggregation of the AD volume (this build's extension) */
    SM_LR_CHECK = 2u,       /* left-right consistency (STMatching/StereoDisparity.cpp:136-147):
                               occluded pixels are written as 0 */
    SM_MEDIAN = 4u,         /* 7x7 median post-filter of the WTA map(s), STMatching's
                               MeanFilter(disp, disp, 3) = ctmf (Toolkit.cpp:33-48); with
                               SM_LR_CHECK both maps are filtered before the check, in the
                               order of StereoDisparity.cpp:119-126 */
    SM_STAGED = 8u,         /* box path through explicit HBM volumes (AD u8 -> SAD u16 -> WTA),
                               the reference's two-kernel data flow (Device.cu:19-64); same
                               output as the fused kernel, bandwidth-bound; not with
                               SM_AGG_GUIDED or SM_LR_CHECK, radius <= 7.  Frames run in launch
                               groups of up to 8 (SM_PARAM_STAGED_GROUP), and the handle keeps the
                               volumes' workspace, 3*P*D (+ P with SM_MEDIAN) bytes per frame of a
                               group: ~6.4 GB at 1080p D=128 with 8-frame groups (capped at 8 GiB),
                               ~0.8 GB with groups of 1.  Lowering SM_PARAM_STAGED_GROUP frees the
                               workspace (after the handle's pending work), so the next staged call
                               allocates the smaller size */
    SM_DEVICE_CU_GRID = 16u /* opt-in emulation of Device.cu's fixed launch geometry (Device.cu:231-233,
                               253): the AD cost only for rows < 256 and cols < 320, 0 elsewhere (the
                               memset, :193-194), and the all-zero map for width > 1024 (the failed
                               <<<rows, cols>>> launch, :191-192).  Equals the default map at exactly
                               320x256; width < 320 or height < 256 (where the reference reads and writes
                               out of bounds) is SM_ERR_INVALID_ARG.  Box aggregation only (no other flag);
                               whole frames only (not the row-band or d-slice group calls).  Uses
                               ~330 KB * num_disp of the handle's volume workspace */
};

/* ---- scalar parameters (sm_set_param_f) ---- */
enum {
    SM_PARAM_GUIDED_EPS = 1,  /* guided-filter epsilon in AD^2 units (default 6.5025 = 1e-4 * 255^2) */
    SM_PARAM_STAGED_GROUP = 2, /* SM_STAGED frames per launch group, 1..8 (default 8): bounds the
                                  handle's staged workspace (see SM_STAGED) */
    SM_PARAM_STAGE_TIMING = 3  /* whether host calls record the upload / match / download split read by
                                  sm_last_stage_ms with two hipEvents (each a marker between the copy and
                                  compute queues, ~10 us per 1080p call together).  2 (default, auto):
                                  recorded once sm_last_stage_ms has been called on the handle (the calls
                                  after that first read), or in every call when the environment sets
                                  SM_VERBOSE; 1: always; 0: never, and sm_last_stage_ms reports 0.
                                  Setting 2 again returns to the unarmed default */
};

typedef struct sm_handle sm_handle;

/* Library / device information. */
SM_API const char *sm_version(void);
SM_API const char *sm_last_error_string(void);      /* thread-local message of the last failure */
SM_API int sm_device_count(int *count);

/* Create a handle on HIP device `device`, sized for frames up to max_width x max_height and
 * up to max_disp disparities (1..256).  Device frame buffers are allocated once here (the
 * reference re-allocates and leaks ~2*P*D bytes per call: Device.cu:185-194). */
SM_API int sm_create(int device, int max_width, int max_height, int max_disp, sm_handle **out);
SM_API int sm_destroy(sm_handle *h);
SM_API int sm_set_param_f(sm_handle *h, int param, float value);

/* Page-locked host memory for frames and maps (hipHostMalloc, portable).  The host entry points
 * take any host pointer; with buffers from here their copies run as DMA straight from / into the
 * caller's memory instead of through the runtime's pageable bounce buffers (the reference's
 * Mat data is pageable: Device.cu:212-216, 287-291).  sm_host_free(NULL) is a no-op. */
SM_API int sm_host_alloc(size_t bytes, void **out);
SM_API int sm_host_free(void *p);

/* Host-pointer entry point — the blockMatching_gpu replacement.
 * left/right: uint8 gray, `height` rows of `width` bytes at row stride `pitch` (>= width).
 * disp_out: uint8, `height` rows at stride `out_pitch`.  Synchronous, like the reference.
 * flags: SM_AGG_BOX | SM_AGG_GUIDED, optionally | SM_LR_CHECK | SM_MEDIAN. */
SM_API int sm_block_match_u8(sm_handle *h, const uint8_t *left, const uint8_t *right,
                             int width, int height, int pitch, int radius, int num_disp,
                             unsigned flags, uint8_t *disp_out, int out_pitch);

/* Same, also returning the right-view disparity (may be NULL) and the LR valid mask
 * (1 = consistent, may be NULL).  Implies SM_LR_CHECK. */
SM_API int sm_block_match_lr_u8(sm_handle *h, const uint8_t *left, const uint8_t *right,
                                int width, int height, int pitch, int radius, int num_disp,
                                unsigned flags, uint8_t *disp_out, uint8_t *right_disp_out,
                                uint8_t *valid_mask_out, int out_pitch);

/* Per-stage timings of the last sm_block_match_* call in ms (hipEvents), mirroring the
 * reference's "upload data / pre calculation / find corr / download data" printouts
 * (Device.cu:218,238,257,292; "pre calculation" is fused into the match stage here).  With the
 * default SM_PARAM_STAGE_TIMING (auto) the first call of this function turns the recording on for
 * the handle's later calls; a call made while recording was off reads 0.  Any pointer may be NULL. */
SM_API int sm_last_stage_ms(sm_handle *h, float *upload_ms, float *match_ms, float *download_ms);

/* Kernel times (ms, hipEvents on the launch stream) of the last SM_STAGED pass, per frame: the
 * pass runs its frames in launch groups of up to 8 (one AD, one SAD and one WTA launch per group),
 * and each figure is the last group's launch time divided by its frame count.  AD volume
 * (kernalPreCal_V2, Device.cu:19-32), SAD volume and WTA (kernalFindCorr's two halves,
 * Device.cu:34-64).  Waits for that pass to finish.  Any pointer may be NULL. */
SM_API int sm_last_staged_kernel_ms(sm_handle *h, float *ad_ms, float *sad_ms, float *wta_ms);

/* ---- device-pointer entry points (inputs already resident in HBM) ----
 * All pointers are device pointers on the handle's device; `stream` is a hipStream_t used as
 * given (NULL = the device's default stream, as in the HIP runtime API).  Asynchronous: nothing
 * waits for completion.  Calls on one handle may use different streams: a pass that uses the
 * handle's workspace (LR, median, staged, guided LR) first waits for the handle's previous pass
 * when that ran on another stream.
 * `batch` frames are stored back to back: frame i starts at ptr + i*frame_stride. */
SM_API int sm_match_device(sm_handle *h, const uint8_t *d_left, const uint8_t *d_right,
                           int width, int height, int pitch, int batch, int64_t frame_stride,
                           int radius, int num_disp, unsigned flags,
                           uint8_t *d_disp, int out_pitch, int64_t out_frame_stride, void *stream);

/* Disparity-slice keys for multi-GPU sharding over d: for every pixel the
 * minimum over valid d in [d_lo, d_hi) of ((SAD << 8) | d), seeded with (50*win^2) << 8.
 * Keys of disjoint slices combine with an elementwise unsigned min (an all-reduce MIN). */
SM_API int sm_slice_keys_device(sm_handle *h, const uint8_t *d_left, const uint8_t *d_right,
                                int width, int height, int pitch, int radius, int d_lo, int d_hi,
                                uint32_t *d_keys, void *stream);

/* Key map -> disparity: d where (key >> 8) < 50*win^2, else 0 (Device.cu:37,57,63). */
SM_API int sm_keys_to_disp_device(sm_handle *h, const uint32_t *d_keys, int width, int height,
                                  int radius, uint8_t *d_disp, int out_pitch, void *stream);

/* Guided-aggregation d-slice keys (the same sharding over d for SM_AGG_GUIDED): per pixel the
 * best d in [d_lo, d_hi) (valid d <= W - x, no threshold) of the guided-filtered cost q, as
 * ((int32)(q * 2^14) << 8) | d; INT32_MAX where no d of the slice is valid.  Keys of disjoint
 * slices combine with an elementwise SIGNED min (q may be negative).  The handle's guided eps
 * applies.  The combined map equals the single-device guided map up to the 2^-14 quantisation of q
 * (near-ties of the fp32 costs may resolve to the other d). */
SM_API int sm_guided_slice_keys_device(sm_handle *h, const uint8_t *d_left, const uint8_t *d_right,
                                       int width, int height, int pitch, int radius, int d_lo, int d_hi,
                                       int32_t *d_keys, void *stream);

/* Guided key map -> disparity: d where q < 50 (the Device.cu:37 seed, strict), else 0. */
SM_API int sm_guided_keys_to_disp_device(sm_handle *h, const int32_t *d_keys, int width, int height,
                                         uint8_t *d_disp, int out_pitch, void *stream);

/* d-slice keys of BOTH views from one fused pass (multi-GPU d-slices with the LR check, SURVEY §8e "LR adds
 * a second packed reduction for the right view"): d_left_keys as sm_slice_keys_device (flags SM_AGG_BOX,
 * uint32) or sm_guided_slice_keys_device (SM_AGG_GUIDED, int32), and d_right_keys the right view's keys,
 * C_R(y, u, d) = C_L(y, u + d, d) (StereoHelper.cpp:156-180): per right pixel the minimum over d in
 * [d_lo, d_hi) with u + d < W of (cost << 8) | d, no threshold (:131-154); box: (SAD << 8 | d), guided:
 * (floor(q * 2^14) << 8 | d); INT32_MAX where no d of the slice reaches u.  Box right keys carry the sign bit
 * flipped, (SAD << 8 | d) ^ 0x80000000, because a wide window's key passes 2^31 from r = 91: right keys of
 * disjoint slices combine with a SIGNED elementwise MIN for both aggregations (box left keys: unsigned, as
 * sm_slice_keys_device's; guided left keys: signed).  Box radius <= 15 (fused right view) or 16..127 through
 * the wide path (width 4..4096); guided radius <= 7.  Uses the handle's right-view / volume workspace. */
SM_API int sm_slice_keys_lr_device(sm_handle *h, const uint8_t *d_left, const uint8_t *d_right, int width, int height,
                                   int pitch, int radius, int d_lo, int d_hi, unsigned flags, void *d_left_keys,
                                   void *d_right_keys, void *stream);

/* Combined right-view keys -> dR: the d field (low byte) of each of n keys (box or guided). */
SM_API int sm_right_keys_to_disp_device(sm_handle *h, const void *d_keys, int64_t n, uint8_t *d_disp, void *stream);

/* The left-right check of StereoDisparity.cpp:136-147 on device maps: d = dL(x); occluded when x - d < 0, d == 0
 * or |d - dR(x - d)| > 1; d_out = occluded ? 0 : d (may alias d_left_disp), d_mask (may be NULL) = !occluded. */
SM_API int sm_lr_check_device(sm_handle *h, const uint8_t *d_left_disp, const uint8_t *d_right_disp, int width,
                              int height, int pitch, uint8_t *d_out, uint8_t *d_mask, int out_pitch, void *stream);

/* Wait for all work queued on `stream`.  NULL means the default stream, as it does for every
 * device entry point, and also waits for the handle's own stream. */
SM_API int sm_stream_sync(sm_handle *h, void *stream);

/* ---- caller-side steps in front of the path (SURVEY §8f "next") ----
 * BGR(A) -> gray exactly as the reference's caller does it (Caller.cpp:15-16, OpenCV 2.4
 * cvtColor CV_BGR2GRAY, 8-bit fixed point): Y = (1868 B + 9617 G + 4899 R + 8192) >> 14.
 * `channels` is 3 (BGR) or 4 (BGRA; alpha ignored). */
SM_API int sm_bgr_to_gray_device(sm_handle *h, const uint8_t *d_bgr, int width, int height, int pitch,
                                 int channels, uint8_t *d_gray, int gray_pitch, void *stream);

/* Rectification remap with CV_32FC1 maps, the reference's kernalRemap (Device.cu:127-167):
 * bilinear, out-of-range taps -> 0, round half to even + saturate.  map_pitch in floats. */
SM_API int sm_remap_u8_device(sm_handle *h, const uint8_t *d_src, int width, int height, int pitch,
                              const float *d_mapx, const float *d_mapy, int map_pitch,
                              uint8_t *d_dst, int dst_pitch, void *stream);

/* ---- the AD cost volume itself ----
 * dif[d][y][x] = |L(y,x) - R(y,x-d)| for x >= d, else 0, as d-major planes [num_disp][height][width]
 * (PreCal, BlockMatching.cpp:89-109; kernalPreCal_V2 + memset, Device.cu:19-32,193-194).  The
 * matching entry points never build it; this is for callers of the reference's PreCal.
 * Device form: d_dif holds num_disp*width*height bytes.  Host form: synchronous, dif_out likewise.
 * width <= 4096. */
SM_API int sm_ad_volume_device(sm_handle *h, const uint8_t *d_left, const uint8_t *d_right, int width, int height,
                               int pitch, int num_disp, uint8_t *d_dif, void *stream);
SM_API int sm_ad_volume_u8(sm_handle *h, const uint8_t *left, const uint8_t *right, int width, int height,
                           int pitch, int num_disp, uint8_t *dif_out);

/* u16 SAD volume sad[d][y][x] = zero-padded (2r+1)^2 window sum of the AD plane d, radius <= 7
 * (the volume kernalFindAllSAD / getAllSAD build, Device.cu:67-103 / BlockMatching.cpp:191-261,
 * without their uint8 truncation).  d_sad holds num_disp*width*height uint16. */
SM_API int sm_sad_volume_device(sm_handle *h, const uint8_t *d_left, const uint8_t *d_right, int width, int height,
                                int pitch, int radius, int num_disp, uint16_t *d_sad, void *stream);

/* getAllSAD (BlockMatching.cpp:191-261; BlockMatching.h:11): every window SAD, PIXEL-major
 * sad[(y*width + x)*num_disp + d], stored as uint8 (the reference's uchar store truncates mod 256,
 * :258), and 255 where x + d > width (:245-249).  Any radius (r <= 7 and width <= 4096 go through the
 * AD and u16 SAD volumes of SM_STAGED plus a transpose; other sizes through a direct kernel).
 * Device form: d_sad holds width*height*num_disp bytes, asynchronous on `stream`, uses the handle's
 * volume workspace (~4*P*num_disp bytes).  Host form: synchronous, sad_out likewise sized. */
SM_API int sm_all_sad_device(sm_handle *h, const uint8_t *d_left, const uint8_t *d_right, int width, int height,
                             int pitch, int radius, int num_disp, uint8_t *d_sad, void *stream);
SM_API int sm_all_sad_u8(sm_handle *h, const uint8_t *left, const uint8_t *right, int width, int height,
                         int pitch, int radius, int num_disp, uint8_t *sad_out);

/* ---- post-filter ----
 * (2r+1)^2 median with replicate borders, r in 1..3: ctmf (STMatching/ctmf.c:378-433) as called
 * by MeanFilter (Toolkit.cpp:33-48).  Not in place: d_src and d_dst must not overlap. */
SM_API int sm_median_u8_device(sm_handle *h, const uint8_t *d_src, int width, int height, int pitch,
                               int radius, uint8_t *d_dst, int dst_pitch, void *stream);

/* Host-pointer, synchronous forms of the two steps above (the reference's cvtColor_gpu /
 * remap_gpu, Device.cuh:51-52).  Buffers are staged through the handle. */
SM_API int sm_bgr_to_gray_u8(sm_handle *h, const uint8_t *bgr, int width, int height, int pitch, int channels,
                             uint8_t *gray, int gray_pitch);
SM_API int sm_remap_u8(sm_handle *h, const uint8_t *src, int width, int height, int pitch, const float *mapx,
                       const float *mapy, int map_pitch, uint8_t *dst, int dst_pitch);

/* ---- rectification maps (the step before the remap) ----
 * The reference's remapTest (Caller.cpp:27-74) builds its maps with Rectify (Utility.cpp:228-234):
 * OpenCV 2.4 stereoRectify(K1, D1, K2, D2, size, R, T, R1, R2, P1, P2, Q, CV_CALIB_ZERO_DISPARITY)
 * (alpha = -1, newImageSize = size) and initUndistortRectifyMap(Kk, Dk, Rk, Pk, size, CV_32FC1).
 * Matrices are row-major doubles: K 3x3, R 3x3 (r_len 9) or a rotation vector (r_len 3), T 3,
 * R1/R2 3x3, P1/P2 3x4, Q 4x4.  dist: ndist = 0, 4, 5 or 8 coefficients k1 k2 p1 p2 [k3 [k4 k5 k6]].
 * sm_stereo_rectify is host-only math (no device, no handle). */
SM_API int sm_stereo_rectify(const double *K1, const double *dist1, int ndist1, const double *K2,
                             const double *dist2, int ndist2, int width, int height, const double *R,
                             int r_len, const double *T, double *R1, double *R2, double *P1, double *P2,
                             double *Q);
/* CV_32FC1 maps for one camera on the GPU (map_pitch in floats).  Device form: asynchronous on
 * `stream`; host form: synchronous, maps staged through the handle. */
SM_API int sm_init_rectify_map_device(sm_handle *h, const double *K, const double *dist, int ndist,
                                      const double *R, const double *P, int width, int height,
                                      float *d_mapx, float *d_mapy, int map_pitch, void *stream);
SM_API int sm_init_rectify_map(sm_handle *h, const double *K, const double *dist, int ndist,
                               const double *R, const double *P, int width, int height, float *mapx,
                               float *mapy, int map_pitch);

/* imread -> cvtColor -> blockMatching_gpu in one call (Caller.cpp:12-19): BGR(A) host frames
 * are uploaded, converted to gray on the GPU and matched.  Synchronous. */
SM_API int sm_block_match_bgr_u8(sm_handle *h, const uint8_t *left_bgr, const uint8_t *right_bgr,
                                 int width, int height, int pitch, int channels, int radius,
                                 int num_disp, unsigned flags, uint8_t *disp_out, int out_pitch);

/* STMatching's segment-tree stereo, ST-1 (stereo_disparity_normal, StereoDisparity.cpp:57-89; SURVEY
 * §8f rank 4): BGR host frames (3 bytes per pixel, row pitch `pitch`) -> truncated colour + gradient
 * cost over d in [0, max_level) -> segment-tree aggregation on the left view's colour tree
 * (sigma, TAU = 1200) -> WTA -> 7x7 median -> disparity x scale (saturated), uint8 [height][out_pitch].
 * The cost, the filter, the WTA and the median run on the GPU; the tree (a sequential Kruskal / BFS,
 * as in the reference) is built on the host from the GPU's edge weights.  Synchronous.
 * Reference defaults (STMatching/main.cpp:49-51): max_level 60, scale 4, sigma 0.1. */
SM_API int sm_segment_tree_match_bgr_u8(sm_handle *h, const uint8_t *left_bgr, const uint8_t *right_bgr,
                                        int width, int height, int pitch, int max_level, int scale, float sigma,
                                        uint8_t *disp_out, int out_pitch);
/* STMatching's ST-2 (stereo_disparity_iteration, StereoDisparity.cpp:91-160; main.cpp's method 1), same
 * arguments and output as sm_segment_tree_match_bgr_u8: first-pass left and right maps on colour trees
 * of each view (sigma SIGMA_ONE = 0.08, Toolkit.h:35; the right cost taken from the left's,
 * StereoHelper.cpp:156-180), each WTA + 7x7 median; the left-right check (:129-147); then a colour +
 * depth tree (CColorDepthWeight, SegmentTree.cpp:196-219) on the left view, the first left map and
 * the check's mask, filtered with `sigma`, WTA, 7x7 median, x scale.  The three trees' segment_graph
 * passes run on the host (the first two on two threads), their BFS on the GPU; everything O(P*D) runs
 * on the GPU.  Synchronous. */
SM_API int sm_segment_tree_refined_bgr_u8(sm_handle *h, const uint8_t *left_bgr, const uint8_t *right_bgr,
                                          int width, int height, int pitch, int max_level, int scale, float sigma,
                                          uint8_t *disp_out, int out_pitch);
/* last segment-tree call (either method): tree-build time (the host's segment_graph passes and the BFS,
 * until its level count is known), whole-call time (ms) and the last tree's BFS level count */
SM_API int sm_last_segment_tree_stats(sm_handle *h, float *tree_ms, float *total_ms, int *levels);
/* diagnostics: the last call's last tree (ST-1 its colour tree, ST-2 the colour + depth tree) in BFS
 * order, as SegmentTree.cpp:97-130 lays it out: ints = rank[P] (pixel -> BFS index), parent[P],
 * first[P] (first child), child[P] (count | distance bytes << 8), level offsets[levels + 1]
 * (n_ints >= 4P + levels + 1); pdist[P] = distance byte to the parent, n_bytes == P exactly (the last
 * call's pixel count; another value is SM_ERR_INVALID_ARG, so a stale width x height cannot mis-slice).
 * Synchronous. */
SM_API int sm_last_segment_tree_arrays(sm_handle *h, int *ints, int64_t n_ints, uint8_t *pdist, int64_t n_bytes,
                                       int *levels);

/* ---- several GPUs from one host thread (sm_create_group) ----
 * A group holds one handle and one host worker thread per device (devices == NULL: 0..ngpu-1;
 * a device may repeat).  Calls are synchronous, like sm_block_match_u8.
 *  - sm_group_block_match[_lr]_u8: ONE frame in row bands of whole 32-row tiles, one band per
 *    device, each matched from its rows plus the window halo (r; guided max(2r, 16); +3 with
 *    SM_MEDIAN) and downloaded straight into its rows of disp_out.  Every flag is row-local, so
 *    the result equals sm_block_match[_lr]_u8 bit for bit (the guided bands start on the full
 *    frame's tile grid).  No device-to-device traffic: the host frame is the gather point.
 *  - sm_group_block_match_batch_u8: nframes independent pairs, frame f on member f mod ngpu. */
typedef struct sm_group sm_group;
SM_API int sm_create_group(int ngpu, const int *devices, int max_width, int max_height, int max_disp,
                           sm_group **out);
SM_API int sm_destroy_group(sm_group *g);
SM_API int sm_group_size(const sm_group *g, int *n);
SM_API int sm_group_set_param_f(sm_group *g, int param, float value);
SM_API int sm_group_block_match_u8(sm_group *g, const uint8_t *left, const uint8_t *right, int width,
                                   int height, int pitch, int radius, int num_disp, unsigned flags,
                                   uint8_t *disp_out, int out_pitch);
SM_API int sm_group_block_match_lr_u8(sm_group *g, const uint8_t *left, const uint8_t *right, int width,
                                      int height, int pitch, int radius, int num_disp, unsigned flags,
                                      uint8_t *disp_out, uint8_t *right_disp_out, uint8_t *valid_mask_out,
                                      int out_pitch);
SM_API int sm_group_block_match_batch_u8(sm_group *g, const uint8_t *const *lefts,
                                         const uint8_t *const *rights, int nframes, int width, int height,
                                         int pitch, int radius, int num_disp, unsigned flags,
                                         uint8_t *const *disps, int out_pitch);
/* ONE frame sharded over the disparity range, the north star's split (Device.cu:43-61: every d
 * plane is independent, so no halo): member k computes packed keys (SAD << 8 | d; guided:
 * (int)(q * 2^14) << 8 | d) for d in [k*D/n, (k+1)*D/n) on its own device, one RCCL MIN
 * reduce-scatter over xGMI gives each member the global argmin of 1/n of the pixels (the
 * reference's first-smallest-d tie rule survives the MIN), each member finalises its pixels to
 * uint8 (the Device.cu:37 threshold) and one RCCL all-gather assembles the map on every member;
 * member 0's copy is downloaded into disp_out.  Bit-identical to sm_block_match_u8 for box
 * aggregation; guided keys quantise q to 2^-14, so two fp32 costs closer than that may resolve
 * differently from a single pass.  flags: 0 (box) or SM_AGG_GUIDED, optionally | SM_LR_CHECK: each
 * member also emits the right view's keys for its slice from the same fused pass
 * (sm_slice_keys_lr_device), a second MIN reduce-scatter + all-gather forms dR, and member 0 applies
 * StereoDisparity.cpp:136-147 before the download (box LR: any radius the wide path takes).  Members must be distinct
 * devices; RCCL (librccl.so.1) is loaded on first use and one communicator per member is created
 * with ncclCommInitAll.
 * Failure handling: the call runs in two phases.  Phase 1 (upload, slice keys, stream sync) runs on
 * every member; if any member fails there, the call returns its error before any collective is
 * enqueued.  In phase 2 (the collectives) a member that cannot take part aborts its communicator
 * and the others, which poll their streams instead of blocking, abort theirs; the call returns the
 * error and the next call re-creates the communicators.  Test hook: the environment variable
 * SM_DSLICE_FAULT="<member>:keys" or "<member>:collective" injects a failure of that member in
 * phase 1 or in place of its phase-2 collectives. */
SM_API int sm_group_dslice_block_match_u8(sm_group *g, const uint8_t *left, const uint8_t *right, int width,
                                          int height, int pitch, int radius, int num_disp, unsigned flags,
                                          uint8_t *disp_out, int out_pitch);

/* The d-slice plan shared by sm_group_dslice_block_match_u8 and the torch path (sharding.py): for a
 * frame of `pixels` pixels split over `members`, member `member` scans d in [*d_lo, *d_hi) =
 * [member*num_disp/members, (member+1)*num_disp/members) (empty when members > num_disp), the keys
 * are padded to *padded_pixels = members * *chunk pixels with the "no match" key, and the MIN
 * reduce-scatter hands the member pixels [member * *chunk, (member+1) * *chunk).  Host-only (no
 * device, no handle); any output pointer may be NULL. */
SM_API int sm_dslice_plan(int64_t pixels, int num_disp, int members, int member, int *d_lo, int *d_hi,
                          int64_t *chunk, int64_t *padded_pixels);

/* The d-slice split rehearsed on ONE device: the `members` members of sm_group_dslice_block_match_u8
 * run one after another on this handle through the same per-member key pass, padding and
 * finalisation; the RCCL MIN reduce-scatter is an elementwise MIN of their key maps and the
 * all-gather puts chunk k at offset k*chunk.  The map must equal sm_block_match_u8's (box) for any
 * member count; it lets the plan for n > 1 be checked on a one-GPU machine.  flags: 0 or
 * SM_AGG_GUIDED, optionally | SM_LR_CHECK (the right keys' MIN and the LR check as in the group call);
 * members 1..64.  Synchronous. */
SM_API int sm_dslice_rehearse_u8(sm_handle *h, const uint8_t *left, const uint8_t *right, int width,
                                 int height, int pitch, int radius, int num_disp, unsigned flags,
                                 int members, uint8_t *disp_out, int out_pitch);

#ifdef __cplusplus
}
#endif
#endif /* SM_HIP_H */
