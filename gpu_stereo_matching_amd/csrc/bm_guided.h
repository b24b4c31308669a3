// bm_guided.h — guided-filter cost aggregation (absent from the reference).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sm {

// Guided-filter aggregation + WTA over d in [0, D), D <= 256, radius <= 7, `batch` frames in one
// launch.  valid_mode as MatchArgs (0: left view, threshold 50 and d <= W - x;  1: mirrored right
// view, d <= x, no threshold).  No workspace: every intermediate lives in LDS.
hipError_t launch_guided_match(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int batch,
                               int64_t frame_stride, int radius, int D, float eps, int valid_mode, uint8_t* disp,
                               int out_pitch, int64_t out_frame_stride, hipStream_t s);

// Same, with the fused right view (valid_mode 0 only): the right-view disparity of STMatching's rule
// C_R(y, u, d) = C_L(y, u + d, d), strict < from d = 0, no threshold (StereoHelper.cpp:131-180), is
// written to `right` ([batch][H][rpitch], frame stride rstride).  gpart: per-tile right-key
// partials, guided_right_partial_bytes(...) bytes.  gpart == nullptr: left view only.
hipError_t launch_guided_match_lr(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int batch,
                                  int64_t frame_stride, int radius, int D, float eps, int valid_mode, uint8_t* disp,
                                  int out_pitch, int64_t out_frame_stride, int* gpart, uint8_t* right, int rpitch,
                                  int64_t rstride, hipStream_t s);
size_t guided_right_partial_bytes(int W, int H, int radius, int D, int batch);

// d-slice keys of the guided path (multi-GPU sharding over d): per pixel of each frame
// ([batch][H][W] int32), ((int)(q * 2^14) << 8) | d for the best d in [d_lo, d_hi) (valid d <= W - x,
// no threshold), INT_MAX if none is valid.  Keys of disjoint slices combine with a signed min.
hipError_t launch_guided_slice_keys(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int batch,
                                    int64_t frame_stride, int radius, int d_lo, int d_hi, float eps, int* keys,
                                    hipStream_t s);
// The same slice pass with the fused right view (LR over d-slices): also the right view's slice keys
// (cost field of q_R = q_L(u + d, d), 2^-14 fixed point) | d for the best d in the slice with u + d < W
// (StereoHelper.cpp:156-180; INT_MAX where none), [batch][H][W] int32, combined with a signed min.
// gpart: guided_right_partial_bytes(W, H, radius, d_hi - d_lo, batch) bytes.
hipError_t launch_guided_slice_lr_keys(const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int batch,
                                       int64_t frame_stride, int radius, int d_lo, int d_hi, float eps, int* keys,
                                       int* right_keys, int* gpart, hipStream_t s);
// combined keys -> disparity with the Device.cu:37 threshold q < 50
hipError_t launch_guided_keys_to_disp(const int* keys, int W, int H, uint8_t* disp, int out_pitch, hipStream_t s);

}  // namespace sm
