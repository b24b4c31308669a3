// sm_capi.hip — the C ABI (include/sm_hip.h): handles, buffers, streams, entry points.
//
// Replaces blockMatching_gpu (BlockMatching/Device.cu:173-301).  Differences from the
// reference that are deliberate and documented in DESIGN.md:
//   * buffers are allocated once per handle, not per call, and are freed (Device.cu leaks
//     ~2*P*D bytes and the output buffer per call, :185-194, :300);
//   * every HIP call is checked and surfaced as an int status + sm_last_error_string()
//     (the reference never checks, so its W > 1024 launch failure returns all zeros, :253);
//   * any frame size works (the reference's fixed (8,10,D)x(32,32) grid covers 320x256 only, :231-233).
#include <dlfcn.h>
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <cstdio>
#include <cstring>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <functional>
#include <map>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sm_hip.h"
#include "bm_common.h"
#include "bm_guided.h"
#include "bm_segtree.h"

struct sm_handle {
    int device = 0;
    int max_w = 0, max_h = 0, max_d = 0;
    hipStream_t stream = nullptr;
    // frame buffers (one frame; batched device calls use caller memory)
    uint8_t* d_left = nullptr;
    uint8_t* d_right = nullptr;
    uint8_t* d_disp = nullptr;
    // LR workspace (grown on demand): mirrored L, mirrored R, mirrored right disparity
    uint8_t* d_lr = nullptr;
    size_t lr_bytes = 0;
    // AD volume staging of the host PreCal entry point (grown on demand)
    uint8_t* d_vol = nullptr;
    size_t vol_bytes = 0;
    // float maps of the host remap entry point (grown on demand)
    float* d_maps = nullptr;
    size_t maps_bytes = 0;
    // right-map / mask staging of the host LR entry point (grown on demand)
    uint8_t* d_aux = nullptr;
    size_t aux_bytes = 0;
    // fused right view: per-tile right-key partials (grown on demand)
    uint32_t* d_rpart = nullptr;
    size_t rpart_bytes = 0;
    // BGR staging for sm_block_match_bgr_u8 (grown on demand)
    uint8_t* d_bgr = nullptr;
    size_t bgr_bytes = 0;
    float guided_eps = 6.5025f;  // 1e-4 * 255^2 (AD units)
    int staged_group = 8;        // SM_STAGED frames per launch group (SM_PARAM_STAGED_GROUP)
    // host calls record the upload / match / download split (SM_PARAM_STAGE_TIMING): 0 off, 1 on, 2 auto
    // (default: on once sm_last_stage_ms has been called on the handle, or when SM_VERBOSE is set)
    int stage_timing = 2;
    bool stage_requested = false;
    // The workspaces above are shared by every call on the handle while calls run on the stream
    // they are given: the end of each pass is recorded here, and a pass on another stream waits
    // for it first, so two streams never write the same workspace at once.
    hipEvent_t scratch_ev = nullptr;
    hipStream_t scratch_stream = nullptr;
    bool scratch_pending = false;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    float stage_ms[3] = {0.f, 0.f, 0.f};
    // RCCL d-slice group mode (sm_group_dslice_block_match_u8): slice keys, this member's reduced
    // key chunk, its uint8 chunk and the gathered map (grown on demand)
    uint8_t* d_dsl = nullptr;
    size_t dsl_bytes = 0;
    // segment-tree path (sm_segment_tree_match_bgr_u8): device workspace and the last call's stats
    sm::StWorkspace st;
    sm::StStats st_stats;
    float st_total_ms = 0.f;
    bool st_valid = false;
    // staged box path: events around the last launch group's AD / SAD / WTA kernels
    // (sm_last_staged_kernel_ms reports them per frame of that group)
    hipEvent_t kev[4] = {nullptr, nullptr, nullptr, nullptr};
    int kev_frames = 1;
    bool kev_valid = false;
};

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

#define SM_HIP(call)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (call);                                                               \
        if (e_ != hipSuccess)                                                                 \
            return fail(e_ == hipErrorOutOfMemory ? SM_ERR_OUT_OF_MEMORY : SM_ERR_LAUNCH,      \
                        "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, __LINE__); \
    } while (0)

int check_geometry(const sm_handle* h, int width, int height, int pitch, int radius, int num_disp) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (width <= 0 || height <= 0) return fail(SM_ERR_INVALID_ARG, "bad frame size %dx%d", width, height);
    if (pitch < width) return fail(SM_ERR_INVALID_ARG, "pitch %d < width %d", pitch, width);
    if (radius < 0 || radius > 127) return fail(SM_ERR_INVALID_ARG, "radius %d out of [0,127]", radius);
    if (num_disp < 1 || num_disp > sm::kMaxDisp)
        return fail(SM_ERR_INVALID_ARG, "num_disp %d out of [1,%d] (uint8 disparity output)", num_disp, sm::kMaxDisp);
    const int64_t win = 2 * radius + 1;
    if (((int64_t)50 * win * win) >= (int64_t)1 << 23)
        return fail(SM_ERR_INVALID_ARG, "radius %d too large for the 32-bit (SAD<<8|d) key", radius);
    return SM_OK;
}

uint32_t seed_key(int radius) {
    const uint32_t win = 2u * (uint32_t)radius + 1u;
    return (50u * win * win) << 8;  // Device.cu:37 start value, d field 0
}

int ensure_lr(sm_handle* h, size_t bytes) {
    if (h->lr_bytes >= bytes) return SM_OK;
    if (h->d_lr) (void)hipFree(h->d_lr);
    h->d_lr = nullptr;
    h->lr_bytes = 0;
    SM_HIP(hipMalloc(&h->d_lr, bytes));
    h->lr_bytes = bytes;
    return SM_OK;
}

int ensure_rpart(sm_handle* h, size_t bytes) {
    if (h->rpart_bytes >= bytes) return SM_OK;
    if (h->d_rpart) (void)hipFree(h->d_rpart);
    h->d_rpart = nullptr;
    h->rpart_bytes = 0;
    SM_HIP(hipMalloc(&h->d_rpart, bytes));
    h->rpart_bytes = bytes;
    return SM_OK;
}

// Host<->device 2-D copy.  Contiguous rows (both pitches == row bytes) go as one 1-D copy: the
// 2-D path takes a slow per-row route for widths that are not a multiple of 4 (measured 5.7 ms
// instead of 0.02 ms to upload a 463x370 pair).
// Pitched host buffers are gathered into / scattered from a contiguous host vector around one
// 1-D copy (the pageable 2-D path is the slow one, pitched or not).
thread_local std::vector<uint8_t> g_host_rows;

hipError_t copy2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t row_bytes, size_t rows,
                  hipMemcpyKind kind, hipStream_t s) {
    if (dpitch == row_bytes && spitch == row_bytes) return hipMemcpyAsync(dst, src, row_bytes * rows, kind, s);
    if (kind == hipMemcpyHostToDevice && dpitch == row_bytes) {
        g_host_rows.resize(row_bytes * rows);
        for (size_t r = 0; r < rows; ++r)
            std::memcpy(g_host_rows.data() + r * row_bytes, static_cast<const uint8_t*>(src) + r * spitch, row_bytes);
        // a pageable source is staged before the call returns, so the vector may be reused
        return hipMemcpyAsync(dst, g_host_rows.data(), row_bytes * rows, kind, s);
    }
    if (kind == hipMemcpyDeviceToHost && spitch == row_bytes) {
        g_host_rows.resize(row_bytes * rows);
        hipError_t e = hipMemcpyAsync(g_host_rows.data(), src, row_bytes * rows, kind, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return e;
        for (size_t r = 0; r < rows; ++r)
            std::memcpy(static_cast<uint8_t*>(dst) + r * dpitch, g_host_rows.data() + r * row_bytes, row_bytes);
        return hipSuccess;
    }
    return hipMemcpy2DAsync(dst, dpitch, src, spitch, row_bytes, rows, kind, s);
}

int ensure_vol(sm_handle* h, size_t bytes) {
    if (h->vol_bytes >= bytes) return SM_OK;
    if (h->d_vol) (void)hipFree(h->d_vol);
    h->d_vol = nullptr;
    h->vol_bytes = 0;
    // 64 readable bytes past the end: box_sad_kernel reads whole 8-byte words at the planes' last bytes
    SM_HIP(hipMalloc(&h->d_vol, bytes + 64));
    h->vol_bytes = bytes;
    return SM_OK;
}

// Staged box path through AD (u8) + SAD (u16) volume workspaces, in launch groups of up to
// kStagedGroup frames (workspace <= kStagedBytes): one AD, one SAD and one WTA launch per group, as
// the fused path batches frames per launch.  The SAD launch sees the group's g*D planes as one
// volume; the WTA launch takes the frame from blockIdx.y.
constexpr int kStagedGroup = 8;
constexpr int64_t kStagedBytes = (int64_t)8 << 30;
int run_staged(sm_handle* h, const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int batch, int64_t fstride,
               int radius, int D, bool med, uint8_t* disp, int opitch, int64_t ostride, hipStream_t s) {
    const int64_t P = (int64_t)W * H;
    if (W > 4096) return fail(SM_ERR_INVALID_ARG, "SM_STAGED: width %d exceeds 4096", W);
    const int64_t per_frame = 3 * P * D + (med ? P : 0);
    int group = (int)std::min<int64_t>(h->staged_group, std::max<int64_t>(1, kStagedBytes / per_frame));
    group = std::min(group, std::max(batch, 1));
    int rc = ensure_vol(h, (size_t)(per_frame * group));
    if (rc) return rc;
    uint8_t* ad = h->d_vol;
    uint16_t* sad = reinterpret_cast<uint16_t*>(h->d_vol + group * P * D);
    uint8_t* raw = h->d_vol + 3 * group * P * D;
    if (!h->kev[0])
        for (auto& e : h->kev) SM_HIP(hipEventCreate(&e));
    h->kev_valid = false;
    for (int f0 = 0; f0 < batch; f0 += group) {
        const int g = std::min(group, batch - f0);
        const bool last = f0 + g >= batch;   // the last group's kernels are bracketed by events
        if (last) SM_HIP(hipEventRecord(h->kev[0], s));
        SM_HIP(sm::launch_ad_volume(L + f0 * fstride, R + f0 * fstride, W, H, pitch, fstride, g, D, ad, P * D, s));
        if (last) SM_HIP(hipEventRecord(h->kev[1], s));
        SM_HIP(sm::launch_box_sad_volume(ad, W, H, radius, g * D, sad, s));
        if (last) SM_HIP(hipEventRecord(h->kev[2], s));
        uint8_t* out = disp + f0 * ostride;
        SM_HIP(sm::launch_volume_wta(sad, W, H, D, g, seed_key(radius), med ? raw : out, med ? W : opitch,
                                     med ? P : ostride, s));
        if (last) SM_HIP(hipEventRecord(h->kev[3], s));
        if (med) SM_HIP(sm::launch_median(raw, W, H, W, P, g, 3, out, opitch, ostride, s));
        if (last) h->kev_frames = g;
    }
    h->kev_valid = batch > 0;
    return SM_OK;
}

// Core device-side pass over `batch` frames.  Workspace planes (d_lr) are dense W x H frames.
//   left map  : matched straight into `disp`, or into a workspace plane when SM_MEDIAN filters it
//               into `disp` afterwards (StereoDisparity.cpp:85/119);
//   right map : fused with the left pass for box r <= 15 and for guided (right keys from
//               the left costs, bm_guided.hip); box r = 16..127 takes it from the wide kernel's LDS
//               atomic-min row (bm_wide.hip); only frames the wide path rejects (W > 4096, or planes of
//               2^31 bytes and up) match the mirrored pair (valid d <= x, no threshold), kept mirrored;
//   LR check  : StereoDisparity.cpp:136-147 on the (median-filtered, :119-126) maps.
// SM_STRIP_LR=0 (read once) keeps box + LR at r 16..37 on the separable path (A/B)
bool strip_lr_enabled() {
    static const bool on = [] {
#ifdef SM_STRIP_LR_OFF
        return false;   // A/B builds
#endif
        const char* e = std::getenv("SM_STRIP_LR");
        return !(e && e[0] == '0');
    }();
    return on;
}

int run_device_body(sm_handle* h, const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int batch,
                    int64_t fstride, int radius, int D, unsigned flags, uint8_t* disp, int opitch, int64_t ostride,
                    uint8_t* right_out, uint8_t* mask_out, int apitch, int64_t astride, hipStream_t s) {
    const bool guided = (flags & SM_AGG_GUIDED) != 0;
    const bool lr = (flags & SM_LR_CHECK) != 0 || right_out || mask_out;
    const bool med = (flags & SM_MEDIAN) != 0;
    constexpr int kMedianRadius = 3;   // MeanFilter(disp, disp, 3)
    const int64_t P = (int64_t)W * H;
    const int64_t PB = P * batch;
    const bool fused_right = lr && !guided && radius <= sm::kMaxBoxRadius;
    const bool guided_right = lr && guided;   // right view fused into the guided pass (bm_guided.hip)
    // box r > 15: the separable wide-window path (bm_wide.hip), right view included; wider frames keep the
    // direct generic kernel and the mirrored LR pass
    const bool wide = !guided && sm::wide_path(radius, W, H, pitch);
    if ((flags & SM_DEVICE_CU_GRID) != 0) {   // Device.cu's launch geometry, frame by frame (bm_literal.hip)
        if (flags != SM_DEVICE_CU_GRID || lr)
            return fail(SM_ERR_INVALID_ARG, "SM_DEVICE_CU_GRID is box aggregation only (flags 0x%x)", flags);
        if (W < 320 || H < 256)
            return fail(SM_ERR_INVALID_ARG,
                        "SM_DEVICE_CU_GRID: %dx%d is below the 320x256 the reference's fixed grid assumes "
                        "(Device.cu:231-233 reads and writes outside the frame)", W, H);
        int rc = ensure_vol(h, sm::literal_workspace_bytes(D));
        if (rc) return rc;
        for (int f = 0; f < batch; ++f)
            SM_HIP(sm::launch_device_cu_literal(L + f * fstride, R + f * fstride, W, H, pitch, radius, D,
                                                reinterpret_cast<uint32_t*>(h->d_vol), disp + f * ostride, opitch,
                                                s));
        return SM_OK;
    }
    if ((flags & SM_STAGED) != 0) {
        if (guided || lr || radius > sm::kMaxFastRadius)
            return fail(SM_ERR_INVALID_ARG, "SM_STAGED supports box aggregation without LR, radius <= %d",
                        sm::kMaxFastRadius);
        return run_staged(h, L, R, W, H, pitch, batch, fstride, radius, D, med, disp, opitch, ostride, s);
    }

    // workspace: [left raw (med)] [right (lr)] [right filtered (lr && med)] [mirrored L, R (lr, not fused)]
    const bool mirrored = lr && !fused_right && !guided_right && !wide;
    const int64_t n_planes = (med ? 1 : 0) + (lr ? 1 : 0) + (lr && med ? 1 : 0) + (mirrored ? 2 : 0);
    if (n_planes > 0) {
        int rc = ensure_lr(h, (size_t)(n_planes * PB));
        if (rc) return rc;
    }
    uint8_t* ws = h->d_lr;
    uint8_t* left_raw = med ? ws : nullptr;
    if (med) ws += PB;
    uint8_t* right_map = lr ? ws : nullptr;   // plain (fused) or mirrored
    if (lr) ws += PB;
    uint8_t* right_med = (lr && med) ? ws : nullptr;
    if (lr && med) ws += PB;
    uint8_t* mL = mirrored ? ws : nullptr;
    uint8_t* mR = mL ? mL + PB : nullptr;

    // ---- left map ----
    uint8_t* lmap = med ? left_raw : disp;
    const int lpitch = med ? W : opitch;
    const int64_t lstride = med ? P : ostride;
    sm::MatchArgs a{};
    a.left = L;
    a.right = R;
    a.W = W;
    a.H = H;
    a.pitch = pitch;
    a.frame_stride = fstride;
    a.radius = radius;
    a.d_lo = 0;
    a.d_hi = D;
    a.valid_mode = 0;
    a.seed_key = seed_key(radius);
    a.thresh_key = seed_key(radius);
    a.disp = lmap;
    a.out_pitch = lpitch;
    a.out_frame_stride = lstride;
    a.keys = nullptr;
    a.rpart = nullptr;
    if (fused_right) {
        int rc = ensure_rpart(h, sm::box_right_partial_bytes(W, H, radius, D, batch));
        if (rc) return rc;
        a.rpart = h->d_rpart;
        if (!med) {   // match + right view + check in one pass over the partials
            SM_HIP(sm::launch_box_match_lr(a, batch, 1, right_out, mask_out, apitch, astride, s));
            return SM_OK;
        }
        SM_HIP(sm::launch_box_match_lr(a, batch, 0, right_map, nullptr, W, P, s));
    } else if (guided_right) {
        int rc = ensure_rpart(h, sm::guided_right_partial_bytes(W, H, radius, D, batch));
        if (rc) return rc;
        SM_HIP(sm::launch_guided_match_lr(L, R, W, H, pitch, batch, fstride, radius, D, h->guided_eps, 0, lmap, lpitch,
                                         lstride, reinterpret_cast<int*>(h->d_rpart), right_map, W, P, s));
    } else if (guided) {
        SM_HIP(sm::launch_guided_match(L, R, W, H, pitch, batch, fstride, radius, D, h->guided_eps, 0, lmap, lpitch,
                                      lstride, s));
    } else if (wide) {
        // r 16..37: the strip kernel (bm_strip.hip); without the right view it needs no workspace, with it the
        // right keys go through the volume workspace (4 B per pixel) and their low byte is dR
        if (!lr && sm::strip_path(a)) {
            SM_HIP(sm::launch_box_match_strip(a, batch, s));
        } else if (lr && strip_lr_enabled() && sm::strip_path(a)) {
            int rc = ensure_vol(h, (size_t)PB * 4);
            if (rc) return rc;
            uint32_t* rk = reinterpret_cast<uint32_t*>(h->d_vol);
            SM_HIP(hipMemsetAsync(rk, 0xFF, (size_t)PB * 4, s));
            SM_HIP(sm::launch_box_match_strip_lr(a, batch, rk, s));
            SM_HIP(sm::launch_keys_low_byte(rk, PB, right_map, s));
        } else {
            int rc = ensure_vol(h, sm::wide_workspace_bytes(W, H, D, batch));
            if (rc) return rc;
            SM_HIP(sm::launch_box_match_wide(a, batch, reinterpret_cast<uint16_t*>(h->d_vol), lr ? right_map : nullptr,
                                             W, P, s));
        }
    } else if (radius > sm::kMaxBoxRadius && sm::strip_path(a)) {
        // frames past the separable path's limits (wider than 4096 columns): the strip kernel has none (the
        // mirrored right view below takes it too)
        SM_HIP(sm::launch_box_match_strip(a, batch, s));
    } else {
        SM_HIP(sm::launch_box_match(a, batch, s));
    }
    if (med) SM_HIP(sm::launch_median(left_raw, W, H, W, P, batch, kMedianRadius, disp, opitch, ostride, s));
    if (!lr) return SM_OK;

    // ---- right map on the mirrored pair (StereoHelper.cpp:156-180 + :131-154), box r > 7 ----
    if (mirrored) {
        SM_HIP(sm::launch_mirror(R, W, H, pitch, fstride, batch, mL, W, P, s));
        SM_HIP(sm::launch_mirror(L, W, H, pitch, fstride, batch, mR, W, P, s));
        {
            sm::MatchArgs b = a;
            b.left = mL;
            b.right = mR;
            b.pitch = W;
            b.frame_stride = P;
            b.valid_mode = 1;
            b.seed_key = 0xFFFFFFFFu;
            b.thresh_key = 0xFFFFFFFFu;
            b.disp = right_map;
            b.out_pitch = W;
            b.out_frame_stride = P;
            if (radius > sm::kMaxBoxRadius && sm::strip_path(b))   // frames wider than the separable path takes
                SM_HIP(sm::launch_box_match_strip(b, batch, s));
            else
                SM_HIP(sm::launch_box_match(b, batch, s));
        }
    }
    const uint8_t* rcheck = right_map;
    if (med) {   // the median commutes with the mirror, so a mirrored map is filtered as is
        SM_HIP(sm::launch_median(right_map, W, H, W, P, batch, kMedianRadius, right_med, W, P, s));
        rcheck = right_med;
    }
    SM_HIP(sm::launch_lr_check(disp, opitch, ostride, rcheck, W, P, mirrored ? 1 : 0, W, H, batch, disp, opitch,
                               ostride, right_out, mask_out, apitch, astride, s));
    return SM_OK;
}

// run_device_body on stream s, ordered after the handle's previous pass when that ran on another
// stream (the workspaces d_lr / d_rpart / d_vol are per handle).
// A pass without median, LR, staged volumes or the wide path's V planes touches no workspace: it neither
// waits for nor records the scratch event (round 4: the marker cost the host call ~µs; SM_SCRATCH_EVENT=1,
// read once, keeps both for every pass, for A/B).  A box pass at r 16..127 writes its V planes into d_vol
// (and may grow it), so it is ordered like the others.
bool scratch_event_forced() {
    static const bool on = [] {
        const char* e = getenv("SM_SCRATCH_EVENT");
        return e && e[0] == '1';
    }();
    return on;
}

int run_device(sm_handle* h, const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int batch,
               int64_t fstride, int radius, int D, unsigned flags, uint8_t* disp, int opitch, int64_t ostride,
               uint8_t* right_out, uint8_t* mask_out, int apitch, int64_t astride, hipStream_t s) {
    const bool uses_ws = (flags & (SM_STAGED | SM_MEDIAN | SM_LR_CHECK | SM_DEVICE_CU_GRID)) != 0 || right_out || mask_out ||
                         (!(flags & SM_AGG_GUIDED) && sm::wide_path(radius, W, H, pitch)) || scratch_event_forced();
    if (uses_ws && h->scratch_pending && h->scratch_stream != s) SM_HIP(hipStreamWaitEvent(s, h->scratch_ev, 0));
    const int rc = run_device_body(h, L, R, W, H, pitch, batch, fstride, radius, D, flags, disp, opitch, ostride,
                                   right_out, mask_out, apitch, astride, s);
    if (uses_ws) {
        SM_HIP(hipEventRecord(h->scratch_ev, s));
        h->scratch_stream = s;
        h->scratch_pending = true;
    }
    return rc;
}

// Page-locked blocks from sm_host_alloc: a map the caller receives into one of them is written by the
// kernel straight over PCIe (zero-copy), with no separate device-to-host copy.
std::mutex g_host_mu;
std::map<uintptr_t, size_t> g_host_blocks;

void host_blocks_add(void* p, size_t n) {
    std::lock_guard<std::mutex> lk(g_host_mu);
    g_host_blocks[(uintptr_t)p] = n;
}

void host_blocks_remove(void* p) {
    std::lock_guard<std::mutex> lk(g_host_mu);
    g_host_blocks.erase((uintptr_t)p);
}

// Device address of [p, p + bytes) when that range lies in one sm_host_alloc block, else nullptr.
uint8_t* host_block_device_ptr(void* p, size_t bytes) {
    uintptr_t base = 0;
    {
        std::lock_guard<std::mutex> lk(g_host_mu);
        auto it = g_host_blocks.upper_bound((uintptr_t)p);
        if (it == g_host_blocks.begin()) return nullptr;
        --it;
        if ((uintptr_t)p + bytes > it->first + it->second) return nullptr;
        base = it->first;
    }
    void* dbase = nullptr;
    if (hipHostGetDevicePointer(&dbase, reinterpret_cast<void*>(base), 0) != hipSuccess || !dbase) {
        (void)hipGetLastError();
        return nullptr;
    }
    return static_cast<uint8_t*>(dbase) + ((uintptr_t)p - base);
}

bool verbose_env() {
    static const bool on = getenv("SM_VERBOSE") != nullptr;
    return on;
}

// SM_ZERO_COPY=0 keeps the device buffer + download for every call (A/B timing)
bool zero_copy_enabled() {
    static const bool on = [] {
        const char* e = getenv("SM_ZERO_COPY");
        return !(e && e[0] == '0');
    }();
    return on;
}

bool start_event_forced() {
    static const bool on = [] {
        const char* e = getenv("SM_START_EVENT");
        return e && e[0] == '1';
    }();
    return on;
}

// SM_PAIR_COPY=0 (A/B only): a contiguous host pair still goes up as two copies
bool pair_copy_enabled() {
    static const bool on = [] {
        const char* e = getenv("SM_PAIR_COPY");
        return !(e && e[0] == '0');
    }();
    return on;
}

// Host-pointer pass over one frame (or one row band of a frame: sm_group_*).  Only result rows
// [keep0, keep1) are downloaded, into disp_out / right_out / mask_out pointing at row keep0.
int host_match_rows(sm_handle* h, const uint8_t* left, const uint8_t* right, int width, int height, int pitch,
                    int radius, int num_disp, unsigned flags, int keep0, int keep1, uint8_t* disp_out,
                    uint8_t* right_out, uint8_t* mask_out, int out_pitch);

int host_match(sm_handle* h, const uint8_t* left, const uint8_t* right, int width, int height, int pitch,
               int radius, int num_disp, unsigned flags, uint8_t* disp_out, uint8_t* right_out, uint8_t* mask_out,
               int out_pitch) {
    return host_match_rows(h, left, right, width, height, pitch, radius, num_disp, flags, 0, height, disp_out,
                           right_out, mask_out, out_pitch);
}

int host_match_rows(sm_handle* h, const uint8_t* left, const uint8_t* right, int width, int height, int pitch,
                    int radius, int num_disp, unsigned flags, int keep0, int keep1, uint8_t* disp_out,
                    uint8_t* right_out, uint8_t* mask_out, int out_pitch) {
    int rc = check_geometry(h, width, height, pitch, radius, num_disp);
    if (rc) return rc;
    if (!left || !right || !disp_out) return fail(SM_ERR_INVALID_ARG, "null image pointer");
    if (out_pitch < width) return fail(SM_ERR_INVALID_ARG, "out_pitch %d < width %d", out_pitch, width);
    if (keep0 < 0 || keep1 > height || keep0 >= keep1) return fail(SM_ERR_INVALID_ARG, "bad kept rows");
    if (width > h->max_w || height > h->max_h || num_disp > h->max_d)
        return fail(SM_ERR_CAPACITY, "frame %dx%d/D=%d exceeds handle capacity %dx%d/D=%d", width, height, num_disp,
                    h->max_w, h->max_h, h->max_d);
    SM_HIP(hipSetDevice(h->device));
    hipStream_t s = h->stream;
    const int64_t P = (int64_t)width * height;
    uint8_t* aux = nullptr;
    if (right_out || mask_out) {
        if (h->aux_bytes < (size_t)(2 * P)) {
            if (h->d_aux) (void)hipFree(h->d_aux);
            h->d_aux = nullptr;
            h->aux_bytes = 0;
            SM_HIP(hipMalloc(&h->d_aux, (size_t)(2 * P)));
            h->aux_bytes = (size_t)(2 * P);
        }
        aux = h->d_aux;
    }
    // zero-copy map: a whole-frame call whose map goes to an sm_host_alloc block and is only written by
    // the last kernel (no LR check, which reads the left map back)
    uint8_t* mapped = nullptr;
    if (zero_copy_enabled() && keep0 == 0 && keep1 == height && !right_out && !mask_out && !(flags & SM_LR_CHECK))
        mapped = host_block_device_ptr(disp_out, (size_t)(height - 1) * out_pitch + width);
    // stage split events (SM_PARAM_STAGE_TIMING): each costs a marker between the copy and compute
    // queues, ~10 us per 1080p call for the two (profiles/microbench/r03_roundtrip_pair_block.txt); the
    // start event likewise only when the split is recorded (round 4; SM_START_EVENT=1, read once, records
    // it in every call as before, for A/B)
    const bool ev = h->stage_timing == 1 || (h->stage_timing == 2 && (h->stage_requested || verbose_env()));
    if (ev || start_event_forced()) SM_HIP(hipEventRecord(h->ev[0], s));
    // a pair with the right frame right after the left one (one sm_host_alloc block of 2 frames, or any
    // contiguous (2, H, W) array) goes up as one copy into d_left .. d_left + 2P: one DMA transfer
    // instead of two
    uint8_t* dR = h->d_right;
    if (pitch == width && reinterpret_cast<uintptr_t>(right) == reinterpret_cast<uintptr_t>(left) + (uintptr_t)P &&
        pair_copy_enabled()) {
        dR = h->d_left + P;
        SM_HIP(hipMemcpyAsync(h->d_left, left, (size_t)(2 * P), hipMemcpyHostToDevice, s));
    } else {
        SM_HIP(copy2d(h->d_left, width, left, pitch, width, height, hipMemcpyHostToDevice, s));
        SM_HIP(copy2d(h->d_right, width, right, pitch, width, height, hipMemcpyHostToDevice, s));
    }
    if (ev) SM_HIP(hipEventRecord(h->ev[1], s));
    rc = run_device(h, h->d_left, dR, width, height, width, 1, P, radius, num_disp, flags,
                    mapped ? mapped : h->d_disp, mapped ? out_pitch : width, P, right_out ? aux : nullptr,
                    mask_out ? aux + P : nullptr, width, P, s);
    if (rc) return rc;
    if (ev) SM_HIP(hipEventRecord(h->ev[2], s));
    const int64_t k0 = (int64_t)keep0 * width;
    const int nk = keep1 - keep0;
    if (!mapped) SM_HIP(copy2d(disp_out, out_pitch, h->d_disp + k0, width, width, nk, hipMemcpyDeviceToHost, s));
    if (right_out) SM_HIP(copy2d(right_out, out_pitch, aux + k0, width, width, nk, hipMemcpyDeviceToHost, s));
    if (mask_out) SM_HIP(copy2d(mask_out, out_pitch, aux + P + k0, width, width, nk, hipMemcpyDeviceToHost, s));
    SM_HIP(hipEventRecord(h->ev[3], s));
    SM_HIP(hipEventSynchronize(h->ev[3]));
    if (ev) {
        SM_HIP(hipEventElapsedTime(&h->stage_ms[0], h->ev[0], h->ev[1]));
        SM_HIP(hipEventElapsedTime(&h->stage_ms[1], h->ev[1], h->ev[2]));
        SM_HIP(hipEventElapsedTime(&h->stage_ms[2], h->ev[2], h->ev[3]));
    } else {
        h->stage_ms[0] = h->stage_ms[1] = h->stage_ms[2] = 0.f;
    }
    return SM_OK;
}

// ---- multi-GPU group (sm_create_group): one handle and one persistent host thread per device ----
// Pageable host copies block their calling thread, so each device gets its own worker thread; a
// call hands every worker its job (a row band of one frame, or a share of a frame batch) and
// waits for all of them.
struct GroupWorker {
    sm_handle* h = nullptr;
    std::thread th;
    std::mutex m;
    std::condition_variable cv;
    std::function<int()> job;
    bool has_job = false, done = false, quit = false;
    int rc = SM_OK;
    std::string err;

    void loop() {
        for (;;) {
            std::function<int()> j;
            {
                std::unique_lock<std::mutex> lk(m);
                cv.wait(lk, [&] { return has_job || quit; });
                if (quit) return;
                j = std::move(job);
                has_job = false;
            }
            const int r = j();
            std::lock_guard<std::mutex> lk(m);
            rc = r;
            err = r ? std::string(g_err) : std::string();
            done = true;
            cv.notify_all();
        }
    }
};

}  // namespace

struct sm_group {
    std::vector<GroupWorker*> w;
    // one RCCL communicator per member for the d-slice mode, created on first use (ncclCommInitAll)
    std::vector<ncclComm_t> comms;
};

namespace {

// Runs jobs[k] on worker k (jobs may be shorter than the group: the rest stay idle) and returns the
// first failure, its message re-raised on the calling thread.
int group_run(sm_group* g, std::vector<std::function<int()>>& jobs) {
    const size_t n = jobs.size() < g->w.size() ? jobs.size() : g->w.size();
    for (size_t k = 0; k < n; ++k) {
        GroupWorker* w = g->w[k];
        std::lock_guard<std::mutex> lk(w->m);
        w->job = std::move(jobs[k]);
        w->has_job = true;
        w->done = false;
        w->cv.notify_all();
    }
    int rc = SM_OK;
    std::string err;
    for (size_t k = 0; k < n; ++k) {
        GroupWorker* w = g->w[k];
        std::unique_lock<std::mutex> lk(w->m);
        w->cv.wait(lk, [&] { return w->done; });
        if (w->rc && !rc) {
            rc = w->rc;
            err = "device " + std::to_string(w->h->device) + ": " + w->err;
        }
    }
    if (rc) return fail(rc, "%s", err.c_str());
    return SM_OK;
}

// RCCL is loaded on first use of the d-slice mode, not linked: callers that never shard a frame over
// disparities carry no RCCL dependency.  The soname matches the copy PyTorch-ROCm ships, so inside a
// torch process dlopen returns the already-loaded library (one RCCL per process).
struct RcclApi {
    decltype(&ncclCommInitAll) init_all;
    decltype(&ncclCommDestroy) destroy;
    decltype(&ncclReduceScatter) reduce_scatter;
    decltype(&ncclAllGather) all_gather;
    decltype(&ncclGetErrorString) error_string;
    decltype(&ncclCommAbort) abort;
    decltype(&ncclCommGetAsyncError) async_error;
};

const RcclApi* rccl_api() {
    static std::mutex mu;
    static RcclApi api;
    static int state = 0;   // 0 untried, 1 loaded, -1 unavailable
    std::lock_guard<std::mutex> lk(mu);
    if (state == 0) {
        void* lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!lib) lib = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        state = -1;
        if (lib) {
            api.init_all = reinterpret_cast<decltype(api.init_all)>(dlsym(lib, "ncclCommInitAll"));
            api.destroy = reinterpret_cast<decltype(api.destroy)>(dlsym(lib, "ncclCommDestroy"));
            api.reduce_scatter = reinterpret_cast<decltype(api.reduce_scatter)>(dlsym(lib, "ncclReduceScatter"));
            api.all_gather = reinterpret_cast<decltype(api.all_gather)>(dlsym(lib, "ncclAllGather"));
            api.error_string = reinterpret_cast<decltype(api.error_string)>(dlsym(lib, "ncclGetErrorString"));
            api.abort = reinterpret_cast<decltype(api.abort)>(dlsym(lib, "ncclCommAbort"));
            api.async_error = reinterpret_cast<decltype(api.async_error)>(dlsym(lib, "ncclCommGetAsyncError"));
            if (api.init_all && api.destroy && api.reduce_scatter && api.all_gather && api.error_string && api.abort &&
                api.async_error)
                state = 1;
        }
    }
    return state == 1 ? &api : nullptr;
}

#define SM_RCCL(api, call)                                                                         \
    do {                                                                                           \
        ncclResult_t r_ = (call);                                                                  \
        if (r_ != ncclSuccess)                                                                     \
            return fail(SM_ERR_LAUNCH, "%s failed: %s (%s:%d)", #call, (api)->error_string(r_), __FILE__, \
                        __LINE__);                                                                 \
    } while (0)

int group_comms(sm_group* g) {
    if (!g->comms.empty()) return SM_OK;
    const RcclApi* api = rccl_api();
    if (!api) return fail(SM_ERR_DEVICE, "d-slice mode: librccl.so.1 not loadable (%s)", dlerror());
    const int n = (int)g->w.size();
    std::vector<int> devs(n);
    for (int k = 0; k < n; ++k) {
        devs[k] = g->w[k]->h->device;
        for (int j = 0; j < k; ++j)
            if (devs[j] == devs[k])
                return fail(SM_ERR_INVALID_ARG, "d-slice mode needs distinct devices (device %d twice)", devs[k]);
    }
    std::vector<ncclComm_t> comms(n, nullptr);
    SM_RCCL(api, api->init_all(comms.data(), n, devs.data()));
    g->comms = comms;
    return SM_OK;
}

// ---- the d-slice split (sm_group_dslice_block_match_u8, sm_dslice_rehearse_u8) ----
// One plan for every path that shards a frame over d: the C group call, its one-device rehearsal and
// the torch path (sharding.py calls sm_dslice_plan).  Member k of n scans d in [kD/n, (k+1)D/n)
// (Device.cu:43-61: the d planes are independent); the P keys are padded with the "no match" key to
// Ppad = n * chunk so that the MIN reduce-scatter hands member k the pixels [k*chunk, (k+1)*chunk),
// and the all-gather puts chunk k back at offset k*chunk.
// The pair itself is split by rows (round 4): member k uploads only image rows
// [k*rows_per, (k+1)*rows_per) of each frame over its own PCIe link, into slot k of an n*rows_per-row
// buffer, and an in-place RCCL all-gather over xGMI assembles both frames on every member before the
// key pass.  No halo is needed: the gathered frames are the whole pair.
struct DslicePlan {
    int lo, hi;
    int64_t chunk, padded;
    int rows_per, row_lo, row_hi;   // this member's upload rows [row_lo, row_hi) (empty past the frame)
};

DslicePlan dslice_plan(int64_t P, int D, int n, int k, int H = 1) {
    DslicePlan p;
    p.lo = (int)((int64_t)k * D / n);
    p.hi = (int)((int64_t)(k + 1) * D / n);
    p.chunk = (P + n - 1) / n;
    p.padded = p.chunk * n;
    p.rows_per = (H + n - 1) / n;
    p.row_lo = std::min(H, k * p.rows_per);
    p.row_hi = std::min(H, (k + 1) * p.rows_per);
    return p;
}

// keys no d of the slice improves: the Device.cu:37 seed (box) / INT32_MAX (guided, signed keys)
uint32_t dslice_none_key(int radius, bool guided) { return guided ? 0x7FFFFFFFu : seed_key(radius); }
// right-view keys no d of the slice reaches (no seed: StereoHelper.cpp:131-154 has no threshold): INT32_MAX for
// both aggregations, since box right keys are sign-flipped (kRightKeyFlip) and every right-key MIN is signed
uint32_t dslice_none_rkey(bool) { return 0x7FFFFFFFu; }

// One d-sliced frame: geometry, aggregation and whether the LR check runs (SM_LR_CHECK: a second key map
// for the right view, C_R(u, d) = C_L(u + d, d), reduced with its own MIN; StereoHelper.cpp:156-180)
struct DsliceCfg {
    int W, H, radius, D;
    bool guided, lr;
    int64_t P() const { return (int64_t)W * H; }
};

int ensure_dsl(sm_handle* h, size_t need) {
    if (h->dsl_bytes >= need) return SM_OK;
    if (h->d_dsl) (void)hipFree(h->d_dsl);
    h->d_dsl = nullptr;
    h->dsl_bytes = 0;
    SM_HIP(hipMalloc(&h->d_dsl, need));
    h->dsl_bytes = need;
    return SM_OK;
}

// Test hook (include/sm_hip.h): SM_DSLICE_FAULT="<member>:<phase>" makes that member fail in phase
// "keys" (before any collective) or "collective" (instead of enqueuing its reduce-scatter).
bool dslice_fault(int k, const char* phase) {
    const char* e = getenv("SM_DSLICE_FAULT");
    if (!e) return false;
    const char* colon = strchr(e, ':');
    return colon && atoi(e) == k && strcmp(colon + 1, phase) == 0;
}

// The slice pass over [d_lo, d_hi) of frames already on the device (pitch `pitch`): left keys, and with
// `rkeys` the right view's keys from the same fused pass (its per-tile partials in the handle's rpart
// workspace).  Keys are [H][W]; no padding.
int slice_keys_pass(sm_handle* h, const uint8_t* dL, const uint8_t* dR, int W, int H, int pitch, int radius, int d_lo,
                    int d_hi, bool guided, uint32_t* keys, uint32_t* rkeys, hipStream_t s) {
    const int64_t P = (int64_t)W * H;
    if (guided) {
        if (!rkeys) {
            SM_HIP(sm::launch_guided_slice_keys(dL, dR, W, H, pitch, 1, P, radius, d_lo, d_hi, h->guided_eps,
                                                reinterpret_cast<int*>(keys), s));
            return SM_OK;
        }
        int rc = ensure_rpart(h, sm::guided_right_partial_bytes(W, H, radius, d_hi - d_lo, 1));
        if (rc) return rc;
        SM_HIP(sm::launch_guided_slice_lr_keys(dL, dR, W, H, pitch, 1, P, radius, d_lo, d_hi, h->guided_eps,
                                               reinterpret_cast<int*>(keys), reinterpret_cast<int*>(rkeys),
                                               reinterpret_cast<int*>(h->d_rpart), s));
        return SM_OK;
    }
    sm::MatchArgs a{};
    a.left = dL;
    a.right = dR;
    a.W = W;
    a.H = H;
    a.pitch = pitch;
    a.frame_stride = P;
    a.radius = radius;
    a.d_lo = d_lo;
    a.d_hi = d_hi;
    a.valid_mode = 0;
    a.seed_key = seed_key(radius);
    a.thresh_key = seed_key(radius);
    a.keys = keys;
    if (!rkeys) {
        if (sm::strip_path(a)) {   // r 16..37: the strip kernel (bm_strip.hip), at any width
            SM_HIP(sm::launch_box_match_strip(a, 1, s));
            return SM_OK;
        }
        if (sm::wide_path(radius, W, H, pitch)) {   // the wide-window path (bm_wide.hip)
            int rc = ensure_vol(h, sm::wide_workspace_bytes(W, H, d_hi - d_lo, 1));
            if (rc) return rc;
            SM_HIP(sm::launch_box_match_wide(a, 1, reinterpret_cast<uint16_t*>(h->d_vol), nullptr, 0, 0, s));
            return SM_OK;
        }
        SM_HIP(sm::launch_box_match(a, 1, s));
        return SM_OK;
    }
    if (sm::wide_path(radius, W, H, pitch)) {   // r 16..127: the wide path's right row, keys sign-flipped
        int rc = ensure_vol(h, sm::wide_workspace_bytes(W, H, d_hi - d_lo, 1));
        if (rc) return rc;
        SM_HIP(sm::launch_box_match_wide(a, 1, reinterpret_cast<uint16_t*>(h->d_vol), nullptr, 0, 0, s, rkeys));
        return SM_OK;
    }
    int rc = ensure_rpart(h, sm::box_right_partial_bytes(W, H, radius, d_hi - d_lo, 1));
    if (rc) return rc;
    a.rpart = h->d_rpart;
    SM_HIP(sm::launch_box_slice_lr_keys(a, 1, rkeys, s));
    return SM_OK;
}

// Member-side key pass over its slice: keys[0, padded) (and rkeys with LR) on stream s from the frames
// already on the device (dL / dR, pitch W).
int dslice_keys(sm_handle* h, const DslicePlan& p, const DsliceCfg& c, const uint8_t* dL, const uint8_t* dR,
                uint32_t* keys, uint32_t* rkeys, hipStream_t s) {
    const int64_t P = c.P();
    const uint32_t none = dslice_none_key(c.radius, c.guided), rnone = dslice_none_rkey(c.guided);
    if (p.padded > P) SM_HIP(hipMemsetD32Async(keys + P, (int)none, (size_t)(p.padded - P), s));
    if (rkeys && p.padded > P) SM_HIP(hipMemsetD32Async(rkeys + P, (int)rnone, (size_t)(p.padded - P), s));
    if (p.hi <= p.lo) {   // more members than disparities: an empty slice contributes "no match"
        SM_HIP(hipMemsetD32Async(keys, (int)none, (size_t)P, s));
        if (rkeys) SM_HIP(hipMemsetD32Async(rkeys, (int)rnone, (size_t)P, s));
        return SM_OK;
    }
    return slice_keys_pass(h, dL, dR, c.W, c.H, c.W, c.radius, p.lo, p.hi, c.guided, keys, rkeys, s);
}

// A reduced key chunk -> uint8 (the Device.cu:37 threshold, after the MIN); a right-view chunk -> its d field
int dslice_finalise(const uint32_t* mine, int64_t chunk, int radius, bool guided, uint8_t* mine8, hipStream_t s) {
    if (guided)
        SM_HIP(sm::launch_guided_keys_to_disp(reinterpret_cast<const int*>(mine), (int)chunk, 1, mine8, (int)chunk, s));
    else
        SM_HIP(sm::launch_keys_to_disp(mine, (int)chunk, 1, seed_key(radius), mine8, (int)chunk, s));
    return SM_OK;
}

// Member workspace: keys [padded] | reduced chunk [chunk] | uint8 chunk [chunk] | gathered map [padded] |
// gathered left frame [n * rows_per * W] | gathered right frame [same] | with LR the right view's
// keys [padded] | reduced chunk [chunk] | uint8 chunk [chunk] | gathered right map [padded]
// (each region 256-B aligned)
struct DsliceWs {
    uint32_t* keys;
    uint32_t* mine;
    uint8_t* mine8;
    uint8_t* map;
    uint8_t* gl;
    uint8_t* gr;
    uint32_t* rkeys;
    uint32_t* rmine;
    uint8_t* rmine8;
    uint8_t* rmap;
    int64_t slot;   // bytes of one member's row slot (rows_per * W)
    size_t bytes;
};
inline int64_t a256(int64_t v) { return (v + 255) & ~(int64_t)255; }
DsliceWs dslice_ws(uint8_t* base, const DslicePlan& p, int n, int W, bool lr) {
    DsliceWs w;
    w.slot = (int64_t)p.rows_per * W;
    int64_t o = 0;
    w.keys = reinterpret_cast<uint32_t*>(base + o);
    o += a256(p.padded * 4);
    w.mine = reinterpret_cast<uint32_t*>(base + o);
    o += a256(p.chunk * 4);
    w.mine8 = base + o;
    o += a256(p.chunk);
    w.map = base + o;
    o += a256(p.padded);
    w.gl = base + o;
    o += a256(n * w.slot);
    w.gr = base + o;
    o += a256(n * w.slot);
    w.rkeys = w.rmine = nullptr;
    w.rmine8 = w.rmap = nullptr;
    if (lr) {
        w.rkeys = reinterpret_cast<uint32_t*>(base + o);
        o += a256(p.padded * 4);
        w.rmine = reinterpret_cast<uint32_t*>(base + o);
        o += a256(p.chunk * 4);
        w.rmine8 = base + o;
        o += a256(p.chunk);
        w.rmap = base + o;
        o += a256(p.padded);
    }
    w.bytes = (size_t)o;
    return w;
}

// Member k's rows of the pair into its slot of the gathered frames (host -> device, its own PCIe link).
int dslice_upload_rows(const DslicePlan& p, const DsliceWs& w, int k, const uint8_t* left, const uint8_t* right, int W,
                       int pitch, hipStream_t s) {
    const int nr = p.row_hi - p.row_lo;
    if (nr <= 0) return SM_OK;   // a member past the frame's last row contributes a pad slot only
    const int64_t off = (int64_t)p.row_lo * pitch;
    SM_HIP(copy2d(w.gl + k * w.slot, W, left + off, pitch, W, nr, hipMemcpyHostToDevice, s));
    SM_HIP(copy2d(w.gr + k * w.slot, W, right + off, pitch, W, nr, hipMemcpyHostToDevice, s));
    return SM_OK;
}

// Phase 1 of member k (its worker thread): workspace and the upload of its rows, then a stream sync
// so that every local failure (allocation, copy) is known before any member enqueues a collective.  A
// member that fails here returns before phase 2 starts, so nobody waits on it.
int dslice_member_upload(sm_handle* h, int k, int n, const uint8_t* left, const uint8_t* right, const DsliceCfg& c,
                         int pitch) {
    const DslicePlan p = dslice_plan(c.P(), c.D, n, k, c.H);
    SM_HIP(hipSetDevice(h->device));
    hipStream_t s = h->stream;
    if (dslice_fault(k, "keys")) return fail(SM_ERR_LAUNCH, "d-slice member %d: injected fault (keys)", k);
    int rc = ensure_dsl(h, dslice_ws(nullptr, p, n, c.W, c.lr).bytes);
    if (rc) return rc;
    const bool wide = !c.guided && sm::wide_path(c.radius, c.W, c.H, c.W);
    if (c.lr && p.hi > p.lo && !wide) {   // the right view's per-tile partials, before any collective
        rc = ensure_rpart(h, c.guided ? sm::guided_right_partial_bytes(c.W, c.H, c.radius, p.hi - p.lo, 1)
                                      : sm::box_right_partial_bytes(c.W, c.H, c.radius, p.hi - p.lo, 1));
        if (rc) return rc;
    }
    // a box slice at r 16..127 runs the wide path (right keys included), whose V planes live in d_vol: sized
    // here too, so that its allocation cannot fail after the pair all-gathers are enqueued
    if (wide && p.hi > p.lo) {
        rc = ensure_vol(h, sm::wide_workspace_bytes(c.W, c.H, p.hi - p.lo, 1));
        if (rc) return rc;
    }
    const DsliceWs w = dslice_ws(h->d_dsl, p, n, c.W, c.lr);
    rc = dslice_upload_rows(p, w, k, left, right, c.W, pitch, s);
    if (rc) return rc;
    SM_HIP(hipStreamSynchronize(s));
    return SM_OK;
}

// Shared by the members of one phase-2 call: a member that cannot take part raises `abort`, and
// every member then aborts its communicator instead of waiting for the missing peer.
struct DsliceSync {
    std::atomic<bool> abort{false};
};

// Phase 2 of member k: in-place all-gathers of the pair's row slots, the slice keys, MIN reduce-scatter,
// finalise, all-gather of the map, member 0 downloads.  With LR the right view's keys take the same
// reduce-scatter / finalise (their d field) / all-gather, and member 0 applies StereoDisparity.cpp:136-147
// to the gathered maps before the download.  Waits by polling its stream and the shared abort flag (and
// RCCL's async error), so that no member blocks forever on a collective a failed peer never joined (the
// ncclCommAbort pattern).  On any failure the member's communicator is aborted and its slot set to null
// (the group re-creates them).
int dslice_member_collect(sm_handle* h, const RcclApi* api, ncclComm_t* comm, DsliceSync* sync, int k, int n,
                          const DsliceCfg& c, uint8_t* disp_out, int out_pitch) {
    const DslicePlan p = dslice_plan(c.P(), c.D, n, k, c.H);
    const DsliceWs w = dslice_ws(h->d_dsl, p, n, c.W, c.lr);
    hipStream_t s = h->stream;
    // every failure of phase 2 goes through bail, so the others stop polling for this member
    auto bail = [&](int code, const char* what) {
        sync->abort.store(true);
        if (*comm) (void)api->abort(*comm);
        *comm = nullptr;
        return fail(code, "d-slice member %d: %s", k, what);
    };
    if (hipSetDevice(h->device) != hipSuccess) return bail(SM_ERR_LAUNCH, "hipSetDevice failed");
    if (dslice_fault(k, "collective")) return bail(SM_ERR_LAUNCH, "injected fault (collective)");
    // the pair: every member's row slot to every member (in place: slot k is this member's send buffer)
    if (api->all_gather(w.gl + k * w.slot, w.gl, (size_t)w.slot, ncclUint8, *comm, s) != ncclSuccess ||
        api->all_gather(w.gr + k * w.slot, w.gr, (size_t)w.slot, ncclUint8, *comm, s) != ncclSuccess)
        return bail(SM_ERR_LAUNCH, "ncclAllGather (pair rows) failed");
    if (dslice_keys(h, p, c, w.gl, w.gr, w.keys, w.rkeys, s)) return bail(SM_ERR_LAUNCH, "slice keys launch failed");
    // box keys (SAD << 8 | d) compare as unsigned (the right view's too); guided keys are signed
    const ncclDataType_t kt = c.guided ? ncclInt32 : ncclUint32;
    if (api->reduce_scatter(w.keys, w.mine, (size_t)p.chunk, kt, ncclMin, *comm, s) != ncclSuccess)
        return bail(SM_ERR_LAUNCH, "ncclReduceScatter failed");
    // right keys: signed for both aggregations (box right keys are sign-flipped, kRightKeyFlip)
    if (c.lr && api->reduce_scatter(w.rkeys, w.rmine, (size_t)p.chunk, ncclInt32, ncclMin, *comm, s) != ncclSuccess)
        return bail(SM_ERR_LAUNCH, "ncclReduceScatter (right keys) failed");
    if (dslice_finalise(w.mine, p.chunk, c.radius, c.guided, w.mine8, s) ||
        (c.lr && sm::launch_keys_low_byte(w.rmine, p.chunk, w.rmine8, s) != hipSuccess))
        return bail(SM_ERR_LAUNCH, "finalise launch failed");
    if (api->all_gather(w.mine8, w.map, (size_t)p.chunk, ncclUint8, *comm, s) != ncclSuccess)
        return bail(SM_ERR_LAUNCH, "ncclAllGather failed");
    if (c.lr && api->all_gather(w.rmine8, w.rmap, (size_t)p.chunk, ncclUint8, *comm, s) != ncclSuccess)
        return bail(SM_ERR_LAUNCH, "ncclAllGather (right map) failed");
    if (c.lr && k == 0 &&
        sm::launch_lr_check(w.map, c.W, c.P(), w.rmap, c.W, c.P(), 0, c.W, c.H, 1, w.map, c.W, c.P(), nullptr, nullptr,
                            c.W, c.P(), s) != hipSuccess)
        return bail(SM_ERR_LAUNCH, "LR check launch failed");
    for (;;) {
        const hipError_t q = hipStreamQuery(s);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) return bail(SM_ERR_LAUNCH, hipGetErrorString(q));
        ncclResult_t async = ncclSuccess;
        if (api->async_error(*comm, &async) != ncclSuccess || async != ncclSuccess)
            return bail(SM_ERR_LAUNCH, "RCCL asynchronous error");
        if (sync->abort.load()) return bail(SM_ERR_LAUNCH, "aborted: another member failed");
        std::this_thread::yield();
    }
    if (k == 0) {
        const hipError_t e = copy2d(disp_out, out_pitch, w.map, c.W, c.W, c.H, hipMemcpyDeviceToHost, s);
        if (e != hipSuccess || hipStreamSynchronize(s) != hipSuccess) return bail(SM_ERR_LAUNCH, "map download failed");
    }
    return SM_OK;
}

// Rows a band must see on each side of its output rows: the aggregation window (2r for the
// guided filter's nested windows, at least 16 so that the guided kernel's 8-row float running
// sums of the kept rows start on rows the band holds exactly) plus the median's 3.
int group_halo(int radius, unsigned flags) {
    int h = (flags & SM_AGG_GUIDED) ? (2 * radius > 16 ? 2 * radius : 16) : radius;
    return h + ((flags & SM_MEDIAN) ? 3 : 0);
}

int group_bands(sm_group* g, const uint8_t* left, const uint8_t* right, int width, int height, int pitch,
                int radius, int num_disp, unsigned flags, uint8_t* disp_out, uint8_t* right_out, uint8_t* mask_out,
                int out_pitch) {
    if (!g) return fail(SM_ERR_INVALID_ARG, "null group");
    if (!left || !right || !disp_out) return fail(SM_ERR_INVALID_ARG, "null image pointer");
    if (flags & SM_DEVICE_CU_GRID)   // the literal grid is anchored at the frame's corner: not row-local
        return fail(SM_ERR_INVALID_ARG, "SM_DEVICE_CU_GRID needs whole frames (sm_group_block_match_batch_u8)");
    if (width <= 0 || height <= 0 || pitch < width || out_pitch < width)
        return fail(SM_ERR_INVALID_ARG, "bad frame geometry %dx%d pitch %d out_pitch %d", width, height, pitch,
                    out_pitch);
    // bands of whole 32-row tiles; each band's input starts on a 32-row boundary so that its tile
    // grid is the full frame's (the kept rows are then bit-identical to a single-device pass)
    constexpr int kAlign = 32;
    const int n = (int)g->w.size();
    const int tiles = (height + kAlign - 1) / kAlign;
    const int per = ((tiles + n - 1) / n) * kAlign;
    const int halo = group_halo(radius, flags);
    std::vector<std::function<int()>> jobs;
    for (int k = 0; k < n; ++k) {
        const int y0 = k * per, y1 = (k + 1) * per < height ? (k + 1) * per : height;
        if (y0 >= height) break;
        const int a = y0 - halo <= 0 ? 0 : ((y0 - halo) / kAlign) * kAlign;
        const int b = y1 + halo < height ? y1 + halo : height;
        sm_handle* h = g->w[k]->h;
        const int64_t ro = (int64_t)a * pitch, oo = (int64_t)y0 * out_pitch;
        jobs.push_back([=]() -> int {
            return host_match_rows(h, left + ro, right + ro, width, b - a, pitch, radius, num_disp, flags, y0 - a,
                                   y1 - a, disp_out + oo, right_out ? right_out + oo : nullptr,
                                   mask_out ? mask_out + oo : nullptr, out_pitch);
        });
    }
    return group_run(g, jobs);
}

}  // namespace

extern "C" {

SM_API const char* sm_version(void) { return "gpu_stereo_matching_amd 0.1.0 (gfx950)"; }

SM_API const char* sm_last_error_string(void) { return g_err; }

SM_API int sm_device_count(int* count) {
    if (!count) return fail(SM_ERR_INVALID_ARG, "null count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    *count = n;
    return SM_OK;
}

SM_API int sm_create(int device, int max_width, int max_height, int max_disp, sm_handle** out) {
    if (!out) return fail(SM_ERR_INVALID_ARG, "null out");
    *out = nullptr;
    if (max_width <= 0 || max_height <= 0 || max_disp < 1 || max_disp > sm::kMaxDisp)
        return fail(SM_ERR_INVALID_ARG, "bad capacity %dx%d/D=%d", max_width, max_height, max_disp);
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(SM_ERR_DEVICE, "no HIP device visible");
    if (device < 0 || device >= n) return fail(SM_ERR_DEVICE, "device %d out of range (%d visible)", device, n);
    hipDeviceProp_t prop;
    SM_HIP(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(SM_ERR_DEVICE, "device %d is %s; this library is built for gfx950 only", device, prop.gcnArchName);
    SM_HIP(hipSetDevice(device));
    sm_handle* h = new (std::nothrow) sm_handle();
    if (!h) return fail(SM_ERR_OUT_OF_MEMORY, "host alloc");
    h->device = device;
    h->max_w = max_width;
    h->max_h = max_height;
    h->max_d = max_disp;
    const size_t P = (size_t)max_width * max_height;
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    // the pair's device frames are one allocation, so a host pair that sits in one block (right frame
    // right after the left one) uploads as one DMA copy into d_left .. d_left + 2P (host_match_rows then
    // reads the right frame at d_left + P).  d_right itself starts 256-B aligned (at
    // d_left + P it was not even dword-aligned for odd max sizes).
    const size_t Pa = (P + 255) & ~(size_t)255;
    if (e == hipSuccess) e = hipMalloc(&h->d_left, 2 * Pa);
    if (e == hipSuccess) h->d_right = h->d_left + Pa;
    if (e == hipSuccess) e = hipMalloc(&h->d_disp, P);
    for (int i = 0; i < 4 && e == hipSuccess; ++i) e = hipEventCreate(&h->ev[i]);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->scratch_ev, hipEventDisableTiming);
    if (e != hipSuccess) {
        sm_destroy(h);
        return fail(e == hipErrorOutOfMemory ? SM_ERR_OUT_OF_MEMORY : SM_ERR_DEVICE, "sm_create: %s",
                    hipGetErrorString(e));
    }
    *out = h;
    return SM_OK;
}

SM_API int sm_destroy(sm_handle* h) {
    if (!h) return SM_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    if (h->scratch_ev && h->scratch_pending) (void)hipEventSynchronize(h->scratch_ev);   // device calls on other streams
    (void)hipFree(h->d_left);   // d_right lies in the same allocation
    (void)hipFree(h->d_disp);
    (void)hipFree(h->d_lr);
    (void)hipFree(h->d_rpart);
    (void)hipFree(h->d_aux);
    (void)hipFree(h->d_maps);
    (void)hipFree(h->d_vol);
    (void)hipFree(h->d_bgr);
    (void)hipFree(h->d_dsl);
    for (auto& ev : h->ev)
        if (ev) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : h->kev)
        if (ev) (void)hipEventDestroy(ev);
    if (h->scratch_ev) (void)hipEventDestroy(h->scratch_ev);
    if (h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return SM_OK;
}

SM_API int sm_set_param_f(sm_handle* h, int param, float value) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (param == SM_PARAM_GUIDED_EPS) {
        if (!(value > 0.f)) return fail(SM_ERR_INVALID_ARG, "guided eps must be > 0");
        h->guided_eps = value;
        return SM_OK;
    }
    if (param == SM_PARAM_STAGED_GROUP) {
        const int g = (int)value;
        if ((float)g != value || g < 1 || g > kStagedGroup)
            return fail(SM_ERR_INVALID_ARG, "staged launch group must be an integer in [1, %d]", kStagedGroup);
        if (g < h->staged_group && h->d_vol) {
            // a smaller group bounds the workspace from now on: drop the larger volume once
            // the handle's pending work is done, and let the next staged call allocate the new size
            SM_HIP(hipSetDevice(h->device));
            SM_HIP(hipStreamSynchronize(h->stream));
            if (h->scratch_pending) SM_HIP(hipEventSynchronize(h->scratch_ev));
            SM_HIP(hipFree(h->d_vol));
            h->d_vol = nullptr;
            h->vol_bytes = 0;
        }
        h->staged_group = g;
        return SM_OK;
    }
    if (param == SM_PARAM_STAGE_TIMING) {
        if (value != 0.f && value != 1.f && value != 2.f) return fail(SM_ERR_INVALID_ARG, "stage timing is 0, 1 or 2");
        h->stage_timing = (int)value;
        if (h->stage_timing == 2) h->stage_requested = false;   // back to the default: unarmed until read
        return SM_OK;
    }

    return fail(SM_ERR_INVALID_ARG, "unknown param %d", param);
}

SM_API int sm_host_alloc(size_t bytes, void** out) {
    if (!out) return fail(SM_ERR_INVALID_ARG, "null out pointer");
    *out = nullptr;
    if (bytes == 0) return fail(SM_ERR_INVALID_ARG, "zero-byte host allocation");
    // portable: usable by every device's handle (a group's members copy from one frame); mapped: the
    // kernels may write a map straight into it (host_match_rows)
    SM_HIP(hipHostMalloc(out, bytes, hipHostMallocPortable | hipHostMallocMapped));
    host_blocks_add(*out, bytes);
    return SM_OK;
}

SM_API int sm_host_free(void* p) {
    if (!p) return SM_OK;
    host_blocks_remove(p);
    SM_HIP(hipHostFree(p));
    return SM_OK;
}

SM_API int sm_block_match_u8(sm_handle* h, const uint8_t* left, const uint8_t* right, int width, int height,
                             int pitch, int radius, int num_disp, unsigned flags, uint8_t* disp_out, int out_pitch) {
    return host_match(h, left, right, width, height, pitch, radius, num_disp, flags, disp_out, nullptr, nullptr,
                      out_pitch);
}

SM_API int sm_block_match_lr_u8(sm_handle* h, const uint8_t* left, const uint8_t* right, int width, int height,
                                int pitch, int radius, int num_disp, unsigned flags, uint8_t* disp_out,
                                uint8_t* right_disp_out, uint8_t* valid_mask_out, int out_pitch) {
    return host_match(h, left, right, width, height, pitch, radius, num_disp, flags | SM_LR_CHECK, disp_out,
                      right_disp_out, valid_mask_out, out_pitch);
}

SM_API int sm_last_staged_kernel_ms(sm_handle* h, float* ad_ms, float* sad_ms, float* wta_ms) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (!h->kev_valid) return fail(SM_ERR_INVALID_ARG, "no SM_STAGED pass has run on this handle");
    SM_HIP(hipEventSynchronize(h->kev[3]));
    float t[3];
    for (int i = 0; i < 3; ++i) {
        SM_HIP(hipEventElapsedTime(&t[i], h->kev[i], h->kev[i + 1]));
        t[i] /= (float)h->kev_frames;
    }
    if (ad_ms) *ad_ms = t[0];
    if (sad_ms) *sad_ms = t[1];
    if (wta_ms) *wta_ms = t[2];
    return SM_OK;
}

SM_API int sm_last_stage_ms(sm_handle* h, float* upload_ms, float* match_ms, float* download_ms) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    h->stage_requested = true;   // auto mode: the calls from now on record the split
    if (upload_ms) *upload_ms = h->stage_ms[0];
    if (match_ms) *match_ms = h->stage_ms[1];
    if (download_ms) *download_ms = h->stage_ms[2];
    return SM_OK;
}

SM_API int sm_match_device(sm_handle* h, const uint8_t* d_left, const uint8_t* d_right, int width, int height,
                           int pitch, int batch, int64_t frame_stride, int radius, int num_disp, unsigned flags,
                           uint8_t* d_disp, int out_pitch, int64_t out_frame_stride, void* stream) {
    int rc = check_geometry(h, width, height, pitch, radius, num_disp);
    if (rc) return rc;
    if (!d_left || !d_right || !d_disp) return fail(SM_ERR_INVALID_ARG, "null device pointer");
    if (batch < 1) return fail(SM_ERR_INVALID_ARG, "batch %d < 1", batch);
    if (out_pitch < width) return fail(SM_ERR_INVALID_ARG, "out_pitch < width");
    if (batch > 1 && (frame_stride < (int64_t)pitch * height || out_frame_stride < (int64_t)out_pitch * height))
        return fail(SM_ERR_INVALID_ARG, "frame strides overlap");
    SM_HIP(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    return run_device(h, d_left, d_right, width, height, pitch, batch, frame_stride, radius, num_disp, flags, d_disp,
                      out_pitch, out_frame_stride, nullptr, nullptr, width, (int64_t)width * height, s);
}

SM_API int sm_slice_keys_device(sm_handle* h, const uint8_t* d_left, const uint8_t* d_right, int width, int height,
                                int pitch, int radius, int d_lo, int d_hi, uint32_t* d_keys, void* stream) {
    int rc = check_geometry(h, width, height, pitch, radius, d_hi > 0 ? d_hi : 1);
    if (rc) return rc;
    if (d_lo < 0 || d_hi <= d_lo || d_hi > sm::kMaxDisp)
        return fail(SM_ERR_INVALID_ARG, "bad slice [%d,%d)", d_lo, d_hi);
    if (!d_left || !d_right || !d_keys) return fail(SM_ERR_INVALID_ARG, "null device pointer");
    SM_HIP(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    // radius > 15 runs the wide-window path through the handle's volume workspace: ordered after the handle's
    // last workspace pass on another stream, as run_device orders its passes
    const bool ws = sm::wide_path(radius, width, height, pitch);
    if (ws && h->scratch_pending && h->scratch_stream != s) SM_HIP(hipStreamWaitEvent(s, h->scratch_ev, 0));
    rc = slice_keys_pass(h, d_left, d_right, width, height, pitch, radius, d_lo, d_hi, false, d_keys, nullptr, s);
    if (ws) {
        SM_HIP(hipEventRecord(h->scratch_ev, s));
        h->scratch_stream = s;
        h->scratch_pending = true;
    }
    return rc;
}

SM_API int sm_keys_to_disp_device(sm_handle* h, const uint32_t* d_keys, int width, int height, int radius,
                                  uint8_t* d_disp, int out_pitch, void* stream) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (!d_keys || !d_disp || width <= 0 || height <= 0 || out_pitch < width || radius < 0)
        return fail(SM_ERR_INVALID_ARG, "bad keys_to_disp arguments");
    SM_HIP(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    SM_HIP(sm::launch_keys_to_disp(d_keys, width, height, seed_key(radius), d_disp, out_pitch, s));
    return SM_OK;
}

SM_API int sm_guided_slice_keys_device(sm_handle* h, const uint8_t* d_left, const uint8_t* d_right, int width,
                                       int height, int pitch, int radius, int d_lo, int d_hi, int32_t* d_keys,
                                       void* stream) {
    int rc = check_geometry(h, width, height, pitch, radius, d_hi > 0 ? d_hi : 1);
    if (rc) return rc;
    if (radius > sm::kMaxFastRadius)
        return fail(SM_ERR_INVALID_ARG, "guided aggregation: radius %d > %d", radius, sm::kMaxFastRadius);
    if (d_lo < 0 || d_hi <= d_lo || d_hi > sm::kMaxDisp)
        return fail(SM_ERR_INVALID_ARG, "bad slice [%d,%d)", d_lo, d_hi);
    if (!d_left || !d_right || !d_keys) return fail(SM_ERR_INVALID_ARG, "null device pointer");
    SM_HIP(hipSetDevice(h->device));
    SM_HIP(sm::launch_guided_slice_keys(d_left, d_right, width, height, pitch, 1, (int64_t)pitch * height, radius,
                                        d_lo, d_hi, h->guided_eps, d_keys, (hipStream_t)stream));
    return SM_OK;
}

SM_API int sm_guided_keys_to_disp_device(sm_handle* h, const int32_t* d_keys, int width, int height,
                                         uint8_t* d_disp, int out_pitch, void* stream) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (!d_keys || !d_disp || width <= 0 || height <= 0 || out_pitch < width)
        return fail(SM_ERR_INVALID_ARG, "bad guided_keys_to_disp arguments");
    SM_HIP(hipSetDevice(h->device));
    SM_HIP(sm::launch_guided_keys_to_disp(d_keys, width, height, d_disp, out_pitch, (hipStream_t)stream));
    return SM_OK;
}

SM_API int sm_slice_keys_lr_device(sm_handle* h, const uint8_t* d_left, const uint8_t* d_right, int width, int height,
                                   int pitch, int radius, int d_lo, int d_hi, unsigned flags, void* d_left_keys,
                                   void* d_right_keys, void* stream) {
    int rc = check_geometry(h, width, height, pitch, radius, d_hi > 0 ? d_hi : 1);
    if (rc) return rc;
    if ((flags & ~(unsigned)SM_AGG_GUIDED) != 0u)
        return fail(SM_ERR_INVALID_ARG, "slice LR keys: flags 0x%x (SM_AGG_BOX or SM_AGG_GUIDED)", flags);
    const bool guided = (flags & SM_AGG_GUIDED) != 0;
    if (guided ? radius > sm::kMaxFastRadius
               : radius > sm::kMaxBoxRadius && !sm::wide_path(radius, width, height, pitch))
        return fail(SM_ERR_INVALID_ARG, "slice LR keys: radius %d > %d%s", radius,
                    guided ? sm::kMaxFastRadius : sm::kMaxBoxRadius,
                    guided ? "" : " outside the wide path (width 4..4096, frame < 2^31 bytes)");
    if (d_lo < 0 || d_hi <= d_lo || d_hi > sm::kMaxDisp)
        return fail(SM_ERR_INVALID_ARG, "bad slice [%d,%d)", d_lo, d_hi);
    if (!d_left || !d_right || !d_left_keys || !d_right_keys) return fail(SM_ERR_INVALID_ARG, "null device pointer");
    if ((int64_t)width * height > (int64_t)h->max_w * h->max_h)
        return fail(SM_ERR_CAPACITY, "frame %dx%d exceeds handle capacity", width, height);
    SM_HIP(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    // the right view's per-tile partials live in the handle's workspace: ordered after the handle's last
    // workspace pass on another stream, as run_device orders its passes
    if (h->scratch_pending && h->scratch_stream != s) SM_HIP(hipStreamWaitEvent(s, h->scratch_ev, 0));
    rc = slice_keys_pass(h, d_left, d_right, width, height, pitch, radius, d_lo, d_hi, guided,
                         static_cast<uint32_t*>(d_left_keys), static_cast<uint32_t*>(d_right_keys), s);
    SM_HIP(hipEventRecord(h->scratch_ev, s));
    h->scratch_stream = s;
    h->scratch_pending = true;
    return rc;
}

SM_API int sm_right_keys_to_disp_device(sm_handle* h, const void* d_keys, int64_t n, uint8_t* d_disp, void* stream) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (!d_keys || !d_disp || n < 0) return fail(SM_ERR_INVALID_ARG, "bad right_keys_to_disp arguments");
    SM_HIP(hipSetDevice(h->device));
    SM_HIP(sm::launch_keys_low_byte(static_cast<const uint32_t*>(d_keys), n, d_disp, (hipStream_t)stream));
    return SM_OK;
}

SM_API int sm_lr_check_device(sm_handle* h, const uint8_t* d_left_disp, const uint8_t* d_right_disp, int width,
                              int height, int pitch, uint8_t* d_out, uint8_t* d_mask, int out_pitch, void* stream) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (!d_left_disp || !d_right_disp || !d_out || width <= 0 || height <= 0 || pitch < width || out_pitch < width)
        return fail(SM_ERR_INVALID_ARG, "bad lr_check arguments");
    if (d_right_disp == d_out) return fail(SM_ERR_INVALID_ARG, "lr_check: the right map cannot be the output");
    SM_HIP(hipSetDevice(h->device));
    const int64_t P = (int64_t)width * height;
    SM_HIP(sm::launch_lr_check(d_left_disp, pitch, P, d_right_disp, pitch, P, 0, width, height, 1, d_out, out_pitch, P,
                               nullptr, d_mask, out_pitch, P, (hipStream_t)stream));
    return SM_OK;
}

SM_API int sm_bgr_to_gray_device(sm_handle* h, const uint8_t* d_bgr, int width, int height, int pitch, int channels,
                                 uint8_t* d_gray, int gray_pitch, void* stream) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (!d_bgr || !d_gray || width <= 0 || height <= 0 || (channels != 3 && channels != 4) ||
        pitch < width * channels || gray_pitch < width)
        return fail(SM_ERR_INVALID_ARG, "bad bgr_to_gray arguments");
    SM_HIP(hipSetDevice(h->device));
    SM_HIP(sm::launch_bgr_to_gray(d_bgr, width, height, pitch, channels, d_gray, gray_pitch, (hipStream_t)stream));
    return SM_OK;
}

SM_API int sm_remap_u8_device(sm_handle* h, const uint8_t* d_src, int width, int height, int pitch,
                              const float* d_mapx, const float* d_mapy, int map_pitch, uint8_t* d_dst, int dst_pitch,
                              void* stream) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (!d_src || !d_mapx || !d_mapy || !d_dst || width <= 0 || height <= 0 || pitch < width || map_pitch < width ||
        dst_pitch < width)
        return fail(SM_ERR_INVALID_ARG, "bad remap arguments");
    SM_HIP(hipSetDevice(h->device));
    SM_HIP(sm::launch_remap(d_src, width, height, pitch, d_mapx, d_mapy, map_pitch, d_dst, dst_pitch,
                            (hipStream_t)stream));
    return SM_OK;
}

SM_API int sm_bgr_to_gray_u8(sm_handle* h, const uint8_t* bgr, int width, int height, int pitch, int channels,
                             uint8_t* gray, int gray_pitch) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (!bgr || !gray || width <= 0 || height <= 0 || (channels != 3 && channels != 4) || pitch < width * channels ||
        gray_pitch < width)
        return fail(SM_ERR_INVALID_ARG, "bad BGR layout");
    if (width > h->max_w || height > h->max_h) return fail(SM_ERR_CAPACITY, "frame exceeds handle capacity");
    SM_HIP(hipSetDevice(h->device));
    hipStream_t s = h->stream;
    const size_t need = (size_t)width * channels * height;
    if (h->bgr_bytes < need) {
        if (h->d_bgr) (void)hipFree(h->d_bgr);
        h->d_bgr = nullptr;
        h->bgr_bytes = 0;
        SM_HIP(hipMalloc(&h->d_bgr, need));
        h->bgr_bytes = need;
    }
    SM_HIP(copy2d(h->d_bgr, (size_t)width * channels, bgr, pitch, (size_t)width * channels, height,
                            hipMemcpyHostToDevice, s));
    SM_HIP(sm::launch_bgr_to_gray(h->d_bgr, width, height, width * channels, channels, h->d_left, width, s));
    SM_HIP(copy2d(gray, gray_pitch, h->d_left, width, width, height, hipMemcpyDeviceToHost, s));
    SM_HIP(hipStreamSynchronize(s));
    return SM_OK;
}

SM_API int sm_remap_u8(sm_handle* h, const uint8_t* src, int width, int height, int pitch, const float* mapx,
                       const float* mapy, int map_pitch, uint8_t* dst, int dst_pitch) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (!src || !mapx || !mapy || !dst || width <= 0 || height <= 0 || pitch < width || map_pitch < width ||
        dst_pitch < width)
        return fail(SM_ERR_INVALID_ARG, "bad remap arguments");
    if (width > h->max_w || height > h->max_h) return fail(SM_ERR_CAPACITY, "frame exceeds handle capacity");
    SM_HIP(hipSetDevice(h->device));
    hipStream_t s = h->stream;
    const size_t plane = (size_t)width * height;
    if (h->maps_bytes < 2 * plane * sizeof(float)) {
        if (h->d_maps) (void)hipFree(h->d_maps);
        h->d_maps = nullptr;
        h->maps_bytes = 0;
        SM_HIP(hipMalloc(&h->d_maps, 2 * plane * sizeof(float)));
        h->maps_bytes = 2 * plane * sizeof(float);
    }
    float* dmx = h->d_maps;
    float* dmy = h->d_maps + plane;
    SM_HIP(copy2d(dmx, width * sizeof(float), mapx, (size_t)map_pitch * sizeof(float), width * sizeof(float),
                            height, hipMemcpyHostToDevice, s));
    SM_HIP(copy2d(dmy, width * sizeof(float), mapy, (size_t)map_pitch * sizeof(float), width * sizeof(float),
                            height, hipMemcpyHostToDevice, s));
    SM_HIP(copy2d(h->d_left, width, src, pitch, width, height, hipMemcpyHostToDevice, s));
    SM_HIP(sm::launch_remap(h->d_left, width, height, width, dmx, dmy, width, h->d_right, width, s));
    SM_HIP(copy2d(dst, dst_pitch, h->d_right, width, width, height, hipMemcpyDeviceToHost, s));
    SM_HIP(hipStreamSynchronize(s));
    return SM_OK;
}

SM_API int sm_stereo_rectify(const double* K1, const double* dist1, int ndist1, const double* K2, const double* dist2,
                             int ndist2, int width, int height, const double* R, int r_len, const double* T, double* R1,
                             double* R2, double* P1, double* P2, double* Q) {
    if (!K1 || !K2 || !R || !T || !R1 || !R2 || !P1 || !P2 || !Q || width <= 0 || height <= 0)
        return fail(SM_ERR_INVALID_ARG, "bad stereo_rectify arguments");
    auto ndist_ok = [](int n, const double* d) { return (n == 0 || n == 4 || n == 5 || n == 8) && (n == 0 || d); };
    if (!ndist_ok(ndist1, dist1) || !ndist_ok(ndist2, dist2))
        return fail(SM_ERR_INVALID_ARG, "distortion vectors hold 0, 4, 5 or 8 coefficients");
    if (r_len != 9 && r_len != 3) return fail(SM_ERR_INVALID_ARG, "R is a 3x3 matrix (9) or a rotation vector (3)");
    if (!sm::stereo_rectify(K1, dist1, ndist1, K2, dist2, ndist2, width, height, R, r_len, T, R1, R2, P1, P2, Q))
        return fail(SM_ERR_INVALID_ARG, "singular rotation matrix");
    return SM_OK;
}

namespace {
int check_map_args(const sm_handle* h, const double* K, const double* dist, int ndist, const double* R,
                   const double* P, int width, int height, const float* mx, const float* my, int map_pitch) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (!K || !R || !P || !mx || !my || width <= 0 || height <= 0 || map_pitch < width)
        return fail(SM_ERR_INVALID_ARG, "bad rectify-map arguments");
    if (!(ndist == 0 || ndist == 4 || ndist == 5 || ndist == 8) || (ndist && !dist))
        return fail(SM_ERR_INVALID_ARG, "distortion vectors hold 0, 4, 5 or 8 coefficients");
    return SM_OK;
}
}  // namespace

SM_API int sm_init_rectify_map_device(sm_handle* h, const double* K, const double* dist, int ndist, const double* R,
                                      const double* P, int width, int height, float* d_mapx, float* d_mapy,
                                      int map_pitch, void* stream) {
    int rc = check_map_args(h, K, dist, ndist, R, P, width, height, d_mapx, d_mapy, map_pitch);
    if (rc) return rc;
    SM_HIP(hipSetDevice(h->device));
    const hipError_t e = sm::launch_rectify_map(K, dist, ndist, R, P, width, height, d_mapx, d_mapy, map_pitch,
                                                (hipStream_t)stream);
    if (e == hipErrorInvalidValue) return fail(SM_ERR_INVALID_ARG, "P[:, :3] * R is singular");
    SM_HIP(e);
    return SM_OK;
}

SM_API int sm_init_rectify_map(sm_handle* h, const double* K, const double* dist, int ndist, const double* R,
                               const double* P, int width, int height, float* mapx, float* mapy, int map_pitch) {
    int rc = check_map_args(h, K, dist, ndist, R, P, width, height, mapx, mapy, map_pitch);
    if (rc) return rc;
    SM_HIP(hipSetDevice(h->device));
    hipStream_t s = h->stream;
    const size_t plane = (size_t)width * height;
    if (h->maps_bytes < 2 * plane * sizeof(float)) {
        if (h->d_maps) (void)hipFree(h->d_maps);
        h->d_maps = nullptr;
        h->maps_bytes = 0;
        SM_HIP(hipMalloc(&h->d_maps, 2 * plane * sizeof(float)));
        h->maps_bytes = 2 * plane * sizeof(float);
    }
    float* dmx = h->d_maps;
    float* dmy = h->d_maps + plane;
    const hipError_t e = sm::launch_rectify_map(K, dist, ndist, R, P, width, height, dmx, dmy, width, s);
    if (e == hipErrorInvalidValue) return fail(SM_ERR_INVALID_ARG, "P[:, :3] * R is singular");
    SM_HIP(e);
    SM_HIP(copy2d(mapx, (size_t)map_pitch * sizeof(float), dmx, width * sizeof(float), width * sizeof(float), height,
                  hipMemcpyDeviceToHost, s));
    SM_HIP(copy2d(mapy, (size_t)map_pitch * sizeof(float), dmy, width * sizeof(float), width * sizeof(float), height,
                  hipMemcpyDeviceToHost, s));
    SM_HIP(hipStreamSynchronize(s));
    return SM_OK;
}

SM_API int sm_ad_volume_device(sm_handle* h, const uint8_t* d_left, const uint8_t* d_right, int width, int height,
                               int pitch, int num_disp, uint8_t* d_dif, void* stream) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (!d_left || !d_right || !d_dif || width <= 0 || height <= 0 || pitch < width || num_disp < 1 ||
        num_disp > sm::kMaxDisp)
        return fail(SM_ERR_INVALID_ARG, "bad AD-volume arguments");
    if (width > 4096) return fail(SM_ERR_INVALID_ARG, "width %d exceeds the AD-volume kernel's 4096 columns", width);
    SM_HIP(hipSetDevice(h->device));
    SM_HIP(sm::launch_ad_volume(d_left, d_right, width, height, pitch, (int64_t)pitch * height, 1, num_disp, d_dif,
                                (int64_t)width * height * num_disp, (hipStream_t)stream));
    return SM_OK;
}

SM_API int sm_ad_volume_u8(sm_handle* h, const uint8_t* left, const uint8_t* right, int width, int height, int pitch,
                           int num_disp, uint8_t* dif_out) {
    int rc = check_geometry(h, width, height, pitch, 0, num_disp);
    if (rc) return rc;
    if (!left || !right || !dif_out) return fail(SM_ERR_INVALID_ARG, "null image pointer");
    if (width > h->max_w || height > h->max_h || num_disp > h->max_d)
        return fail(SM_ERR_CAPACITY, "frame %dx%d/D=%d exceeds handle capacity", width, height, num_disp);
    if (width > 4096) return fail(SM_ERR_INVALID_ARG, "width %d exceeds the AD-volume kernel's 4096 columns", width);
    SM_HIP(hipSetDevice(h->device));
    hipStream_t s = h->stream;
    const size_t need = (size_t)width * height * num_disp;
    rc = ensure_vol(h, need);
    if (rc) return rc;
    SM_HIP(copy2d(h->d_left, width, left, pitch, width, height, hipMemcpyHostToDevice, s));
    SM_HIP(copy2d(h->d_right, width, right, pitch, width, height, hipMemcpyHostToDevice, s));
    SM_HIP(sm::launch_ad_volume(h->d_left, h->d_right, width, height, width, (int64_t)width * height, 1, num_disp,
                                h->d_vol, (int64_t)need, s));
    SM_HIP(hipMemcpyAsync(dif_out, h->d_vol, need, hipMemcpyDeviceToHost, s));
    SM_HIP(hipStreamSynchronize(s));
    return SM_OK;
}

SM_API int sm_sad_volume_device(sm_handle* h, const uint8_t* d_left, const uint8_t* d_right, int width, int height,
                                int pitch, int radius, int num_disp, uint16_t* d_sad, void* stream) {
    int rc = check_geometry(h, width, height, pitch, radius, num_disp);
    if (rc) return rc;
    if (!d_left || !d_right || !d_sad) return fail(SM_ERR_INVALID_ARG, "null pointer");
    if (radius > sm::kMaxFastRadius) return fail(SM_ERR_INVALID_ARG, "SAD volume: radius %d > 7", radius);
    if (width > 4096) return fail(SM_ERR_INVALID_ARG, "SAD volume: width %d exceeds 4096", width);
    SM_HIP(hipSetDevice(h->device));
    const int64_t P = (int64_t)width * height;
    rc = ensure_vol(h, (size_t)(P * num_disp));
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    SM_HIP(sm::launch_ad_volume(d_left, d_right, width, height, pitch, (int64_t)pitch * height, 1, num_disp,
                                h->d_vol, P * num_disp, s));
    SM_HIP(sm::launch_box_sad_volume(h->d_vol, width, height, radius, num_disp, d_sad, s));
    return SM_OK;
}

namespace {
// getAllSAD's volume (P * D device bytes, pixel-major) on stream s into `out`, or, with out == nullptr,
// into the first P * D bytes of the handle's d_vol (*where says which).  r <= 7 and W <= 4096: AD volume
// -> u16 SAD volume in d_vol -> transpose (the AD volume at the start of d_vol is consumed by the SAD
// kernel before the transpose overwrites it, in stream order); otherwise the direct kernel.
int run_all_sad(sm_handle* h, const uint8_t* L, const uint8_t* R, int W, int H, int pitch, int radius, int D,
                uint8_t* out, uint8_t** where, hipStream_t s) {
    const int64_t P = (int64_t)W * H;
    if (radius <= sm::kMaxFastRadius && W <= 4096) {
        const int64_t ad_bytes = (P * D + 255) & ~(int64_t)255;   // the u16 volume starts 256-B aligned
        int rc = ensure_vol(h, (size_t)(ad_bytes + 2 * P * D));
        if (rc) return rc;
        uint16_t* sad = reinterpret_cast<uint16_t*>(h->d_vol + ad_bytes);
        if (!out) out = h->d_vol;
        SM_HIP(sm::launch_ad_volume(L, R, W, H, pitch, (int64_t)pitch * H, 1, D, h->d_vol, P * D, s));
        SM_HIP(sm::launch_box_sad_volume(h->d_vol, W, H, radius, D, sad, s));
        SM_HIP(sm::launch_all_sad_transpose(sad, W, H, D, out, s));
    } else {
        if (!out) {
            int rc = ensure_vol(h, (size_t)(P * D));
            if (rc) return rc;
            out = h->d_vol;
        }
        SM_HIP(sm::launch_all_sad_generic(L, R, W, H, pitch, radius, D, out, s));
    }
    if (where) *where = out;
    return SM_OK;
}
}  // namespace

SM_API int sm_all_sad_device(sm_handle* h, const uint8_t* d_left, const uint8_t* d_right, int width, int height,
                             int pitch, int radius, int num_disp, uint8_t* d_out, void* stream) {
    int rc = check_geometry(h, width, height, pitch, radius, num_disp);
    if (rc) return rc;
    if (!d_left || !d_right || !d_out) return fail(SM_ERR_INVALID_ARG, "null device pointer");
    SM_HIP(hipSetDevice(h->device));
    hipStream_t s = (hipStream_t)stream;
    // d_vol is handle workspace: order after a pass of this handle on another stream, as run_device does
    if (h->scratch_pending && h->scratch_stream != s) SM_HIP(hipStreamWaitEvent(s, h->scratch_ev, 0));
    rc = run_all_sad(h, d_left, d_right, width, height, pitch, radius, num_disp, d_out, nullptr, s);
    SM_HIP(hipEventRecord(h->scratch_ev, s));
    h->scratch_stream = s;
    h->scratch_pending = true;
    return rc;
}

SM_API int sm_all_sad_u8(sm_handle* h, const uint8_t* left, const uint8_t* right, int width, int height, int pitch,
                         int radius, int num_disp, uint8_t* sad_out) {
    int rc = check_geometry(h, width, height, pitch, radius, num_disp);
    if (rc) return rc;
    if (!left || !right || !sad_out) return fail(SM_ERR_INVALID_ARG, "null image pointer");
    if (width > h->max_w || height > h->max_h || num_disp > h->max_d)
        return fail(SM_ERR_CAPACITY, "frame %dx%d/D=%d exceeds handle capacity", width, height, num_disp);
    SM_HIP(hipSetDevice(h->device));
    hipStream_t s = h->stream;
    if (h->scratch_pending && h->scratch_stream != s) SM_HIP(hipStreamWaitEvent(s, h->scratch_ev, 0));
    const size_t need = (size_t)width * height * num_disp;
    SM_HIP(copy2d(h->d_left, width, left, pitch, width, height, hipMemcpyHostToDevice, s));
    SM_HIP(copy2d(h->d_right, width, right, pitch, width, height, hipMemcpyHostToDevice, s));
    uint8_t* vol = nullptr;
    rc = run_all_sad(h, h->d_left, h->d_right, width, height, width, radius, num_disp, nullptr, &vol, s);
    if (rc) return rc;
    SM_HIP(hipMemcpyAsync(sad_out, vol, need, hipMemcpyDeviceToHost, s));
    SM_HIP(hipStreamSynchronize(s));
    h->scratch_pending = false;   // the handle's stream has drained
    return SM_OK;
}

SM_API int sm_median_u8_device(sm_handle* h, const uint8_t* d_src, int width, int height, int pitch, int radius,
                               uint8_t* d_dst, int dst_pitch, void* stream) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (!d_src || !d_dst || width <= 0 || height <= 0 || pitch < width || dst_pitch < width)
        return fail(SM_ERR_INVALID_ARG, "bad median arguments");
    if (radius < 1 || radius > 3) return fail(SM_ERR_INVALID_ARG, "median radius %d out of [1,3]", radius);
    SM_HIP(hipSetDevice(h->device));
    SM_HIP(sm::launch_median(d_src, width, height, pitch, (int64_t)pitch * height, 1, radius, d_dst, dst_pitch,
                             (int64_t)dst_pitch * height, (hipStream_t)stream));
    return SM_OK;
}

namespace {
// segment-tree stereo behind both C entry points: refined = false ST-1, true ST-2
int segment_tree_call(sm_handle* h, const uint8_t* left_bgr, const uint8_t* right_bgr, int width, int height,
                      int pitch, int max_level, int scale, float sigma, uint8_t* disp_out, int out_pitch,
                      bool refined) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (!left_bgr || !right_bgr || !disp_out) return fail(SM_ERR_INVALID_ARG, "null image pointer");
    if (width < 2 || height < 1 || pitch < 3 * width || out_pitch < width)
        return fail(SM_ERR_INVALID_ARG, "bad frame geometry %dx%d (pitch %d, out_pitch %d)", width, height, pitch,
                    out_pitch);
    if (max_level < 1 || max_level > sm::kMaxDisp) return fail(SM_ERR_INVALID_ARG, "max_level %d out of [1,256]", max_level);
    if (scale < 0) return fail(SM_ERR_INVALID_ARG, "scale %d < 0", scale);
    if (!(sigma > 0.f)) return fail(SM_ERR_INVALID_ARG, "sigma must be > 0");
    if (width > h->max_w || height > h->max_h || max_level > h->max_d)
        return fail(SM_ERR_CAPACITY, "frame %dx%d/D=%d exceeds handle capacity %dx%d/D=%d", width, height, max_level,
                    h->max_w, h->max_h, h->max_d);
    SM_HIP(hipSetDevice(h->device));
    const auto t0 = std::chrono::steady_clock::now();
    const size_t row = (size_t)width * 3, need = 2 * row * height;
    if (h->bgr_bytes < need) {
        if (h->d_bgr) (void)hipFree(h->d_bgr);
        h->d_bgr = nullptr;
        h->bgr_bytes = 0;
        SM_HIP(hipMalloc(&h->d_bgr, need));
        h->bgr_bytes = need;
    }
    hipStream_t s = h->stream;
    if (h->scratch_pending && h->scratch_stream != s) SM_HIP(hipStreamWaitEvent(s, h->scratch_ev, 0));
    uint8_t* dl = h->d_bgr;
    uint8_t* dr = h->d_bgr + row * height;
    SM_HIP(copy2d(dl, row, left_bgr, pitch, row, height, hipMemcpyHostToDevice, s));
    SM_HIP(copy2d(dr, row, right_bgr, pitch, row, height, hipMemcpyHostToDevice, s));
    h->st_valid = false;
    constexpr float kTau = 1200.0f;   // TAU, Toolkit.h:34
    if (refined)
        SM_HIP(sm::segment_tree_refined_match(h->st, dl, dr, width, height, (int)row, max_level, scale, sigma, kTau,
                                              h->d_disp, s, &h->st_stats));
    else
        SM_HIP(sm::segment_tree_match(h->st, dl, dr, width, height, (int)row, max_level, scale, sigma, kTau, h->d_disp,
                                      s, &h->st_stats));
    SM_HIP(copy2d(disp_out, out_pitch, h->d_disp, width, width, height, hipMemcpyDeviceToHost, s));
    SM_HIP(hipStreamSynchronize(s));
    h->st_total_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    h->st_valid = true;
    return SM_OK;
}
}  // namespace

SM_API int sm_segment_tree_match_bgr_u8(sm_handle* h, const uint8_t* left_bgr, const uint8_t* right_bgr, int width,
                                        int height, int pitch, int max_level, int scale, float sigma,
                                        uint8_t* disp_out, int out_pitch) {
    try {
        return segment_tree_call(h, left_bgr, right_bgr, width, height, pitch, max_level, scale, sigma, disp_out,
                                 out_pitch, false);
    } catch (const std::bad_alloc&) {   // the host tree's buffers: no C++ exception crosses the C ABI
        return fail(SM_ERR_OUT_OF_MEMORY, "segment tree: host allocation failed");
    }
}

SM_API int sm_segment_tree_refined_bgr_u8(sm_handle* h, const uint8_t* left_bgr, const uint8_t* right_bgr, int width,
                                          int height, int pitch, int max_level, int scale, float sigma,
                                          uint8_t* disp_out, int out_pitch) {
    try {
        return segment_tree_call(h, left_bgr, right_bgr, width, height, pitch, max_level, scale, sigma, disp_out,
                                 out_pitch, true);
    } catch (const std::bad_alloc&) {
        return fail(SM_ERR_OUT_OF_MEMORY, "segment tree: host allocation failed");
    }
}

SM_API int sm_last_segment_tree_stats(sm_handle* h, float* tree_ms, float* total_ms, int* levels) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (!h->st_valid) return fail(SM_ERR_INVALID_ARG, "no segment-tree call has completed on this handle");
    if (tree_ms) *tree_ms = h->st_stats.tree_ms;
    if (total_ms) *total_ms = h->st_total_ms;
    if (levels) *levels = h->st_stats.levels;
    return SM_OK;
}

SM_API int sm_last_segment_tree_arrays(sm_handle* h, int* ints, int64_t n_ints, uint8_t* pdist, int64_t n_bytes,
                                       int* levels) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    if (!h->st_valid || h->st.last_P <= 0) return fail(SM_ERR_INVALID_ARG, "no segment-tree call has completed on this handle");
    const int64_t P = h->st.last_P, nlev = h->st.last_nlev, need = 4 * P + nlev + 1;
    // n_bytes must be the last call's pixel count exactly: a caller slicing the ints by its own width *
    // height would mis-slice them after a call on another frame shape
    if (!ints || !pdist || n_ints < need || n_bytes != P)
        return fail(SM_ERR_INVALID_ARG, "need >= %lld ints and exactly %lld pdist bytes (the last call's pixels)",
                    (long long)need, (long long)P);
    SM_HIP(hipSetDevice(h->device));
    SM_HIP(hipStreamSynchronize(h->stream));
    SM_HIP(hipMemcpy(ints, h->st.tree_i, (size_t)need * sizeof(int), hipMemcpyDeviceToHost));
    SM_HIP(hipMemcpy(pdist, h->st.tree_b, (size_t)P, hipMemcpyDeviceToHost));
    if (levels) *levels = (int)nlev;
    return SM_OK;
}

SM_API int sm_block_match_bgr_u8(sm_handle* h, const uint8_t* left_bgr, const uint8_t* right_bgr, int width,
                                 int height, int pitch, int channels, int radius, int num_disp, unsigned flags,
                                 uint8_t* disp_out, int out_pitch) {
    int rc = check_geometry(h, width, height, width, radius, num_disp);
    if (rc) return rc;
    if (!left_bgr || !right_bgr || !disp_out) return fail(SM_ERR_INVALID_ARG, "null image pointer");
    if ((channels != 3 && channels != 4) || pitch < width * channels || out_pitch < width)
        return fail(SM_ERR_INVALID_ARG, "bad BGR layout");
    if (width > h->max_w || height > h->max_h || num_disp > h->max_d)
        return fail(SM_ERR_CAPACITY, "frame exceeds handle capacity");
    SM_HIP(hipSetDevice(h->device));
    const size_t row = (size_t)width * channels, need = 2 * row * height;
    if (h->bgr_bytes < need) {
        if (h->d_bgr) (void)hipFree(h->d_bgr);
        h->d_bgr = nullptr;
        h->bgr_bytes = 0;
        SM_HIP(hipMalloc(&h->d_bgr, need));
        h->bgr_bytes = need;
    }
    hipStream_t s = h->stream;
    uint8_t* dl = h->d_bgr;
    uint8_t* dr = h->d_bgr + row * height;
    const int64_t P = (int64_t)width * height;
    // the stage split under the same SM_PARAM_STAGE_TIMING rule as the gray host calls
    const bool ev = h->stage_timing == 1 || (h->stage_timing == 2 && (h->stage_requested || verbose_env()));
    if (ev) SM_HIP(hipEventRecord(h->ev[0], s));
    SM_HIP(copy2d(dl, row, left_bgr, pitch, row, height, hipMemcpyHostToDevice, s));
    SM_HIP(copy2d(dr, row, right_bgr, pitch, row, height, hipMemcpyHostToDevice, s));
    if (ev) SM_HIP(hipEventRecord(h->ev[1], s));
    SM_HIP(sm::launch_bgr_to_gray(dl, width, height, (int)row, channels, h->d_left, width, s));
    SM_HIP(sm::launch_bgr_to_gray(dr, width, height, (int)row, channels, h->d_right, width, s));
    rc = run_device(h, h->d_left, h->d_right, width, height, width, 1, P, radius, num_disp, flags, h->d_disp, width, P,
                    nullptr, nullptr, width, P, s);
    if (rc) return rc;
    if (ev) SM_HIP(hipEventRecord(h->ev[2], s));
    SM_HIP(copy2d(disp_out, out_pitch, h->d_disp, width, width, height, hipMemcpyDeviceToHost, s));
    SM_HIP(hipEventRecord(h->ev[3], s));
    SM_HIP(hipEventSynchronize(h->ev[3]));
    if (ev) {
        SM_HIP(hipEventElapsedTime(&h->stage_ms[0], h->ev[0], h->ev[1]));
        SM_HIP(hipEventElapsedTime(&h->stage_ms[1], h->ev[1], h->ev[2]));
        SM_HIP(hipEventElapsedTime(&h->stage_ms[2], h->ev[2], h->ev[3]));
    } else {
        h->stage_ms[0] = h->stage_ms[1] = h->stage_ms[2] = 0.f;
    }
    return SM_OK;
}

SM_API int sm_stream_sync(sm_handle* h, void* stream) {
    if (!h) return fail(SM_ERR_INVALID_ARG, "null handle");
    SM_HIP(hipSetDevice(h->device));
    if (stream) {
        SM_HIP(hipStreamSynchronize((hipStream_t)stream));
        return SM_OK;
    }
    // NULL: the default stream, which is what NULL means to every device entry point, and the
    // handle's own stream (host entry points, FrameStream-style callers)
    SM_HIP(hipStreamSynchronize(nullptr));
    SM_HIP(hipStreamSynchronize(h->stream));
    return SM_OK;
}


SM_API int sm_create_group(int ngpu, const int* devices, int max_width, int max_height, int max_disp,
                           sm_group** out) {
    if (!out) return fail(SM_ERR_INVALID_ARG, "null out");
    *out = nullptr;
    if (ngpu < 1 || ngpu > 64) return fail(SM_ERR_INVALID_ARG, "group size %d out of [1, 64]", ngpu);
    sm_group* g = new (std::nothrow) sm_group();
    if (!g) return fail(SM_ERR_OUT_OF_MEMORY, "host alloc");
    for (int k = 0; k < ngpu; ++k) {
        sm_handle* h = nullptr;
        const int rc = sm_create(devices ? devices[k] : k, max_width, max_height, max_disp, &h);
        if (rc) {
            const std::string msg = g_err;
            sm_destroy_group(g);
            return fail(rc, "group member %d: %s", k, msg.c_str());
        }
        GroupWorker* w = new (std::nothrow) GroupWorker();
        if (!w) {
            sm_destroy(h);
            sm_destroy_group(g);
            return fail(SM_ERR_OUT_OF_MEMORY, "host alloc");
        }
        w->h = h;
        w->th = std::thread([w] { w->loop(); });
        g->w.push_back(w);
    }
    *out = g;
    return SM_OK;
}

SM_API int sm_destroy_group(sm_group* g) {
    if (!g) return SM_OK;
    if (!g->comms.empty()) {
        const RcclApi* api = rccl_api();
        for (ncclComm_t c : g->comms)
            if (c && api) (void)api->destroy(c);
    }
    for (GroupWorker* w : g->w) {
        {
            std::lock_guard<std::mutex> lk(w->m);
            w->quit = true;
            w->cv.notify_all();
        }
        if (w->th.joinable()) w->th.join();
        sm_destroy(w->h);
        delete w;
    }
    delete g;
    return SM_OK;
}

SM_API int sm_group_size(const sm_group* g, int* n) {
    if (!g || !n) return fail(SM_ERR_INVALID_ARG, "null argument");
    *n = (int)g->w.size();
    return SM_OK;
}

SM_API int sm_group_set_param_f(sm_group* g, int param, float value) {
    if (!g) return fail(SM_ERR_INVALID_ARG, "null group");
    for (GroupWorker* w : g->w) {
        const int rc = sm_set_param_f(w->h, param, value);
        if (rc) return rc;
    }
    return SM_OK;
}

SM_API int sm_group_block_match_u8(sm_group* g, const uint8_t* left, const uint8_t* right, int width, int height,
                                   int pitch, int radius, int num_disp, unsigned flags, uint8_t* disp_out,
                                   int out_pitch) {
    return group_bands(g, left, right, width, height, pitch, radius, num_disp, flags, disp_out, nullptr, nullptr,
                       out_pitch);
}

SM_API int sm_group_block_match_lr_u8(sm_group* g, const uint8_t* left, const uint8_t* right, int width, int height,
                                      int pitch, int radius, int num_disp, unsigned flags, uint8_t* disp_out,
                                      uint8_t* right_disp_out, uint8_t* valid_mask_out, int out_pitch) {
    return group_bands(g, left, right, width, height, pitch, radius, num_disp, flags | SM_LR_CHECK, disp_out,
                       right_disp_out, valid_mask_out, out_pitch);
}

SM_API int sm_group_dslice_block_match_u8(sm_group* g, const uint8_t* left, const uint8_t* right, int width,
                                          int height, int pitch, int radius, int num_disp, unsigned flags,
                                          uint8_t* disp_out, int out_pitch) {
    if (!g) return fail(SM_ERR_INVALID_ARG, "null group");
    if (!left || !right || !disp_out) return fail(SM_ERR_INVALID_ARG, "null image pointer");
    if (flags & SM_DEVICE_CU_GRID)   // the literal grid is anchored at the frame's corner: not row-local
        return fail(SM_ERR_INVALID_ARG, "SM_DEVICE_CU_GRID needs whole frames (sm_group_block_match_batch_u8)");
    if (width <= 0 || height <= 0 || pitch < width || out_pitch < width)
        return fail(SM_ERR_INVALID_ARG, "bad frame geometry %dx%d pitch %d out_pitch %d", width, height, pitch,
                    out_pitch);
    if ((flags & ~(unsigned)(SM_AGG_GUIDED | SM_LR_CHECK)) != 0u)
        return fail(SM_ERR_INVALID_ARG,
                    "d-slice mode: flags 0x%x (box or SM_AGG_GUIDED, optionally SM_LR_CHECK; no median, staged)", flags);
    const bool guided = (flags & SM_AGG_GUIDED) != 0;
    const DsliceCfg cfg{width, height, radius, num_disp, guided, (flags & SM_LR_CHECK) != 0};
    if (cfg.lr && !guided && radius > sm::kMaxBoxRadius && !sm::wide_path(radius, width, height, width))
        return fail(SM_ERR_INVALID_ARG, "d-slice LR: box radius %d > %d needs the wide path (width <= %d)", radius,
                    sm::kMaxBoxRadius, sm::kMaxWideWidth);
    for (GroupWorker* w : g->w) {
        int rc = check_geometry(w->h, width, height, width, radius, num_disp);
        if (rc) return rc;
        if (width > w->h->max_w || height > w->h->max_h || num_disp > w->h->max_d)
            return fail(SM_ERR_CAPACITY, "frame %dx%d/D=%d exceeds member capacity", width, height, num_disp);
    }
    if (guided && radius > sm::kMaxFastRadius)
        return fail(SM_ERR_INVALID_ARG, "guided aggregation: radius %d > %d", radius, sm::kMaxFastRadius);
    int rc = group_comms(g);
    if (rc) return rc;
    const int n = (int)g->w.size();
    // phase 1 on every member: workspace + the upload of its rows, stream synchronised (no collective yet)
    std::vector<std::function<int()>> jobs;
    for (int k = 0; k < n; ++k) {
        sm_handle* h = g->w[k]->h;
        jobs.push_back([=]() -> int { return dslice_member_upload(h, k, n, left, right, cfg, pitch); });
    }
    rc = group_run(g, jobs);
    if (rc) return rc;
    // phase 2: the collectives, entered by every member or aborted by all
    const RcclApi* api = rccl_api();
    DsliceSync sync;
    jobs.clear();
    for (int k = 0; k < n; ++k) {
        sm_handle* h = g->w[k]->h;
        ncclComm_t* c = &g->comms[k];
        DsliceSync* sy = &sync;
        jobs.push_back([=]() -> int { return dslice_member_collect(h, api, c, sy, k, n, cfg, disp_out, out_pitch); });
    }
    rc = group_run(g, jobs);
    if (sync.abort.load()) {   // some communicators were aborted: drop the rest, re-create on next use
        for (ncclComm_t& c : g->comms)
            if (c) (void)api->destroy(c);
        g->comms.clear();
    }
    return rc;
}

SM_API int sm_dslice_plan(int64_t pixels, int num_disp, int members, int member, int* d_lo, int* d_hi,
                          int64_t* chunk, int64_t* padded_pixels) {
    if (pixels <= 0 || num_disp < 1 || members < 1 || member < 0 || member >= members)
        return fail(SM_ERR_INVALID_ARG, "d-slice plan: pixels %lld, num_disp %d, member %d of %d", (long long)pixels,
                    num_disp, member, members);
    const DslicePlan p = dslice_plan(pixels, num_disp, members, member);
    if (d_lo) *d_lo = p.lo;
    if (d_hi) *d_hi = p.hi;
    if (chunk) *chunk = p.chunk;
    if (padded_pixels) *padded_pixels = p.padded;
    return SM_OK;
}

SM_API int sm_dslice_rehearse_u8(sm_handle* h, const uint8_t* left, const uint8_t* right, int width, int height,
                                 int pitch, int radius, int num_disp, unsigned flags, int members, uint8_t* disp_out,
                                 int out_pitch) {
    int rc = check_geometry(h, width, height, pitch, radius, num_disp);
    if (rc) return rc;
    if (!left || !right || !disp_out) return fail(SM_ERR_INVALID_ARG, "null image pointer");
    if (out_pitch < width) return fail(SM_ERR_INVALID_ARG, "out_pitch %d < width %d", out_pitch, width);
    if (members < 1 || members > 64) return fail(SM_ERR_INVALID_ARG, "members %d out of [1, 64]", members);
    if ((flags & ~(unsigned)(SM_AGG_GUIDED | SM_LR_CHECK)) != 0u)
        return fail(SM_ERR_INVALID_ARG, "d-slice mode: flags 0x%x (box or SM_AGG_GUIDED, optionally SM_LR_CHECK)",
                    flags);
    const bool guided = (flags & SM_AGG_GUIDED) != 0;
    if (guided && radius > sm::kMaxFastRadius)
        return fail(SM_ERR_INVALID_ARG, "guided aggregation: radius %d > %d", radius, sm::kMaxFastRadius);
    const DsliceCfg cfg{width, height, radius, num_disp, guided, (flags & SM_LR_CHECK) != 0};
    if (cfg.lr && !guided && radius > sm::kMaxBoxRadius && !sm::wide_path(radius, width, height, width))
        return fail(SM_ERR_INVALID_ARG, "d-slice LR: box radius %d > %d needs the wide path (width <= %d)", radius,
                    sm::kMaxBoxRadius, sm::kMaxWideWidth);
    if (width > h->max_w || height > h->max_h || num_disp > h->max_d)
        return fail(SM_ERR_CAPACITY, "frame %dx%d/D=%d exceeds handle capacity", width, height, num_disp);
    const int64_t P = (int64_t)width * height;
    const int n = members;
    const DslicePlan p0 = dslice_plan(P, num_disp, n, 0, height);
    // workspace: one member's layout (its gathered frames are the all-gather's result, shared by every
    // rehearsed member) followed by the other members' key maps [n - 1][padded] (and right key maps)
    const DsliceWs w = dslice_ws(nullptr, p0, n, width, cfg.lr);
    const int nk = cfg.lr ? 2 : 1;
    rc = ensure_dsl(h, w.bytes + (size_t)(nk * (n - 1) * p0.padded * 4));
    if (rc) return rc;
    SM_HIP(hipSetDevice(h->device));
    hipStream_t s = h->stream;
    const DsliceWs ws = dslice_ws(h->d_dsl, p0, n, width, cfg.lr);
    uint32_t* extra = reinterpret_cast<uint32_t*>(h->d_dsl + w.bytes);
    auto keys_of = [&](int k) { return k == 0 ? ws.keys : extra + (int64_t)(k - 1) * p0.padded; };
    auto rkeys_of = [&](int k) {
        return !cfg.lr ? nullptr : k == 0 ? ws.rkeys : extra + (int64_t)(n - 1 + k - 1) * p0.padded;
    };
    uint8_t* map = ws.map;
    // the row-split upload: member k's rows into slot k of the gathered frames, which is where the
    // in-place all-gather leaves them on every member; the pad rows of the last slots are never read
    for (int k = 0; k < n; ++k) {
        rc = dslice_upload_rows(dslice_plan(P, num_disp, n, k, height), ws, k, left, right, width, pitch, s);
        if (rc) return rc;
    }
    for (int k = 0; k < n; ++k) {   // every member's key pass, into its own buffers
        rc = dslice_keys(h, dslice_plan(P, num_disp, n, k, height), cfg, ws.gl, ws.gr, keys_of(k), rkeys_of(k), s);
        if (rc) return rc;
    }
    // the reduce-scatter's MIN (into member 0's buffers: left keys signed for guided, unsigned for box; right
    // keys signed for both, box ones being sign-flipped), then each member's chunk finalised into slot k
    for (int k = 1; k < n; ++k) {
        if (guided)
            SM_HIP(sm::launch_min_keys(reinterpret_cast<int*>(ws.keys), reinterpret_cast<const int*>(keys_of(k)),
                                       p0.padded, s));
        else
            SM_HIP(sm::launch_min_keys_u32(ws.keys, keys_of(k), p0.padded, s));
        if (cfg.lr)
            SM_HIP(sm::launch_min_keys(reinterpret_cast<int*>(ws.rkeys), reinterpret_cast<const int*>(rkeys_of(k)),
                                       p0.padded, s));
    }
    for (int k = 0; k < n; ++k) {
        const DslicePlan p = dslice_plan(P, num_disp, n, k, height);
        rc = dslice_finalise(ws.keys + k * p.chunk, p.chunk, radius, guided, map + k * p.chunk, s);
        if (rc) return rc;
        if (cfg.lr) SM_HIP(sm::launch_keys_low_byte(ws.rkeys + k * p.chunk, p.chunk, ws.rmap + k * p.chunk, s));
    }
    if (cfg.lr)
        SM_HIP(sm::launch_lr_check(map, width, P, ws.rmap, width, P, 0, width, height, 1, map, width, P, nullptr, nullptr,
                                   width, P, s));
    SM_HIP(copy2d(disp_out, out_pitch, map, width, width, height, hipMemcpyDeviceToHost, s));
    SM_HIP(hipStreamSynchronize(s));
    return SM_OK;
}

SM_API int sm_group_block_match_batch_u8(sm_group* g, const uint8_t* const* lefts, const uint8_t* const* rights,
                                         int nframes, int width, int height, int pitch, int radius, int num_disp,
                                         unsigned flags, uint8_t* const* disps, int out_pitch) {
    if (!g) return fail(SM_ERR_INVALID_ARG, "null group");
    if (nframes < 0 || (nframes > 0 && (!lefts || !rights || !disps)))
        return fail(SM_ERR_INVALID_ARG, "bad frame arrays");
    const int n = (int)g->w.size();
    std::vector<std::function<int()>> jobs;
    for (int k = 0; k < n && k < nframes; ++k) {
        sm_handle* h = g->w[k]->h;
        jobs.push_back([=]() -> int {
            for (int f = k; f < nframes; f += n) {   // frame f on member f mod n, in order
                const int rc = host_match(h, lefts[f], rights[f], width, height, pitch, radius, num_disp, flags,
                                          disps[f], nullptr, nullptr, out_pitch);
                if (rc) return rc;
            }
            return SM_OK;
        });
    }
    return group_run(g, jobs);
}

}  // extern "C"
