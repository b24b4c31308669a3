// stereo_bm.hpp — header-only C++ adapter that keeps the reference's host API (Device.cuh:50-52)
//   void blockMatching_gpu(Mat &h_left, Mat &h_right, Mat &h_disparity,
//                          int SADWindowSize, int searchRange);
//   void remap_gpu(Mat &left, Mat &right, Mat &mapX1, Mat &mapY1, Mat &mapX2, Mat &mapY2,
//                  int rows, int cols, int total, uchar *result);
//   void cvtColor_gpu(uchar3 *src, uchar *dst, int rows, int cols);
// and all of BlockMatching.h (BlockMatching.h:8-15: testBM / PreCal / getDisp / getAllSAD and the
// compareDiff / compareDisp / compareSAD checks), on top of the C ABI in
// sm_hip.h, so a Main.cpp / Caller.cpp (singleFrame, remapTest, cvtColorTest) shaped caller
// compiles and runs unchanged apart from the include.  Host-only:
// compile it with a plain C++ compiler (it declares the host type uchar3 the reference's callers
// cast to).
//
// Works with cv::Mat when OpenCV is available (define SM_WITH_OPENCV before including, after
// including <opencv2/core/core.hpp>), and with the minimal sm::Mat below otherwise (this image
// has no OpenCV).  Any Mat-like type with rows, cols, data, step and a create(rows, cols, type)
// member, or sm::Mat's (rows, cols, CV_8UC1) constructor, is accepted.
//
// Behaviour vs the reference (Device.cu:173-301):
//   same arguments, same disparity values (bit-exact), same four stdout stage lines in ms
//   ("upload data", "pre calculation", "find corr", "download data", Device.cu:218,238,257,292;
//   "pre calculation" reads 0 because the AD cost is fused into the match kernel, and a multi-GPU
//   group call, which has no single upload/download, reports its whole wall time as "find corr");
//   BlockMatching.h's functions print BlockMatching.cpp's lines ("prep location", "precalculate
//   diff", "main loop", in seconds) with the GPU call's wall time on the last line the reference
//   prints for that function; SM_QUIET silences every line;
//   the output Mat owns its memory (the reference wraps a leaked new[] buffer, :185/:300);
//   errors are reported on std::cerr and leave an all-zero map, like the reference's silent
//   launch failure but visible.
#pragma once

#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <memory>
#include <mutex>
#include <vector>

#include "sm_hip.h"

#ifndef CV_8UC1
#define CV_8UC1 0
#endif
#ifndef CV_32FC1
#define CV_32FC1 5
#endif
#ifndef CV_64FC1
#define CV_64FC1 6
#endif

// the host vector type the reference's callers cast BGR data to (Caller.cpp:92, Device.cuh:52)
struct uchar3 {
    unsigned char x, y, z;
};
typedef unsigned char uchar;

namespace sm {

// Minimal single-channel image (the subset of cv::Mat that the reference's path uses): 8-bit by
// default, CV_32FC1 for remap maps (elem = 4), CV_64FC1 for calibration matrices (elem = 8).
struct Mat {
    int rows = 0, cols = 0;
    size_t step = 0;                     // bytes per row
    size_t elem = 1;                     // bytes per element (1: CV_8UC1, 4: CV_32FC1)
    uint8_t* data = nullptr;
    std::shared_ptr<std::vector<uint8_t>> store;

    Mat() = default;
    Mat(int r, int c, int type = CV_8UC1) { create(r, c, type); }
    // wrap external memory (not owned), like cv::Mat(rows, cols, CV_8UC1, ptr)
    Mat(int r, int c, int type, void* ptr, size_t stp = 0)
        : rows(r), cols(c), elem(elem_size(type)), data(static_cast<uint8_t*>(ptr)) {
        step = stp ? stp : (size_t)c * elem;
    }
    static size_t elem_size(int type) { return type == CV_64FC1 ? 8 : type == CV_32FC1 ? 4 : 1; }
    void create(int r, int c, int type = CV_8UC1) {
        const size_t e = elem_size(type);
        if (r == rows && c == cols && e == elem && store) return;
        rows = r;
        cols = c;
        elem = e;
        step = (size_t)c * e;
        store = std::make_shared<std::vector<uint8_t>>((size_t)r * step, 0);
        data = store->data();
    }
    template <typename T> T* ptr(int r = 0) { return reinterpret_cast<T*>(data + (size_t)r * step); }
    template <typename T> const T* ptr(int r = 0) const { return reinterpret_cast<const T*>(data + (size_t)r * step); }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    size_t total() const { return (size_t)rows * cols; }
};

struct Size {                            // cv::Size: (width, height)
    int width = 0, height = 0;
    Size() = default;
    Size(int w, int h) : width(w), height(h) {}
};

namespace detail {

// SM_QUIET in the environment silences the reference's stdout lines (stage timings, BlockMatching.cpp's
// step lines)
inline bool quiet() { return std::getenv("SM_QUIET") != nullptr; }

// SM_DEVICE=k picks the device; SM_DEVICES=a,b,... (two or more) also builds a group handle
// (sm_create_group) over those devices, and blockMatching_gpu / testBM / getDisp then split each
// frame into row bands, one per device (bit-identical results).  SM_GROUP_MODE=dslice splits the
// disparity range over the devices instead (sm_group_dslice_block_match_u8: RCCL MIN reduce-scatter
// + all-gather over xGMI, the north star's split; bit-identical for box aggregation).
struct Engine {
    sm_handle* h = nullptr;
    sm_group* g = nullptr;
    int w = 0, hgt = 0, d = 0;
    ~Engine() {
        if (g) sm_destroy_group(g);
        if (h) sm_destroy(h);
    }
    static std::vector<int> device_list() {
        std::vector<int> v;
        if (const char* e = std::getenv("SM_DEVICES")) {
            std::stringstream ss(e);
            std::string tok;
            while (std::getline(ss, tok, ','))
                if (!tok.empty()) v.push_back(std::atoi(tok.c_str()));
        }
        return v;
    }
    bool ensure(int width, int height, int ndisp) {
        if (h && width <= w && height <= hgt && ndisp <= d) return true;
        if (g) sm_destroy_group(g);
        if (h) sm_destroy(h);
        h = nullptr;
        g = nullptr;
        w = width > 1920 ? width : 1920;
        hgt = height > 1080 ? height : 1080;
        d = 256;
        const std::vector<int> devs = device_list();
        int dev = devs.empty() ? 0 : devs[0];
        if (const char* e = std::getenv("SM_DEVICE")) dev = std::atoi(e);
        if (sm_create(dev, w, hgt, d, &h) != SM_OK) {
            std::cerr << "sm_create: " << sm_last_error_string() << std::endl;
            h = nullptr;
            return false;
        }
        // the d-slice mode runs through a group even on one device (a one-rank communicator)
        const char* mode = std::getenv("SM_GROUP_MODE");
        std::vector<int> gdevs = devs;
        if (gdevs.empty() && mode && std::string(mode) == "dslice") gdevs.push_back(dev);
        if ((gdevs.size() > 1 || (mode && std::string(mode) == "dslice")) &&
            sm_create_group((int)gdevs.size(), gdevs.data(), w, hgt, d, &g) != SM_OK) {
            std::cerr << "sm_create_group: " << sm_last_error_string() << std::endl;
            g = nullptr;
            return false;
        }
        return true;
    }
};

inline Engine& engine() {
    static thread_local Engine e;   // one handle per host thread (sm_hip.h threading contract)
    return e;
}

template <typename M> inline size_t row_step(const M& m) { return (size_t)m.step; }

template <typename M> inline void make_output(M& out, int rows, int cols) { out.create(rows, cols, CV_8UC1); }

}  // namespace detail

// Mat-agnostic implementation (cv::Mat or sm::Mat).
// stage_lines: print Device.cu's four stage lines (blockMatching_gpu); BlockMatching.h's functions
// print their own.
template <typename M>
inline int block_matching(const M& h_left, const M& h_right, M& h_disparity, int SADWindowSize, int searchRange,
                          unsigned flags = SM_AGG_BOX, bool stage_lines = false) {
    const int rows = h_left.rows, cols = h_left.cols;
    detail::make_output(h_disparity, rows, cols);
    if (h_right.rows != rows || h_right.cols != cols) {
        std::cerr << "blockMatching_gpu: left/right sizes differ" << std::endl;
        return SM_ERR_INVALID_ARG;
    }
    detail::Engine& e = detail::engine();
    if (!e.ensure(cols, rows, searchRange)) return SM_ERR_DEVICE;
    const char* mode = std::getenv("SM_GROUP_MODE");
    const bool dslice = e.g && mode && std::string(mode) == "dslice" && (flags & ~(unsigned)SM_AGG_GUIDED) == 0u;
    // the stage lines read the upload / match / download split of this call only: the handle stays at the
    // auto default (no event markers) for testBM / getDisp / PreCal / getAllSAD
    // (a literal SM_DEVICE_CU_GRID call runs on e.h even when a group exists, so it is timed there: ADVICE r5)
    const bool timed = stage_lines && !detail::quiet() && (!e.g || (flags & SM_DEVICE_CU_GRID));
    if (timed) sm_set_param_f(e.h, SM_PARAM_STAGE_TIMING, 1.f);
    const auto t0 = std::chrono::steady_clock::now();
    // Device.cu's literal launch geometry (SM_DEVICE_CU_GRID) is a whole-frame pass: one device
    int rc = (flags & SM_DEVICE_CU_GRID) ? sm_block_match_u8(e.h, h_left.data, h_right.data, cols, rows,
                                                             (int)detail::row_step(h_left), SADWindowSize, searchRange,
                                                             flags, h_disparity.data, (int)detail::row_step(h_disparity))
             : dslice ? sm_group_dslice_block_match_u8(e.g, h_left.data, h_right.data, cols, rows,
                                                     (int)detail::row_step(h_left), SADWindowSize, searchRange, flags,
                                                     h_disparity.data, (int)detail::row_step(h_disparity))
             : e.g ? sm_group_block_match_u8(e.g, h_left.data, h_right.data, cols, rows, (int)detail::row_step(h_left),
                                           SADWindowSize, searchRange, flags, h_disparity.data,
                                           (int)detail::row_step(h_disparity))
                 : sm_block_match_u8(e.h, h_left.data, h_right.data, cols, rows, (int)detail::row_step(h_left),
                                     SADWindowSize, searchRange, flags, h_disparity.data,
                                     (int)detail::row_step(h_disparity));
    if (timed) sm_set_param_f(e.h, SM_PARAM_STAGE_TIMING, 2.f);
    if (rc != SM_OK) {
        std::cerr << "blockMatching_gpu: " << sm_last_error_string() << std::endl;
        for (int r = 0; r < rows; ++r) std::memset(h_disparity.data + (size_t)r * detail::row_step(h_disparity), 0, cols);
        return rc;
    }
    if (stage_lines && !detail::quiet()) {
        float up = 0, mt = 0, dn = 0;
        if (e.g && !(flags & SM_DEVICE_CU_GRID))   // row bands / d-slices on several devices: one wall time
            mt = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
        else
            sm_last_stage_ms(e.h, &up, &mt, &dn);
        std::cout << "upload data : " << up << std::endl;        // Device.cu:218
        std::cout << "pre calculation : " << 0 << std::endl;     // Device.cu:238 (fused into find corr)
        std::cout << "find corr : " << mt << std::endl;          // Device.cu:257
        std::cout << "download data : " << dn << std::endl;      // Device.cu:292
    }
    return rc;
}

// remap_gpu (Device.cu:303-342): both views rectified on the GPU; `result` receives the left
// view (the reference copies back only d_left_gpu_data, :341).  Maps are CV_32FC1.
template <typename M, typename F>
inline int remap(const M& left, const M& right, const F& mapX1, const F& mapY1, const F& mapX2, const F& mapY2,
                 int rows, int cols, uint8_t* result, uint8_t* right_result = nullptr) {
    detail::Engine& e = detail::engine();
    if (!e.ensure(cols, rows, 1)) return SM_ERR_DEVICE;
    const int mp = (int)(detail::row_step(mapX1) / sizeof(float));
    int rc = sm_remap_u8(e.h, left.data, cols, rows, (int)detail::row_step(left),
                         reinterpret_cast<const float*>(mapX1.data), reinterpret_cast<const float*>(mapY1.data), mp,
                         result, cols);
    if (rc == SM_OK && right_result)
        rc = sm_remap_u8(e.h, right.data, cols, rows, (int)detail::row_step(right),
                         reinterpret_cast<const float*>(mapX2.data), reinterpret_cast<const float*>(mapY2.data),
                         (int)(detail::row_step(mapX2) / sizeof(float)), right_result, cols);
    if (rc != SM_OK) std::cerr << "remap_gpu: " << sm_last_error_string() << std::endl;
    return rc;
}

}  // namespace sm

// ---- the reference's free functions, unchanged signatures (Device.cuh:50-52) ----

// BGR -> gray of a rows x cols packed uchar3 image.  Computes what the reference's callers use,
// OpenCV 2.4 cvtColor(CV_BGR2GRAY) (Y = (1868 B + 9617 G + 4899 R + 8192) >> 14); the
// reference's own kernalCvtColor applies the luma weights to B,G,R swapped (Device.cu:136-143)
// and is deliberately not reproduced.
inline void cvtColor_gpu(uchar3* src, uchar* dst, int rows, int cols) {
    sm::detail::Engine& e = sm::detail::engine();
    if (!e.ensure(cols, rows, 1)) return;
    if (sm_bgr_to_gray_u8(e.h, reinterpret_cast<const uint8_t*>(src), cols, rows, cols * 3, 3, dst, cols) != SM_OK)
        std::cerr << "cvtColor_gpu: " << sm_last_error_string() << std::endl;
}

#ifdef SM_WITH_OPENCV
using SmHostMat = cv::Mat;
#else
using SmHostMat = sm::Mat;
#endif
// SM_DEVICE_CU_GRID=1 in the environment reproduces Device.cu's literal output, launch geometry included
// (AD only for rows < 256, cols < 320; all zero for cols > 1024: Device.cu:231-233, 253); the default is the
// intended getDisp semantics at every size.
inline void blockMatching_gpu(SmHostMat& h_left, SmHostMat& h_right, SmHostMat& h_disparity, int SADWindowSize,
                              int searchRange) {
    const char* lit = std::getenv("SM_DEVICE_CU_GRID");
    const unsigned flags = (lit && lit[0] == '1') ? (unsigned)SM_DEVICE_CU_GRID : (unsigned)SM_AGG_BOX;
    sm::block_matching(h_left, h_right, h_disparity, SADWindowSize, searchRange, flags, true);
}
inline void remap_gpu(SmHostMat& left, SmHostMat& right, SmHostMat& mapX1, SmHostMat& mapY1, SmHostMat& mapX2,
                      SmHostMat& mapY2, int rows, int cols, int /*total*/, uchar* result) {
    sm::remap(left, right, mapX1, mapY1, mapX2, mapY2, rows, cols, result);
}

// ---- BlockMatching.h (BlockMatching.h:8-15): the reference's CPU entry points, same signatures
//      and outputs, computed on the GPU ----
namespace sm {
namespace detail {
// BlockMatching.cpp's step lines (cout << label << seconds, :32,49,84 / :136,153,188 / :215,232).  The
// tap table and the AD volume are not separate steps here (0); `main` is the GPU call's wall time.
inline void cpu_lines(double main_s, bool with_main) {
    if (quiet()) return;
    std::cout << "prep location " << 0 << std::endl;
    std::cout << "precalculate diff " << (with_main ? 0.0 : main_s) << std::endl;
    if (with_main) std::cout << "main loop " << main_s << std::endl;
}
inline double seconds_since(std::chrono::steady_clock::time_point t0) {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
}  // namespace detail
}  // namespace sm

// testBM / getDisp: the disparity map of getDisp (BlockMatching.cpp:7-87, :111-189), bit-exact.
inline void testBM(const SmHostMat& left0, const SmHostMat& right0, SmHostMat& disparity, int SAD, int searchRange) {
    const auto t0 = std::chrono::steady_clock::now();
    sm::block_matching(left0, right0, disparity, SAD, searchRange);
    sm::detail::cpu_lines(sm::detail::seconds_since(t0), true);
}
inline void getDisp(const SmHostMat& left0, const SmHostMat& right0, uchar* disparity, int SAD, int searchRange) {
    sm::detail::Engine& e = sm::detail::engine();
    if (!e.ensure(left0.cols, left0.rows, searchRange)) return;
    const int lp = (int)sm::detail::row_step(left0);
    const auto t0 = std::chrono::steady_clock::now();
    if ((e.g ? sm_group_block_match_u8(e.g, left0.data, right0.data, left0.cols, left0.rows, lp, SAD, searchRange,
                                       SM_AGG_BOX, disparity, left0.cols)
             : sm_block_match_u8(e.h, left0.data, right0.data, left0.cols, left0.rows, lp, SAD, searchRange,
                                 SM_AGG_BOX, disparity, left0.cols)) != SM_OK)
        std::cerr << "getDisp: " << sm_last_error_string() << std::endl;
    sm::detail::cpu_lines(sm::detail::seconds_since(t0), true);
}
// PreCal (BlockMatching.cpp:89-109): the AD volume, searchRange d-major planes of rows*cols bytes.
// Entries with x < d are written as 0 (the reference leaves them at the caller's memset 0).  The
// reference's PreCal prints nothing.
inline void PreCal(const SmHostMat& left0, const SmHostMat& right0, uchar* dif_, int /*SAD*/, int searchRange) {
    sm::detail::Engine& e = sm::detail::engine();
    if (!e.ensure(left0.cols, left0.rows, searchRange)) return;
    if (sm_ad_volume_u8(e.h, left0.data, right0.data, left0.cols, left0.rows, (int)sm::detail::row_step(left0),
                        searchRange, dif_) != SM_OK)
        std::cerr << "PreCal: " << sm_last_error_string() << std::endl;
}
// getAllSAD (BlockMatching.cpp:191-261): every window SAD, pixel-major data_dm[p * searchRange + d],
// truncated to uchar, 255 where col + d > cols; bit-exact (sm_all_sad_u8).
inline void getAllSAD(const SmHostMat& left0, const SmHostMat& right0, uchar* data_dm, int SAD, int searchRange) {
    sm::detail::Engine& e = sm::detail::engine();
    if (!e.ensure(left0.cols, left0.rows, searchRange)) return;
    const auto t0 = std::chrono::steady_clock::now();
    if (sm_all_sad_u8(e.h, left0.data, right0.data, left0.cols, left0.rows, (int)sm::detail::row_step(left0), SAD,
                      searchRange, data_dm) != SM_OK)
        std::cerr << "getAllSAD: " << sm_last_error_string() << std::endl;
    sm::detail::cpu_lines(sm::detail::seconds_since(t0), false);
}
// The reference's debugging cross-checks (BlockMatching.cpp:263-308), same output format: the
// reference result is recomputed (PreCal / getDisp / getAllSAD above) and every mismatching index is
// printed; compareDiff and compareSAD end with "-1" and no newline.
inline void compareDiff(const SmHostMat& left0, const SmHostMat& right0, uchar* GPUresult, int SADWindowSize,
                        int searchRange, int total) {
    std::vector<uchar> ref((size_t)total * searchRange, 0);
    PreCal(left0, right0, ref.data(), SADWindowSize, searchRange);
    for (size_t i = 0; i < (size_t)searchRange * total; i++)
        if (ref[i] != GPUresult[i]) std::cout << i << std::endl;
    std::cout << -1;
}
inline void compareDisp(const SmHostMat& left, const SmHostMat& right, uchar* GPUresult, int SADWindowSize,
                        int searchRange, int cols, int rows) {
    std::vector<uchar> ref((size_t)rows * cols);
    getDisp(left, right, ref.data(), SADWindowSize, searchRange);
    for (size_t i = 0; i < (size_t)rows; i++)
        for (size_t j = 0; j < (size_t)cols; j++)
            if (ref[i * cols + j] != GPUresult[i * cols + j]) {
                std::cout << "[" << i << ":" << j << "]" << std::endl;
                std::cout << "CPU = " << (int)ref[i * cols + j] << ", GPU = " << (int)GPUresult[i * cols + j]
                          << std::endl;
            }
}
inline void compareSAD(const SmHostMat& left, const SmHostMat& right, uchar* GPUresult, int SADWindowSize,
                       int searchRange, int cols, int rows) {
    const size_t total = (size_t)rows * cols;
    std::vector<uchar> allSAD((size_t)searchRange * total, 255);
    getAllSAD(left, right, allSAD.data(), SADWindowSize, searchRange);
    for (size_t i = 0; i < (size_t)searchRange * total; i++)
        if (allSAD[i] != GPUresult[i]) std::cout << i << std::endl;
    std::cout << -1;
}

// ---- Utility.h (Utility.h:26-27, :42): the calibration load and Rectify in front of remap_gpu ----
namespace sm {
namespace detail {

// Every `name: !!opencv-matrix` node of an OpenCV FileStorage YAML file (the block form
// FileStorage writes: rows / cols / dt / data: [ ... ]), as CV_64FC1 — LoadDataBatch converts each
// matrix with convertTo(..., CV_64F), Utility.cpp:29-40.  Values are rounded through float first
// when dt is 'f', as FileStorage stores them in a CV_32F Mat.
inline bool read_opencv_matrix(const std::string& text, const std::string& name, Mat& out) {
    size_t pos = 0;
    for (;;) {
        pos = text.find(name, pos);
        if (pos == std::string::npos) return false;
        const bool start = pos == 0 || text[pos - 1] == ' ' || text[pos - 1] == '\n' || text[pos - 1] == '\t';
        size_t q = pos + name.size();
        while (q < text.size() && text[q] == ' ') ++q;
        if (start && q < text.size() && text[q] == ':') break;
        pos = q;
    }
    auto field = [&](const char* key) -> std::string {
        const size_t k = text.find(key, pos);
        if (k == std::string::npos) return std::string();
        size_t v = text.find(':', k) + 1;
        while (v < text.size() && text[v] == ' ') ++v;
        size_t e = v;
        while (e < text.size() && text[e] != '\n' && text[e] != '\r') ++e;
        return text.substr(v, e - v);
    };
    const int rows = std::atoi(field("rows").c_str()), cols = std::atoi(field("cols").c_str());
    const std::string dt = field("dt");
    const size_t lb = text.find('[', text.find("data", pos)), rb = text.find(']', lb);
    if (rows <= 0 || cols <= 0 || lb == std::string::npos || rb == std::string::npos) return false;
    std::string body = text.substr(lb + 1, rb - lb - 1);
    for (char& c : body)
        if (c == ',' || c == '\n' || c == '\r') c = ' ';
    std::istringstream is(body);
    out.create(rows, cols, CV_64FC1);
    for (int i = 0; i < rows * cols; ++i) {
        double v;
        if (!(is >> v)) return false;
        out.ptr<double>(i / cols)[i % cols] = (!dt.empty() && dt[0] == 'f') ? (double)(float)v : v;
    }
    return true;
}

template <typename M> inline std::vector<double> to_f64(const M& m) {   // CV_64FC1 Mat -> row-major vector
    std::vector<double> v;
    for (int r = 0; r < m.rows; ++r)
        for (int c = 0; c < m.cols; ++c) v.push_back(reinterpret_cast<const double*>(m.data + (size_t)r * m.step)[c]);
    return v;
}

}  // namespace detail

// LoadData (Utility.cpp:17-23): one matrix by name (CV_64FC1).
inline Mat LoadData(const std::string& filename, const std::string& varName) {
    std::ifstream f(filename);
    std::stringstream ss;
    ss << f.rdbuf();
    Mat m;
    if (!detail::read_opencv_matrix(ss.str(), varName, m)) std::cerr << "LoadData: no matrix " << varName << std::endl;
    return m;
}

// LoadDataBatch (Utility.cpp:25-42): LeftMat, RightMat, LeftDist, RightDist, RotationVec,
// TranslationVec, each as CV_64FC1.  Returns false (and says which) when the file or a node is missing.
inline bool LoadDataBatch(const std::string& filename, Mat& camMat1, Mat& camMat2, Mat& distCoe1, Mat& distCoe2,
                          Mat& R, Mat& T) {
    std::ifstream f(filename);
    if (!f) {
        std::cerr << "LoadDataBatch: cannot open " << filename << std::endl;
        return false;
    }
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    const char* names[6] = {"LeftMat", "RightMat", "LeftDist", "RightDist", "RotationVec", "TranslationVec"};
    Mat* outs[6] = {&camMat1, &camMat2, &distCoe1, &distCoe2, &R, &T};
    for (int i = 0; i < 6; ++i)
        if (!detail::read_opencv_matrix(text, names[i], *outs[i])) {
            std::cerr << "LoadDataBatch: no matrix " << names[i] << " in " << filename << std::endl;
            return false;
        }
    return true;
}

// Rectify (Utility.cpp:228-234): stereoRectify(..., CV_CALIB_ZERO_DISPARITY) on the host, then the
// CV_32FC1 maps of both cameras computed on the GPU (sm_init_rectify_map).  Inputs are CV_64FC1
// (what LoadDataBatch returns); R is 3x3 or a 3-vector.
template <typename M, typename F>
inline int Rectify(const M& camMat1, const M& camMat2, const M& distCoe1, const M& distCoe2, const M& R, const M& T,
                   Size imageSize, F& mapX1, F& mapY1, F& mapX2, F& mapY2) {
    const std::vector<double> K1 = detail::to_f64(camMat1), K2 = detail::to_f64(camMat2);
    const std::vector<double> d1 = detail::to_f64(distCoe1), d2 = detail::to_f64(distCoe2);
    const std::vector<double> Rv = detail::to_f64(R), Tv = detail::to_f64(T);
    if (K1.size() != 9 || K2.size() != 9 || Tv.size() != 3 || (Rv.size() != 9 && Rv.size() != 3)) {
        std::cerr << "Rectify: bad matrix sizes" << std::endl;
        return SM_ERR_INVALID_ARG;
    }
    double R1[9], R2[9], P1[12], P2[12], Q[16];
    const int w = imageSize.width, h = imageSize.height;
    int rc = sm_stereo_rectify(K1.data(), d1.empty() ? nullptr : d1.data(), (int)d1.size(), K2.data(),
                               d2.empty() ? nullptr : d2.data(), (int)d2.size(), w, h, Rv.data(), (int)Rv.size(),
                               Tv.data(), R1, R2, P1, P2, Q);
    detail::Engine& e = detail::engine();
    if (rc == SM_OK && !e.ensure(w, h, 1)) rc = SM_ERR_DEVICE;
    if (rc == SM_OK) {
        mapX1.create(h, w, CV_32FC1), mapY1.create(h, w, CV_32FC1), mapX2.create(h, w, CV_32FC1), mapY2.create(h, w, CV_32FC1);
        rc = sm_init_rectify_map(e.h, K1.data(), d1.empty() ? nullptr : d1.data(), (int)d1.size(), R1, P1, w, h,
                                 reinterpret_cast<float*>(mapX1.data), reinterpret_cast<float*>(mapY1.data),
                                 (int)(mapX1.step / sizeof(float)));
    }
    if (rc == SM_OK)
        rc = sm_init_rectify_map(e.h, K2.data(), d2.empty() ? nullptr : d2.data(), (int)d2.size(), R2, P2, w, h,
                                 reinterpret_cast<float*>(mapX2.data), reinterpret_cast<float*>(mapY2.data),
                                 (int)(mapX2.step / sizeof(float)));
    if (rc != SM_OK) std::cerr << "Rectify: " << sm_last_error_string() << std::endl;
    return rc;
}

}  // namespace sm
