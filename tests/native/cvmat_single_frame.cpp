// Compile (and, on a GPU box, run) test of include/stereo_bm.hpp's SM_WITH_OPENCV branch
// (stereo_bm.hpp:235-243): the reference's callers pass cv::Mat (Caller.cpp:9-25), whose `step` is a
// cv::MatStep, not a size_t.  OpenCV is absent from this image, so the few cv::Mat members the
// adapter touches are declared below: rows, cols, uchar* data, a MatStep `step` convertible to
// size_t, and create(rows, cols, type).  This stand-in claims nothing about OpenCV itself; it only
// proves the adapter instantiates and runs on a Mat whose step is a MatStep.  Rows are padded to a
// multiple of 64 bytes, as cv::Mat rows of a ROI or an aligned allocator can be, so the pitched
// upload / download paths run too.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>
#include <memory>
#include <string>
#include <vector>

typedef unsigned char uchar;
namespace cv {
struct MatStep {
    size_t p[2] = {0, 1};
    operator size_t() const { return p[0]; }
    size_t operator[](int i) const { return p[i]; }
};
struct Mat {
    int rows = 0, cols = 0;
    uchar* data = nullptr;
    MatStep step;
    std::shared_ptr<std::vector<uchar>> buf;
    void create(int r, int c, int /*type*/) {
        rows = r;
        cols = c;
        step.p[0] = ((size_t)c + 63) & ~(size_t)63;
        buf = std::make_shared<std::vector<uchar>>(step.p[0] * r, 0xAB);
        data = buf->data();
    }
};
}  // namespace cv
#define CV_8UC1 0
#define SM_WITH_OPENCV
#include "stereo_bm.hpp"

static bool read_pgm(const char* path, cv::Mat& m) {
    std::ifstream f(path, std::ios::binary);
    std::string magic;
    int w = 0, h = 0, maxv = 0;
    if (!(f >> magic >> w >> h >> maxv) || magic != "P5" || maxv != 255) return false;
    f.get();
    m.create(h, w, CV_8UC1);
    for (int r = 0; r < h; ++r) f.read(reinterpret_cast<char*>(m.data + r * (size_t)m.step), w);
    return (bool)f;
}

// singleFrame() (Caller.cpp:9-25) on cv::Mat: blockMatching_gpu(g1, g2, disp, 5, 64), then the map
// written as PGM (imshow in the reference); also testBM, the BlockMatching.h entry point.
int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s left.pgm right.pgm out.pgm SAD range\n", argv[0]);
        return 2;
    }
    cv::Mat g1, g2, disp, disp2;
    if (!read_pgm(argv[1], g1) || !read_pgm(argv[2], g2)) return 2;
    const int sad = std::atoi(argv[4]), range = std::atoi(argv[5]);
    blockMatching_gpu(g1, g2, disp, sad, range);
    testBM(g1, g2, disp2, sad, range);
    std::ofstream o(argv[3], std::ios::binary);
    o << "P5\n" << disp.cols << " " << disp.rows << "\n255\n";
    for (int r = 0; r < disp.rows; ++r) {
        if (std::memcmp(disp.data + r * (size_t)disp.step, disp2.data + r * (size_t)disp2.step, disp.cols) != 0) {
            std::fprintf(stderr, "testBM and blockMatching_gpu differ in row %d\n", r);
            return 3;
        }
        o.write(reinterpret_cast<const char*>(disp.data + r * (size_t)disp.step), disp.cols);
    }
    return o ? 0 : 4;
}
