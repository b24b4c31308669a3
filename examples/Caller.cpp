// Caller.cpp — the reference's demos (BlockMatching/Caller.cpp) on the MI355X engine.
// Without OpenCV in this image, images are 8-bit PGM (gray already: the reference converts with
// cvtColor(CV_BGR2GRAY) at Caller.cpp:15-16; tests/golden holds the converted pairs) and the
// disparity is written as PGM instead of imshow.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <string>
#include <utility>
#include <vector>

#include "Caller.h"
#include "stereo_bm.hpp"

static bool read_pgm(const std::string& path, sm::Mat& m) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return false;
    std::string magic;
    int w = 0, h = 0, maxv = 0;
    f >> magic >> w >> h >> maxv;
    f.get();
    if (magic != "P5" || w <= 0 || h <= 0 || maxv != 255) return false;
    m.create(h, w);
    f.read(reinterpret_cast<char*>(m.data), (std::streamsize)m.total());
    return (bool)f;
}

static bool write_pgm(const std::string& path, const sm::Mat& m) {
    std::ofstream f(path, std::ios::binary);
    if (!f) return false;
    f << "P5\n" << m.cols << " " << m.rows << "\n255\n";
    for (int r = 0; r < m.rows; ++r) f.write(reinterpret_cast<const char*>(m.ptr<uint8_t>(r)), m.cols);
    return (bool)f;
}

static std::string env_or(const char* k, const char* dflt) {
    const char* v = std::getenv(k);
    return v ? std::string(v) : std::string(dflt);
}

void singleFrame() {
    sm::Mat g1, g2, disp;
    const std::string left = env_or("SM_LEFT", "view1_.pgm"), right = env_or("SM_RIGHT", "view5_.pgm");
    if (!read_pgm(left, g1) || !read_pgm(right, g2)) {
        std::cerr << "cannot read " << left << " / " << right << std::endl;
        std::exit(2);
    }
    const int sad = std::atoi(env_or("SM_SAD", "5").c_str());        // Caller.cpp:19: 5, 64
    const int range = std::atoi(env_or("SM_RANGE", "64").c_str());
    auto t0 = std::chrono::steady_clock::now();
    blockMatching_gpu(g1, g2, disp, sad, range);
    auto t1 = std::chrono::steady_clock::now();
    std::cout << "GPU : " << std::chrono::duration<double>(t1 - t0).count() << std::endl;   // Caller.cpp:21
    write_pgm(env_or("SM_OUT", "disp.pgm"), disp);                    // imshow("disp", disp) in the reference
}

// remapTest (Caller.cpp:27-74): the reference's chain on the gray, already-resized pair —
// LoadDataBatch (the YAML calibration, SM_CALIB) -> Rectify (stereoRectify + the CV_32FC1 maps on the
// GPU) -> remap_gpu.  Both rectified views are written as PGM (SM_OUT, SM_OUT2) instead of imshow,
// and the four maps as raw float32 planes (SM_MAPS, optional).
void remapTest() {
    sm::Mat left, right, mapX1, mapY1, mapX2, mapY2;
    sm::Mat camMat1, camMat2, distCoe1, distCoe2, R, T;
    if (!read_pgm(env_or("SM_LEFT", "left_320x200.pgm"), left) ||
        !read_pgm(env_or("SM_RIGHT", "right_320x200.pgm"), right)) {
        std::cerr << "cannot read the pair" << std::endl;
        std::exit(2);
    }
    const int rows = left.rows, cols = left.cols, total = rows * cols;
    if (!sm::LoadDataBatch(env_or("SM_CALIB", "Calib_Data_OpenCV.yml"), camMat1, camMat2, distCoe1, distCoe2, R, T))
        std::exit(2);
    if (sm::Rectify(camMat1, camMat2, distCoe1, distCoe2, R, T, sm::Size(cols, rows), mapX1, mapY1, mapX2, mapY2) !=
        SM_OK)
        std::exit(3);
    sm::Mat result(rows, cols), result2(rows, cols);
    auto t0 = std::chrono::steady_clock::now();
    remap_gpu(left, right, mapX1, mapY1, mapX2, mapY2, rows, cols, total, result.data);
    auto t1 = std::chrono::steady_clock::now();
    std::cout << "GPU Remap : " << std::chrono::duration<double, std::milli>(t1 - t0).count() << std::endl;
    sm::remap(left, right, mapX1, mapY1, mapX2, mapY2, rows, cols, result.data, result2.data);
    write_pgm(env_or("SM_OUT", "remap_left.pgm"), result);
    write_pgm(env_or("SM_OUT2", "remap_right.pgm"), result2);
    const std::string maps = env_or("SM_MAPS", "");
    if (!maps.empty()) {
        std::ofstream f(maps, std::ios::binary);
        for (const sm::Mat* m : {&mapX1, &mapY1, &mapX2, &mapY2})
            f.write(reinterpret_cast<const char*>(m->data), (std::streamsize)(m->step * rows));
    }
}

// cvtColorTest (Caller.cpp:76-113): BGR -> gray with cvtColor_gpu on a binary PPM (P6, RGB order on
// disk, swapped to BGR in memory like imread), written as PGM.
void cvtColorTest() {
    std::ifstream f(env_or("SM_BGR", "view1_.ppm"), std::ios::binary);
    std::string magic;
    int w = 0, h = 0, maxv = 0;
    if (!(f >> magic >> w >> h >> maxv) || magic != "P6" || maxv != 255) {
        std::cerr << "cannot read PPM" << std::endl;
        std::exit(2);
    }
    f.get();
    std::vector<uchar3> bgr((size_t)w * h);
    f.read(reinterpret_cast<char*>(bgr.data()), (std::streamsize)(bgr.size() * 3));
    for (auto& p : bgr) std::swap(p.x, p.z);                           // RGB on disk -> BGR (imread order)
    sm::Mat gray(h, w);
    auto t0 = std::chrono::steady_clock::now();
    cvtColor_gpu(bgr.data(), gray.data, h, w);
    auto t1 = std::chrono::steady_clock::now();
    std::cout << "GPU cvtColor : " << std::chrono::duration<double, std::milli>(t1 - t0).count() << std::endl;
    write_pgm(env_or("SM_OUT", "gray.pgm"), gray);
}

// Not a reference demo: all seven BlockMatching.h functions through the adapter (the reference uses
// them to cross-check its GPU path, Device.cu:241-243, 265-268, 297; BlockMatching.cpp:263-308).
// Writes the testBM and getDisp maps (PGM), the AD volume (raw, D planes) and the getAllSAD volume
// (raw, pixel-major), then runs compareDiff / compareDisp / compareSAD on the results as computed
// and once more with one planted mismatch each (stdout sections "== compareX clean|planted").
void blockMatchingApiTest() {
    sm::Mat g1, g2, disp;
    if (!read_pgm(env_or("SM_LEFT", "view1_.pgm"), g1) || !read_pgm(env_or("SM_RIGHT", "view5_.pgm"), g2)) {
        std::cerr << "cannot read the pair" << std::endl;
        std::exit(2);
    }
    const int sad = std::atoi(env_or("SM_SAD", "5").c_str());
    const int range = std::atoi(env_or("SM_RANGE", "64").c_str());
    const int rows = g1.rows, cols = g1.cols, total = rows * cols;
    testBM(g1, g2, disp, sad, range);
    write_pgm(env_or("SM_OUT", "disp.pgm"), disp);
    sm::Mat disp2(rows, cols);
    getDisp(g1, g2, disp2.data, sad, range);
    write_pgm(env_or("SM_OUT2", "disp2.pgm"), disp2);
    std::vector<uchar> dif((size_t)total * range, 0);
    PreCal(g1, g2, dif.data(), sad, range);
    {
        std::ofstream f(env_or("SM_VOL", "dif.u8"), std::ios::binary);
        f.write(reinterpret_cast<const char*>(dif.data()), (std::streamsize)dif.size());
    }
    std::vector<uchar> all((size_t)total * range, 0);
    getAllSAD(g1, g2, all.data(), sad, range);
    {
        std::ofstream f(env_or("SM_SADVOL", "allsad.u8"), std::ios::binary);
        f.write(reinterpret_cast<const char*>(all.data()), (std::streamsize)all.size());
    }
    std::cout << "== compareDiff clean" << std::endl;
    compareDiff(g1, g2, dif.data(), sad, range, total);
    std::cout << std::endl << "== compareDisp clean" << std::endl;
    compareDisp(g1, g2, disp2.data, sad, range, cols, rows);
    std::cout << "== compareSAD clean" << std::endl;
    compareSAD(g1, g2, all.data(), sad, range, cols, rows);
    std::cout << std::endl;
    dif[7] ^= 1;
    disp2.data[1 * cols + 2] ^= 1;
    all[5] ^= 1;
    std::cout << "== compareDiff planted" << std::endl;
    compareDiff(g1, g2, dif.data(), sad, range, total);
    std::cout << std::endl << "== compareDisp planted" << std::endl;
    compareDisp(g1, g2, disp2.data, sad, range, cols, rows);
    std::cout << "== compareSAD planted" << std::endl;
    compareSAD(g1, g2, all.data(), sad, range, cols, rows);
    std::cout << std::endl;
}
