// Caller.cpp — singleFrame() as in BlockMatching/Caller.cpp:9-25, on the MI355X engine.
// Without OpenCV in this image, images are 8-bit PGM (gray already: the reference converts with
// cvtColor(CV_BGR2GRAY) at Caller.cpp:15-16; tests/golden holds the converted pairs) and the
// disparity is written as PGM instead of imshow.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <string>

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

void remapTest() { std::cout << "remapTest: rectification is outside this engine's scope" << std::endl; }
void cvtColorTest() { std::cout << "cvtColorTest: gray conversion is outside this engine's scope" << std::endl; }
