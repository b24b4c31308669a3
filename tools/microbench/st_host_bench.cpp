// Host segment-tree build time (csrc/bm_segtree_host.h) on one view: reads W, H (int32) and W*H*3 BGR
// bytes, forms the colour weights on the 3x3-median guide as st_weights_kernel does, and reports the best
// of N builds.  usage: st_host_bench FILE [threads] [iters]
// Built against a given copy of the header to compare versions on the same host (-I DIR).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "bm_segtree_host.h"

using namespace sm::st_host;

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "rb");
    if (!f) return 2;
    int wh[2];
    if (fread(wh, 4, 2, f) != 2) return 2;
    const int W = wh[0], H = wh[1], P = W * H;
    std::vector<uint8_t> bgr((size_t)P * 3);
    if (fread(bgr.data(), 1, bgr.size(), f) != bgr.size()) return 2;
    fclose(f);
#ifdef SM_HAVE_PAR
    if (argc > 2) g_par_threads = atoi(argv[2]);
#endif
    const int iters = argc > 3 ? atoi(argv[3]) : 20;
    std::vector<uint8_t> g((size_t)P * 3), wr(P, 0), wu(P, 0);
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            for (int c = 0; c < 3; ++c) {
                uint8_t v[9];
                int k = 0;
                for (int i = -1; i <= 1; ++i)
                    for (int j = -1; j <= 1; ++j)
                        v[k++] = bgr[((size_t)std::min(std::max(y + i, 0), H - 1) * W + std::min(std::max(x + j, 0), W - 1)) * 3 + c];
                std::nth_element(v, v + 4, v + 9);
                g[((size_t)y * W + x) * 3 + c] = v[4];
            }
    for (int p = 0; p < P; ++p) {
        const int x = p % W;
        for (int c = 0; c < 3; ++c) {
            if (x + 1 < W) wr[p] = std::max(wr[p], (uint8_t)std::abs(g[p * 3 + c] - g[(p + 1) * 3 + c]));
            if (p >= W) wu[p] = std::max(wu[p], (uint8_t)std::abs(g[p * 3 + c] - g[(p - W) * 3 + c]));
        }
    }
    double best = 1e30;
    int levels = 0;
    for (int it = 0; it < iters; ++it) {
        const auto t0 = std::chrono::steady_clock::now();
        HostTree t;
        if (!build_tree(wr.data(), wu.data(), W, H, 1200.f, t)) return 1;
        best = std::min(best, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        levels = (int)t.lev.size() - 1;
    }
    printf("%dx%d levels %d threads %s: build_tree best %.3f ms\n", W, H, levels, argc > 2 ? argv[2] : "default", best);
    return 0;
}
