// Host segment-tree build time (csrc/bm_segtree_host.h) on one view: reads W, H (int32) and W*H*3 BGR
// bytes, forms the colour weights on the 3x3-median guide as st_weights_kernel does, and reports the best
// of N builds.  usage: st_host_bench FILE [threads] [iters]
// Built against a given copy of the header to compare versions on the same host (-I DIR).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>

// phase times of tree_from_edges (first pass, second pass + neighbour lists, BFS)
static std::chrono::steady_clock::time_point g_mark[4];
#define SM_ST_PHASE(k) (g_mark[(k) + 1] = std::chrono::steady_clock::now())
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
    // as the GPU path since round 4: the sorted edges are given, one tree object is reused across builds
    double best = 1e30, ph[3] = {0, 0, 0};
    int levels = 0;
    HostTree t;
    const std::vector<Edge> e0 = sorted_edges_u8(wr.data(), wu.data(), W, P);
    std::vector<Edge> e;
    auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    for (int it = 0; it < iters; ++it) {
        e = e0;
        g_mark[0] = std::chrono::steady_clock::now();
        if (!tree_from_edges(e.data(), (int)e.size(), P, W, 1200.f, 1.0f, t)) return 1;
        const double tot = ms(g_mark[0], g_mark[3]);
        if (tot < best) {
            best = tot;
            for (int k = 0; k < 3; ++k) ph[k] = ms(g_mark[k], g_mark[k + 1]);
        }
        levels = (int)t.lev.size() - 1;
    }
    printf("%dx%d levels %d threads %s: tree_from_edges best %.3f ms (first pass %.3f, second pass + lists %.3f, "
           "BFS %.3f)\n", W, H, levels, argc > 2 ? argv[2] : "default", best, ph[0], ph[1], ph[2]);
    return 0;
}
