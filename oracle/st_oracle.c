/*
 * st_oracle.c — CPU restatement of the reference's segment-tree stereo (STMatching, ST-1 /
 * "ST_RAW": StereoDisparity.cpp:57-89), the checker of the GPU segment-tree path.
 *
 * TEST INFRASTRUCTURE ONLY, like bm_oracle.c: nothing in the product links, loads or calls it.
 * The reference's STMatching sources need OpenCV, absent here, so they are unbuildable; this file
 * restates their algorithm in plain C, citing the lines it follows.  Parity with the reference
 * binary is therefore unpinned; the float operations are written in the reference's
 * order (no FMA contraction: the Makefile passes -ffp-contract=off).
 *
 * ST-2 ("ST_REFINED", StereoDisparity.cpp:91-160) reuses these pieces: ora_st2_disp below.
 *
 * Pipeline (ST_RAW):
 *   1. cost volume  C[y][x][d]: truncated colour + gradient cost   (StereoHelper.cpp:37-129)
 *   2. guide        3x3 median of the left BGR image (ctmf, r = 1)  (SegmentTree.cpp:183-194, Toolkit.cpp:33-48)
 *   3. tree         4-neighbour edges, Kruskal with Felzenszwalb's  (SegmentTree.cpp:38-139,
 *                   size threshold, then the rest of the MST with    segment-graph.h:48-101,
 *                   a cross-segment penalty; BFS order from pixel 0  disjoint-set.h:30-82)
 *   4. filter       leaf-to-root and root-to-leaf passes             (SegmentTree.cpp:141-181)
 *   5. WTA, 7x7 median (ctmf r = 3), x scale                         (StereoHelper.cpp:131-154, StereoDisparity.cpp:82-88)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ORA_API __attribute__((visibility("default")))

void ora_median_u8(const uint8_t *src, int W, int H, int r, uint8_t *dst);   /* bm_oracle.c (ctmf) */

/* rgb_2_gray, StereoHelper.cpp:37 (in = B, G, R) */
static uint8_t st_gray(const uint8_t *in) { return (uint8_t)(0.299 * in[2] + 0.587 * in[1] + 0.114 * in[0] + 0.5); }

/* GetGradient, StereoHelper.cpp:39-73 (W >= 2) */
static void st_gradient(const uint8_t *bgr, int W, int H, float *g)
{
    uint8_t *gray = (uint8_t *)malloc((size_t)W);
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W; ++x) gray[x] = st_gray(bgr + ((size_t)y * W + x) * 3);
        float *row = g + (size_t)y * W;
        float plus = gray[1], minus = gray[0];
        row[0] = plus - minus + 127.5f;
        for (int x = 1; x < W - 1; ++x) {
            plus = gray[x + 1];
            minus = gray[x - 1];
            row[x] = 0.5f * (plus - minus) + 127.5f;
        }
        plus = gray[W - 1];
        minus = gray[W - 2];
        row[W - 1] = plus - minus + 127.5f;
    }
    free(gray);
}

/* GetMatchingCost, StereoHelper.cpp:75-129: C[(y*W + x)*D + d]; right pixels left of column 0 repeat
 * column 0 (:107-110) */
ORA_API void ora_st_cost(const uint8_t *L, const uint8_t *R, int W, int H, int D, float *cost)
{
    float *gL = (float *)malloc((size_t)W * H * sizeof(float));
    float *gR = (float *)malloc((size_t)W * H * sizeof(float));
    st_gradient(L, W, H, gL);
    st_gradient(R, W, H, gR);
    const double max_color_difference = 7, max_gradient_difference = 2;
    const double weight_on_color = 0.11, weight_on_gradient = 1.0 - weight_on_color;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            for (int d = 0; d < D; ++d) {
                const int xs = x >= d ? x - d : 0;
                const uint8_t *l = L + ((size_t)y * W + x) * 3, *r = R + ((size_t)y * W + xs) * 3;
                double costColor = 0, costGradient;
                for (int c = 0; c < 3; ++c) costColor += abs(l[c] - r[c]);
                costColor = costColor / 3 < max_color_difference ? costColor / 3 : max_color_difference;
                costGradient = fabsf(gL[(size_t)y * W + x] - gR[(size_t)y * W + xs]);
                costGradient = costGradient < max_gradient_difference ? costGradient : max_gradient_difference;
                cost[((size_t)y * W + x) * D + d] = (float)(weight_on_color * costColor + weight_on_gradient * costGradient);
            }
    free(gL);
    free(gR);
}

/* ---- disjoint-set forest, disjoint-set.h:30-82 (union by rank; find compresses x only) ---- */
typedef struct { int rank, p, size; } st_elt;
static int st_find(st_elt *e, int x)
{
    int y = x;
    while (y != e[y].p) y = e[y].p;
    e[x].p = y;
    return y;
}
static void st_join(st_elt *e, int x, int y)
{
    if (x != e[x].p) x = st_find(e, x);
    if (y != e[y].p) y = st_find(e, y);
    if (x == y) return;
    if (e[x].rank > e[y].rank) {
        e[y].p = x;
        e[x].size += e[y].size;
    } else {
        e[x].p = y;
        e[y].size += e[x].size;
        if (e[x].rank == e[y].rank) e[y].rank++;
    }
}

typedef struct { float w; int a, b; } st_edge;
/* edge::operator<, SegmentTree.h:99-112: by weight, then b, then a */
static int st_edge_cmp(const void *pa, const void *pb)
{
    const st_edge *x = (const st_edge *)pa, *y = (const st_edge *)pb;
    if (x->w != y->w) return x->w < y->w ? -1 : 1;
    if (x->b != y->b) return x->b < y->b ? -1 : 1;
    return (x->a > y->a) - (x->a < y->a);
}

/* MeanFilter(img, img, 1) of a BGR image: ctmf r = 1 per channel (SegmentTree.cpp:185, :199) */
static uint8_t *st_guide(const uint8_t *bgr, int W, int H)
{
    const int P = W * H;
    uint8_t *ch = (uint8_t *)malloc((size_t)P), *med = (uint8_t *)malloc((size_t)P * 3), *tmp = (uint8_t *)malloc((size_t)P);
    for (int c = 0; c < 3; ++c) {
        for (int p = 0; p < P; ++p) ch[p] = bgr[(size_t)p * 3 + c];
        ora_median_u8(ch, W, H, 1, tmp);
        for (int p = 0; p < P; ++p) med[(size_t)p * 3 + c] = tmp[p];
    }
    free(ch);
    free(tmp);
    return med;
}

/* max channel |diff| of two guide pixels (CColorWeight::GetWeight, SegmentTree.cpp:189-194) */
static int st_color_diff(const uint8_t *med, int p, int q)
{
    int m = 0;
    for (int c = 0; c < 3; ++c) {
        const int v = abs(med[(size_t)p * 3 + c] - med[(size_t)q * 3 + c]);
        m = v > m ? v : m;
    }
    return m;
}

/* edges of SegmentTree.cpp:44-62 (right neighbour, then the one above).  disp == NULL: CColorWeight
 * (weight = max channel |diff|, :189-194); else CColorDepthWeight (:196-219): where both ends are in
 * `mask`, 0.5 * |disp diff| / level + 0.5 * colour / 255, else colour / 255 */
static st_edge *st_edges(const uint8_t *med, int W, int H, const uint8_t *disp, const uint8_t *mask, float level,
                         int *nE)
{
    st_edge *edges = (st_edge *)malloc(sizeof(st_edge) * (size_t)W * H * 2);
    int E = 0;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            const int p = y * W + x;
            for (int k = 0; k < 2; ++k) {
                int q;
                if (k == 0) {
                    if (x >= W - 1) continue;
                    q = p + 1;
                } else {
                    if (y < 1) continue;
                    q = p - W;
                }
                const int m = st_color_diff(med, p, q);
                float w;
                if (!disp) {
                    w = (float)m;
                } else if (mask[p] && mask[q]) {
                    const float dispValue = (float)abs(disp[p] - disp[q]) / level;
                    const float colorValue = (float)m / 255.0f;
                    w = 0.5f * dispValue + (1.0f - 0.5f) * colorValue;
                } else {
                    w = (float)m / 255.0f;
                }
                edges[E].a = p;
                edges[E].b = q;
                edges[E].w = w;
                ++E;
            }
        }
    *nE = E;
    return edges;
}

/* BuildSegmentTree (SegmentTree.cpp:38-139) from its edge list (consumed): segment_graph, the
 * node-based graph with dist = min(int(w * wscale + 0.5), 255) (wscale = GetScale(): 1 for
 * CColorWeight, 255 for CColorDepthWeight), BFS from pixel 0.  Outputs per BFS position i: node[i]
 * (pixel id), parent[i] (BFS position, -1 at the root), pdist[i] (edge distance to the parent),
 * first[i] / nchild[i] (children occupy BFS positions first .. first + nchild - 1) and cdist[4 * i + k].
 * Returns the number of BFS levels (-1 if the tree does not span the image). */
static int st_tree_from_edges(st_edge *edges, int E, int P, float tau, float wscale, int *node, int *parent,
                              uint8_t *pdist, int *first, uint8_t *nchild, uint8_t *cdist)
{
    /* segment_graph, segment-graph.h:48-101 */
    qsort(edges, (size_t)E, sizeof(st_edge), st_edge_cmp);
    st_elt *u = (st_elt *)malloc(sizeof(st_elt) * (size_t)P);
    for (int i = 0; i < P; ++i) u[i] = (st_elt){0, i, 1};
    float *thr = (float *)malloc(sizeof(float) * (size_t)P);
    for (int i = 0; i < P; ++i) thr[i] = tau / 1;
    uint8_t *mask = (uint8_t *)calloc((size_t)E, 1);
    for (int i = 0; i < E; ++i) {
        int a = st_find(u, edges[i].a), b = st_find(u, edges[i].b);
        if (a != b && edges[i].w <= thr[a] && edges[i].w <= thr[b]) {
            mask[i] = 255;
            st_join(u, a, b);
            a = st_find(u, a);
            thr[a] = edges[i].w + tau / u[a].size;
        }
    }
    for (int i = 0; i < E; ++i) {
        const int a = st_find(u, edges[i].a), b = st_find(u, edges[i].b);
        if (a != b) {
            const int size_min = u[a].size < u[b].size ? u[a].size : u[b].size;
            st_join(u, a, b);
            mask[i] = 255;
            if (size_min > 50) edges[i].w += 5;   /* MIN_SIZE_SEG, PENALTY_CROSS_SEG */
        }
    }
    free(thr);
    free(u);
    /* node-based graph, SegmentTree.cpp:71-95: neighbours in sorted-edge order */
    int *adj = (int *)malloc(sizeof(int) * (size_t)P * 4);
    uint8_t *adjd = (uint8_t *)malloc((size_t)P * 4), *na = (uint8_t *)calloc((size_t)P, 1);
    for (int i = 0; i < E; ++i) {
        if (!mask[i]) continue;
        const int pa = edges[i].a, pb = edges[i].b;
        int dis = (int)(edges[i].w * wscale + 0.5f);
        dis = dis < 255 ? dis : 255;
        adj[pa * 4 + na[pa]] = pb;
        adjd[pa * 4 + na[pa]++] = (uint8_t)dis;
        adj[pb * 4 + na[pb]] = pa;
        adjd[pb * 4 + na[pb]++] = (uint8_t)dis;
    }
    free(mask);
    /* BFS from pixel 0, SegmentTree.cpp:97-130 */
    uint8_t *vis = (uint8_t *)calloc((size_t)P, 1);
    int *level = (int *)malloc(sizeof(int) * (size_t)P);
    node[0] = 0;
    parent[0] = -1;
    pdist[0] = 0;
    level[0] = 0;
    vis[0] = 1;
    int start = 0, end = 1, levels = 1;
    while (start < end) {
        const int i = start++, p = node[i];
        first[i] = end;
        nchild[i] = 0;
        for (int k = 0; k < na[p]; ++k) {
            const int q = adj[p * 4 + k];
            if (vis[q]) continue;   /* the father (a tree has no other visited neighbour) */
            vis[q] = 1;
            cdist[4 * i + nchild[i]] = adjd[p * 4 + k];
            nchild[i]++;
            node[end] = q;
            parent[end] = i;
            pdist[end] = adjd[p * 4 + k];
            level[end] = level[i] + 1;
            if (level[end] + 1 > levels) levels = level[end] + 1;
            ++end;
        }
    }
    free(level);
    free(vis);
    free(adj);
    free(adjd);
    free(na);
    return end == P ? levels : -1;
}

/* BuildSegmentTree with CColorWeight on `bgr` (SegmentTree.cpp:38-139, :183-194) */
ORA_API int ora_st_tree(const uint8_t *bgr, int W, int H, float tau, int *node, int *parent, uint8_t *pdist,
                        int *first, uint8_t *nchild, uint8_t *cdist)
{
    uint8_t *med = st_guide(bgr, W, H);
    int E;
    st_edge *edges = st_edges(med, W, H, NULL, NULL, 0.f, &E);
    free(med);
    const int levels = st_tree_from_edges(edges, E, W * H, tau, 1.0f, node, parent, pdist, first, nchild, cdist);
    free(edges);
    return levels;
}

/* BuildSegmentTree with CColorDepthWeight(img, disp, mask, maxLevel) (SegmentTree.cpp:196-219, scale 255) */
ORA_API int ora_st_tree_depth(const uint8_t *bgr, const uint8_t *disp, const uint8_t *mask, int W, int H, int level,
                              float tau, int *node, int *parent, uint8_t *pdist, int *first, uint8_t *nchild,
                              uint8_t *cdist)
{
    uint8_t *med = st_guide(bgr, W, H);
    int E;
    st_edge *edges = st_edges(med, W, H, disp, mask, (float)level, &E);
    free(med);
    const int levels = st_tree_from_edges(edges, E, W * H, tau, 255.0f, node, parent, pdist, first, nchild, cdist);
    free(edges);
    return levels;
}

/* Filter, SegmentTree.cpp:141-181, on the pixel-major volume cost[p * D + d] (in place) */
ORA_API void ora_st_filter(const int *node, const int *parent, const uint8_t *pdist, const int *first,
                           const uint8_t *nchild, const uint8_t *cdist, int P, int D, float sigma, float *cost)
{
    float table[256];
    sigma = sigma > 0.01f ? sigma : 0.01f;
    for (int i = 0; i <= 255; ++i) table[i] = expf(-(float)i / (255 * sigma));
    float *buf = (float *)malloc(sizeof(float) * (size_t)P * D);
    memcpy(buf, cost, sizeof(float) * (size_t)P * D);
    for (int i = P - 1; i >= 0; --i) {   /* leaf to root */
        float *c = buf + (size_t)node[i] * D;
        for (int z = 0; z < nchild[i]; ++z) {
            const float *cc = buf + (size_t)node[first[i] + z] * D;
            const float w = table[cdist[4 * i + z]];
            for (int k = 0; k < D; ++k) c[k] += cc[k] * w;
        }
    }
    memcpy(cost + (size_t)node[0] * D, buf + (size_t)node[0] * D, sizeof(float) * D);
    for (int i = 1; i < P; ++i) {       /* root to leaf */
        float *f = cost + (size_t)node[i] * D;
        const float *cur = buf + (size_t)node[i] * D, *fa = cost + (size_t)node[parent[i]] * D;
        const float w = table[pdist[i]];
        for (int k = 0; k < D; ++k) f[k] = w * (fa[k] - w * cur[k]) + cur[k];
    }
    free(buf);
}

typedef struct {
    int *node, *parent, *first;
    uint8_t *pdist, *nchild, *cdist;
} st_tree_buf;

static void st_tree_alloc(st_tree_buf *t, int P)
{
    t->node = (int *)malloc(sizeof(int) * (size_t)P);
    t->parent = (int *)malloc(sizeof(int) * (size_t)P);
    t->first = (int *)malloc(sizeof(int) * (size_t)P);
    t->pdist = (uint8_t *)malloc((size_t)P);
    t->nchild = (uint8_t *)malloc((size_t)P);
    t->cdist = (uint8_t *)calloc((size_t)P * 4, 1);
}

static void st_tree_free(st_tree_buf *t)
{
    free(t->node);
    free(t->parent);
    free(t->first);
    free(t->pdist);
    free(t->nchild);
    free(t->cdist);
}

/* GetDisparity_WTA (StereoHelper.cpp:131-154): strict < from d = 0, pixel-major cost */
static void st_wta(const float *cost, int P, int D, uint8_t *disp)
{
    for (int p = 0; p < P; ++p) {
        const float *c = cost + (size_t)p * D;
        int m = 0;
        float v = c[0];
        for (int d = 1; d < D; ++d)
            if (c[d] < v) {
                v = c[d];
                m = d;
            }
        disp[p] = (uint8_t)m;
    }
}

/* filter `cost` on `t`, WTA, 7x7 median (MeanFilter r = 3) into out */
static void st_aggregate(const st_tree_buf *t, int W, int H, int D, float sigma, float *cost, uint8_t *out)
{
    const int P = W * H;
    ora_st_filter(t->node, t->parent, t->pdist, t->first, t->nchild, t->cdist, P, D, sigma, cost);
    uint8_t *disp = (uint8_t *)malloc((size_t)P);
    st_wta(cost, P, D, disp);
    ora_median_u8(disp, W, H, 3, out);
    free(disp);
}

static void st_scale(uint8_t *m, int P, int scale)
{
    for (int p = 0; p < P; ++p) {
        const int v = m[p] * scale;
        m[p] = (uint8_t)(v > 255 ? 255 : v);
    }
}

/* stereo_disparity_normal (StereoDisparity.cpp:57-89): cost, tree on the left view, filter, float WTA
 * (strict < from d = 0, StereoHelper.cpp:131-154), 7x7 median (MeanFilter r = 3), x scale (saturated).
 * Returns the tree's BFS level count (-1 if the tree does not span the image). */
ORA_API int ora_st_disp(const uint8_t *Lbgr, const uint8_t *Rbgr, int W, int H, int D, int scale, float sigma,
                        float tau, uint8_t *out)
{
    const int P = W * H;
    float *cost = (float *)malloc(sizeof(float) * (size_t)P * D);
    ora_st_cost(Lbgr, Rbgr, W, H, D, cost);
    st_tree_buf t;
    st_tree_alloc(&t, P);
    const int levels = ora_st_tree(Lbgr, W, H, tau, t.node, t.parent, t.pdist, t.first, t.nchild, t.cdist);
    if (levels > 0) {
        st_aggregate(&t, W, H, D, sigma, cost, out);
        st_scale(out, P, scale);
    }
    st_tree_free(&t);
    free(cost);
    return levels;
}

/* GetRightMatchingCostFromLeft (StereoHelper.cpp:156-180), pixel-major: the right view's cost at
 * (y, x, d) is the left view's at (y, x + d, d); where x + d >= W it repeats d - 1's.
 * W < D (max_level wider than the frame): the reference's second loop starts at x = w - maxLevel
 * (StereoHelper.cpp:168), a negative column, so it writes into row y - 1 and, for y = 0, before the
 * buffer: undefined behaviour with no defined output.  This port clamps the start to x = 0, the
 * in-bounds reading (every pixel then takes the per-pixel rule above); results for W < D are
 * therefore PARITY UNPINNED, a defined extension, not reference behaviour. */
ORA_API void ora_st_right_cost(const float *left, int W, int H, int D, float *right)
{
    memcpy(right, left, sizeof(float) * (size_t)W * H * D);
    for (int y = 0; y < H; ++y) {
        for (int x = 0; x < W - D; ++x)
            for (int d = 0; d < D; ++d)
                right[((size_t)y * W + x) * D + d] = left[((size_t)y * W + x + d) * D + d];
        for (int x = W - D > 0 ? W - D : 0; x < W; ++x)
            for (int d = 0; d < D; ++d) {
                if (x + d < W) right[((size_t)y * W + x) * D + d] = left[((size_t)y * W + x + d) * D + d];
                else right[((size_t)y * W + x) * D + d] = right[((size_t)y * W + x) * D + d - 1];
            }
    }
}

/* stereo_disparity_iteration, ST-2 (StereoDisparity.cpp:91-160):
 *   left / right maps on CColorWeight trees of each view with sigma = SIGMA_ONE (0.08, Toolkit.h:35), the
 *   right cost taken from the left's (GetRightMatchingCostFromLeft), each WTA + 7x7 median;
 *   the left-right check (:129-147): mask = !(x - d < 0 || d == 0 || |d - dR(x - d)| > 1);
 *   a CColorDepthWeight tree on the left view, the filtered left map and the mask, with `sigma`; its
 *   WTA + 7x7 median, x scale.
 * Optional outputs (NULL to skip): the first-pass left / right maps and the mask.  Returns the last
 * tree's BFS level count (-1 if a tree does not span the image). */
ORA_API int ora_st2_disp(const uint8_t *Lbgr, const uint8_t *Rbgr, int W, int H, int D, int scale, float sigma,
                         float tau, uint8_t *out, uint8_t *left1, uint8_t *right1, uint8_t *mask_out)
{
    const int P = W * H;
    const float sigma_one = 0.08f;
    float *costL = (float *)malloc(sizeof(float) * (size_t)P * D);
    float *costR = (float *)malloc(sizeof(float) * (size_t)P * D);
    float *cost2 = (float *)malloc(sizeof(float) * (size_t)P * D);
    ora_st_cost(Lbgr, Rbgr, W, H, D, costL);
    ora_st_right_cost(costL, W, H, D, costR);
    memcpy(cost2, costL, sizeof(float) * (size_t)P * D);   /* the reference recomputes the same volume (:150) */
    uint8_t *dL = (uint8_t *)malloc((size_t)P), *dR = (uint8_t *)malloc((size_t)P), *mask = (uint8_t *)malloc((size_t)P);
    st_tree_buf t;
    st_tree_alloc(&t, P);
    int levels = ora_st_tree(Lbgr, W, H, tau, t.node, t.parent, t.pdist, t.first, t.nchild, t.cdist);
    if (levels > 0) {
        st_aggregate(&t, W, H, D, sigma_one, costL, dL);
        levels = ora_st_tree(Rbgr, W, H, tau, t.node, t.parent, t.pdist, t.first, t.nchild, t.cdist);
    }
    if (levels > 0) {
        st_aggregate(&t, W, H, D, sigma_one, costR, dR);
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                const int d = dL[y * W + x];
                int occ = 1;
                if (x - d >= 0) {
                    const int dc = dR[y * W + x - d];
                    occ = (d == 0 || abs(d - dc) > 1);
                }
                mask[y * W + x] = (uint8_t)!occ;
            }
        levels = ora_st_tree_depth(Lbgr, dL, mask, W, H, D, tau, t.node, t.parent, t.pdist, t.first, t.nchild,
                                   t.cdist);
    }
    if (levels > 0) {
        st_aggregate(&t, W, H, D, sigma, cost2, out);
        st_scale(out, P, scale);
        if (left1) memcpy(left1, dL, (size_t)P);
        if (right1) memcpy(right1, dR, (size_t)P);
        if (mask_out) memcpy(mask_out, mask, (size_t)P);
    }
    st_tree_free(&t);
    free(dL);
    free(dR);
    free(mask);
    free(costL);
    free(costR);
    free(cost2);
    return levels;
}
