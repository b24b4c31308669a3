"""The device BFS's algorithm (csrc/bm_segtree.hip, gpu_bfs) restated in plain Python and checked
against a FIFO BFS (SegmentTree.cpp:97-130's order: from pixel 0, a node's children in neighbour-list
order) on random spanning trees of small grids.  It pins the math the kernels implement: the Euler tour
built from the lists, ranking it roots the tree (parent = the neighbour whose arc comes first, subtree
size from the gap), the tour's prefix sums of {+-1, +-preorder offset} give depth and preorder, and the
preorder stably sorted by depth is the BFS order.  The kernels themselves are compared with the host
BFS on the GPU (tests/test_gpu_segtree.py::test_device_bfs_equals_host_bfs)."""
import random
from collections import deque

import pytest


def _random_tree(W, H, rng):
    P = W * H
    edges = [(p, p + 1) for p in range(P) if p % W + 1 < W] + [(p, p + W) for p in range(P - W)]
    rng.shuffle(edges)
    par = list(range(P))

    def find(x):
        while par[x] != x:
            par[x] = par[par[x]]
            x = par[x]
        return x

    adj = [[] for _ in range(P)]   # (neighbour, distance byte) in the order the edges joined
    for a, b in edges:
        ra, rb = find(a), find(b)
        if ra != rb:
            par[ra] = rb
            d = rng.randrange(256)
            adj[a].append((b, d))
            adj[b].append((a, d))
    return adj


def _fifo_bfs(adj):
    order, parent = [0], {0: -1}
    q = deque([0])
    while q:
        p = q.popleft()
        for c, _ in adj[p]:
            if c == parent[p]:
                continue
            parent[c] = p
            order.append(c)
            q.append(c)
    return order


def _tour_bfs(adj):
    P = len(adj)
    L = 2 * (P - 1)
    # slot of p in the list of its k-th neighbour q: arc p -> q reversed
    back = {(p, k): next(z for z, (r, _) in enumerate(adj[q]) if r == p)
            for p in range(P) for k, (q, _) in enumerate(adj[p])}
    nxt = {}
    for (p, k), j in back.items():
        q = adj[p][k][0]
        arc = (q, (j + 1) % len(adj[q]))
        nxt[(p, k)] = None if arc == (0, 0) else arc        # the arc into the start arc ends the tour
    dist = {}
    for a in nxt:                                            # the ranks pointer jumping computes
        c, b = 0, a
        while nxt[b] is not None:
            b, c = nxt[b], c + 1
        dist[a] = c
    psl, size = {0: None}, {0: P}
    for p in range(1, P):
        for k, (q, _) in enumerate(adj[p]):
            da, db = dist[(p, k)], dist[(q, back[(p, k)])]
            if db > da:
                psl[p], size[p] = k, (db - da + 1) // 2
    offs = [0] * P
    for p in range(P):
        run = 1
        for k, (c, _) in enumerate(adj[p]):
            if k != psl[p]:
                offs[c], run = run, run + size[c]
    tw, tv = [None] * L, [None] * L
    for p in range(P):
        for k, (q, _) in enumerate(adj[p]):
            pos = L - 1 - dist[(p, k)]
            tw[pos], tv[pos] = ((-1, -offs[p]), -1) if k == psl[p] else ((1, offs[q]), q)
    keys, vals = [0] * P, [0] * P
    dep = pre = 0
    for pos in range(L):
        dep, pre = dep + tw[pos][0], pre + tw[pos][1]
        if tv[pos] >= 0:
            keys[pre], vals[pre] = dep, tv[pos]
    return [vals[i] for i in sorted(range(P), key=lambda i: (keys[i], i))]


@pytest.mark.parametrize("W,H", [(2, 1), (2, 2), (3, 5), (7, 4), (1, 9), (13, 11), (30, 20)])
def test_tour_order_is_fifo_bfs(W, H):
    rng = random.Random(W * 1000 + H)
    for _ in range(10):
        adj = _random_tree(W, H, rng)
        assert _tour_bfs(adj) == _fifo_bfs(adj)
