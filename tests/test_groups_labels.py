"""CPU check of the identity the device filterSmallGroups relies on (pmvs_filter.hip, filter_pass):
the reference's labelling -- a BFS from every unlabelled patch in collect order over DIRECTED
neighbour edges (filter.cpp:520-562) -- gives patch j the smallest index from which j is
reachable.  Checked on random directed graphs against the fixpoint the device computes
(lab[j] = min over edges i -> j of lab[i], with pointer jumping lab[j] = lab[lab[j]])."""
from collections import deque

import numpy as np


def bfs_labels(n, adj):
    lab = [-1] * n
    nid = -1
    root = []
    for pid in range(n):
        if lab[pid] != -1:
            continue
        nid += 1
        root.append(pid)
        lab[pid] = nid
        q = deque([pid])
        while q:
            u = q.popleft()
            for v in adj[u]:
                if lab[v] == -1:
                    lab[v] = nid
                    q.append(v)
    return [root[x] for x in lab]  # label as the root's index


def fixpoint_labels(n, adj):
    lab = list(range(n))
    changed = True
    while changed:
        changed = False
        for u in range(n):
            for v in adj[u]:
                if lab[u] < lab[v]:
                    lab[v] = lab[u]
                    changed = True
        for u in range(n):
            if lab[lab[u]] < lab[u]:
                lab[u] = lab[lab[u]]
                changed = True
    return lab


def test_bfs_labels_are_min_reachable_index():
    rng = np.random.default_rng(7)
    for trial in range(300):
        n = int(rng.integers(1, 60))
        p = float(rng.uniform(0.0, 0.12))
        adj = [[int(v) for v in np.nonzero(rng.random(n) < p)[0] if v != u] for u in range(n)]
        a, b = bfs_labels(n, adj), fixpoint_labels(n, adj)
        assert a == b, (trial, n)
        sizes_a = np.bincount(a, minlength=n)
        assert (sizes_a[a] == np.bincount(b, minlength=n)[b]).all()
