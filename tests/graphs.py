"""Test graphs and features, restated from the reference's tests.

* g20: the hand-built 20-node graph of tests/compute/test_kernel.py:338-351
  (self-loops, hubs 0/1 -> 2..17 -> 18/19, back-edges 18/19 -> 0/1).
* features: np.random.seed(31) uniform(-1, 1) with shapes (N, 5, 3, 4) /
  (N, 5, 3, 4, 10) for dot and the broadcast variants of
  test_kernel.py:33-74, value ranges adjusted for div/add/sub (:204-223).
* powerlaw: a Chung-Lu style skewed graph (heavy in-degree hubs) for the
  load-balanced kernels.
"""
import numpy as np

D1, D2, D3, D4 = 5, 3, 4, 10
CODE = {"u": 0, "v": 1, "e": 2}


def g20():
    src, dst = [], []
    for i in range(20):
        src.append(i)
        dst.append(i)
    for i in range(2, 18):
        src += [0, 1, i, i]
        dst += [i, i, 18, 19]
    src += [18, 18, 19, 19]
    dst += [0, 1, 0, 1]
    return np.array(src, np.int64), np.array(dst, np.int64), 20


def er_graph(n=100, p=0.1, seed=0, self_loops=True):
    rng = np.random.default_rng(seed)
    a = rng.random((n, n)) < p
    np.fill_diagonal(a, False)
    u, v = np.nonzero(a)
    if self_loops:
        u = np.concatenate([u, np.arange(n)])
        v = np.concatenate([v, np.arange(n)])
    return u.astype(np.int64), v.astype(np.int64), n


def powerlaw(n, m, seed=0, alpha=1.1, zero_frac=0.2):
    """Skewed in-degrees (a few hubs with thousands of in-edges), some empty rows."""
    rng = np.random.default_rng(seed)
    w = (np.arange(1, n + 1, dtype=np.float64)) ** (-alpha)
    w[rng.random(n) < zero_frac] = 0.0
    w /= w.sum()
    perm = rng.permutation(n)
    dst = perm[rng.choice(n, size=m, p=w)]
    src = rng.integers(0, n, m)
    return src.astype(np.int64), dst.astype(np.int64), n


def features(n_nodes, n_edges, broadcast="none", op="none"):
    np.random.seed(31)
    if op == "dot":
        full, small = (D1, D2, D3, D4), (D2, 1, D4)
    else:
        full, small = (D1, D2, D3), (D2, 1)
    u = np.random.uniform(-1, 1, (n_nodes,) + (small if broadcast == "u" else full))
    e = np.random.uniform(-1, 1, (n_edges,) + (small if broadcast == "e" else full))
    v = np.random.uniform(-1, 1, (n_nodes,) + (small if broadcast == "v" else full))
    return u, v, e


def binary_case_features(n, m, lhs, rhs, op, broadcast):
    u, v, e = features(n, m, broadcast, op)
    if op == "div":
        if rhs == "u":
            u = (u + 3) / 2
        elif rhs == "v":
            v = (v + 3) / 2
        elif rhs == "e":
            e = (e + 3) / 2
    if op in ("add", "sub"):
        u, v, e = u / 2, v / 2, e / 2
    return {"u": u.astype(np.float32), "v": v.astype(np.float32), "e": e.astype(np.float32)}
