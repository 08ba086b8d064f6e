"""Seeded synthetic power-law edge lists for the benchmark configs (the real datasets
need network downloads).

``chung_lu_edges`` draws the same edges on every process and every run for a seed:
multi-rank jobs build the graph independently on each rank and must agree on it
(``th.multinomial`` on the device gave a different draw per call for the same
generator state, so ranks disagreed on the C5 partition).  The weights' prefix sum is
formed on the host in fp64; the device draws uniforms from a seeded generator and
inverts the CDF with a binary search -- both order-independent."""
import torch as th

__all__ = ["chung_lu_edges"]


def chung_lu_edges(n, m, alpha, seed, device):
    """(src, dst) int32 device tensors of ``m`` edges over ``n`` nodes; each end drawn
    independently with probability proportional to w_i = rank_i^-alpha, ranks
    permuted by ``seed`` (Chung-Lu, in-/out-degrees ~ power law)."""
    gc = th.Generator().manual_seed(int(seed))
    w = th.arange(1, n + 1, dtype=th.float64).pow(-float(alpha))
    w = w[th.randperm(n, generator=gc)]
    cdf = th.cumsum(w, 0)
    cdf /= cdf[-1].item()
    cdf = cdf.to(device)
    g = th.Generator(device=device)
    g.manual_seed(int(seed))
    ends = []
    for _ in range(2):
        u = th.rand(m, generator=g, device=device, dtype=th.float64)
        ends.append(th.searchsorted(cdf, u, right=True).clamp_(max=n - 1).to(th.int32))
        del u
    return ends[0], ends[1]
