"""TEST INFRASTRUCTURE: numpy restatement of the device label-propagation
partitioner (``dgl-hack_amd/csrc/partition.hip``, ``DGLMIPartitionLabelProp``),
round by round with the same counter-based hashes, so the GPU labels can be
checked bit-exactly.  The reference itself partitions with METIS
(``src/graph/metis_partition.cc:19-66``), which is absent here; this pins our
own replacement, not the reference."""
import numpy as np

M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def admit_hash(v, rnd, seed):
    inner = splitmix(np.uint64(seed) ^ (np.uint64(1) << np.uint64(56)))
    h = splitmix(inner ^ (np.uint64(rnd) << np.uint64(40)) ^ np.asarray(v, np.uint64))
    return (h >> np.uint64(32)).astype(np.int64)


def _cut(hist, room):
    """bins admitted whole, room left for the straddling bin (k_admit_cut)."""
    b = 0
    while b < 256:
        if hist[b] > room:
            break
        room -= hist[b]
        b += 1
    return b, room


def labelprop(n, src, dst, k, rounds, slack, weight, seed, init):
    """Labels after `rounds` rounds (int32), loads (int64), cut edges."""
    src = np.asarray(src, np.int64)
    dst = np.asarray(dst, np.int64)
    lab = np.asarray(init, np.int64).copy()
    w = np.ones(n, np.int64) if weight is None else np.asarray(weight, np.int64)
    load = np.bincount(lab, weights=w, minlength=k).astype(np.int64)
    total = int(load.sum())
    cap = int((1.0 + slack) * float(total) / k) + 1
    nonself = src != dst
    s, d = src[nonself], dst[nonself]
    v_all = np.arange(n, dtype=np.int64)
    for r in range(rounds if k > 1 else 0):
        hist = np.bincount(d * k + lab[s], minlength=n * k) + np.bincount(s * k + lab[d], minlength=n * k)
        hist = hist.reshape(n, k)
        half = (splitmix(np.uint64(seed) ^ v_all.astype(np.uint64) ^
                         (np.uint64(r) << np.uint64(48))) & np.uint64(1)) == 0
        want = np.full(n, -1, np.int64)
        for v in range(n):
            cur = lab[v]
            best = cur
            hv = hist[v]
            for p in range(k):
                if p == best:
                    continue
                c, cb = hv[p], hv[best]
                if c > cb or (c == cb and best != cur and
                              (load[p] < load[best] or (load[p] == load[best] and p < best))):
                    best = p
            if best != cur and hv[best] > hv[cur] and half[v]:
                want[v] = best
        h = admit_hash(v_all, r, seed)
        ba, bb = h >> 24, (h >> 16) & 255
        cand = want >= 0
        hist_a = np.zeros((k, 256), np.int64)
        np.add.at(hist_a, (want[cand], ba[cand]), w[cand])
        cut_a, rem_a = zip(*[_cut(hist_a[p], cap - load[p]) for p in range(k)])
        hist_b = np.zeros((k, 256), np.int64)
        sel = cand & (ba == np.array(cut_a + (0,))[np.where(cand, want, k)])
        np.add.at(hist_b, (want[sel], bb[sel]), w[sel])
        cut_b = [256 if cut_a[p] >= 256 else _cut(hist_b[p], rem_a[p])[0] for p in range(k)]
        delta = np.zeros(k, np.int64)
        for v in np.nonzero(cand)[0]:
            p = want[v]
            if not (ba[v] < cut_a[p] or (ba[v] == cut_a[p] and bb[v] < cut_b[p])):
                continue
            delta[lab[v]] -= w[v]
            delta[p] += w[v]
            lab[v] = p
        load += delta
    cut = int((lab[src] != lab[dst]).sum())
    return lab.astype(np.int32), load, cut
