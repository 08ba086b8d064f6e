"""Synthetic stand-ins for the citation datasets the reference's examples load
(``dgl.data.load_data``, network downloads): a planted-partition graph with
Cora's sizes (2708 nodes, 10556 edges + self-loops, 1433 features, 7 classes)
whose labels are learnable from structure and features, and the usual
train / val / test masks."""
import numpy as np
import torch as th


def planted_cora(seed=0, n=2708, m=10556, feats=1433, classes=7, p_in=0.9, signal=0.5):
    rs = np.random.RandomState(seed)
    labels = rs.randint(0, classes, n)
    by_class = [np.nonzero(labels == c)[0] for c in range(classes)]
    src = rs.randint(0, n, m)
    same = rs.rand(m) < p_in
    dst = np.where(same, [rs.choice(by_class[labels[s]]) for s in src], rs.randint(0, n, m))
    x = (rs.rand(n, feats) < 0.01).astype(np.float32)
    centers = rs.randn(classes, feats).astype(np.float32) * signal / np.sqrt(feats) * 10
    x += centers[labels]
    idx = rs.permutation(n)
    train, val, test = idx[:140], idx[140:640], idx[1708:2708]
    masks = []
    for sel in (train, val, test):
        mk = np.zeros(n, bool)
        mk[sel] = True
        masks.append(th.from_numpy(mk))
    return src, dst, n, th.from_numpy(x), th.from_numpy(labels), masks
