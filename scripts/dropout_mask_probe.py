"""Where the C3 training step with GATConv's own attention-dropout mask spends its time:
each step of the mask preparation (ones, nn.Dropout, DGLMIGatKeepBits) and the fused
forward / backward with the module's mask against the hashed one, HIP events.  Prints one
JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dgl-hack_amd"))
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import torch as th  # noqa: E402

from bench_configs import chung_lu, timeit  # noqa: E402


def main():
    dev = th.device("cuda", 0)
    from dgl import backend as B
    from dgl import kernel as K
    n, m = 232965, 114615892
    g = chung_lu(n, m, 0.4, 3, dev)
    gidx = g._graph.get_immutable_gidx(dev)
    H, D, p = 8, 8, 0.6
    drop = th.nn.Dropout(p)
    ones = th.ones(m, H, 1, device=dev)
    res = {"edges": m, "heads": H, "p": p}
    res["ones_ms"] = timeit(lambda: th.ones(m, H, 1, device=dev), 10, 2)
    res["nn_dropout_ms"] = timeit(lambda: drop(ones), 10, 2)
    t = drop(ones)
    res["native_dropout_ms"] = timeit(lambda: th.native_dropout(ones, p, True), 10, 2)
    res["keep_bits_ms"] = timeit(lambda: K.gat_keep_bits(t), 10, 2)
    keep = K.gat_keep_bits(t)
    scale = 1.0 / (1.0 - p)
    ft = th.randn(n, H, D, device=dev, requires_grad=True)
    el = th.randn(n, H, 1, device=dev, requires_grad=True)
    er = th.randn(n, H, 1, device=dev, requires_grad=True)
    go = th.randn(n, H, D, device=dev)

    def run(**kw):
        out = B.fused_gat(g, ft, el, er, 0.2, **kw)
        th.autograd.grad(out, (ft, el, er), go)
    for order in ("pos,pos", "eid,eid", "eid,pos", "pos,eid"):
        os.environ["DGLMI_GAT_KEEP_ORDER"] = order
        res["fused_fwd_bwd_keep_%s_ms" % order.replace(",", "_")] = timeit(
            lambda: run(keep=keep, keep_scale=scale), 10, 2)
    os.environ.pop("DGLMI_GAT_KEEP_ORDER")
    res["keep_gather_in_ms"] = timeit(lambda: K.gat_keep_walk_order(gidx, keep, ft, "in"), 10, 2)
    res["keep_gather_out_ms"] = timeit(lambda: K.gat_keep_walk_order(gidx, keep, ft, "out"), 10, 2)
    res["fused_fwd_bwd_keep_ms"] = timeit(lambda: run(keep=keep, keep_scale=scale), 10, 2)
    res["fused_fwd_bwd_hashed_ms"] = timeit(lambda: run(attn_drop=p, seed=7), 10, 2)
    res["fused_fwd_bwd_nodrop_ms"] = timeit(lambda: run(), 10, 2)
    with th.no_grad():
        res["fused_fwd_keep_ms"] = timeit(lambda: B.fused_gat(g, ft, el, er, 0.2, keep=keep, keep_scale=scale), 10, 2)
        res["fused_fwd_hashed_ms"] = timeit(lambda: B.fused_gat(g, ft, el, er, 0.2, attn_drop=p, seed=7), 10, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
