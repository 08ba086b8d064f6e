"""Times the MFMA projection (DGLMIProject: k_project / k_project_tile) against
torch.matmul (hipBLASLt) on the bracketing GEMM shapes of the configs, HIP events on the
launch stream, and reports TFLOP/s and the fraction of the 157.3 TF fp32 MFMA peak
(MI355X_MICROARCH.md).  Shapes (M, K -> N, weight layout):
  C3 fwd  232965 x 602 -> 64   W = fc.weight.t()   (gatconv.py:127-132)
  C3 dX   232965 x 64 -> 602   W = fc.weight
  C5 fwd  5000000 x 64 -> 256  (R-GCN relation-major Y = X [W_0..W_3])
  C5 dX   5000000 x 256 -> 64
  C2 fwd  169343 x 128 -> 128  k_project and, with DGLMI_PROJECT_TILE=1, k_project_tile
Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "dgl-hack_amd"))
import torch as th  # noqa: E402

from dgl import kernel as K  # noqa: E402

PEAK_TF = 157.3
# k_project_tile instances A/B'd per shape (kernels_project.hip kTileCfgs indices)
CFGS = {"c3_fwd": (8, 10), "c5_dx": (6, 9), "c3_dx": (3, 11), "c5_fwd": (2,)}


def timeit(fn, reps=20):
    for _ in range(5):
        fn()
    th.cuda.synchronize()
    s, e = th.cuda.Event(enable_timing=True), th.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    th.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    dev = th.device("cuda", 0)
    g = th.Generator(device=dev).manual_seed(0)
    shapes = [("c3_fwd", 232965, 602, 64, "t"), ("c3_dx", 232965, 64, 602, "n"),
              ("c5_fwd", 5000000, 64, 256, "n"), ("c5_dx", 5000000, 256, 64, "t"),
              ("c2_fwd", 169343, 128, 128, "t")]
    out = {}
    for name, m, k, n, lay in shapes:
        x = th.randn(m, k, device=dev, generator=g)
        w = th.randn(n, k, device=dev, generator=g).t() if lay == "t" else \
            th.randn(k, n, device=dev, generator=g)
        flops = 2.0 * m * k * n
        rec = {"m": m, "k": k, "n": n}
        ref = x.double()[:4096] @ w.double()
        variants = [("mfma", "0", None)]
        if name == "c2_fwd":
            variants.append(("mfma_tile", "1", None))
        for cfg in CFGS.get(name, ()):
            variants.append(("mfma_cfg%d" % cfg, "0", str(cfg)))
            if k % 4:
                variants.append(("mfma_cfg%d_regstage" % cfg, "0", str(cfg)))
        for label, env, cfg in variants:
            os.environ["DGLMI_PROJECT_GLDS"] = "0" if label.endswith("_regstage") else "1"
            os.environ["DGLMI_PROJECT_TILE"] = env
            if cfg is None:
                os.environ.pop("DGLMI_PROJECT_CFG", None)
            else:
                os.environ["DGLMI_PROJECT_CFG"] = cfg
            ms = timeit(lambda: K.project_mfma(x, w))
            y = K.project_mfma(x, w)
            err = float(((y[:4096].double() - ref).abs() / (x.double()[:4096].abs() @ w.double().abs() + 1e-30)).max())
            rec[label] = {"ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1),
                          "frac_peak": round(flops / ms / 1e9 / PEAK_TF, 3), "rel_err": err}
        os.environ["DGLMI_PROJECT_TILE"] = "0"
        os.environ.pop("DGLMI_PROJECT_CFG", None)
        ms = timeit(lambda: th.matmul(x, w))
        rec["torch_matmul"] = {"ms": round(ms, 4), "tflops": round(flops / ms / 1e9, 1),
                               "frac_peak": round(flops / ms / 1e9 / PEAK_TF, 3)}
        out[name] = rec
        del x, w
        th.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
