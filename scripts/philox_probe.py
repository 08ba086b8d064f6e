"""Which element -> Philox draw mapping does torch.native_dropout use on this build?

Builds nothing: loads scripts/philox_probe.so (hipcc --offload-arch=gfx950 -shared -fPIC
scripts/philox_probe.hip -o scripts/philox_probe.so) and compares, for several shapes,
seeds and generator offsets, torch's mask with the probe's candidate mappings under the
launch geometry torch's fused dropout computes (256-thread blocks, grid capped at
CUs x maxThreadsPerCU / 256; the generator offset advanced by the draws per thread).

    python scripts/philox_probe.py
"""
import ctypes
import json
import os

import torch as th

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "philox_probe.so"))
    lib.philox_probe.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint64,
                                 ctypes.c_float, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    dev = th.device("cuda:0")
    props = th.cuda.get_device_properties(dev)
    cus, mtp = props.multi_processor_count, props.max_threads_per_multi_processor
    gen = th.cuda.default_generators[0]
    res = {"cus": cus, "max_threads_per_cu": mtp, "rows": []}
    p = 0.6
    keep = float(th.tensor(1.0 - p, dtype=th.float32))
    shapes = [(13, 1, 1), (1001, 3, 1), (1001, 2, 1), (4099, 8, 1), (70001, 5, 1), (3_000_001, 2, 1),
              (5_000_001, 3, 1), (2_000_000, 8, 1), (114_615_892, 8, 1)]
    for shape in shapes:
        n = shape[0] * shape[1] * shape[2]
        for seed, pre in ((0, 0), (123456789012, 3)):
            th.manual_seed(seed)
            for _ in range(pre):  # move the generator offset off zero
                th.native_dropout(th.empty(1000, device=dev), 0.5, True)
            s0, off0 = gen.initial_seed(), gen.get_offset()
            _, m = th.native_dropout(th.empty(shape, device=dev), p, True)
            off1 = gen.get_offset()
            grid = min(cus * (mtp // 256), (n + 255) // 256)
            want_inc = ((n - 1) // (256 * grid * 4) + 1) * 4
            row = {"shape": list(shape), "seed": s0, "offset": off0, "offset_inc": off1 - off0,
                   "predicted_inc": want_inc, "grid": grid}
            ref = m.reshape(-1).to(th.uint8)
            out = th.empty(n, dtype=th.uint8, device=dev)
            for v in range(4):
                rc = lib.philox_probe(n, grid * 256, s0, off0, keep, v, ctypes.c_void_p(out.data_ptr()),
                                      ctypes.c_void_p(th.cuda.current_stream().cuda_stream))
                assert rc == 0
                row["v%d_mismatch" % v] = int((out != ref).sum())
            row["kept_frac"] = float(ref.float().mean())
            res["rows"].append(row)
            print(json.dumps(row), flush=True)
            del m, ref, out
    print(json.dumps(res))


if __name__ == "__main__":
    main()
