"""Generate tests/golden/kernel_g20.npz -- golden vectors of the CPU oracle.

The reference library cannot run here, so these vectors come
from the oracle's deterministic single-thread restatement on the reference's
own test graph and seed (tests/compute/test_kernel.py:33-74, 338-351); the
oracle itself is pinned by tests/golden/spmat_kat.json and by the UDF
cross-check in tests/test_oracle_cpu.py.  Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.dirname(HERE)):
    if p not in sys.path:
        sys.path.insert(0, p)

from oracle import oracle as O  # noqa: E402
from graphs import CODE, binary_case_features, g20  # noqa: E402

CASES = [
    # (lhs, op, rhs, reducer, broadcast)
    ("u", "use_lhs", None, "sum", "none"),
    ("u", "use_lhs", None, "max", "none"),
    ("u", "use_lhs", None, "mean", "none"),
    ("e", "use_lhs", None, "sum", "none"),
    ("u", "mul", "e", "sum", "e"),
    ("u", "mul", "e", "sum", "none"),
    ("u", "add", "v", "none", "none"),
    ("u", "dot", "v", "none", "none"),
    ("e", "sub", "v", "none", "v"),
    ("e", "div", "v", "none", "v"),
    ("v", "sub", "u", "min", "u"),
    ("e", "dot", "u", "max", "e"),
]


def cases():
    src, dst, n = g20()
    m = len(src)
    g = O.RefGraph(src, dst, n)
    for lhs, op, rhs, red, bc in CASES:
        name = "%s_%s_%s_%s_%s" % (lhs, op, rhs, red, bc)
        d = binary_case_features(n, m, lhs, rhs or "u", "mul" if op == "use_lhs" else op, bc)
        out_rows = m if red == "none" else n
        if op == "use_lhs":
            x = d[lhs]
            out = O.copy_reduce(red, g, CODE[lhs], x, out_rows)
            go = np.linspace(-1, 1, out.size, dtype=np.float32).reshape(out.shape)
            _, gx = O.copy_reduce(red, g, CODE[lhs], x, out_rows, grad_out=go)
            yield name, {"x": x, "out": out, "grad_out": go, "grad_x": gx}
        else:
            l, r = d[lhs], d[rhs]
            out = O.binary_reduce(red, op, g, CODE[lhs], CODE[rhs], l, r, out_rows)
            go = np.linspace(-1, 1, out.size, dtype=np.float32).reshape(out.shape)
            _, gl, gr = O.binary_reduce(red, op, g, CODE[lhs], CODE[rhs], l, r, out_rows,
                                        grad_out=go)
            yield name, {"lhs": l, "rhs": r, "out": out, "grad_out": go, "grad_lhs": gl,
                         "grad_rhs": gr}


def main():
    arrays = {"src": g20()[0], "dst": g20()[1]}
    for name, arrs in cases():
        for k, v in arrs.items():
            arrays[name + "/" + k] = v
    np.savez_compressed(os.path.join(HERE, "kernel_g20.npz"), **arrays)
    print("wrote", len(arrays), "arrays")


if __name__ == "__main__":
    main()
