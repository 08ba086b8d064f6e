#!/usr/bin/env python3
"""Rehearsal diagnostics: N processes sharing one GPU each run th.unique over
175 M int64 keys (what partition_stats does at C4 size) and log progress per
process; a sort whose tiles spin on their predecessors can stall when other
processes' kernels hold the CUs."""
import sys
import time

import torch as th


def main():
    r = int(sys.argv[1])
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 175_000_000
    log = open("gpurun_out/contention_%d.log" % r, "a")
    g = th.Generator(device="cuda:0")
    g.manual_seed(r)
    k = th.randint(0, 80_000_000, (n,), device="cuda:0", generator=g)
    th.cuda.synchronize()
    for i in range(3):
        t = time.time()
        u = th.unique(k)
        th.cuda.synchronize()
        log.write("unique %d: %.2fs (%d)\n" % (i, time.time() - t, u.numel()))
        log.flush()


if __name__ == "__main__":
    main()
