"""Worker for tests/test_bench_guard_cpu.py (gloo, CPU): one rank fails or stalls
inside a bench side line while its peer waits in a collective."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch as th  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def main():
    mode = sys.argv[1]
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    res = {"metric": "guard-test", "value": 1.0}
    guard = bench.SideLineGuard(dist, rank, res, budget_s=float(os.environ.get("BUDGET", "300")))
    guard.start("c4")
    try:
        if mode == "raise" and rank == 1:
            raise RuntimeError("injected failure")
        if mode == "raise0" and rank == 0:
            raise RuntimeError("injected failure on rank 0")
        if mode == "raiselast" and rank == dist.get_world_size() - 1:
            raise RuntimeError("injected failure on the last rank")
        if mode == "stall" and rank == 1:
            time.sleep(600)
        t = th.ones(1)
        dist.all_reduce(t)  # the peer of a failing rank waits here
        res["c4"] = {"value": float(t.item())}
    except Exception as exc:  # noqa: BLE001
        guard.fail(exc)
    guard.phase = None
    guard.finish()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
