"""Probe: can two RCCL ranks share one GPU on the 1-GPU box?

If they can, the N = 2 bench path (RCCL all-to-all-v, all-reduce) can be rehearsed
on the real collective library before the driver's 8-GPU run; if RCCL refuses a
duplicate device it says so within seconds.  Each rank all-reduces and
all-to-all-v's a small tensor and prints the result as one JSON line.
"""
import json
import os
import subprocess
import sys


def worker():
    import torch as th
    import torch.distributed as dist
    rank = int(os.environ["RANK"])
    dev = th.device("cuda:0")
    th.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    x = th.full((1024,), float(rank + 1), device=dev)
    dist.all_reduce(x)
    send = th.arange(8, dtype=th.float32, device=dev) + 100 * rank
    recv = th.empty(8, device=dev)
    dist.all_to_all_single(recv, send, [4, 4], [4, 4])
    th.cuda.synchronize()
    print(json.dumps({"rank": rank, "allreduce": float(x[0]), "a2a": recv.tolist()}), flush=True)
    dist.destroy_process_group()


def main():
    n = 2
    env = dict(os.environ, WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
    procs = [subprocess.Popen([sys.executable, __file__, "--worker"],
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r))) for r in range(n)]
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=90))
        except subprocess.TimeoutExpired:
            p.kill()
            rcs.append(-9)
    print(json.dumps({"probe": "rccl_same_device", "rcs": rcs}), flush=True)
    sys.exit(0 if all(r == 0 for r in rcs) else 1)


if __name__ == "__main__":
    if "--worker" in sys.argv:
        worker()
    else:
        main()
