"""Helpers to run world_size-N process groups in tests (127.0.0.1 rendezvous)."""
import os
import socket

import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _entry(rank, world, port, fn, args, backend="gloo"):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if backend == "nccl":  # RCCL: one rank per GPU (cuda:rank)
        import torch
        torch.cuda.set_device(rank)
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", rank))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    try:
        fn(rank, world, *args)
    finally:
        dist.destroy_process_group()


def run_world(fn, world=2, args=(), backend="gloo"):
    mp.spawn(_entry, args=(world, free_port(), fn, args, backend), nprocs=world, join=True)
