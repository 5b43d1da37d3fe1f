"""The bench's multi-rank timing on CPU (gloo, world_size 2): every rank gets
the slowest rank's wall time, and the job value counts all ranks' audio."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    t = bench.max_over_ranks(0.5 + rank, world, torch.device("cpu"))
    out[rank] = t
    dist.barrier()
    dist.destroy_process_group()


def test_max_over_ranks_gloo():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    assert dict(out) == {0: 1.5, 1: 1.5}


def test_max_over_ranks_single():
    import bench
    assert bench.max_over_ranks(0.25, 1, torch.device("cpu")) == 0.25
