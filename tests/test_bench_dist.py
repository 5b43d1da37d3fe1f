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


def test_bench_gpus_flag_launches_ranks():
    """`python bench.py --gpus 2` with no launcher starts two ranks itself;
    the JSON reports n_gpus == 2 and the slowest rank's time (rank 1 sleeps
    twice as long as rank 0)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--plumbing"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["world_from_dist"] == 2
    assert len(res["rank_s"]) == 2 and res["elapsed"] == max(res["rank_s"])
    assert res["rank_s"][1] >= 0.1


def test_bench_rejects_world_mismatch():
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--plumbing"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def test_bench_launcher_stops_peers_of_a_failed_rank():
    """A rank that dies (here: exit 3 before the rendezvous) makes the
    launcher stop its peers — rank 0 would otherwise wait in the gloo
    rendezvous until its timeout — and return the failing exit code."""
    import subprocess
    import sys
    import time
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["SBK_PLUMBING_FAIL_RANK"] = "1"
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--plumbing"],
                       capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-500:])  # the failing rank's code, not a terminated peer's -15
    assert time.perf_counter() - t0 < 90
