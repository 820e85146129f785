"""bench.py's multi-process timing path on CPU: world_size 2 over gloo.

Each rank runs a fake step of a different length; the reported time must be
the max over ranks, identical on both ranks, and cover exactly K steps."""
import os
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    import time
    import bench
    w, r, local = bench.dist_init()
    calls = {"n": 0}

    def step():
        calls["n"] += 1
        time.sleep(0.01 * (r + 1))

    dt = bench.timed_steps(step, lambda: None, w, steps=5, warmup=2)
    q.put((r, dt, calls["n"]))
    import torch.distributed as dist
    dist.destroy_process_group()


def test_two_rank_max_timing():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    res.sort()
    (r0, dt0, n0), (r1, dt1, n1) = res
    assert n0 == n1 == 7
    assert dt0 == dt1                 # both ranks report the max
    assert dt0 >= 5 * 0.02 * 0.95     # rank 1's 5 timed steps of 20 ms dominate
