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


def _sharded_worker(rank, world, port, q):
    """bench.py's N > 1 flow on the CPU oracle (test infrastructure: the
    bench itself only ever builds HIP engines): the replica leg, then the
    limb-sharded sort over the gloo host transport (bench.shard_spec "host")
    timed by the same barrier / max-over-ranks helper."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), OMP_NUM_THREADS="2")
    sys.path.insert(0, ROOT)
    import bench
    import sfhe
    from oracle import slotsim
    w, r, _ = bench.dist_init()
    N, logn = 8, 12
    depth, rots = sfhe.direct_sort_params(N, "oracle")
    spec = dict(N=N, logn=logn, secure=False, depth=depth, rots=rots, cfg=slotsim.default_sign_config(N))
    kw = dict(mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots)
    rep = bench.replica_leg(lambda: sfhe.Engine("oracle", seed=11 + r, **kw), spec, w, steps=1, warmup=0)
    eng = sfhe.Engine("oracle", seed=20251205 + N, shard=bench.shard_spec("host", r, w), **kw)
    eng.set_quiet(True)
    sorter = eng.sorter(N)
    ct = eng.encrypt(bench.input_vector(N).tolist())
    out = {}

    def step():
        out["ct"] = sorter.sort(ct, *spec["cfg"])

    dt = bench.timed_steps(step, eng.sync, w, steps=1, warmup=0)
    line = bench.fallback_line(rep, spec, w, type("A", (), {"steps": 1, "warmup": 0, "workload": "t"})(), "test")
    q.put((r, dt, rep["value"], out["ct"].download(), eng.shard_tail(), line["scaling"]))
    import torch.distributed as dist
    dist.destroy_process_group()


def test_two_rank_sharded_bench_flow(oracle_lib):
    import numpy as np
    import sfhe
    from oracle import slotsim
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + os.getpid() % 1000
    procs = [ctx.Process(target=_sharded_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (_, dt0, v0, ct0, tail0, sc0), (_, dt1, v1, ct1, tail1, sc1) = res
    assert dt0 == dt1 and v0 == v1 and v0 > 0          # max over ranks, on both
    assert tail0 == tail1 == 16 and sc0 == "weak"
    assert np.array_equal(ct0, ct1)                   # both ranks hold the whole result
    N = 8
    depth, rots = sfhe.direct_sort_params(N, "oracle")
    ref = sfhe.Engine("oracle", mult_depth=depth, ring_dim=1 << 12, batch_size=N, rotations=rots,
                      seed=20251205 + N)
    ref.set_quiet(True)
    want = ref.sorter(N).sort(ref.encrypt(slotsim.input_vector(N).tolist()), *slotsim.default_sign_config(N))
    assert np.array_equal(ct0, want.download())       # and it is the unsharded sort's
