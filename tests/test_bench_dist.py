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


def _sharded_worker(rank, world, port, q, groups=1, N=8):
    """bench.py's N > 1 flow on the CPU oracle (test infrastructure: the
    bench itself only ever builds HIP engines): the replica leg, then the
    multi-GPU sort over the gloo host transport (bench.comm_spec "host":
    `groups` batch groups, each limb-sharded over world // groups ranks)
    timed by the same barrier / max-over-ranks helper."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), OMP_NUM_THREADS="2")
    sys.path.insert(0, ROOT)
    import bench
    import sfhe
    from oracle import slotsim
    w, r, _ = bench.dist_init()
    logn = 12
    depth, rots = sfhe.direct_sort_params(N, "oracle")
    spec = dict(N=N, logn=logn, secure=False, depth=depth, rots=rots, cfg=slotsim.default_sign_config(N))
    kw = dict(mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots)
    # the replica leg on DirectSort<8> (its flow does not depend on N)
    d8, r8 = sfhe.direct_sort_params(8, "oracle")
    spec8 = dict(spec, N=8, depth=d8, rots=r8, cfg=slotsim.default_sign_config(8))
    rep = bench.replica_leg(lambda: sfhe.Engine("oracle", seed=11 + r, mult_depth=d8, ring_dim=1 << logn,
                                                batch_size=8, rotations=r8), spec8, w, steps=1, warmup=0)
    shard, grp = bench.comm_spec("host", r, w, groups)
    eng = sfhe.Engine("oracle", seed=20251205 + N, shard=shard, groups=grp, **kw)
    eng.set_quiet(True)
    sorter = eng.sorter(N)
    ct = eng.encrypt(bench.input_vector(N).tolist())
    out = {}

    def step():
        out["ct"] = sorter.sort(ct, *spec["cfg"])

    dt = bench.timed_steps(step, eng.sync, w, steps=1, warmup=0)
    # the bench's collective attribution (its profiling sort): one more sort with the counters on
    eng.comm_stats_reset(timed=True)
    step()
    comm = eng.comm_stats()
    line = bench.fallback_line(rep, spec, w, type("A", (), {"steps": 1, "warmup": 0, "workload": "t"})(), "test")
    q.put((r, dt, rep["value"], out["ct"].download(), eng.shard_tail(), line["scaling"],
           bench.parallelism(w, groups, "gloo", eng.shard_tail()), comm))
    import torch.distributed as dist
    dist.destroy_process_group()


@pytest.mark.parametrize("world,groups,N,label", [
    (2, 1, 8, "limb-shard x2 (replicated tail <= 16 limbs) over gloo"),
    (4, 2, 64, "batch-split x2 * limb-shard x2 (replicated tail <= 16 limbs) over gloo"),
])
def test_sharded_bench_flow(oracle_lib, world, groups, N, label):
    """W = 2: limb sharding alone (DirectSort<8>, one batch); W = 4: the
    bench's default layout, two batch groups of two limb-sharded ranks
    (DirectSort<64> @ 2^12: two batches per phase, one per group)."""
    import numpy as np
    import sfhe
    from oracle import slotsim
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 30500 + os.getpid() % 1000 + 7 * world
    procs = [ctx.Process(target=_sharded_worker, args=(r, world, port, q, groups, N)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    dts = {t[1] for t in res}
    assert len(dts) == 1 and res[0][2] > 0            # max over ranks, on every rank
    assert all(t[4] == 16 and t[5] == "weak" and t[6] == label for t in res)
    ct0 = res[0][3]
    for t in res[1:]:
        assert np.array_equal(ct0, t[3])              # every rank holds the whole result
    for t in res:  # every rank exchanged data in its sort, and timed it
        c = t[7]
        assert c["calls"] > 0 and c["bytes"] > 0 and c["ms"] > 0, c
    per = world // groups                             # (rank = group * per + in-group rank)
    for g in range(groups):                           # one batch group's ranks issue the same collectives
        assert len({t[7]["calls"] for t in res[g * per:(g + 1) * per]}) == 1, [t[7] for t in res]
    depth, rots = sfhe.direct_sort_params(N, "oracle")
    ref = sfhe.Engine("oracle", mult_depth=depth, ring_dim=1 << 12, batch_size=N, rotations=rots,
                      seed=20251205 + N)
    ref.set_quiet(True)
    want = ref.sorter(N).sort(ref.encrypt(slotsim.input_vector(N).tolist()), *slotsim.default_sign_config(N))
    assert np.array_equal(ct0, want.download())       # and it is the unsharded sort's
