"""The multi-GPU sort over real RCCL ranks, one process per visible GPU
(until now every RCCL call ran on a one-rank
communicator).  bench.py's layout at W GPUs -- two batch groups of W/2 ranks
(the sort's two batches per phase, parts all-gathered over a group
communicator) each limb-sharded over its own communicator, or limb sharding
over all W ranks -- must give every rank the unsharded sort's ciphertext,
residue for residue, eagerly and through the captured graph (collectives
inside it).  Needs at least two visible GPUs: skipped on a one-GPU box (the
driver's 8-GPU node runs bench.py --gpus N); tests/test_gpu_shard.py covers the
same layouts with thread ranks on one GPU."""
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _visible_gpus() -> int:
    import torch
    return torch.cuda.device_count()  # (counts devices without initialising them)


def _rank(rank, world, port, groups, N, logn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "sorting-fhe_amd", "python"))
    try:
        import numpy as np
        import bench
        import sfhe
        w, r, local = bench.dist_init()  # gloo: the RCCL ids travel over it
        depth, rots = sfhe.direct_sort_params(N, "hip")
        kw = dict(mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots, seed=20251205 + N,
                  device=local)
        cfg = bench.sign_config(N)
        x = bench.input_vector(N)
        ref = sfhe.Engine("hip", **kw)
        ref.set_quiet(True)
        want = ref.sorter(N).sort(ref.encrypt(x.tolist()), *cfg).download()
        ref.close()
        shard, grp = bench.comm_spec("rccl", r, w, groups)
        e = sfhe.Engine("hip", shard=shard, groups=grp, **kw)
        e.set_quiet(True)
        s = e.sorter(N)
        ct = e.encrypt(x.tolist())
        ok = []
        for _ in range(3):  # eager, captured, replayed
            bench.barrier(w)
            ok.append(bool(np.array_equal(s.sort(ct, *cfg).download(), want)))
        nodes = s.graph_nodes()
        e.close()
        q.put((r, ok, nodes, None))
        import torch.distributed as dist
        dist.destroy_process_group()
    except Exception as ex:  # noqa: BLE001 -- reported to the parent
        q.put((rank, [], 0, repr(ex)))


@pytest.mark.parametrize("groups", [2, 1])
def test_rccl_multi_rank_sort_bitexact(hip_lib, groups):
    n = _visible_gpus()
    if n < 2:
        pytest.skip(f"{n} visible GPU(s): the multi-rank RCCL sort needs at least 2")
    world = min(n, 8) // 2 * 2  # an even world: two batch groups
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + os.getpid() % 1000 + groups
    procs = [ctx.Process(target=_rank, args=(r, world, port, groups, 256, 16, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=600) for _ in procs], key=lambda t: t[0])
    for p in procs:
        p.join(120)
    for r, ok, nodes, err in res:
        assert err is None, f"rank {r}: {err}"
        assert ok == [True, True, True], f"rank {r}: eager / captured / replayed bit-exact: {ok}"
        assert nodes > 0, f"rank {r}: no graph"
