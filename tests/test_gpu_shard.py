"""Limb sharding on the HIP product: W ranks as threads sharing device 0
(each its own context and streams), exchanging limbs through the host
transport (ThreadComm), must reproduce the unsharded HIP residues bit for
bit -- every op at W = 2, 3, whole sorts up to the metric sort and config 5's
at W = 8.  The RCCL transport runs on a one-rank communicator (RCCL does not
place two ranks on one GPU), which takes the sharded path with every
exchange an RCCL call, eagerly and captured into the sort's hipGraph; the
multi-GPU run is bench.py --gpus N on a node.
"""
import numpy as np
import pytest

import sfhe
from oracle import slotsim
from test_shard import OPS_KW, compare, ops_program, sort_program

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,tail", [(2, 0), (3, 0), (3, 3)])
def test_sharded_ops_bitexact_hip(hip_lib, world, tail, monkeypatch):
    monkeypatch.setenv("SFHE_SHARD_TAIL", str(tail))  # dealt rows (and the replicated tail below 4 limbs)
    ref = ops_program(sfhe.Engine("hip", **OPS_KW))
    outs = sfhe.run_sharded_threads("hip", world, ops_program, **OPS_KW)
    for r in range(world):
        compare(ref, outs[r])


def test_sharded_sort_bitexact_hip(hip_lib):
    N = 8
    depth, rots = sfhe.direct_sort_params(N, "hip")
    kw = dict(mult_depth=depth, ring_dim=1 << 12, batch_size=N, rotations=rots, seed=777)
    ref = sort_program(sfhe.Engine("hip", **kw), N)
    outs = sfhe.run_sharded_threads("hip", 2, lambda e: sort_program(e, N), **kw)
    for r in range(2):
        compare(ref, outs[r])
    # and the unsharded HIP result is the oracle's (tests/test_gpu_parity.py covers the rest)
    ora = sort_program(sfhe.Engine("oracle", **kw), N)
    assert np.array_equal(ref["sort"], ora["sort"])


@pytest.mark.parametrize("N,logn,world", [(64, 15, 3), (128, 16, 4), (256, 17, 2), (256, 17, 4),
                                           (256, 16, 8), (256, 17, 8)])
def test_sharded_sort_large_bitexact_hip(hip_lib, N, logn, world):
    """Larger rings and limb counts (31 Q limbs at N=128), more ranks, the
    metric sort (DirectSort<256> at ring 2^16) and BASELINE config 5's sort
    (DirectSort<256> at ring 2^17, 35 Q limbs) at W = 8 -- the node's GPU
    count, every rank a thread on this one GPU with its own context and
    streams -- each with the default replicated tail (levels of at most 16
    limbs on every rank)."""
    depth, rots = sfhe.direct_sort_params(N, "hip")
    kw = dict(mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots, seed=4099)
    ref = sort_program(sfhe.Engine("hip", **kw), N)
    assert np.max(np.abs(ref["dec"][:N] - np.sort(slotsim.input_vector(N)))) < 0.01
    outs = sfhe.run_sharded_threads("hip", world, lambda e: sort_program(e, N), **kw)
    for r in range(world):
        compare(ref, outs[r])


@pytest.mark.parametrize("N,logn,world,groups", [(256, 16, 2, 2), (256, 16, 8, 2), (256, 17, 4, 2)])
def test_batch_split_sort_bitexact_hip(hip_lib, N, logn, world, groups):
    """The bench's multi-GPU layout as thread ranks on this GPU: two batch
    groups (each runs one of the sort's two batches per phase; parts
    all-gathered over the host transport), each group limb-sharded over
    world // groups ranks -- the metric sort at W = 2 (split only) and W = 8
    (2 x 4), config 5's at W = 4 -- bit-identical to the unsplit sort."""
    depth, rots = sfhe.direct_sort_params(N, "hip")
    kw = dict(mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots, seed=4099)
    ref = sort_program(sfhe.Engine("hip", **kw), N)
    outs = sfhe.run_split_threads("hip", world, groups, lambda e: sort_program(e, N), **kw)
    for r in range(world):
        compare(ref, outs[r])


RCCL_SCRIPT = r"""
import os, sys
sys.path.insert(0, {py!r}); sys.path.insert(0, {tests!r})
import numpy as np
import sfhe
from oracle import slotsim
from test_shard import OPS_KW, compare, ops_program
os.environ["SFHE_SHARD_TAIL"] = "3"
uid = sfhe.comm_uid("hip")
assert uid is not None and len(uid) == 128
e = sfhe.Engine("hip", shard=("rccl", 0, 1, uid), **OPS_KW)
ref = sfhe.Engine("hip", **OPS_KW)
compare(ops_program(ref), ops_program(e))
e.close(); ref.close()
print("RCCL communicator OK", flush=True)
# the sharded sort through RCCL (a one-rank communicator takes the sharded
# path: every ModUp / ModDown all-gather and rescale broadcast is an RCCL
# call), captured into the sort's hipGraph with its collectives and replayed
os.environ["SFHE_SHARD_TAIL"] = {tail!r}
# special-prime tiers (DESIGN.md §4b) run at replicated levels only: below the
# largest tier bound (10 limbs) a small tail would have the sharded sort take
# them at fewer levels than the unsharded one, so both run without them there
if int({tail!r}) < 10:
    os.environ["SFHE_KS_TIERS"] = "0"
N, logn = {N}, {logn}
depth, rots = sfhe.direct_sort_params(N, "hip")
kw = dict(mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots, seed=4099)
cfg = slotsim.default_sign_config(N)
x = slotsim.input_vector(N)
ref = sfhe.Engine("hip", **kw); ref.set_quiet(True)
want = ref.sorter(N).sort(ref.encrypt(x.tolist()), *cfg).download()
ref.close()
uid, uid2 = sfhe.comm_uid("hip"), sfhe.comm_uid("hip")
# and a one-group batch communicator: every part of both phases through ncclAllGather
e = sfhe.Engine("hip", shard=("rccl", 0, 1, uid), groups=("rccl", 0, 1, uid2), **kw); e.set_quiet(True)
assert e.groups() == (0, 1)
s = e.sorter(N)
ct = e.encrypt(x.tolist())
outs = [s.sort(ct, *cfg) for _ in range(3)]   # eager, captured, replayed
nodes = s.graph_nodes()
for o in outs:
    assert np.array_equal(o.download(), want)
y = x[::-1].copy()
o = s.sort(e.encrypt(y.tolist()), *cfg)       # a new input through the graph
err = float(np.max(np.abs(np.array(e.decrypt(o))[:N] - np.sort(y))))
assert err < 0.01, err
print(f"RCCL sharded sort N={{N}} 2^{{logn}}: graph of {{nodes}} nodes, bit-exact vs unsharded, err {{err:.3g}}", flush=True)
assert nodes > 100, nodes
e.close()
print("RCCL graph OK")
"""


@pytest.mark.parametrize("N,logn,tail", [(64, 14, "3"), (256, 16, "16")])
def test_rccl_single_rank_communicator(hip_lib, N, logn, tail):
    """sfhe_comm_uid + sfhe_shard_rccl (ncclCommInitRank) on one rank: the
    context takes the sharded code path with every exchange an RCCL call
    (ncclAllGather / ncclBroadcast, not the one-rank device copy); the sort
    also has a one-group batch communicator (sfhe_groups_rccl) through which
    every batch part is all-gathered.  The op
    program, then DirectSort<N> sorted eagerly, captured into a hipGraph
    WITH its RCCL collectives, and replayed -- all bit-identical to the
    unsharded sort.  Own process: RCCL's threads and the HIP runtime are torn
    down with it."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = RCCL_SCRIPT.format(py=os.path.join(os.path.dirname(here), "sorting-fhe_amd", "python"), tests=here,
                              N=N, logn=logn, tail=tail)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    print(r.stdout[-3000:])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "RCCL communicator OK" in r.stdout and "RCCL graph OK" in r.stdout
