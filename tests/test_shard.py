"""Limb sharding on the CPU oracle: W ranks, each holding the
RNS limbs i with i % W == rank, must produce exactly the residues of the
unsharded context -- every evaluator op, and a whole DirectSort.

The ranks run as threads of this process over ThreadComm (host-memory
all-gather / broadcast through the C ABI's sfhe_shard_host), and as two
processes over torch.distributed gloo (GlooComm), the transport a CPU-only
multi-process job would use.  RCCL (sfhe_shard_rccl) is the GPU path
(tests/test_gpu_shard.py, bench.py --shard).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import sfhe
from oracle import slotsim

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

OPS_KW = dict(mult_depth=6, ring_dim=1 << 12, batch_size=16, seed=4242, rotations=[1, 3, -2])


def ops_program(e):
    """Every evaluator op the sort uses, down to the last level (where a rank
    of W = 3 holds no limb); returns the downloaded residues and a decryption."""
    rng = np.random.default_rng(11)
    a = rng.uniform(-1, 1, 16).tolist()
    b = rng.uniform(-1, 1, 16).tolist()
    ca, cb = e.encrypt(a), e.encrypt(b)
    x = e.mult(ca, cb)
    x2 = e.mult(x, x)
    res = {
        "enc": ca,
        "add": e.add(ca, cb),
        "sub": e.sub(ca, cb),
        "mult": x,
        "mult_const": e.mult_const(ca, -3.75),
        "add_const": e.add_const(ca, 0.5),
        "mult_plain": e.mult_plain(ca, list(range(16)), 16),
        "rotate1": e.rotate(ca, 1),
        "rotate-2": e.rotate(x, -2),
        "mixed_level": e.add(x2, ca),
        "deep": e.mult(e.mult(e.mult(e.mult(x2, x), cb), ca), x),
        "cheb": e.chebyshev(ca, [0.1, 0.5, -0.25, 0.125, 0.05]),
    }
    out = {k: v.download() for k, v in res.items()}
    out["dec"] = np.array(e.decrypt(res["deep"]))
    out["levels"] = np.array([v.level for v in res.values()])
    return out


def sort_program(e, N):
    e.set_quiet(True)
    x = slotsim.input_vector(N).tolist()
    s = e.sorter(N)
    r = s.sort(e.encrypt(x), *slotsim.default_sign_config(N))
    return {"sort": r.download(), "dec": np.array(e.decrypt(r))}


def compare(ref, got):
    assert sorted(ref) == sorted(got)
    for k, v in ref.items():
        assert got[k].shape == v.shape, k
        bad = int(np.count_nonzero(got[k] != v))
        assert bad == 0, f"{k}: {bad} of {v.size} values differ"


@pytest.mark.parametrize("world,tail", [(2, 0), (3, 0), (2, 3), (3, 4), (3, 16)])
def test_sharded_ops_bitexact_oracle(oracle_lib, world, tail, monkeypatch):
    """tail: SFHE_SHARD_TAIL, the limb count at and below which every rank
    holds every row (0: dealt at every level; 3 / 4: the program crosses into
    the replicated tail -- rescales, level adjustments, lifts and weighted-sum
    inputs gathered there; 16: replicated throughout)."""
    monkeypatch.setenv("SFHE_SHARD_TAIL", str(tail))
    ref = ops_program(sfhe.Engine("oracle", **OPS_KW))
    assert ref["levels"].max() == OPS_KW["mult_depth"]  # "deep" reached the last level
    outs = sfhe.run_sharded_threads("oracle", world, ops_program, **OPS_KW)
    for r in range(world):
        compare(ref, outs[r])


@pytest.mark.parametrize("N,logn,world", [(8, 12, 2), (64, 13, 2), (64, 13, 3), (64, 13, 4), (8, 12, 8)])
def test_sharded_sort_bitexact_oracle(oracle_lib, N, logn, world):
    """Whole DirectSort<N> limb-sharded over W thread ranks (the default
    replicated tail of 16 limbs: the rank's first levels are dealt, the
    placement replicated).  W = 8: 3-4 dealt rows per rank above the tail."""
    depth, rots = sfhe.direct_sort_params(N, "oracle")
    kw = dict(mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots, seed=777)
    ref = sort_program(sfhe.Engine("oracle", **kw), N)
    assert np.max(np.abs(ref["dec"][:N] - np.sort(slotsim.input_vector(N)))) < 0.01
    outs = sfhe.run_sharded_threads("oracle", world, lambda e: sort_program(e, N), **kw)
    for r in range(world):
        compare(ref, outs[r])


def test_shard_argument_errors(oracle_lib):
    e = sfhe.Engine("oracle", keygen=False, mult_depth=2, ring_dim=1 << 12)
    with pytest.raises(sfhe.SfheError):
        e.shard_host(3, 2, sfhe.ThreadComm(2))  # rank outside the world
    e2 = sfhe.Engine("oracle", mult_depth=2, ring_dim=1 << 12)
    with pytest.raises(sfhe.SfheError):  # after key generation
        e2.shard_host(0, 2, sfhe.ThreadComm(2))
    assert sfhe.comm_uid("oracle") is None  # the oracle has no RCCL
    with pytest.raises(sfhe.SfheError):
        sfhe.Engine("oracle", keygen=False, mult_depth=2, ring_dim=1 << 12, shard=("rccl", 0, 2, bytes(128)))


GLOO_SCRIPT = r"""
import sys
import numpy as np
sys.path.insert(0, {py!r}); sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
import torch.distributed as dist
import sfhe
from test_shard import ops_program, OPS_KW
rank = int(sys.argv[1])
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{port}", rank=rank, world_size=2)
e = sfhe.Engine("oracle", shard=("host", rank, 2, sfhe.GlooComm()), **OPS_KW)
out = ops_program(e)
np.savez({path!r} + str(rank) + ".npz", **out)
dist.barrier()
dist.destroy_process_group()
"""


def test_sharded_ops_gloo_two_processes(oracle_lib, tmp_path):
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    path = str(tmp_path / "rank")
    code = GLOO_SCRIPT.format(py=os.path.join(ROOT, "sorting-fhe_amd", "python"), root=ROOT,
                              tests=os.path.join(ROOT, "tests"), port=port, path=path)
    # dealt rows above 3 limbs, the replicated tail below: both across processes
    env = dict(os.environ, OMP_NUM_THREADS="4", SFHE_SHARD_TAIL="3")
    procs = [subprocess.Popen([sys.executable, "-c", code, str(r)], env=env) for r in range(2)]
    try:
        for p in procs:
            assert p.wait(timeout=600) == 0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    ref = ops_program(sfhe.Engine("oracle", **OPS_KW))
    for r in range(2):
        z = np.load(f"{path}{r}.npz")
        compare(ref, {k: z[k] for k in z.files})


GLOO_SORT_SCRIPT = r"""
import sys
import numpy as np
sys.path.insert(0, {py!r}); sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
import torch.distributed as dist
import sfhe
from test_shard import sort_program
rank = int(sys.argv[1])
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:{port}", rank=rank, world_size={W})
kw = {kw!r}
e = sfhe.Engine("oracle", shard=("host", rank, {W}, sfhe.GlooComm()), **kw)
out = sort_program(e, {N})
np.savez({path!r} + str(rank) + ".npz", **out)
dist.barrier()
dist.destroy_process_group()
"""


@pytest.mark.parametrize("N,logn,W,overlap", [(8, 12, 2, None), (64, 13, 2, None), (64, 13, 4, None), (64, 13, 4, "0")])
def test_sharded_sort_gloo_two_processes(oracle_lib, tmp_path, N, logn, W, overlap):
    """A whole DirectSort<N> limb-sharded over W PROCESSES (one per 'GPU',
    gloo host transport): every exchange of a real sharded sort (ModUp /
    ModDown all-gathers, rescale broadcasts) crosses a process boundary;
    every rank's result is bit-identical to the unsharded sort.  The ModUp
    is the overlapped form by default (each rank converts its own rows while
    the all-gather brings the rest, then adds the rest's part: DESIGN.md §7);
    overlap "0" runs the unsplit form (SFHE_SHARD_OVERLAP=0) at W = 4."""
    import socket
    depth, rots = sfhe.direct_sort_params(N, "oracle")
    kw = dict(mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots, seed=777)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    path = str(tmp_path / "rank")
    code = GLOO_SORT_SCRIPT.format(py=os.path.join(ROOT, "sorting-fhe_amd", "python"), root=ROOT,
                                   tests=os.path.join(ROOT, "tests"), port=port, path=path, kw=kw, N=N, W=W)
    env = dict(os.environ, OMP_NUM_THREADS=str(max(1, 8 // W)))
    if overlap is not None:
        env["SFHE_SHARD_OVERLAP"] = overlap
    procs = [subprocess.Popen([sys.executable, "-c", code, str(r)], env=env) for r in range(W)]
    try:
        for p in procs:
            assert p.wait(timeout=900) == 0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    ref = sort_program(sfhe.Engine("oracle", **kw), N)
    for r in range(W):
        z = np.load(f"{path}{r}.npz")
        compare(ref, {k: z[k] for k in z.files})


@pytest.mark.parametrize("world,groups", [(1, 1), (2, 2), (4, 2)])
def test_batch_split_sort_bitexact_oracle(oracle_lib, world, groups):
    """DirectSort<64> @ 2^12 has B = 2 batches in both phases (P = 32): with
    two batch groups each group runs one batch and all-gathers the parts
    (sfhe_groups_host); W = 4 also limb-shards each group over two ranks.
    Every rank's result is bit-identical to the unsplit sort.  (1, 1): one
    group that still gathers every part through its communicator."""
    N, logn = 64, 12
    depth, rots = sfhe.direct_sort_params(N, "oracle")
    kw = dict(mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots, seed=777)

    def prog(e):
        e.op_stats(reset=True)
        out = sort_program(e, N)
        return out, e.op_stats()["tensor"]

    ref, ref_tensors = prog(sfhe.Engine("oracle", **kw))
    assert np.max(np.abs(ref["dec"][:N] - np.sort(slotsim.input_vector(N)))) < 0.01
    outs = sfhe.run_split_threads("oracle", world, groups, prog, **kw)
    for r in range(world):
        compare(ref, outs[r][0])
        if groups > 1:  # one of the two batches per rank: about half the ct x ct products
            assert outs[r][1] < 0.6 * ref_tensors, (outs[r][1], ref_tensors)


def test_batch_groups_arguments(oracle_lib):
    e = sfhe.Engine("oracle", keygen=False, mult_depth=2, ring_dim=1 << 12)
    assert e.groups() == (0, 1)
    with pytest.raises(sfhe.SfheError):
        e.groups_host(2, 2, sfhe.ThreadComm(2))  # group outside the groups
    e.groups_host(1, 2, sfhe.ThreadComm(2))
    assert e.groups() == (1, 2)
    with pytest.raises(sfhe.SfheError):
        e.groups_host(0, 2, sfhe.ThreadComm(2))  # already set
    e2 = sfhe.Engine("oracle", mult_depth=2, ring_dim=1 << 12)
    with pytest.raises(sfhe.SfheError):  # after key generation
        e2.groups_host(0, 2, sfhe.ThreadComm(2))
    with pytest.raises(sfhe.SfheError):  # the oracle has no RCCL
        e2.groups_rccl(0, 2, bytes(128))


@pytest.mark.parametrize("world,tail", [(3, 4), (2, 0), (4, 16)])
def test_sliced_keys_oracle(oracle_lib, world, tail, monkeypatch):
    """each rank keeps only its slice of every switching key --
    the Q rows of the replicated tail, its own dealt Q rows above it and the P
    rows (sfp_key_geom) -- and every op stays bit-identical to the unsharded
    context (the sharded tests above run with sliced keys by default)."""
    monkeypatch.setenv("SFHE_SHARD_TAIL", str(tail))
    ref_e = sfhe.Engine("oracle", **OPS_KW)
    info = ref_e.info()
    nq, npr = info["num_q"], info["num_p"]
    assert ref_e.key_rows() == nq + npr
    ref = ops_program(ref_e)

    def prog(e):
        out = ops_program(e)
        out["key_rows"] = np.array([e.key_rows()])
        return out

    outs = sfhe.run_sharded_threads("oracle", world, prog, **OPS_KW)
    t = min(tail, nq)
    for r in range(world):
        want = t + sum(1 for p in range(t, nq) if p % world == r) + npr
        assert int(outs[r].pop("key_rows")[0]) == want
        assert want < nq + npr or t == nq  # (a tail over every limb: nothing to slice)
        compare(ref, outs[r])
    monkeypatch.setenv("SFHE_KEY_SLICE", "0")  # whole keys: the same residues
    outs = sfhe.run_sharded_threads("oracle", world, prog, **OPS_KW)
    for r in range(world):
        assert int(outs[r].pop("key_rows")[0]) == nq + npr
        compare(ref, outs[r])
