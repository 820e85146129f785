"""Limb sharding on the HIP product: W ranks as threads sharing device 0
(each its own context and streams), exchanging limbs through the host
transport (ThreadComm), must reproduce the unsharded HIP residues bit for
bit -- every op at W = 2, 3 and a whole DirectSort<8> at W = 2.  The RCCL
transport is exercised by the communicator set-up (a one-rank communicator;
RCCL does not place two ranks on one GPU) and by bench.py --shard on a node.
"""
import numpy as np
import pytest

import sfhe
from oracle import slotsim
from test_shard import OPS_KW, compare, ops_program, sort_program

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_ops_bitexact_hip(hip_lib, world):
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


@pytest.mark.parametrize("N,logn,world", [(64, 15, 3), (128, 16, 4), (256, 17, 2), (256, 17, 3), (256, 17, 4)])
def test_sharded_sort_large_bitexact_hip(hip_lib, N, logn, world):
    """Larger rings and limb counts (31 Q limbs at N=128), more ranks, and
    BASELINE config 5's sort itself (DirectSort<256> at ring 2^17, 35 Q
    limbs) at W = 2, 3, 4."""
    depth, rots = sfhe.direct_sort_params(N, "hip")
    kw = dict(mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots, seed=4099)
    ref = sort_program(sfhe.Engine("hip", **kw), N)
    assert np.max(np.abs(ref["dec"][:N] - np.sort(slotsim.input_vector(N)))) < 0.01
    outs = sfhe.run_sharded_threads("hip", world, lambda e: sort_program(e, N), **kw)
    for r in range(world):
        compare(ref, outs[r])


RCCL_SCRIPT = r"""
import sys
sys.path.insert(0, {py!r}); sys.path.insert(0, {tests!r})
import sfhe
from oracle import slotsim
from test_shard import OPS_KW, compare, ops_program
uid = sfhe.comm_uid("hip")
assert uid is not None and len(uid) == 128
e = sfhe.Engine("hip", shard=("rccl", 0, 1, uid), **OPS_KW)
ref = sfhe.Engine("hip", **OPS_KW)
compare(ops_program(ref), ops_program(e))
e.close(); ref.close()
print("RCCL communicator OK")
"""


def test_rccl_single_rank_communicator(hip_lib):
    """sfhe_comm_uid + sfhe_shard_rccl (ncclCommInitRank) on one rank, then the
    op program through the RCCL-configured context.  Own process: RCCL's
    threads and the HIP runtime are torn down with it."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = RCCL_SCRIPT.format(py=os.path.join(os.path.dirname(here), "sorting-fhe_amd", "python"), tests=here)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "RCCL communicator OK" in r.stdout
