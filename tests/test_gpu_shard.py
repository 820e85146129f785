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


def test_rccl_single_rank_communicator(hip_lib):
    uid = sfhe.comm_uid("hip")
    assert uid is not None and len(uid) == 128
    e = sfhe.Engine("hip", shard=("rccl", 0, 1, uid), **OPS_KW)
    ref = sfhe.Engine("hip", **OPS_KW)
    compare(ops_program(ref), ops_program(e))
