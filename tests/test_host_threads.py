"""The sort with each lane issued by its own host thread (SFHE_HOST_THREADS=1,
the reference's OpenMP batch loop, /root/reference/src/sort_algo.h:438-492)
against the oracle, residue for residue.  Pins the device pool's cross-thread
frees during another lane's batched ops (core/context.cpp ~DeviceBuffer /
EndBatch: a block freed by one lane's thread while the other lane's batch is
open goes through the lane / region checks, not onto the batching lane's free
list).  The knob is read once per process, so the HIP sort runs in a child
process and hands its residues back as a .npy file."""
import os
import subprocess
import sys

import numpy as np
import pytest

import sfhe
from oracle import slotsim

HERE = os.path.dirname(os.path.abspath(__file__))
PY = os.path.join(os.path.dirname(HERE), "sorting-fhe_amd", "python")

# N = 64 at ring 2^12: N^2 = 4096 > 2048 slots, so two batches on two lanes
N, RING, SEED = 64, 1 << 12, 4321

CHILD = """
import sys, numpy as np
sys.path[:0] = sys.argv[1:3]
import sfhe
from oracle import slotsim
N, ring, seed, out, backend = int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), sys.argv[6], sys.argv[7]
depth, rots = sfhe.direct_sort_params(N, backend)
e = sfhe.Engine(backend, mult_depth=depth, ring_dim=ring, batch_size=N, seed=seed, rotations=rots)
e.set_quiet(True)
x = slotsim.input_vector(N).tolist()
r = e.sorter(N).sort(e.encrypt(x), *slotsim.default_sign_config(N))
np.save(out, r.download())
print("max_err", float(np.max(np.abs(np.array(e.decrypt(r)) - np.sort(x)))))
"""


def _child_sort(backend, out, threads):
    env = dict(os.environ, SFHE_HOST_THREADS=threads)
    r = subprocess.run([sys.executable, "-u", "-c", CHILD, os.path.dirname(HERE), PY, str(N), str(RING),
                        str(SEED), out, backend], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    err = float(r.stdout.split("max_err")[-1])
    assert err < 0.01, err
    return np.load(out)


def _same(got, ref):
    assert got.shape == ref.shape
    bad = int(np.count_nonzero(got != ref))
    assert bad == 0, f"{bad} of {ref.size} residues differ"


@pytest.mark.gpu
def test_host_thread_lanes_bitexact(hip_lib, oracle_lib, tmp_path):
    got = _child_sort("hip", str(tmp_path / "hip.npy"), "1")
    depth, rots = sfhe.direct_sort_params(N, "hip")
    o = sfhe.Engine("oracle", mult_depth=depth, ring_dim=RING, batch_size=N, seed=SEED, rotations=rots)
    o.set_quiet(True)
    x = slotsim.input_vector(N).tolist()
    _same(got, o.sorter(N).sort(o.encrypt(x), *slotsim.default_sign_config(N)).download())


def test_host_thread_lanes_oracle(oracle_lib, tmp_path):
    """The host-side half on the CPU: the oracle build (same context.cpp pool,
    lane and batch code) with one host thread per lane gives the residues of
    the default single issuing thread."""
    _same(_child_sort("oracle", str(tmp_path / "t.npy"), "1"), _child_sort("oracle", str(tmp_path / "s.npy"), "0"))
