"""The Chebyshev PS recursion's q / r subtrees on lanes (SFHE_PS_LANES,
core/chebyshev.cpp): a sort phase that runs one batch per GPU (config 3, a
batch-split rank) evaluates its placement series on up to four lanes.  Same
operations on other streams: the result is bit-identical.  The knob is read
once per process, so each variant runs in its own process."""
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
PY = os.path.join(os.path.dirname(HERE), "sorting-fhe_amd", "python")

CODE = r"""
import sys
sys.path[:0] = [{py!r}, {tests!r}, {root!r}]
import numpy as np
import sfhe
from oracle import slotsim
N, logn = {N}, {logn}
d, r = sfhe.direct_sort_params(N, {backend!r})
e = sfhe.Engine({backend!r}, mult_depth=d, ring_dim=1 << logn, batch_size=N, rotations=r, seed=5)
e.set_quiet(True)
s = e.sorter(N)
x = slotsim.input_vector(N)
outs = [s.sort(e.encrypt(x.tolist()), *slotsim.default_sign_config(N)) for _ in range({reps})]
err = float(np.max(np.abs(np.array(e.decrypt(outs[-1]))[:N] - np.sort(x))))
assert err < 0.01, err
np.save({path!r}, np.stack([o.download() for o in outs]))
"""


def run(backend, N, logn, lanes, path, reps=1):
    env = dict(os.environ)
    env.pop("SFHE_PS_LANES", None)
    if lanes:
        env["SFHE_PS_LANES"] = str(lanes)
    code = CODE.format(py=PY, tests=HERE, root=os.path.dirname(HERE), N=N, logn=logn, backend=backend,
                       path=str(path), reps=reps)
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=900)
    return np.load(str(path) + ".npy" if not str(path).endswith(".npy") else str(path))


def test_ps_lanes_bitexact_oracle(oracle_lib, tmp_path):
    """DirectSort<64> at ring 2^13: one batch per phase, so the placement's
    series runs on 4 lanes with the knob."""
    a = run("oracle", 64, 13, 0, tmp_path / "a.npy")
    b = run("oracle", 64, 13, 4, tmp_path / "b.npy")
    assert np.array_equal(a, b)


@pytest.mark.gpu
def test_ps_lanes_bitexact_hip(hip_lib, tmp_path):
    """Config 3 (DirectSort<128> @ 2^16, one batch): eager, captured and
    replayed sorts with the series on 4 lanes, bit-identical to one lane."""
    a = run("hip", 128, 16, 0, tmp_path / "a.npy", reps=3)
    b = run("hip", 128, 16, 4, tmp_path / "b.npy", reps=3)
    assert np.array_equal(a, b)
