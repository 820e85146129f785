"""GPU acceptance at the BASELINE.json configurations (DirectSortTest shape).

Oracle: the float64 slot-level re-enactment (oracle/slotsim.py) and std::sort
of the input.  Bars:
  * the reference's own gate: max |out - sort(x)| < 0.01 and final level ==
    multDepth (tests/DirectSortTest.cpp:140-141, :194), at every size the
    reference's DirectSortTest instantiates at ring 2^17 / HEStd_128_classic
    (DirectSortTest.cpp:35-37, :203-208: N = 256, 512, 1024 here);
  * a measured bar (~3x the error measured on MI355X, DESIGN.md §2,
    tools/precision_table.py): with the engine's precision choices (exact
    ModDown, lazy rescaling, the self comparison moved off the sign's steep
    point, the doubled sinc in the rebased variable) the rank is within
    ~1e-6 of exact and the sort is limited by the placement's
    Paterson-Stockmeyer noise; test_precision_attribution measures each
    choice against the reference's order of operations.
"""
import numpy as np
import pytest

import sfhe
from oracle import slotsim

pytestmark = pytest.mark.gpu


def run_sort(N, logn, secure=False, debug=False, scale_bits=40):
    depth, rots = sfhe.direct_sort_params(N, "hip")
    e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, secure=secure,
                    rotations=rots, seed=20251205 + N, scaling_mod_size=scale_bits)
    e.set_quiet(True)
    x = slotsim.input_vector(N)
    s = e.sorter(N, debug=debug)
    out = s.sort(e.encrypt(x.tolist()), *slotsim.default_sign_config(N))
    return e, x, out, depth


@pytest.mark.parametrize("N,logn,secure,scale_bits,tol", [
    (8, 17, True, 40, 1e-6),       # config 1 (DirectSortTest N=8: ring 2^17, 128-bit; measured 2.3e-7)
    (128, 16, False, 40, 3e-5),    # config 3 (measured 1.1e-5, approximation floor 9.6e-6)
    (256, 16, False, 40, 8e-5),    # metric config (measured 2.6e-5)
    (256, 16, False, 50, 2 ** -19),  # same circuit, 50-bit scale: noise-limited
    (256, 17, True, 40, 1.2e-4),   # DirectSortTest N=256 / config 5 shape on one GPU (4.0e-5)
    (512, 17, True, 40, 3e-4),     # DirectSortTest N=512 (9.8e-5)
    (1024, 17, True, 40, 7e-4),    # DirectSortTest N=1024 (2.2e-4)
])
def test_direct_sort(N, logn, secure, scale_bits, tol):
    e, x, out, depth = run_sort(N, logn, secure, scale_bits=scale_bits)
    assert out.level == depth
    got = np.array(e.decrypt(out))
    exact = np.sort(x)
    err = np.max(np.abs(got - exact))
    sim, _ = slotsim.direct_sort(x, N, 1 << logn)
    print(f"N={N} ring=2^{logn} max err {err:.3g} (log2 {np.log2(err):.2f}); vs slotsim "
          f"{np.max(np.abs(got - sim)):.3g}")
    assert err < 0.01
    assert np.max(np.abs(got - sim)) < tol


PREC_CHILD = r"""
import json, numpy as np, sfhe
from oracle import slotsim
N, logn = 256, 16
depth, rots = sfhe.direct_sort_params(N, "hip")
e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots, seed=20251205 + N)
e.set_quiet(True)
x = slotsim.input_vector(N)
s = e.sorter(N)
ct = e.encrypt(x.tolist())
r = s.rank(ct, *slotsim.default_sign_config(N))
rank = np.array(e.decrypt(r))
out = s.place(r, ct)
assert out.level == depth
print(json.dumps({"rank": float(np.max(np.abs(rank - np.argsort(np.argsort(x))))),
                  "sort": float(np.max(np.abs(np.array(e.decrypt(out)) - np.sort(x))))}))
"""


def _prec(env):
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    child = dict(os.environ, **env)
    child["PYTHONPATH"] = os.pathsep.join([os.path.join(root, "sorting-fhe_amd", "python"), root])
    p = subprocess.run([sys.executable, "-c", PREC_CHILD], cwd=root, env=child, capture_output=True, text=True,
                       timeout=110)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


def test_precision_attribution():
    """Metric config (N=256 @ 2^16, 40-bit scale): the rank's and the sort's
    error with each of the engine's precision choices switched off in turn
    (each knob is read once per process, so every variant is a child
    process).  DESIGN.md §2 tabulates the same measurement."""
    base = _prec({})
    no_off = _prec({"SFHE_SELF_OFFSET": "0"})   # self comparison at the sign's steep point (reference)
    no_lazy = _prec({"SFHE_LAZY": "0"})          # every product rescaled at once
    no_reb = _prec({"SFHE_SINC_REBASE": "0"})    # doubled sinc in the reference's variable
    print(f"default {base}\nno self offset {no_off}\nno lazy rescaling {no_lazy}\nno sinc rebase {no_reb}")
    assert base["rank"] < 5e-6 and base["sort"] < 8e-5       # measured 1.1e-6 / 2.6e-5
    assert no_off["rank"] > 20 * base["rank"]                 # ~1e-4: the self term's sign gain
    # lazy rescaling moves the sort's error by less than its run-to-run
    # spread here (2.6e-5 .. 4.4e-5 across op orders); it matters for hybrid1
    # (test_hybrid1.py's 1.8e-6 gate).  Both stay inside the gate:
    assert no_lazy["rank"] < 5e-6 and no_lazy["sort"] < 8e-5
    assert no_reb["sort"] > 20 * base["sort"]                 # giant steps at +-1 on the hits


def test_rank_matches_oracle():
    N, logn = 64, 16
    depth, rots = sfhe.direct_sort_params(N, "hip")
    e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots)
    x = slotsim.input_vector(N)
    s = e.sorter(N)
    cfg = slotsim.default_sign_config(N)
    rank = np.array(e.decrypt(s.rank(e.encrypt(x.tolist()), *cfg)))
    sim = slotsim.construct_rank(x, N, 1 << logn, cfg)
    assert np.max(np.abs(rank - np.argsort(np.argsort(x)))) < 1e-3
    assert np.max(np.abs(rank - sim)) < 1e-4


@pytest.mark.parametrize("cfg", [(4, 3, 3), (3, 4, 2)])
def test_sign_config2(cfg):
    """BASELINE config 2: sign() on one ciphertext at ring 2^15, depth 30, scale 50."""
    e = sfhe.Engine("hip", mult_depth=30, ring_dim=1 << 15, batch_size=1 << 14, scaling_mod_size=50)
    rng = np.random.default_rng(99)
    mag = rng.uniform(2 ** -7, 1.0, 1 << 14)
    x = mag * rng.choice([-1.0, 1.0], size=mag.size)
    out = e.sign(e.encrypt(x.tolist()), *cfg)
    got = np.array(e.decrypt(out))
    ref = slotsim.composite_sign(x, *cfg)
    assert out.level == slotsim.sign_depth(*cfg)
    assert np.max(np.abs(got - ref)) < 1e-3
    assert np.all(np.sign(got) == np.sign(x))


def test_compare_reference_vectors():
    """tests/CompareTest.cpp:13-63: depth 50, scale 59, ring 2^12;
    compare({1,5,3,4},{2,4,3,3}) with CompositeSign(4,3,3) = {0,1,0.5,1} +- 0.1."""
    e = sfhe.Engine("hip", mult_depth=50, ring_dim=1 << 12, batch_size=4, scaling_mod_size=59)
    a = e.encrypt([1.0, 5.0, 3.0, 4.0])
    b = e.encrypt([2.0, 4.0, 3.0, 3.0])
    got = np.array(e.decrypt(e.compare(a, b, 4, 3, 3)))
    assert np.max(np.abs(got - np.array([0, 1, 0.5, 1]))) < 0.1


def test_pool_is_steady_across_sorts():
    """Repeated sorts reuse the device pool: lanes take lane 0's pre-fork free
    blocks, so the pool does not grow per sort (it once grew ~6.5 GB per sort at
    N=256 until HBM ran out and a full release stalled a sort for seconds)."""
    N, logn = 64, 14
    depth, rots = sfhe.direct_sort_params(N, "hip")
    e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots)
    e.set_quiet(True)
    s = e.sorter(N)
    ct = e.encrypt(slotsim.input_vector(N).tolist())
    cfg = slotsim.default_sign_config(N)
    sizes = []
    for _ in range(6):
        o = s.sort(ct, *cfg)
        e.sync()
        del o
        sizes.append(e.pool_bytes())
    assert sizes[-1] - sizes[2] <= 0.05 * sizes[2], sizes  # lane timing may vary reuse slightly
