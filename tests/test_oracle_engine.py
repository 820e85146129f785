"""The CKKS engine's host layer on the CPU oracle backend (no GPU).

These exercise the same host code the product runs (context, keys, encoder,
key switching, Chebyshev PS, sign, DirectSort) with the C oracle prims, at
ring sizes the oracle finishes in seconds.  Bars are the reference tests'
own: CompareTest +-0.1, SignTest +-0.1 + sign agreement, RotationTest 1e-6,
DirectSortTest < 0.01 and level == multDepth.
"""
import json
import os

import numpy as np
import pytest

import sfhe
from oracle import cheb, slotsim

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF = json.load(open(os.path.join(GOLD, "reference_params.json")))


def test_encrypt_decrypt_and_ext_precision(oracle_lib):
    x = np.linspace(-1, 1, 64)
    errs = {}
    for sc in ("FLEXIBLEAUTO", "FLEXIBLEAUTOEXT"):
        e = sfhe.Engine("oracle", mult_depth=3, ring_dim=1 << 13, batch_size=64, scaling=sc)
        ct = e.encrypt(x.tolist())
        assert ct.level == 0 and ct.slots == 64
        errs[sc] = np.max(np.abs(np.array(e.decrypt(ct)) - x))
    assert errs["FLEXIBLEAUTO"] < 2 ** -20
    assert errs["FLEXIBLEAUTOEXT"] < errs["FLEXIBLEAUTO"] / 4  # fresh noise divided by q_ext


def test_arithmetic_and_levels(oracle_lib):
    e = sfhe.Engine("oracle", mult_depth=6, ring_dim=1 << 12, batch_size=16)
    rng = np.random.default_rng(3)
    a, b = rng.uniform(-1, 1, 16), rng.uniform(-1, 1, 16)
    ca, cb = e.encrypt(a.tolist()), e.encrypt(b.tolist())
    chk = lambda ct, ref, tol=1e-5: np.testing.assert_allclose(e.decrypt(ct), ref, atol=tol)
    chk(e.add(ca, cb), a + b)
    chk(e.sub(ca, cb), a - b)
    m = e.mult(ca, cb)
    assert m.level == 1
    chk(m, a * b)
    chk(e.mult_const(ca, -2.5), -2.5 * a)
    chk(e.add_const(ca, 0.25), a + 0.25)
    chk(e.mult_plain(ca, list(range(16)), 16), a * np.arange(16), 1e-4)
    # mixed levels align automatically
    chk(e.add(m, ca), a * b + a)
    sq = e.mult(e.mult(m, m), m)
    assert sq.level == 3
    chk(sq, (a * b) ** 3)


@pytest.mark.parametrize("r", [1, 2, 3, 5, 8, -1, 15])
def test_rotation(oracle_lib, r):
    """RotationTest (tests/RotationTest.cpp:73-170): left rotation, 1e-6."""
    e = sfhe.Engine("oracle", mult_depth=2, ring_dim=1 << 12, batch_size=16,
                    scaling_mod_size=50, rotations=[1, 2, 3, 5, 8, -1, 15])
    x = np.arange(16) / 16.0
    got = np.array(e.decrypt(e.rotate(e.encrypt(x.tolist()), r)))
    np.testing.assert_allclose(got, np.roll(x, -r), atol=1e-6)


@pytest.mark.parametrize("lazy_product", [False, True])
def test_rotate_sum(oracle_lib, lazy_product):
    """EvalRotateSum (output aggregation: one ModDown for all terms) equals the
    sum of the individual rotations, on canonical inputs and on lazily
    rescaled products (the vecRotsOpt / blind-rotation giant steps)."""
    rots = [1, 2, 3, 5, 8, 0, 15]
    e = sfhe.Engine("oracle", mult_depth=3, ring_dim=1 << 12, batch_size=16,
                    scaling_mod_size=50, rotations=[r for r in rots if r % 16])
    rng = np.random.default_rng(11)
    xs = [rng.uniform(-1, 1, 16) for _ in rots]
    cts = [e.encrypt(x.tolist()) for x in xs]
    if lazy_product:
        cts = [e.mult_const(c, 0.5) for c in cts]
        xs = [0.5 * x for x in xs]
    got = e.rotate_sum(cts, rots)
    ref = sum(np.roll(x, -r) for x, r in zip(xs, rots))
    np.testing.assert_allclose(e.decrypt(got), ref, atol=1e-6)
    sep = cts[0]
    for c, r in zip(cts, rots):
        t = e.rotate(c, r)
        sep = t if c is cts[0] else e.add(sep, t)
    assert got.level == sep.level
    np.testing.assert_allclose(e.decrypt(got), e.decrypt(sep), atol=1e-6)


def test_compare_reference_vectors(oracle_lib):
    """tests/CompareTest.cpp:13-63, verbatim parameters."""
    t = REF["compare_test"]
    e = sfhe.Engine("oracle", mult_depth=t["mult_depth"], ring_dim=1 << t["ring_dim_log2"],
                    batch_size=len(t["a"]), scaling_mod_size=t["scaling_mod_size"])
    out = e.compare(e.encrypt(t["a"]), e.encrypt(t["b"]), *t["composite_sign_config"])
    np.testing.assert_allclose(e.decrypt(out), t["expected"], atol=t["tolerance"])


@pytest.mark.parametrize("cfg", [(3, 2, 2), (4, 3, 3)])
def test_sign_matches_slot_simulation(oracle_lib, cfg):
    """SignTest shape (tests/SignTest.cpp:17-121) at ring 2^12, depth 30, scale 50."""
    e = sfhe.Engine("oracle", mult_depth=30, ring_dim=1 << 12, batch_size=512, scaling_mod_size=50)
    rng = np.random.default_rng(5)
    x = rng.uniform(2 ** -5, 1, 512) * rng.choice([-1, 1], 512)
    out = e.sign(e.encrypt(x.tolist()), *cfg)
    got = np.array(e.decrypt(out))
    assert out.level == slotsim.sign_depth(*cfg)
    assert np.all(np.sign(got) == np.sign(x))
    assert np.max(np.abs(got - slotsim.composite_sign(x, *cfg))) < 1e-4


def test_chebyshev_ps(oracle_lib):
    """EvalChebyshevSeriesPS on the doubled sinc of N=8 (degree 70, depth 7)."""
    c = cheb.doubled_sinc_coeffs(8)
    e = sfhe.Engine("oracle", mult_depth=9, ring_dim=1 << 12, batch_size=64, scaling_mod_size=50)
    x = np.linspace(-0.99, 0.99, 64)
    out = e.chebyshev(e.encrypt(x.tolist()), c.tolist())
    assert out.level == cheb.ps_depth(len(c) - 1)
    np.testing.assert_allclose(e.decrypt(out), cheb.cheb_eval(c, x), atol=1e-6)


@pytest.mark.parametrize("N", [4, 8, 16])
def test_direct_sort(oracle_lib, N):
    """DirectSortTest (tests/DirectSortTest.cpp:96-210) on the oracle at ring 2^12."""
    depth, rots = sfhe.direct_sort_params(N, "oracle")
    e = sfhe.Engine("oracle", mult_depth=depth, ring_dim=1 << 12, batch_size=N, rotations=rots,
                    seed=20251205 + N)
    e.set_quiet(True)
    x = slotsim.input_vector(N)
    out = e.sorter(N).sort(e.encrypt(x.tolist()), *slotsim.default_sign_config(N))
    assert out.level == depth
    got = np.array(e.decrypt(out))
    assert np.max(np.abs(got - np.sort(x))) < 0.01
    sim, _ = slotsim.direct_sort(x, N, 1 << 12)
    assert np.max(np.abs(got - sim)) < 2 ** -12


def test_sort_rank_and_place_split(oracle_lib):
    """constructRank then rotationIndexCheckN == sort (sort_algo.h:752-774)."""
    N = 8
    depth, rots = sfhe.direct_sort_params(N, "oracle")
    e = sfhe.Engine("oracle", mult_depth=depth, ring_dim=1 << 12, batch_size=N, rotations=rots)
    e.set_quiet(True)
    x = slotsim.input_vector(N)
    s = e.sorter(N)
    ct = e.encrypt(x.tolist())
    rank = s.rank(ct, *slotsim.default_sign_config(N))
    np.testing.assert_allclose(e.decrypt(rank), np.argsort(np.argsort(x)), atol=1e-3)
    out = s.place(rank, ct)
    np.testing.assert_allclose(e.decrypt(out), np.sort(x), atol=0.01)


def test_depth_exhaustion_is_an_error(oracle_lib):
    e = sfhe.Engine("oracle", mult_depth=1, ring_dim=1 << 12, batch_size=4)
    c = e.encrypt([0.5, 0.5, 0.5, 0.5])
    c2 = e.mult(c, c)
    with pytest.raises(sfhe.SfheError):
        e.mult(c2, c2)


def test_debug_sort_repeats(oracle_lib, capfd):
    """A debug sorter (DebugEncryption's PRINT_PT decrypts inside sort(),
    src/sort_algo.h:755-770) sorted three times: on the oracle the graph
    capture the second sort attempts is refused, the sorter falls back to
    eager sorts (DirectSort::sortDebug), and every sort returns the same
    ciphertext and prints the same sections; the second and third the same
    text."""
    N = 8
    depth, rots = sfhe.direct_sort_params(N, "oracle")
    e = sfhe.Engine("oracle", mult_depth=depth, ring_dim=1 << 12, batch_size=N, rotations=rots, seed=7)
    s = e.sorter(N, debug=True)
    x = slotsim.input_vector(N)
    ct = e.encrypt(x.tolist())
    cfg = slotsim.default_sign_config(N)
    outs, texts = [], []
    for _ in range(3):
        capfd.readouterr()
        outs.append(s.sort(ct, *cfg).download())
        texts.append(capfd.readouterr().out)
    for t in texts:
        assert t.count("Constructed Rank") == 1 and t.count("Final Output") == 1
    assert np.array_equal(outs[0], outs[1]) and np.array_equal(outs[1], outs[2])
    assert texts[1] == texts[2]
    np.testing.assert_allclose(np.array(e.decrypt(e.sorter(N).sort(ct, *cfg)))[:N], np.sort(x), atol=0.01)


WAVES_CHILD = r"""
import hashlib, sys
import sfhe
from oracle import slotsim
N = 16
depth, rots = sfhe.direct_sort_params(N, "oracle")
e = sfhe.Engine("oracle", mult_depth=depth, ring_dim=1 << 12, batch_size=N, rotations=rots, seed=5)
e.set_quiet(True)
o = e.sorter(N).sort(e.encrypt(slotsim.input_vector(N).tolist()), *slotsim.default_sign_config(N))
e2 = sfhe.Engine("oracle", mult_depth=30, ring_dim=1 << 12, batch_size=8, scaling_mod_size=50, seed=6)
s = e2.sign(e2.encrypt([0.3, -0.2, 0.05, -0.7]), 4, 3, 3)
print(hashlib.sha256(o.download().tobytes() + s.download().tobytes()).hexdigest())
"""


def test_ps_waves_same_values(oracle_lib):
    """The level-synchronous Chebyshev PS and polynomial powers (EvalMultMany
    waves, the default) against the recursive order (SFHE_PS_WAVES=0): the
    same operations on the same operands, so the same residues -- a whole
    DirectSort<16> and a CompositeSign(4,3,3) (knob read once per process:
    child processes)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(root, "sorting-fhe_amd", "python"), root]))
    out = []
    for w in ("1", "0"):
        p = subprocess.run([sys.executable, "-c", WAVES_CHILD], env=dict(env, SFHE_PS_WAVES=w), capture_output=True,
                           text=True, timeout=600)
        assert p.returncode == 0, p.stderr[-2000:]
        out.append(p.stdout.strip().splitlines()[-1])
    assert out[0] == out[1]
