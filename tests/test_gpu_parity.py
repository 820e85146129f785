"""GPU parity: the HIP product against the CPU oracle, bit for bit.

Both libraries run the same host CKKS layer with the same seed, so keys,
encryptions and every homomorphic result are identical integers iff the
gfx950 kernels compute exactly what the plain-C oracle (oracle/prims_ref.c,
independent 128-bit '%' arithmetic) computes.  Sizes are chosen so the
oracle finishes in seconds.
"""
import numpy as np
import pytest

import sfhe
from oracle import cheb, slotsim

pytestmark = pytest.mark.gpu


def pair(ring, depth, batch, rotations=(), scaling=40, secure=False, seed=1234):
    kw = dict(mult_depth=depth, ring_dim=ring, batch_size=batch, scaling_mod_size=scaling,
              secure=secure, seed=seed, rotations=rotations)
    return sfhe.Engine("hip", **kw), sfhe.Engine("oracle", **kw)


def same(a, b):
    x, y = a.download(), b.download()
    assert x.shape == y.shape
    bad = int(np.count_nonzero(x != y))
    assert bad == 0, f"{bad} of {x.size} residues differ"


def test_backend_is_hip(hip_lib, oracle_lib):
    assert hip_lib.sfhe_backend() == b"hip-gfx950"
    assert oracle_lib.sfhe_backend() == b"oracle-c"


@pytest.mark.parametrize("logn", [12, 13, 15, 16, 17])
def test_encrypt_bitexact(hip_lib, oracle_lib, logn):
    depth = 4 if logn < 17 else 2
    g, o = pair(1 << logn, depth, 8)
    v = [0.5, -0.25, 0.125, 0.75, -1.0, 0.3, 0.2, 0.1]
    cg, co = g.encrypt(v), o.encrypt(v)
    same(cg, co)
    assert np.allclose(g.decrypt(cg), v, atol=1e-6)


def test_ops_bitexact(hip_lib, oracle_lib):
    g, o = pair(1 << 13, 8, 16, rotations=[1, 3, -2, 8])
    rng = np.random.default_rng(7)
    a = rng.uniform(-1, 1, 16).tolist()
    b = rng.uniform(-1, 1, 16).tolist()
    ca = (g.encrypt(a), o.encrypt(a))
    cb = (g.encrypt(b), o.encrypt(b))
    ops = {
        "add": lambda e, x, y: e.add(x, y),
        "sub": lambda e, x, y: e.sub(x, y),
        "mult": lambda e, x, y: e.mult(x, y),
        "mult_const": lambda e, x, y: e.mult_const(x, -3.75),
        "add_const": lambda e, x, y: e.add_const(x, 0.5),
        "mult_plain": lambda e, x, y: e.mult_plain(x, list(range(16)), 16),
        "rotate1": lambda e, x, y: e.rotate(x, 1),
        "rotate-2": lambda e, x, y: e.rotate(x, -2),
        "rotate8": lambda e, x, y: e.rotate(x, 8),
        "mixed_level": lambda e, x, y: e.add(e.mult(x, y), x),
    }
    for name, f in ops.items():
        rg, ro = f(g, ca[0], cb[0]), f(o, ca[1], cb[1])
        same(rg, ro)
    # correctness of one of them against plaintext
    got = np.array(g.decrypt(g.mult(ca[0], cb[0])))
    assert np.max(np.abs(got - np.array(a) * np.array(b))) < 1e-6


def test_chebyshev_and_sign_bitexact(hip_lib, oracle_lib):
    g, o = pair(1 << 12, 30, 8, scaling=50)
    v = [0.02, -0.02, 0.01, -0.01, 0.009, -0.009, 1, -1]
    cg, co = g.encrypt(v), o.encrypt(v)
    sg, so = g.sign(cg, 4, 3, 3), o.sign(co, 4, 3, 3)
    same(sg, so)
    assert sg.level == 27
    got = np.array(g.decrypt(sg))
    assert np.all(np.sign(got) == np.sign(v)) and np.max(np.abs(np.abs(got) - 1)) < 0.1
    x = np.linspace(-0.9, 0.9, 8).tolist()
    c = cheb.doubled_sinc_coeffs(4)
    hg = g.chebyshev(g.encrypt(x), c.tolist())
    ho = o.chebyshev(o.encrypt(x), c.tolist())
    same(hg, ho)
    assert np.max(np.abs(np.array(g.decrypt(hg)) - cheb.cheb_eval(c, np.array(x)))) < 1e-5


@pytest.mark.parametrize("N", [4, 8, 16])
def test_direct_sort_bitexact(hip_lib, oracle_lib, N):
    depth, rots = sfhe.direct_sort_params(N, "hip")
    g, o = pair(1 << 12, depth, N, rotations=rots)
    x = slotsim.input_vector(N).tolist()
    cfg = slotsim.default_sign_config(N)
    outs = []
    for e in (g, o):
        e.set_quiet(True)
        s = e.sorter(N)
        outs.append(s.sort(e.encrypt(x), *cfg))
    same(outs[0], outs[1])
    assert outs[0].level == depth
    got = np.array(g.decrypt(outs[0]))
    assert np.max(np.abs(got - np.sort(x))) < 0.01


@pytest.mark.gpu
@pytest.mark.parametrize("logn", [10, 11])
def test_small_ring_bitexact(hip_lib, oracle_lib, logn):
    """Rings below 2^12 (k_ntt_small: one single-pass block per row) -- the
    ring the reference's k-way unit tests use (tests/k-way/MaskingTest.cpp:15,
    tests/KWaySortTest.cpp:24): encrypt, multiply, rotate, rescale bit for bit
    against the oracle."""
    raw = {}
    for backend in ("hip", "oracle"):
        e = sfhe.Engine(backend, mult_depth=4, ring_dim=1 << logn, batch_size=8, rotations=[1, -2],
                        seed=77, device=0)
        e.set_quiet(True)
        a = e.encrypt([0.5, -0.25, 0.125, 0.75, 0.1, 0.2, 0.3, 0.4])
        b = e.rotate(e.mult(a, a), 1)
        c = e.rotate(e.mult_const(b, 0.5), -2)
        raw[backend] = c.download()
        got = np.array(e.decrypt(c))[:8]
        x = np.array([0.5, -0.25, 0.125, 0.75, 0.1, 0.2, 0.3, 0.4]) ** 2 * 0.5
        assert np.allclose(got, np.roll(np.roll(x, -1), 2), atol=1e-4), (backend, got)
    assert np.array_equal(raw["hip"], raw["oracle"])
