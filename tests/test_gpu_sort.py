"""GPU acceptance at the BASELINE.json configurations (DirectSortTest shape).

Oracle: the float64 slot-level re-enactment (oracle/slotsim.py) and std::sort
of the input.  Bars:
  * the reference's own gate: max |out - sort(x)| < 0.01 and final level ==
    multDepth (tests/DirectSortTest.cpp:140-141, :194), at every size the
    reference's DirectSortTest instantiates at ring 2^17 / HEStd_128_classic
    (DirectSortTest.cpp:35-37, :203-208: N = 256, 512, 1024 here);
  * a measured bar (4x the error measured on MI355X): the
    rank's CKKS noise (the self comparison's sign gain ~2^11 at d = 0) is
    what remains once the placement evaluates the doubled sinc in the
    rebased variable; evaluated as the reference orders it (SFHE_SINC_REBASE
    =0) the placement adds ~2^-6.7 at N=256 (test_precision_attribution).
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
    (8, 17, True, 40, 2 ** -12),     # config 1 (DirectSortTest N=8: ring 2^17, 128-bit)
    (128, 16, False, 40, 3e-4),      # config 3 (measured 7.4e-5)
    (256, 16, False, 40, 1.5e-3),    # metric config (measured 3.7e-4)
    (256, 16, False, 50, 2 ** -19),  # same circuit, 50-bit scale (measured 4.9e-7): noise-limited
    (256, 17, True, 40, 3.5e-3),     # DirectSortTest N=256 / config 5 shape on one GPU (8.3e-4)
    (512, 17, True, 40, 4e-3),       # DirectSortTest N=512 (9.3e-4)
    (1024, 17, True, 40, 7.5e-3),    # DirectSortTest N=1024 (1.8e-3)
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


def test_precision_attribution(monkeypatch):
    """Metric config (N=256 @ 2^16, 40-bit scale), stage by stage against
    slotsim: the rank's error, the sort's error with the placement's doubled
    sinc evaluated in the rebased variable (default), and as the reference
    orders it (SFHE_SINC_REBASE=0: every PS giant step T_{2^i} sits at +-1 on
    the hits z = 0, so noise grows 4x per doubling)."""
    N, logn = 256, 16
    depth, rots = sfhe.direct_sort_params(N, "hip")
    e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots,
                    seed=20251205 + N)
    e.set_quiet(True)
    x = slotsim.input_vector(N)
    cfg = slotsim.default_sign_config(N)
    s = e.sorter(N)
    ct = e.encrypt(x.tolist())
    r = s.rank(ct, *cfg)
    rank = np.array(e.decrypt(r))
    sim = slotsim.construct_rank(x, N, 1 << logn, cfg)
    rank_err = np.max(np.abs(rank - sim))
    errs = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("SFHE_SINC_REBASE", mode)
        out = s.place(r, ct)
        assert out.level == depth
        errs[mode] = np.max(np.abs(np.array(e.decrypt(out)) - np.sort(x)))
    print(f"rank err {rank_err:.3g} (log2 {np.log2(rank_err):.2f}); sort err rebased {errs['1']:.3g} "
          f"(log2 {np.log2(errs['1']):.2f}), reference order {errs['0']:.3g} (log2 {np.log2(errs['0']):.2f})")
    assert rank_err < 2e-3          # measured 4.2e-4 (2^-11.2)
    assert errs["1"] < 2e-3         # measured 3.7e-4 (2^-11.4)
    assert errs["0"] < 0.02         # measured 9.8e-3 (2^-6.7)
    assert errs["1"] * 8 < errs["0"]


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
