"""sort_hybrid, sort_hybrid2 and rotationIndexCheck2N (SURVEY.md §8(b):
sort_hybrid* are part of the sort_algo.h surface; reference src/sort_algo.h
:894-1062 rotationIndexCheckHybrid / sort_hybrid, :1233-1389 -Hybrid2 /
sort_hybrid2, :537-656 blindRotationOpt2N / rotationIndexCheck2N).

Oracle: oracle/slotsim.py's float64 re-enactment of the same placements and
std::sort; the reference's own gates (tests/DirectSortHTest.cpp,
tests/DirectSortH2Test.cpp): final level == multDepth, max error < 0.01.
The depth tables of both tests are reproduced by the SURVEY Appendix B model
(slotsim.hybrid_depth).  CPU tests run the C oracle at small rings; the GPU
tests check HIP against the oracle bit for bit and run the tests' own
configurations (ring 2^17, HEStd_128_classic).
"""
import numpy as np
import pytest

import sfhe
from oracle import slotsim

SIZES = [4, 8, 16, 32, 64, 128, 256, 512, 1024]


@pytest.mark.parametrize("variant", [0, 2])
def test_hybrid_params_match_depth_model(oracle_lib, variant):
    for N in SIZES:
        depth, rots = sfhe.hybrid_params(N, variant, "oracle")
        assert depth == slotsim.hybrid_depth(N, variant), (N, variant)
        assert rots == sfhe.hybrid1_params(N, "oracle")[1]  # the three hybrid tests share their keys


def run_hybrid(backend, N, logn, variant, secure=False):
    depth, rots = sfhe.hybrid_params(N, variant, backend)
    e = sfhe.Engine(backend, mult_depth=depth, ring_dim=1 << logn, batch_size=N, secure=secure,
                    rotations=rots, seed=20251205 + N, device=0)
    e.set_quiet(True)
    x = slotsim.input_vector(N)
    s = e.sorter(N, rotations=rots)
    out = s.sort_hybrid(e.encrypt(x.tolist()), *slotsim.default_sign_config(N), variant=variant)
    return e, x, out, depth


@pytest.mark.parametrize("variant", [0, 2])
def test_hybrid_oracle(oracle_lib, variant):
    N = 8
    e, x, out, depth = run_hybrid("oracle", N, 12, variant)
    assert out.level == depth
    got = np.array(e.decrypt(out))[:N]
    sim, _ = slotsim.sort_hybrid(x, N, 1 << 12, variant)
    err = np.max(np.abs(got - np.sort(x)))
    print(f"hybrid variant {variant} N={N} @2^12 (oracle): max err {err:.3g}, vs slotsim "
          f"{np.max(np.abs(got - sim)):.3g}")
    assert err < 0.01
    assert np.max(np.abs(got - sim)) < 1e-4


def test_rotation_index_check_2n_oracle(oracle_lib):
    """rank (constructRank) then the 2N-block placement: the sorted array."""
    N, logn = 8, 12
    depth, rots = sfhe.direct_sort_params(N, "oracle")
    e = sfhe.Engine("oracle", mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots,
                    seed=20251205 + N)
    e.set_quiet(True)
    x = slotsim.input_vector(N)
    s = e.sorter(N)
    ct = e.encrypt(x.tolist())
    out = s.place_2n(s.rank(ct, *slotsim.default_sign_config(N)), ct)
    err = np.max(np.abs(np.array(e.decrypt(out))[:N] - np.sort(x)))
    print(f"rotationIndexCheck2N N={N} @2^12: max err {err:.3g}, level {out.level}/{depth}")
    assert out.level == depth
    assert err < 0.01


@pytest.mark.gpu
@pytest.mark.parametrize("variant", [0, 2])
def test_hybrid_bitexact_hip_vs_oracle(hip_lib, oracle_lib, variant):
    raw = {}
    for backend in ("hip", "oracle"):
        e, x, out, depth = run_hybrid(backend, 8, 12, variant)
        assert out.level == depth
        raw[backend] = out.download()
    assert np.array_equal(raw["hip"], raw["oracle"])


@pytest.mark.gpu
@pytest.mark.parametrize("variant,N,tol", [
    (0, 64, 3e-4),     # DirectSortHTest: scaled-sinc series below 256 (measured 1.3e-4)
    (0, 256, 4e-6),    # composite-sign indicator (3,4,2) (measured 1.65e-6)
    (2, 64, 3e-4),     # DirectSortH2Test (measured 1.3e-4)
    (2, 128, 2e-3),    # (measured 1.0e-3: the series' Paterson-Stockmeyer noise)
])
def test_hybrid_directsorthtest_config(hip_lib, variant, N, tol):
    """DirectSortHTest / DirectSortH2Test configuration: ring 2^17,
    HEStd_128_classic, the tests' depths and keys; gates = measured x ~2
     and the reference's 0.01."""
    e, x, out, depth = run_hybrid("hip", N, 17, variant, secure=True)
    assert out.level == depth
    got = np.array(e.decrypt(out))[:N]
    err = np.max(np.abs(got - np.sort(x)))
    print(f"hybrid variant {variant} N={N} @2^17: max err {err:.3g} (log2 {np.log2(err):.2f})")
    assert err < 0.01
    assert err < tol
