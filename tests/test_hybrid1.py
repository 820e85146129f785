"""sort_hybrid1: DirectSort<N>::sort_hybrid1 =
constructRank + rotationIndexCheckHybrid1 (reference src/sort_algo.h:815-891,
:1067-1229; MEHP24 indicatorAdv / signAdv, src/mehp24/mehp24_utils.cpp:166-174,
:246-261).

Oracle: oracle/slotsim.py's float64 re-enactment of the same schedule and
std::sort; the reference's own gates (tests/DirectSortH1Test.cpp:197-256):
final level == multDepth, max error < 0.01.  CPU tests run the C oracle at
small rings; the GPU tests run the product at DirectSortH1Test's ring 2^17 /
HEStd_128_classic and check the HIP ciphertext bit for bit against the oracle
at a small ring.
"""
import numpy as np
import pytest

import sfhe
from oracle import slotsim

SIZES = [4, 8, 16, 32, 64, 128, 256, 512, 1024]


def test_hybrid1_params_match_depth_model(oracle_lib):
    """The DirectSortH1Test depth table is rank + [2 + 4 (dg_i + 2)] + 3."""
    for N in SIZES:
        depth, rots = sfhe.hybrid1_params(N, "oracle")
        assert depth == slotsim.hybrid1_depth(N), N
        # every amount sumColumnsToTarget / transposeColumnTarget rotates by
        # on batch 0 is a key (the composer would otherwise chain steps)
        m = min(N, 256)
        need = {m >> (i + 1) for i in range(int(np.log2(m)))} | \
               {m * (m - 1) // (2 << i) for i in range(int(np.log2(m)))}
        assert need <= set(rots), (N, sorted(need - set(rots)))


def test_slotsim_hybrid1_sorts():
    for N, ring in ((4, 1 << 12), (8, 1 << 12), (32, 1 << 12), (128, 1 << 15), (512, 1 << 17)):
        x = slotsim.input_vector(N)
        out, _ = slotsim.sort_hybrid1(x, N, ring)
        assert np.max(np.abs(out - np.sort(x))) < 1e-3, N


def run_hybrid1(backend, N, logn, secure=False, seed=None):
    depth, rots = sfhe.hybrid1_params(N, backend)
    e = sfhe.Engine(backend, mult_depth=depth, ring_dim=1 << logn, batch_size=N, secure=secure,
                    rotations=rots, seed=seed or 20251205 + N, device=0)
    e.set_quiet(True)
    x = slotsim.input_vector(N)
    s = e.sorter(N, rotations=rots)
    out = s.sort_hybrid1(e.encrypt(x.tolist()), *slotsim.default_sign_config(N))
    return e, x, out, depth


@pytest.mark.parametrize("N", [8, 16])
def test_hybrid1_oracle(oracle_lib, N):
    e, x, out, depth = run_hybrid1("oracle", N, 12)
    assert out.level == depth
    got = np.array(e.decrypt(out))[:N]  # result->SetLength(N) (DirectSortH1Test.cpp:206)
    sim, _ = slotsim.sort_hybrid1(x, N, 1 << 12)
    err = np.max(np.abs(got - np.sort(x)))
    print(f"hybrid1 N={N} @2^12 (oracle): max err {err:.3g}, vs slotsim {np.max(np.abs(got - sim)):.3g}")
    assert err < 0.01
    assert np.max(np.abs(got - sim)) < 1e-3


@pytest.mark.gpu
def test_hybrid1_bitexact_hip_vs_oracle(hip_lib, oracle_lib):
    raw = {}
    for backend in ("hip", "oracle"):
        e, x, out, depth = run_hybrid1(backend, 8, 12)
        assert out.level == depth
        raw[backend] = out.download()
    assert np.array_equal(raw["hip"], raw["oracle"])


@pytest.mark.gpu
@pytest.mark.parametrize("N,tol,exact_tol", [(64, 1e-6, 2e-5), (256, 3e-6, 1.8e-6)])
def test_hybrid1_directsorth1test_config(hip_lib, N, tol, exact_tol):
    """DirectSortH1Test's configuration: ring 2^17, HEStd_128_classic, its
    depth and keys.  The reference publishes N=256 over 10 trials: max error
    1.33e-6 .. 1.74e-6, log2 -19.13 .. -19.52 (comparison/experimental_results/
    ours_hybrid1/trials/trial_*/size_256.txt; total_results.txt:151-174).
    Measured here 1.67e-6 (2^-19.19): gated at 1.8e-6, the top of
    the reference's range.  N=64 sits on the approximation floor (slotsim
    9.2e-6)."""
    import time
    t0 = time.perf_counter()
    e, x, out, depth = run_hybrid1("hip", N, 17, secure=True)
    got = np.array(e.decrypt(out))[:N]  # result->SetLength(N) (DirectSortH1Test.cpp:206)
    dt = time.perf_counter() - t0
    assert out.level == depth
    sim, _ = slotsim.sort_hybrid1(x, N, 1 << 17)
    err = np.max(np.abs(got - np.sort(x)))
    print(f"hybrid1 N={N} @2^17: max err {err:.3g} (log2 {np.log2(err):.2f}), vs slotsim "
          f"{np.max(np.abs(got - sim)):.3g}; {dt:.1f} s incl. keygen")
    assert err < 0.01
    assert err < exact_tol
    assert np.max(np.abs(got - sim)) < tol


def _published():
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "hybrid1_published.json")) as f:
        return json.load(f)["by_N"]


def test_published_fixture_matches_params(oracle_lib):
    """The published runs used the depths and sign configurations this engine
    takes for DirectSortH1Test (hybrid1_params / default_sign_config)."""
    pub = _published()
    assert sorted(int(n) for n in pub) == SIZES
    for N in SIZES:
        p = pub[str(N)]
        assert p["ring_dim"] == 1 << 17 and p["scaling_mod_size"] == 40
        assert p["mult_depth"] == sfhe.hybrid1_params(N, "oracle")[0], N
        assert tuple(p["sign"]) == tuple(slotsim.default_sign_config(N)), N
        assert all(t["level"] == p["mult_depth"] for t in p["trials"])


# Engine max error / the largest of the reference's 10 published trials,
# allowed per N.  1.25 everywhere the engine is at or below
# the reference; DESIGN.md §2 attributes any N listed with a larger factor.
HYBRID1_RATIO = {N: 1.25 for N in SIZES}


@pytest.mark.gpu
@pytest.mark.parametrize("N", SIZES)
def test_hybrid1_published_outputs(hip_lib, N):
    """sort_hybrid1 at DirectSortH1Test's configuration (ring 2^17,
    HEStd_128_classic, its depth / keys / sign configuration) against every
    output the reference publishes (comparison/experimental_results/
    ours_hybrid1/total_results.txt:1-224 and trials/trial_*/size_*.txt, 10
    trials per N, extracted to tests/golden/hybrid1_published.json): final
    level == depth (the reference's Result Level), and the max error within
    HYBRID1_RATIO[N] x the largest published trial error."""
    pub = _published()[str(N)]
    e, x, out, depth = run_hybrid1("hip", N, 17, secure=True)
    got = np.array(e.decrypt(out))[:N]
    err = float(np.max(np.abs(got - np.sort(x))))
    pmax = max(t["max_err"] for t in pub["trials"])
    pmin = min(t["max_err"] for t in pub["trials"])
    sim, _ = slotsim.sort_hybrid1(x, N, 1 << 17)
    floor = float(np.max(np.abs(sim - np.sort(x))))
    print(f"hybrid1 N={N}: max err {err:.3g} (log2 {np.log2(err):.2f}); published {pmin:.3g}..{pmax:.3g} "
          f"(log2 {pub['max_err_log2']:.2f}); slotsim floor {floor:.3g}; ratio {err / pmax:.2f}")
    assert out.level == depth == pub["mult_depth"]
    assert err <= HYBRID1_RATIO[N] * pmax, (N, err, pmax)
