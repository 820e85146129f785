"""k-way sorting network and BitonicSort through the C ABI (SURVEY.md §8(f)
rows 2-3; reference src/kway_adapter.h, src/k-way/*, src/sort_algo.h:1393-1487).

The reference's own k-way tests (tests/k-way/*, tests/KWaySortTest.cpp) and
BitonicSortTest run unchanged in tests/test_reference_sources.py (CPU oracle)
and tests/test_gpu_reference_sources.py (MI355X); here the ABI entries are
checked on small rings against std::sort, and the HIP path bit for bit
against the oracle.
"""
import numpy as np
import pytest

import sfhe


def test_kway_params(oracle_lib):
    """KWayAdapter<N>::getSizeParameters (kway_adapter.h:41-64)."""
    b, d, budget, rots = sfhe.kway_params(1024, "oracle")
    assert (b, d, budget) == (1024, 40, (5, 5))
    assert sorted(rots) == sorted([s * (1 << i) for i in range(10) for s in (1, -1)])
    b, d, budget, rots = sfhe.kway_params(729, "oracle")
    assert (b, budget) == (1024, (5, 5))
    b, d, budget, _ = sfhe.kway_params(27, "oracle")
    assert (b, budget) == (32, (4, 4))


def run_kway(backend, k, M, logn=12):
    N = k ** M
    batch, depth, budget, rots = sfhe.kway_params(N, backend)
    e = sfhe.Engine(backend, mult_depth=depth, ring_dim=1 << logn, batch_size=batch, scaling_mod_size=59,
                    rotations=rots, seed=11, device=0)
    e.set_quiet(True)
    e.bootstrap_setup(budget, batch)
    x = np.random.default_rng(k * 100 + M).permutation(N) / N
    out = e.kway_sort(e.encrypt(x.tolist()), k, M, 3, 2, 2, depth)
    return e, x, out


@pytest.mark.slow
@pytest.mark.parametrize("k,M", [(2, 3), (3, 2)])
def test_kway_sort_oracle(oracle_lib, k, M):
    e, x, out = run_kway("oracle", k, M)
    got = np.array(e.decrypt(out))[: len(x)]
    err = np.max(np.abs(got - np.sort(x)))
    print(f"k={k} M={M}: max err {err:.3g}")
    assert err < 0.01


def test_kway_sort_errors(oracle_lib):
    e = sfhe.Engine("oracle", mult_depth=10, ring_dim=1 << 12, batch_size=8, seed=3)
    e.set_quiet(True)
    ct = e.encrypt([0.1] * 8)
    with pytest.raises(sfhe.SfheError, match="k must be"):
        e.kway_sort(ct, 4, 2)
    with pytest.raises(sfhe.SfheError, match="exceeds"):
        e.kway_sort(ct, 2, 4)


@pytest.mark.slow
def test_bitonic_sort_oracle(oracle_lib):
    """BitonicSortTest's configuration (ring 2^12, depth 58, scale 59, {3,3})
    through sfhe_sorter_sort_bitonic."""
    N = 4
    rots = [r for i in range(2) for r in (1 << i, -(1 << i))]
    e = sfhe.Engine("oracle", mult_depth=58, ring_dim=1 << 12, batch_size=N, scaling_mod_size=59,
                    rotations=rots, seed=4)
    e.set_quiet(True)
    e.bootstrap_setup((3, 3), N)
    x = np.array([123.73, 115.91, 245.11, 250.48])
    out = e.sorter(N, rotations=rots).sort_bitonic(e.encrypt(x.tolist()))
    got = np.array(e.decrypt(out))[:N]
    assert np.max(np.abs(got - np.sort(x))) < 1e-3


@pytest.mark.gpu
def test_kway_bitexact_hip_vs_oracle(hip_lib, oracle_lib):
    raw = {}
    for backend in ("hip", "oracle"):
        e, x, out = run_kway(backend, 2, 2)
        assert np.max(np.abs(np.array(e.decrypt(out))[:4] - np.sort(x))) < 0.01
        raw[backend] = out.download()
    assert np.array_equal(raw["hip"], raw["oracle"])


def test_kway_schedule_matches_reference_masking():
    """The network schedule pinned to the reference's own code: the reference's
    src/k-way/Masking.cpp, compiled where it lies (oracle/Makefile `ref`), and
    the engine's algo/k-way/Masking.cpp print identical sortType /
    getRotateDistance / genIndices / genMask output for every stage of every
    k in {2, 3, 5} network up to 1024 slots."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    ref = os.environ.get("SFHE_REFERENCE", "/root/reference")
    if not os.path.isfile(os.path.join(ref, "src", "k-way", "Masking.cpp")):
        pytest.skip("reference sources absent")
    subprocess.run(["make", "-C", os.path.join(root, "oracle"), "ref"], check=True, stdout=subprocess.DEVNULL)
    outs = [subprocess.run([os.path.join(root, "oracle", "_ref", f"masking_dump_{w}")], capture_output=True,
                           text=True, check=True).stdout for w in ("ref", "engine")]
    assert outs[0].count("stage=") > 100
    assert outs[0] == outs[1]


@pytest.mark.slow
def test_kway_handle_oracle(oracle_lib):
    """sfhe_kway_create / sfhe_kway_run: a persistent KWayAdapter; repeated
    sorts of one input agree bit for bit."""
    N, k, M = 8, 2, 3
    batch, depth, budget, rots = sfhe.kway_params(N, "oracle")
    e = sfhe.Engine("oracle", mult_depth=depth, ring_dim=1 << 12, batch_size=batch, scaling_mod_size=59,
                    rotations=rots, seed=11)
    e.set_quiet(True)
    e.bootstrap_setup(budget, batch)
    x = np.random.default_rng(3).permutation(N) / N
    ct = e.encrypt(x.tolist())
    s = e.kway(k, M)
    a = s.sort(ct, 3, 2, 2, depth)
    b = s.sort(ct, 3, 2, 2, depth)
    assert np.array_equal(a.download(), b.download())
    assert np.max(np.abs(np.array(e.decrypt(a))[:N] - np.sort(x))) < 0.01
    import ctypes
    h = ctypes.c_void_p()
    assert e.lib.sfhe_kway_create(e.ctx, 12, 2, 3, ctypes.byref(h)) != sfhe.SFHE_OK
    assert "k^M" in e.lib.sfhe_last_error().decode()


@pytest.mark.gpu
@pytest.mark.parametrize("N,k,M,logn,chunk", [(8, 2, 3, 12, None), (27, 3, 3, 13, None), (8, 2, 3, 12, "2")])
def test_kway_graph_replay_hip(hip_lib, oracle_lib, N, k, M, logn, chunk, monkeypatch):
    """The k-way network as a hipGraph (BASELINE config 4): a persistent
    adapter sorts eagerly, then captures the whole sort -- every stage's
    comparisons, masked rotations and sub-sorters with the bootstraps between
    them -- and replays it.  Eager, captured and replayed sorts are the
    oracle's residues bit for bit; a new input through the replayed graph
    sorts correctly.  chunk = "2": SFHE_KWAY_CHUNK=2 (read at every sort), so
    the six stages of M = 3 are captured as a CHAIN of three graphs, each
    reading the previous one's output (config 4's N = 1024 runs four)."""
    if chunk is not None:
        monkeypatch.setenv("SFHE_KWAY_CHUNK", chunk)
    batch, depth, budget, rots = sfhe.kway_params(N, "hip")
    kw = dict(mult_depth=depth, ring_dim=1 << logn, batch_size=batch, scaling_mod_size=59, rotations=rots,
              seed=11)
    x = np.random.default_rng(3).permutation(N) / N
    ref = sfhe.Engine("oracle", **kw)
    ref.set_quiet(True)
    ref.bootstrap_setup(budget, batch)
    want = ref.kway(k, M).sort(ref.encrypt(x.tolist()), 3, 2, 2, depth).download()
    e = sfhe.Engine("hip", **kw)
    e.set_quiet(True)
    e.bootstrap_setup(budget, batch)
    s = e.kway(k, M)
    ct = e.encrypt(x.tolist())
    outs = [s.sort(ct, 3, 2, 2, depth) for _ in range(3)]  # eager, captured, replayed
    nodes = s.graph_nodes()
    print(f"k-way N={N} (k={k}, M={M}) @ 2^{logn}, chunk {chunk or 14}: graph of {nodes} nodes")
    assert nodes > 100
    for i, o in enumerate(outs):
        assert np.array_equal(o.download(), want), f"sort {i} differs from the oracle"
    y = np.random.default_rng(4).permutation(N) / N
    o = s.sort(e.encrypt(y.tolist()), 3, 2, 2, depth)
    assert np.max(np.abs(np.array(e.decrypt(o))[:N] - np.sort(y))) < 0.01
