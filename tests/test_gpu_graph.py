"""hipGraph replay of DirectSort<N>::sort (north_star: the Chebyshev tree,
rotations and rank-matrix EvalMults run as a hipGraph).

The sorter runs the first sort of a shape eagerly, captures the second and
replays the graph afterwards.  The op sequence is data-independent (reference
src/sort_algo.h:752-774), so every replay must be bit-identical to the eager
sort of the same input on the same sorter (same zero-cache encryption), for
the captured input and for a different one copied into the graph's buffer.
"""
import numpy as np
import pytest

import sfhe
from oracle import slotsim

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("N,logn", [(64, 14), (256, 16)])
def test_graph_replay_bitexact(N, logn, monkeypatch):
    depth, rots = sfhe.direct_sort_params(N, "hip")
    e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots,
                    seed=20251205 + N)
    e.set_quiet(True)
    x = slotsim.input_vector(N)
    cfg = slotsim.default_sign_config(N)
    s = e.sorter(N)
    ct = e.encrypt(x.tolist())
    monkeypatch.setenv("SFHE_GRAPH", "1")
    eager = s.sort(ct, *cfg)             # first sort of the shape: eager
    assert s.graph_nodes() == 0
    cap = s.sort(ct, *cfg)               # captured, then launched
    nodes = s.graph_nodes()
    rep = s.sort(ct, *cfg)               # replayed
    assert nodes > 100, nodes
    ref = eager.download()
    assert np.array_equal(cap.download(), ref)
    assert np.array_equal(rep.download(), ref)
    assert cap.level == rep.level == depth
    # a different input: copied into the graph's input buffer
    y = slotsim.input_vector(N)[::-1].copy()
    ct2 = e.encrypt(y.tolist())
    g2 = s.sort(ct2, *cfg)
    monkeypatch.setenv("SFHE_GRAPH", "0")
    e2 = s.sort(ct2, *cfg)
    assert np.array_equal(g2.download(), e2.download())
    err = np.max(np.abs(np.array(e.decrypt(g2)) - np.sort(y)))
    print(f"N={N}: graph of {nodes} nodes, replay bit-identical to eager; max err {err:.3g}")
    assert err < 0.01


def test_graph_pool_steady(monkeypatch):
    """Replays allocate nothing new: the graph owns its blocks, the pool
    stays flat across sorts (outputs are clones the caller frees)."""
    N, logn = 64, 14
    depth, rots = sfhe.direct_sort_params(N, "hip")
    e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots)
    e.set_quiet(True)
    monkeypatch.setenv("SFHE_GRAPH", "1")
    s = e.sorter(N)
    ct = e.encrypt(slotsim.input_vector(N).tolist())
    cfg = slotsim.default_sign_config(N)
    sizes = []
    for _ in range(8):
        o = s.sort(ct, *cfg)
        e.sync()
        del o
        sizes.append(e.pool_bytes())
    assert s.graph_nodes() > 0
    assert sizes[-1] == sizes[3], sizes


@pytest.mark.parametrize("force_fail", [False, True])
def test_graph_lazy_inputs(force_fail, monkeypatch):
    """ADVICE r3 (high / medium): sorts of inputs that are lazy products
    (EvalMult(ct, 1.0): deferred, rescaled by their first consumer).  Three
    different arrays through one sorter -- eager, captured, replayed -- must
    each come back sorted; with the capture forced to fail
    (SFHE_CAPTURE_FORCE_FAIL=1) the sorter falls back to eager sorts and the
    results are the same values."""
    N, logn = 64, 14
    depth, rots = sfhe.direct_sort_params(N, "hip")
    e = sfhe.Engine("hip", mult_depth=depth + 1, ring_dim=1 << logn, batch_size=N, rotations=rots,
                    seed=20251205 + N)
    e.set_quiet(True)
    cfg = slotsim.default_sign_config(N)
    s = e.sorter(N)
    monkeypatch.setenv("SFHE_GRAPH", "1")
    rng = np.random.default_rng(5)
    for i in range(3):
        y = rng.permutation(N) / N + i * 0.3 / N
        lazy = e.mult_const(e.encrypt(y.tolist()), 1.0)
        if i == 1 and force_fail:
            monkeypatch.setenv("SFHE_CAPTURE_FORCE_FAIL", "1")
        out = s.sort(lazy, *cfg)
        monkeypatch.delenv("SFHE_CAPTURE_FORCE_FAIL", raising=False)
        err = float(np.max(np.abs(np.array(e.decrypt(out))[:N] - np.sort(y))))
        print(f"input {i}: max err {err:.3g}, graph nodes {s.graph_nodes()}")
        assert err < 1e-3, (i, err)
        if i >= 1:
            assert (s.graph_nodes() > 0) == (not force_fail)


def test_debug_sort_graphs(capfd, monkeypatch):
    """A debug sorter (DebugEncryption: the PRINT_PT decrypts of the input,
    the rank and the output inside sort(), reference src/sort_algo.h:755-770,
    as DirectSortTest times it) replays two graphs -- the rank and the
    placement -- with the decrypts between them: outputs bit-identical to the
    eager debug sort, and the printed decryptions the same text."""
    N, logn = 64, 14
    depth, rots = sfhe.direct_sort_params(N, "hip")
    e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots,
                    seed=20251205 + N)
    cfg = slotsim.default_sign_config(N)
    s = e.sorter(N, debug=True)
    ct = e.encrypt(slotsim.input_vector(N).tolist())
    monkeypatch.setenv("SFHE_GRAPH", "1")
    outs, texts = [], []
    for _ in range(3):                   # eager, captured, replayed
        capfd.readouterr()
        outs.append(s.sort(ct, *cfg).download())
        e.sync()
        texts.append(capfd.readouterr().out)
    nodes = s.graph_nodes()
    assert nodes > 100, nodes
    monkeypatch.setenv("SFHE_GRAPH", "0")
    capfd.readouterr()
    eager = s.sort(ct, *cfg).download()
    e.sync()
    eager_text = capfd.readouterr().out
    assert "Constructed Rank" in eager_text and "Final Output" in eager_text
    for o in outs:
        assert np.array_equal(o, eager)
    # the captured and the replayed sort print what the eager one prints (the
    # first sort's text differs: it sees its input at N slots, and sort()
    # leaves the input at the layout's S slots, :711)
    assert texts[1] == eager_text
    assert texts[2] == eager_text
    print(f"debug sort: two graphs of {nodes} nodes, replay bit-identical to eager")
