"""Stacked launches (prims.h sfp_stack_*, DESIGN.md §4 "stacked batches";
SFHE_STACK_BATCHES=1 -- off by default, two streams measured faster):
the sort's batches run the same op sequence on their lanes; inside a stacked
region their identical ops are issued as ONE launch each (NTT passes, fused
key-switch passes, conversions, ModDown+rescale conversions), the rest in an
order that keeps each lane's sequence and every cross-lane event.

Per-row arithmetic is unchanged, so every result must be the oracle's residue
for residue -- at two batches (N = 128 @ 2^14, two lanes) and at four
(N = 256 @ 2^15: four lanes, pairs merged among four heads), eager, captured
and replayed.  tests/test_gpu_parity_sort.py does the same at the metric
shape."""
import numpy as np
import pytest

import sfhe

pytestmark = pytest.mark.gpu


def sort_pair(N, logn):
    depth, rots = sfhe.direct_sort_params(N, "hip")
    kw = dict(mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots, seed=4711 + N)
    x = (np.random.default_rng(N).permutation(N) / N).tolist()
    cfg = (3, 3, 2) if N <= 128 else (3, 4, 2)
    res = {}
    for backend in ("oracle", "hip"):
        e = sfhe.Engine(backend, **kw)
        e.set_quiet(True)
        s = e.sorter(N)
        ct = e.encrypt(x)
        outs = [s.sort(ct, *cfg) for _ in range(3 if backend == "hip" else 1)]
        res[backend] = (e, s, outs)
    return res, x


@pytest.mark.parametrize("N,logn,batches", [(128, 14, 2), (256, 15, 4)])
def test_stacked_sort_bitexact(hip_lib, oracle_lib, N, logn, batches, monkeypatch):
    monkeypatch.setenv("SFHE_STACK_BATCHES", "1")  # (off by default: DESIGN.md §4)
    res, x = sort_pair(N, logn)
    eo, _, (ref,) = res["oracle"]
    eh, sh, outs = res["hip"]
    want = ref.download()
    for k, o in enumerate(outs):  # eager, captured, replayed
        got = o.download()
        assert got.shape == want.shape
        bad = int(np.count_nonzero(got != want))
        assert bad == 0, f"sort {k}: {bad} of {got.size} residues differ"
    merged, single = eh.stack_stats()
    print(f"N={N} @ 2^{logn}: {batches} batches, {merged} merged pairs, {single} alone, "
          f"graph {sh.graph_nodes()} nodes")
    assert merged > 0, "the batches' launches were never merged"
    assert np.max(np.abs(np.array(eh.decrypt(outs[-1]))[:N] - np.sort(x))) < 0.01
    eo.close()
    eh.close()
