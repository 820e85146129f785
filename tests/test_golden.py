"""Oracle and host logic against the reference's own data (tests/golden/,
extracted by tests/golden/make_golden.py) and the derived expectations."""
import json
import os

import numpy as np
import pytest

import sfhe
from oracle import cheb, slotsim

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REF = json.load(open(os.path.join(GOLD, "reference_params.json")))
DER = json.load(open(os.path.join(GOLD, "derived_expectations.json")))


@pytest.mark.parametrize("N", [4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048])
def test_size_parameters_match_reference(oracle_lib, N):
    want = REF["direct_sort_size_parameters"]["by_N"][str(N)]
    depth, rots = sfhe.direct_sort_params(N, "oracle")
    assert depth == want["mult_depth"]
    assert list(rots) == want["rotations"]


@pytest.mark.parametrize("N", [4, 8, 16, 32, 64, 128, 256, 512, 1024])
def test_depth_model_reproduces_reference_table(N):
    # Appendix B model: rank + placement levels with DirectSortTest's sign configs
    want = REF["direct_sort_size_parameters"]["by_N"][str(N)]["mult_depth"]
    assert slotsim.direct_sort_depth(N) == want


def test_sign_coefficients_match_reference():
    c = REF["sign_coefficients"]
    assert slotsim.G3 == c["g3"]
    assert slotsim.F3 == c["f3"]
    assert list(slotsim.G4_CHEB) == c["g4_chebyshev"]
    assert list(slotsim.F4) == c["f4"]


def test_ps_depth_table():
    table = DER["chebyshev_ps_depth_table"]
    for i, (deg, depth) in enumerate(table):
        assert cheb.ps_depth(deg) == depth
        if i + 1 < len(table):
            assert cheb.ps_depth(deg + 1) == depth + 1


@pytest.mark.parametrize("N", [4, 8, 16, 32, 64, 128, 256])
def test_doubled_sinc_tables(oracle_lib, N):
    """C++ generator (the product's table) == numpy restatement, including the
    reference generator's %g (6 significant digit) printing."""
    cxx = np.array(sfhe.doubled_sinc_coeffs(N, "oracle"))
    py = cheb.doubled_sinc_coeffs(N)
    assert len(cxx) - 1 == DER["doubled_sinc_degree"][str(N)]
    assert len(cxx) == len(py)
    assert np.array_equal(cxx, py)


def test_decompose_reference_numbers(oracle_lib):
    d = REF["decompose_test"]
    for algo in (0, 1, 2):  # NAF, BNAF, BINARY
        for num in d["numbers"]:
            steps = sfhe.decompose(d["N"], d["keys"], num, d["wrap"], algo, "oracle")
            # DecomposeTest: the steps recompose the amount (identity steps dropped)
            assert sum(s for _, s in steps) % d["wrap"] == num % d["wrap"]
    assert sfhe.decompose(128, d["keys"], 127, 128, 0, "oracle") == [tuple(x) for x in DER["decompose_naf_127"]]


@pytest.mark.parametrize("N,ring", [(8, 1 << 7), (16, 1 << 9), (16, 1 << 8), (32, 1 << 10)])
def test_slot_simulation_sorts(N, ring):
    """SURVEY App. C validation table: the float64 re-enactment sorts."""
    x = slotsim.input_vector(N)
    out, rank = slotsim.direct_sort(x, N, ring)
    assert np.max(np.abs(rank - np.argsort(np.argsort(x)))) < 1e-6
    assert np.max(np.abs(out - np.sort(x))) < 2e-6


def test_composite_sign_precision():
    """comparison (sign+1)/2 error over |d| >= 1/N."""
    for (n, dg, df), N, bound in [((3, 2, 2), 8, 2 ** -24.4), ((3, 3, 2), 128, 2 ** -16.6),
                                  ((3, 4, 2), 256, 2 ** -24.7)]:
        d = np.concatenate([np.arange(1, N + 1), -np.arange(1, N + 1)]) / N
        err = np.max(np.abs(slotsim.composite_sign(d, n, dg, df) - np.sign(d))) / 2
        assert err < bound, (n, dg, df, N, err)
