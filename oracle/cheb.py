"""ORACLE (test infrastructure only): numpy restatement of the reference's
Chebyshev coefficient generators.

Reference:
  utils/generate_cheb_doubled_coeffs.cpp:11-49  (doubled sinc, threshold 1e-8,
      trim trailing |c| < 1e-8, printed with default 6-significant-digit
      ostream formatting at :43)
  utils/generate_cheb_coeffs.cpp:11-64           (scaled sinc: odd terms 0,
      even |c| < 1e-6 -> 0, trim trailing |c| < 1e-15)
  src/comparison.h:27-78                         (Sinc<N>::scaled_sinc /
      doubled_sinc, instantiated as Sinc<2N>)
  tests/SincTest.cpp:17-39                       (evaluation convention
      p(x) = c0/2 + sum_k c_k T_k(x))
The interpolation itself is OpenFHE 1.1.4's EvalChebyshevCoefficients
(external, not vendored): the published Chebyshev-node interpolation
  c_i = 2/d * sum_j f(cos(pi (j+1/2)/d)) cos(pi i (j+1/2)/d),  i < d,
computed here as an unnormalised DCT-II.
"""
from __future__ import annotations

import numpy as np
from scipy.fft import dct

INTERP_DEGREE = 13011  # generate_cheb_doubled_coeffs.cpp:12


def cheb_interp(f, a: float, b: float, d: int) -> np.ndarray:
    j = np.arange(d, dtype=np.float64)
    x = np.cos(np.pi / d * (j + 0.5)) * 0.5 * (b - a) + 0.5 * (b + a)
    return dct(f(x), type=2) / d


def _sinc_period(N2: int):
    def s(y):
        out = np.ones_like(y)
        m = np.abs(y) >= 1e-10
        out[m] = np.sin(np.pi * N2 * y[m]) / (np.pi * N2 * y[m])
        return out
    return s


def doubled_sinc(N: int):
    """Sinc<2N>::doubled_sinc: S(x) + S(x + 1/2), S(x) = sin(2 pi N x)/(2 pi N x)."""
    s = _sinc_period(2 * N)
    return lambda x: s(x) + s(x + 0.5)


def round6g(c: np.ndarray) -> np.ndarray:
    return np.array([float(f"{v:.6g}") for v in c])


def doubled_sinc_coeffs(N: int, d: int = INTERP_DEGREE) -> np.ndarray:
    c = cheb_interp(doubled_sinc(N), -1.0, 1.0, d)
    c = np.where(np.abs(c) >= 1e-8, c, 0.0)
    nz = np.nonzero(np.abs(c) >= 1e-8)[0]
    c = c[: nz[-1] + 1] if len(nz) else c[:0]
    return round6g(c)


def scaled_sinc_coeffs(N: int, d: int = INTERP_DEGREE) -> np.ndarray:
    c = cheb_interp(_sinc_period(2 * N), -1.0, 1.0, d)
    c = np.where((np.arange(len(c)) % 2 == 0) & (np.abs(c) >= 1e-6), c, 0.0)
    nz = np.nonzero(np.abs(c) >= 1e-15)[0]
    c = c[: nz[-1] + 1] if len(nz) else c[:0]
    return round6g(c)


def cheb_eval(c: np.ndarray, x: np.ndarray) -> np.ndarray:
    """p(x) = c0/2 + sum_{k>=1} c_k T_k(x) (SincTest.cpp:17-39)."""
    cc = np.array(c, dtype=np.float64).copy()
    if len(cc):
        cc[0] *= 0.5
    return np.polynomial.chebyshev.chebval(x, cc)


# OpenFHE EvalChebyshevSeriesPS depth for inputs in [-1, 1] (SURVEY.md
# §8(a) a-12(iv)); pinned by the reference's per-N multDepth tables.
_PS_BOUNDS = [5, 13, 27, 59, 119, 247, 495, 1007, 2031, 4031, 8127]


def ps_depth(degree: int) -> int:
    if degree <= 1:
        return 1
    if degree == 2:
        return 2
    for i, ub in enumerate(_PS_BOUNDS):
        if degree <= ub:
            return 3 + i
    raise ValueError(degree)
