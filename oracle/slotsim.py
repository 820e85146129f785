"""ORACLE (test infrastructure only): float64 slot-level re-enactment of the
reference's DirectSort<N>::sort (no CKKS noise).

Every CKKS ciphertext is modelled by its periodic slot vector; rotations are
left rotations (np.roll by -r), plaintext masks are the reference's 0/1
vectors, and the sign / sinc approximations are the exact polynomials the
reference evaluates.  Restated from:
  src/sort_algo.h:206-306  mask / index / checking-vector generators
  src/sort_algo.h:326-366  vecRotsOpt          src/sort_algo.h:368-506 constructRank
  src/sort_algo.h:561-584  blindRotationOptN   src/sort_algo.h:658-750 rotationIndexCheckN
  src/comparison.cpp:4-22  compare             src/sign.cpp:9-185 composite sign
  src/sort_algo.h:894-1062, :1067-1229, :1233-1389  the hybrid placements
  tests/utils.h:28-51      getVectorWithMinDiff (seeded instead of random_device)
"""
from __future__ import annotations

import math

import numpy as np

from . import cheb

# ---- sign polynomials (src/sign.cpp:17-21, :40-44, :68-75, :81-88) ----
G3 = [4589 / 1024, -16577 / 1024, 25614 / 1024, -12860 / 1024]
F3 = [35 / 16, -35 / 16, 21 / 16, -5 / 16]
G4_CHEB = [0.0, 1.077117252745569, 0.0, -0.36166113998402755, 0.0, 0.2137420717859748, 0.0,
           -0.15635204788780485, 0.0, 0.11749645501187332, 0.0, -0.10074154666447852, 0.0,
           0.08002086947825496, 0.0, -0.07533558758484624, 0.0, 0.059514472116534836, 0.0,
           -0.06146663712787884, 0.0, 0.04570084927999001, 0.0, -0.05403683682999072, 0.0,
           0.03364293851188723, 0.0, -0.054459493266273494]
F4 = [3.14208984375, -7.33154296875, 13.19677734375, -15.71044921875, 12.21923828125,
      -5.99853515625, 1.69189453125, -0.20947265625]


def odd_poly(c, x):
    return sum(ci * x ** (2 * i + 1) for i, ci in enumerate(c))


def composite_sign(x, n: int, dg: int, df: int):
    """compositeSign<n>: g applied max(dg,1) times (sign.cpp:173-178), then f df times."""
    y = np.asarray(x, dtype=np.float64)
    for _ in range(max(dg, 1)):
        y = odd_poly(G3, y) if n == 3 else cheb.cheb_eval(G4_CHEB, y)
    for _ in range(df):
        y = odd_poly(F3, y) if n == 3 else odd_poly(F4, y)
    return y


def sign_depth(n: int, dg: int, df: int) -> int:
    return 3 * (max(dg, 1) + df) if n == 3 else 5 * max(dg, 1) + 4 * df


def default_sign_config(N: int):
    """DirectSortTest.cpp:113-121."""
    if N <= 16:
        return (3, 2, 2)
    if N <= 128:
        return (3, 3, 2)
    if N <= 512:
        return (3, 4, 2)
    return (3, 5, 2)


def direct_sort_depth(N: int, cfg=None) -> int:
    n, dg, df = cfg or default_sign_config(N)
    deg = len(cheb.doubled_sinc_coeffs(N)) - 1
    return 2 + sign_depth(n, dg, df) + 1 + cheb.ps_depth(deg) + 2


def np_rank(N: int, P: int) -> int:
    return min(1 << (int(math.log2(N)) // 2), P)


def np_place(N: int) -> int:
    if N <= 256:
        return 1 << (int(math.log2(N)) // 2)
    return 8 if N <= 1024 else 4


def input_vector(N: int, seed: int | None = None) -> np.ndarray:
    """getVectorWithMinDiff(N, 0, 1, 1/N) with std::mt19937(20251205+N)-style seeding."""
    rng = np.random.default_rng(20251205 + N if seed is None else seed)
    return rng.permutation(N).astype(np.float64) / N


def rot(v, r):
    return np.roll(v, -r)


def _mask(S, N, k):
    m = np.zeros(S)
    m[k * N:(k + 1) * N] = 1.0
    return m


def construct_rank(x, N, ring, cfg, sign_fn=None):
    P = min(N, ring // 2 // N)
    B, S = N // P, N * P
    npr = np_rank(N, P)
    base = np.tile(x, S // N)  # periodic packing with period N
    pre = [rot(base, i) for i in range(npr)]
    sgn = sign_fn or (lambda d: composite_sign(d, *cfg))
    rank = np.zeros(S)
    for b in range(B):
        giants = []
        for j in range(P // npr):
            shift = b * P + j * npr
            T = np.zeros(S)
            for i in range(npr):
                T += pre[i] * rot(_mask(S, N, npr * j + i), -shift)
            giants.append(rot(T, shift))
        shifted = sum(giants)
        rank += (sgn(base - shifted) + 1.0) * 0.5
    s = S // 2
    while s >= N:
        rank = rank + rot(rank, s)
        s //= 2
    return rank[:N] - 0.5


def rotation_index_check(rank, x, N, ring):
    P = min(N, ring // 2 // N)
    B, S = N // P, N * P
    npp = np_place(N)
    coeffs = cheb.doubled_sinc_coeffs(N)
    imr = np.tile(np.arange(N) - rank, S // N)
    xs = np.tile(x, S // N)
    out = np.zeros(S)
    for b in range(B):
        chk = np.array([(b * P + s // N) % N for s in range(S)], dtype=np.float64)
        z = (imr - chk) / N / 2
        masked = cheb.cheb_eval(coeffs, z) * xs
        mi = [rot(masked, i) for i in range(npp)]
        res = np.zeros(S)
        for i in range((S // N) // npp):
            tmp = np.zeros(S)
            for j in range(npp):
                tmp += mi[j] * rot(_mask(S, N, npp * i + j), j)
            res += rot(tmp, b * P + i * npp)
        out += res
    s = S // 2
    while s >= N:
        out = out + rot(out, s)
        s //= 2
    return out[:N]


def direct_sort(x, N, ring, cfg=None):
    cfg = cfg or default_sign_config(N)
    rank = construct_rank(np.asarray(x, dtype=np.float64), N, ring, cfg)
    return rotation_index_check(rank, np.asarray(x, dtype=np.float64), N, ring), rank


# ---- hybrid placement I (sort_hybrid1): src/sort_algo.h:815-891 (matrix
# helpers), :1067-1229 (rotationIndexCheckHybrid1, sort_hybrid1);
# src/mehp24/mehp24_utils.cpp:166-174 (indicatorAdv), :246-261 (signAdv) ----
def sign_adv(x, dg: int, df: int):
    """signAdv: dg x g3, (df - 1) x f3, then 1/2 + f3/2 (coeffF3_final)."""
    y = np.asarray(x, dtype=np.float64)
    for _ in range(dg):
        y = odd_poly(G3, y)
    for _ in range(df - 1):
        y = odd_poly(F3, y)
    return 0.5 + 0.5 * odd_poly(F3, y)


def indicator_adv(c, b: float, dg: int, df: int):
    tmp = np.asarray(c, dtype=np.float64) / b
    return sign_adv(tmp + 0.5 / b, dg, df) * (1.0 - sign_adv(tmp - 0.5 / b, dg, df))


def hybrid1_dg(N: int) -> int:
    return int((math.log2(N) + 1) / 2)  # uint32_t dg_i = (log2(N) + 1) / 2 (:1126)


def hybrid1_depth(N: int, cfg=None) -> int:
    """rank + [2 + 4 (dg_i + 2)] + 3."""
    n, dg, df = cfg or default_sign_config(N)
    return 2 + sign_depth(n, dg, df) + 2 + 4 * (hybrid1_dg(N) + 2) + 3


def _binary_path(idx: int, m: int):
    bits = int(math.ceil(math.log2(m)))
    return [(idx >> (bits - 1 - i)) & 1 for i in range(bits)]


def sum_columns_to_target(c, m: int, col: int):
    step = m >> 1
    for bit in _binary_path(col, m):
        c = c + rot(c, -step if bit else step)
        step >>= 1
    msk = np.zeros(len(c))
    msk[np.arange(m) * m + col] = 1.0
    return c * msk


def transpose_column_target(c, m: int, row: int):
    step = m * (m - 1) // 2
    for bit in _binary_path(row, m):
        c = c + rot(c, -step if bit else step)
        step >>= 1
    msk = np.zeros(len(c))
    msk[m * row + np.arange(m)] = 1.0
    return c * msk


def rotation_index_check_hybrid1(rank, x, N, ring):
    maxa = 256
    num_slots, num_batch = (ring // 2, N // maxa) if N > maxa else (N * N, 1)
    M = min(N, maxa)
    rk = np.tile(np.asarray(rank, dtype=np.float64), num_slots // N)
    xs = np.tile(np.asarray(x, dtype=np.float64), num_slots // N)
    rots_rank = [rot(rk, k * maxa) for k in range(num_batch)]
    rots_in = [rot(xs, k * maxa) for k in range(num_batch)]
    dg = hybrid1_dg(N)
    out = np.zeros(num_slots)
    for b in range(num_batch):
        sub = np.zeros(num_slots)
        for i in range(M):
            sub[i * M:(i + 1) * M] = b * M + i
        acc = np.zeros(num_slots)
        for k in range(num_batch):
            acc = acc + rots_in[k] * indicator_adv(sub - rots_rank[k], N, dg, 2)
        acc = sum_columns_to_target(acc, N // num_batch, b)
        out = out + transpose_column_target(acc, N // num_batch, b)
    return out[:N]


def sort_hybrid1(x, N, ring, cfg=None):
    cfg = cfg or default_sign_config(N)
    rank = construct_rank(np.asarray(x, dtype=np.float64), N, ring, cfg)
    return rotation_index_check_hybrid1(rank, np.asarray(x, dtype=np.float64), N, ring), rank


# ---- hybrid placements with rank / N (src/sort_algo.h:894-1062 sort_hybrid,
# :1233-1389 sort_hybrid2); src/comparison.cpp:24-40 (Comparison::indicator) ----
def indicator(x, c: float, cfg):
    """step(x + c) * (1 - step(x - c)), step(d) = (sign(d) + 1) / 2."""
    step = lambda d: (composite_sign(d, *cfg) + 1.0) * 0.5  # noqa: E731
    return step(np.asarray(x) + c) * (1.0 - step(np.asarray(x) - c))


def hybrid_depth(N: int, variant: int, cfg=None) -> int:
    """hybrid / hybrid2 depth tables."""
    n, dg, df = cfg or default_sign_config(N)
    rank = 2 + sign_depth(n, dg, df)
    ps = cheb.ps_depth(len(cheb.scaled_sinc_coeffs(N)) - 1)
    if variant == 2 or N < 256:
        return rank + 1 + ps + 3
    dgi = 4 if N < 512 else 5
    return rank + 1 + (3 * (dgi + 2) + 2) + 3


def rotation_index_check_hybrid(rank, x, N, ring, variant: int):
    maxa = 256
    num_slots, num_batch = (ring // 2, N // maxa) if N > maxa else (N * N, 1)
    M = min(N, maxa)
    r = np.tile(np.asarray(rank, dtype=np.float64), num_slots // N) / N
    xs = np.tile(np.asarray(x, dtype=np.float64), num_slots // N)
    rots_rank = [rot(r, k * maxa) for k in range(num_batch)]
    rots_in = [rot(xs, k * maxa) for k in range(num_batch)]
    coeffs = cheb.scaled_sinc_coeffs(N)
    out = np.zeros(num_slots)
    for b in range(num_batch):
        sub = np.zeros(num_slots)
        for i in range(M):
            sub[i * M:(i + 1) * M] = (b * M + i) / N
        acc = np.zeros(num_slots)
        for k in range(num_batch):
            d = sub - rots_rank[k]
            if variant == 2 or N < 256:
                ind = cheb.cheb_eval(coeffs, d)
            else:
                ind = indicator(d, 0.5 / N, (3, 4 if N < 512 else 5, 2))
            acc = acc + rots_in[k] * ind
        acc = sum_columns_to_target(acc, N // num_batch, b)
        out = out + transpose_column_target(acc, N // num_batch, b)
    return out[:N]


def sort_hybrid(x, N, ring, variant: int = 0, cfg=None):
    cfg = cfg or default_sign_config(N)
    rank = construct_rank(np.asarray(x, dtype=np.float64), N, ring, cfg)
    return rotation_index_check_hybrid(rank, np.asarray(x, dtype=np.float64), N, ring, variant), rank
