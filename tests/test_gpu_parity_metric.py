"""GPU parity at the metric shape with the default kernels.

tests/test_gpu_parity.py proves the HIP product bit-exact against the C
oracle on small rings; this file does it on the parameters the metric sort
actually runs -- ring 2^16, depth 34 (35 Q limbs, dnum 3 -> alpha 12, K 13
special primes), scale 40, FP64 NTT / conversion kernels on (SFHE_NTT_FP
default) -- and once at ring 2^17 (BASELINE config 5's ring).  That covers
the kernels only these shapes reach:

  * the FP64 INTT / NTT at n = 2^16 (the logn = 16 `colUnroll` COL pass) and
    2^17;
  * ModUp's `k_convf<13>` conversions with 12-source digits (alpha = 12) and
    ModDown's 13-source P -> Q conversion, fused with the rescale in
    `k_mdrsf` (relinearisation) and unfused (rotations);
  * the key inner product over 3 digits, lazily rescaled rotations, the
    rotation sum's shared ModDown (EvalRotateSum), the Chebyshev PS with its
    weighted-sum leaves, and a composite sign that walks the chain from 35
    limbs down to 23.

Every result is compared residue for residue with the oracle's (same host
layer, same seed: identical integers iff the gfx950 kernels compute what
oracle/prims_ref.c computes with exact 128-bit '%')."""
import numpy as np
import pytest

import sfhe
from oracle import cheb

pytestmark = pytest.mark.gpu


def program(e, N=256):
    """Ops of the metric sort at its own parameters; returns name -> Ct."""
    e.set_quiet(True)
    rng = np.random.default_rng(2026)
    a = (rng.permutation(N) / N).tolist()
    b = rng.uniform(-1, 1, N).tolist()
    x, y = e.encrypt(a), e.encrypt(b)
    out = {"encrypt": x}
    m = e.mult(x, y)                      # tensor + relinearisation (+ fused ModDown/rescale)
    out["mult"] = m
    out["rotate_lazy"] = e.rotate(m, 1)   # a deferred product rotated before its rescale
    out["rotate"] = e.rotate(x, 16)
    out["rotate_sum"] = e.rotate_sum([x, y, e.mult_const(x, 0.5)], [1, 16, 128])
    out["mult_plain"] = e.mult_plain(y, [float(i % 2) for i in range(N)], N)
    out["mult_deep"] = e.mult(e.mult(m, m), x)
    out["sign"] = e.sign(e.sub(x, y), 3, 2, 2)     # 12 levels: 35 -> 23 limbs
    z = e.mult_const(e.sub(x, y), 0.25)
    out["chebyshev"] = e.chebyshev(z, cheb.doubled_sinc_coeffs(8).tolist())  # degree 70, PS depth 7
    return out


def compare_programs(logn, depth, N=256):
    kw = dict(mult_depth=depth, ring_dim=1 << logn, batch_size=N, scaling_mod_size=40, secure=False,
              seed=4242, rotations=[1, 16, 128])
    outs = {}
    for backend in ("hip", "oracle"):
        e = sfhe.Engine(backend, **kw)
        info = e.info()
        assert (info["num_q"], info["dnum"]) == (depth + 1, 3), info
        res = program(e, N)
        outs[backend] = {k: (v.download(), v.level) for k, v in res.items()}
        if backend == "hip":
            dec = np.array(e.decrypt(res["mult"]))[:N]
        e.close()
    for k in outs["hip"]:
        g, lg = outs["hip"][k]
        o, lo = outs["oracle"][k]
        assert lg == lo, (k, lg, lo)
        bad = int(np.count_nonzero(g != o))
        assert bad == 0, f"{k}: {bad} of {g.size} residues differ"
    return outs, dec


def test_metric_shape_bitexact(hip_lib, oracle_lib):
    """Ring 2^16, depth 34: the metric sort's parameters."""
    outs, dec = compare_programs(16, 34)
    rng = np.random.default_rng(2026)
    a = rng.permutation(256) / 256
    b = rng.uniform(-1, 1, 256)
    assert np.max(np.abs(dec - a * b)) < 1e-6
    assert outs["hip"]["sign"][1] == 12


def test_config5_ring_bitexact(hip_lib, oracle_lib):
    """Ring 2^17, depth 34: BASELINE config 5's ring (n = 512 x 256 in the NTT)."""
    compare_programs(17, 34)
