"""Plaintext encoding on the device (SURVEY §7 hard part
6: the sort encodes its in-loop masks, reference src/sort_algo.h:341-357,
:573-574, :715-717).

sfp_encode runs the host encoder's special inverse FFT (core/encoder.cpp)
operation for operation and must give bit-identical encodings.  Two engines
with the same seed draw identical keys and encryption randomness, so their
ciphertexts agree residue for residue iff the plaintext encodings agree: one
encodes on the host (SFHE_HOST_ENCODE=1, read per encoding), the other on
the device.  CPU: the oracle's C restatement of sfp_encode; GPU: the HIP
kernels (k_enc_*)."""
import numpy as np
import pytest

import sfhe

CASES = [
    # (slots, values)
    (8, [0.5, -0.25, 0.125, 0.75, -1.0, 0.3, 0.2, 0.1]),
    (16, list(np.random.default_rng(1).uniform(-1, 1, 16))),
    (2048, [float(i % 2) for i in range(2048)]),                  # a 0/1 mask, one LDS tile
    (2048, list(np.random.default_rng(2).uniform(-1, 1, 1500))),  # zero padding
    (1, [0.75]),
]


def program(e, monkeypatch, host, cases, big=None):
    monkeypatch.setenv("SFHE_HOST_ENCODE", "1" if host else "0")
    e.op_stats(reset=True)
    out = []
    for slots, v in cases:
        ct = e.encrypt(v, slots)
        out.append(ct.download())
        # a plaintext product at a deeper level (the masks' use)
        out.append(e.mult_plain(e.mult_const(ct, 0.5), v, slots).download())
    if big:
        slots, v = big
        out.append(e.encrypt(v, slots).download())
    return out, e.encode_counts()


def check(backend, logn, monkeypatch, big_slots):
    kw = dict(mult_depth=4, ring_dim=1 << logn, batch_size=8, seed=31337)
    rng = np.random.default_rng(3)
    big = (big_slots, [float(x) for x in (rng.permutation(big_slots) % 2)])  # a full-ring 0/1 mask
    res = {}
    for host in (True, False):
        e = sfhe.Engine(backend, **kw)
        e.set_plaintext_cache(False)
        res[host] = program(e, monkeypatch, host, CASES, big)
        e.close()
    (h_out, (hd, hh)), (d_out, (dd, dh)) = res[True], res[False]
    assert hd == 0 and hh > 0, (hd, hh)
    assert dh == 0 and dd == hh, (dd, dh, hh)  # every encoding took the device path
    for i, (a, b) in enumerate(zip(h_out, d_out)):
        bad = int(np.count_nonzero(a != b))
        assert bad == 0, f"output {i}: {bad} of {a.size} residues differ"


def test_device_encoding_bitexact_oracle(oracle_lib, monkeypatch):
    check("oracle", 13, monkeypatch, 1 << 12)


def test_large_values_stay_on_the_host(oracle_lib, monkeypatch):
    """Values whose scaled coefficients could need the encoder's 2^shift range
    extension are encoded on the host."""
    monkeypatch.setenv("SFHE_HOST_ENCODE", "0")
    e = sfhe.Engine("oracle", mult_depth=2, ring_dim=1 << 12, batch_size=8, scaling_mod_size=59, seed=5)
    e.op_stats(reset=True)
    ct = e.encrypt([300.0, -1.0, 2.0], 8)
    d, h = e.encode_counts()
    assert h == 1 and d == 0
    assert np.allclose(np.array(e.decrypt(ct))[:3], [300.0, -1.0, 2.0], atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("logn", [14, 16, 17])
def test_device_encoding_bitexact_hip(hip_lib, monkeypatch, logn):
    """The HIP kernels, up to the metric ring (2^16: 32768-slot masks, four
    global stages then 2048-value LDS tiles) and 2^17."""
    check("hip", logn, monkeypatch, 1 << (logn - 1))


def sort_encodings(backend, monkeypatch, logn, N):
    """A DirectSort<N>'s downloaded result with every mask encoded on the
    host, and with the masks of each giant step encoded as one device batch
    (sfp_encode_batch / sfp_ntt_batch, core/context.cpp encodeBatch)."""
    from oracle import slotsim
    depth, rots = sfhe.direct_sort_params(N, backend)
    kw = dict(mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots, seed=99)
    out = {}
    for host in (True, False):
        monkeypatch.setenv("SFHE_HOST_ENCODE", "1" if host else "0")
        e = sfhe.Engine(backend, **kw)
        e.set_quiet(True)
        e.set_plaintext_cache(False)
        e.op_stats(reset=True)
        r = e.sorter(N).sort(e.encrypt(slotsim.input_vector(N).tolist()), *slotsim.default_sign_config(N))
        out[host] = (r.download(), e.encode_counts())
        e.close()
    (h, (hd, hh)), (d, (dd, dh)) = out[True], out[False]
    assert hd == 0 and dh == 0 and dd == hh > 0, (hd, hh, dd, dh)
    assert np.array_equal(h, d)


def test_batched_mask_encodings_bitexact_oracle(oracle_lib, monkeypatch):
    sort_encodings("oracle", monkeypatch, 12, 8)


@pytest.mark.gpu
def test_batched_mask_encodings_bitexact_hip(hip_lib, monkeypatch):
    """The metric sort's masks (16 per giant step, 32768 slots): batched on
    the device, bit-identical to the host encoder."""
    sort_encodings("hip", monkeypatch, 16, 256)


@pytest.mark.gpu
def test_batched_encodings_chunked_hip(hip_lib, monkeypatch):
    """a batch whose values exceed the argument ring is
    encoded in chunks (ringPut refuses oversize uploads instead of writing past
    the pinned ring).  With a 1 MiB ring every giant step's 16 masks of 32768
    slots (4 MiB of values) take several chunks; the sort stays bit-identical
    to the host encoder."""
    monkeypatch.setenv("SFHE_ARG_RING_MB", "1")
    sort_encodings("hip", monkeypatch, 16, 256)
