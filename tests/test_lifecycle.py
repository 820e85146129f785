"""Context lifecycle: creating and destroying contexts
repeatedly releases everything they allocated -- the device's per-lane
scratch, conversion tables, twiddle tables and pools belong to the context
(sfp_dev) and are freed by sfp_destroy.  CPU: the oracle backend; GPU: the
product, with the device's free memory read back through hipMemGetInfo of the
HIP runtime the product library itself loaded (torch's bundled runtime is a
second copy that does not see the library's device)."""
import gc

import numpy as np
import pytest

import sfhe


def cycle(backend, rounds, logn=13):
    for i in range(rounds):
        e = sfhe.Engine(backend, mult_depth=6, ring_dim=1 << logn, batch_size=8, rotations=[1, 2],
                        seed=100 + i, device=0)
        e.set_quiet(True)
        a = e.encrypt([0.5, -0.25, 0.125, 0.0])
        b = e.mult(a, e.rotate(a, 1))  # key switching: conversion tables, scratch
        got = np.array(e.decrypt(b))[:3]
        assert np.allclose(got, [-0.125, -0.03125, 0.0], atol=1e-3), got
        del a, b  # ciphertexts hold their context; the last reference frees it
        e.close()
        del e
        gc.collect()


def test_context_churn_oracle(oracle_lib):
    cycle("oracle", 5)


@pytest.mark.gpu
def test_context_churn_hip_releases_device_memory(hip_lib):
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime libsfhe.so linked (already loaded)

    def free_bytes():
        assert hip.hipDeviceSynchronize() == 0
        free, total = ctypes.c_size_t(), ctypes.c_size_t()
        assert hip.hipMemGetInfo(ctypes.byref(free), ctypes.byref(total)) == 0
        return free.value

    cycle("hip", 2)  # warm: runtime / code-object state that stays for the process
    free0 = free_bytes()
    cycle("hip", 12)
    free1 = free_bytes()
    print(f"free before {free0 / 2**30:.2f} GiB, after 12 contexts {free1 / 2**30:.2f} GiB")
    assert free0 - free1 < 64 << 20, (free0, free1)
