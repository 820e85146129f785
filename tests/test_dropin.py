"""The reference's C++ call surface, unchanged: tests/cxx/direct_sort_drop_in.cpp
follows DirectSortTest's SetUp + SortTest (getSizeParameters, GenCryptoContext,
KeyGen, EvalMultKeyGen, EvalRotateKeyGen, DebugEncryption::encryptInput,
DirectSort<N>::sort, Decrypt) and is compiled against this engine's headers
only.  CPU: linked to the oracle library.  GPU: linked to libsfhe.so at
DirectSortTest's own parameters (ring 2^17, HEStd_128_classic)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "cxx", "direct_sort_drop_in.cpp")
CS = os.path.join(ROOT, "sorting-fhe_amd", "csrc")


def build(tmp_path, libdir, libname):
    exe = str(tmp_path / f"dropin_{libname}")
    subprocess.run(["g++", "-O2", "-std=c++17", "-fopenmp", "-DENABLE_PRINT_PT",
                    f"-I{CS}/core", f"-I{CS}/algo", f"-I{CS}", SRC, "-o", exe, f"-L{libdir}",
                    f"-l{libname}", f"-Wl,-rpath,{libdir}"], check=True)
    return exe


def run(exe, *args, timeout=600):
    r = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=timeout)
    line = [l for l in r.stdout.splitlines() if l.startswith("DROPIN")]
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-2000:])
    return line[-1]


def test_dropin_oracle(tmp_path, oracle_lib):
    exe = build(tmp_path, os.path.join(ROOT, "oracle", "_build"), "sfhe_oracle")
    print(run(exe, 8, 12, 0))


@pytest.mark.gpu
def test_dropin_hip_directsorttest_config(tmp_path, hip_lib):
    exe = build(tmp_path, os.path.join(ROOT, "sorting-fhe_amd", "build"), "sfhe")
    print(run(exe, 8, 17, 1))   # DirectSortTest<8>: ring 2^17, 128-bit security
    print(run(exe, 256, 16, 0))  # metric config through the C++ surface
