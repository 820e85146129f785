"""The facade's layout stamp: a C++ caller compiled
against engine headers whose object layouts differ from the library's gets a
clean OpenFHEException from GenCryptoContext instead of heap corruption.

tests/cxx/abi_stamp.cpp is compiled twice against the oracle library (the
same host layer as the product): as is, it creates a context; with
-DSFHE_LAYOUT_SALT=1 (its stamp no longer the library's) GenCryptoContext
throws before any object crosses the boundary."""
import os
import subprocess

import pytest

import sfhe

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "sorting-fhe_amd", "csrc")


def build(tmp_path, extra):
    libdir = os.path.dirname(sfhe.ORACLE_LIB)
    exe = str(tmp_path / ("abi" + ("_salt" if extra else "")))
    cmd = (["g++", "-O1", "-std=c++17", "-I" + os.path.join(CSRC, "core"), "-I" + CSRC,
            "-I" + os.path.join(ROOT, "include")] + extra +
           [os.path.join(HERE, "cxx", "abi_stamp.cpp"), "-o", exe, "-L" + libdir, "-lsfhe_oracle",
            "-Wl,-rpath," + libdir, "-lpthread"])
    subprocess.run(cmd, check=True)
    return exe


def test_matching_caller_creates_context(oracle_lib, tmp_path):
    p = subprocess.run([build(tmp_path, [])], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "context ring 4096" in p.stdout


def test_mismatched_caller_gets_clean_exception(oracle_lib, tmp_path):
    p = subprocess.run([build(tmp_path, ["-DSFHE_LAYOUT_SALT=1"])], capture_output=True, text=True, timeout=120)
    assert p.returncode == 3, p.stdout + p.stderr
    assert "do not match the library's" in p.stdout and "caller stamp" in p.stdout, p.stdout


def test_c_abi_version(oracle_lib):
    assert oracle_lib.sfhe_abi_version() == sfhe.ABI_VERSION
