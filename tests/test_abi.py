"""The C ABI (include/sfhe.h): both libraries load and export every declared
symbol.  No compute call goes to the product library here (no GPU)."""
import ctypes
import os
import re

import sfhe

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "sfhe.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sfhe_\w+)\s*\(", src)))


def test_header_matches_binding_list():
    assert header_functions() == sorted(sfhe.ABI_SYMBOLS)


def test_product_library_exports_every_symbol():
    lib = ctypes.CDLL(sfhe.PRODUCT_LIB)  # load only: no HIP call is made
    missing = [s for s in header_functions() if not hasattr(lib, s)]
    assert not missing, missing


def test_oracle_library_exports_every_symbol(oracle_lib):
    missing = [s for s in header_functions() if not hasattr(oracle_lib, s)]
    assert not missing, missing


def test_abi_version_and_backends(oracle_lib):
    lib = ctypes.CDLL(sfhe.PRODUCT_LIB)
    lib.sfhe_abi_version.restype = ctypes.c_int
    lib.sfhe_backend.restype = ctypes.c_char_p
    assert lib.sfhe_abi_version() == sfhe.ABI_VERSION == 3
    assert lib.sfhe_backend() == b"hip-gfx950"
    assert oracle_lib.sfhe_backend() == b"oracle-c"


def test_params_default(oracle_lib):
    p = sfhe.Params()
    oracle_lib.sfhe_params_default(ctypes.byref(p))
    assert (p.scaling_mod_size, p.first_mod_size, p.security_level) == (40, 60, 0)
    assert p.scaling_technique == 3  # FLEXIBLEAUTOEXT, OpenFHE's default


def test_errors_are_codes_not_crashes(oracle_lib):
    with __import__("pytest").raises(sfhe.SfheError):
        sfhe.Engine("oracle", mult_depth=2, ring_dim=1000)  # not a power of two
    with __import__("pytest").raises(sfhe.SfheError):
        sfhe.direct_sort_params(3, "oracle")
