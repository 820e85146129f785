"""Every kernel the product library's host code can launch has device code
for gfx950 (CPU test; reads the built libsfhe.so, runs nothing on a GPU).

A __global__ template specialisation named only inside a conditional
expression got a host-side handle but no device code: the launch aborted the
process with "Cannot find Symbol with name: _Z11k_modup_col..." (round 5).
The handles are the library's `_Z<len>k_...` data symbols (nm); the device
kernels are the `.name` notes of the gfx950 code object in `.hip_fatbin`.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "sorting-fhe_amd", "build", "libsfhe.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _tool(name):
    p = os.path.join(LLVM, name)
    return p if os.path.exists(p) else shutil.which(name)


def test_every_launchable_kernel_has_device_code(tmp_path):
    bundler, readelf = _tool("clang-offload-bundler"), _tool("llvm-readelf")
    if not (os.path.exists(LIB) and bundler and readelf and shutil.which("objcopy") and shutil.which("nm")):
        pytest.skip("needs the built libsfhe.so and the ROCm LLVM tools")
    fat, co = tmp_path / "fat.bin", tmp_path / "k.co"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", LIB, str(fat)], check=True)
    subprocess.run([bundler, "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([readelf, "--notes", str(co)], check=True, capture_output=True, text=True).stdout
    device = set(re.findall(r"^\s+\.name:\s+(_Z\S+)$", notes, re.M))
    syms = subprocess.run(["nm", LIB], check=True, capture_output=True, text=True).stdout
    host = set(re.findall(r"^[0-9a-f]+ [VvDdBbRr] (_Z\d+k_\w+)$", syms, re.M))
    assert len(device) > 100 and len(host) > 100, (len(device), len(host))
    missing = sorted(host - device)
    assert not missing, f"{len(missing)} kernel handles without gfx950 code, e.g. {missing[:3]}"
