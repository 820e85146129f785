"""Build the reference's own test and benchmark sources UNCHANGED against this
engine (DirectSortTest, SortNBenchmark, CompareTest,
SignTest, RotationTest, DecomposeTest must compile and link as-is).

Container-only (needs /root/reference; nothing is copied from it): every
source is compiled where it lies, with the engine's reference-level headers
(sorting-fhe_amd/csrc/{core,algo}) first on the include path, the reference's
tests/ directory only for its utils.h / memory_tracker.h, and the gtest /
google-benchmark shims of tests/cxx/shim (the reference's googletest and
benchmark submodules are empty).  Each program is linked twice:
  <name>_oracle  against oracle/_build/libsfhe_oracle.so (runs here, on CPU)
  <name>_hip     against sorting-fhe_amd/build/libsfhe.so (the product; runs
                 on the GPU box from the tree: tests/test_gpu_reference_sources.py)
into tests/cxx/build/ (git-ignored build output).

    python tests/cxx/reference_harness.py [--jobs 8]
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("SFHE_REFERENCE", "/root/reference")
OUT = os.path.join(HERE, "build")
CSRC = os.path.join(ROOT, "sorting-fhe_amd", "csrc")
SHIM = os.path.join(HERE, "shim")
PSTL = next((os.path.join("/usr/include/c++", v, "pstl") for v in sorted(os.listdir("/usr/include/c++"), reverse=True)
             if os.path.isdir(os.path.join("/usr/include/c++", v, "pstl"))), "/usr/include")
LIBS = {
    "oracle": (os.path.join(ROOT, "oracle", "_build"), "sfhe_oracle"),
    "hip": (os.path.join(ROOT, "sorting-fhe_amd", "build"), "sfhe"),
}

# program -> (sources relative to the reference, needs gtest_main, needs memory_tracker)
PROGRAMS = {
    "DirectSortTest": (["tests/DirectSortTest.cpp"], True, True),
    "DirectSortH1Test": (["tests/DirectSortH1Test.cpp"], True, True),
    "DirectSortHTest": (["tests/DirectSortHTest.cpp"], True, True),
    "DirectSortH2Test": (["tests/DirectSortH2Test.cpp"], True, True),
    "DirectSortNTest": (["tests/DirectSortNTest.cpp"], True, False),
    "SincTest": (["tests/SincTest.cpp"], False, False),
    "DirectSortBenchmark": (["benchmarks/DirectSortBenchmark.cpp"], False, False),
    "SincBenchmark": (["benchmarks/SincBenchmark.cpp"], False, False),
    "RotationBenchmark": (["benchmarks/RotationBenchmark.cpp"], False, False),
    "CompareTest": (["tests/CompareTest.cpp"], False, False),
    "SignTest": (["tests/SignTest.cpp"], False, False),
    "RotationTest": (["tests/RotationTest.cpp"], True, False),
    "DecomposeTest": (["tests/DecomposeTest.cpp"], True, False),
    "SortNBenchmark": (["benchmarks/SortNBenchmark.cpp"], False, False),
    # BitonicSort<N> + CKKS bootstrapping, SURVEY §8(f) rows 2-3
    "BitonicSortTest": (["tests/BitonicSortTest.cpp"], True, False),
    "BitonicSortBenchmark": (["benchmarks/BitonicSortBenchmark.cpp"], False, False),
    # the k-way network (src/k-way/*, src/kway_adapter.h; SURVEY §8(f) row 2, BASELINE config 4)
    "KWaySortTest": (["tests/KWaySortTest.cpp"], False, False),
    "KWayMaskingTest": (["tests/k-way/MaskingTest.cpp"], False, False),
    "KWayEvalUtilsTest": (["tests/k-way/EvalUtilsTest.cpp"], False, False),
    "KWaySortUtilsTest": (["tests/k-way/SortUtilsTest.cpp"], False, False),
    "KWaySorterTest": (["tests/k-way/SorterTest.cpp"], False, False),
    "KWaySort2Test": (["tests/k-way/KWaySort2Test.cpp"], False, True),
    "KWaySort3Test": (["tests/k-way/KWaySort3Test.cpp"], False, True),
    "KWaySort5Test": (["tests/k-way/KWaySort5Test.cpp"], False, True),
    "KWaySort235Test": (["tests/k-way/KWaySort235Test.cpp"], False, False),
    # the FHERMA-style server (src/sort.h SortContext + src/main.cpp), SURVEY §8(f) row 4
    "main": (["src/main.cpp"], False, False),
}

# the engine's own test programs (no reference sources; always buildable)
OWN = {"fherma_client": os.path.join(HERE, "fherma_client.cpp")}


def _engine_mtime() -> float:
    """Newest engine header: objects compiled against older headers are stale."""
    t = 0.0
    for d, _, fs in list(os.walk(CSRC)) + list(os.walk(SHIM)):
        for f in fs:
            if f.endswith(".h"):
                t = max(t, os.path.getmtime(os.path.join(d, f)))
    return t


def build_own():
    built = {}
    for name, src in OWN.items():
        for backend, (libdir, lib) in LIBS.items():
            exe = os.path.join(OUT, f"{name}_{backend}")
            os.makedirs(OUT, exist_ok=True)
            if not _fresh(exe, src):
                _atomic(["g++"] + flags() + [src, "-o"], exe,
                        ["-L" + libdir, "-l" + lib, "-Wl,-rpath," + libdir, "-lpthread"])
            built[(name, backend)] = exe
    return built


def available() -> bool:
    return os.path.isdir(os.path.join(REF, "tests")) and os.path.isfile(os.path.join(REF, "tests", "DirectSortTest.cpp"))


def _forwarders() -> str:
    """Include directory of one-line forwarding headers to reference sources
    the engine does not re-provide: src/sort.h (SortContext, the FHERMA-style
    serialized I/O glue of src/main.cpp) calls only the lbcrypto facade, so
    the reference's own file is compiled where it lies (its quote-includes of
    sort_algo.h / sign.h / comparison.h / openfhe.h resolve to the engine's
    headers through -I-)."""
    d = os.path.join(OUT, "forward")
    os.makedirs(d, exist_ok=True)
    for name, target in {"sort.h": os.path.join(REF, "src", "sort.h")}.items():
        text = f'#include "{target}"\n'
        path = os.path.join(d, name)
        if not (os.path.exists(path) and open(path).read() == text):
            with open(path, "w") as f:
                f.write(text)
    return d


def flags():
    # -I- first: #include "x" never resolves next to the including source
    # file, so the reference's src/main.cpp picks up this engine's
    # sort_algo.h, not the reference's own (every -I after it serves both
    # include forms; libstdc++'s pstl headers quote-include their siblings,
    # hence their directory)
    return ["-O2", "-std=c++17", "-fopenmp", "-DENABLE_PRINT_PT", "-I-",
            "-I" + _forwarders(),
            "-I" + os.path.join(CSRC, "core"), "-I" + os.path.join(CSRC, "algo"), "-I" + os.path.join(CSRC, "algo", "k-way"),
            "-I" + CSRC,
            "-I" + os.path.join(ROOT, "include"), "-I" + SHIM, "-I" + os.path.join(REF, "tests"),
            # the k-way tests include "../utils.h" from tests/k-way (test .cpp files only there)
            "-I" + os.path.join(REF, "tests", "k-way"),
            "-I" + PSTL, "-w"]


def _fresh(out: str, *deps: str) -> bool:
    return os.path.exists(out) and os.path.getmtime(out) >= max([os.path.getmtime(d) for d in deps] +
                                                                [_engine_mtime()])


def _atomic(cmd_before_out, out, cmd_after_out=()):
    """Run a compiler writing to a private temp name, then rename over `out`:
    concurrent pytest-xdist workers never see a half-written file."""
    tmp = f"{out}.tmp{os.getpid()}"
    subprocess.run(list(cmd_before_out) + [tmp] + list(cmd_after_out), check=True)
    os.replace(tmp, out)


def compile_obj(src: str, obj: str):
    os.makedirs(os.path.dirname(obj), exist_ok=True)
    if _fresh(obj, src):
        return
    _atomic(["g++"] + flags() + ["-c", src, "-o"], obj)


def build(jobs: int = 8, programs=None):
    if not available():
        raise FileNotFoundError(f"reference sources not found under {REF}")
    programs = programs or list(PROGRAMS)
    objs = {}
    work = []
    extra = {"gtest_main": os.path.join(SHIM, "gtest_main.cc"),
             "memory_tracker": os.path.join(REF, "tests", "memory_tracker.cpp")}
    for k, src in extra.items():
        objs[k] = os.path.join(OUT, "obj", k + ".o")
        work.append((src, objs[k]))
    for p in programs:
        srcs, _, _ = PROGRAMS[p]
        for s in srcs:
            o = os.path.join(OUT, "obj", p + "_" + os.path.basename(s) + ".o")
            objs[(p, s)] = o
            work.append((os.path.join(REF, s), o))
    with ThreadPoolExecutor(jobs) as ex:
        for f in [ex.submit(compile_obj, s, o) for s, o in work]:
            f.result()
    built = {}
    for p in programs:
        srcs, gmain, mtrack = PROGRAMS[p]
        o = [objs[(p, s)] for s in srcs]
        if gmain:
            o.append(objs["gtest_main"])
        if mtrack:
            o.append(objs["memory_tracker"])
        for backend, (libdir, lib) in LIBS.items():
            exe = os.path.join(OUT, f"{p}_{backend}")
            if not _fresh(exe, *o):
                _atomic(["g++", "-fopenmp", "-o"], exe,
                        o + ["-L" + libdir, "-l" + lib, "-Wl,-rpath," + libdir, "-lpthread"])
            built[(p, backend)] = exe
    return built


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=8)
    a = ap.parse_args()
    built = build_own()
    if available():
        built.update(build(a.jobs))
    for (p, b), exe in sorted(built.items()):
        print(f"{p:16s} {b:7s} {exe}")


if __name__ == "__main__":
    sys.exit(main())
