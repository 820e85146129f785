"""The reference's unchanged tests/benchmark on the MI355X product library.

Runs the binaries tests/cxx/reference_harness.py built in the container from
the reference's own sources (every program of its PROGRAMS table: the
DirectSort / hybrid / N / sinc / rotation / compare / sign / decompose /
bitonic / k-way tests and benchmarks, and src/main.cpp) linked to
sorting-fhe_amd/build/libsfhe.so; nothing here reads /root/reference.  Skips when the prebuilt binaries are absent.
"""
import os
import re
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "cxx", "build")

pytestmark = pytest.mark.gpu


CSRC = os.path.join(os.path.dirname(HERE), "sorting-fhe_amd", "csrc")


def _newest_header() -> float:
    t = 0.0
    for d, _, fs in os.walk(CSRC):
        for f in fs:
            if f.endswith(".h"):
                t = max(t, os.path.getmtime(os.path.join(d, f)))
    return t


def exe(name):
    p = os.path.join(BUILD, name + "_hip")
    if not os.access(p, os.X_OK):
        pytest.skip(f"{name}_hip not built (tests/cxx/reference_harness.py runs where the reference is)")
    # the programs compile the engine's headers (sort_algo.h, openfhe.h,
    # state.h) into themselves: one built before a header change disagrees
    # with the library on object layouts, which corrupts memory at run time
    # (120 s of slack: a copy that does not keep mtimes stamps files seconds apart)
    assert os.path.getmtime(p) >= _newest_header() - 120, (
        f"{name}_hip is older than the engine headers: rebuild it (python tests/cxx/reference_harness.py)")
    return p


def run(path, *args, timeout=280):
    p = subprocess.run([path, *args], capture_output=True, text=True, timeout=timeout)
    return p.returncode, p.stdout + p.stderr


def test_direct_sort_test_all_sizes(hip_lib):
    """DirectSortTest.cpp as-is: N = 4 ... 1024 at ring 2^17, HEStd_128_classic,
    DebugEncryption (PRINT_PT inside the timed sort), gate max error < 0.01 and
    final level == multDepth, for every one of its nine instantiations."""
    rc, out = run(exe("DirectSortTest"))
    errs = [float(x) for x in re.findall(r"Maximum error: ([0-9.e+-]+)", out)]
    times = [int(x) for x in re.findall(r"Execution time: (\d+) ms", out)]
    print("max errors:", errs, "\nexecution ms (as-test):", times)
    assert rc == 0, out[-4000:]
    assert "9 tests ran, 0 failed" in out
    assert len(errs) == 9 and max(errs) < 0.01


def test_rotation_test(hip_lib):
    """RotationTest.cpp as-is (ring 2^17, depth 45, scale 59): composed
    rotations (NAF chains through non-key amounts), rotation trees, forward /
    backward round trips and rotate-and-add at 16384 slots."""
    rc, out = run(exe("RotationTest"))
    check_rotation_test_output(out)


def check_rotation_test_output(out):
    """RotateVector, RotateForwardAndBackward (r in [-128, 128], NAF chains)
    and RotateLargerThanNWithMask pass.  RotateTreeVector fails in the
    reference itself: it encrypts 8 values with batch size 128
    (tests/RotationTest.cpp:33-35, :70), so the ciphertext has 128 slots
    (MakeCKKSPackedPlaintext pads with zeros) while the test expects a cyclic
    rotation of 8 (:76-86); and RotationTree<8>'s NAF folds -N/2 = -4 into +4
    (src/rotation.h:128-135), a different rotation at 128 slots.  Every
    mismatch must be exactly a slot that this 128-slot rotation fills with a
    padding zero."""
    def naf_total(r, N=8):  # sum of the NAF steps (src/rotation.h:111-140)
        tot, b = 0, 0
        while r:
            if r & 1:
                z = -1 if r & 2 else 1
                w = z << b
                tot += -w if w == -N // 2 else w
                r -= z
            r >>= 1
            b += 1
        return tot
    for t in ("RotateVector", "RotateForwardAndBackward", "RotateLargerThanNWithMask"):
        assert f"[       OK ] RotationComposerTest.{t}" in out, out[-4000:]
    assert "4 tests ran, 1 failed" in out, out[-4000:]
    got = {(int(r), int(i)) for i, r in re.findall(r"Mismatch at index (\d+) for rotation (-?\d+)", out)}
    want = {(r, i) for r in range(-4, 5) for i in range(8)
            if not 0 <= (i + naf_total(r)) % 128 < 8 or (i + naf_total(r)) % 128 != (i + r) % 8}
    assert got == want, (sorted(got ^ want), out[-3000:])
    assert all(a == "0" for a in re.findall(r"actual: ([0-9.e+-]+) vs [0-9.]+ \(tolerance 1e-06\)", out)), out[-3000:]


def test_compare_and_decompose(hip_lib):
    rc, out = run(exe("CompareTest"))
    assert rc == 0 and "1 tests ran, 0 failed" in out, out[-3000:]
    rc, out = run(exe("DecomposeTest"))
    assert rc == 0 and "1 tests ran, 0 failed" in out, out[-3000:]


def test_sign_test(hip_lib):
    """As on the oracle: VerySmallElementsTest passes; CompositeSignTest fails
    exactly as the reference's own polynomial composition does (0.78775 vs
    its +-0.1 bar around 1, tests/test_reference_sources.py)."""
    rc, out = run(exe("SignTest"))
    assert "[       OK ] ArraySortTest.VerySmallElementsTest" in out, out[-3000:]
    m = re.search(r"actual: ([0-9.]+) vs 1 \(tolerance 0\.1\)", out)
    assert m and abs(float(m.group(1)) - 0.787755) < 1e-3 and out.count("Failure") == 1, out[-3000:]


def test_sortn_benchmark_direct(hip_lib):
    """benchmarks/SortNBenchmark.cpp as-is, BM_DirectSort<N>.  It sorts with
    SignConfig(CompositeSignConfig(4, 3, 3)) (SortNBenchmark.cpp:100) on the
    depth DirectSort<N>::getSizeParameters budgets for CompositeSign(3, dg, df)
    (src/sort_algo.h:94-198): CompositeSign<4> costs 5 levels per g4 (PS
    degree 27) and 4 per f4, so the rank alone needs 2 + 3*5 + 3*4 = 29 levels
    against N=4's whole budget of 23.  The reference's own benchmark therefore
    exhausts the modulus chain in constructRank; the engine must fail the same
    way (a C++ exception out of sort()), not silently return garbage."""
    rc, out = run(exe("SortNBenchmark"), "--benchmark_filter=BM_DirectSort<4>")
    assert rc != 0 and "multiplicative depth exhausted" in out, out[-3000:]


def test_direct_sort_h1_test(hip_lib):
    """tests/DirectSortH1Test.cpp as-is (sort_hybrid1):
    N = 4 ... 256 at ring 2^17, HEStd_128_classic, its own depth / key
    tables; gates: level == multDepth, max error < 0.01.  The reference
    publishes 93.53 s and 2^-19.30 at N=256 (comparison/experimental_results/
    ours_hybrid1/total_results.txt:151-174)."""
    rc, out = run(exe("DirectSortH1Test"), "--gtest_filter=*/0.*:*/1.*:*/2.*:*/3.*:*/4.*:*/5.*:*/6.*",
                  timeout=600)
    errs = [float(x) for x in re.findall(r"Maximum error: ([0-9.e+-]+)", out)]
    times = [int(x) for x in re.findall(r"Execution time: (\d+) ms", out)]
    print("max errors:", errs, "\nexecution ms:", times)
    assert rc == 0, out[-4000:]
    assert "7 tests ran, 0 failed" in out
    assert len(errs) == 7 and max(errs) < 0.01


def test_direct_sort_h1_test_large(hip_lib):
    """tests/DirectSortH1Test.cpp as-is, the two largest sizes: N = 512 and
    1024 (depth 53 / 56, CompositeSign(3,4,2) / (3,5,2)), which the reference
    publishes at 2^-18.51 and 2^-17.85."""
    rc, out = run(exe("DirectSortH1Test"), "--gtest_filter=*/7.*:*/8.*", timeout=600)
    errs = [float(x) for x in re.findall(r"Maximum error: ([0-9.e+-]+)", out)]
    times = [int(x) for x in re.findall(r"Execution time: (\d+) ms", out)]
    print("max errors:", errs, "\nexecution ms:", times)
    assert rc == 0, out[-4000:]
    assert "2 tests ran, 0 failed" in out
    assert len(errs) == 2 and max(errs) < 0.01


def test_bitonic_sort_test(hip_lib):
    """tests/BitonicSortTest.cpp as-is: BitonicSort<4> at ring 2^12, depth 58,
    two meta-bootstraps (EvalBootstrap(ct, 2, 20)); max error < 1, none > 0.1."""
    rc, out = run(exe("BitonicSortTest"))
    assert rc == 0 and "1 tests ran, 0 failed" in out, out[-3000:]
    err = float(re.search(r"Maximum error: ([0-9.e+-]+)", out).group(1))
    print("BitonicSortTest max error", err)
    assert err < 1e-3


def test_sortn_benchmark_bitonic(hip_lib):
    """benchmarks/SortNBenchmark.cpp as-is, BM_BitonicSort<4> and <8>: ring
    2^17, depth 58, levelBudget {4,4} (SortNBenchmark.cpp:62-91) -- the
    bitonic half of the benchmark runs to completion on the engine."""
    rc, out = run(exe("SortNBenchmark"), "--benchmark_filter=BM_BitonicSort<(4|8)>", timeout=600)
    print(out[-1500:])
    assert rc == 0, out[-3000:]
    assert re.search(r"BM_BitonicSort<4>\S*\s+[0-9.]+ ms", out) and re.search(r"BM_BitonicSort<8>\S*\s+[0-9.]+ ms", out)


@pytest.mark.parametrize("prog,count", [("KWayMaskingTest", 4), ("KWaySortUtilsTest", 11), ("KWayEvalUtilsTest", 6),
                                        ("KWaySorterTest", 7), ("KWaySortTest", 1)])
def test_kway_unit_tests(hip_lib, prog, count):
    """The k-way unit tests and KWaySortTest (512 at ring 2^10) on the product."""
    rc, out = run(exe(prog), timeout=400)
    assert rc == 0 and f"{count} tests ran, 0 failed" in out, out[-3000:]


def test_kway_sort2_test(hip_lib):
    """tests/k-way/KWaySort2Test.cpp as-is: KWayAdapter<N>, k = 2, at ring 2^17,
    HEStd_128_classic, depth 40, scale 59, levelBudget {4,4} / {5,5}, sparse
    slots = N, CompositeSign(3, d_f, d_g) with lazy bootstrapping; max error
    < 0.01 and none >= 0.01.  N = 4 .. 1024 (BASELINE config 4 is N = 1024)."""
    rc, out = run(exe("KWaySort2Test"), timeout=900)
    errs = [float(x) for x in re.findall(r"Maximum error: ([0-9.e+-]+)", out)]
    times = [int(x) for x in re.findall(r"Execution time: (\d+) ms", out)]
    print("max errors:", errs, "\nexecution ms:", times)
    assert rc == 0, out[-4000:]
    assert "9 tests ran, 0 failed" in out


@pytest.mark.parametrize("prog,count", [("KWaySort3Test", 5), ("KWaySort5Test", 3)])
def test_kway_sort35_test(hip_lib, prog, count):
    """tests/k-way/KWaySort{3,5}Test.cpp as-is: k = 3 (N = 9 .. 729) and k = 5
    (N = 25 .. 625) at ring 2^17, the 3- / 4- / 5- / mixed 2..5-sorter stages."""
    rc, out = run(exe(prog), timeout=900)
    errs = [float(x) for x in re.findall(r"Maximum error: ([0-9.e+-]+)", out)]
    times = [int(x) for x in re.findall(r"Execution time: (\d+) ms", out)]
    print(prog, "max errors:", errs, "\nexecution ms:", times)
    assert rc == 0, out[-4000:]
    assert f"{count} tests ran, 0 failed" in out


def test_direct_sort_htest(hip_lib):
    """tests/DirectSortHTest.cpp as-is (sort_hybrid): N = 4 ...
    1024 at ring 2^17, HEStd_128_classic, its own depth / key tables; the
    scaled-sinc series below N = 256, the composite-sign indicator from 256
    on.  Gates: level == multDepth, max error < 0.01, every instantiation."""
    rc, out = run(exe("DirectSortHTest"), timeout=400)
    errs = [float(x) for x in re.findall(r"Maximum error: ([0-9.e+-]+)", out)]
    print("max errors:", errs)
    assert rc == 0, out[-4000:]
    assert "9 tests ran, 0 failed" in out
    assert len(errs) == 9 and max(errs) < 0.01


def test_direct_sort_h2test(hip_lib):
    """tests/DirectSortH2Test.cpp as-is (sort_hybrid2: the scaled-sinc series
    at every N) for N = 4 ... 128, at ring 2^17, HEStd_128_classic; gates:
    level == multDepth, max error < 0.01.

    N >= 256 is not gated: there the series' own Paterson-Stockmeyer noise
    exceeds 0.01.  tools/prec_probe.cpp h2s isolates it -- the series on a
    FRESH encryption of the exact differences errs 1.6e-4 / 1.6e-3 / 1.8e-2
    at N = 64 / 128 / 256, all of it at the hits x = 0, where every giant
    step T_{2^i}(0) = +-1 multiplies its rounding noise by 4 per doubling;
    the rank's own error explains < 3e-5 (profiles/r03_h2_series_attribution.txt).
    The reference's sort_hybrid switches to the composite-sign indicator at
    N >= 256 for this reason (sort_algo.h:894-1062); it publishes no hybrid2
    results."""
    rc, out = run(exe("DirectSortH2Test"), "--gtest_filter=*/0.*:*/1.*:*/2.*:*/3.*:*/4.*:*/5.*", timeout=400)
    errs = [float(x) for x in re.findall(r"Maximum error: ([0-9.e+-]+)", out)]
    print("max errors:", errs)
    assert rc == 0, out[-4000:]
    assert "6 tests ran, 0 failed" in out
    assert len(errs) == 6 and max(errs) < 0.01


def test_direct_sort_h2test_large_fails_as_attributed(hip_lib):
    """tests/DirectSortH2Test.cpp as-is at N = 256, 512, 1024 (VERDICT r3
    item 7): the reference's own test cannot pass at 40-bit scale, and the
    engine fails it exactly the attributed way -- each sort completes at its
    level, and only the max-error gate trips, with errors of the size the
    Paterson-Stockmeyer rounding noise at the hits x = 0 predicts
    (0.026 / 0.072 / 0.25 measured in round 3), never a
    crash, an exception or a level mismatch.  The scaled sinc must hold on all
    of [-1, 1] (its hits sit at x = 0, where every giant step T_{2^i} is at an
    extremum), so no affine re-expansion moves them (that is what rescues the
    doubled sinc in DirectSort); the reference's sort_hybrid
    switches to the composite-sign indicator at N >= 256 for this reason.

    The test draws a fresh input every run (tests/utils.h shuffles with
    std::random_device), and at N = 256 the error straddles the gate
    (0.0097 ... 0.026 over runs): N = 256 may pass or fail, N = 512 and 1024
    always fail.

    Gates per N, from the runs on record (each the maximum over the N hits of
    the series' rounding noise, so it spreads from run to run): N = 256
    0.0097 / 0.026 (rounds 3, 5), N = 512 0.072 / 0.073, N = 1024 0.25 /
    0.381 (round 3; round 5, gpurun_out/r05m_gpu_tests.log).  Each window is
    the observed range widened x2 to x3 on either side; and the attributed
    mechanism (noise x4 per giant-step doubling, one more doubling per
    doubling of N) makes the error grow with N, which is asserted too --
    a regression of a different kind (a wrong level, a wrong polynomial)
    breaks either the windows or the order."""
    rc, out = run(exe("DirectSortH2Test"), "--gtest_filter=*/6.*:*/7.*:*/8.*", timeout=600)
    errs = [float(x) for x in re.findall(r"Maximum error: ([0-9.e+-]+)", out)]
    levels = [int(x) for x in re.findall(r"Result Level: (\d+)", out)]
    print("max errors:", errs, "levels:", levels)
    assert rc != 0
    assert "3 tests ran, 3 failed" in out or "3 tests ran, 2 failed" in out, out[-3000:]
    assert len(errs) == 3, errs
    windows = ((0.004, 0.08), (0.025, 0.22), (0.08, 0.9))  # N = 256 (either side of 0.01), 512, 1024
    assert all(lo < e < hi for e, (lo, hi) in zip(errs, windows)), errs
    assert errs[1] > 0.01 and errs[2] > 0.01, errs  # 512 and 1024 fail the reference's gate
    assert errs[0] < errs[1] < errs[2], errs  # grows with N, as the attribution predicts
    assert "unexpected exception" not in out, out[-3000:]
    assert "Use the level returned" not in out, out[-3000:]  # the level gate holds


def test_direct_sort_ntest(hip_lib):
    """tests/DirectSortNTest.cpp as-is (ring 2^13, HEStd_NotSet, the depth of
    DirectSort<N>::getSizeParameters, CompositeSign(3, 6, 3) at every N).

    Every test that can run passes: RotationIndexCheck / -WithNoise
    (rotationIndexCheckN on exact and +-0.001-noisy ranks) for N = 4 ... 512,
    ConstructRank for N = 64 ... 2048.  The rest fail in the reference the
    same way, by construction of the test: (3, 6, 3) costs more levels than
    getSizeParameters budgets for the default sign config at N <= 32 (rank)
    and at every N (rank + placement, SortTest), so the modulus chain runs out
    (OpenFHE throws on a rescale past the last tower; the engine throws
    "no levels left"); and N = 1024, 2048 need N*N <= 4096 slots for the
    placement's batches, so rotationIndexCheckN sums an empty vector
    (EvalAddMany throws on an empty input, as OpenFHE's does)."""
    rc, out = run(exe("DirectSortNTest"), timeout=400)
    ok = set(re.findall(r"\[       OK \] DirectSort/DirectSortTestFixture/(\d+)\.(\w+)", out))
    bad = set(re.findall(r"\[  FAILED  \] DirectSort/DirectSortTestFixture/(\d+)\.(\w+)", out))
    want_ok = {(str(i), t) for i in range(8) for t in ("RotationIndexCheck", "RotationIndexCheckWithNoise")}
    want_ok |= {(str(i), "ConstructRank") for i in range(4, 10)}
    assert ok == want_ok, (sorted(ok ^ want_ok), out[-3000:])
    assert len(ok) + len(bad) == 40
    # the failures are exceptions, never numerical mismatches
    assert "Mismatch at index" not in out, out[-3000:]
    exc = re.findall(r"unexpected exception: (.*)", out)
    assert len(exc) == len(bad)
    assert all("no levels left" in e or "EvalAddMany of an empty vector" in e for e in exc), exc


def test_sinc_test(hip_lib):
    """tests/SincTest.cpp as-is: the scaled-sinc Chebyshev series
    (selectCoefficients<N>) for N = 4 ... 1024, in plaintext and encrypted on
    65536 slots at ring 2^17.  The plaintext error checks the coefficient
    tables (approximation floor <= 1.2e-6, measured); the encrypted error adds
    the Paterson-Stockmeyer noise (measured 1.1e-6 .. 1.5e-4, gate 2x)."""
    rc, out = run(exe("SincTest"), timeout=300)
    assert rc == 0, out[-3000:]
    plain = [float(x) for x in re.findall(r"L_inf \(plain\) = ([0-9.e+-]+)", out)]
    enc = [float(x) for x in re.findall(r"L_inf \(enc\) = ([0-9.e+-]+)", out)]
    print("plain L_inf:", plain, "\nencrypted L_inf:", enc)
    assert len(plain) == 9 and len(enc) == 9
    assert max(plain) < 1.2e-6
    gates = [3e-6] * 5 + [6e-6, 3e-5, 1.6e-4, 3e-4]   # measured x ~2 (N = 4 ... 1024)
    assert all(e < g for e, g in zip(enc, gates)), list(zip(enc, gates))


def test_direct_sort_benchmark(hip_lib):
    """benchmarks/DirectSortBenchmark.cpp as-is: DirectSort<128> and its
    constructRank with CompositeSign(4, 3, 3) at ring 2^17, depth 44 (the
    FHERMA configuration); the sort ends at level 42 (rank 29 + placement 13
    levels: config.json's depth leaves two unused)."""
    rc, out = run(exe("DirectSortBenchmark"), timeout=300)
    print(out[-600:])
    assert rc == 0, out[-3000:]
    assert "Final Level: 42" in out
    assert re.search(r"BM_DirectSort<128>\s+[0-9.]+ ms", out) and re.search(r"BM_ConstructRank<128>\s+[0-9.]+ ms", out)


def test_rotation_and_sinc_benchmarks(hip_lib):
    """benchmarks/RotationBenchmark.cpp (EvalRotate / EvalFastRotation chains
    of 1 .. 14, RotationComposer batch and tree rotations at 128 slots) and
    benchmarks/SincBenchmark.cpp (scalar scaled_sinc) as-is."""
    rc, out = run(exe("RotationBenchmark"), timeout=300)
    print(out[-1500:])
    assert rc == 0, out[-3000:]
    for name in ["BM_Rotations/14", "BM_FastRotations/14", "BM_BatchRotations", "BM_BatchTreeRotations"]:
        assert re.search(re.escape(name) + r"\s+[0-9.]+ ms", out), name
    rc, out = run(exe("SincBenchmark"), timeout=60)
    assert rc == 0 and "BM_ScaledSincJ" in out, out[-2000:]
