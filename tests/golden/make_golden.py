#!/usr/bin/env python3
"""Generate tests/golden/*.json from the reference's own files (data only).

Runs in the build container, where /root/reference is mounted; the GPU box
and the test suite only read the committed JSON.  Extracted:

* reference_params.json
    - DirectSort<N>::getSizeParameters depth and rotation-key lists
      (src/sort_algo.h:87-201)
    - CompositeSign<3> g3/f3 and CompositeSign<4> g4 (Chebyshev) / f4
      coefficients (src/sign.cpp:9-158)
    - CompareTest inputs / expected outputs / tolerance (tests/CompareTest.cpp:13-63)
    - DecomposeTest key set and numbers (tests/DecomposeTest.cpp:10-13, :64-75)
* hybrid1_published.json
    - the reference's only published outputs: sort_hybrid1 per N (summary
      and each of the 10 trials: ring, depth, sign configuration, time, max /
      average error, result level) from comparison/experimental_results/
      ours_hybrid1/{total_results.txt, trials/trial_*/size_*.txt}
* derived_expectations.json (computed here, recorded with their derivation):
    - the Chebyshev-PS depth table of the reference's OpenFHE (SURVEY a-12 iv)
    - Decomposer NAF(127) = {64, 64, -1} recorded in SURVEY 8(c) from the
      reference's own Decomposer<128>
"""
import json
import os
import re

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def read(rel):
    with open(os.path.join(REF, rel)) as f:
        return f.read()


def nums(s):
    return [float(x) if any(c in x for c in ".eE") else int(x)
            for x in re.findall(r"-?\d+(?:\.\d+)?(?:[eE][-+]?\d+)?", s)]


def size_parameters():
    src = read("src/sort_algo.h")
    start = src.index("static void getSizeParameters")
    end = src.index("parameters.SetScalingModSize(modSize);", start)
    body = src[start:end]
    mod = int(re.search(r"int modSize = (\d+);", body).group(1))
    out = {}
    for m in re.finditer(r"case (\d+):(.*?)break;", body, re.S):
        N = int(m.group(1))
        blk = m.group(2)
        depth = int(re.search(r"multDepth = (\d+);", blk).group(1))
        rots = re.search(r"rotations = \{(.*?)\};", blk, re.S)
        out[str(N)] = {"mult_depth": depth, "rotations": nums(rots.group(1)) if rots else []}
    return {"scaling_mod_size": mod, "by_N": out}


def sign_coefficients():
    src = read("src/sign.cpp")
    c3 = src[src.index("struct CompositeSign<3>"):src.index("struct CompositeSign<4>")]
    g3 = c3[c3.index("g_n("):c3.index("f_n(")]
    f3 = c3[c3.index("f_n("):]

    def frac(block):
        return [float(a) / float(b) for a, b in
                re.findall(r"constexpr double c\d+ = (-?\d+\.\d+) / (\d+\.\d+);", block)]

    c4 = src[src.index("struct CompositeSign<4>"):]
    g4 = re.search(r"std::vector<double> coeffs = \{(.*?)\};", c4, re.S).group(1)
    f4blk = c4[c4.index("f_n("):]
    f4 = [float(v) for v in re.findall(r"constexpr double c\d+ = (-?\d+\.\d+);", f4blk)]
    return {"g3": frac(g3), "f3": frac(f3), "g4_chebyshev": nums(g4), "f4": f4[:8]}


def compare_test():
    src = read("tests/CompareTest.cpp")
    vec = lambda name: nums(re.search(r"std::vector<double> %s = \{(.*?)\};" % name, src).group(1))
    cfg = nums(re.search(r"CompositeSignConfig\((.*?)\)", src).group(1))
    return {
        "scaling_mod_size": int(re.search(r"scalingModSize = (\d+);", src).group(1)),
        "mult_depth": int(re.search(r"multDepth = (\d+);", src).group(1)),
        "ring_dim_log2": int(re.search(r"SetRingDim\(1 << (\d+)\)", src).group(1)),
        "a": vec("a"), "b": vec("b"), "expected": vec("expected"),
        "composite_sign_config": cfg,
        "tolerance": float(re.search(r"EXPECT_NEAR\(.*?, ([\d.]+)\);", src).group(1)),
    }


def decompose_test():
    src = read("tests/DecomposeTest.cpp")
    keys = nums(re.search(r"std::vector<int>\{(.*?)\}", src).group(1))
    numbers = nums(re.search(r"testNumbers = \{(.*?)\};", src, re.S).group(1))
    return {"N": 128, "keys": keys, "numbers": numbers, "wrap": 128}


def hybrid1_published():
    base = "comparison/experimental_results/ours_hybrid1"
    total = read(base + "/total_results.txt")
    out = {}
    for blk in total.split("Results for N = ")[1:]:
        N = int(re.match(r"(\d+)", blk).group(1))
        g = lambda pat: re.search(pat, blk).group(1)
        cfg = nums(g(r"CompositeSign\(([^)]*)\)"))
        out[str(N)] = {"ring_dim": int(g(r"Ring Dimension\s*:\s*(\d+)")),
                       "mult_depth": int(g(r"Multiplicative Depth:\s*(\d+)")),
                       "scaling_mod_size": int(g(r"Scaling Mod Size\s*:\s*(\d+)")),
                       "sign": cfg,
                       "avg_time_s": float(g(r"Average Time\s*:\s*([\d.]+)s")),
                       "max_err_log2": float(g(r"Max Error \(log2\):\s*(-?[\d.]+)")),
                       "avg_err_log2": float(g(r"Average Error \(log2\):\s*(-?[\d.]+)")),
                       "trials": []}
    for t in range(1, 11):
        for N in out:
            txt = read(f"{base}/trials/trial_{t}/size_{N}.txt")
            m = re.search(r"Maximum error: ([-\d.e+]+) \(log2: (-?[\d.]+)\)", txt)
            a = re.search(r"Average error: ([-\d.e+]+) \(log2: (-?[\d.]+)\)", txt)
            out[N]["trials"].append({
                "trial": t,
                "time_ms": int(re.search(r"Execution time: (\d+) ms", txt).group(1)),
                "max_err": float(m.group(1)), "max_err_log2": float(m.group(2)),
                "avg_err": float(a.group(1)), "avg_err_log2": float(a.group(2)),
                "level": int(re.search(r"Result Level: (\d+)", txt).group(1))})
    return {"_source": f"extracted from /root/reference/{base} by tests/golden/make_golden.py (data only)",
            "by_N": out}


def main():
    ref = {
        "_source": "extracted from /root/reference by tests/golden/make_golden.py (data only)",
        "direct_sort_size_parameters": size_parameters(),
        "sign_coefficients": sign_coefficients(),
        "compare_test": compare_test(),
        "decompose_test": decompose_test(),
    }
    with open(os.path.join(HERE, "reference_params.json"), "w") as f:
        json.dump(ref, f, indent=1)
    with open(os.path.join(HERE, "hybrid1_published.json"), "w") as f:
        json.dump(hybrid1_published(), f, indent=1)
    derived = {
        "_source": "derived expectations (see SURVEY.md a-12 (iv) and 8(c))",
        "chebyshev_ps_depth_table": [[5, 3], [13, 4], [27, 5], [59, 6], [119, 7], [247, 8],
                                     [495, 9], [1007, 10], [2031, 11], [4031, 12], [8127, 13]],
        "decompose_naf_127": [[1, 64], [1, 64], [-1, -1]],
        "doubled_sinc_degree": {"4": 42, "8": 70, "16": 126, "32": 232, "64": 438, "128": 848,
                                "256": 1662, "512": 3280, "1024": 6510},
    }
    with open(os.path.join(HERE, "derived_expectations.json"), "w") as f:
        json.dump(derived, f, indent=1)
    print("wrote", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
