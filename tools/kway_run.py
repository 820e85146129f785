"""k-way sort at BASELINE config 4 (developer tool, GPU): KWayAdapter<1024>
(k = 2, M = 10) at ring 2^17 with bootstrapping, as bench.py's kway leg; a
cold and a warm sort.  With SFHE_BOOT_TRACE=1 the engine prints every
bootstrap's synchronised time, which this tool totals per sort (the
bootstrapping share of the k-way time).

    SFHE_BOOT_TRACE=1 python tools/kway_run.py [--N 1024] [--sorts 2]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sorting-fhe_amd", "python"))
import numpy as np  # noqa: E402
import sfhe  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=1024)
    ap.add_argument("--k", type=int, default=2)
    ap.add_argument("--sorts", type=int, default=2)
    a = ap.parse_args()
    M = round(np.log(a.N) / np.log(a.k))
    batch, depth, budget, rots = sfhe.kway_params(a.N)
    eng = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << 17, batch_size=batch, scaling_mod_size=59,
                      secure=True, rotations=rots, seed=7 + a.N)
    eng.set_quiet(True)
    t0 = time.perf_counter()
    eng.bootstrap_setup(budget, batch)
    print(f"bootstrap setup {time.perf_counter() - t0:.1f} s", flush=True)
    x = np.random.default_rng(a.N).permutation(a.N) / a.N
    ct = eng.encrypt(x.tolist())
    sorter = eng.kway(a.k, M)
    for i in range(a.sorts):
        eng.sync()
        sys.stderr.write(f"SORT {i} begin\n")
        sys.stderr.flush()
        t0 = time.perf_counter()
        out = sorter.sort(ct, 3, 2, 5, depth)
        eng.sync()
        dt = time.perf_counter() - t0
        sys.stderr.write(f"SORT {i} end {dt * 1e3:.1f} ms\n")
        sys.stderr.flush()
        err = float(np.max(np.abs(np.array(eng.decrypt(out))[:a.N] - np.sort(x))))
        print(f"sort {i}: {dt:.2f} s, level {out.level}, max err {err:.3g}", flush=True)


if __name__ == "__main__":
    main()
