"""Config-5 shaped sort under a graph (developer tool): DirectSort<256> at ring
2^17 (HEStd_128_classic), the first sort eager, the second captured into a
hipGraph, then `--replays` graph replays; prints the per-sort time and the
error.  Used to profile the 2^17 graph (rocprofv3 --kernel-trace) and to
reproduce the round-2 profiler crash with SFHE_CRASH_TRACE=1.

    python tools/c5_graph.py [--replays 3] [--N 256] [--logn 17]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sorting-fhe_amd", "python"))
import sfhe  # noqa: E402
from oracle import slotsim  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replays", type=int, default=3)
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--logn", type=int, default=17)
    a = ap.parse_args()
    N = a.N
    depth, rots = sfhe.direct_sort_params(N, "hip")
    t0 = time.time()
    e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << a.logn, batch_size=N, secure=a.logn >= 17,
                    rotations=rots, seed=20251205 + N)
    e.set_quiet(True)
    print(f"setup {time.time() - t0:.1f} s", flush=True)
    x = slotsim.input_vector(N)
    ct = e.encrypt(x.tolist())
    s = e.sorter(N)
    cfg = slotsim.default_sign_config(N)
    for i in range(2 + a.replays):
        e.sync()
        t0 = time.perf_counter()
        out = s.sort(ct, *cfg)
        e.sync()
        kind = "eager" if i == 0 else ("capture" if i == 1 else "replay")
        print(f"sort {i} ({kind}): {1e3 * (time.perf_counter() - t0):.1f} ms, graph nodes {s.graph_nodes()}",
              flush=True)
    err = np.max(np.abs(np.array(e.decrypt(out))[:N] - np.sort(x)))
    print(f"max err {err:.3g} level {out.level}/{depth}", flush=True)


if __name__ == "__main__":
    main()
