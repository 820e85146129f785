#!/usr/bin/env python3
"""Where the cold sort's time goes (developer tool; bench.py's trials.cold_ms).

Runs the metric sort (DirectSort<256>, ring 2^16, depth 34) three times
eagerly with SFHE_PHASES=1 (device-synchronised phase marks on stderr:
core/sort_algo.h PhaseTimer): the first sort of a fresh sorter (mask
generation, encodings, first-use uploads), then two warm eager sorts.  The
per-phase difference between the first and the warm sorts is the host-side
first-use cost of each phase.

    python tools/cold_probe.py > gpurun_out/cold_probe.txt 2>&1
"""
import os
import sys
import time

os.environ["SFHE_PHASES"] = "1"
os.environ["SFHE_GRAPH"] = "0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sorting-fhe_amd", "python"))
import sfhe  # noqa: E402
import bench  # noqa: E402

N, logn = 256, 16
depth, rots = sfhe.direct_sort_params(N, "hip")
t0 = time.perf_counter()
e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots, seed=7)
e.set_quiet(True)
print(f"context + keys: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
ct = e.encrypt(bench.input_vector(N).tolist())
e.sync()
t0 = time.perf_counter()
s = e.sorter(N)
e.sync()
print(f"sorter: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
for k in range(3):
    sys.stderr.write(f"==== sort {k} ({'cold' if k == 0 else 'warm, eager'})\n")
    sys.stderr.flush()
    e.sync()
    t0 = time.perf_counter()
    o = s.sort(ct, *bench.sign_config(N))
    e.sync()
    print(f"sort {k}: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
    del o
