#!/usr/bin/env python3
"""Per-phase device-synchronised wall time of DirectSort<N>::sort
(SFHE_PHASES=1, diagnostics only: the phase syncs serialise the lanes).
    python tools/phases.py [N] [logn]"""
import os, sys, time
os.environ["SFHE_PHASES"] = "1"
sys.path.insert(0, "sorting-fhe_amd/python"); sys.path.insert(0, ".")
import sfhe, bench
N = int(sys.argv[1]) if len(sys.argv) > 1 else 256
logn = int(sys.argv[2]) if len(sys.argv) > 2 else 16
depth, rots = sfhe.direct_sort_params(N, "hip")
e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots)
e.set_quiet(True)
s = e.sorter(N)
ct = e.encrypt(bench.input_vector(N).tolist())
for i in range(3):
    print(f"--- sort {i}", file=sys.stderr, flush=True)
    t0 = time.perf_counter(); o = s.sort(ct, *bench.sign_config(N)); e.sync(); del o
    print(f"total {1e3*(time.perf_counter()-t0):.1f} ms", file=sys.stderr, flush=True)
