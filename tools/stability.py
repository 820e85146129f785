"""Per-sort wall times over a long loop (diagnostics for run-to-run variance).
    python tools/stability.py [sorts]   -> one line per sort: t_since_start_s ms"""
import sys, time
sys.path.insert(0, "sorting-fhe_amd/python"); sys.path.insert(0, ".")
import sfhe, bench
N, logn = 256, 16
depth, rots = sfhe.direct_sort_params(N, "hip")
e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots)
e.set_quiet(True)
s = e.sorter(N)
ct = e.encrypt(bench.input_vector(N).tolist())
T0 = time.perf_counter()
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 60):
    e.sync(); t0 = time.perf_counter(); o = s.sort(ct, 3, 4, 2); e.sync(); t1 = time.perf_counter(); del o
    print(f"{t0 - T0:8.3f} {1e3 * (t1 - t0):8.2f}", flush=True)
