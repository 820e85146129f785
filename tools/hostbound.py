import sys, time
sys.path.insert(0, "sorting-fhe_amd/python"); sys.path.insert(0, ".")
import sfhe, bench
N, logn = 256, 16
depth, rots = sfhe.direct_sort_params(N, "hip")
e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots)
e.set_quiet(True)
s = e.sorter(N)
ct = e.encrypt(bench.input_vector(N).tolist())
for _ in range(2):
    o = s.sort(ct, 3, 4, 2); del o
e.sync()
for _ in range(3):
    t0 = time.perf_counter(); o = s.sort(ct, 3, 4, 2); t1 = time.perf_counter(); e.sync(); t2 = time.perf_counter(); del o
    print(f"enqueue {1e3*(t1-t0):.1f} ms, total {1e3*(t2-t0):.1f} ms")
