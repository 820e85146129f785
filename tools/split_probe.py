#!/usr/bin/env python3
"""One rank's share of a batch-split metric sort, emulated on one GPU
(developer tool).

Rank 0 of two batch groups runs batch 0 of each phase and all-gathers the
parts; here the group communicator is a host stand-in that hands back the
rank's own part for both groups, so the sort runs exactly rank 0's
operations (its result is wrong: the other batch is a copy).  Host-transport
contexts run eagerly, so both sides are timed eagerly (SFHE_GRAPH=0): the
ratio of one rank's time to the unsplit sort's is the W = 2 estimate.

    python tools/split_probe.py > gpurun_out/split_probe.txt 2>&1
"""
import ctypes as C
import os
import sys
import time

os.environ["SFHE_GRAPH"] = "0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sorting-fhe_amd", "python"))
import sfhe  # noqa: E402
import bench  # noqa: E402


class SelfComm:
    """allgather: the rank's own block in every slot (no second rank)."""
    world = 2

    def allgather(self, rank, send, recv, nbytes):
        for r in range(self.world):
            C.memmove(recv + r * nbytes, send, nbytes)


def run(groups, reps=5):
    N, logn = 256, 16
    depth, rots = sfhe.direct_sort_params(N, "hip")
    g = ("host", 0, 2, SelfComm()) if groups else None
    e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots, seed=7, groups=g)
    e.set_quiet(True)
    s = e.sorter(N)
    ct = e.encrypt(bench.input_vector(N).tolist())
    ts = []
    for _ in range(reps + 1):
        e.sync()
        t0 = time.perf_counter()
        o = s.sort(ct, *bench.sign_config(N))
        e.sync()
        ts.append((time.perf_counter() - t0) * 1e3)
        del o
    e.close()
    return sorted(ts[1:])[len(ts[1:]) // 2]


full = run(False)
half = run(True)
print(f"metric sort, eager: unsplit {full:.1f} ms, one rank of a 2-group batch split {half:.1f} ms, "
      f"ratio {full / half:.2f}")
