#!/usr/bin/env python3
"""Rows per NTT launch in one sort of a rocprofv3 kernel trace (developer
tool): the grid's y extent is the launch's row count (k_ntt: blockIdx.y =
row).  Prints the distribution over the median-length segment's NTT passes.

    python tools/ntt_rows.py gpurun_out/prof/run_kernel_trace.csv [--gap-us 300]
"""
import argparse
import collections
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap-us", type=float, default=300.0)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         int(r["Grid_Size_Y"])))
    rows.sort()
    segs, cur, end = [], [], None
    for r in rows:
        if end is not None and r[0] - end > a.gap_us * 1e3:
            segs.append(cur)
            cur = []
        cur.append(r)
        end = r[1] if end is None else max(end, r[1])
    segs.append(cur)
    big = [s for s in segs if len(s) > 1000]
    seg = sorted(big, key=len)[len(big) // 2]
    ys = [r[3] for r in seg if "k_ntt<" in r[2]]  # not k_ntt_ks (the fused key inner product)
    dur = [(r[1] - r[0]) / 1e3 for r in seg if "k_ntt<" in r[2]]
    print(f"segment of {len(seg)} kernels: {len(ys)} NTT passes")
    print(f"rows per pass: mean {statistics.mean(ys):.1f}, median {statistics.median(ys)}, "
          f"row-weighted mean {sum(y * y for y in ys) / sum(ys):.1f}")
    hist = collections.Counter()
    t = collections.Counter()
    for y, d in zip(ys, dur):
        b = 1 if y <= 1 else 4 if y <= 4 else 8 if y <= 8 else 16 if y <= 16 else 32 if y <= 32 else 64 if y <= 64 else 128
        hist[b] += 1
        t[b] += d
    print("rows <=   passes   ms     us/pass")
    for b in sorted(hist):
        print(f"{b:7d} {hist[b]:8d} {t[b] / 1e3:6.2f} {t[b] / hist[b]:9.2f}")


if __name__ == "__main__":
    main()
