#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace (csv) into sorts and summarise one of them.

    python tools/trace_segments.py gpurun_out/prof/run_kernel_trace.csv [--gap-us 300] [--seg K]

A sort is a run of kernels with no idle gap longer than --gap-us (the bench
synchronises the device between sorts).  Prints every segment (kernels,
wall span, GPU-busy union), then a per-kernel table of segment --seg
(default: the median-length segment among the graph-replayed ones, i.e. the
last run of equal-length segments).
"""
import argparse
import collections
import csv


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--gap-us", type=float, default=300.0)
    ap.add_argument("--seg", type=int, default=-1)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]),
                         int(r["Workgroup_Size_X"])))
    rows.sort()
    segs, cur, end = [], [], None
    for r in rows:
        if end is not None and r[0] - end > a.gap_us * 1e3:
            segs.append(cur)
            cur = []
        cur.append(r)
        end = r[1] if end is None else max(end, r[1])
    if cur:
        segs.append(cur)

    def busy(seg):
        tot, ce, cs = 0, None, None
        for s, e, *_ in seg:
            if ce is None or s > ce:
                if ce is not None:
                    tot += ce - cs
                cs, ce = s, e
            else:
                ce = max(ce, e)
        return tot + (ce - cs)

    big = [i for i, s in enumerate(segs) if len(s) > 500]
    for i, s in enumerate(segs):
        if len(s) > 500:
            span = max(r[1] for r in s) - s[0][0]
            print(f"seg {i:3d}: {len(s):6d} kernels, span {span/1e6:8.2f} ms, busy {busy(s)/1e6:8.2f} ms")
    # default: the first whole sort -- the first segment with (nearly) the
    # largest kernel count (a timed sort; later ones may be split by gaps or
    # followed by other legs' segments)
    most = max(len(segs[i]) for i in big)
    whole = [i for i in big if len(segs[i]) >= 0.99 * most]
    k = a.seg if a.seg >= 0 else whole[0]
    seg = segs[k]
    agg = collections.defaultdict(lambda: [0, 0])
    for s, e, name, *_ in seg:
        agg[name][0] += 1
        agg[name][1] += e - s
    tot = sum(v[1] for v in agg.values())
    span = max(r[1] for r in seg) - seg[0][0]
    print(f"\nsegment {k}: span {span/1e6:.2f} ms, busy {busy(seg)/1e6:.2f} ms, sum of kernel durations {tot/1e6:.2f} ms")
    print(f"{'kernel':34s} {'calls':>7s} {'ms':>8s} {'avg us':>8s} {'share':>6s}")
    for name, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{name:34s} {c:7d} {d/1e6:8.2f} {d/c/1e3:8.2f} {100*d/tot:5.1f}%")


if __name__ == "__main__":
    main()
