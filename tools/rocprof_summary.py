#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace database (rocpd sqlite output).

    python tools/rocprof_summary.py gpurun_out/prof/run_results.db [--n 65536] [--sorts K]

Prints, per kernel: launches, total / average duration, share of GPU time,
and for the kernels whose algorithmic bytes follow from the grid shape
(NTT passes: 16 B per coefficient in+out), the achieved GB/s.
"""
import argparse
import collections
import sqlite3


def short(name: str) -> str:
    s = name.split("(")[0].replace("void ", "")
    return s


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--n", type=int, default=65536, help="ring dimension of the run")
    ap.add_argument("--sorts", type=int, default=0, help="divide totals by this many sorts")
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    db = sqlite3.connect(a.db)
    rows = db.execute("select name, duration, grid_x, grid_y, grid_z from kernels").fetchall()
    agg = collections.defaultdict(lambda: [0, 0, 0.0])
    total = 0
    for name, dur, gx, gy, gz in rows:
        k = short(name)
        agg[k][0] += 1
        agg[k][1] += dur
        total += dur
        if k.startswith("k_ntt<"):
            agg[k][2] += gy * a.n * 16.0  # one pass reads and writes every coefficient once
    print(f"{'kernel':34s} {'calls':>8s} {'total ms':>10s} {'avg us':>8s} {'share':>6s} {'GB/s':>8s}")
    for k, (c, d, b) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        bw = f"{b / d:8.1f}" if b else "       -"
        print(f"{k:34s} {c:8d} {d / 1e6:10.3f} {d / c / 1e3:8.2f} {100.0 * d / total:5.1f}% {bw}")
    print(f"total GPU kernel time {total / 1e6:.3f} ms over {len(rows)} dispatches")
    if a.sorts:
        print(f"per sort: {total / 1e6 / a.sorts:.3f} ms GPU time, {len(rows) / a.sorts:.0f} dispatches")


if __name__ == "__main__":
    main()
