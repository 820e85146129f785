#!/usr/bin/env python3
"""GPU utilisation from a rocprofv3 kernel trace (csv): busy-interval union,
summed kernel time (>= union when lanes overlap), and per-kernel shares.
    python tools/trace_util.py run_kernel_trace.csv [--last-ms W]"""
import argparse, collections, csv
ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--last-ms", type=float, default=0.0, help="only the final W ms of the trace")
a = ap.parse_args()
rows = list(csv.DictReader(open(a.trace)))
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", ""))
            for r in rows)
end = max(e for _, e, _ in iv)
if a.last_ms:
    iv = [x for x in iv if x[0] >= end - a.last_ms * 1e6]
start = iv[0][0]
union = 0; cur_s, cur_e = iv[0][0], iv[0][1]
for s, e, _ in iv[1:]:
    if s > cur_e:
        union += cur_e - cur_s; cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
union += cur_e - cur_s
tot = sum(e - s for s, e, _ in iv)
wall = end - start
print(f"window {wall/1e6:.2f} ms, GPU busy (union) {union/1e6:.2f} ms ({100*union/wall:.0f}%), "
      f"summed kernel time {tot/1e6:.2f} ms (avg concurrency {tot/max(union,1):.2f}), {len(iv)} kernels")
agg = collections.defaultdict(lambda: [0, 0])
for s, e, k in iv:
    agg[k][0] += 1; agg[k][1] += e - s
for k, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:14]:
    print(f"  {k:26s} {c:6d} {d/1e6:8.2f} ms {100*d/tot:5.1f}%  avg {d/c/1e3:6.2f} us")
