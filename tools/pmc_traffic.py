#!/usr/bin/env python3
"""HBM traffic per launch of the hot kernel families from two rocprofv3 PMC
passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950):

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d F -o run -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d W -o run -- python3 bench.py ...
    python tools/pmc_traffic.py F/run_counter_collection.csv W/run_counter_collection.csv \
        --n 65536 --out profiles/pmc_traffic.json

Corrections (/opt/skills/guides/MI355X_MICROARCH.md, HBM section): counters
are in KiB; FETCH_SIZE reports half the bytes of a 16-B-per-lane coalesced
streaming read (x2); WRITE_SIZE is exact for 16-B-per-lane stores.  The NTT
and k_conv / k_ks_inner read and write 16 B per lane where contiguous.

Algorithmic bytes per launch (prims.h): NTT pass 16 B x coefficients of the
launch (rows from the grid: k_ntt<INV, COL, LE> runs n / 2^LE threads per row).
"""
import argparse
import collections
import csv
import hashlib
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def family(name: str):
    s = name.split("(")[0].replace("void ", "")
    if s.startswith("k_ntt_ks"):  # the fused ModUp ROW pass + key inner product
        return "ks_inner"
    if s.startswith("k_ntt"):
        return "ntt"
    if s.startswith("k_conv") or s.startswith("k_mdrs"):
        return "conv"
    if s == "k_ks_inner":
        return "ks_inner"
    return None


def load(path, counter):
    per = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter:
                continue
            per[int(r["Dispatch_Id"])] = (r["Kernel_Name"], int(r["Grid_Size"]), float(r["Counter_Value"]))
    return per


def ntt_rows(name: str, grid: int, n: int) -> int:
    """Rows of one k_ntt<INV, COL, LE> launch: each thread of a pass holds
    2^LE words, so a row takes n / 2^LE threads (Grid_Size = total threads)."""
    m = re.search(r"k_ntt<\s*\w+,\s*\w+,\s*(\d+)", name)
    le = int(m.group(1)) if m else 3
    return grid * (1 << le) // n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--mb-log", default=None,
                    help="microbench stdout: its CONV_ALGO line gives the conversion launches' algorithmic bytes")
    a = ap.parse_args()
    conv_algo = None
    if a.mb_log:
        with open(a.mb_log) as f:
            for line in f:
                m = re.match(r"CONV_ALGO launches=(\d+) bytes=([\d.e+]+)", line)
                if m:
                    conv_algo = (int(m.group(1)), float(m.group(2)))
    fe = load(a.fetch_csv, "FETCH_SIZE")
    wr = load(a.write_csv, "WRITE_SIZE")
    acc = collections.defaultdict(lambda: {"launches": 0, "fetch": 0.0, "write": 0.0, "algo": 0.0})
    # the two passes run the same deterministic program: pair dispatches by
    # order within each family
    fam_f = collections.defaultdict(list)
    fam_w = collections.defaultdict(list)
    # the microbench's plain NTT sweep comes before its first key-switch
    # kernel: NTT launches before that one read and write exactly the tile
    # (and the twiddles); those after it carry the key switch's prologues /
    # epilogues (lift, pre-multiply, the rescale's (a - x) P^-1 and tensor rows)
    ks_first = min((i for i, (nm, _, _) in fe.items()
                    if re.match(r"(void )?k_(conv|mdrs|modup|ntt_ks|ks_inner)", nm)), default=None)
    plain_f = []
    for i, (name, grid, v) in sorted(fe.items()):
        if family(name):
            fam_f[family(name)].append((name, grid, v))
            if family(name) == "ntt":
                plain_f.append(ks_first is None or i < ks_first)
    for _, (name, grid, v) in sorted(wr.items()):
        if family(name):
            fam_w[family(name)].append((name, grid, v))
    out = {}
    for fam in fam_f:
        F, W = fam_f[fam], fam_w.get(fam, [])
        if fam == "conv" and conv_algo:  # the launches the microbench's byte count covers: the last L
            L = conv_algo[0]
            F, W = F[-L:], W[-L:]
        k = min(len(F), len(W))
        fetch = sum(v for _, _, v in F[:k]) * 1024 * 2
        write = sum(v for _, _, v in W[:k]) * 1024
        entry = {"launches": k, "hbm_bytes_per_launch": (fetch + write) / k,
                 "fetch_bytes_per_launch": fetch / k, "write_bytes_per_launch": write / k}
        if fam == "ntt":
            algo = sum(16.0 * ntt_rows(nm, g, a.n) * a.n for nm, g, _ in F[:k])
            entry["algorithmic_bytes_per_launch"] = algo / k
            entry["traffic_over_algorithmic"] = (fetch + write) / algo
            # the excess located by pass (forward / inverse x COL / ROW)
            by = collections.defaultdict(lambda: [0, 0.0, 0.0, 0.0])
            for (nm, g, vf), (_, _, vw), plain in zip(F[:k], W[:k], plain_f):
                m = re.search(r"k_ntt<\s*(\w+),\s*(\w+)", nm)
                key = ("inverse" if m and m.group(1) == "true" else "forward") + " " + \
                      ("COL" if m and m.group(2) == "true" else "ROW")
                for kk in (key, key + (" (plain sweep)" if plain else " (key-switch prims)")):
                    b = by[kk]
                    b[0] += 1
                    b[1] += vf * 1024 * 2
                    b[2] += vw * 1024
                    b[3] += 16.0 * ntt_rows(nm, g, a.n) * a.n
            entry["by_pass"] = {key: {"launches": b[0], "fetch_over_read": b[1] / (b[3] / 2),
                                      "write_over_written": b[2] / (b[3] / 2),
                                      "traffic_over_algorithmic": (b[1] + b[2]) / b[3]}
                                for key, b in sorted(by.items())}
        if fam == "conv" and conv_algo and k == conv_algo[0]:
            entry["algorithmic_bytes_per_launch"] = conv_algo[1] / k
            entry["traffic_over_algorithmic"] = (fetch + write) / conv_algo[1]
        out[fam] = entry
    src = os.path.join(ROOT, "sorting-fhe_amd", "csrc", "hip", "prims_hip.hip")
    with open(src, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()[:16]
    j = {"kernel_source_sha": sha, "ring_dim": a.n,
         "corrections": "KiB->B; FETCH_SIZE x2 (gfx950 16-B/lane streaming read); WRITE_SIZE x1",
         "families": out}
    with open(a.out, "w") as f:
        json.dump(j, f, indent=1)
    print(json.dumps(j, indent=1))


if __name__ == "__main__":
    main()
