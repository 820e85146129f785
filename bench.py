#!/usr/bin/env python3
"""Benchmark: encrypted rank sort (DirectSort<N>::sort) on MI355X.

Contract (see task README): ``python bench.py --gpus N --steps K --warmup W``
prints ONE JSON line on rank 0.  A step is one ``DirectSort<N>::sort`` of one
encrypted array (reference src/sort_algo.h:752-774, timed like
tests/DirectSortTest.cpp:129-136) at the metric configuration of
BASELINE.json: N=256, ring 2^16, depth 34, CompositeSign(3,4,2), scale 40.

Multi-GPU: one process per GPU.  Default: every rank sorts its own array
(independent replicas, no data-path collective) -> weak scaling; value =
comparisons/s of the whole job = world * N^2 * K / max-over-ranks(time).
``--shard rccl``: the ranks limb-shard ONE sort (rank r holds
the RNS limbs i % world == r; RCCL all-gather at ModUp / ModDown, broadcast at
rescale) -> strong scaling; value = N^2 * K / max-over-ranks(time).
``--shard host`` runs the same over the gloo host transport (a rehearsal of
the sharded bench on one GPU: SFHE_BENCH_DEVICE=0 puts every rank on it).

Extra fields: ``roofline`` (dominant kernel family, timed live with HIP
events on the engine's stream over the timed region) and ``cpu_baseline``
(the C oracle on a bounded sample, rank 0 only, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sorting-fhe_amd", "python"))

import sfhe  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md

WORKLOADS = {
    # name: (N, logn, secure)
    "directsort_n256_2e16": (256, 16, False),  # metric config (BASELINE.json)
    "directsort_n128_2e16": (128, 16, False),  # config 3
    "directsort_n256_2e17": (256, 17, True),   # config 5 shape (single GPU)
    "directsort_n8_2e17": (8, 17, True),       # config 1 shape
}


def input_vector(N: int):
    """Seeded random permutation of {k/N} (restates tests/utils.h:28-51 with
    std::mt19937(20251205+N) semantics replaced by numpy's generator; the
    sort's cost does not depend on the permutation)."""
    import numpy as np
    rng = np.random.default_rng(20251205 + N)
    return (rng.permutation(N) / N).astype(float)


def sign_config(N: int):
    # SignConfig(CompositeSignConfig(3, dg, df)) of DirectSortTest.cpp:104-118
    if N <= 16:
        return (3, 2, 2)
    if N <= 128:
        return (3, 3, 2)
    return (3, 4, 2)


def dist_init():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("SFHE_BENCH_BACKEND", "gloo")
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return world, rank, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(world, x: float) -> float:
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed_steps(step, sync, world: int, steps: int, warmup: int, before_timed=None) -> float:
    """W untimed warmup steps, then exactly K steps bracketed by a barrier and
    a device sync on both sides; returns the max over ranks of the K-step
    wall time (seconds)."""
    for _ in range(warmup):
        step()
    sync()
    if before_timed:
        before_timed()
    barrier(world)
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    t1 = time.perf_counter()
    barrier(world)
    return max_over_ranks(world, t1 - t0)


def cpu_baseline(N, logn, secure, depth, seconds, gpu_bytes_per_sort):
    """Bounded CPU sample on the C oracle (test infrastructure; never the
    measured path): EvalMult + relinearise + rescale on the metric context's
    top level, repeated for ~`seconds`; the sort time is extrapolated with
    the same algorithmic-byte model the GPU run reports (op_stats)."""
    import numpy as np
    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    eng = sfhe.Engine("oracle", mult_depth=depth, ring_dim=1 << logn, batch_size=N, secure=secure,
                      seed=99)
    rng = np.random.default_rng(1)
    a = eng.encrypt(rng.uniform(-1, 1, N).tolist())
    b = eng.encrypt(rng.uniform(-1, 1, N).tolist())
    eng.op_stats(reset=True)
    reps = 0
    t0 = time.perf_counter()
    while True:
        c = eng.mult(a, b)
        del c
        reps += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    bps = eng.op_stats()["algo_bytes"] / dt
    sort_s = gpu_bytes_per_sort / bps
    info = eng.info()
    return {
        "value": N * N / sort_s,
        "unit": "cmp/s",
        "cores": cores,
        "kind": "port",
        "sample": (f"C oracle (OpenMP, {cores} threads): {reps} x EvalMult+relin+rescale at the top "
                   f"level ({info['num_q']} Q limbs, n=2^{logn}) in {dt:.1f} s = {bps / 1e9:.2f} "
                   f"algorithmic GB/s; sort time extrapolated over "
                   f"{gpu_bytes_per_sort / 1e9:.1f} GB/sort -> {sort_s:.1f} s/sort"),
        "sort_seconds": sort_s,
    }


def pmc_traffic(family: str):
    """HBM bytes per launch for `family` from the committed PMC summary
    (tools/pmc_traffic.py output), if it was taken on the current kernels."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            j = json.load(f)
    except (OSError, ValueError):
        return None
    src = os.path.join(ROOT, "sorting-fhe_amd", "csrc", "hip", "prims_hip.hip")
    import hashlib
    with open(src, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()[:16]
    if j.get("kernel_source_sha") != sha:
        return None
    return j.get("families", {}).get(family, {}).get("hbm_bytes_per_launch")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="directsort_n256_2e16", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-seconds", type=float, default=15.0)
    ap.add_argument("--trials", type=int, default=10,
                    help="per-sort trials after the timed region (median/min/max, pure and as-test)")
    ap.add_argument("--shard", choices=("rccl", "host"), default=None,
                    help="limb-shard one sort over the ranks instead of running replicas")
    args = ap.parse_args(argv)

    world, rank, local = dist_init()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    N, logn, secure = WORKLOADS[args.workload]
    depth, rots = sfhe.direct_sort_params(N, "hip")
    cfg = sign_config(N)

    device = int(os.environ.get("SFHE_BENCH_DEVICE", local))
    shard, seed = None, 20251205 + N + 7919 * rank
    if args.shard and world > 1:
        import torch.distributed as dist
        seed = 20251205 + N  # every rank builds the same keys
        if args.shard == "rccl":
            uid = [sfhe.comm_uid("hip") if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            shard = ("rccl", rank, world, uid[0])
        else:
            shard = ("host", rank, world, sfhe.GlooComm())
    eng = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, secure=secure,
                      rotations=rots, seed=seed, device=device, shard=shard)
    eng.set_quiet(True)
    sorter = eng.sorter(N)
    x = input_vector(N)
    ct = eng.encrypt(x.tolist())  # input resident in HBM before timing

    period = int(os.environ.get("SFHE_BENCH_TIMING_PERIOD", "13"))
    families = ("ntt", "conv", "ks_inner")

    def step():
        out = sorter.sort(ct, *cfg)
        del out

    def start_counters():
        eng.op_stats(reset=True)
        for fam in families:
            eng.kernel_timing(fam, period)

    dt = timed_steps(step, eng.sync, world, args.steps, args.warmup, start_counters)
    stats = eng.op_stats()
    kt = {fam: eng.kernel_timing_read(fam) for fam in families}
    for fam in families:
        eng.kernel_timing(fam, 0)

    # per-sort trials, "pure" (plain Encryption, SortNBenchmark)
    # and "as-test" (DebugEncryption: the three PRINT_PT decrypts inside sort(),
    # DirectSortTest.cpp:129-136), median / min / max like run_experiments.sh
    def trial_ms(srt, k):
        ts = []
        for _ in range(k):
            eng.sync()
            t0 = time.perf_counter()
            o = srt.sort(ct, *cfg)
            eng.sync()
            ts.append((time.perf_counter() - t0) * 1e3)
            del o
        return ts

    def stats3(ts):
        import statistics
        return {"median": statistics.median(ts), "min": min(ts), "max": max(ts)} if ts else None
    trials = None
    if args.trials > 0:
        pure = trial_ms(sorter, args.trials)
        as_test = trial_ms(eng.sorter(N, debug=True), args.trials)
        trials = {"count": args.trials, "pure_ms": stats3(pure), "as_test_ms": stats3(as_test),
                  "note": "each trial one sort with a device sync on both sides (rank-local, after the timed region)"}

    # dominant timed family: estimated total time = timed ms * launches / timed
    def est_ms(k):
        return k["ms"] * k["launches"] / k["timed"] if k["timed"] else 0.0
    dom = max(families, key=lambda f: est_ms(kt[f]))
    k = kt[dom]
    achieved = k["bytes"] / (k["ms"] / 1e3) / 1e9 if k["ms"] else 0.0
    traffic = pmc_traffic(dom)
    roofline = {
        "bound": "hbm",
        "kernel": {"ntt": "k_ntt (both passes, fwd+inv)", "conv": "k_conv",
                   "ks_inner": "k_ks_inner"}[dom],
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        "traffic": traffic,
        "avg_launch_us": k["ms"] / k["timed"] * 1e3 if k["timed"] else None,
        "algorithmic_bytes_per_launch": k["bytes"] / k["timed"] if k["timed"] else None,
        "launches_per_sort": k["launches"] / args.steps,
        "share_of_sort": est_ms(k) / 1e3 / dt,
        "timing": f"HIP events on the engine stream around every {period}th launch, timed region",
    }
    kernels = {f: {"launches_per_sort": kt[f]["launches"] / args.steps,
                   "ms_per_sort": est_ms(kt[f]) / args.steps,
                   "GBps": (kt[f]["bytes"] / (kt[f]["ms"] / 1e3) / 1e9) if kt[f]["ms"] else None}
               for f in families}

    sort_s = dt / args.steps
    sorts = 1 if shard else world  # concurrent sorts in the job
    value = sorts * N * N * args.steps / dt
    result = {
        "metric": "encrypted rank-sort homomorphic comparisons/s (N^2 per DirectSort<N>::sort)",
        "value": value,
        "unit": "cmp/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": sort_s * 1e3,
        "sort_seconds": sort_s,
        "higher_is_better": True,
        "scaling": "strong" if shard else "weak",
        "vs_baseline": None,
        "dtype": "u64 (RNS residues, 40/60-bit primes)",
        "data": "synthetic: seeded permutation of {k/N}, CKKS-encrypted",
        "config": {"workload": args.workload, "N": N, "ring_dim": 1 << logn, "mult_depth": depth,
                   "sign": list(cfg), "scale_bits": 40, "secure": secure,
                   "parallelism": f"limb-shard x{world} ({args.shard})" if shard else f"replicas x{world}"},
        "algorithmic_gb_per_sort": stats["algo_bytes"] / args.steps / 1e9,
        "roofline": roofline,
        "kernels": kernels,
        "trials": trials,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(N, logn, secure, depth, args.cpu_sample_seconds,
                                                  stats["algo_bytes"] / args.steps)
        except Exception as e:  # the oracle is optional on a box without its build
            result["cpu_baseline"] = {"value": None, "error": str(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
