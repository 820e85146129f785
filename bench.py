#!/usr/bin/env python3
"""Benchmark: encrypted rank sort (DirectSort<N>::sort) on MI355X.

Contract (see task README): ``python bench.py --gpus N --steps K --warmup W``
prints ONE JSON line on rank 0.  A step is one ``DirectSort<N>::sort`` of one
encrypted array (reference src/sort_algo.h:752-774, timed like
tests/DirectSortTest.cpp:129-136) at the metric configuration of
BASELINE.json: N=256, ring 2^16, depth 34, CompositeSign(3,4,2), scale 40.

Multi-GPU (one process per GPU; BASELINE north_star: "encrypted-sort
wall-clock ... at 1, 2, 4 and 8 MI355X"): at N > 1 the headline is the
wall-clock of ONE metric sort over all ranks -> scaling "strong", value =
N^2 * K / max-over-ranks(time).  The ranks form G = 2 batch groups (``--split``;
the sort's two independent batches per phase, one per group, parts
all-gathered over RCCL) of N/G ranks, and each group limb-shards its batch
(in-group rank r holds the RNS limbs i % (N/G) == r above the
replicated tail; RCCL all-gather at ModUp / ModDown, broadcast at rescale).
The whole sort is one hipGraph with its collectives.  ``--split 1``: limb
sharding over all N ranks.  The ranks' independent replica sorts (each GPU its own
array, no data-path collective) are measured first and reported as the
extra field ``replicas``; should the sharded leg fail or stall, the line
carries the replica throughput as the headline and says so.
``--replicas`` makes the replicas the headline (weak scaling);
``--shard host`` runs the sharded sort over the gloo host transport (a
rehearsal on one GPU: SFHE_BENCH_DEVICE=0 puts every rank on it).

Extra fields: ``roofline`` (dominant kernel family: HIP events around each of
its launches during one profiling sort after the timed region, lanes
serialised as under rocprofv3), ``cpu_baseline`` (one real DirectSort<N> on
the C oracle, rank 0 only, N=1 only) and ``trials`` (pure / as-test / cold).
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


PUBLISHED_CPU = ("reference OpenFHE CPU, sort_hybrid1 N=256 @ ring 2^17 (sibling placement, same "
                 "constructRank): 93.53 s average, comparison/experimental_results/ours_hybrid1/"
                 "total_results.txt:151-174")


def cpu_baseline(N, logn, secure, depth, rots, cfg):
    """One real DirectSort<N>::sort on the C oracle (test infrastructure;
    never the measured path): the same parameters, input and op trace as the
    GPU steps, on every host thread the box gives the process (OpenMP), cold
    (a fresh sorter: host mask generation and encoding inside the timed sort,
    as in the reference's DirectSortTest).  Key generation is not timed."""
    import numpy as np
    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
    t0 = time.perf_counter()
    eng = sfhe.Engine("oracle", mult_depth=depth, ring_dim=1 << logn, batch_size=N, secure=secure,
                      rotations=rots, seed=20251205 + N)
    eng.set_quiet(True)
    setup_s = time.perf_counter() - t0
    x = input_vector(N)
    ct = eng.encrypt(x.tolist())
    sorter = eng.sorter(N)
    t0 = time.perf_counter()
    out = sorter.sort(ct, *cfg)
    sort_s = time.perf_counter() - t0
    err = float(np.max(np.abs(np.array(eng.decrypt(out)) - np.sort(x))))
    return {
        "value": N * N / sort_s,
        "unit": "cmp/s",
        "cores": cores,
        "kind": "port",
        "sample": (f"one full DirectSort<{N}>::sort (ring 2^{logn}, depth {depth}) on the C oracle "
                   f"(u128-% RNS primitives, OpenMP {cores} threads), cold: {sort_s:.1f} s/sort "
                   f"(key generation {setup_s:.1f} s, untimed); max err {err:.2g}"),
        "sort_seconds": sort_s,
        "published_reference": PUBLISHED_CPU,
    }


PUBLISHED_HYBRID1_S = 93.5315  # comparison/experimental_results/ours_hybrid1/total_results.txt:151-174


def hybrid1_leg(device, N=256, logn=17, trials=3):
    """DirectSort<256>::sort_hybrid1 at DirectSortH1Test's configuration (ring
    2^17, HEStd_128_classic, depth 49, its rotation keys): the only path the
    reference publishes timings for (93.53 s average on its CPU machine)."""
    import numpy as np
    depth, rots = sfhe.hybrid1_params(N)
    eng = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, secure=True,
                      rotations=rots, seed=20251205 + N, device=device)
    eng.set_quiet(True)
    x = input_vector(N)
    ct = eng.encrypt(x.tolist())
    s = eng.sorter(N, rotations=rots)
    ts = []
    for _ in range(trials + 1):
        eng.sync()
        t0 = time.perf_counter()
        out = s.sort_hybrid1(ct, *sign_config(N))
        eng.sync()
        ts.append((time.perf_counter() - t0) * 1e3)
    err = float(np.max(np.abs(np.array(eng.decrypt(out))[:N] - np.sort(x))))
    import statistics
    med = statistics.median(ts[1:])
    return {"workload": f"sort_hybrid1 N={N} @ ring 2^{logn} (DirectSortH1Test config, depth {depth})",
            "ms_median": med, "ms_cold": ts[0], "trials": trials, "level": out.level, "max_err": err,
            "published_reference_s": PUBLISHED_HYBRID1_S,
            "speedup_vs_published": PUBLISHED_HYBRID1_S * 1e3 / med}


def kway_leg(device, k=2, M=10, logn=17):
    """BASELINE config 4: the k-way network KWayAdapter<1024>::sort (k = 2,
    M = 10: 55 stages) at ring 2^17, HEStd_128_classic, depth 40, scale 59,
    bootstrapping {5,5} over 1024 sparse slots, CompositeSign(3, d_f = 2,
    d_g = 5) as tests/k-way/KWaySort2Test.cpp:124-157 passes it.  Two sorts on
    one persistent adapter: cold (encodes the masks and bootstrapping
    diagonals) and warm; `ms` is the warm one.  The reference publishes no
    k-way timing."""
    import numpy as np
    N = k ** M
    batch, depth, budget, rots = sfhe.kway_params(N)
    eng = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=batch, scaling_mod_size=59,
                      secure=True, rotations=rots, seed=7 + N, device=device)
    eng.set_quiet(True)
    t0 = time.perf_counter()
    eng.bootstrap_setup(budget, batch)
    setup_s = time.perf_counter() - t0
    x = np.random.default_rng(N).permutation(N) / N
    ct = eng.encrypt(x.tolist())
    sorter = eng.kway(k, M)
    ms = []
    for _ in range(3):  # cold (encodes masks / diagonals), captured into a hipGraph, replayed
        eng.sync()
        t0 = time.perf_counter()
        out = sorter.sort(ct, 3, 2, 5, depth)  # (3, d_f, d_g) as the test passes it
        eng.sync()
        ms.append((time.perf_counter() - t0) * 1e3)
    err = float(np.max(np.abs(np.array(eng.decrypt(out))[:N] - np.sort(x))))
    # where the warm sort's kernel time goes, each family's
    # nodes of the captured chain replayed alone (HIP events on the engine
    # stream), and the dominant family's algorithmic rate against HBM peak
    fams = {}
    for f in ("ntt", "conv", "ntt_ks", "ks_inner", "other"):
        try:
            f_ms, f_n, f_b = sorter.graph_family_time(f, reps=1)
        except sfhe.SfheError:
            continue
        fams[f] = {"ms_per_sort": f_ms, "launches_per_sort": f_n, "algorithmic_gb_per_sort": f_b / 1e9 or None,
                   "avg_launch_us": f_ms / f_n * 1e3 if f_n else None,
                   "frac": (f_b / (f_ms / 1e3) / (HBM_PEAK_GBS * 1e9)) if (f_b and f_ms) else None}
    dom = max((f for f in fams if fams[f]["algorithmic_gb_per_sort"]), key=lambda f: fams[f]["ms_per_sort"],
              default=None)
    roof = None
    if dom:
        d = fams[dom]
        roof = {"bound": "hbm", "family": dom, "achieved": d["algorithmic_gb_per_sort"] / (d["ms_per_sort"] / 1e3),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": d["frac"], "avg_launch_us": d["avg_launch_us"],
                "algorithmic_bytes_per_launch": d["algorithmic_gb_per_sort"] * 1e9 / d["launches_per_sort"],
                "launches_per_sort": d["launches_per_sort"],
                "timing": "the family's kernel nodes of the k-way sort's captured chain of graphs, re-instantiated "
                          "alone in captured order and replayed once each, HIP events on the engine stream"}
    return {"workload": f"k-way sort N={N} (k={k}, M={M}) @ ring 2^{logn}, depth {depth}, bootstrapping {budget}",
            "roofline": roof, "families": fams,
            "ms": ms[-1], "ms_cold": ms[0], "ms_capture": ms[1], "graph_nodes": sorter.graph_nodes(),
            "note": "ms: the replay of the whole sort's hipGraph (stages + bootstraps); ms_capture: the "
                    "second sort, which captures it",
            "bootstrap_keygen_s": setup_s, "level": out.level, "max_err": err,
            "stages": M + M * (M - 1) // 2 * ((k + 1) // 2)}


def c5_leg(device, world=1, rank=0, steps=2, groups=1):
    """BASELINE config 5's sort: DirectSort<256> at ring 2^17 (DirectSortTest's
    ring, HEStd_128_classic, ~40 limbs).  world == 1: one GPU, unsharded (the
    reference point).  world > 1: the ranks split one sort's batches over
    `groups` groups and limb-shard each group's share over RCCL (SURVEY
    §8(e)): per-sort wall-clock at W GPUs.  Run after the replica
    measurement, as an extra field; a watchdog (SFHE_C5_TIMEOUT s, default
    240) prints the line without it and exits with status 2 if the collective
    path stalls."""
    import numpy as np
    N, logn, secure = WORKLOADS["directsort_n256_2e17"]
    depth, rots = sfhe.direct_sort_params(N, "hip")
    shard = grp = None
    transport = os.environ.get("SFHE_C5_TRANSPORT", "rccl")  # "host": gloo rehearsal (ranks may share a GPU)
    if world > 1:
        shard, grp = comm_spec(transport, rank, world, groups)
    t0 = time.perf_counter()
    eng = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, secure=secure,
                      rotations=rots, seed=20251205 + N, device=device, shard=shard, groups=grp)
    eng.set_quiet(True)
    setup_s = time.perf_counter() - t0
    x = input_vector(N)
    ct = eng.encrypt(x.tolist())
    sorter = eng.sorter(N)
    cfg = sign_config(N)
    holder = {}

    def step():
        holder["out"] = sorter.sort(ct, *cfg)

    dt = timed_steps(step, eng.sync, world, steps, 1)
    err = float(np.max(np.abs(np.array(eng.decrypt(holder["out"]))[:N] - np.sort(x))))
    return {"workload": f"DirectSort<{N}> @ ring 2^{logn} (HEStd_128_classic, depth {depth})",
            "parallelism": parallelism(world, groups, transport, eng.shard_tail()) if world > 1
            else "1 GPU, unsharded",
            "ms_per_sort": dt / steps * 1e3, "setup_s": setup_s, "max_err": err, "level": holder["out"].level}


def pmc_traffic(family: str):
    """HBM traffic / algorithmic bytes for `family` from the committed PMC
    summary (tools/pmc_traffic.py over tools/profile_round.sh's two PMC passes
    on the kernel microbenchmark), if it was taken on the current kernels."""
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
    return j.get("families", {}).get(family, {}).get("traffic_over_algorithmic")


def comm_spec(mode: str, rank: int, world: int, groups: int):
    """Engine(shard=..., groups=...) arguments of the multi-GPU sort: `groups`
    batch groups of world // groups ranks (rank = group * per + r), each group
    limb-sharded over its own communicator when per > 1, and a group
    communicator per in-group rank r joining the groups (sfhe_groups_*).
    RCCL: each communicator's unique id made by one of its members and shared
    with all_gather_object; host: gloo subgroups.  Collective over all ranks."""
    import torch.distributed as dist
    per = world // groups
    g, r = divmod(rank, per)
    if mode == "host":
        limb = [dist.new_group(list(range(h * per, (h + 1) * per))) for h in range(groups)]
        cross = [dist.new_group([h * per + j for h in range(groups)]) for j in range(per)]
        shard = ("host", r, per, sfhe.GlooComm(limb[g])) if per > 1 else None
        grp = ("host", g, groups, sfhe.GlooComm(cross[r])) if groups > 1 else None
        return shard, grp
    mine = {}
    if per > 1 and r == 0:
        mine[f"limb{g}"] = sfhe.comm_uid("hip")
    if groups > 1 and g == 0:
        mine[f"cross{r}"] = sfhe.comm_uid("hip")
    every = [None] * world
    dist.all_gather_object(every, mine)
    uids = {}
    for m in every:
        uids.update(m)
    shard = ("rccl", r, per, uids[f"limb{g}"]) if per > 1 else None
    grp = ("rccl", g, groups, uids[f"cross{r}"]) if groups > 1 else None
    return shard, grp


def parallelism(world: int, groups: int, mode: str, tail: int) -> str:
    per = world // groups
    parts = []
    if groups > 1:
        parts.append(f"batch-split x{groups}")
    if per > 1:
        parts.append(f"limb-shard x{per} (replicated tail <= {tail} limbs)")
    return " * ".join(parts) + f" over {mode}"


def replica_leg(make_engine, spec, world, steps, warmup):
    """Every rank sorts its own array on its own GPU (no data-path
    collective): the job's throughput, world * N^2 per sort time.  Measured
    with the same barrier / max-over-ranks timing as the headline."""
    N, cfg = spec["N"], spec["cfg"]
    eng = make_engine()
    eng.set_quiet(True)
    sorter = eng.sorter(N)
    ct = eng.encrypt(input_vector(N).tolist())
    holder = {}

    def step():
        holder["out"] = sorter.sort(ct, *cfg)

    dt = timed_steps(step, eng.sync, world, steps, warmup)
    nodes = sorter.graph_nodes()
    holder.clear()
    del sorter, ct
    eng.close()
    return {"value": world * N * N * steps / dt, "unit": "cmp/s", "ms_per_step": dt / steps * 1e3,
            "scaling": "weak", "parallelism": f"replicas x{world}", "graph_nodes": nodes,
            "note": "each rank sorts its own array (independent replicas, no data-path collective)"}


def fallback_line(replicas, spec, world, args, why):
    """The metric line when the sharded headline could not be measured: the
    replica throughput, labelled as such."""
    N = spec["N"]
    return {"metric": "encrypted rank-sort homomorphic comparisons/s (N^2 per DirectSort<N>::sort)",
            "value": replicas["value"], "unit": "cmp/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": replicas["ms_per_step"],
            "sort_seconds": replicas["ms_per_step"] / 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u64 (RNS residues, 40/60-bit primes)",
            "data": "synthetic: seeded permutation of {k/N}, CKKS-encrypted",
            "config": {"workload": args.workload, "N": N, "ring_dim": 1 << spec["logn"],
                       "mult_depth": spec["depth"], "sign": list(spec["cfg"]), "scale_bits": 40,
                       "secure": spec["secure"], "parallelism": f"replicas x{world}"},
            "replicas": replicas, "sharded_error": why}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="directsort_n256_2e16", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--trials", type=int, default=10,
                    help="per-sort trials after the timed region (median/min/max, pure and as-test)")
    ap.add_argument("--no-kway", dest="kway", action="store_false",
                    help="skip the k-way leg (BASELINE config 4: N=1024 @ 2^17, one ~14 s sort)")
    ap.add_argument("--no-hybrid1", dest="hybrid1", action="store_false",
                    help="skip the sort_hybrid1 leg (N=256 @ 2^17, the published-timing path)")
    ap.add_argument("--no-c5", dest="c5", action="store_false",
                    help="skip the config-5 leg (N=256 @ 2^17: unsharded at N=1, limb-sharded over RCCL at N>1)")
    ap.add_argument("--c5-eager", action="store_true",
                    help="run the config-5 leg without graph replay (profiling: replaying the 2^17 sort's graph "
                         "under rocprofv3's kernel tracer crashes inside the profiler, DESIGN.md §5)")
    ap.add_argument("--shard", choices=("rccl", "host"), default=None,
                    help="transport of the multi-GPU headline sort at N > 1 (default rccl)")
    ap.add_argument("--split", type=int, default=None,
                    help="batch groups of the multi-GPU sort (default 2 when N is even and the sort has an "
                         "even batch count, else 1; 1 = limb sharding over all ranks)")
    ap.add_argument("--replicas", action="store_true",
                    help="at N > 1, make the independent replica sorts the headline (weak scaling)")
    args = ap.parse_args(argv)

    world, rank, local = dist_init()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    N, logn, secure = WORKLOADS[args.workload]
    depth, rots = sfhe.direct_sort_params(N, "hip")
    cfg = sign_config(N)

    device = int(os.environ.get("SFHE_BENCH_DEVICE", local))
    mode = None if (world == 1 or args.replicas) else (args.shard or "rccl")
    spec = dict(N=N, logn=logn, secure=secure, depth=depth, rots=rots, cfg=cfg)
    replicas = None
    if mode:  # the safe number first: every rank sorts its own array
        replicas = replica_leg(lambda: sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N,
                                                   secure=secure, rotations=rots, seed=20251205 + N + 7919 * rank,
                                                   device=device),
                               spec, world, args.steps, args.warmup)
    # DirectSort's batches per phase (RankLayout: P = min(N, n/2/N) partitions, B = N/P)
    batches = N // min(N, (1 << logn) // 2 // N)
    groups = args.split if args.split else (2 if world % 2 == 0 and batches % 2 == 0 else 1)
    if world % groups:
        raise SystemExit(f"--split {groups} does not divide --gpus {world}")
    shard = grp = None
    seed = 20251205 + N + 7919 * rank
    if mode:
        seed = 20251205 + N  # every rank builds the same keys
        shard, grp = comm_spec(mode, rank, world, groups)
    limit = float(os.environ.get("SFHE_SHARD_TIMEOUT", "600"))
    dog = None
    if mode:  # a stalled collective: report the replicas, then fail loudly
        import threading

        def stalled():
            if rank == 0:
                print(json.dumps(fallback_line(replicas, spec, world, args, f"sharded leg stalled after {limit:.0f} s")),
                      flush=True)
            sys.stderr.write(f"bench: sharded leg stalled after {limit:.0f} s\n")
            sys.stderr.flush()
            os._exit(2)
        dog = threading.Timer(limit, stalled)
        dog.daemon = True
        dog.start()
    try:
        eng = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, secure=secure,
                          rotations=rots, seed=seed, device=device, shard=shard, groups=grp)
    except Exception as e:  # noqa: BLE001 -- the sharded context could not be built
        if not mode:
            raise
        if rank == 0:
            print(json.dumps(fallback_line(replicas, spec, world, args, f"sharded context: {e}")), flush=True)
        sys.exit(3)
    eng.set_quiet(True)
    sorter = eng.sorter(N)
    x = input_vector(N)
    ct = eng.encrypt(x.tolist())  # input resident in HBM before timing

    families = ("ntt", "conv", "ks_inner", "ntt_ks")
    kernel_name = {"ntt": "k_ntt (both passes, fwd+inv)", "conv": "k_convf / k_mdrsf",
                   "ks_inner": "k_ks_inner", "ntt_ks": "k_ntt_ks (ModUp ROW pass + key inner product)"}

    def step():
        out = sorter.sort(ct, *cfg)
        del out

    # cold sort: a fresh sorter's first sort (host mask generation + encoding)
    eng.sync()
    t0 = time.perf_counter()
    step()
    eng.sync()
    cold_ms = (time.perf_counter() - t0) * 1e3

    dt = timed_steps(step, eng.sync, world, args.steps, args.warmup)
    tail = eng.shard_tail()

    # profiling leg (after the timed region): one EAGER sort (SFHE_GRAPH=0)
    # with the lanes serialised on one stream and every launch of each family
    # bracketed by HIP events on that stream -- per-launch durations as
    # rocprofv3 measures them (no other lane's kernels inside a timed
    # interval).  Batched ops merge here as in the captured sort (prims.h
    # sfp_batch_*), a merged launch timed as one launch with the bytes of all
    # of its ops; stacked lane regions (SFHE_STACK_BATCHES) are off in both.
    graph_nodes = sorter.graph_nodes()
    stk0 = eng.stack_stats()
    eng.sync()
    os.environ["SFHE_GRAPH"] = "0"  # per-launch timing needs the eager path
    eng.serialize_lanes(True)
    for fam in families:
        eng.kernel_timing(fam, 1)
    eng.op_stats(reset=True)
    if mode:
        eng.comm_stats_reset(timed=True)
    t0 = time.perf_counter()
    step()
    eng.sync()
    serial_ms = (time.perf_counter() - t0) * 1e3
    stats = eng.op_stats()  # the SURVEY §8(d) byte model over one (eager) sort
    collectives = None
    if mode:  # each rank's exchange share of a sort, so the 1 -> 8 curve decomposes
        mine = dict(eng.comm_stats(), rank=rank, serial_sort_ms=serial_ms)
        import torch.distributed as dist
        every = [None] * world
        dist.all_gather_object(every, mine)
        collectives = {
            "per_rank": every,
            "source": "the profiling sort after the timed region (eager, lanes serialised on one stream)",
            "note": "calls = all-gathers / broadcasts this rank issued in one sort (ModUp / ModDown "
                    "all-gathers and rescale broadcasts at dealt levels, one batch-group all-gather per "
                    "phase); bytes = what it received; ms = their summed duration (HIP events on the "
                    "engine stream around each RCCL call); serial_sort_ms - ms = that sort's compute. "
                    "The timed graph issues the same collectives"}
    stk1 = eng.stack_stats()
    kt = {fam: eng.kernel_timing_read(fam) for fam in families}
    for fam in families:
        eng.kernel_timing(fam, 0)
    eng.serialize_lanes(False)
    os.environ.pop("SFHE_GRAPH", None)

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
        # the as-test sorter is a fresh sorter: its first sort runs eagerly and
        # its second captures the rank / placement graphs (the
        # 96 ms as-test "outlier" was that capture inside the trials); both
        # are reported apart, then the trials replay like the pure ones
        dbg = eng.sorter(N, debug=True)
        as_test_first = trial_ms(dbg, 2)
        as_test = trial_ms(dbg, args.trials)
        trials = {"count": args.trials, "pure_ms": stats3(pure), "as_test_ms": stats3(as_test),
                  "pure_each_ms": pure, "as_test_each_ms": as_test,
                  "as_test_first_two_ms": as_test_first,
                  "cold_ms": cold_ms,
                  "note": "each trial one sort with a device sync on both sides (rank-local, after the "
                          "timed region); cold_ms = the first sort of a fresh sorter (mask generation + "
                          "encoding), before the warmup; as_test_first_two_ms = the debug sorter's eager "
                          "first sort and its graph-capturing second, before its trials"}

    ms_step = dt / args.steps * 1e3
    kernels = {}
    for f in families:
        k = kt[f]
        kernels[f] = {"kernel": kernel_name[f], "launches_per_sort": k["launches"],
                      "ms_per_sort": k["ms"], "avg_launch_us": k["ms"] / k["timed"] * 1e3 if k["timed"] else None,
                      "algorithmic_bytes_per_launch": k["bytes"] / k["timed"] if k["timed"] else None,
                      "GBps": k["bytes"] / (k["ms"] / 1e3) / 1e9 if k["ms"] else None}
        # a family's kernel time cannot exceed the sort it is part of
        assert k["ms"] <= max(ms_step, serial_ms) * 1.02, (f, k["ms"], ms_step, serial_ms)
    dom = max(families, key=lambda f: kt[f]["ms"])
    assert dom == "ntt", dom  # the roofline kernel
    # The dominant family's kernels exactly as the timed region ran them: the
    # NTT nodes of the sort's captured graph, replayed alone back to back and
    # timed with HIP events on the engine's stream (no other lane's kernels
    # inside the interval, no per-launch event overhead) -- what rocprofv3
    # reports as their durations.  Eager runs (SFHE_GRAPH=0) fall back to the
    # per-launch events of the serialised profiling sort.
    try:
        if os.environ.get("SFHE_NO_GRAPH_REPLAY"):  # (set by tools/profile_round.sh under rocprofv3)
            raise sfhe.SfheError("graph replay disabled")
        r_ms, r_launch, r_bytes = sorter.graph_ntt_time(reps=5)
        timing = ("the NTT kernel nodes of the timed region's captured sort graph, re-instantiated alone "
                  "in captured order and replayed 5x, timed with HIP events on the engine stream; "
                  "achieved = algorithmic bytes (16 B per coefficient per pass) / replay time")
    except sfhe.SfheError:
        r_ms, r_launch, r_bytes = kt[dom]["ms"], kt[dom]["timed"], kt[dom]["bytes"]
        timing = ("HIP events around every launch of the family on the stream it runs on, during one "
                  f"profiling sort after the timed region with the lanes serialised ({serial_ms:.1f} ms)")
    achieved = r_bytes / (r_ms / 1e3) / 1e9 if r_ms else 0.0
    # every family of the captured sort replayed alone the same way: where the
    # sort's kernel time goes ("all" = every kernel node back to back, i.e.
    # without the two lanes' overlap; the timed sort is shorter by that overlap)
    graph_breakdown = None
    if not os.environ.get("SFHE_NO_GRAPH_REPLAY"):
        try:
            graph_breakdown = {}
            for f in ("ntt", "conv", "ntt_ks", "ks_inner", "other", "all"):
                f_ms, f_n, f_b = sorter.graph_family_time(f, reps=3)
                graph_breakdown[f] = {"ms_per_sort": f_ms, "launches_per_sort": f_n}
                if f_b:  # NTT, conversion and k_ntt_ks families: algorithmic bytes -> rate and frac
                    graph_breakdown[f].update(algorithmic_gb_per_sort=f_b / 1e9,
                                              frac=f_b / (f_ms / 1e3) / (HBM_PEAK_GBS * 1e9))
        except sfhe.SfheError:
            graph_breakdown = None
    ratio = pmc_traffic(dom)
    roofline = {
        "bound": "hbm",
        "kernel": kernel_name[dom],
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        # HBM bytes per launch: the PMC ratio (FETCH_SIZE x2 + WRITE_SIZE, KiB -> B, over the
        # same kernels on tools/microbench at 1..96 limbs) x this sort's algorithmic bytes per launch
        "traffic": ratio * r_bytes / r_launch if (ratio and r_launch) else None,
        "traffic_over_algorithmic": ratio,
        "avg_launch_us": r_ms / r_launch * 1e3 if r_launch else None,
        "algorithmic_bytes_per_launch": r_bytes / r_launch if r_launch else None,
        "launches_per_sort": r_launch,
        "ms_per_sort": r_ms,
        "timing": timing,
    }

    sort_s = dt / args.steps
    sorts = 1 if mode else world  # concurrent sorts in the job
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
        "scaling": "strong" if mode else "weak",
        "vs_baseline": None,
        "dtype": "u64 (RNS residues, 40/60-bit primes)",
        "data": "synthetic: seeded permutation of {k/N}, CKKS-encrypted",
        "config": {"workload": args.workload, "N": N, "ring_dim": 1 << logn, "mult_depth": depth,
                   "sign": list(cfg), "scale_bits": 40, "secure": secure,
                   "parallelism": (parallelism(world, groups, mode, tail) if mode
                                   else f"replicas x{world}")},
        "algorithmic_gb_per_sort": stats["algo_bytes"] / 1e9,
        "graph": {"replayed": graph_nodes > 0, "nodes": graph_nodes,
                  "note": "timed steps replay the sort as one hipGraph (captured during warmup; "
                          "SFHE_GRAPH=0 runs them eagerly)"},
        # the sort's algorithmic bytes over the timed sort's wall time, against HBM peak
        "whole_sort_frac": stats["algo_bytes"] / sort_s / (HBM_PEAK_GBS * 1e9),
        "batched_ops": {"merged_launches_per_sort": stk1[0] - stk0[0],
                        "alone_launches_per_sort": stk1[1] - stk0[1],
                        "source": "the serialised eager profiling sort after the timed region",
                        "note": "launches of batched ops (prims.h sfp_batch_*: independent ops of one lane, "
                                "e.g. one Chebyshev PS level's products) issued as ONE merged launch of 2-8 "
                                "ops, and those issued alone; the captured sort records the same merged "
                                "launches.  Stacked lane regions (SFHE_STACK_BATCHES=1) are off"},
        "roofline": roofline,
        "kernels": kernels,
        "kernels_source": ("the serialised eager profiling sort after the timed region (SFHE_GRAPH=0, lanes on "
                           f"one stream, {serial_ms:.1f} ms): HIP events around every launch of each family; "
                           "batched ops merged as in the timed graph, a merged launch counted as one.  The "
                           "timed graph's own kernels: roofline (NTT) and graph_breakdown (every family)"),
        "graph_breakdown": graph_breakdown,
        "trials": trials,
        "cpu_baseline": None,
    }
    if collectives:
        result["collectives"] = collectives
    if replicas:
        result["replicas"] = replicas
    if dog:
        dog.cancel()
    def leg(name):  # progress on stderr (a crash inside a leg names it)
        sys.stderr.write(f"bench: {name}\n")
        sys.stderr.flush()

    leg(f"timed region done: {dt / args.steps * 1e3:.2f} ms per sort")
    if args.c5 and (world == 1 or mode == "rccl"):
        import threading

        def c5_stalled():  # the collective path hung: report what was measured, then fail loudly
            if rank == 0:
                result["c5"] = {"error": f"timeout after {c5_limit:.0f} s (collective stalled)"}
                print(json.dumps(result), flush=True)
            sys.stderr.write(f"bench: c5 leg stalled after {c5_limit:.0f} s\n")
            sys.stderr.flush()
            os._exit(2)
        c5_limit = float(os.environ.get("SFHE_C5_TIMEOUT", "240"))
        c5_dog = threading.Timer(c5_limit, c5_stalled)
        c5_dog.daemon = True
        c5_dog.start()
        if args.c5_eager:
            os.environ["SFHE_GRAPH"] = "0"  # read per sort by the sorter
        leg("c5 leg")
        try:
            # config 5's sort has one batch per phase at 2^17: nothing to split,
            # so its ranks limb-shard over all N
            result["c5"] = c5_leg(device, world, rank, groups=1)
        except Exception as e:  # noqa: BLE001 -- an extra leg must not lose the metric line
            result["c5"] = {"error": str(e)}
        c5_dog.cancel()
    if rank == 0 and world == 1 and args.hybrid1:
        leg("hybrid1 leg")
        try:
            result["hybrid1"] = hybrid1_leg(device)
        except Exception as e:  # noqa: BLE001 -- an extra leg must not lose the metric line
            result["hybrid1"] = {"error": str(e)}
    if rank == 0 and world == 1 and args.kway:
        leg("kway leg")
        try:
            result["kway"] = kway_leg(device)
        except Exception as e:  # noqa: BLE001
            result["kway"] = {"error": str(e)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        leg("cpu baseline")
        try:
            result["cpu_baseline"] = cpu_baseline(N, logn, secure, depth, rots, cfg)
        except Exception as e:  # the oracle is optional on a box without its build
            result["cpu_baseline"] = {"value": None, "error": str(e)}
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
