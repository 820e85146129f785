"""Precision table (developer tool, GPU): max |decrypted - exact| of every sort
at the configurations the GPU tests gate, with the engine's precision
choices on (default) or off (SFHE_LAZY=0 SFHE_SELF_OFFSET=0 SFHE_SINC_REBASE=0,
the reference's order of operations), next to the noise-free slot simulation
(oracle/slotsim.py: the approximation floor).  DESIGN.md §2 quotes its output.

    python tools/precision_table.py [--quick] > gpurun_out/precision.txt
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sorting-fhe_amd", "python"))
import sfhe  # noqa: E402
from oracle import slotsim  # noqa: E402

DIRECT = [(8, 17, True), (128, 16, False), (256, 16, False), (256, 17, True), (512, 17, True), (1024, 17, True)]
HYBRID = [("hybrid1", 64), ("hybrid1", 256), ("hybrid", 64), ("hybrid", 256), ("hybrid2", 64), ("hybrid2", 128),
          ("hybrid2", 256)]


def direct(N, logn, secure):
    depth, rots = sfhe.direct_sort_params(N, "hip")
    e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, secure=secure, rotations=rots,
                    seed=20251205 + N)
    e.set_quiet(True)
    x = slotsim.input_vector(N)
    s = e.sorter(N)
    ct = e.encrypt(x.tolist())
    cfg = slotsim.default_sign_config(N)
    r = s.rank(ct, *cfg)
    rank = np.array(e.decrypt(r))
    out = s.place(r, ct)
    got = np.array(e.decrypt(out))
    sim, srank = slotsim.direct_sort(x, N, 1 << logn)
    return dict(rank=np.max(np.abs(rank - np.argsort(np.argsort(x)))), sort=np.max(np.abs(got - np.sort(x))),
                floor=np.max(np.abs(sim - np.sort(x))), level=out.level, depth=depth)


def hybrid(kind, N, logn=17):
    if kind == "hybrid1":
        depth, rots = sfhe.hybrid1_params(N, "hip")
    else:
        depth, rots = sfhe.hybrid_params(N, 2 if kind == "hybrid2" else 0, "hip")
    e = sfhe.Engine("hip", mult_depth=depth, ring_dim=1 << logn, batch_size=N, secure=True, rotations=rots,
                    seed=20251205 + N)
    e.set_quiet(True)
    x = slotsim.input_vector(N)
    s = e.sorter(N, rotations=rots)
    ct = e.encrypt(x.tolist())
    cfg = slotsim.default_sign_config(N)
    if kind == "hybrid1":
        out = s.sort_hybrid1(ct, *cfg)
        sim, _ = slotsim.sort_hybrid1(x, N, 1 << logn)
        floor = np.max(np.abs(sim - np.sort(x)))
    else:
        out = s.sort_hybrid(ct, *cfg, variant=2 if kind == "hybrid2" else 0)
        floor = float("nan")
    got = np.array(e.decrypt(out))[:N]
    return dict(sort=np.max(np.abs(got - np.sort(x))), floor=floor, level=out.level, depth=depth)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="skip N >= 512")
    a = ap.parse_args()
    mode = "reference order" if os.environ.get("SFHE_LAZY") == "0" else "engine default"
    print(f"# precision table ({mode}): SFHE_LAZY={os.environ.get('SFHE_LAZY', '1')} "
          f"SFHE_SELF_OFFSET={os.environ.get('SFHE_SELF_OFFSET', '1')} "
          f"SFHE_SINC_REBASE={os.environ.get('SFHE_SINC_REBASE', '1')}", flush=True)
    for N, logn, secure in DIRECT:
        if a.quick and N >= 512:
            continue
        t = time.time()
        r = direct(N, logn, secure)
        print(f"DirectSort N={N:4d} 2^{logn} rank {r['rank']:.3e}  sort {r['sort']:.3e} (log2 {np.log2(r['sort']):6.2f})"
              f"  floor {r['floor']:.3e}  level {r['level']}/{r['depth']}  {time.time() - t:.1f}s", flush=True)
    for kind, N in HYBRID:
        t = time.time()
        r = hybrid(kind, N)
        print(f"{kind:8s} N={N:4d} 2^17 sort {r['sort']:.3e} (log2 {np.log2(r['sort']):6.2f})  floor {r['floor']:.3e}"
              f"  level {r['level']}/{r['depth']}  {time.time() - t:.1f}s", flush=True)


if __name__ == "__main__":
    main()
