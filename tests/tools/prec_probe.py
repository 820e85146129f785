"""Developer probe (not collected by pytest): rank / sort error of DirectSort<N>
against slotsim and the exact sort, on the chosen backend.
  python tests/tools/prec_probe.py N logn [secure] [scale_bits] [backend]"""
import os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "sorting-fhe_amd", "python"))
import sfhe
from oracle import slotsim

N = int(sys.argv[1]); logn = int(sys.argv[2])
secure = len(sys.argv) > 3 and sys.argv[3] == "1"
sb = int(sys.argv[4]) if len(sys.argv) > 4 else 40
be = sys.argv[5] if len(sys.argv) > 5 else "hip"
t0 = time.time()
depth, rots = sfhe.direct_sort_params(N, be)
e = sfhe.Engine(be, mult_depth=depth, ring_dim=1 << logn, batch_size=N, rotations=rots,
                seed=20251205 + N, scaling_mod_size=sb, secure=secure)
e.set_quiet(True)
x = slotsim.input_vector(N)
cfg = slotsim.default_sign_config(N)
s = e.sorter(N)
ct = e.encrypt(x.tolist())
print(f"N={N} logn={logn} secure={secure} scale={sb} depth={depth} setup {time.time()-t0:.1f}s "
      f"primes={len(e.primes())}", flush=True)
t = time.time()
r = s.rank(ct, *cfg)
rank = np.array(e.decrypt(r))
true = np.argsort(np.argsort(x)).astype(float)
sim = slotsim.construct_rank(x, N, 1 << logn, cfg)
er = np.max(np.abs(rank - true))
print(f"  rank {time.time()-t:.2f}s err vs argsort {er:.3g} (log2 {np.log2(er):.2f}) vs slotsim "
      f"{np.max(np.abs(rank-sim)):.3g} level {r.level}", flush=True)
t = time.time()
out = s.place(r, ct)
got = np.array(e.decrypt(out))
es = np.max(np.abs(got - np.sort(x)))
print(f"  place {time.time()-t:.2f}s sort err {es:.3g} (log2 {np.log2(es):.2f}) level {out.level} "
      f"depth {depth}", flush=True)
for i in range(3):
    t = time.time(); o = s.sort(ct, *cfg); e.sync()
    print(f"  sort trial {i}: {1e3*(time.time()-t):.1f} ms", flush=True)
got = np.array(e.decrypt(o)); es = np.max(np.abs(got - np.sort(x)))
print(f"  sort() err {es:.3g} (log2 {np.log2(es):.2f}) pool {e.pool_bytes()/2**30:.1f} GiB", flush=True)
