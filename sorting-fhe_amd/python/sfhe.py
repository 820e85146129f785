"""ctypes binding of the C ABI in include/sfhe.h.

The product library is ``sorting-fhe_amd/build/libsfhe.so`` (HIP, gfx950).
``load("oracle")`` loads ``oracle/_build/libsfhe_oracle.so``, the CPU oracle
build -- test infrastructure only (tests/, __graft_entry__.smoke and the
bench's cpu_baseline leg); product code paths call ``load()`` and fail
loudly when the HIP library is missing.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
REPO_ROOT = os.path.dirname(PKG_ROOT)
PRODUCT_LIB = os.path.join(PKG_ROOT, "build", "libsfhe.so")
ORACLE_LIB = os.path.join(REPO_ROOT, "oracle", "_build", "libsfhe_oracle.so")

SFHE_OK = 0
HESTD_128_CLASSIC = 0
HESTD_NOTSET = 3

# every symbol include/sfhe.h declares (checked by tests/test_abi.py)
ABI_SYMBOLS = [
    "sfhe_abi_version", "sfhe_last_error", "sfhe_backend", "sfhe_params_default",
    "sfhe_context_create", "sfhe_context_destroy", "sfhe_keygen", "sfhe_rotate_keygen",
    "sfhe_context_info", "sfhe_context_primes", "sfhe_set_plaintext_cache", "sfhe_set_quiet",
    "sfhe_sync", "sfhe_op_stats", "sfhe_encrypt", "sfhe_decrypt", "sfhe_ct_free",
    "sfhe_ct_clone", "sfhe_ct_info", "sfhe_ct_set_slots", "sfhe_ct_download", "sfhe_eval_add",
    "sfhe_eval_sub", "sfhe_eval_add_const", "sfhe_eval_mult_const", "sfhe_eval_mult_plain",
    "sfhe_eval_mult", "sfhe_eval_rotate", "sfhe_eval_rotate_sum", "sfhe_eval_chebyshev", "sfhe_sign", "sfhe_compare",
    "sfhe_direct_sort_params", "sfhe_doubled_sinc_coeffs", "sfhe_sorter_create",
    "sfhe_sorter_destroy", "sfhe_sorter_sort", "sfhe_sorter_rank", "sfhe_sorter_place",
    "sfhe_decompose", "sfhe_kernel_timing", "sfhe_kernel_timing_read",
    "sfhe_comm_uid", "sfhe_shard_rccl", "sfhe_shard_host", "sfhe_pool_bytes", "sfhe_live_contexts",
    "sfhe_serialize_lanes", "sfhe_stack_stats", "sfhe_comm_stats_reset", "sfhe_comm_stats", "sfhe_sorter_graph_nodes", "sfhe_sorter_create_rot",
    "sfhe_sorter_sort_hybrid1", "sfhe_hybrid1_params", "sfhe_sorter_graph_ntt_time",
    "sfhe_sorter_graph_family_time",
    "sfhe_sorter_sort_hybrid", "sfhe_hybrid_params", "sfhe_sorter_place_2n",
    "sfhe_bootstrap_setup", "sfhe_bootstrap_depth", "sfhe_bootstrap",
    "sfhe_sorter_sort_bitonic", "sfhe_kway_sort", "sfhe_kway_params",
    "sfhe_save", "sfhe_load", "sfhe_ct_save", "sfhe_ct_load",
    "sfhe_kway_create", "sfhe_kway_run", "sfhe_kway_destroy", "sfhe_kway_graph_nodes", "sfhe_kway_graph_family_time", "sfhe_shard_tail",
    "sfhe_key_rows",
    "sfhe_groups_rccl", "sfhe_groups_host", "sfhe_groups",
    "sfhe_encode_counts", "sfhe_bootstrap_graphs",
]


class SfheError(RuntimeError):
    pass


class Params(C.Structure):
    _fields_ = [
        ("mult_depth", C.c_uint32),
        ("scaling_mod_size", C.c_uint32),
        ("first_mod_size", C.c_uint32),
        ("batch_size", C.c_uint32),
        ("ring_dim", C.c_uint32),
        ("security_level", C.c_int32),
        ("num_large_digits", C.c_uint32),
        ("device", C.c_int32),
        ("seed", C.c_uint64),
        ("scaling_technique", C.c_int32),
    ]


_VP = C.c_void_p
_PVP = C.POINTER(C.c_void_p)
_U32 = C.c_uint32
_PU32 = C.POINTER(C.c_uint32)
_SZ = C.c_size_t
_PSZ = C.POINTER(C.c_size_t)
_PD = C.POINTER(C.c_double)
_PI32 = C.POINTER(C.c_int32)
_PU64 = C.POINTER(C.c_uint64)

# host collectives of sfhe_shard_host (sfhe_allgather_fn / sfhe_bcast_fn)
_AG = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t)
_BC = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.c_size_t, C.c_int)

_SIGS = {
    "sfhe_abi_version": (C.c_int, []),
    "sfhe_last_error": (C.c_char_p, []),
    "sfhe_backend": (C.c_char_p, []),
    "sfhe_params_default": (None, [C.POINTER(Params)]),
    "sfhe_context_create": (C.c_int, [C.POINTER(Params), _PVP]),
    "sfhe_context_destroy": (None, [_VP]),
    "sfhe_keygen": (C.c_int, [_VP]),
    "sfhe_rotate_keygen": (C.c_int, [_VP, _PI32, _SZ]),
    "sfhe_context_info": (C.c_int, [_VP, _PU32, _PU32, _PU32, _PU32, _PU32]),
    "sfhe_context_primes": (C.c_int, [_VP, _PU64, _SZ, _PSZ]),
    "sfhe_set_plaintext_cache": (C.c_int, [_VP, C.c_int]),
    "sfhe_set_quiet": (C.c_int, [_VP, C.c_int]),
    "sfhe_sync": (C.c_int, [_VP]),
    "sfhe_op_stats": (C.c_int, [_VP, _PU64, _PD, C.c_int]),
    "sfhe_encrypt": (C.c_int, [_VP, _PD, _SZ, _U32, _U32, _PVP]),
    "sfhe_decrypt": (C.c_int, [_VP, _VP, _PD, _SZ, _PSZ]),
    "sfhe_ct_free": (None, [_VP]),
    "sfhe_ct_clone": (C.c_int, [_VP, _PVP]),
    "sfhe_ct_info": (C.c_int, [_VP, _PU32, _PU32, _PU32]),
    "sfhe_ct_set_slots": (C.c_int, [_VP, _U32]),
    "sfhe_ct_download": (C.c_int, [_VP, _VP, _PU64, _SZ]),
    "sfhe_eval_add": (C.c_int, [_VP, _VP, _VP, _PVP]),
    "sfhe_eval_sub": (C.c_int, [_VP, _VP, _VP, _PVP]),
    "sfhe_eval_add_const": (C.c_int, [_VP, _VP, C.c_double, _PVP]),
    "sfhe_eval_mult_const": (C.c_int, [_VP, _VP, C.c_double, _PVP]),
    "sfhe_eval_mult_plain": (C.c_int, [_VP, _VP, _PD, _SZ, _U32, _PVP]),
    "sfhe_eval_mult": (C.c_int, [_VP, _VP, _VP, _PVP]),
    "sfhe_eval_rotate": (C.c_int, [_VP, _VP, C.c_int32, _PVP]),
    "sfhe_eval_rotate_sum": (C.c_int, [_VP, C.POINTER(_VP), C.POINTER(C.c_int32), C.c_size_t, _PVP]),
    "sfhe_bootstrap_setup": (C.c_int, [_VP, _U32, _U32, _U32]),
    "sfhe_bootstrap_depth": (C.c_int, [_VP, _U32, _U32, _U32, _PU32]),
    "sfhe_bootstrap": (C.c_int, [_VP, _VP, _U32, _U32, _PVP]),
    "sfhe_eval_chebyshev": (C.c_int, [_VP, _VP, _PD, _SZ, C.c_double, C.c_double, _PVP]),
    "sfhe_sign": (C.c_int, [_VP, _VP, C.c_int, C.c_int, C.c_int, _PVP]),
    "sfhe_compare": (C.c_int, [_VP, _VP, _VP, C.c_int, C.c_int, C.c_int, _PVP]),
    "sfhe_direct_sort_params": (C.c_int, [_U32, _PU32, _PI32, _SZ, _PSZ]),
    "sfhe_doubled_sinc_coeffs": (C.c_int, [_U32, _PD, _SZ, _PSZ]),
    "sfhe_sorter_create": (C.c_int, [_VP, _U32, C.c_int, _PVP]),
    "sfhe_sorter_destroy": (None, [_VP]),
    "sfhe_sorter_sort": (C.c_int, [_VP, _VP, C.c_int, C.c_int, C.c_int, _PVP]),
    "sfhe_sorter_rank": (C.c_int, [_VP, _VP, C.c_int, C.c_int, C.c_int, _PVP]),
    "sfhe_sorter_place": (C.c_int, [_VP, _VP, _VP, _PVP]),
    "sfhe_sorter_graph_nodes": (C.c_int, [_VP, _PU64]),
    "sfhe_sorter_create_rot": (C.c_int, [_VP, _U32, C.c_int, _PI32, _SZ, _PVP]),
    "sfhe_sorter_sort_hybrid1": (C.c_int, [_VP, _VP, C.c_int, C.c_int, C.c_int, _PVP]),
    "sfhe_hybrid1_params": (C.c_int, [_U32, _PU32, _PI32, _SZ, _PSZ]),
    "sfhe_sorter_sort_hybrid": (C.c_int, [_VP, _VP, C.c_int, C.c_int, C.c_int, C.c_int, _PVP]),
    "sfhe_hybrid_params": (C.c_int, [_U32, C.c_int, _PU32, _PI32, _SZ, _PSZ]),
    "sfhe_sorter_place_2n": (C.c_int, [_VP, _VP, _VP, _PVP]),
    "sfhe_sorter_sort_bitonic": (C.c_int, [_VP, _VP, C.c_int, C.c_int, C.c_int, _PVP]),
    "sfhe_save": (C.c_int, [_VP, C.c_char_p]),
    "sfhe_kway_create": (C.c_int, [_VP, _U32, C.c_int, C.c_int, _PVP]),
    "sfhe_kway_run": (C.c_int, [_VP, _VP, C.c_int, C.c_int, C.c_int, _U32, _PVP]),
    "sfhe_kway_destroy": (None, [_VP]),
    "sfhe_kway_graph_nodes": (C.c_int, [_VP, _PU64]),
    "sfhe_kway_graph_family_time": (C.c_int, [_VP, _U32, C.c_int, _PD, _PU64, _PD]),
    "sfhe_load": (C.c_int, [C.c_char_p, _PVP]),
    "sfhe_ct_save": (C.c_int, [_VP, _VP, C.c_char_p]),
    "sfhe_ct_load": (C.c_int, [_VP, C.c_char_p, _PVP]),
    "sfhe_kway_sort": (C.c_int, [_VP, _VP, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _U32, _PVP]),
    "sfhe_kway_params": (C.c_int, [_U32, _PU32, _PU32, _PU32, _PU32, _PI32, _SZ, _PSZ]),
    "sfhe_sorter_graph_ntt_time": (C.c_int, [_VP, C.c_int, _PD, _PU64, _PD]),
    "sfhe_sorter_graph_family_time": (C.c_int, [_VP, C.c_uint32, C.c_int, _PD, _PU64, _PD]),
    "sfhe_kernel_timing": (C.c_int, [_VP, _U32, _U32]),
    "sfhe_serialize_lanes": (C.c_int, [_VP, C.c_int]),
    "sfhe_stack_stats": (C.c_int, [_VP, _PU64, _PU64]),
    "sfhe_comm_stats_reset": (C.c_int, [_VP, C.c_int]),
    "sfhe_comm_stats": (C.c_int, [_VP, _PU64, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "sfhe_kernel_timing_read": (C.c_int, [_VP, _U32, _PU64, _PU64, _PD, _PD]),
    "sfhe_decompose": (C.c_int, [_U32, _PI32, _SZ, C.c_int32, C.c_int32, C.c_int, _PI32, _PI32, _SZ, _PSZ]),
    "sfhe_comm_uid": (C.c_int, [_VP]),
    "sfhe_pool_bytes": (C.c_int, [_VP, _PU64]),
    "sfhe_live_contexts": (C.c_int, []),
    "sfhe_shard_rccl": (C.c_int, [_VP, C.c_int, C.c_int, _VP]),
    "sfhe_shard_host": (C.c_int, [_VP, C.c_int, C.c_int, _AG, _BC, _VP]),
    "sfhe_shard_tail": (C.c_int, [_VP, _PU32]),
    "sfhe_key_rows": (C.c_int, [_VP, _PU32]),
    "sfhe_groups_rccl": (C.c_int, [_VP, C.c_int, C.c_int, _VP]),
    "sfhe_groups_host": (C.c_int, [_VP, C.c_int, C.c_int, _AG, _VP]),
    "sfhe_groups": (C.c_int, [_VP, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "sfhe_encode_counts": (C.c_int, [_VP, _PU64, _PU64]),
    "sfhe_bootstrap_graphs": (C.c_int, [_VP, _PU64]),
}

_libs: dict = {}


def lib_path(backend: str = "hip") -> str:
    # SFHE_PRODUCT_LIB: an alternative HIP build (tools: kernel-variant sweeps)
    return os.environ.get("SFHE_PRODUCT_LIB", PRODUCT_LIB) if backend == "hip" else ORACLE_LIB


ABI_VERSION = 3  # include/sfhe.h SFHE_ABI_VERSION


def load(backend: str = "hip"):
    """Load the engine library.  backend='hip' is the product (raises if the
    HIP build is absent); backend='oracle' is the CPU oracle (tests only)."""
    if backend in _libs:
        return _libs[backend]
    path = lib_path(backend)
    if not os.path.exists(path):
        raise SfheError(
            f"{backend} library not built: {path} is missing "
            f"(run `make -C sorting-fhe_amd` for the HIP product, `make -C oracle` for the oracle)")
    lib = C.CDLL(path)
    for name, (res, args) in _SIGS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    # the ctypes structures and signatures above are those of include/sfhe.h
    # at SFHE_ABI_VERSION: refuse a library built from another version
    if lib.sfhe_abi_version() != ABI_VERSION:
        raise SfheError(f"{path}: C ABI version {lib.sfhe_abi_version()}, this binding speaks {ABI_VERSION} "
                        "(rebuild the library or use the matching sfhe.py)")
    _libs[backend] = lib
    return lib


def _darr(v: Sequence[float]):
    a = (C.c_double * len(v))(*[float(x) for x in v])
    return a


class Engine:
    """Thin object wrapper; one CKKS context + key pair."""

    def __init__(self, backend: str = "hip", *, mult_depth: int, ring_dim: int = 0,
                 batch_size: int = 0, scaling_mod_size: int = 40, first_mod_size: int = 60,
                 secure: bool = False, num_large_digits: int = 0, seed: int = 0x5EED5EED2025,
                 device: int = 0, rotations: Sequence[int] = (), keygen: bool = True,
                 scaling: str = "FLEXIBLEAUTOEXT", shard=None, groups=None):
        """shard: None, ("rccl", rank, world, uid) or ("host", rank, world, comm)
        (limb sharding, include/sfhe.h; every rank passes the same params).
        groups: None, ("rccl", group, groups, uid) or ("host", group, groups,
        comm): the sort's batches split over batch groups (sfhe_groups_*)."""
        self.lib = load(backend)
        self.backend = backend
        p = Params()
        self.lib.sfhe_params_default(C.byref(p))
        p.mult_depth = mult_depth
        p.ring_dim = ring_dim
        p.batch_size = batch_size
        p.scaling_mod_size = scaling_mod_size
        p.first_mod_size = first_mod_size
        p.security_level = HESTD_128_CLASSIC if secure else HESTD_NOTSET
        p.num_large_digits = num_large_digits
        p.seed = seed
        p.device = device
        p.scaling_technique = {"FLEXIBLEAUTO": 2, "FLEXIBLEAUTOEXT": 3}[scaling]
        self.ctx = C.c_void_p()
        self._chk(self.lib.sfhe_context_create(C.byref(p), C.byref(self.ctx)))
        self._comm_refs = None
        if shard is not None:
            kind, rank, world, arg = shard
            if kind == "rccl":
                self.shard_rccl(rank, world, arg)
            elif kind == "host":
                self.shard_host(rank, world, arg)
            else:
                raise ValueError(f"unknown shard transport {kind!r}")
        if groups is not None:
            kind, g, G, arg = groups
            if kind == "rccl":
                self.groups_rccl(g, G, arg)
            elif kind == "host":
                self.groups_host(g, G, arg)
            else:
                raise ValueError(f"unknown group transport {kind!r}")
        if keygen:
            self._chk(self.lib.sfhe_keygen(self.ctx))
            if rotations:
                self.rotate_keygen(rotations)

    @classmethod
    def load(cls, directory: str, backend: str = "hip") -> "Engine":
        """A context and keys from sfhe_save's file set (src/sort.h:31-102)."""
        self = cls.__new__(cls)
        self.lib = load(backend)
        self.backend = backend
        self._comm_refs = None
        self.ctx = C.c_void_p()
        self._chk(self.lib.sfhe_load(directory.encode(), C.byref(self.ctx)))
        return self

    def save(self, directory: str):
        self._chk(self.lib.sfhe_save(self.ctx, directory.encode()))

    def save_ct(self, ct: "Ct", path: str):
        self._chk(self.lib.sfhe_ct_save(self.ctx, ct.h, path.encode()))

    def load_ct(self, path: str) -> "Ct":
        return self._new(self.lib.sfhe_ct_load, self.ctx, path.encode())

    # -- plumbing --
    def _chk(self, rc: int):
        if rc != SFHE_OK:
            raise SfheError(f"sfhe error {rc}: {self.lib.sfhe_last_error().decode()}")

    def close(self):
        if self.ctx:
            self.lib.sfhe_context_destroy(self.ctx)
            self.ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _new(self, fn, *args) -> "Ct":
        out = C.c_void_p()
        self._chk(fn(*args, C.byref(out)))
        return Ct(self, out)

    # -- limb sharding --
    def shard_rccl(self, rank: int, world: int, uid: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(bytes(uid))
        self._chk(self.lib.sfhe_shard_rccl(self.ctx, rank, world, buf))

    def shard_host(self, rank: int, world: int, comm):
        """comm: object with allgather(rank, send, recv, nbytes) and
        bcast(rank, buf, nbytes, root) over raw addresses (ThreadComm, GlooComm)."""
        ag = _AG(lambda _u, send, recv, nb: comm.allgather(rank, send, recv, nb))
        bc = _BC(lambda _u, buf, nb, root: comm.bcast(rank, buf, nb, root))
        self._chk(self.lib.sfhe_shard_host(self.ctx, rank, world, ag, bc, None))
        self._comm_refs = (ag, bc, comm)  # the library keeps the raw pointers

    def groups_rccl(self, group: int, groups: int, uid: bytes):
        buf = (C.c_uint8 * 128).from_buffer_copy(bytes(uid))
        self._chk(self.lib.sfhe_groups_rccl(self.ctx, group, groups, buf))

    def groups_host(self, group: int, groups: int, comm):
        """comm: as shard_host's (only its allgather is used)."""
        ag = _AG(lambda _u, send, recv, nb: comm.allgather(group, send, recv, nb))
        self._chk(self.lib.sfhe_groups_host(self.ctx, group, groups, ag, None))
        self._group_refs = (ag, comm)

    def groups(self):
        """(group, groups) of the batch split ((0, 1): unsplit)."""
        g, G = C.c_int(), C.c_int()
        self._chk(self.lib.sfhe_groups(self.ctx, C.byref(g), C.byref(G)))
        return g.value, G.value

    def shard_tail(self) -> int:
        """Replicated-tail limb count of a sharded context (0: unsharded)."""
        v = C.c_uint32()
        self._chk(self.lib.sfhe_shard_tail(self.ctx, C.byref(v)))
        return v.value

    def key_rows(self) -> int:
        """Rows per digit part of this rank's switching keys (a slice when sharded)."""
        v = C.c_uint32()
        self._chk(self.lib.sfhe_key_rows(self.ctx, C.byref(v)))
        return v.value

    # -- context --
    def rotate_keygen(self, idx: Sequence[int]):
        a = (C.c_int32 * len(idx))(*idx)
        self._chk(self.lib.sfhe_rotate_keygen(self.ctx, a, len(idx)))

    def info(self) -> dict:
        v = [C.c_uint32() for _ in range(5)]
        self._chk(self.lib.sfhe_context_info(self.ctx, *[C.byref(x) for x in v]))
        return dict(ring_dim=v[0].value, mult_depth=v[1].value, num_q=v[2].value,
                    num_p=v[3].value, dnum=v[4].value)

    def primes(self) -> list:
        cnt = C.c_size_t()
        self._chk(self.lib.sfhe_context_primes(self.ctx, None, 0, C.byref(cnt)))
        buf = (C.c_uint64 * cnt.value)()
        self._chk(self.lib.sfhe_context_primes(self.ctx, buf, cnt.value, None))
        return list(buf)

    def sync(self):
        self._chk(self.lib.sfhe_sync(self.ctx))

    def set_quiet(self, q: bool = True):
        self._chk(self.lib.sfhe_set_quiet(self.ctx, int(q)))

    def set_plaintext_cache(self, on: bool):
        self._chk(self.lib.sfhe_set_plaintext_cache(self.ctx, int(on)))

    def op_stats(self, reset: bool = False) -> dict:
        c = (C.c_uint64 * 9)()
        b = C.c_double()
        self._chk(self.lib.sfhe_op_stats(self.ctx, c, C.byref(b), int(reset)))
        keys = ["keyswitch", "rescale", "tensor", "ptmult", "constmult", "add", "automorph",
                "ntt_limbs", "wsum_terms"]
        d = dict(zip(keys, list(c)))
        d["algo_bytes"] = b.value
        return d

    def encode_counts(self):
        """(device, host) plaintext encodings since the last op_stats reset."""
        d, h = C.c_uint64(), C.c_uint64()
        self._chk(self.lib.sfhe_encode_counts(self.ctx, C.byref(d), C.byref(h)))
        return d.value, h.value

    def pool_bytes(self) -> int:
        v = C.c_uint64()
        self._chk(self.lib.sfhe_pool_bytes(self.ctx, C.byref(v)))
        return v.value

    KFAM = {"ntt": 0, "conv": 1, "ks_inner": 2, "ntt_ks": 3}

    def kernel_timing(self, family: str, period: int = 1):
        self._chk(self.lib.sfhe_kernel_timing(self.ctx, self.KFAM[family], period))

    def serialize_lanes(self, on: bool = True):
        self._chk(self.lib.sfhe_serialize_lanes(self.ctx, int(on)))

    def stack_stats(self):
        """(merged pairs, launches alone) issued by stacked regions so far."""
        m, s1 = C.c_uint64(), C.c_uint64()
        self._chk(self.lib.sfhe_stack_stats(self.ctx, C.byref(m), C.byref(s1)))
        return m.value, s1.value

    def comm_stats_reset(self, timed: bool = True):
        """Zero the collective counters (timed: also time each eager collective)."""
        self._chk(self.lib.sfhe_comm_stats_reset(self.ctx, 1 if timed else 0))

    def comm_stats(self) -> dict:
        """Collectives this rank issued since comm_stats_reset: calls, bytes received, ms."""
        n, by, ms = C.c_uint64(), C.c_double(), C.c_double()
        self._chk(self.lib.sfhe_comm_stats(self.ctx, C.byref(n), C.byref(by), C.byref(ms)))
        return {"calls": n.value, "bytes": by.value, "ms": ms.value}

    def kernel_timing_read(self, family: str) -> dict:
        la, ti = C.c_uint64(), C.c_uint64()
        ms, by = C.c_double(), C.c_double()
        self._chk(self.lib.sfhe_kernel_timing_read(self.ctx, self.KFAM[family], C.byref(la),
                                                   C.byref(ti), C.byref(ms), C.byref(by)))
        return {"launches": la.value, "timed": ti.value, "ms": ms.value, "bytes": by.value}

    # -- data --
    def encrypt(self, values: Sequence[float], slots: int = 0, level: int = 0) -> "Ct":
        a = _darr(values)
        return self._new(self.lib.sfhe_encrypt, self.ctx, a, len(values), slots, level)

    def decrypt(self, ct: "Ct") -> list:
        n = C.c_size_t()
        self._chk(self.lib.sfhe_decrypt(self.ctx, ct.h, None, 0, C.byref(n)))
        buf = (C.c_double * n.value)()
        self._chk(self.lib.sfhe_decrypt(self.ctx, ct.h, buf, n.value, None))
        return list(buf)

    # -- eval --
    def add(self, a, b):
        return self._new(self.lib.sfhe_eval_add, self.ctx, a.h, b.h)

    def sub(self, a, b):
        return self._new(self.lib.sfhe_eval_sub, self.ctx, a.h, b.h)

    def add_const(self, a, k: float):
        return self._new(self.lib.sfhe_eval_add_const, self.ctx, a.h, float(k))

    def mult_const(self, a, k: float):
        return self._new(self.lib.sfhe_eval_mult_const, self.ctx, a.h, float(k))

    def mult_plain(self, a, values: Sequence[float], slots: int = 0):
        return self._new(self.lib.sfhe_eval_mult_plain, self.ctx, a.h, _darr(values), len(values), slots)

    def mult(self, a, b):
        return self._new(self.lib.sfhe_eval_mult, self.ctx, a.h, b.h)

    def rotate(self, a, r: int):
        return self._new(self.lib.sfhe_eval_rotate, self.ctx, a.h, int(r))

    def rotate_sum(self, cts, rots):
        """sum_k rotate(cts[k], rots[k]) with one shared ModDown (EvalRotateSum)."""
        hs = (_VP * len(cts))(*[c.h for c in cts])
        rs = (C.c_int32 * len(rots))(*[int(r) for r in rots])
        return self._new(self.lib.sfhe_eval_rotate_sum, self.ctx, hs, rs, len(cts))

    def bootstrap_setup(self, level_budget=(5, 5), slots: int = 0):
        """EvalBootstrapSetup + EvalBootstrapKeyGen for `slots`-slot ciphertexts."""
        self._chk(self.lib.sfhe_bootstrap_setup(self.ctx, level_budget[0], level_budget[1], slots))

    def bootstrap_depth(self, level_budget=(5, 5), slots: int = 0) -> int:
        v = C.c_uint32()
        self._chk(self.lib.sfhe_bootstrap_depth(self.ctx, level_budget[0], level_budget[1], slots, C.byref(v)))
        return v.value

    def bootstrap_graphs(self) -> int:
        """Bootstrap shapes replayed from a captured hipGraph so far."""
        v = C.c_uint64()
        self._chk(self.lib.sfhe_bootstrap_graphs(self.ctx, C.byref(v)))
        return v.value

    def bootstrap(self, a, iterations: int = 1, precision: int = 0):
        return self._new(self.lib.sfhe_bootstrap, self.ctx, a.h, iterations, precision)

    def kway(self, k: int, M: int) -> "KWay":
        """A persistent KWayAdapter<k^M> (reuses its encoded masks across sorts)."""
        h = C.c_void_p()
        self._chk(self.lib.sfhe_kway_create(self.ctx, k ** M, k, M, C.byref(h)))
        return KWay(self, h)

    def kway_sort(self, a, k: int, M: int, n: int = 3, dg: int = 2, df: int = 2, mult_depth: int = 40):
        """KWayAdapter<k^M>::sort (reference kway_adapter.h:66-72): the k-way
        network with CompositeSign(n, dg, df) and lazy bootstrapping."""
        return self._new(self.lib.sfhe_kway_sort, self.ctx, a.h, k, M, n, dg, df, mult_depth)

    def chebyshev(self, x, coeffs: Sequence[float], a: float = -1.0, b: float = 1.0):
        return self._new(self.lib.sfhe_eval_chebyshev, self.ctx, x.h, _darr(coeffs), len(coeffs),
                         float(a), float(b))

    def sign(self, x, n: int, dg: int, df: int):
        return self._new(self.lib.sfhe_sign, self.ctx, x.h, n, dg, df)

    def compare(self, a, b, n: int, dg: int, df: int):
        return self._new(self.lib.sfhe_compare, self.ctx, a.h, b.h, n, dg, df)

    def sorter(self, N: int, debug: bool = False, rotations=None) -> "Sorter":
        """DirectSort<N>; rotations = the constructor's rotIndices (None: the
        getSizeParameters list)."""
        h = C.c_void_p()
        if rotations is None:
            self._chk(self.lib.sfhe_sorter_create(self.ctx, N, int(debug), C.byref(h)))
        else:
            buf = (C.c_int32 * len(rotations))(*rotations)
            self._chk(self.lib.sfhe_sorter_create_rot(self.ctx, N, int(debug), buf, len(rotations), C.byref(h)))
        return Sorter(self, h, N)


class Ct:
    def __init__(self, eng: Engine, h):
        self.eng = eng
        self.h = h

    def __del__(self):
        try:
            if self.h:
                self.eng.lib.sfhe_ct_free(self.h)
                self.h = None
        except Exception:
            pass

    def info(self) -> dict:
        v = [C.c_uint32() for _ in range(3)]
        self.eng._chk(self.eng.lib.sfhe_ct_info(self.h, *[C.byref(x) for x in v]))
        return dict(level=v[0].value, slots=v[1].value, limbs=v[2].value)

    @property
    def level(self) -> int:
        return self.info()["level"]

    @property
    def slots(self) -> int:
        return self.info()["slots"]

    def set_slots(self, s: int):
        self.eng._chk(self.eng.lib.sfhe_ct_set_slots(self.h, s))

    def clone(self) -> "Ct":
        return self.eng._new(self.eng.lib.sfhe_ct_clone, self.h)

    def download(self):
        import numpy as np
        n = self.eng.info()["ring_dim"]
        words = 2 * self.info()["limbs"] * n
        buf = np.empty(words, dtype=np.uint64)
        self.eng._chk(self.eng.lib.sfhe_ct_download(
            self.eng.ctx, self.h, buf.ctypes.data_as(_PU64), words))
        return buf


class Sorter:
    def __init__(self, eng: Engine, h, N: int):
        self.eng, self.h, self.N = eng, h, N

    def __del__(self):
        try:
            if self.h:
                self.eng.lib.sfhe_sorter_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def sort(self, ct: Ct, n: int = 3, dg: int = 2, df: int = 2) -> Ct:
        return self.eng._new(self.eng.lib.sfhe_sorter_sort, self.h, ct.h, n, dg, df)

    def rank(self, ct: Ct, n: int = 3, dg: int = 2, df: int = 2) -> Ct:
        return self.eng._new(self.eng.lib.sfhe_sorter_rank, self.h, ct.h, n, dg, df)

    def place(self, rank: Ct, ct: Ct) -> Ct:
        return self.eng._new(self.eng.lib.sfhe_sorter_place, self.h, rank.h, ct.h)

    def sort_hybrid1(self, ct: Ct, n: int = 3, dg: int = 2, df: int = 2) -> Ct:
        """DirectSort<N>::sort_hybrid1 (reference sort_algo.h:1213-1229)."""
        return self.eng._new(self.eng.lib.sfhe_sorter_sort_hybrid1, self.h, ct.h, n, dg, df)

    def sort_hybrid(self, ct: Ct, n: int = 3, dg: int = 2, df: int = 2, variant: int = 0) -> Ct:
        """DirectSort<N>::sort_hybrid (variant 0, reference sort_algo.h:1049-1062) or
        sort_hybrid2 (variant 2, :1376-1389)."""
        return self.eng._new(self.eng.lib.sfhe_sorter_sort_hybrid, self.h, ct.h, variant, n, dg, df)

    def place_2n(self, rank: Ct, ct: Ct) -> Ct:
        """DirectSort<N>::rotationIndexCheck2N (reference sort_algo.h:587-656)."""
        return self.eng._new(self.eng.lib.sfhe_sorter_place_2n, self.h, rank.h, ct.h)

    def sort_bitonic(self, ct: Ct, n: int = 4, dg: int = 3, df: int = 3) -> Ct:
        """BitonicSort<N>::sort (reference sort_algo.h:1421-1486); values in [0, 255]."""
        return self.eng._new(self.eng.lib.sfhe_sorter_sort_bitonic, self.h, ct.h, n, dg, df)

    def graph_ntt_time(self, reps: int = 5):
        """(ms per sort, launches, algorithmic bytes) of the captured sort's
        NTT kernels replayed alone (sfhe_sorter_graph_ntt_time)."""
        ms, n, b = C.c_double(), C.c_uint64(), C.c_double()
        self.eng._chk(self.eng.lib.sfhe_sorter_graph_ntt_time(self.h, reps, C.byref(ms), C.byref(n), C.byref(b)))
        return ms.value, n.value, b.value

    def graph_family_time(self, family: str, reps: int = 3):
        """(ms per sort, launches, NTT algorithmic bytes) of the captured
        sort's kernels of one family (KFAM names, "other" or "all") replayed
        alone (sfhe_sorter_graph_family_time)."""
        f = {**self.eng.KFAM, "other": 4, "all": 5}[family]
        ms, n, b = C.c_double(), C.c_uint64(), C.c_double()
        self.eng._chk(self.eng.lib.sfhe_sorter_graph_family_time(self.h, f, reps, C.byref(ms), C.byref(n),
                                                                 C.byref(b)))
        return ms.value, n.value, b.value

    def graph_nodes(self) -> int:
        v = C.c_uint64()
        self.eng._chk(self.eng.lib.sfhe_sorter_graph_nodes(self.h, C.byref(v)))
        return v.value


def direct_sort_params(N: int, backend: str = "hip"):
    lib = load(backend)
    depth = C.c_uint32()
    cnt = C.c_size_t()
    rc = lib.sfhe_direct_sort_params(N, C.byref(depth), None, 0, C.byref(cnt))
    if rc != SFHE_OK:
        raise SfheError(lib.sfhe_last_error().decode())
    buf = (C.c_int32 * cnt.value)()
    lib.sfhe_direct_sort_params(N, None, buf, cnt.value, None)
    return depth.value, list(buf)


class KWay:
    def __init__(self, eng: "Engine", h):
        self.eng, self.h = eng, h

    def __del__(self):
        try:
            if self.h:
                self.eng.lib.sfhe_kway_destroy(self.h)
                self.h = None
        except Exception:
            pass

    def sort(self, ct: "Ct", n: int = 3, dg: int = 2, df: int = 2, mult_depth: int = 40) -> "Ct":
        return self.eng._new(self.eng.lib.sfhe_kway_run, self.h, ct.h, n, dg, df, mult_depth)

    def graph_nodes(self) -> int:
        """Nodes of the captured sort graph (0: none yet / eager)."""
        v = C.c_uint64()
        self.eng._chk(self.eng.lib.sfhe_kway_graph_nodes(self.h, C.byref(v)))
        return v.value

    def graph_family_time(self, family: str, reps: int = 1):
        """(ms per sort, launches, algorithmic bytes) of the captured sort's
        kernels of one family replayed alone, over its chain of graphs."""
        f = {**self.eng.KFAM, "other": 4, "all": 5}[family]
        ms, n, b = C.c_double(), C.c_uint64(), C.c_double()
        self.eng._chk(self.eng.lib.sfhe_kway_graph_family_time(self.h, f, reps, C.byref(ms), C.byref(n),
                                                               C.byref(b)))
        return ms.value, n.value, b.value


def kway_params(N: int, backend: str = "hip"):
    """KWayAdapter<N>::getSizeParameters: (batch, depth, level budget, rotations)."""
    lib = load(backend)
    b, d, b0, b1, cnt = C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_uint32(), C.c_size_t()
    rc = lib.sfhe_kway_params(N, C.byref(b), C.byref(d), C.byref(b0), C.byref(b1), None, 0, C.byref(cnt))
    if rc != SFHE_OK:
        raise SfheError(f"sfhe error {rc}: {lib.sfhe_last_error().decode()}")
    buf = (C.c_int32 * cnt.value)()
    lib.sfhe_kway_params(N, None, None, None, None, buf, cnt.value, None)
    return b.value, d.value, (b0.value, b1.value), list(buf)


def hybrid_params(N: int, variant: int = 0, backend: str = "hip"):
    """(depth, rotation keys) of tests/DirectSortHTest.cpp (variant 0) or
    tests/DirectSortH2Test.cpp (variant 2) for N."""
    lib = load(backend)
    depth = C.c_uint32()
    cnt = C.c_size_t()
    rc = lib.sfhe_hybrid_params(N, variant, C.byref(depth), None, 0, C.byref(cnt))
    if rc != SFHE_OK:
        raise SfheError(f"sfhe error {rc}: {lib.sfhe_last_error().decode()}")
    buf = (C.c_int32 * cnt.value)()
    lib.sfhe_hybrid_params(N, variant, None, buf, cnt.value, None)
    return depth.value, list(buf)


def hybrid1_params(N: int, backend: str = "hip"):
    """(depth, rotation keys) of tests/DirectSortH1Test.cpp:36-117 for N."""
    lib = load(backend)
    depth = C.c_uint32()
    cnt = C.c_size_t()
    rc = lib.sfhe_hybrid1_params(N, C.byref(depth), None, 0, C.byref(cnt))
    if rc != SFHE_OK:
        raise SfheError(lib.sfhe_last_error().decode())
    buf = (C.c_int32 * cnt.value)()
    lib.sfhe_hybrid1_params(N, None, buf, cnt.value, None)
    return depth.value, list(buf)


def doubled_sinc_coeffs(N: int, backend: str = "hip"):
    lib = load(backend)
    cnt = C.c_size_t()
    rc = lib.sfhe_doubled_sinc_coeffs(N, None, 0, C.byref(cnt))
    if rc != SFHE_OK:
        raise SfheError(lib.sfhe_last_error().decode())
    buf = (C.c_double * cnt.value)()
    lib.sfhe_doubled_sinc_coeffs(N, buf, cnt.value, None)
    return list(buf)


def decompose(N: int, keys: Sequence[int], rotation: int, wrapN: int, algo: int, backend: str = "hip"):
    lib = load(backend)
    k = (C.c_int32 * len(keys))(*keys)
    cap = 64
    v = (C.c_int32 * cap)()
    s = (C.c_int32 * cap)()
    cnt = C.c_size_t()
    rc = lib.sfhe_decompose(N, k, len(keys), rotation, wrapN, algo, v, s, cap, C.byref(cnt))
    if rc == SFHE_OK and cnt.value > cap:  # long chains: ask again with room for all of them
        cap = cnt.value
        v, s = (C.c_int32 * cap)(), (C.c_int32 * cap)()
        rc = lib.sfhe_decompose(N, k, len(keys), rotation, wrapN, algo, v, s, cap, C.byref(cnt))
    if rc != SFHE_OK:
        raise SfheError(lib.sfhe_last_error().decode())
    return [(v[i], s[i]) for i in range(min(cnt.value, cap))]


# ---- limb-sharding transports ------------------------------------------------

def live_contexts(backend: str = "hip") -> int:
    """Engine contexts alive in this process (sfhe_live_contexts)."""
    return load(backend).sfhe_live_contexts()


def comm_uid(backend: str = "hip"):
    """128-byte RCCL unique id (bytes), or None where the backend has no RCCL."""
    lib = load(backend)
    buf = (C.c_uint8 * 128)()
    if lib.sfhe_comm_uid(buf) != SFHE_OK:
        return None
    return bytes(buf)


class ThreadComm:
    """Host collectives between `world` threads of one process (each thread
    one rank; tests).  Callbacks run with the GIL held; the library calls
    them with the GIL released, so the ranks' device work overlaps."""

    def __init__(self, world: int, timeout: float = 600.0):
        import threading
        self.world = world
        self.bar = threading.Barrier(world, timeout=timeout)
        self.slots = [b""] * world

    def allgather(self, rank, send, recv, nbytes):
        self.slots[rank] = C.string_at(send, nbytes) if nbytes else b""
        self.bar.wait()
        for r in range(self.world):
            if nbytes:
                C.memmove(recv + r * nbytes, self.slots[r], nbytes)
        self.bar.wait()

    def bcast(self, rank, buf, nbytes, root):
        if rank == root:
            self.slots[root] = C.string_at(buf, nbytes) if nbytes else b""
        self.bar.wait()
        if rank != root and nbytes:
            C.memmove(buf, self.slots[root], nbytes)
        self.bar.wait()


class GlooComm:
    """Host collectives over an initialised torch.distributed process group
    (gloo: CPU tensors; one process per rank)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist, self.group = dist, group
        self.world = dist.get_world_size(group)

    def allgather(self, rank, send, recv, nbytes):
        import torch
        t = torch.frombuffer(bytearray(C.string_at(send, nbytes)), dtype=torch.uint8)
        outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.world)]
        self.dist.all_gather(outs, t, group=self.group)
        for r, o in enumerate(outs):
            C.memmove(recv + r * nbytes, o.numpy().ctypes.data, nbytes)

    def bcast(self, rank, buf, nbytes, root):
        import torch
        t = torch.frombuffer(bytearray(C.string_at(buf, nbytes)), dtype=torch.uint8)
        # root is a rank of this communicator; torch wants the global rank
        src = root if self.group is None else self.dist.get_global_rank(self.group, root)
        self.dist.broadcast(t, src=src, group=self.group)
        if rank != root:
            C.memmove(buf, t.numpy().ctypes.data, nbytes)


def run_split_threads(backend: str, world: int, groups: int, fn, **engine_kw):
    """Run fn(engine) on `world` thread ranks split into `groups` batch groups
    of world // groups ranks (rank = group * (world // groups) + r); each
    group limb-sharded over its own ThreadComm when it has more than one
    rank.  Returns the per-rank results (rank order)."""
    import threading
    per = world // groups
    if per * groups != world:
        raise ValueError("world must be a multiple of groups")
    limb = [ThreadComm(per) for _ in range(groups)]
    grp = [ThreadComm(groups) for _ in range(per)]
    outs, errs = [None] * world, []

    def body(rank):
        g, r = divmod(rank, per)
        try:
            shard = ("host", r, per, limb[g]) if per > 1 else None
            e = Engine(backend, shard=shard, groups=("host", g, groups, grp[r]), **engine_kw)
            outs[rank] = fn(e)
        except BaseException as ex:  # unblock the other ranks
            errs.append(ex)
            for c in limb + grp:
                c.bar.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    return outs


def run_sharded_threads(backend: str, world: int, fn, **engine_kw):
    """Run fn(engine) on `world` limb-sharded engines, one thread per rank,
    over ThreadComm; returns the per-rank results (rank order)."""
    import threading
    comm = ThreadComm(world)
    outs, errs = [None] * world, []

    def body(r):
        try:
            e = Engine(backend, shard=("host", r, world, comm), **engine_kw)
            outs[r] = fn(e)
        except BaseException as ex:  # unblock the other ranks
            errs.append(ex)
            comm.bar.abort()

    th = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errs:
        raise errs[0]
    return outs
