"""Python mirror of the reference's `KeyCollection<FE, FieldElm>` (src/collect.rs:28-1030),
backed by the HIP engine in libfhh.so. Same method names and argument meaning; errors raise
FhhError where the reference panics.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ._lib import FhhError, FhhStats, check, lib, ptr, u32p, u64p
from .fields import FE255_P, FE_P, limbs10_to_int, int_to_limbs


@dataclass
class Result:
    """collect.rs:39-43: `Result<T> { path: Vec<Vec<bool>>, value: T }`."""
    path: list      # d lists of bools
    value: int      # unreduced FieldElm sum as int (or count in plaintext-count harness mode)


class KeyCollection:
    """One server's key collection (collect.rs:45-1030) on one GPU, or — with `devices` — one
    collection whose clients are sharded over several GPUs (fhh_create_multi: contiguous ranges
    of 64-client words, per-child partials reduced over an in-process RCCL communicator, or on
    the host when a device repeats). The methods are the same either way."""

    def __init__(self, depth: int, n_dims: int, device: int = 0, devices=None):
        # KeyCollection::new(seed, depth) (collect.rs:51-60)
        self.depth = depth
        self.n_dims = n_dims
        self.device = device if devices is None else int(devices[0])
        self.devices = None if devices is None else [int(x) for x in devices]
        self._owner = None
        h = ctypes.c_void_p()
        if devices is None:
            check(lib().fhh_create(ctypes.byref(h), depth, n_dims, device))
        else:
            arr = (ctypes.c_int * len(self.devices))(*self.devices)
            check(lib().fhh_create_multi(ctypes.byref(h), depth, n_dims, arr, len(self.devices)))
        self._h = h

    @classmethod
    def _borrowed(cls, owner: "KeyCollection", handle, device: int):
        """A shard's ctx, owned by `owner` (never destroyed through this object)."""
        kc = cls.__new__(cls)
        kc.depth, kc.n_dims, kc.device, kc.devices = owner.depth, owner.n_dims, device, None
        kc._owner = owner
        kc._h = handle
        return kc

    def shard_info(self):
        """[(device, client_base, n_clients)] per shard and the reduction ("none" / "host" / "rccl")."""
        from ._lib import FHH_REDUCE_NAMES
        out = []
        ns, dev, red = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        base, cnt = ctypes.c_uint64(), ctypes.c_uint64()
        k = 0
        while True:
            self._chk(lib().fhh_shard_info(self._h, k, ctypes.byref(ns), ctypes.byref(dev), ctypes.byref(base),
                                           ctypes.byref(cnt), ctypes.byref(red)))
            out.append((dev.value, base.value, cnt.value))
            k += 1
            if k >= ns.value:
                break
        return out, FHH_REDUCE_NAMES[red.value]

    def shard(self, k: int) -> "KeyCollection":
        """Shard k's one-GPU collection (per-shard calls: the two-party GC + OT, fhh_gb_* / fhh_ev_*)."""
        h = ctypes.c_void_p()
        self._chk(lib().fhh_shard_ctx(self._h, k, ctypes.byref(h)))
        if h.value == (self._h.value if isinstance(self._h, ctypes.c_void_p) else self._h):
            return self
        return KeyCollection._borrowed(self, h, self.shard_info()[0][k][0])

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_owner", None) is not None:   # a borrowed shard ctx
            self._h = None
            return
        if getattr(self, "_h", None):
            lib().fhh_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        check(rc, self._h)

    # ---- keys -----------------------------------------------------------------------
    def add_keys(self, key_idx: np.ndarray, root_seed: np.ndarray, cw_seed: np.ndarray, cw_bits: np.ndarray):
        """Batched `add_key` (collect.rs:62-65). Shapes [n][d][2], [n][d][2][16],
        [n][d][2][L][16], [n][d][2][L] (uint8)."""
        n = key_idx.shape[0]
        d, L = self.n_dims, self.depth
        if key_idx.shape != (n, d, 2) or root_seed.shape != (n, d, 2, 16) or cw_seed.shape != (n, d, 2, L, 16) \
                or cw_bits.shape != (n, d, 2, L):
            raise FhhError("add_keys: shape mismatch")
        a = [np.ascontiguousarray(x, np.uint8) for x in (key_idx, root_seed, cw_seed, cw_bits)]
        self._chk(lib().fhh_add_keys(self._h, n, *[ptr(x) for x in a]))

    def add_keys_bincode(self, request: bytes):
        """The `add_keys` RPC payload (rpc.rs:12-15: `Vec<Vec<(ibDCFKey, ibDCFKey)>>` in bincode
        legacy encoding), decoded on the GPU straight into the device layout."""
        buf = np.frombuffer(bytes(request), np.uint8) if not isinstance(request, np.ndarray) else \
            np.ascontiguousarray(request, np.uint8)
        self._chk(lib().fhh_add_keys_bincode(self._h, ptr(buf), buf.size))

    def num_clients(self) -> int:
        n = ctypes.c_uint64()
        self._chk(lib().fhh_num_clients(self._h, ctypes.byref(n)))
        return n.value

    def export_keys(self):
        n, d, L = self.num_clients(), self.n_dims, self.depth
        ki = np.zeros((n, d, 2), np.uint8)
        rs = np.zeros((n, d, 2, 16), np.uint8)
        cs = np.zeros((n, d, 2, L, 16), np.uint8)
        cb = np.zeros((n, d, 2, L), np.uint8)
        self._chk(lib().fhh_export_keys(self._h, ptr(ki), ptr(rs), ptr(cs), ptr(cb)))
        return ki, rs, cs, cb

    def set_client_base(self, base: int):
        self._chk(lib().fhh_set_client_base(self._h, base))

    # ---- crawl ----------------------------------------------------------------------
    def tree_init(self):
        self._chk(lib().fhh_tree_init(self._h))

    def _crawl(self, fn, share_planes: bool):
        nch = ctypes.c_uint64()
        if not share_planes:
            self._chk(fn(self._h, ctypes.byref(nch), None))
            return int(nch.value), None
        # query size: frontier size * 2^d
        f = ctypes.c_uint64()
        self._chk(lib().fhh_frontier_size(self._h, ctypes.byref(f), None))
        n = self.num_clients()
        nw = (n + 63) // 64
        # a pending (unpruned) crawl becomes the frontier first; size it generously
        C = int(f.value) << self.n_dims
        planes = np.zeros((C, 2 * self.n_dims, nw), np.uint64)
        self._chk(fn(self._h, ctypes.byref(nch), ptr(planes, u64p)))
        return int(nch.value), planes[: nch.value]

    def tree_crawl(self, share_planes: bool = False):
        """Expansion half of `tree_crawl` (collect.rs:370-418). Returns (C, planes|None);
        planes[c][k][w] bit (client % 64) = share bit k of (child c, client)."""
        return self._crawl(lib().fhh_tree_crawl, share_planes)

    def tree_crawl_last(self, share_planes: bool = False):
        return self._crawl(lib().fhh_tree_crawl_last, share_planes)

    def node_sums_fe(self, vals: np.ndarray) -> np.ndarray:
        """collect.rs:487-501: vals [C][n] u64 -> canonical FE sums [C]."""
        v = np.ascontiguousarray(vals, np.uint64)
        out = np.zeros(v.shape[0], np.uint64)
        self._chk(lib().fhh_node_sums_fe(self._h, ptr(v, u64p), ptr(out, u64p)))
        return out

    def node_sums_fe_device(self, vals_dev, ld: int, C: int, fmt: int = 0) -> np.ndarray:
        """collect.rs:487-501 on OT outputs already in device memory (no host round trip):
        vals_dev = one device pointer (int) per shard, rows [C][ld] (C = the pending crawl's
        children); fmt FHH_VALS_FE_U64 / FHH_VALS_FE_BLOCK. Returns canonical FE sums [C]."""
        ptrs = (ctypes.c_void_p * len(vals_dev))(*[int(p) for p in vals_dev])
        out = np.zeros(max(C, 1), np.uint64)
        self._chk(lib().fhh_node_sums_fe_device(self._h, ptrs, ld, fmt, ptr(out, u64p)))
        return out[:C]

    def node_sums_fe255_device(self, vals_dev, ld: int, C: int, fmt: int = 3):
        """collect.rs:891-905 on device-resident FieldElm OT outputs (FHH_VALS_FE255_LIMBS /
        FHH_VALS_FE255_BLOCKPAIR) -> (unreduced ints, canonical ints)."""
        ptrs = (ctypes.c_void_p * len(vals_dev))(*[int(p) for p in vals_dev])
        unr = np.zeros((max(C, 1), 10), np.uint32)
        can = np.zeros((max(C, 1), 8), np.uint32)
        self._chk(lib().fhh_node_sums_fe255_device(self._h, ptrs, ld, fmt, ptr(unr, u32p), ptr(can, u32p)))
        return [limbs10_to_int(r) for r in unr[:C]], [limbs10_to_int(r) for r in can[:C]]

    def node_sums_fe255(self, vals: np.ndarray):
        """collect.rs:891-905: vals [C][n][8] u32 LE limbs -> (unreduced ints, canonical ints)."""
        v = np.ascontiguousarray(vals, np.uint32)
        C = v.shape[0]
        unr = np.zeros((C, 10), np.uint32)
        can = np.zeros((C, 8), np.uint32)
        self._chk(lib().fhh_node_sums_fe255(self._h, ptr(v, u32p), ptr(unr, u32p), ptr(can, u32p)))
        return [limbs10_to_int(r) for r in unr], [limbs10_to_int(r) for r in can]

    def tree_prune(self, keep):
        k = np.ascontiguousarray(np.asarray(keep, bool).astype(np.uint8))
        self._chk(lib().fhh_tree_prune(self._h, ptr(k), k.size))

    def tree_prune_last(self, keep):
        k = np.ascontiguousarray(np.asarray(keep, bool).astype(np.uint8))
        self._chk(lib().fhh_tree_prune_last(self._h, ptr(k), k.size))

    def frontier_size(self):
        a, b = ctypes.c_uint64(), ctypes.c_uint64()
        self._chk(lib().fhh_frontier_size(self._h, ctypes.byref(a), ctypes.byref(b)))
        return int(a.value), int(b.value)

    def final_shares(self):
        """collect.rs:993-1005 -> list of Result(path, value)."""
        nf, lv = ctypes.c_uint64(), ctypes.c_uint32()
        self._chk(lib().fhh_final_shares(self._h, ctypes.byref(nf), ctypes.byref(lv), None, None))
        F, L = int(nf.value), int(lv.value)
        paths = np.zeros((F, self.n_dims, max(L, 1)), np.uint8)
        vals = np.zeros((F, 10), np.uint32)
        if F:
            self._chk(lib().fhh_final_shares(self._h, ctypes.byref(nf), ctypes.byref(lv), ptr(paths),
                                             ptr(vals, u32p)))
        bits = paths[:, :, :L].astype(bool).tolist()
        return [Result(bits[k], limbs10_to_int(vals[k])) for k in range(F)]

    def export_states(self):
        """EvalStates of the frontier (or pending children) as [node][n][d][2] seed/t/y."""
        nn = ctypes.c_uint64()
        self._chk(lib().fhh_export_states(self._h, ctypes.byref(nn), None, None, None))
        F, n, d = int(nn.value), self.num_clients(), self.n_dims
        seeds = np.zeros((F, n, d, 2, 16), np.uint8)
        t = np.zeros((F, n, d, 2), np.uint8)
        y = np.zeros((F, n, d, 2), np.uint8)
        self._chk(lib().fhh_export_states(self._h, ctypes.byref(nn), ptr(seeds), ptr(t), ptr(y)))
        return seeds, t, y

    def stats(self) -> dict:
        s = FhhStats()
        self._chk(lib().fhh_get_stats(self._h, ctypes.byref(s)))
        return {k: getattr(s, k) for k, _ in FhhStats._fields_}

    def set_timing(self, every: int):
        """0: no k_expand events; 1: time every launch; K > 1: every K-th level-loop launch."""
        self._chk(lib().fhh_set_timing(self._h, every))

    def set_variant(self, variant: int):
        """Select the k_expand variant (bit-identical outputs, different speed)."""
        self._chk(lib().fhh_set_variant(self._h, variant))

    def reset_stats(self):
        self._chk(lib().fhh_reset_stats(self._h))

    def reset(self):
        self._chk(lib().fhh_reset(self._h))

    # ---- leader-side static helpers (collect.rs:945-1029) ------------------------------------
    @staticmethod
    def keep_values(nclients: int, threshold: int, vals0, vals1):
        v0 = np.ascontiguousarray(np.asarray(vals0, np.uint64))
        v1 = np.ascontiguousarray(np.asarray(vals1, np.uint64))
        if v0.shape != v1.shape:
            raise FhhError("keep_values: vals0.len() != vals1.len() (collect.rs:946)")
        keep = np.zeros(v0.size, np.uint8)
        check(lib().fhh_keep_values(threshold, ptr(v0, u64p), ptr(v1, u64p), v0.size, ptr(keep)))
        return keep.astype(bool)

    @staticmethod
    def keep_values_last(nclients: int, threshold: int, vals0, vals1):
        if len(vals0) != len(vals1):
            raise FhhError("keep_values_last: vals0.len() != vals1.len() (collect.rs:967)")
        a = np.array([int_to_limbs(v, 10) for v in vals0], np.uint32).reshape(-1, 10)
        b = np.array([int_to_limbs(v, 10) for v in vals1], np.uint32).reshape(-1, 10)
        keep = np.zeros(len(vals0), np.uint8)
        check(lib().fhh_keep_values_last(threshold, ptr(a, u32p), ptr(b, u32p), len(vals0), ptr(keep)))
        return keep.astype(bool)

    @staticmethod
    def final_values(res0, res1):
        if len(res0) != len(res1):
            raise FhhError("final_values: res0.len() != res1.len() (collect.rs:1008)")
        for r0, r1 in zip(res0, res1):
            if r0.path != r1.path:
                raise FhhError("final_values: paths differ (collect.rs:1012)")
        a = np.array([int_to_limbs(r.value, 10) for r in res0], np.uint32).reshape(-1, 10)
        b = np.array([int_to_limbs(r.value, 10) for r in res1], np.uint32).reshape(-1, 10)
        out = np.zeros((len(res0), 8), np.uint32)
        check(lib().fhh_final_values(ptr(a, u32p), ptr(b, u32p), len(res0), ptr(out, u32p)))
        return [Result(r.path, limbs10_to_int(out[k])) for k, r in enumerate(res0)]


def gen_keys_pair(c0: KeyCollection, c1: KeyCollection, left_bits: np.ndarray, right_bits: np.ndarray,
                  root_seeds: np.ndarray):
    """Leader-side batched interval keygen on the GPU (ibDCF.rs:84-188), server 0's keys into
    c0 and server 1's into c1."""
    n, d, L = left_bits.shape
    if right_bits.shape != (n, d, L) or root_seeds.shape != (n, d, 2, 2, 16):
        raise FhhError("gen_keys_pair: shape mismatch")
    lb = np.ascontiguousarray(left_bits, np.uint8)
    rb = np.ascontiguousarray(right_bits, np.uint8)
    rs = np.ascontiguousarray(root_seeds, np.uint8)
    check(lib().fhh_gen_keys_pair(c0.handle, c1.handle, n, ptr(lb), ptr(rb), ptr(rs)), c0.handle)


def sim_eq_count(c0: KeyCollection, c1: KeyCollection, C: int) -> np.ndarray:
    out = np.zeros(C, np.uint64)
    check(lib().fhh_sim_eq_count(c0.handle, c1.handle, ptr(out, u64p)), c0.handle)
    return out


def sim_ot_sums(c0: KeyCollection, c1: KeyCollection, C: int, prf_seed: int, last: bool):
    if last:
        a = np.zeros((C, 10), np.uint32)
        b = np.zeros((C, 10), np.uint32)
        check(lib().fhh_sim_ot_sums(c0.handle, c1.handle, prf_seed, a.ctypes.data, b.ctypes.data), c0.handle)
        return [limbs10_to_int(r) for r in a], [limbs10_to_int(r) for r in b]
    a = np.zeros(C, np.uint64)
    b = np.zeros(C, np.uint64)
    check(lib().fhh_sim_ot_sums(c0.handle, c1.handle, prf_seed, a.ctypes.data, b.ctypes.data), c0.handle)
    return [int(x) for x in a], [int(x) for x in b]


__all__ = ["KeyCollection", "Result", "gen_keys_pair", "sim_eq_count", "sim_ot_sums", "FE_P", "FE255_P"]
