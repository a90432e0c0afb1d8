"""Python mirror of the reference's sketch verification:
`SketchDPFKey::sketch_at` (src/sketch.rs:157-200) and `MulState` (src/mpc.rs:83-220), for
T = FE, backed by the HIP kernels in libfhh.so (fhh_sketch.hip). Both reference files are fully
commented out; the restatement follows the commented text (parity unpinned beyond the
protocol's identities).

The functions take a KeyCollection (the ctx that owns the GPU/stream), like the reference's
methods on the server's collection, and host numpy arrays; `sim_sketch_verify` is the
device-resident in-process leader + two servers (main.rs:14-70 verify_sketches).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ._lib import FhhSketchBatch, check, lib, ptr, u64p
from .fields import FE_P

u8p = ctypes.POINTER(ctypes.c_uint8)


def _u64(a):
    return np.ascontiguousarray(a, dtype=np.uint64)


def sketch_at(kc, seeds: np.ndarray, x: np.ndarray, kx: np.ndarray) -> np.ndarray:
    """sketch_at for n keys: seeds [n][16] (each key's rand_stream = PrgSeed::to_rng),
    x / kx [n][nodes] FE. Returns [n][6] canonical {r_x, r2_x, r_kx, rand1, rand2, rand3}."""
    seeds = np.ascontiguousarray(seeds, dtype=np.uint8)
    x, kx = _u64(x), _u64(kx)
    n = seeds.shape[0]
    nodes = x.shape[1] if x.ndim == 2 else 0
    if seeds.shape != (n, 16) or x.shape != (n, nodes) or kx.shape != x.shape:
        raise ValueError("sketch_at: shapes seeds [n][16], x / kx [n][nodes]")
    out = np.zeros((n, 6), np.uint64)
    check(lib().fhh_sketch_at_fe(kc.handle, n, nodes, ptr(seeds, u8p), ptr(x, u64p), ptr(kx, u64p),
                                 ptr(out, u64p)), kc.handle)
    return out


def mul_cor_share(kc, sketch6, mac_key, mac_key2, triples9) -> np.ndarray:
    """MulState::new + cor_share (mpc.rs:83-158): [n][6] = {d0, d1, d2, e0, e1, e2}."""
    sk, m, m2, tr = _u64(sketch6), _u64(mac_key), _u64(mac_key2), _u64(triples9)
    n = sk.shape[0]
    out = np.zeros((n, 6), np.uint64)
    check(lib().fhh_mul_cor_share_fe(kc.handle, n, ptr(sk, u64p), ptr(m, u64p), ptr(m2, u64p), ptr(tr, u64p),
                                     ptr(out, u64p)), kc.handle)
    return out


def mul_cor(share0, share1) -> np.ndarray:
    """MulState::cor (mpc.rs:160-180)."""
    s0, s1 = _u64(share0), _u64(share1)
    out = np.zeros_like(s0)
    check(lib().fhh_mul_cor_fe(s0.shape[0], ptr(s0, u64p), ptr(s1, u64p), ptr(out, u64p)))
    return out


def mul_out_share(kc, server_idx: bool, sketch6, mac_key, mac_key2, triples9, cor6) -> np.ndarray:
    """MulState::out_share (mpc.rs:182-212)."""
    sk, m, m2, tr, c = _u64(sketch6), _u64(mac_key), _u64(mac_key2), _u64(triples9), _u64(cor6)
    n = sk.shape[0]
    out = np.zeros(n, np.uint64)
    check(lib().fhh_mul_out_share_fe(kc.handle, int(bool(server_idx)), n, ptr(sk, u64p), ptr(m, u64p), ptr(m2, u64p),
                                     ptr(tr, u64p), ptr(c, u64p), ptr(out, u64p)), kc.handle)
    return out


def mul_verify(out0, out1) -> np.ndarray:
    """MulState::verify (mpc.rs:214-220): out0 + out1 == 0."""
    o0, o1 = _u64(out0), _u64(out1)
    ok = np.zeros(o0.shape[0], np.uint8)
    check(lib().fhh_mul_verify_fe(o0.shape[0], ptr(o0, u64p), ptr(o1, u64p), ptr(ok, u8p)))
    return ok.astype(bool)


# ---- synthetic workload (config E: sketch_batch_size keys x frontier nodes) ------------------
def _splitmix(state: np.ndarray) -> np.ndarray:
    z = (state + np.uint64(0x9E3779B97F4A7C15)).astype(np.uint64)
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)).astype(np.uint64)
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)).astype(np.uint64)
    return z ^ (z >> np.uint64(31))


def _rand_fe(seed: int, shape) -> np.ndarray:
    """uniform canonical FE values from a counter-based SplitMix64 stream"""
    n = int(np.prod(shape))
    ctr = np.arange(n, dtype=np.uint64) + np.uint64((seed * 0x632BE59BD9B4E019) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        v = _splitmix(ctr) & np.uint64((1 << 62) - 1)
    v = np.where(v >= np.uint64(FE_P), v - np.uint64(FE_P), v)
    return v.reshape(shape)


def _sub_fe(a, b):
    return np.where(a >= b, a - b, a + (np.uint64(FE_P) - b)).astype(np.uint64)


def _share(v: np.ndarray, seed: int):
    """Share::share (lib.rs:42-49): s0 random, s1 = v - s0."""
    s0 = _rand_fe(seed, v.shape)
    return s0, _sub_fe(v, s0)


def _mul_fe(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    return np.array([(int(p) * int(q)) % FE_P for p, q in zip(a.ravel(), b.ravel())], np.uint64).reshape(a.shape)


@dataclass
class SketchWorkload:
    """Both servers' inputs for one level of sketch verification (SketchDPFKey::gen,
    sketch.rs:84-150, with the DPF outputs replaced by their defining property): key i's
    vector is the one-hot e_{alpha_i} over the frontier (or zero), its MAC vector k_i * x."""
    seeds: np.ndarray           # [n][16]
    x: list                     # per server [n][nodes]
    kx: list
    mac: list                   # per server [n]
    mac2: list
    triples: list               # per server [n][9]
    honest: np.ndarray          # [n] bool: the vector is well formed


def sketch_workload(n_keys: int, n_nodes: int, seed: int = 0x5EED, bad_fraction: float = 0.0) -> SketchWorkload:
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, size=(n_keys, 16), dtype=np.uint8)
    alpha = rng.integers(0, max(n_nodes, 1), size=n_keys)
    k = _rand_fe(seed + 1, (n_keys,))
    k2 = _mul_fe(k, k)
    xv = np.zeros((n_keys, n_nodes), np.uint64)
    if n_nodes:
        xv[np.arange(n_keys), alpha] = 1
    honest = np.ones(n_keys, bool)
    nbad = int(round(bad_fraction * n_keys))
    if nbad and n_nodes > 1:
        bad = rng.choice(n_keys, size=nbad, replace=False)
        # malformed: weight 2 at one node (breaks <r,x>^2 = <r^2,x>)
        xv[bad, alpha[bad]] = 2
        honest[bad] = False
    # k * x with x in {0, 1, 2}: no wide multiply needed
    kxv = np.where(xv == 0, np.uint64(0), np.where(xv == 1, k[:, None], (k[:, None] * np.uint64(2)) % np.uint64(FE_P)))
    kxv = kxv.astype(np.uint64)
    x0, x1 = _share(xv, seed + 2)
    kx0, kx1 = _share(kxv, seed + 3)
    m0, m1 = _share(k, seed + 4)
    q0, q1 = _share(k2, seed + 5)
    # TripleShare::new (mpc.rs:18-45): a, b shared at random, c = a * b shared
    a0, a1 = _rand_fe(seed + 6, (n_keys, 3)), _rand_fe(seed + 7, (n_keys, 3))
    b0, b1 = _rand_fe(seed + 8, (n_keys, 3)), _rand_fe(seed + 9, (n_keys, 3))
    a = (a0 + a1) % np.uint64(FE_P)
    b = (b0 + b1) % np.uint64(FE_P)
    c = _mul_fe(a, b)
    c0, c1 = _share(c, seed + 10)
    t0 = np.stack([a0, b0, c0], axis=2).reshape(n_keys, 9)
    t1 = np.stack([a1, b1, c1], axis=2).reshape(n_keys, 9)
    return SketchWorkload(seeds, [x0, x1], [kx0, kx1], [m0, m1], [q0, q1], [t0, t1], honest)


class DeviceSketchBatch:
    """A SketchWorkload resident in HBM (torch tensors on the ctx's GPU) for
    `sim_sketch_verify`."""

    def __init__(self, wl: SketchWorkload, device: int = 0):
        import torch
        dev = torch.device(f"cuda:{device}")

        def t(a):
            return torch.from_numpy(np.ascontiguousarray(a).view(np.int64)).to(dev)

        self.n_keys, self.n_nodes = wl.x[0].shape
        self.seeds = torch.from_numpy(np.ascontiguousarray(wl.seeds)).to(dev)
        self.x = [t(v) for v in wl.x]
        self.kx = [t(v) for v in wl.kx]
        self.mac = [t(v) for v in wl.mac]
        self.mac2 = [t(v) for v in wl.mac2]
        self.triples = [t(v) for v in wl.triples]
        self.sketch = [torch.zeros((self.n_keys, 6), dtype=torch.int64, device=dev) for _ in range(2)]
        self.ok = torch.zeros(self.n_keys, dtype=torch.uint8, device=dev)
        self.out_shares = torch.zeros((2, self.n_keys), dtype=torch.int64, device=dev)

    def struct(self, force_sequential: bool = False) -> FhhSketchBatch:
        b = FhhSketchBatch()
        b.n_keys = self.n_keys
        b.n_nodes = self.n_nodes
        b.force_sequential = int(force_sequential)
        b.seeds_dev = self.seeds.data_ptr()
        for s in range(2):
            b.x_dev[s] = self.x[s].data_ptr()
            b.kx_dev[s] = self.kx[s].data_ptr()
            b.mac_dev[s] = self.mac[s].data_ptr()
            b.mac2_dev[s] = self.mac2[s].data_ptr()
            b.triples_dev[s] = self.triples[s].data_ptr()
            b.sketch_dev[s] = self.sketch[s].data_ptr()
        b.ok_dev = self.ok.data_ptr()
        b.out_shares_dev = self.out_shares.data_ptr()
        return b


def sim_sketch_verify(kc, batch: DeviceSketchBatch, force_sequential: bool = False) -> None:
    """Both servers' sketch_at + MulState cor/out shares + verify, on the GPU (main.rs:14-70)."""
    b = batch.struct(force_sequential)
    check(lib().fhh_sim_sketch_verify_fe(kc.handle, ctypes.byref(b)), kc.handle)
