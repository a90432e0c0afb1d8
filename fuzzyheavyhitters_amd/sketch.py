"""Python mirror of the reference's sketch verification:
`SketchDPFKey::sketch_at` (src/sketch.rs:157-200) and `MulState` (src/mpc.rs:83-220) for
T = FE, and `sketch_at_last` (sketch.rs:202-245) with `MulState<FieldElm>` for the last level
(U = FieldElm, values as 8 x u32 little-endian limbs), backed by the HIP kernels in libfhh.so
(fhh_sketch.hip). Both reference files are fully commented out; the restatement follows the
commented text (parity unpinned beyond the protocol's identities).

The functions take a KeyCollection (the ctx that owns the GPU/stream), like the reference's
methods on the server's collection, and host numpy arrays; `sim_sketch_verify` is the
device-resident in-process leader + two servers (main.rs:14-70 verify_sketches).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ._lib import FhhError, FhhSketchBatch, FhhSketchBatch255, check, lib, ptr, u32p, u64p
from .fields import FE255_P, FE_P

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
        self.triples_levels = getattr(wl, "triples_levels", 0)
        levels = max(1, self.triples_levels)
        self.sketch = [torch.zeros((self.n_keys, 6), dtype=torch.int64, device=dev) for _ in range(2)]
        self.ok = torch.zeros((levels, self.n_keys), dtype=torch.uint8, device=dev)
        self.out_shares = torch.zeros((levels, 2, self.n_keys), dtype=torch.int64, device=dev)
        # the library runs on its own stream: torch's fills and copies must be complete first
        torch.cuda.synchronize(dev)

    def struct(self, force_sequential: bool = False, level: int = 0, n_levels: int = 1) -> FhhSketchBatch:
        b = FhhSketchBatch()
        b.n_keys = self.n_keys
        b.n_nodes = self.n_nodes
        b.force_sequential = int(force_sequential)
        b.level = level
        b.n_levels = n_levels
        b.triples_levels = self.triples_levels
        b.x_level_stride = 0
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


def deal_triples(kc, batch: DeviceSketchBatch, levels: int, seed: int = 0x7121) -> None:
    """Replace the batch's triples by `levels` per-level sets dealt on the GPU (fhh_deal_triples_fe:
    TripleShare::new for every key x level x 3), so level l verifies with triples[l] as
    MulState::new takes them (mpc.rs:94-98)."""
    import torch
    dev = batch.mac[0].device
    batch.triples = [torch.zeros((batch.n_keys, levels, 9), dtype=torch.int64, device=dev) for _ in range(2)]
    batch.triples_levels = levels
    batch.ok = torch.zeros((levels, batch.n_keys), dtype=torch.uint8, device=dev)
    batch.out_shares = torch.zeros((levels, 2, batch.n_keys), dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)   # torch's zero fills run on its stream; the dealer on the ctx's
    check(lib().fhh_deal_triples_fe(kc.handle, batch.n_keys, levels, seed, batch.triples[0].data_ptr(),
                                    batch.triples[1].data_ptr()), kc.handle)


def sim_sketch_verify(kc, batch: DeviceSketchBatch, force_sequential: bool = False, level: int = 0,
                      n_levels: int = 1) -> None:
    """Both servers' sketch_at + MulState cor/out shares + verify, on the GPU (main.rs:14-70), for
    levels [level, level + n_levels): level l's stream seed is the key's seed with bytes 12..15
    ^= l, its triples are triples[l] (batch.triples_levels > 0); ok / out_shares per level."""
    if n_levels < 1 or n_levels > batch.ok.shape[0]:
        raise FhhError(f"sim_sketch_verify: n_levels {n_levels} outside [1, {batch.ok.shape[0]}] "
                       "(levels beyond the first need per-level triples: deal_triples)")
    b = batch.struct(force_sequential, level, n_levels)
    check(lib().fhh_sim_sketch_verify_fe(kc.handle, ctypes.byref(b)), kc.handle)


# ---- U = FieldElm: the last level (sketch_at_last, MulState<FieldElm>) -----------------------
_P255_LIMBS = np.array([(FE255_P >> (32 * k)) & 0xFFFFFFFF for k in range(8)], np.int64)


def int_to_fe8(v: int) -> np.ndarray:
    return np.array([(v >> (32 * k)) & 0xFFFFFFFF for k in range(8)], np.uint32)


def fe8_to_int(a) -> int:
    return sum(int(x) << (32 * k) for k, x in enumerate(np.asarray(a).ravel()))


def _u32(a):
    return np.ascontiguousarray(a, dtype=np.uint32)


def sketch_at_fe255(kc, seeds: np.ndarray, x: np.ndarray, kx: np.ndarray) -> np.ndarray:
    """sketch_at_last for n keys: x / kx [n][nodes][8] -> [n][6][8] canonical."""
    seeds = np.ascontiguousarray(seeds, dtype=np.uint8)
    x, kx = _u32(x), _u32(kx)
    n, F = x.shape[:2]
    if seeds.shape != (n, 16) or x.shape != (n, F, 8) or kx.shape != x.shape:
        raise ValueError("sketch_at_fe255: shapes seeds [n][16], x / kx [n][nodes][8]")
    out = np.zeros((n, 6, 8), np.uint32)
    check(lib().fhh_sketch_at_fe255(kc.handle, n, F, ptr(seeds, u8p), ptr(x, u32p), ptr(kx, u32p),
                                    ptr(out, u32p)), kc.handle)
    return out


def mul_cor_share_fe255(kc, sketch6, mac_key, mac_key2, triples9) -> np.ndarray:
    sk, m, m2, tr = _u32(sketch6), _u32(mac_key), _u32(mac_key2), _u32(triples9)
    n = sk.shape[0]
    out = np.zeros((n, 6, 8), np.uint32)
    check(lib().fhh_mul_cor_share_fe255(kc.handle, n, ptr(sk, u32p), ptr(m, u32p), ptr(m2, u32p), ptr(tr, u32p),
                                        ptr(out, u32p)), kc.handle)
    return out


def mul_cor_fe255(share0, share1) -> np.ndarray:
    s0, s1 = _u32(share0), _u32(share1)
    out = np.zeros_like(s0)
    check(lib().fhh_mul_cor_fe255(s0.shape[0], ptr(s0, u32p), ptr(s1, u32p), ptr(out, u32p)))
    return out


def mul_out_share_fe255(kc, server_idx: bool, sketch6, mac_key, mac_key2, triples9, cor6) -> np.ndarray:
    sk, m, m2, tr, c = _u32(sketch6), _u32(mac_key), _u32(mac_key2), _u32(triples9), _u32(cor6)
    n = sk.shape[0]
    out = np.zeros((n, 8), np.uint32)
    check(lib().fhh_mul_out_share_fe255(kc.handle, int(bool(server_idx)), n, ptr(sk, u32p), ptr(m, u32p),
                                        ptr(m2, u32p), ptr(tr, u32p), ptr(c, u32p), ptr(out, u32p)), kc.handle)
    return out


def mul_verify_fe255(out0, out1) -> np.ndarray:
    o0, o1 = _u32(out0), _u32(out1)
    ok = np.zeros(o0.shape[0], np.uint8)
    check(lib().fhh_mul_verify_fe255(o0.shape[0], ptr(o0, u32p), ptr(o1, u32p), ptr(ok, u8p)))
    return ok.astype(bool)


def _rand_fe8(seed: int, shape) -> np.ndarray:
    """uniform values < 2^254 (< p) as [..., 8] u32 limbs, counter-based SplitMix64"""
    n = int(np.prod(shape)) * 4
    ctr = np.arange(n, dtype=np.uint64) + np.uint64((seed * 0x9E3779B97F4A7C15 + 0x1234567) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        w = _splitmix(ctr).view(np.uint32).reshape(*shape, 8).copy()
    w[..., 7] &= 0x3FFFFFFF
    return w


def _sub_fe8(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """(a - b) mod p on canonical [..., 8] limbs, vectorised"""
    a64, b64 = a.astype(np.int64), b.astype(np.int64)
    out = np.empty_like(a64)
    borrow = np.zeros(a.shape[:-1], np.int64)
    for k in range(8):
        v = a64[..., k] - b64[..., k] - borrow
        borrow = (v < 0).astype(np.int64)
        out[..., k] = v + (borrow << 32)
    carry = np.zeros_like(borrow)
    for k in range(8):   # a - b < 0: add p (the wrap past 2^256 drops out)
        v = out[..., k] + borrow * _P255_LIMBS[k] + carry
        carry = v >> 32
        out[..., k] = v & 0xFFFFFFFF
    return out.astype(np.uint32)


def _share_fe8(v: np.ndarray, seed: int):
    s0 = _rand_fe8(seed, v.shape[:-1])
    return s0, _sub_fe8(v, s0)


def _neg_fe8_fast(a: np.ndarray) -> np.ndarray:
    """p - a for 0 < a < 2^254, vectorised without carries: p - a = (2^255 - 1 - a) - 18, and
    2^255 - 1 - a is the bitwise NOT of a's 255 bits; the -18 borrows past limb 0 only when
    limb 0 < 18 (about 4e-9 per value), fixed up elementwise."""
    out = ~a
    out[..., 7] &= 0x7FFFFFFF
    low = out[..., 0]
    rare = low < 18
    out[..., 0] = low - np.uint32(18)
    if rare.any():
        for idx in zip(*np.nonzero(rare)):
            v = (FE255_P - fe8_to_int(a[idx])) % FE255_P
            out[idx] = int_to_fe8(v)
    return out


def _share_sparse_fe8(shape, idx, vals: np.ndarray, seed: int):
    """Shares of a vector that is zero except vals [m][8] at positions idx (a tuple of index
    arrays into shape): s0 random, s1 = v - s0 = -s0 (+ v at idx)."""
    s0 = _rand_fe8(seed, shape)
    s0[s0[..., 0] == 0, 0] = 1            # nonzero, so -s0 = p - s0 < p (the fast negation)
    s1 = _neg_fe8_fast(s0)
    if len(idx[0]):
        s1[idx] = _add_fe8(s1[idx], vals)
    return s0, s1


def _add_fe8(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """(a + b) mod p on canonical [..., 8] limbs, vectorised"""
    a64, b64 = a.astype(np.int64), b.astype(np.int64)
    out = np.empty_like(a64)
    carry = np.zeros(a.shape[:-1], np.int64)
    for k in range(8):
        v = a64[..., k] + b64[..., k] + carry
        carry = v >> 32
        out[..., k] = v & 0xFFFFFFFF
    # subtract p once where out >= p
    ge = np.ones(a.shape[:-1], bool)
    eq = np.ones(a.shape[:-1], bool)
    for k in range(7, -1, -1):
        gt_k = out[..., k] > _P255_LIMBS[k]
        lt_k = out[..., k] < _P255_LIMBS[k]
        ge = np.where(eq & gt_k, True, np.where(eq & lt_k, False, ge))
        eq &= out[..., k] == _P255_LIMBS[k]
    borrow = np.zeros_like(carry)
    for k in range(8):
        v = out[..., k] - ge * _P255_LIMBS[k] - borrow
        borrow = (v < 0).astype(np.int64)
        out[..., k] = v + (borrow << 32)
    return out.astype(np.uint32)


@dataclass
class SketchWorkload255:
    """Both servers' inputs of the last level's check (U = FieldElm): one-hot vector e_alpha (or
    weight 2 at alpha for a malformed key) over the frontier, its MAC k_last * x, shares of
    mac_key_last / mac_key2_last and the 3 triples_last (sketch.rs:80-149 shape)."""
    seeds: np.ndarray           # [n][16]
    x: list                     # per server [n][nodes][8]
    kx: list
    mac: list                   # per server [n][8]
    mac2: list
    triples: list               # per server [n][9][8]
    honest: np.ndarray


def sketch_workload255(n_keys: int, n_nodes: int, seed: int = 0x5EED, bad_fraction: float = 0.0) -> SketchWorkload255:
    rng = np.random.default_rng([seed, 255])
    seeds = rng.integers(0, 256, size=(n_keys, 16), dtype=np.uint8)
    alpha = rng.integers(0, max(n_nodes, 1), size=n_keys)
    k = _rand_fe8(seed + 1, (n_keys,))
    kint = [fe8_to_int(k[i]) for i in range(n_keys)]
    k2 = np.stack([int_to_fe8(v * v % FE255_P) for v in kint]) if n_keys else np.zeros((0, 8), np.uint32)
    honest = np.ones(n_keys, bool)
    weight = np.ones(n_keys, np.int64)
    nbad = int(round(bad_fraction * n_keys))
    if nbad and n_nodes > 1:
        bad = rng.choice(n_keys, size=nbad, replace=False)
        weight[bad] = 2            # breaks <r,x>^2 = <r^2,x>
        honest[bad] = False
    pos = (np.arange(n_keys), alpha) if n_nodes else (np.zeros(0, np.int64), np.zeros(0, np.int64))
    xw = np.zeros((len(pos[0]), 8), np.uint32)
    xw[:, 0] = weight[: len(pos[0])].astype(np.uint32)
    kxw = (np.stack([int_to_fe8(kint[i] * int(weight[i]) % FE255_P) for i in range(n_keys)])
           if n_keys and n_nodes else np.zeros((0, 8), np.uint32))
    x0, x1 = _share_sparse_fe8((n_keys, n_nodes), pos, xw, seed + 2)
    kx0, kx1 = _share_sparse_fe8((n_keys, n_nodes), pos, kxw, seed + 3)
    m0, m1 = _share_fe8(k, seed + 4)
    q0, q1 = _share_fe8(k2, seed + 5)
    # TripleShare::new (mpc.rs:18-45): a, b shared at random, c = a * b shared
    a0, a1 = _rand_fe8(seed + 6, (n_keys, 3)), _rand_fe8(seed + 7, (n_keys, 3))
    b0, b1 = _rand_fe8(seed + 8, (n_keys, 3)), _rand_fe8(seed + 9, (n_keys, 3))
    c = np.zeros((n_keys, 3, 8), np.uint32)
    for i in range(n_keys):
        for t in range(3):
            av = (fe8_to_int(a0[i, t]) + fe8_to_int(a1[i, t])) % FE255_P
            bv = (fe8_to_int(b0[i, t]) + fe8_to_int(b1[i, t])) % FE255_P
            c[i, t] = int_to_fe8(av * bv % FE255_P)
    c0, c1 = _share_fe8(c, seed + 10)
    t0 = np.stack([a0, b0, c0], axis=2).reshape(n_keys, 9, 8)
    t1 = np.stack([a1, b1, c1], axis=2).reshape(n_keys, 9, 8)
    return SketchWorkload255(seeds, [x0, x1], [kx0, kx1], [m0, m1], [q0, q1], [t0, t1], honest)


class DeviceSketchBatch255:
    """A SketchWorkload255 resident in HBM for `sim_sketch_verify_fe255`."""

    def __init__(self, wl: SketchWorkload255, device: int = 0):
        import torch
        dev = torch.device(f"cuda:{device}")

        def t(a):
            return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).to(dev)

        self.n_keys, self.n_nodes = wl.x[0].shape[:2]
        self.seeds = torch.from_numpy(np.ascontiguousarray(wl.seeds)).to(dev)
        self.x = [t(v) for v in wl.x]
        self.kx = [t(v) for v in wl.kx]
        self.mac = [t(v) for v in wl.mac]
        self.mac2 = [t(v) for v in wl.mac2]
        self.triples = [t(v) for v in wl.triples]
        self.sketch = [torch.zeros((self.n_keys, 6, 8), dtype=torch.int32, device=dev) for _ in range(2)]
        self.ok = torch.zeros(self.n_keys, dtype=torch.uint8, device=dev)
        self.out_shares = torch.zeros((2, self.n_keys, 8), dtype=torch.int32, device=dev)
        torch.cuda.synchronize(dev)

    def struct(self, force_sequential: bool = False, level: int = 0) -> FhhSketchBatch255:
        b = FhhSketchBatch255()
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
        b.level = level
        return b


def sim_sketch_verify_fe255(kc, batch: DeviceSketchBatch255, force_sequential: bool = False, level: int = 0) -> None:
    """The last level's check (U = FieldElm), both servers, on the GPU."""
    b = batch.struct(force_sequential, level)
    check(lib().fhh_sim_sketch_verify_fe255(kc.handle, ctypes.byref(b)), kc.handle)
