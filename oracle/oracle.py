"""ORACLE — TEST INFRASTRUCTURE ONLY.

Python side of the CPU restatement of sks-codes/fuzzyheavyhitters' per-level client-key
evaluation (reference: Rust crate `counttree`, /root/reference, not compilable here).
Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import
this module; the product package never does.

Parity anchors (see tests/test_oracle_kat.py):
  * AES-128: FIPS-197 appendix C.1 vector + zero-key vector, and OpenSSL ``AES_encrypt``.
  * FE (fastfield.rs): the reference's own known answers (fastfield.rs:459-559).
  * ibDCF: comparison semantics derived from ibDCF.rs:84-119,208-227, checked exhaustively.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

u8p = ctypes.POINTER(ctypes.c_uint8)
u64p = ctypes.POINTER(ctypes.c_uint64)


def build() -> str:
    """Compile liboracle.so (Makefile in this directory)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return os.path.join(_HERE, "liboracle.so")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.orc_level_expand.restype = ctypes.c_uint64
        L.orc_fe_new.restype = ctypes.c_uint64
        L.orc_fe_new.argtypes = [ctypes.c_uint64]
        L.orc_fe_value.restype = ctypes.c_uint64
        L.orc_fe_value.argtypes = [ctypes.c_uint64]
        for nm in ("orc_fe_add", "orc_fe_sub", "orc_fe_mul"):
            getattr(L, nm).restype = ctypes.c_uint64
            getattr(L, nm).argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.orc_fe_neg.restype = ctypes.c_uint64
        L.orc_fe_neg.argtypes = [ctypes.c_uint64]
        L.orc_fe_fold_sum.restype = ctypes.c_uint64
        L.orc_sim_prf.restype = ctypes.c_uint64
        L.orc_sim_prf.argtypes = [ctypes.c_uint64] * 4 + [ctypes.c_uint32]
        L.orc_prg_stream_u64.restype = ctypes.c_uint64
        L.orc_prg_stream_u64.argtypes = [u8p, ctypes.c_uint64]
        L.orc_mul_out_share_fe.restype = ctypes.c_uint64
        L.orc_mul_out_share_fe.argtypes = [ctypes.c_int, u64p, ctypes.c_uint64, ctypes.c_uint64, u64p, u64p]
        L.orc_mul_verify_fe.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        _LIB = L
    return _LIB


def _p(a: np.ndarray, t=u8p):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(t)


# --------------------------------------------------------------------------------------
# AES / PRG / ibDCF
# --------------------------------------------------------------------------------------

def aes128_encrypt(key: bytes, block: bytes) -> bytes:
    k = np.frombuffer(key, np.uint8).copy()
    i = np.frombuffer(block, np.uint8).copy()
    o = np.zeros(16, np.uint8)
    lib().orc_aes128_encrypt(_p(k), _p(i), _p(o))
    return o.tobytes()


def aes0(block: bytes, ni: bool = False) -> bytes:
    i = np.frombuffer(block, np.uint8).copy()
    o = np.zeros(16, np.uint8)
    (lib().orc_aes128_zero_encrypt_ni if ni else lib().orc_aes128_zero_encrypt)(_p(i), _p(o))
    return o.tobytes()


def aes_ni_available() -> bool:
    return bool(lib().orc_aes_ni_available())


def sbox() -> np.ndarray:
    o = np.zeros(256, np.uint8)
    lib().orc_sbox(_p(o))
    return o


def zero_round_keys() -> np.ndarray:
    o = np.zeros(176, np.uint8)
    lib().orc_zero_round_keys(_p(o))
    return o


def expand_dir(seed: bytes, direction: int):
    """prg.rs:92-122 (as called from eval_bit). Returns (child_seed, (b0,b1,y0,y1))."""
    s = np.frombuffer(seed, np.uint8).copy()
    o = np.zeros(16, np.uint8)
    b = np.zeros(4, np.uint8)
    lib().orc_expand_dir(_p(s), ctypes.c_int(direction), _p(o), _p(b))
    return o.tobytes(), tuple(int(x) for x in b)


def gen_ibdcf(alpha_bits, side: bool, root0: bytes, root1: bytes):
    """ibDCF.rs:138-164. Returns (cw_seed [L][16] u8, cw_bits [L] nibble)."""
    a = np.asarray(alpha_bits, np.uint8).copy()
    L = a.size
    r0 = np.frombuffer(root0, np.uint8).copy()
    r1 = np.frombuffer(root1, np.uint8).copy()
    cs = np.zeros((L, 16), np.uint8)
    cb = np.zeros(L, np.uint8)
    lib().orc_gen_ibdcf(_p(a), ctypes.c_uint32(L), ctypes.c_int(int(side)), _p(r0), _p(r1), _p(cs), _p(cb))
    return cs, cb


def eval_bit(seed: bytes, t: int, y: int, cw_seed: bytes, cw_bits: int, direction: int):
    """ibDCF.rs:208-227."""
    s = np.frombuffer(seed, np.uint8).copy()
    c = np.frombuffer(cw_seed, np.uint8).copy()
    o = np.zeros(16, np.uint8)
    to = ctypes.c_uint8()
    yo = ctypes.c_uint8()
    lib().orc_eval_bit(_p(s), ctypes.c_int(t), ctypes.c_int(y), _p(c), ctypes.c_uint8(cw_bits),
                       ctypes.c_int(direction), _p(o), ctypes.byref(to), ctypes.byref(yo))
    return o.tobytes(), to.value, yo.value


def eval_ibdcf(key_idx: int, root_seed: bytes, cw_seed, cw_bits, idx_bits):
    """ibDCF.rs:238-250: returns y_bit ^ bit after evaluating the prefix idx_bits."""
    seed, t, y = root_seed, key_idx, key_idx
    for lvl, b in enumerate(idx_bits):
        seed, t, y = eval_bit(seed, t, y, bytes(cw_seed[lvl]), int(cw_bits[lvl]), int(b))
    return y ^ t


@dataclass
class ServerKeys:
    """One server's keys, client-major then dim then (left,right) — the order of
    ``add_key(Vec<(ibDCFKey, ibDCFKey)>)`` (collect.rs:62)."""
    key_idx: np.ndarray   # [n][d][2] u8
    root_seed: np.ndarray  # [n][d][2][16] u8
    cw_seed: np.ndarray    # [n][d][2][L][16] u8 (shared by both servers)
    cw_bits: np.ndarray    # [n][d][2][L] u8 nibble

    @property
    def n(self):
        return self.key_idx.shape[0]


def gen_keys(left_bits: np.ndarray, right_bits: np.ndarray, root_seeds: np.ndarray, nthreads: int = 0):
    """Batched ``gen_interval`` per (client, dim) — ibDCF.rs:166-173.

    left_bits/right_bits: [n][d][L] (0/1); root_seeds: [n][d][2 side][2 server][16].
    Returns (ServerKeys server0, ServerKeys server1)."""
    n, d, L = left_bits.shape
    lb = np.ascontiguousarray(left_bits, np.uint8)
    rb = np.ascontiguousarray(right_bits, np.uint8)
    rs = np.ascontiguousarray(root_seeds, np.uint8)
    cws = np.zeros((n, d, 2, L, 16), np.uint8)
    cwb = np.zeros((n, d, 2, L), np.uint8)
    lib().orc_gen_keys(ctypes.c_uint64(n), ctypes.c_uint32(d), ctypes.c_uint32(L), _p(lb), _p(rb), _p(rs),
                       _p(cws), _p(cwb), ctypes.c_int(nthreads))
    k0 = ServerKeys(np.zeros((n, d, 2), np.uint8), np.ascontiguousarray(rs[:, :, :, 0, :]), cws, cwb)
    k1 = ServerKeys(np.ones((n, d, 2), np.uint8), np.ascontiguousarray(rs[:, :, :, 1, :]), cws, cwb)
    return k0, k1


# --------------------------------------------------------------------------------------
# Collection engine restatement (collect.rs), reference order, no dedup.
# --------------------------------------------------------------------------------------

@dataclass
class States:
    seed: np.ndarray  # [F][n][d][2][16]
    t: np.ndarray     # [F][n][d][2]
    y: np.ndarray


def tree_init(keys: ServerKeys) -> States:
    n, d = keys.key_idx.shape[:2]
    seed = np.zeros((1, n, d, 2, 16), np.uint8)
    t = np.zeros((1, n, d, 2), np.uint8)
    y = np.zeros((1, n, d, 2), np.uint8)
    lib().orc_tree_init(ctypes.c_uint64(n), ctypes.c_uint32(d), _p(np.ascontiguousarray(keys.key_idx)),
                        _p(np.ascontiguousarray(keys.root_seed)), _p(seed), _p(t), _p(y))
    return States(seed, t, y)


def level_expand(keys: ServerKeys, st: States, parent_idx, level: int, nthreads: int = 0, use_ni: bool = True):
    """collect.rs:379-391 for one server. Returns (States of F*2^d children, aes_blocks)."""
    n, d, _, L = keys.cw_bits.shape
    pidx = np.ascontiguousarray(np.asarray(parent_idx, np.uint64))
    F = pidx.size
    C = F << d
    out = States(np.zeros((C, n, d, 2, 16), np.uint8), np.zeros((C, n, d, 2), np.uint8),
                 np.zeros((C, n, d, 2), np.uint8))
    blocks = lib().orc_level_expand(
        ctypes.c_uint64(n), ctypes.c_uint32(d), ctypes.c_uint32(L), ctypes.c_uint32(level),
        _p(keys.cw_seed), _p(keys.cw_bits), ctypes.c_uint64(F), _p(pidx, u64p),
        _p(st.seed), _p(st.t), _p(st.y), _p(out.seed), _p(out.t), _p(out.y),
        ctypes.c_int(nthreads), ctypes.c_int(int(use_ni)))
    return out, int(blocks)


def subset_keys(keys: ServerKeys, clients) -> ServerKeys:
    """The keys of a client sample (in the given order)."""
    idx = np.asarray(clients, np.int64)
    return ServerKeys(np.ascontiguousarray(keys.key_idx[idx]), np.ascontiguousarray(keys.root_seed[idx]),
                      np.ascontiguousarray(keys.cw_seed[idx]), np.ascontiguousarray(keys.cw_bits[idx]))


def replay_states(keys0: ServerKeys, keys1: ServerKeys, keeps, want_levels, nthreads: int = 0):
    """The crawl's expansion (collect.rs:379-391) for the clients in keys0/keys1 along a GIVEN
    frontier: level l expands the children kept at level l - 1 (keeps[l - 1], a bool mask over
    that level's children, e.g. from the run under test, decided over all clients). The EvalStates
    of every child depend only on the client's own keys and the child's path, so a client sample
    evaluated on the full run's frontier must reproduce that run's states exactly.
    Returns {level: (States server 0, States server 1)} for the levels in want_levels."""
    want = set(int(x) for x in want_levels)
    out = {}
    s0, s1 = tree_init(keys0), tree_init(keys1)
    parents = np.zeros(1, np.uint64)
    for lv in range(max(want) + 1):
        c0, _ = level_expand(keys0, s0, parents, lv, nthreads)
        c1, _ = level_expand(keys1, s1, parents, lv, nthreads)
        if lv in want:
            out[lv] = (c0, c1)
        if lv < len(keeps):
            parents = np.nonzero(np.asarray(keeps[lv], bool))[0].astype(np.uint64)
        s0, s1 = c0, c1
    return out


def share_bits(st: States) -> np.ndarray:
    """collect.rs:393-418: [C][n][2d], left dims then right dims."""
    e = st.t ^ st.y                       # [C][n][d][2]
    return np.ascontiguousarray(np.concatenate([e[..., 0], e[..., 1]], axis=-1))


def eq_counts(s0: States, s1: States) -> np.ndarray:
    e0 = share_bits(s0)
    e1 = share_bits(s1)
    return np.all(e0 == e1, axis=-1).sum(axis=1).astype(np.uint64)


# --------------------------------------------------------------------------------------
# Fields (fastfield.rs / field.rs) — exact Python-int restatements.
# --------------------------------------------------------------------------------------
FE_P = (1 << 62) - (1 << 30) - 1           # fastfield.rs:24-28
FE255_P = (1 << 255) - 19                  # field.rs:19 (MODULUS_STR)
FE_MASK = (1 << 62) - 1


def fe_new(v: int) -> int:                 # internal (bit-reduced-once) val
    return int(lib().orc_fe_new(v & ((1 << 64) - 1)))


def fe_value(val: int) -> int:
    return int(lib().orc_fe_value(val))


def fe_fold_sum(vals: np.ndarray) -> int:
    """collect.rs:487-501 with FE add_lazy (field.rs:219-222): internal val."""
    v = np.ascontiguousarray(vals, np.uint64)
    return int(lib().orc_fe_fold_sum(_p(v, u64p), ctypes.c_uint64(v.size)))


def _mix64(z):
    z = (z + np.uint64(0x9E3779B97F4A7C15))
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def sim_prf(seed: int, level: int, child, client, word: int):
    """Harness-defined PRF for simulated OT shares (vectorised over child/client)."""
    with np.errstate(over="ignore"):
        a = _mix64(np.uint64(seed) ^ np.uint64(level))
        b = _mix64(a ^ np.asarray(child, np.uint64))
        c = _mix64(b ^ np.asarray(client, np.uint64))
        return _mix64(c ^ np.uint64(word))


def sim_r0_fe(seed: int, level: int, C: int, n: int) -> np.ndarray:
    """r0 per (child, client), canonical FE: prf & (2^62-1), minus p if >= p."""
    ch = np.arange(C, dtype=np.uint64)[:, None]
    cl = np.arange(n, dtype=np.uint64)[None, :]
    r = sim_prf(seed, level, ch, cl, 0) & np.uint64(FE_MASK)
    return np.where(r >= np.uint64(FE_P), r - np.uint64(FE_P), r)


def sim_r0_fe255(seed: int, level: int, C: int, n: int):
    """r0 per (child, client) as Python ints < p255 (4 prf words, LE, masked to 255 bits)."""
    ch = np.arange(C, dtype=np.uint64)[:, None]
    cl = np.arange(n, dtype=np.uint64)[None, :]
    words = [sim_prf(seed, level, ch, cl, w) for w in range(4)]
    out = np.empty((C, n), dtype=object)
    for c in range(C):
        for i in range(n):
            v = sum(int(words[w][c, i]) << (64 * w) for w in range(4)) & ((1 << 255) - 1)
            out[c, i] = v - FE255_P if v >= FE255_P else v
    return out


def sim_ot_sums_fe(eq: np.ndarray, seed: int, level: int):
    """Server sums of simulated OT outputs (collect.rs:439-501): v0 = r1 = r0+1,
    v1 = r0 if eq else r1. Returns canonical (sum0, sum1) per child."""
    C, n = eq.shape
    r0 = sim_r0_fe(seed, level, C, n)
    s0, s1 = [], []
    for c in range(C):
        r0c = [int(x) for x in r0[c]]
        r1c = [(x + 1) % FE_P for x in r0c]
        s0.append(sum(r1c) % FE_P)
        s1.append(sum(r0c[i] if eq[c, i] else r1c[i] for i in range(n)) % FE_P)
    return s0, s1


def sim_ot_sums_fe255(eq: np.ndarray, seed: int, level: int):
    """As sim_ot_sums_fe for FieldElm; returns the UNREDUCED sums (add_lazy, field.rs:337-339)."""
    C, n = eq.shape
    r0 = sim_r0_fe255(seed, level, C, n)
    s0, s1 = [], []
    for c in range(C):
        r0c = list(r0[c])
        r1c = [(x + 1) % FE255_P for x in r0c]
        s0.append(sum(r1c))
        s1.append(sum(r0c[i] if eq[c, i] else r1c[i] for i in range(n)))
    return s0, s1


def keep_values(threshold: int, v0, v1, p=FE_P):
    """collect.rs:945-964 / 966-989: v = v0 - v1 mod p, keep iff v >= threshold."""
    return [((a % p) - (b % p)) % p >= threshold for a, b in zip(v0, v1)]


# --------------------------------------------------------------------------------------
# In-process two-server crawl (leader.rs:417-440 level loop), GC/OT replaced by plaintext
# equality (mode "count") or simulated OT shares (mode "fe").
# --------------------------------------------------------------------------------------

@dataclass
class CrawlResult:
    n_children: list = field(default_factory=list)  # per level
    counts: list = field(default_factory=list)      # per level: np.ndarray[C]
    keeps: list = field(default_factory=list)       # per level: np.ndarray[C] bool
    sums: list = field(default_factory=list)        # per level (fe mode): (s0, s1)
    final_paths: list = field(default_factory=list)  # [(tuple of d bit-tuples)]
    final_values: list = field(default_factory=list)
    aes_blocks: int = 0
    states0: list = field(default_factory=list)     # optional: per level States
    states1: list = field(default_factory=list)
    level_states: dict = field(default_factory=dict)   # keep_levels: level -> (States0, States1)


def thresholds(frac: float, nclients: int):
    """leader.rs:193-194 (FE, u64) and leader.rs:245-246 (FieldElm, u32)."""
    t = max(1, int(frac * nclients))
    tl = max(1, int(frac * nclients) & 0xFFFFFFFF)
    return t, tl


def crawl(keys0: ServerKeys, keys1: ServerKeys, threshold: float, mode: str = "count", sim_seed: int = 0,
          nthreads: int = 0, keep_states: bool = False, levels: int | None = None,
          max_seconds: float | None = None, keep_levels=None) -> CrawlResult:
    """max_seconds bounds the run (CPU-baseline sampling): stops after the level that
    crosses it; res.n_children then covers only the levels done. keep_levels: record the
    children's States only at these levels (res.level_states[level] = (States0, States1))."""
    keep_set = set(int(x) for x in keep_levels) if keep_levels is not None else set()
    import time
    t_start = time.perf_counter()
    n, d, _, L = keys0.cw_bits.shape
    if levels is None:
        levels = L
    thr, thr_last = thresholds(threshold, n)
    res = CrawlResult()
    s0, s1 = tree_init(keys0), tree_init(keys1)
    parents = np.zeros(1, np.uint64)
    paths = [tuple(() for _ in range(d))]
    for level in range(levels):
        last = level == levels - 1
        c0, b0 = level_expand(keys0, s0, parents, level, nthreads)
        c1, b1 = level_expand(keys1, s1, parents, level, nthreads)
        res.aes_blocks += b0 + b1
        C = c0.t.shape[0]
        eqm = np.all(share_bits(c0) == share_bits(c1), axis=-1)   # [C][n]
        counts = eqm.sum(axis=1).astype(np.uint64)
        if mode == "count":
            keep = counts >= (thr_last if last else thr)
            vals = [int(x) for x in counts]
        elif mode == "fe":
            if last:
                sv0, sv1 = sim_ot_sums_fe255(eqm, sim_seed, level)
                keep = np.array(keep_values(thr_last, sv0, sv1, FE255_P), bool)
                vals = [((a % FE255_P) - (b % FE255_P)) % FE255_P for a, b in zip(sv0, sv1)]
            else:
                sv0, sv1 = sim_ot_sums_fe(eqm, sim_seed, level)
                keep = np.array(keep_values(thr, sv0, sv1, FE_P), bool)
                vals = [(a - b) % FE_P for a, b in zip(sv0, sv1)]
            res.sums.append((sv0, sv1))
        else:
            raise ValueError(mode)
        res.n_children.append(C)
        res.counts.append(counts)
        res.keeps.append(np.asarray(keep, bool))
        if keep_states:
            res.states0.append(c0)
            res.states1.append(c1)
        if level in keep_set:
            res.level_states[level] = (c0, c1)
        child_paths = []
        for p in paths:
            for i in range(1 << d):
                child_paths.append(tuple(p[j] + (bool((i >> j) & 1),) for j in range(d)))
        kept = np.nonzero(np.asarray(keep, bool))[0]
        if last:
            res.final_paths = [child_paths[k] for k in kept]
            res.final_values = [vals[k] for k in kept]
        paths = [child_paths[k] for k in kept]
        parents = kept.astype(np.uint64)
        s0, s1 = c0, c1
        if max_seconds is not None and time.perf_counter() - t_start > max_seconds:
            break
        if parents.size == 0 and not last:
            # reference: an empty frontier makes every later level produce no children
            res.final_paths, res.final_values = [], []
            for _ in range(level + 1, levels):
                res.n_children.append(0)
                res.counts.append(np.zeros(0, np.uint64))
                res.keeps.append(np.zeros(0, bool))
            break
    return res


# --------------------------------------------------------------------------------------
# Bit-string utilities (lib.rs) — restated for the oracle's own key generation.
# --------------------------------------------------------------------------------------

def u32_to_bits(nbits: int, x: int):           # lib.rs:56-65 (LSB first)
    return [bool((x >> i) & 1) for i in range(nbits)]


def msb_u32_to_bits(nbits: int, x: int):       # lib.rs:67-76
    return [bool((x >> i) & 1) for i in reversed(range(nbits))]


def bits_to_u32(bits) -> int:                  # lib.rs:78-88 (MSB first)
    r = 0
    for b in bits:
        r = (r << 1) | int(bool(b))
    return r


def string_to_bits(s: bytes):                  # lib.rs:90-98
    out = []
    for byte in s:
        out += u32_to_bits(8, byte)
    return out


def all_bit_vectors(dim: int):                 # lib.rs:125-129
    return [[bool((i >> j) & 1) for j in range(dim)] for i in range(1 << dim)]


def add_bitstrings(a, b):                      # lib.rs:131-151
    m = max(len(a), len(b))
    a = [False] * (m - len(a)) + list(a)
    b = [False] * (m - len(b)) + list(b)
    out, carry = [], False
    for x, y in zip(reversed(a), reversed(b)):
        s = x ^ y ^ carry
        carry = (x and y) or (y and carry) or (x and carry)
        out.append(s)
    if carry:
        out.append(True)
    return list(reversed(out))


def subtract_bitstrings(a, b):                 # lib.rs:153-183
    m = max(len(a), len(b))
    a = [False] * (m - len(a)) + list(a)
    b = [False] * (m - len(b)) + list(b)
    bt = [not x for x in b]
    carry = True
    for i in reversed(range(m)):
        s = bt[i] ^ carry
        carry = bt[i] and carry
        bt[i] = s
        if not carry:
            break
    out, carry = [], False
    for x, y in zip(reversed(a), reversed(bt)):
        s = x ^ y ^ carry
        carry = (x and y) or (y and carry) or (x and carry)
        out.append(s)
    return list(reversed(out))


def l_inf_ball_bounds(alpha, size: int):
    """ibDCF.rs:175-188: (alpha - size, alpha + size) MSB-first, width max(len, 32)."""
    delta = msb_u32_to_bits(32, size)
    left = subtract_bitstrings(alpha, delta)
    right = add_bitstrings(alpha, delta)
    assert len(left) == len(right), "carry out of add_bitstrings (reference panics, ibDCF.rs:182)"
    return left, right


def i16_to_bitvec(v: int):                     # sample_driving_data.rs:25-28
    u = v & 0xFFFF
    return [bool((u >> (15 - i)) & 1) for i in range(16)]


# ---- sketch + Beaver verification (row a9; sketch.rs / mpc.rs, dead in the reference) -------
def prg_stream_u64(seed: bytes, pos: int) -> int:
    """PrgStream::next_u64 draw `pos` of PrgSeed::to_rng (prg.rs:82-90,161-182)."""
    s = np.frombuffer(bytes(seed), np.uint8).copy()
    return int(lib().orc_prg_stream_u64(_p(s), ctypes.c_uint64(pos)))


u32p = ctypes.POINTER(ctypes.c_uint32)


def fe255_stream_draw(seed: bytes, m: int) -> int:
    """Draw m of the FieldElm stream before rejection (num-bigint gen_biguint(255), see the C)."""
    s = np.frombuffer(bytes(seed), np.uint8).copy()
    out = np.zeros(8, np.uint32)
    lib().orc_fe255_stream_draw(_p(s), ctypes.c_uint64(m), _p(out, u32p))
    return limbs_to_int(out)


def int_to_limbs8(v: int) -> np.ndarray:
    return np.array([(v >> (32 * k)) & 0xFFFFFFFF for k in range(8)], np.uint32)


def limbs_to_int(a) -> int:
    return sum(int(x) << (32 * k) for k, x in enumerate(np.asarray(a, np.uint64).ravel()))


def fe255_op(op: str, a: int, b: int = 0) -> int:
    """orc_fe255_{mul,add,sub,neg} on Python ints (canonical inputs)."""
    x, y, o = int_to_limbs8(a), int_to_limbs8(b), np.zeros(8, np.uint32)
    f = getattr(lib(), "orc_fe255_" + op)
    if op == "neg":
        f(_p(x, u32p), _p(o, u32p))
    else:
        f(_p(x, u32p), _p(y, u32p), _p(o, u32p))
    return limbs_to_int(o)


def sketch_fe255(seeds: np.ndarray, x: np.ndarray, kx: np.ndarray, nthreads: int = 0) -> np.ndarray:
    """sketch_at_last (sketch.rs:202-245), U = FieldElm: x / kx [n][nodes][8] u32 LE limbs ->
    [n][6][8] canonical {r_x, r2_x, r_kx, rand1, rand2, rand3}."""
    seeds = np.ascontiguousarray(seeds, np.uint8)
    x = np.ascontiguousarray(x, np.uint32)
    kx = np.ascontiguousarray(kx, np.uint32)
    n, F = x.shape[:2]
    out = np.zeros((n, 6, 8), np.uint32)
    lib().orc_sketch_fe255_batch(ctypes.c_uint64(n), ctypes.c_uint32(F), _p(seeds), _p(x, u32p), _p(kx, u32p),
                                 _p(out, u32p), ctypes.c_int(nthreads))
    return out


def mul_cor_share_fe255(sketch6, mac, mac2, triples9) -> np.ndarray:
    """MulState::new + cor_share (mpc.rs:83-158), U = FieldElm: [n][6][8]."""
    sk, m, m2, tr = (np.ascontiguousarray(a, np.uint32) for a in (sketch6, mac, mac2, triples9))
    n = sk.shape[0]
    out = np.zeros((n, 6, 8), np.uint32)
    for i in range(n):
        lib().orc_mul_cor_share_fe255(_p(sk[i], u32p), _p(m[i], u32p), _p(m2[i], u32p), _p(tr[i], u32p),
                                      _p(out[i], u32p))
    return out


def mul_out_share_fe255(server_idx: int, sketch6, mac, mac2, triples9, cor6) -> np.ndarray:
    """MulState::out_share (mpc.rs:182-212), U = FieldElm: [n][8]."""
    sk, m, m2, tr, c = (np.ascontiguousarray(a, np.uint32) for a in (sketch6, mac, mac2, triples9, cor6))
    n = sk.shape[0]
    out = np.zeros((n, 8), np.uint32)
    for i in range(n):
        lib().orc_mul_out_share_fe255(int(server_idx), _p(sk[i], u32p), _p(m[i], u32p), _p(m2[i], u32p),
                                      _p(tr[i], u32p), _p(c[i], u32p), _p(out[i], u32p))
    return out


def sketch_verify_fe255(seeds, x0, kx0, x1, kx1, mac, mac2, triples, nthreads: int = 0):
    """main.rs:14-70 at the last level (U = FieldElm), both servers: (ok [n], out_shares [2][n][8])."""
    x0, kx0, x1, kx1 = (np.ascontiguousarray(a, np.uint32) for a in (x0, kx0, x1, kx1))
    mac, mac2, triples = (np.ascontiguousarray(a, np.uint32) for a in (mac, mac2, triples))
    n, F = x0.shape[:2]
    ok = np.zeros(n, np.uint8)
    outs = np.zeros((2, n, 8), np.uint32)
    lib().orc_sketch_verify_fe255_batch(ctypes.c_uint64(n), ctypes.c_uint32(F),
                                        _p(np.ascontiguousarray(seeds, np.uint8)), _p(x0, u32p), _p(kx0, u32p),
                                        _p(x1, u32p), _p(kx1, u32p), _p(mac, u32p), _p(mac2, u32p),
                                        _p(triples, u32p), _p(ok), _p(outs, u32p), ctypes.c_int(nthreads))
    return ok.astype(bool), outs


def sketch_fe(seeds: np.ndarray, x: np.ndarray, kx: np.ndarray, nthreads: int = 0) -> np.ndarray:
    """sketch_at (sketch.rs:157-200), T = FE, for [n] keys -> [n][6] canonical."""
    seeds = np.ascontiguousarray(seeds, np.uint8)
    x = np.ascontiguousarray(x, np.uint64)
    kx = np.ascontiguousarray(kx, np.uint64)
    n, F = x.shape
    out = np.zeros((n, 6), np.uint64)
    lib().orc_sketch_fe_batch(ctypes.c_uint64(n), ctypes.c_uint32(F), _p(seeds), _p(x, u64p), _p(kx, u64p),
                              _p(out, u64p), ctypes.c_int(nthreads))
    return out


def mul_cor_share_fe(sketch6, mac, mac2, triples9) -> np.ndarray:
    """MulState::new + cor_share (mpc.rs:83-158) per key."""
    n = sketch6.shape[0]
    out = np.zeros((n, 6), np.uint64)
    for i in range(n):
        sk = np.ascontiguousarray(sketch6[i], np.uint64)
        tr = np.ascontiguousarray(triples9[i], np.uint64)
        o = np.zeros(6, np.uint64)
        lib().orc_mul_cor_share_fe(_p(sk, u64p), ctypes.c_uint64(int(mac[i])), ctypes.c_uint64(int(mac2[i])),
                                   _p(tr, u64p), _p(o, u64p))
        out[i] = o
    return out


def mul_out_share_fe(server_idx: int, sketch6, mac, mac2, triples9, cor6) -> np.ndarray:
    """MulState::out_share (mpc.rs:182-212) per key."""
    n = sketch6.shape[0]
    out = np.zeros(n, np.uint64)
    for i in range(n):
        sk = np.ascontiguousarray(sketch6[i], np.uint64)
        tr = np.ascontiguousarray(triples9[i], np.uint64)
        c = np.ascontiguousarray(cor6[i], np.uint64)
        out[i] = lib().orc_mul_out_share_fe(int(server_idx), _p(sk, u64p), int(mac[i]), int(mac2[i]), _p(tr, u64p),
                                            _p(c, u64p))
    return out


def sketch_verify_fe(seeds, x0, kx0, x1, kx1, mac, mac2, triples, nthreads: int = 0):
    """main.rs:14-70 verify_sketches for one level, both servers: (ok [n], out shares [2][n]).
    mac / mac2 [2][n], triples [2][n][9]."""
    n, F = x0.shape
    ok = np.zeros(n, np.uint8)
    outs = np.zeros((2, n), np.uint64)
    a = [np.ascontiguousarray(v, np.uint64) for v in (x0, kx0, x1, kx1, mac, mac2, triples)]
    lib().orc_sketch_verify_fe_batch(ctypes.c_uint64(n), ctypes.c_uint32(F), _p(np.ascontiguousarray(seeds, np.uint8)),
                                     *[_p(v, u64p) for v in a], _p(ok), _p(outs, u64p), ctypes.c_int(nthreads))
    return ok.astype(bool), outs


# --------------------------------------------------------------------------------------
# Row f1: garbled-circuit equality test (equalitytest.rs:25-219), see fhh_oracle.c
# --------------------------------------------------------------------------------------
def gc_garble_eq(gb_bits: np.ndarray, ev_bits: np.ndarray, mask: int, key: bytes, delta: bytes,
                 label_nonce: int = 0, gate_base: int = 0):
    """Garbler for n tests of `bits` bits (gb_bits / ev_bits [n][bits] 0/1). Returns
    (tables [n][bits-1][2][16], gb_labels [n][bits+1][16], ev_labels [n][bits][16], decode [n])."""
    g = np.ascontiguousarray(gb_bits, np.uint8)
    e = np.ascontiguousarray(ev_bits, np.uint8)
    n, bits = g.shape
    tables = np.zeros((n, max(bits - 1, 0), 2, 16), np.uint8)
    gbl = np.zeros((n, bits + 1, 16), np.uint8)
    evl = np.zeros((n, bits, 16), np.uint8)
    dec = np.zeros(n, np.uint8)
    k = np.frombuffer(key, np.uint8).copy()
    d = np.frombuffer(delta, np.uint8).copy()
    lib().orc_gc_garble_eq(ctypes.c_uint64(n), ctypes.c_uint32(bits), _p(g), _p(e), ctypes.c_uint32(mask & 1), _p(k),
                           _p(d), ctypes.c_uint64(label_nonce), ctypes.c_uint64(gate_base), _p(tables), _p(gbl),
                           _p(evl), _p(dec))
    return tables, gbl, evl, dec


def gc_eval_eq(tables, gb_labels, ev_labels, decode, gate_base: int = 0) -> np.ndarray:
    """Evaluator: out [n] = eq ^ mask."""
    t = np.ascontiguousarray(tables, np.uint8)
    g = np.ascontiguousarray(gb_labels, np.uint8)
    e = np.ascontiguousarray(ev_labels, np.uint8)
    d = np.ascontiguousarray(decode, np.uint8)
    n, bits = e.shape[0], e.shape[1]
    out = np.zeros(n, np.uint8)
    lib().orc_gc_eval_eq(ctypes.c_uint64(n), ctypes.c_uint32(bits), _p(t), _p(g), _p(e), _p(d),
                         ctypes.c_uint64(gate_base), _p(out))
    return out


def ot_extend(choices: np.ndarray, x0: np.ndarray, x1, delta: bytes, seeds: np.ndarray, s: bytes,
              tweak_base: int = 0, transcript: bool = False, prg: str = "chacha12"):
    """IKNP/ALSZ OT extension (see fhh_oracle.c): choices [m] 0/1, x0 / x1 [m][16] (x1 None:
    x1 = x0 ^ delta), seeds [128][2][16], s 16 bytes. Returns out [m][16] (and U [128][nblk][16],
    Y0, Y1 [m][16] if transcript). prg: the row PRG — "chacha12" (the GPU's since r06) or "aes"
    (AES-128-CTR, the reference's ocelot AesRng form; bench.py's reference-form CPU baseline)."""
    prg_id = {"aes": 0, "chacha12": 1}[prg]
    ch = np.packbits(np.asarray(choices, np.uint8) & 1, bitorder="little")
    m = len(choices)
    a0 = np.ascontiguousarray(x0, np.uint8)
    a1 = None if x1 is None else np.ascontiguousarray(x1, np.uint8)
    sd = np.ascontiguousarray(seeds, np.uint8)
    dl = np.frombuffer(delta if delta is not None else bytes(16), np.uint8).copy()
    sv = np.frombuffer(s, np.uint8).copy()
    out = np.zeros((m, 16), np.uint8)
    nblk = (m + 127) // 128
    u = np.zeros((128, nblk, 16), np.uint8) if transcript else None
    y0 = np.zeros((m, 16), np.uint8) if transcript else None
    y1 = np.zeros((m, 16), np.uint8) if transcript else None
    lib().orc_ot_extend(ctypes.c_uint64(m), _p(np.ascontiguousarray(ch)), _p(a0), None if a1 is None else _p(a1),
                        _p(dl), _p(sd), _p(sv), ctypes.c_uint64(tweak_base), _p(out),
                        None if u is None else _p(u), None if y0 is None else _p(y0),
                        None if y1 is None else _p(y1), ctypes.c_int(prg_id))
    return (out, u, y0, y1) if transcript else out


def chacha_block(rounds: int, key: bytes, ctr: int, nonce: int = 0) -> bytes:
    """The ChaCha block function of the OT row PRG (fhh_oracle.c orc_chacha_block): 64 bytes."""
    out = np.zeros(64, np.uint8)
    k = np.frombuffer(key, np.uint8).copy()
    assert k.size == 32
    lib().orc_chacha_block(ctypes.c_uint32(rounds), _p(k), ctypes.c_uint64(ctr), ctypes.c_uint64(nonce), _p(out))
    return out.tobytes()


def gc_set_ni(on: bool) -> None:
    """Row f1's AES (labels, TCCR, OT PRG and cr_hash) on AES-NI (the default where the CPU has it,
    as swanky's fixed-key AES does) or on the byte-wise FIPS-197 path."""
    lib().orc_gc_set_ni(ctypes.c_int(1 if on else 0))


def gc_get_ni() -> bool:
    return bool(lib().orc_gc_get_ni())


def gc_garble_eq_cot(gb_bits: np.ndarray, ev_zero: np.ndarray, mask: int, delta: bytes, gate_base: int = 0,
                     share: bool = False):
    """The r05 garbler (fhh_oracle.c orc_gc_garble_eq_cot): the evaluator's zero labels ev_zero
    [n][bits][16] come from the labels C-OT; the garbler's string and mask are folded into the circuit.
    Returns (tables [n][bits-1][2][16], decode [n]); share (r05c, orc_gc_garble_eq_cot_share): also
    the garbler's FE node values [n] and the 8-B share message y [n] from the output labels."""
    g = np.ascontiguousarray(gb_bits, np.uint8)
    z = np.ascontiguousarray(ev_zero, np.uint8)
    n, bits = g.shape
    tables = np.zeros((n, max(bits - 1, 0), 2, 16), np.uint8)
    dec = np.zeros(n, np.uint8)
    d = np.frombuffer(delta, np.uint8).copy()
    gv = np.zeros(n, np.uint64) if share else None
    y = np.zeros(n, np.uint64) if share else None
    lib().orc_gc_garble_eq_cot_share(ctypes.c_uint64(n), ctypes.c_uint32(bits), _p(g), _p(z),
                                     ctypes.c_uint32(mask & 1), _p(d), ctypes.c_uint64(gate_base), _p(tables),
                                     _p(dec), None if gv is None else _p(gv), None if y is None else _p(y))
    return (tables, dec, gv, y) if share else (tables, dec)


def gc_eval_eq_cot(tables, ev_active, decode, gate_base: int = 0, share_y=None):
    """The r05 evaluator: out [n] = eq ^ mask from its OT'd labels ev_active [n][bits][16]; with share_y
    (r05c) also its FE node values [n] from its output label: returns (out, values)."""
    t = np.ascontiguousarray(tables, np.uint8)
    e = np.ascontiguousarray(ev_active, np.uint8)
    d = np.ascontiguousarray(decode, np.uint8)
    n, bits = e.shape[0], e.shape[1]
    out = np.zeros(n, np.uint8)
    y = None if share_y is None else np.ascontiguousarray(share_y, np.uint64)
    ev = np.zeros(n, np.uint64) if y is not None else None
    lib().orc_gc_eval_eq_cot_share(ctypes.c_uint64(n), ctypes.c_uint32(bits), _p(t), _p(e), _p(d),
                                   ctypes.c_uint64(gate_base), _p(out), None if y is None else _p(y),
                                   None if ev is None else _p(ev))
    return (out, ev) if y is not None else out


def gt_garble(gb_bits: np.ndarray, ev_zero: np.ndarray, mask: int, delta: bytes, gate_base: int = 0):
    """r05d, the FE levels' garbled table (fhh_oracle.c orc_gt_garble): from the labels OT's zero labels
    ev_zero [n][bits][16] and the garbler's bits, its messages [n][2^bits - 1] u64 (row 0 carries none)
    and its node values [n] (r1 = v + mask)."""
    g = np.ascontiguousarray(gb_bits, np.uint8)
    z = np.ascontiguousarray(ev_zero, np.uint8)
    n, bits = g.shape
    msgs = np.zeros((n, (1 << bits) - 1), np.uint64)
    gv = np.zeros(n, np.uint64)
    d = np.frombuffer(delta, np.uint8).copy()
    lib().orc_gt_garble(ctypes.c_uint64(n), ctypes.c_uint32(bits), _p(g), _p(z), ctypes.c_uint32(mask & 1), _p(d),
                        ctypes.c_uint64(gate_base), _p(msgs), _p(gv))
    return msgs, gv


def gt_eval(ev_active: np.ndarray, msgs: np.ndarray, gate_base: int = 0) -> np.ndarray:
    """r05d: the evaluator's node values [n] from its OT'd labels [n][bits][16] and the table's messages."""
    e = np.ascontiguousarray(ev_active, np.uint8)
    m = np.ascontiguousarray(msgs, np.uint64)
    n, bits = e.shape[0], e.shape[1]
    ev = np.zeros(n, np.uint64)
    lib().orc_gt_eval(ctypes.c_uint64(n), ctypes.c_uint32(bits), _p(e), _p(m), ctypes.c_uint64(gate_base), _p(ev))
    return ev


def gt_garble_ring32(gb_bits: np.ndarray, ev_zero: np.ndarray, mask: int, delta: bytes, gate_base: int = 0):
    """r06 (fhh_oracle.c orc_gt_garble_ring32): gt_garble with Z_2^32 shares — messages [n][2^bits - 1] u32 and the
    garbler's values [n] u32."""
    g = np.ascontiguousarray(gb_bits, np.uint8)
    z = np.ascontiguousarray(ev_zero, np.uint8)
    n, bits = g.shape
    msgs = np.zeros((n, (1 << bits) - 1), np.uint32)
    gv = np.zeros(n, np.uint32)
    d = np.frombuffer(delta, np.uint8).copy()
    lib().orc_gt_garble_ring32(ctypes.c_uint64(n), ctypes.c_uint32(bits), _p(g), _p(z), ctypes.c_uint32(mask & 1),
                               _p(d), ctypes.c_uint64(gate_base), _p(msgs), _p(gv))
    return msgs, gv


def gt_eval_ring32(ev_active: np.ndarray, msgs: np.ndarray, gate_base: int = 0) -> np.ndarray:
    """r06: the evaluator's Z_2^32 values [n] from its OT'd labels and the table's 4-B messages."""
    e = np.ascontiguousarray(ev_active, np.uint8)
    m = np.ascontiguousarray(msgs, np.uint32)
    n, bits = e.shape[0], e.shape[1]
    ev = np.zeros(n, np.uint32)
    lib().orc_gt_eval_ring32(ctypes.c_uint64(n), ctypes.c_uint32(bits), _p(e), _p(m), ctypes.c_uint64(gate_base),
                             _p(ev))
    return ev


COT_LABELS, COT_FE, COT_FE255, COT_RAW = 1, 2, 3, 4


def cot_extend(mode: int, choices: np.ndarray, seeds: np.ndarray, s: bytes, delta: bytes | None = None,
               mask: int = 0, ctr_off: int = 0):
    """Correlated OT extension (fhh_oracle.c orc_cot_extend). Returns (sender_out, out, U, y):
    mode 1: sender_out = x0 [m][16], out [m][16], y [m][16]; mode 2: sender values [m] u64, out [m]
    u64, y [m] u64; mode 3 (m even, pairs with one choice): sender values / out [m/2][32] BlockPairs,
    y [m][16]; mode 4 (the IKNP correlation, unhashed): sender_out = q [m][16], out = t [m][16] =
    q ^ r s, y unused (zeros)."""
    ch = np.packbits(np.asarray(choices, np.uint8) & 1, bitorder="little")
    m = len(choices)
    sd = np.ascontiguousarray(seeds, np.uint8)
    sv = np.frombuffer(s, np.uint8).copy()
    dl = np.frombuffer(delta if delta is not None else bytes(16), np.uint8).copy()
    nblk = (m + 127) // 128
    u = np.zeros((128, nblk, 16), np.uint8)
    if mode == COT_FE:
        sx = np.zeros(m, np.uint64)
        out = np.zeros(m, np.uint64)
        y = np.zeros(m, np.uint64)
    elif mode == COT_FE255:
        sx = np.zeros((m // 2, 32), np.uint8)
        out = np.zeros((m // 2, 32), np.uint8)
        y = np.zeros((m, 16), np.uint8)
    else:
        sx = np.zeros((m, 16), np.uint8)
        out = np.zeros((m, 16), np.uint8)
        y = np.zeros((m, 16), np.uint8)
    lib().orc_cot_extend(ctypes.c_uint64(m), ctypes.c_uint32(mode), _p(np.ascontiguousarray(ch)), _p(dl),
                         ctypes.c_uint32(mask & 1), _p(sd), _p(sv), ctypes.c_uint64(ctr_off),
                         sx.ctypes.data_as(u8p), out.ctypes.data_as(u8p), _p(u), y.ctypes.data_as(u8p))
    return sx, out, u, y


def cot_extend_ss(ss_k: int, mode: int, choices: np.ndarray, seeds: np.ndarray, s: bytes, delta: bytes | None = None,
                  mask: int = 0, ctr_off: int = 0):
    """cot_extend on SoftSpoken OT extension with k = ss_k bits per chunk (fhh_oracle.c cot_rows / ss_ggm;
    ss_k = 1 is IKNP). Returns (sender_out, out, U [128 / ss_k][nblk][16], y, corr [128 / ss_k][ss_k][2][16]):
    U and the GGM corrections are the receiver's messages."""
    assert ss_k in (1, 2, 4)
    ch = np.packbits(np.asarray(choices, np.uint8) & 1, bitorder="little")
    m = len(choices)
    sd = np.ascontiguousarray(seeds, np.uint8)
    sv = np.frombuffer(s, np.uint8).copy()
    dl = np.frombuffer(delta if delta is not None else bytes(16), np.uint8).copy()
    nblk = (m + 127) // 128
    u = np.zeros((128 // ss_k, nblk, 16), np.uint8)
    corr = np.zeros((128 // ss_k, ss_k, 2, 16), np.uint8)
    if mode == COT_FE:
        sx, out, y = np.zeros(m, np.uint64), np.zeros(m, np.uint64), np.zeros(m, np.uint64)
    elif mode == COT_FE255:
        sx, out, y = np.zeros((m // 2, 32), np.uint8), np.zeros((m // 2, 32), np.uint8), np.zeros((m, 16), np.uint8)
    else:
        sx, out, y = np.zeros((m, 16), np.uint8), np.zeros((m, 16), np.uint8), np.zeros((m, 16), np.uint8)
    lib().orc_cot_extend_ss(ctypes.c_uint32(ss_k), ctypes.c_uint64(m), ctypes.c_uint32(mode),
                            _p(np.ascontiguousarray(ch)), _p(dl), ctypes.c_uint32(mask & 1), _p(sd), _p(sv),
                            ctypes.c_uint64(ctr_off), sx.ctypes.data_as(u8p), out.ctypes.data_as(u8p), _p(u),
                            y.ctypes.data_as(u8p), _p(corr))
    return sx, out, u, y, corr
