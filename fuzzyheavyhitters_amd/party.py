"""The two servers' halves of a level's garbled-circuit equality test + OT, each on its own ctx
(fhh_gb_* / fhh_ev_* in include/fhh.h), and a leader level loop driving them
(src/bin/leader.rs:417-440 over src/collect.rs:370-505 with gc_sender = true on server 0).

Each server holds only its own secrets and draws them itself, as the reference's server threads do
(`AesRng::new()` per channel, collect.rs:431; `OtSender::init` / `OtReceiver::init` per channel and
level, collect.rs:454,460):

  * the garbler (server 0): its mask per chunk (os.urandom), and the base-OT receiver's side of each
    level's Chou–Orlandi runs (its choice bits s, its seed; the labels run's s is its free-XOR Delta);
  * the evaluator (server 1): the base-OT sender's side (its seed, hence both keys of every base OT).

Only protocol messages cross between them: the CO15 messages A and B of each base-OT run, then per
chunk u1, y1 (empty since r05b: the labels OT needs no reply), gc, u2, y2 (both empty at the FE levels
since r05c: the share rides in gc, taken from the circuit's output labels; the share OT and its base-OT
run remain at the FieldElm level). In a deployment they go over the servers' channel; here `Channel` copies
each one into a buffer the receiving party owns (`fhh_memcpy_device`, or a bytes copy for the host
messages) and counts the bytes. `GarblerParty` and `EvaluatorParty` keep the two sides' state apart;
nothing of one is handed to the other except through a Channel.
"""
from __future__ import annotations

import ctypes
import os
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass, field

import numpy as np

from ._lib import FhhEvCfg, FhhGbCfg, check, lib, u8p, u32p, u64p
from .collection import KeyCollection
from .fields import limbs10_to_int


def test_cfgs(prf_seed: int, level: int):
    """TEST MODE: (fhh_gb_cfg, fhh_ev_cfg) of fhh_sim_crawl's in-process material for this level
    (fhh_gc_party_test_cfgs): one seed derives both parties' secrets — reproducible, not private."""
    gb, ev = FhhGbCfg(), FhhEvCfg()
    check(lib().fhh_gc_party_test_cfgs(prf_seed, level, ctypes.byref(gb), ctypes.byref(ev)))
    return gb, ev


class Channel:
    """One direction of the servers' channel. mode "copy": a device message becomes a copy in memory
    the receiving party owns (a torch buffer on its GPU, reused across levels) — the bytes a
    deployment moves over the network, moved here device to device. mode "inplace" (both parties on
    one GPU): the receiver reads the message where the sender's ctx produced it. That is safe in
    this protocol order because each party's messages live in their own buffers (gc, U, y) and a
    party rewrites one only after the peer's call that consumed it has returned (every call returns
    after its device work is complete). Host messages (the base OTs' A and B) are copied as bytes."""

    def __init__(self, device: int, mode: str = "copy"):
        import threading
        import torch
        if mode not in ("copy", "inplace"):
            raise ValueError(f"Channel mode {mode!r}")
        self.torch = torch
        self.device = device
        self.mode = mode
        self.bufs: dict = {}
        self.bytes = 0
        self.host_bytes = 0
        self._lock = threading.Lock()

    def send(self, name: str, src_ptr: int, nbytes: int) -> int:
        if self.mode == "inplace":
            self.bytes += nbytes
            return src_ptr
        buf = self.bufs.get(name)
        if buf is None or buf.numel() < nbytes:
            buf = self.torch.empty(max(nbytes, 1), dtype=self.torch.uint8, device=f"cuda:{self.device}")
            self.torch.cuda.synchronize(self.device)
            self.bufs[name] = buf
        if nbytes:
            check(lib().fhh_memcpy_device(self.device, ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(src_ptr),
                                          nbytes))
        self.bytes += nbytes
        return buf.data_ptr()

    def send_host(self, data: bytes) -> bytes:
        """A host message (thread-safe: base-OT runs go ahead of the crawl on worker threads)."""
        with self._lock:
            self.host_bytes += len(data)
        return bytes(data)


def _rand(n: int) -> np.ndarray:
    return np.frombuffer(os.urandom(n), np.uint8).copy()


def _co15_check(rc: int):
    if rc != 0:
        msg = lib().fhh_base_ot_last_error()
        raise RuntimeError(f"base OT failed ({rc}): {msg.decode() if msg else ''}")


class GarblerParty:
    """Server 0's side: the OT-extension sender (base-OT receiver) and the garbler."""

    def __init__(self, kc: KeyCollection):
        self.kc = kc

    # -- base OTs: the CO15 receiver with choice bits s (OtSender::init's base OTs, collect.rs:454).
    # The labels kind's s is the circuit's free-XOR Delta (its bit 0, the colour bit, is 1)
    def co15_receive(self, A: bytes, colour: bool = False):
        s = _rand(16)
        if colour:
            s[0] |= 1
        seed = _rand(32)
        Av = np.frombuffer(A, np.uint8).copy()
        B = np.zeros((128, 65), np.uint8)
        chosen = np.zeros((128, 16), np.uint8)
        _co15_check(lib().fhh_co15_receiver(128, Av.ctypes.data_as(u8p), s.ctypes.data_as(u8p),
                                            seed.ctypes.data_as(u8p), B.ctypes.data_as(u8p),
                                            chosen.ctypes.data_as(u8p)))
        return B.tobytes(), (chosen, s)

    def chunk_cfg(self, base, child_begin: int, child_count: int, form: int = 0) -> FhhGbCfg:
        """The garbler's material for one chunk: a fresh mask (AesRng::new() per channel, collect.rs:431;
        its string is folded into the circuit, so it draws no labels) and the level's base OTs (both
        kinds; the labels kind's s is the circuit's Delta)."""
        cfg = FhhGbCfg()
        cfg.mask = os.urandom(1)[0] & 1
        chosen = np.zeros((2, 128, 16), np.uint8)    # [kind][128][16]; kind 1 only at the FieldElm level
        choice = np.zeros((2, 16), np.uint8)
        for w, b in enumerate(base):
            chosen[w], choice[w] = b[0], b[1]
        ctypes.memmove(cfg.base_chosen, chosen.tobytes(), chosen.nbytes)
        ctypes.memmove(cfg.base_choice, choice.tobytes(), choice.nbytes)
        cfg.child_begin, cfg.child_count = child_begin, child_count
        cfg.form = form
        return cfg


class EvaluatorParty:
    """Server 1's side: the OT-extension receiver (base-OT sender) and the evaluator."""

    def __init__(self, kc: KeyCollection):
        self.kc = kc

    # -- base OTs: the CO15 sender (OtReceiver::init's base OTs, collect.rs:460)
    def co15_start(self):
        seed = _rand(32)
        A = np.zeros(65, np.uint8)
        _co15_check(lib().fhh_co15_sender_start(seed.ctypes.data_as(u8p), A.ctypes.data_as(u8p)))
        return A.tobytes(), seed

    def co15_finish(self, seed: np.ndarray, B: bytes) -> np.ndarray:
        Bv = np.frombuffer(B, np.uint8).copy()
        pairs = np.zeros((128, 2, 16), np.uint8)
        _co15_check(lib().fhh_co15_sender_finish(128, seed.ctypes.data_as(u8p), Bv.ctypes.data_as(u8p),
                                                 pairs.ctypes.data_as(u8p)))
        return pairs

    @staticmethod
    def chunk_cfg(base, child_begin: int, child_count: int, form: int = 0) -> FhhEvCfg:
        cfg = FhhEvCfg()
        pairs = np.zeros((2, 128, 2, 16), np.uint8)  # [kind][128][2][16]; kind 1 only at the FieldElm level
        for w, b in enumerate(base):
            pairs[w] = b
        ctypes.memmove(cfg.base_pairs, pairs.tobytes(), pairs.nbytes)
        cfg.child_begin, cfg.child_count = child_begin, child_count
        cfg.form = form
        return cfg


def base_ot_run(gb: GarblerParty, ev: EvaluatorParty, to_gb: Channel, to_ev: Channel, colour: bool = False):
    """One Chou–Orlandi run of 128 OTs between the parties (the OT extension's init,
    collect.rs:454,460): A from the evaluator, B back from the garbler (colour: the labels kind, whose s
    is the free-XOR Delta). Returns (the garbler's (chosen, s), the evaluator's pairs) — each side's
    own result."""
    A, seed_e = ev.co15_start()
    B, gb_side = gb.co15_receive(to_gb.send_host(A), colour=colour)
    ev_side = ev.co15_finish(seed_e, to_ev.send_host(B))
    return gb_side, ev_side


def _out():
    return ctypes.c_void_p(), ctypes.c_uint64()


def run_chunk(gb: KeyCollection, ev: KeyCollection, cfg_gb: FhhGbCfg, cfg_ev: FhhEvCfg, to_gb: Channel,
              to_ev: Channel) -> dict:
    """One chunk's GC + OT, each call on its own server's ctx with its own cfg; returns the message
    sizes (u1, y1, gc, u2, y2)."""
    L = lib()
    u1, u1n = _out()
    check(L.fhh_ev_ot_labels(ev.handle, ctypes.byref(cfg_ev), ctypes.byref(u1), ctypes.byref(u1n)), ev.handle)
    u1_rx = to_gb.send("u", u1.value or 0, u1n.value)
    y1, y1n = _out()
    check(L.fhh_gb_ot_labels(gb.handle, ctypes.byref(cfg_gb), ctypes.c_void_p(u1_rx), u1n.value, ctypes.byref(y1),
                             ctypes.byref(y1n)), gb.handle)
    gc, gcn = _out()
    check(L.fhh_gb_garble(gb.handle, ctypes.byref(gc), ctypes.byref(gcn)), gb.handle)
    y1_rx = to_ev.send("y1", y1.value or 0, y1n.value)
    gc_rx = to_ev.send("gc", gc.value or 0, gcn.value)
    u2, u2n = _out()
    check(L.fhh_ev_evaluate(ev.handle, ctypes.c_void_p(gc_rx), gcn.value, ctypes.c_void_p(y1_rx), y1n.value,
                            ctypes.byref(u2), ctypes.byref(u2n)), ev.handle)
    u2_rx = to_gb.send("u", u2.value or 0, u2n.value)
    y2, y2n = _out()
    check(L.fhh_gb_ot_shares(gb.handle, ctypes.c_void_p(u2_rx), u2n.value, ctypes.byref(y2), ctypes.byref(y2n)),
          gb.handle)
    y2_rx = to_ev.send("y2", y2.value or 0, y2n.value)
    check(L.fhh_ev_ot_shares(ev.handle, ctypes.c_void_p(y2_rx), y2n.value), ev.handle)
    return {"u1": u1n.value, "y1": y1n.value, "gc": gcn.value, "u2": u2n.value, "y2": y2n.value}


def party_sums(kc: KeyCollection, C: int, last: bool):
    """fhh_party_node_sums: FE sums [C] (ints), or (unreduced, canonical) FieldElm sums at the last level."""
    if not last:
        out = np.zeros(max(C, 1), np.uint64)
        check(lib().fhh_party_node_sums(kc.handle, out.ctypes.data_as(u64p), None), kc.handle)
        return out[:C]
    unr = np.zeros((max(C, 1), 10), np.uint32)
    can = np.zeros((max(C, 1), 8), np.uint32)
    check(lib().fhh_party_node_sums(kc.handle, unr.ctypes.data_as(u32p), can.ctypes.data_as(u32p)), kc.handle)
    return [limbs10_to_int(r) for r in unr[:C]]


@dataclass
class TwoPartyResult:
    level_children: list = field(default_factory=list)
    counts: list = field(default_factory=list)           # per level v0 - v1 (the leader's view)
    level_bytes: list = field(default_factory=list)      # per level message sizes {u1, y1, gc, u2, y2}
    final: list = field(default_factory=list)            # Result(path, value): final_values
    base_ot_runs: int = 0                                # Chou–Orlandi runs (128 OTs each)
    base_ot_bytes: int = 0                               # their messages (A, B) over the channel
    base_ot_wait_s: float = 0.0                          # crawl time spent waiting for base OTs


# bytes per test of both parties' chunk buffers at d = 1 (gc message 81, labels 32 + 32, OT matrices
# and messages ~150, node values 16, with headroom): the auto chunk size's divisor
_PARTY_BYTES_PER_TEST = 512


def chunk_windows(C: int, chunk_children: int):
    """[(begin, count)] covering [0, C) in chunks of chunk_children (0: one window, the whole level)."""
    if chunk_children <= 0 or C <= chunk_children:
        return [(0, 0)]
    return [(b, min(chunk_children, C - b)) for b in range(0, C, chunk_children)]


def two_party_crawl(c0: KeyCollection, c1: KeyCollection, threshold: float, nclients_total: int | None = None,
                    material: str = "fresh", prf_seed: int = 0, levels: int = 0, expect_counts=None,
                    channel: str = "copy", timing: dict | None = None, record: bool = True,
                    chunk_children: int | None = None, chunk_bytes: int = 64 << 30,
                    level_log: list | None = None, base_ot_every: str = "level",
                    base_ot_workers: int | None = None, base_ot_ahead: int = 8,
                    form: str = "table", ot_ss_k: int = 1) -> TwoPartyResult:
    """The leader's level loop (leader.rs:417-440) with the GC + OT of every level split between the
    two servers' ctxs (server 0 garbles / sends, server 1 evaluates / receives): crawl both, run the
    level's protocol through the channel, take each server's node sums from its own device
    (fhh_party_node_sums), keep_values on the leader, prune both.

    material "fresh" (the default, a deployment's behaviour): each party draws its own secrets —
    the garbler a mask per chunk; its Delta is the labels base-OT run's s (per base-OT run: one per
    level, or one per crawl with base_ot_every "crawl"), so the chunks sharing a Delta stay independent
    through their disjoint row-PRG ranges of the run (ctr_off, party_session) and the level and test
    index in every gate tweak — and every level's two OT extensions start
    from real Chou–Orlandi base OTs run between the parties over the channel (base_ot_every "level",
    as the reference inits per level, collect.rs:454,460; "crawl": one run per OT kind for the whole
    crawl, the library extending it from a running counter). The runs are computed `base_ot_ahead`
    levels ahead on `base_ot_workers` host threads (the ctypes calls release the GIL).
    material "test": fhh_gc_party_test_cfgs(prf_seed, level) — one seed for both sides, ideal base
    OTs, reproducible (tests).

    A multi-device collection runs one protocol instance per shard over its own channel (the
    reference splits a level's tests over several channels, collect.rs:423-430). `expect_counts`
    (tests): per-level v0 - v1 to compare against as the crawl goes. `channel`: "copy" or "inplace"
    (both parties of a pair on one GPU). `timing` (a dict) accumulates the host wall seconds of each
    phase: crawl, gcot, node_sums, keep, prune. A level's tests run in chunks of `chunk_children`
    children (None: as many as `chunk_bytes` of both parties' buffers hold at ~512 B per test; 0: the
    whole level), one protocol instance per chunk. `level_log` (a list) receives one (level, children,
    crawl_s, gcot_s, node_sums_s) tuple per level. `form`: "table" (the FE levels' test as one garbled
    table where 2d <= 4, r05d) or "circuit" (the half-gates circuit at every level, r05c) — a public
    protocol choice both parties make alike. `ot_ss_k` (r06, public like form): 1 = IKNP OT extension, 2 / 4 =
    SoftSpoken with k = ot_ss_k (the U messages carry 128 / k rows + the GGM corrections)."""
    if ot_ss_k not in (1, 2, 4):
        raise ValueError(f"two_party_crawl: ot_ss_k {ot_ss_k!r}")
    if material not in ("fresh", "test"):
        raise ValueError(f"two_party_crawl: material {material!r}")
    if form not in ("table", "circuit"):
        raise ValueError(f"two_party_crawl: form {form!r}")
    form_id = 0 if form == "table" else 1
    if base_ot_every not in ("level", "crawl"):
        raise ValueError(f"two_party_crawl: base_ot_every {base_ot_every!r}")
    L = levels or c0.depth
    n_total = nclients_total if nclients_total is not None else c0.num_clients()
    thr = max(1, int(threshold * n_total))
    thr_last = max(1, min(int(threshold * n_total), 0xFFFFFFFF))
    S = len(c0.shard_info()[0])
    shards = [(c0.shard(k), c1.shard(k)) for k in range(S)] if S > 1 else [(c0, c1)]
    if channel == "inplace" and any(a.device != b.device for a, b in shards):
        raise ValueError("two_party_crawl: an in-place channel needs both parties of a pair on one GPU")
    chans = [(Channel(a.device, channel), Channel(b.device, channel)) for a, b in shards]
    parties = [(GarblerParty(a), EvaluatorParty(b)) for a, b in shards]
    res = TwoPartyResult()
    shard_clients = [a.num_clients() for a, _ in shards]
    # base OTs: a pool computing each (level, shard)'s CO15 runs (labels; + the share OT's at the last level) ahead
    pool = None
    pending: dict = {}
    if material == "fresh":
        nworkers = base_ot_workers or min(16, os.cpu_count() or 4)
        pool = ThreadPoolExecutor(max_workers=nworkers)

        def runs(k, kinds):
            gbp, evp = parties[k]
            to_gb, to_ev = chans[k]
            # kind 0 labels (s = Delta: colour bit), kind 1 the share OT — at the FieldElm level only (r05c)
            return [base_ot_run(gbp, evp, to_gb, to_ev, colour=(w == 0)) for w in range(kinds)]

        def submit(lv):
            key = 0 if base_ot_every == "crawl" else lv
            kinds = 2 if (base_ot_every == "crawl" or lv == L - 1) else 1
            for k in range(len(shards)):
                if shard_clients[k] and (key, k) not in pending:
                    pending[(key, k)] = pool.submit(runs, k, kinds)

        for lv in range(min(L, base_ot_ahead)):
            submit(lv)

    def level_base(lv, k):
        key = 0 if base_ot_every == "crawl" else lv
        t = time.perf_counter()
        got = pending[(key, k)].result()
        res.base_ot_wait_s += time.perf_counter() - t
        if base_ot_every == "level":
            del pending[(key, k)]
        return [g for g, _ in got], [e for _, e in got]

    c0.tree_init()
    c1.tree_init()
    from .fields import FE255_P, FE_P
    tm = timing if timing is not None else {}
    for k in ("crawl", "gcot", "node_sums", "keep", "prune"):
        tm.setdefault(k, 0.0)
    clock = time.perf_counter
    if chunk_children is None:
        chunk_children = max(1, chunk_bytes // (_PARTY_BYTES_PER_TEST * max(1, max(shard_clients))))
    try:
        for lv in range(L):
            last = lv == L - 1
            if pool is not None and lv + base_ot_ahead < L:
                submit(lv + base_ot_ahead)
            t0 = clock()
            C0, _ = (c0.tree_crawl_last if last else c0.tree_crawl)()
            C1, _ = (c1.tree_crawl_last if last else c1.tree_crawl)()
            assert C0 == C1
            t1 = clock()
            sizes = {}
            for k, ((a, b), (to_gb, to_ev)) in enumerate(zip(shards, chans)):
                if shard_clients[k] == 0:
                    continue
                gbp, evp = parties[k]
                if material == "fresh":
                    gb_base, ev_base = level_base(lv, k)
                for j, (cb, cc) in enumerate(chunk_windows(C0, chunk_children)):
                    if material == "fresh":
                        cfg_gb = gbp.chunk_cfg(gb_base, cb, cc, form_id)
                        cfg_ev = evp.chunk_cfg(ev_base, cb, cc, form_id)
                    else:
                        cfg_gb, cfg_ev = test_cfgs(prf_seed ^ (k << 40) ^ (j << 48), lv)
                        cfg_gb.child_begin, cfg_gb.child_count = cb, cc
                        cfg_ev.child_begin, cfg_ev.child_count = cb, cc
                        cfg_gb.form = cfg_ev.form = form_id
                    cfg_gb.ot_ss_k = cfg_ev.ot_ss_k = ot_ss_k
                    for name, v in run_chunk(a, b, cfg_gb, cfg_ev, to_gb, to_ev).items():
                        sizes[name] = sizes.get(name, 0) + v
            res.level_bytes.append(sizes)
            t2 = clock()
            s0 = party_sums(c0, C0, last)
            s1 = party_sums(c1, C1, last)
            t3 = clock()
            res.level_children.append(C0)
            if not last:
                keep = KeyCollection.keep_values(n_total, thr, s0, s1)
                t4 = clock()
                c0.tree_prune(keep)
                c1.tree_prune(keep)
            else:
                keep = KeyCollection.keep_values_last(n_total, thr_last, s0, s1)
                t4 = clock()
                c0.tree_prune_last(keep)
                c1.tree_prune_last(keep)
            t5 = clock()
            tm["crawl"] += t1 - t0
            tm["gcot"] += t2 - t1
            tm["node_sums"] += t3 - t2
            tm["keep"] += t4 - t3
            tm["prune"] += t5 - t4
            if level_log is not None:
                level_log.append((lv, int(C0), t1 - t0, t2 - t1, t3 - t2))
            if not (record or expect_counts is not None):
                continue
            if not last:
                res.counts.append(((s0.astype(object) - s1.astype(object)) % FE_P).astype(np.uint64))
            else:
                res.counts.append(np.array([((a % FE255_P) - (b % FE255_P)) % FE255_P for a, b in zip(s0, s1)],
                                           np.uint64))
            if expect_counts is not None and not np.array_equal(res.counts[-1], np.asarray(expect_counts[lv], np.uint64)):
                bad = np.nonzero(res.counts[-1] != np.asarray(expect_counts[lv], np.uint64))[0]
                raise ValueError(f"two-party crawl: level {lv}: {bad.size} of {C0} children differ (first {bad[:5]}: "
                                 f"{res.counts[-1][bad[:5]]} vs {np.asarray(expect_counts[lv])[bad[:5]]})")
    finally:
        if pool is not None:
            for f in pending.values():
                f.cancel()
            pool.shutdown(wait=True)
    res.final = KeyCollection.final_values(c0.final_shares(), c1.final_shares())
    res.base_ot_bytes = sum(a.host_bytes + b.host_bytes for a, b in chans)
    res.base_ot_runs = res.base_ot_bytes // (65 + 128 * 65) if res.base_ot_bytes else 0
    return res


__all__ = ["Channel", "GarblerParty", "EvaluatorParty", "base_ot_run", "test_cfgs", "run_chunk", "party_sums",
           "two_party_crawl", "TwoPartyResult", "chunk_windows"]
