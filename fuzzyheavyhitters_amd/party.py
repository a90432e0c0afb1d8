"""The two servers' halves of a level's garbled-circuit equality test + OT, each on its own ctx
(fhh_gb_* / fhh_ev_* in include/fhh.h), and a leader level loop driving them
(src/bin/leader.rs:417-440 over src/collect.rs:370-505 with gc_sender = true on server 0).

Only the protocol's messages cross between the two KeyCollections: the garbled circuit, and
U / Y of the two OT extensions (the evaluator's input labels, then the share conversion). In a
deployment they go over the servers' channel; here `Channel` copies each one into a buffer the
receiving party owns (`fhh_memcpy_device`) and counts the bytes.
"""
from __future__ import annotations

import ctypes
import time
from dataclasses import dataclass, field

import numpy as np

from ._lib import FhhGcPartyCfg, check, lib, u64p, u32p
from .collection import KeyCollection, Result
from .fields import limbs10_to_int


def level_cfg(prf_seed: int, level: int) -> FhhGcPartyCfg:
    """The in-process level loop's material for this level (fhh_sim_crawl gc = 2, ideal base OTs):
    a two-party run with it reproduces fhh_sim_crawl's transcripts. A deployment draws fresh
    randomness and runs real base OTs (fhh_co15_*) instead."""
    cfg = FhhGcPartyCfg()
    check(lib().fhh_gc_party_level_cfg(prf_seed, level, ctypes.byref(cfg)))
    return cfg


class Channel:
    """One direction of the servers' channel. mode "copy": a message becomes a copy in memory the
    receiving party owns (a torch buffer on its GPU, reused across levels) — the bytes a deployment
    moves over the network, moved here device to device. mode "inplace" (both parties on one GPU):
    the receiver reads the message where the sender's ctx produced it. That is safe in this protocol
    order because each party's messages live in their own buffers (gc, U, Y0 | Y1) and a party
    rewrites one only after the peer's call that consumed it has returned (every call returns after
    its device work is complete)."""

    def __init__(self, device: int, mode: str = "copy"):
        import torch
        if mode not in ("copy", "inplace"):
            raise ValueError(f"Channel mode {mode!r}")
        self.torch = torch
        self.device = device
        self.mode = mode
        self.bufs: dict = {}
        self.bytes = 0

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


def _out():
    return ctypes.c_void_p(), ctypes.c_uint64()


def run_level(gb: KeyCollection, ev: KeyCollection, cfg_gb: FhhGcPartyCfg, cfg_ev: FhhGcPartyCfg,
              to_gb: Channel, to_ev: Channel) -> dict:
    """One level's GC + OT, each call on its own server's ctx; returns the message sizes."""
    L = lib()
    gc, gcn = _out()
    check(L.fhh_gb_garble(gb.handle, ctypes.byref(cfg_gb), ctypes.byref(gc), ctypes.byref(gcn)), gb.handle)
    u1, u1n = _out()
    check(L.fhh_ev_ot_labels(ev.handle, ctypes.byref(cfg_ev), ctypes.byref(u1), ctypes.byref(u1n)), ev.handle)
    gc_rx = to_ev.send("gc", gc.value or 0, gcn.value)
    u1_rx = to_gb.send("u", u1.value or 0, u1n.value)
    y1, y1n = _out()
    check(L.fhh_gb_ot_labels(gb.handle, ctypes.c_void_p(u1_rx), u1n.value, ctypes.byref(y1), ctypes.byref(y1n)),
          gb.handle)
    y1_rx = to_ev.send("y", y1.value or 0, y1n.value)
    u2, u2n = _out()
    check(L.fhh_ev_evaluate(ev.handle, ctypes.c_void_p(gc_rx), gcn.value, ctypes.c_void_p(y1_rx), y1n.value,
                            ctypes.byref(u2), ctypes.byref(u2n)), ev.handle)
    u2_rx = to_gb.send("u", u2.value or 0, u2n.value)
    y2, y2n = _out()
    check(L.fhh_gb_ot_shares(gb.handle, ctypes.c_void_p(u2_rx), u2n.value, ctypes.byref(y2), ctypes.byref(y2n)),
          gb.handle)
    y2_rx = to_ev.send("y", y2.value or 0, y2n.value)
    check(L.fhh_ev_ot_shares(ev.handle, ctypes.c_void_p(y2_rx), y2n.value), ev.handle)
    return {"gc": gcn.value, "u1": u1n.value, "y1": y1n.value, "u2": u2n.value, "y2": y2n.value}


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
    level_bytes: list = field(default_factory=list)      # per level message sizes {gc, u1, y1, u2, y2}
    final: list = field(default_factory=list)            # Result(path, value): final_values


# bytes per test of both parties' chunk buffers at d = 1 (gc message 81, labels 32 + 32, OT matrices
# and messages 160, OT 2 messages / outputs 48, with headroom): the auto chunk size's divisor
_PARTY_BYTES_PER_TEST = 512


def chunk_windows(C: int, chunk_children: int):
    """[(begin, count)] covering [0, C) in chunks of chunk_children (0: one window, the whole level)."""
    if chunk_children <= 0 or C <= chunk_children:
        return [(0, 0)]
    return [(b, min(chunk_children, C - b)) for b in range(0, C, chunk_children)]


def two_party_crawl(c0: KeyCollection, c1: KeyCollection, threshold: float, nclients_total: int | None = None,
                    prf_seed: int = 0, levels: int = 0, cfg_fn=None, expect_counts=None,
                    channel: str = "copy", timing: dict | None = None, record: bool = True,
                    chunk_children: int | None = None, chunk_bytes: int = 64 << 30,
                    level_log: list | None = None) -> TwoPartyResult:
    """The leader's level loop (leader.rs:417-440) with the GC + OT of every level split between
    the two servers' ctxs (server 0 garbles / sends, server 1 evaluates / receives): crawl both,
    run the level's protocol through the channel, take each server's node sums from its own
    device (fhh_party_node_sums), keep_values on the leader, prune both. `cfg_fn(level)` gives the
    level's fhh_gc_party_cfg (default: level_cfg(prf_seed, level), fhh_sim_crawl's material); for a
    multi-device collection `cfg_fn(level, shard)`, one protocol instance per shard.
    `expect_counts` (tests): per-level v0 - v1 to compare against as the crawl goes (raises at the
    first level that differs instead of crawling on a wrong frontier). `channel`: "copy" (every
    message copied into a buffer of the receiver) or "inplace" (the receiver reads the sender's
    buffer; both shards of a pair must share a GPU). `timing` (a dict) accumulates the host wall
    seconds of each phase of the level loop: crawl, gcot, node_sums, keep, prune (every call returns
    after its device work, so these are the phases' elapsed times). record=False skips the per-level
    v0 - v1 records (res.counts) the timed bench does not need. A level's tests run in chunks of
    `chunk_children` children (None: as many as `chunk_bytes` of both parties' buffers hold at
    ~512 B per test; 0: the whole level), one protocol instance per chunk (fhh_gc_party_cfg
    child_begin / child_count; the default material varies per chunk, a custom cfg_fn's does not),
    and the node sums follow the level's last chunk. `level_log` (a list) receives one
    (level, children, crawl_s, gcot_s, node_sums_s) tuple per level."""
    L = levels or c0.depth
    n_total = nclients_total if nclients_total is not None else c0.num_clients()
    thr = max(1, int(threshold * n_total))
    thr_last = max(1, min(int(threshold * n_total), 0xFFFFFFFF))
    user_cfg = cfg_fn

    def chunk_cfg(lv, k, j, S):
        if user_cfg is None:
            return level_cfg(prf_seed ^ (k << 40) ^ (j << 48), lv)
        return user_cfg(lv) if S == 1 else user_cfg(lv, k)
    # a multi-device collection runs each shard's protocol over its own channel (the reference
    # splits a level's tests over several channels, collect.rs:423-430)
    S = len(c0.shard_info()[0])
    shards = [(c0.shard(k), c1.shard(k)) for k in range(S)] if S > 1 else [(c0, c1)]
    if channel == "inplace" and any(a.device != b.device for a, b in shards):
        raise ValueError("two_party_crawl: an in-place channel needs both parties of a pair on one GPU")
    chans = [(Channel(a.device, channel), Channel(b.device, channel)) for a, b in shards]
    res = TwoPartyResult()
    c0.tree_init()
    c1.tree_init()
    from .fields import FE255_P, FE_P
    tm = timing if timing is not None else {}
    for k in ("crawl", "gcot", "node_sums", "keep", "prune"):
        tm.setdefault(k, 0.0)
    clock = time.perf_counter
    shard_clients = [a.num_clients() for a, _ in shards]
    if chunk_children is None:
        chunk_children = max(1, chunk_bytes // (_PARTY_BYTES_PER_TEST * max(1, max(shard_clients))))
    for lv in range(L):
        last = lv == L - 1
        t0 = clock()
        C0, _ = (c0.tree_crawl_last if last else c0.tree_crawl)()
        C1, _ = (c1.tree_crawl_last if last else c1.tree_crawl)()
        assert C0 == C1
        t1 = clock()
        sizes = {}
        for k, ((a, b), (to_gb, to_ev)) in enumerate(zip(shards, chans)):
            if shard_clients[k] == 0:
                continue
            for j, (cb, cc) in enumerate(chunk_windows(C0, chunk_children)):
                cfg = chunk_cfg(lv, k, j, S)
                cfg.child_begin, cfg.child_count = cb, cc
                for name, v in run_level(a, b, cfg, cfg, to_gb, to_ev).items():
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
            res.counts.append(np.array([((a % FE255_P) - (b % FE255_P)) % FE255_P for a, b in zip(s0, s1)], np.uint64))
        if expect_counts is not None and not np.array_equal(res.counts[-1], np.asarray(expect_counts[lv], np.uint64)):
            bad = np.nonzero(res.counts[-1] != np.asarray(expect_counts[lv], np.uint64))[0]
            raise ValueError(f"two-party crawl: level {lv}: {bad.size} of {C0} children differ (first {bad[:5]}: "
                             f"{res.counts[-1][bad[:5]]} vs {np.asarray(expect_counts[lv])[bad[:5]]})")
    res.final = KeyCollection.final_values(c0.final_shares(), c1.final_shares())
    return res


__all__ = ["Channel", "level_cfg", "run_level", "party_sums", "two_party_crawl", "TwoPartyResult", "chunk_windows"]
