"""OT extension on the GPU (the OT of SURVEY §8 row f1): IKNP in the ALSZ form, mirroring
`ocelot::ot::{AlszSender, AlszReceiver}` as the reference uses them (equalitytest.rs:67-82,
collect.rs:437-471), backed by fhh_ot.hip. Both parties run in one process; the 128 base OTs
are ideal. See include/fhh.h (fhh_ot_batch) for the exact construction."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from ._lib import check, lib, ptr


def ot_extend(kc, choices, x0, x1=None, delta=None, base_seeds=None, base_choice=None, tweak_base: int = 0,
              transcript: bool = False, seed: int | None = None):
    """m OTs: returns the receiver's messages out [m][16] with out[j] = (x1 if choices[j] else x0)[j]
    (x1 None: correlated OT, x1 = x0 ^ delta). With transcript, also (U [128][ceil(m/128)][16],
    Y0, Y1 [m][16]) — the two protocol messages.

    The base-OT material (the receiver's seed pairs, the sender's choice bits) must be fresh for
    every batch, as the reference's OtSender/OtReceiver::init per batch draws it
    (collect.rs:454-471): the row PRG restarts at counter 0, so reused material repeats the pads
    and U ^ U' would reveal the receiver's choices. When omitted it is drawn from os.urandom;
    `seed` (tests only) makes it reproducible instead."""
    ch = np.ascontiguousarray(np.asarray(choices).astype(np.uint8) & 1)
    m = ch.size
    a0 = np.ascontiguousarray(x0, np.uint8).reshape(m, 16)
    a1 = None if x1 is None else np.ascontiguousarray(x1, np.uint8).reshape(m, 16)
    if a1 is None and delta is None:
        raise ValueError("ot_extend: x1 or delta required")
    def fresh(k):
        if seed is not None:
            return np.random.default_rng([seed, k]).integers(0, 256, (128 * 2 * 16,) if k == 0 else (16,),
                                                            dtype=np.uint8)
        return np.frombuffer(os.urandom(128 * 2 * 16 if k == 0 else 16), np.uint8).copy()
    seeds = (fresh(0).reshape(128, 2, 16) if base_seeds is None
             else np.ascontiguousarray(base_seeds, np.uint8).reshape(128, 2, 16))
    s = fresh(1) if base_choice is None else np.frombuffer(bytes(base_choice), np.uint8).copy()
    d = np.frombuffer(bytes(delta), np.uint8).copy() if delta is not None else np.zeros(16, np.uint8)
    out = np.zeros((m, 16), np.uint8)
    nb = (m + 127) // 128
    u = np.zeros((128, nb, 16), np.uint8) if transcript else None
    y0 = np.zeros((m, 16), np.uint8) if transcript else None
    y1 = np.zeros((m, 16), np.uint8) if transcript else None
    check(lib().fhh_ot_extend_host(kc.handle, m, ptr(ch), ptr(a0), ptr(a1) if a1 is not None else None, ptr(d),
                                   ptr(seeds), ptr(s), tweak_base, ptr(out), ptr(u) if transcript else None,
                                   ptr(y0) if transcript else None, ptr(y1) if transcript else None), kc.handle)
    return (out, u, y0, y1) if transcript else out


def cot_extend(kc, mode: int, choices, base_seeds, base_choice, delta=None, mask: int = 0, ctr_off: int = 0,
               transcript: bool = False, ss_k: int = 1):
    """Correlated OT extension on the GPU (fhh_cot_extend_host; the r05 protocol's two OTs, see
    include/fhh.h FHH_COT_*): returns (sender_out, out) and, with transcript, (U, y) — and with ss_k > 1
    (r06, SoftSpoken OT extension with k = ss_k: fhh_cot_extend_ss_host) also the GGM corrections,
    (U [128 / ss_k][ceil(m / 128)][16], y, corr [128 / ss_k][ss_k][2][16]).
    mode 1 (labels): sender_out = x0 [m][16] (x1 = x0 ^ delta), out [m][16]; mode 2 (FE share):
    sender values / out [m] u64 (the garbler's r1 = v + mask, the receiver's share); mode 3 (FieldElm,
    OT pairs with one choice): sender values / out [m/2][32] BlockPairs; mode 4 (FHH_COT_RAW, the labels
    OT since r05b): sender_out = q [m][16], out = t [m][16] = q ^ r s, no y (zeros)."""
    if ss_k not in (1, 2, 4):
        raise ValueError("cot_extend: ss_k must be 1, 2 or 4")
    from ._lib import FHH_COT_FE, FHH_COT_FE255, FHH_COT_LABELS
    if mode == FHH_COT_LABELS and delta is None:
        raise ValueError("cot_extend: the labels mode needs delta (x1 = x0 ^ delta)")
    ch = np.ascontiguousarray(np.asarray(choices).astype(np.uint8) & 1)
    m = ch.size
    seeds = np.ascontiguousarray(base_seeds, np.uint8).reshape(128, 2, 16)
    s = np.frombuffer(bytes(base_choice), np.uint8).copy()
    d = np.frombuffer(bytes(delta), np.uint8).copy() if delta is not None else np.zeros(16, np.uint8)
    if mode == FHH_COT_FE:
        sx, out, y = np.zeros(m, np.uint64), np.zeros(m, np.uint64), np.zeros(m, np.uint64)
    elif mode == FHH_COT_FE255:
        sx, out, y = np.zeros((m // 2, 32), np.uint8), np.zeros((m // 2, 32), np.uint8), np.zeros((m, 16), np.uint8)
    else:
        sx, out, y = np.zeros((m, 16), np.uint8), np.zeros((m, 16), np.uint8), np.zeros((m, 16), np.uint8)
    u = np.zeros((128 // ss_k, (m + 127) // 128, 16), np.uint8) if transcript else None
    u8 = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
    if ss_k == 1:
        check(lib().fhh_cot_extend_host(kc.handle, m, mode, ptr(ch), ptr(d), int(mask) & 1, ptr(seeds), ptr(s),
                                        ctr_off, u8(sx), u8(out), ptr(u) if transcript else None,
                                        u8(y) if transcript else None), kc.handle)
        return (sx, out, u, y) if transcript else (sx, out)
    corr = np.zeros((128 // ss_k, ss_k, 2, 16), np.uint8) if transcript else None
    check(lib().fhh_cot_extend_ss_host(kc.handle, ss_k, m, mode, ptr(ch), ptr(d), int(mask) & 1, ptr(seeds), ptr(s),
                                       ctr_off, u8(sx), u8(out), ptr(u) if transcript else None,
                                       u8(y) if transcript else None, ptr(corr) if transcript else None), kc.handle)
    return (sx, out, u, y, corr) if transcript else (sx, out)
