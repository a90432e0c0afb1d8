"""Python mirror of the reference's garbled-circuit equality test:
`multiple_gb_equality_test` / `multiple_ev_equality_test` (src/equalitytest.rs:25-105) and the
`eq_gc` test's use of them (:222-266), backed by the HIP kernels in libfhh.so (fhh_gc.hip).

The two parties run in one process on one GPU: server 0's kernel garbles, server 1's evaluates.
The evaluator's input labels are handed over as an ideal OT would (the reference runs ALSZ OT
extension over its channel); the garbled tables, the garbler's active labels and the decoding
bits are the wire message, materialised in HBM between the two kernels. Garbling scheme and
label formats: include/fhh.h (fhh_gc_batch) and DESIGN.md §5.3.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ._lib import FhhGcBatch, check, lib, ptr, u64p

u8p = ctypes.POINTER(ctypes.c_uint8)


def _block(v) -> bytes:
    b = bytes(v)
    if len(b) != 16:
        raise ValueError("16-byte block expected")
    return b


@dataclass
class GcTranscript:
    """What the garbler sends (tables, its active labels incl. the mask wire, decoding bits) and
    what OT delivers to the evaluator (its active labels), AoS per test."""
    tables: np.ndarray      # [n][bits-1][2][16]
    gb_labels: np.ndarray   # [n][bits+1][16]
    ev_labels: np.ndarray   # [n][bits][16]
    decode: np.ndarray      # [n]


def equality_test(kc, gb_inputs, ev_inputs, mask: int, label_key, delta, label_nonce: int = 0, gate_base: int = 0,
                  transcript: bool = False):
    """Garble + evaluate n equality tests on the GPU. gb_inputs / ev_inputs: [n][bits] 0/1
    (the `Vec<u16>` share strings). Returns the evaluator's bits eq XOR mask [n] (and the
    transcript if asked)."""
    g = np.ascontiguousarray(np.asarray(gb_inputs).astype(np.uint8) & 1)
    e = np.ascontiguousarray(np.asarray(ev_inputs).astype(np.uint8) & 1)
    if g.ndim != 2 or g.shape != e.shape:
        raise ValueError("equality_test: inputs must both be [n][bits]")
    n, bits = g.shape
    out = np.zeros(n, np.uint8)
    key = np.frombuffer(_block(label_key), np.uint8).copy()
    dl = np.frombuffer(_block(delta), np.uint8).copy()
    tr = None
    if transcript:
        tr = GcTranscript(np.zeros((n, max(bits - 1, 0), 2, 16), np.uint8), np.zeros((n, bits + 1, 16), np.uint8),
                          np.zeros((n, bits, 16), np.uint8), np.zeros(n, np.uint8))
    check(lib().fhh_gc_equality_host(kc.handle, n, bits, ptr(g), ptr(e), int(mask) & 1, ptr(key), ptr(dl),
                                     label_nonce, gate_base,
                                     ptr(tr.tables) if tr else None, ptr(tr.gb_labels) if tr else None,
                                     ptr(tr.ev_labels) if tr else None, ptr(tr.decode) if tr else None, ptr(out)),
          kc.handle)
    return (out, tr) if transcript else out


def multiple_equality_test(kc, gb_value, ev_value, seed: int = 0):
    """Both parties of `multiple_gb_equality_test` + `multiple_ev_equality_test` for one
    channel: returns (masks, results) with masks[i] ^ results[i] == (gb_value[i] == ev_value[i])
    (the eq_gc assertion, equalitytest.rs:258-265). One mask bit per call: the reference draws
    `rng.clone().gen_bool()` per test from a clone that never advances (:38-43)."""
    rng = np.random.default_rng(seed)
    key = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    delta = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    mask = int(rng.integers(0, 2))
    res = equality_test(kc, gb_value, ev_value, mask, key, delta)
    return [bool(mask)] * len(res), [bool(r) for r in res]


class DeviceGcBatch:
    """G groups x N tests resident in HBM (torch tensors on the ctx's GPU): input bit planes
    [G][bits][nw] and the SoA transcript / output buffers of fhh_gc_batch."""

    def __init__(self, gb_planes: np.ndarray, ev_planes: np.ndarray, clients: int, mask: int, label_key, delta,
                 device: int = 0, label_nonce: int = 0, gate_base: int = 0):
        import torch
        dev = torch.device(f"cuda:{device}")
        G, bits, nw = gb_planes.shape
        if ev_planes.shape != gb_planes.shape or nw * 64 < clients or not 1 <= bits <= 8:
            raise ValueError("DeviceGcBatch: planes [G][bits][nw], nw >= ceil(clients / 64), bits in 1..8")
        self.G, self.bits, self.nw, self.N = G, bits, nw, clients
        n = G * clients
        self.n = n

        def t(a):
            return torch.from_numpy(np.ascontiguousarray(a, np.uint64).view(np.int64)).to(dev)

        self.gb_planes, self.ev_planes = t(gb_planes), t(ev_planes)
        u8 = torch.uint8
        self.tables = torch.empty((max(bits - 1, 1) * 2, n, 16), dtype=u8, device=dev)
        self.gb_labels = torch.empty((bits + 1, n, 16), dtype=u8, device=dev)
        self.ev_labels = torch.empty((bits, n, 16), dtype=u8, device=dev)
        self.decode = torch.empty(n, dtype=u8, device=dev)
        self.out = torch.empty(n, dtype=u8, device=dev)
        torch.cuda.synchronize(dev)   # the library runs on its own stream
        self.mask, self.key, self.delta = int(mask) & 1, _block(label_key), _block(delta)
        self.label_nonce, self.gate_base = label_nonce, gate_base

    def struct(self) -> FhhGcBatch:
        b = FhhGcBatch()
        b.groups, b.clients, b.words, b.bits, b.mask = self.G, self.N, self.nw, self.bits, self.mask
        b.label_key[:] = list(self.key)
        b.delta[:] = list(self.delta)
        b.label_nonce, b.gate_base = self.label_nonce, self.gate_base
        b.gb_planes_dev, b.ev_planes_dev = self.gb_planes.data_ptr(), self.ev_planes.data_ptr()
        b.tables_dev, b.gb_labels_dev = self.tables.data_ptr(), self.gb_labels.data_ptr()
        b.ev_labels_dev, b.decode_dev, b.out_dev = self.ev_labels.data_ptr(), self.decode.data_ptr(), self.out.data_ptr()
        return b


def equality_device(kc, batch: DeviceGcBatch) -> None:
    """Garbler then evaluator over a device-resident batch (fhh_gc_equality_device)."""
    b = batch.struct()
    check(lib().fhh_gc_equality_device(kc.handle, ctypes.byref(b)), kc.handle)


def planes_from_bits(bits_gn: np.ndarray) -> np.ndarray:
    """[G][N][bits] 0/1 -> bit planes [G][bits][ceil(N/64)] u64 (bit i % 64 of word i / 64)."""
    G, N, bits = bits_gn.shape
    nw = (N + 63) // 64
    pad = np.zeros((G, nw * 64, bits), np.uint8)
    pad[:, :N] = bits_gn & 1
    packed = np.packbits(pad.transpose(0, 2, 1).reshape(G, bits, nw, 64), axis=-1, bitorder="little")
    return np.ascontiguousarray(packed).view(np.uint64).reshape(G, bits, nw)


def equality_test_cot(kc, gb_inputs, ev_inputs, mask: int, base_seeds, base_choice, gate_base: int = 0,
                      ctr_off: int = 0, share: bool = False):
    """The labels step on the GPU (fhh_gc_cot_host): the evaluator's input labels by the labels OT (its
    bits are the choice bits; since r05b the IKNP correlation itself: zero label q_j, active label t_j,
    Delta = base_choice, whose bit 0 must be 1), garbling with the garbler's string and mask folded into
    the circuit, evaluation. Returns (out [n], dict of the transcript: tables, ev_zero, ev_active,
    decode; share (r05c): also gb_share, ev_share, share_y — the FE share from the output labels)."""
    g = np.ascontiguousarray(np.asarray(gb_inputs).astype(np.uint8) & 1)
    e = np.ascontiguousarray(np.asarray(ev_inputs).astype(np.uint8) & 1)
    if g.ndim != 2 or g.shape != e.shape:
        raise ValueError("equality_test_cot: inputs must both be [n][bits]")
    n, bits = g.shape
    seeds = np.ascontiguousarray(base_seeds, np.uint8).reshape(128, 2, 16)
    s = np.frombuffer(bytes(base_choice), np.uint8).copy()
    tr = {"tables": np.zeros((n, max(bits - 1, 0), 2, 16), np.uint8), "ev_zero": np.zeros((n, bits, 16), np.uint8),
          "ev_active": np.zeros((n, bits, 16), np.uint8), "decode": np.zeros(n, np.uint8)}
    out = np.zeros(n, np.uint8)
    sh = [np.zeros(n, np.uint64) for _ in range(3)] if share else [None] * 3
    check(lib().fhh_gc_cot_host(kc.handle, n, bits, ptr(g), ptr(e), int(mask) & 1, gate_base, ptr(seeds),
                                ptr(s), ctr_off, ptr(tr["tables"]), ptr(tr["ev_zero"]), ptr(tr["ev_active"]),
                                ptr(tr["decode"]), ptr(out), *(None if a is None else ptr(a, u64p) for a in sh)),
          kc.handle)
    if share:
        tr["gb_share"], tr["ev_share"], tr["share_y"] = sh
    return out, tr


def table_cot(kc, gb_inputs, ev_inputs, mask: int, base_seeds, base_choice, gate_base: int = 0, ctr_off: int = 0,
              ring32: bool = False):
    """r05d, the FE levels' form (fhh_gt_cot_host, bits <= 4): the labels OT, then one garbled table
    of 2^bits rows for "the share of eq ^ mask" (Yao's garbled gate, point-and-permute) instead of the
    half-gates chain. Returns dict: msgs [n][2^bits - 1] u64, gb_share / ev_share [n] (gb - ev = eq mod
    p), ev_zero / ev_active [n][bits][16]. ring32 (r06, bits <= 2; fhh_gt_cot_ring32_host): the shares in
    Z_2^32 (4-B messages; gb - ev = eq mod 2^32), returned zero-extended in the same arrays."""
    g = np.ascontiguousarray(np.asarray(gb_inputs).astype(np.uint8) & 1)
    e = np.ascontiguousarray(np.asarray(ev_inputs).astype(np.uint8) & 1)
    if g.ndim != 2 or g.shape != e.shape:
        raise ValueError("table_cot: inputs must both be [n][bits]")
    n, bits = g.shape
    seeds = np.ascontiguousarray(base_seeds, np.uint8).reshape(128, 2, 16)
    s = np.frombuffer(bytes(base_choice), np.uint8).copy()
    tr = {"ev_zero": np.zeros((n, bits, 16), np.uint8), "ev_active": np.zeros((n, bits, 16), np.uint8),
          "msgs": np.zeros((n, (1 << bits) - 1), np.uint64), "gb_share": np.zeros(n, np.uint64),
          "ev_share": np.zeros(n, np.uint64)}
    fn = lib().fhh_gt_cot_ring32_host if ring32 else lib().fhh_gt_cot_host
    check(fn(kc.handle, n, bits, ptr(g), ptr(e), int(mask) & 1, gate_base, ptr(seeds), ptr(s),
             ctr_off, ptr(tr["ev_zero"]), ptr(tr["ev_active"]), ptr(tr["msgs"], u64p),
             ptr(tr["gb_share"], u64p), ptr(tr["ev_share"], u64p)), kc.handle)
    return tr
