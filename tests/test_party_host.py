"""Host-side pieces of the two-party GC + OT driver (no GPU): the chunk windows a level's tests run
in (fhh_gc_party_cfg child_begin / child_count; the reference splits a level's tests over its
channels, collect.rs:423-430) and the ctypes layouts of fhh_gb_cfg / fhh_ev_cfg against include/fhh.h."""
import ctypes

import pytest


@pytest.mark.parametrize("C,chunk", [(0, 3), (1, 3), (5, 0), (5, 5), (5, 6), (7, 3), (476, 134), (1000, 1)])
def test_chunk_windows_cover_the_level_in_order(C, chunk):
    from fuzzyheavyhitters_amd.party import chunk_windows
    w = chunk_windows(C, chunk)
    if chunk <= 0 or C <= chunk:
        assert w == [(0, 0)]   # one instance, the whole level
        return
    assert w[0][0] == 0
    assert all(cnt > 0 and cnt <= chunk for _, cnt in w)
    assert all(b1 == b0 + c0 for (b0, c0), (b1, _) in zip(w, w[1:]))   # in order, no gap, no overlap
    assert w[-1][0] + w[-1][1] == C


def test_party_cfg_layouts_match_header():
    """fhh_gb_cfg / fhh_ev_cfg (include/fhh.h): the ctypes mirrors have the C layout (no padding on
    x86-64: every field is naturally aligned), the chunk window last (the garbler's: before r06's ot_ss_k)."""
    from fuzzyheavyhitters_amd._lib import FhhEvCfg, FhhGbCfg
    gb = 4 + 4 + 2 * 128 * 16 + 2 * 16 + 8 + 8 + 4 + 4
    ev = 2 * 128 * 2 * 16 + 4 + 4 + 8 + 8
    assert ctypes.sizeof(FhhGbCfg) == gb and ctypes.sizeof(FhhEvCfg) == ev
    assert FhhGbCfg.ot_ss_k.offset == gb - 8 and FhhEvCfg.ot_ss_k.offset == ev - 20
    for T, end in ((FhhGbCfg, gb - 8), (FhhEvCfg, ev)):
        assert T.child_begin.offset == end - 16 and T.child_count.offset == end - 8
        cfg = T()
        assert cfg.child_begin == 0 and cfg.child_count == 0   # zero-initialised: the whole level


def test_evaluator_cfg_carries_no_garbler_secret():
    """the evaluator's half never receives the garbler's secrets. fhh_ev_cfg holds only
    its base-OT key pairs and the chunk window; the mask, the base-OT receiver's choice bits (the labels
    kind's s is the circuit's Delta since r05b) and chosen keys exist only in fhh_gb_cfg, and the share
    PRF key is gone (the share values come from the correlated OT itself), as is the label key (the r05
    garbler draws no labels)."""
    from fuzzyheavyhitters_amd._lib import FhhEvCfg, FhhGbCfg
    ev_fields = {f for f, _ in FhhEvCfg._fields_}
    gb_fields = {f for f, _ in FhhGbCfg._fields_}
    # form, ot_ss_k: public protocol choices
    assert ev_fields == {"base_pairs", "form", "ot_ss_k", "child_begin", "child_count"}
    for secret in ("mask", "base_chosen", "base_choice"):
        assert secret in gb_fields and secret not in ev_fields
    assert "delta" not in gb_fields | ev_fields
    assert not any("seed" in f for f in gb_fields | ev_fields)
    # and the header agrees: the evaluator's entry points take only fhh_ev_cfg
    import os
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "fhh.h")).read()
    for fn in ("fhh_ev_ot_labels", "fhh_ev_evaluate", "fhh_ev_ot_shares"):
        decl = hdr[hdr.index("int " + fn + "("):]
        decl = decl[:decl.index(";")]
        assert "fhh_gb_cfg" not in decl and "mask" not in decl and "delta" not in decl


def test_party_python_sides_hold_their_own_material():
    """party.GarblerParty / EvaluatorParty draw their material themselves (os.urandom): the garbler's
    choice bits s of two base-OT runs differ and the labels run's s (the circuit's Delta) has its colour
    bit set, a chunk config carries the garbler's own s and chosen keys, and the evaluator's config is
    built from its own base-OT pairs only."""
    import numpy as np
    from fuzzyheavyhitters_amd.party import EvaluatorParty, GarblerParty
    gp, ep = GarblerParty(None), EvaluatorParty(None)
    sides = []
    for colour in (True, True, False):
        A, seed = ep.co15_start()
        B, (chosen, s) = gp.co15_receive(A, colour=colour)
        pairs = ep.co15_finish(seed, B)
        assert np.array_equal(chosen, pairs[np.arange(128), (np.unpackbits(s, bitorder="little"))])
        sides.append(s)
    assert sides[0][0] & 1 and sides[1][0] & 1 and bytes(sides[0]) != bytes(sides[1])
    base_gb = [(np.full((128, 16), 3, np.uint8), sides[0]), (np.full((128, 16), 5, np.uint8), sides[2])]
    a = GarblerParty(None).chunk_cfg(base_gb, 0, 3)
    assert bytes(a.base_choice)[:16] == bytes(sides[0]) and bytes(a.base_chosen)[:1] == b"\x03"
    pairs = [np.full((128, 2, 16), 7, np.uint8), np.full((128, 2, 16), 9, np.uint8)]
    e = EvaluatorParty.chunk_cfg(pairs, 3, 3)
    assert bytes(e.base_pairs)[:4] == b"\x07" * 4 and bytes(e.base_pairs)[-4:] == b"\x09" * 4
    assert (e.child_begin, e.child_count) == (3, 3)
