"""Host-side pieces of the two-party GC + OT driver (no GPU): the chunk windows a level's tests run
in (fhh_gc_party_cfg child_begin / child_count; the reference splits a level's tests over its
channels, collect.rs:423-430) and the ctypes layout of fhh_gc_party_cfg against include/fhh.h."""
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


def test_party_cfg_layout_matches_header():
    """fhh_gc_party_cfg (include/fhh.h): the r04 chunk fields follow the base-OT arrays; the ctypes
    mirror must have the C layout (no padding on x86-64: every field is naturally aligned)."""
    from fuzzyheavyhitters_amd._lib import FhhGcPartyCfg
    size = 16 + 16 + 4 + 4 + 8 + 2 * 128 * 2 * 16 + 2 * 128 * 16 + 2 * 16 + 8 + 8
    assert ctypes.sizeof(FhhGcPartyCfg) == size
    assert FhhGcPartyCfg.child_begin.offset == size - 16
    assert FhhGcPartyCfg.child_count.offset == size - 8
    cfg = FhhGcPartyCfg()
    assert cfg.child_begin == 0 and cfg.child_count == 0   # zero-initialised: the whole level
