"""The C-ABI library loads and exports every symbol include/fhh.h declares (no GPU calls)."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "fhh.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    names = set(re.findall(r"\b(fhh_[a-z0-9_]+)\s*\(", hdr))
    return sorted(n for n in names if n not in ("fhh_allreduce_fn",))


def test_library_exports_header(fhh):
    lib = fhh.lib()
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), f"libfhh.so does not export {s}"
    from fuzzyheavyhitters_amd._lib import EXPORTS
    assert sorted(EXPORTS) == syms


def test_host_only_entry_points(fhh):
    """Pure-host helpers run without a GPU: keep_values / final_values arithmetic."""
    import numpy as np
    from fuzzyheavyhitters_amd.collection import KeyCollection
    P = fhh.FE_P
    keep = KeyCollection.keep_values(10, 3, [5, 2 + P, 7], [1, 0, 5])
    assert list(keep) == [True, False, False]
    P2 = fhh.FE255_P
    k2 = KeyCollection.keep_values_last(10, 2, [P2 + 5, 3 * P2 + 1, 7], [2, P2 + 0, 6])
    assert list(k2) == [True, False, False]
    from fuzzyheavyhitters_amd.collection import Result
    fv = KeyCollection.final_values([Result([[True]], 2 * P2 + 9)], [Result([[True]], 4)])
    assert fv[0].value == 5
    fv = KeyCollection.final_values([Result([[True]], 1)], [Result([[True]], 4)])
    assert fv[0].value == P2 - 3


def test_create_fails_cleanly_without_gpu(fhh):
    import torch
    if torch.cuda.is_available():
        return
    lib = fhh.lib()
    h = ctypes.c_void_p()
    rc = lib.fhh_create(ctypes.byref(h), 8, 1, 0)
    assert rc != 0
    assert lib.fhh_last_error(None)


def test_sketch_impl_switch_validates(fhh):
    """fhh_sketch_set_impl (the k_sketch_fe A/B switch) accepts 0..4 and rejects the rest; no GPU
    call is made."""
    lib = fhh.lib()
    assert lib.fhh_sketch_set_impl(5) != 0
    assert lib.fhh_sketch_set_impl(-1) != 0
    for impl in (1, 2, 3, 4, 0):
        assert lib.fhh_sketch_set_impl(impl) == 0


def sketch_plan(lib, n, nodes, waves=4096):
    import ctypes
    nm, lm, lt = ctypes.c_uint64(), ctypes.c_int(), ctypes.c_int()
    assert lib.fhh_sketch_plan(n, nodes, waves, ctypes.byref(nm), ctypes.byref(lm), ctypes.byref(lt)) == 0
    return nm.value, lm.value, lt.value


def test_sketch_plan(fhh):
    """k_sketch_fe's launch plan (host arithmetic): configs[4] (100k keys x 256 nodes on 4096 waves)
    runs 3 full rounds at 8 lanes per key and the 1 696 keys left at 64 (29 passes instead of the 36
    of 8 lanes throughout); small launches take one launch at the lanes-per-key with the fewest
    passes; every plan covers the keys exactly once with a power-of-two lanes-per-key."""
    lib = fhh.lib()
    assert sketch_plan(lib, 100_000, 256) == (98_304, 8, 64)
    assert sketch_plan(lib, 98_304, 256) == (98_304, 8, 8)       # whole rounds: one launch
    assert sketch_plan(lib, 1001, 256) == (1001, 64, 64)         # one round of 2 passes
    assert sketch_plan(lib, 1, 0) == (1, 8, 8)
    assert sketch_plan(lib, 40_000, 256)[0] < 40_000             # the GPU test's split case
    for n in (1, 7, 64, 4095, 4097, 32_768, 33_000, 100_000, 250_001, 1_000_000):
        for nodes in (0, 1, 13, 256, 1000):
            n_main, lm, lt = sketch_plan(lib, n, nodes)
            assert 0 < n_main <= n and lm in (8, 16, 32, 64) and lt in (8, 16, 32, 64)
            if n_main < n:   # a split: whole rounds of the main launch
                assert n_main % (4096 * (64 // lm)) == 0
    import ctypes
    x = ctypes.c_uint64()
    y = ctypes.c_int()
    assert lib.fhh_sketch_plan(10, 10, 0, ctypes.byref(x), ctypes.byref(y), ctypes.byref(y)) != 0
