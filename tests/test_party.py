"""The two servers' halves of the GC equality test + OT, each on its own ctx (fhh_gb_* / fhh_ev_*;
src/collect.rs:419-482 with gc_sender = true on server 0 and false on server 1,
src/equalitytest.rs:25-106). Only protocol messages cross (party.Channel copies them into memory the
receiving server owns): the Chou–Orlandi base-OT messages of every level and the four messages per
chunk (two of them empty at the FE levels since r05c/r05d). Each server draws its own material (material="fresh"), or both come from one test seed
(material="test"); either way the leader's output equals the in-process GC + OT crawl
(fhh_sim_config.gc = 2) level by level, and its heavy hitters equal the plaintext recount."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _keys(wl, L, d, devices=None):
    import fuzzyheavyhitters_amd as fhh
    c0 = fhh.KeyCollection(L, d, devices=devices)
    c1 = fhh.KeyCollection(L, d, devices=devices)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    return c0, c1


def _assert_same_crawl(a, b):
    assert list(a.level_children) == list(b.level_children)
    for lv, (x, y) in enumerate(zip(a.counts, b.counts)):
        assert np.array_equal(np.asarray(x, np.uint64), np.asarray(y, np.uint64)), f"level {lv}"
    assert [(r.path, r.value) for r in a.final] == [(r.path, r.value) for r in b.final]


@pytest.mark.parametrize("material", ["fresh", "test"])
@pytest.mark.parametrize("channel", ["copy", "inplace"])
@pytest.mark.parametrize("d,n,L,thr", [(1, 300, 24, 0.02), (2, 200, 12, 0.05), (1, 64 * 3, 20, 0.03)],
                         ids=["d1", "d2", "whole-words"])
def test_two_party_equals_in_process_gc_ot(d, n, L, thr, channel, material):
    """Level by level: the leader's v0 - v1 per child and the final heavy hitters of the split run
    equal fhh_sim_crawl(gc = "ot") (both parties in one device loop), whether each server drew its own
    material and ran CO15 base OTs with the other ("fresh") or both sides come from one test seed, and
    whether each message is copied into the receiver's buffer or read where the sender produced it."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    wl = workload.zipf_workload(n, max(L, 32), d, num_sites=5, seed=3 + d)
    wl.left, wl.right = wl.left[:, :, :L].copy(), wl.right[:, :, :L].copy()
    c0, c1 = _keys(wl, L, d)
    ref = fhh.sim_crawl(c0, c1, thr, mode="fe", prf_seed=77, gc="ot")
    p0, p1 = _keys(wl, L, d)
    got = fhh.two_party_crawl(p0, p1, thr, prf_seed=77, channel=channel, material=material)
    _assert_same_crawl(ref, got)
    assert len(got.final) > 0
    if material == "fresh":   # one CO15 run per level (labels) + the FieldElm level's share OT, A + 128 B each
        assert got.base_ot_runs == L + 1 and got.base_ot_bytes == (L + 1) * 65 * 129
    t = max(1, int(thr * n))
    cnt, paths, vals = workload.plaintext_crawl(wl.left, wl.right, t, t)
    assert sorted(tuple(tuple(int(b) for b in p) for p in r.path) for r in got.final) == sorted(paths)
    # message sizes (the bytes that would cross the servers' channel)
    lb = got.level_bytes[0]
    C0, bits = int(got.level_children[0]), 2 * d
    # r06: d = 1 runs the tile-major table (OT index over whole 512-client tiles), d = 2 the row-major one
    npad = (n + 511) // 512 * 512 if bits <= 2 else (n + 63) // 64 * 64
    # r05d: the FE levels' gc message is the garbled table's rows 1 .. 2^bits - 1, 8 B each
    assert lb["gc"] == C0 * n * ((1 << bits) - 1) * 8
    # r05b: the labels OT is the IKNP correlation itself (no reply); r05c: no share OT at the FE levels
    assert lb["u1"] == 16 * ((C0 * bits * npad + 8191) // 8192 * 8192)
    assert lb["y1"] == 0 and lb["u2"] == 0 and lb["y2"] == 0
    # the FieldElm level keeps its share OT: U and 16 B per OT, 2 OTs per test
    lbl, Cl = got.level_bytes[-1], int(got.level_children[-1])
    assert lbl["gc"] == Cl * n * (2 * (bits - 1) * 16 + 1) and lbl["y2"] == Cl * n * 2 * 16


@pytest.mark.parametrize("ss_k", [2, 4])
@pytest.mark.parametrize("form", ["table", "circuit"])
@pytest.mark.parametrize("d,n,L,thr", [(1, 300, 20, 0.02), (2, 200, 12, 0.05)], ids=["d1", "d2"])
def test_two_party_softspoken(d, n, L, thr, form, ss_k):
    """r06: both parties on SoftSpoken OT extension (ot_ss_k = 2, 4; each its own material and CO15 base
    OTs over the channel) equal the in-process SoftSpoken crawl and the IKNP run level by level; the U
    messages shrink to 128 / k rows plus 4 KiB of GGM corrections."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    wl = workload.zipf_workload(n, 32, d, num_sites=5, seed=60 + d)
    wl.left, wl.right = wl.left[:, :, :L].copy(), wl.right[:, :, :L].copy()
    gc = "ot" if form == "table" else "ot-circuit"
    c0, c1 = _keys(wl, L, d)
    ref = fhh.sim_crawl(c0, c1, thr, mode="fe", prf_seed=5, gc=gc, ot_ss_k=ss_k)
    p0, p1 = _keys(wl, L, d)
    got = fhh.two_party_crawl(p0, p1, thr, form=form, ot_ss_k=ss_k)
    _assert_same_crawl(ref, got)
    t0, t1 = _keys(wl, L, d)
    iknp = fhh.two_party_crawl(t0, t1, thr, form=form)
    _assert_same_crawl(iknp, got)
    bits = 2 * d
    for lv, (a, b) in enumerate(zip(got.level_bytes, iknp.level_bytes)):
        C = int(got.level_children[lv])
        for key in ("u1", "u2"):
            if b.get(key, 0):
                assert a[key] == b[key] // ss_k + 4096, (lv, key)
        assert a["gc"] == b["gc"] and a["y2"] == b["y2"]
    assert len(got.final) > 0


@pytest.mark.parametrize("d,n,L,thr", [(1, 300, 20, 0.02), (2, 200, 12, 0.05)], ids=["d1", "d2"])
def test_two_party_circuit_form(d, n, L, thr):
    """form="circuit" (both parties: the half-gates circuit + output-label share at every FE level,
    r05c) equals fhh_sim_crawl(gc="ot-circuit") and the table form level by level; its gc message is the
    tables, the 8-B share y and the decoding bit per test."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    wl = workload.zipf_workload(n, 32, d, num_sites=5, seed=40 + d)
    wl.left, wl.right = wl.left[:, :, :L].copy(), wl.right[:, :, :L].copy()
    c0, c1 = _keys(wl, L, d)
    ref = fhh.sim_crawl(c0, c1, thr, mode="fe", prf_seed=5, gc="ot-circuit")
    p0, p1 = _keys(wl, L, d)
    got = fhh.two_party_crawl(p0, p1, thr, form="circuit")
    _assert_same_crawl(ref, got)
    t0, t1 = _keys(wl, L, d)
    _assert_same_crawl(got, fhh.two_party_crawl(t0, t1, thr, form="table"))
    lb, C0, bits = got.level_bytes[0], int(got.level_children[0]), 2 * d
    assert lb["gc"] == C0 * n * (2 * (bits - 1) * 16 + 8 + 1) and lb["u2"] == 0 and lb["y2"] == 0


def test_two_party_fresh_randomness_same_output():
    """Independently drawn material (each party's own label keys, Deltas, masks and CO15 base OTs) in
    two runs: every transcript differs, the leader's output does not, and equals the test-seed run's;
    with one base-OT run per OT kind for the whole crawl (the library continues its counters) too."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    n, L = 250, 20
    wl = workload.zipf_workload(n, 32, 1, num_sites=4, seed=12)
    wl.left, wl.right = wl.left[:, :, :L].copy(), wl.right[:, :, :L].copy()
    runs = []
    for kw in (dict(material="test", prf_seed=1), dict(material="fresh"), dict(material="fresh"),
               dict(material="fresh", base_ot_every="crawl")):
        a0, a1 = _keys(wl, L, 1)
        runs.append(fhh.two_party_crawl(a0, a1, 0.02, **kw))
    for r in runs[1:]:
        _assert_same_crawl(runs[0], r)
    assert runs[3].base_ot_runs == 2 and runs[1].base_ot_runs == L + 1


@pytest.mark.parametrize("channel", ["copy", "inplace"])
def test_two_party_multi_device_shards(channel):
    """A multi-device collection runs one protocol instance per shard over its own channel (the
    reference spreads a level's tests over several channels, collect.rs:423-430) and reduces the
    parties' device-resident sums over its shards: same output as the one-GPU in-process crawl."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    n, L = 64 * 7 + 11, 24
    wl = workload.zipf_workload(n, 32, 1, num_sites=6, seed=31)
    wl.left, wl.right = wl.left[:, :, :L].copy(), wl.right[:, :, :L].copy()
    c0, c1 = _keys(wl, L, 1)
    ref = fhh.sim_crawl(c0, c1, 0.02, mode="fe", prf_seed=5, gc="ot")
    g0, g1 = _keys(wl, L, 1, devices=[0, 0, 0])
    got = fhh.two_party_crawl(g0, g1, 0.02, channel=channel)
    _assert_same_crawl(ref, got)


def test_party_calls_out_of_order_refused():
    """Each half checks the protocol order and the message sizes (FHH_E_STATE / FHH_E_ARG)."""
    from fuzzyheavyhitters_amd import party, workload
    from fuzzyheavyhitters_amd._lib import lib
    wl = workload.zipf_workload(100, 32, 1, num_sites=3, seed=1)
    c0, c1 = _keys(wl, 32, 1)
    out, nb = ctypes.c_void_p(), ctypes.c_uint64()
    gb, ev = party.test_cfgs(1, 0)
    assert lib().fhh_ev_ot_labels(c1.handle, ctypes.byref(ev), ctypes.byref(out), ctypes.byref(nb)) == -2   # no crawl
    c0.tree_init()
    c1.tree_init()
    c0.tree_crawl()
    c1.tree_crawl()
    assert lib().fhh_gb_garble(c0.handle, ctypes.byref(out), ctypes.byref(nb)) == -2        # before the labels OT
    assert lib().fhh_ev_evaluate(c1.handle, None, 0, None, 0, ctypes.byref(out), ctypes.byref(nb)) == -2
    assert lib().fhh_ev_ot_labels(c1.handle, ctypes.byref(ev), ctypes.byref(out), ctypes.byref(nb)) == 0
    u, un = out.value, nb.value
    assert lib().fhh_gb_ot_labels(c0.handle, ctypes.byref(gb), out, 12345, ctypes.byref(out), ctypes.byref(nb)) == -1
    assert b"expected" in lib().fhh_last_error(c0.handle)
    assert lib().fhh_gb_ot_labels(c0.handle, ctypes.byref(gb), ctypes.c_void_p(u), un, ctypes.byref(out),
                                  ctypes.byref(nb)) == 0
    assert lib().fhh_gb_ot_shares(c0.handle, None, 0, ctypes.byref(out), ctypes.byref(nb)) == -2   # before garble


@pytest.mark.parametrize("chunk", [None, 150], ids=["whole-levels", "chunks-of-150"])
def test_two_party_configs1_full_size(chunk):
    """configs[1] at full size (100 000 Zipf clients, data_len 512, threshold 0.001): the split
    GC + OT crawl — each server drawing its own material, and every level's OT extension on
    Chou–Orlandi base OTs run between the servers over the channel (513 runs: the share OT at the
    FieldElm level only) — equals the
    in-process GC + OT crawl level by level, and both equal the plaintext recount (222 heavy hitters);
    with each level's tests in one protocol instance, and in chunks of 150 children, one instance per
    chunk (the 1M configuration's shape). Prints the bytes that would cross the channel."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    n, L = 100_000, 512
    wl = workload.zipf_workload(n, L, 1, num_sites=10_000, zipf_s=1.03, seed=0x5EED)
    c0, c1 = _keys(wl, L, 1)
    ref = fhh.sim_crawl(c0, c1, 0.001, mode="fe", prf_seed=7, gc="ot")
    del c0, c1
    p0, p1 = _keys(wl, L, 1)
    got = fhh.two_party_crawl(p0, p1, 0.001, expect_counts=ref.counts, material="fresh",
                              chunk_children=chunk, channel="inplace" if chunk else "copy")
    _assert_same_crawl(ref, got)
    assert len(got.final) == 222
    assert got.base_ot_runs == L + 1
    print(f"base OTs: {got.base_ot_runs} CO15 runs, {got.base_ot_bytes} B, crawl waited {got.base_ot_wait_s:.3f} s")
    if chunk:
        assert max(got.level_children) > chunk
    tot = {k: sum(lb[k] for lb in got.level_bytes) for k in got.level_bytes[0]}
    print("configs[1] two-party channel bytes per crawl:", tot, "max per level:",
          max(sum(lb.values()) for lb in got.level_bytes))


@pytest.mark.parametrize("chunk,devices", [(1, None), (3, None), (2, [0, 0])], ids=["1-child", "3-children", "2-shards"])
def test_two_party_chunked_children(chunk, devices):
    """A level's tests in chunks of children, one protocol instance per chunk (fhh_gc_party_cfg
    child_begin / child_count; the reference splits a level's tests over its channels,
    collect.rs:423-430), each chunk with its own label key, Delta, mask and base OTs: the leader's
    v0 - v1 per child and the heavy hitters equal the in-process crawl's (the node sums follow the
    level's last chunk)."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    n, L = 64 * 4 + 9, 24
    wl = workload.zipf_workload(n, 32, 1, num_sites=6, seed=41)
    wl.left, wl.right = wl.left[:, :, :L].copy(), wl.right[:, :, :L].copy()
    c0, c1 = _keys(wl, L, 1)
    ref = fhh.sim_crawl(c0, c1, 0.02, mode="fe", prf_seed=9, gc="ot")
    p0, p1 = _keys(wl, L, 1, devices=devices)
    got = fhh.two_party_crawl(p0, p1, 0.02, prf_seed=9, channel="inplace", chunk_children=chunk, material="test")
    _assert_same_crawl(ref, got)
    assert max(ref.level_children) > chunk   # some level really ran in several chunks


def test_party_chunks_out_of_order_refused():
    """Chunks run in order and cover the level before the node sums (FHH_E_STATE)."""
    from fuzzyheavyhitters_amd import party, workload
    from fuzzyheavyhitters_amd._lib import lib
    wl = workload.zipf_workload(100, 32, 1, num_sites=3, seed=1)
    c0, c1 = _keys(wl, 32, 1)
    c0.tree_init()
    c1.tree_init()
    C, _ = c0.tree_crawl()
    c1.tree_crawl()
    assert C == 2
    out, nb = ctypes.c_void_p(), ctypes.c_uint64()
    gb, ev = party.test_cfgs(1, 0)
    ev.child_begin, ev.child_count = 1, 1        # the level's first chunk must start at child 0
    assert lib().fhh_ev_ot_labels(c1.handle, ctypes.byref(ev), ctypes.byref(out), ctypes.byref(nb)) == -2
    for cfg in (gb, ev):
        cfg.child_begin, cfg.child_count = 0, 1
    to_gb, to_ev = party.Channel(0, "inplace"), party.Channel(0, "inplace")
    party.run_chunk(c0, c1, gb, ev, to_gb, to_ev)   # child 0 only
    sums = np.zeros(2, np.uint64)
    assert lib().fhh_party_node_sums(c0.handle, sums.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), None) == -2
    for cfg in (gb, ev):
        cfg.child_begin = 1
    party.run_chunk(c0, c1, gb, ev, to_gb, to_ev)   # child 1: the level is covered
    assert lib().fhh_party_node_sums(c0.handle, sums.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), None) == 0
