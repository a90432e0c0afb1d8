"""One KeyCollection over several GPUs (fhh_create_multi; SURVEY §8(b) `fhh_create(..., devices,
n_devices)`, §8(e); north_star: "clients shard across the 8 GPUs, per-GPU partial prefix counts
combined with an RCCL all-reduce"). The reference server holds one KeyCollection
(src/bin/server.rs:44-52, 332-335; src/collect.rs:28-37); a multi-device collection must answer
every KeyCollection call exactly as the one-GPU collection does.

CPU: the placement (whole 64-client words per shard) and a numpy model of the share-plane gather.
GPU: a device list that repeats device 0 (two / three shards on one GPU: the host reduction, the
same fan-out code as distinct GPUs) against the one-GPU collection — the drop-in path level by
level (planes, FE and FieldElm node sums, prune, final shares), the device level loop, host
add_keys and the bincode payload, and node sums of device-resident values."""
import ctypes

import numpy as np
import pytest


@pytest.mark.parametrize("n,S", [(1, 1), (100, 4), (130, 2), (64 * 7 + 5, 3), (100_000, 8), (1_000_000, 8),
                                 (1_000_000, 3)])
def test_shard_plan_layout(n, S):
    """fhh_shard_plan: contiguous ranges covering [0, n) in client order, each starting on a
    64-client word, every shard but the last holding whole words, balanced to one word."""
    import fuzzyheavyhitters_amd as fhh
    plan = fhh.shard_plan(n, S)
    assert len(plan) == S
    pos = 0
    nw = (n + 63) // 64
    for k, (b, c) in enumerate(plan):
        assert b == pos and b % 64 == 0 or c == 0
        if c:
            pos = b + c
        words = (c + 63) // 64
        assert abs(words - nw / S) <= 1
        if k < S - 1 and c:
            assert c % 64 == 0 or b + c == n
    assert pos == n


def test_share_plane_gather_model():
    """What crawl_level's strided copy does for a shard: its planes [C][2d][nw_k] land in the
    collection's [C][2d][nw] rows at word base_k / 64 — reassembling the one-GPU planes."""
    import fuzzyheavyhitters_amd as fhh
    rng = np.random.default_rng(3)
    n, C, bits = 64 * 11 + 17, 5, 4
    nw = (n + 63) // 64
    full = rng.integers(0, 1 << 63, (C, bits, nw), dtype=np.uint64)
    full[:, :, -1] &= np.uint64((1 << (n % 64)) - 1)
    out = np.zeros_like(full)
    for b, c in fhh.shard_plan(n, 3):
        w0, wk = b // 64, (c + 63) // 64
        shard_planes = full[:, :, w0:w0 + wk].copy()      # what the shard computes on its clients
        out.reshape(C * bits, nw)[:, w0:w0 + wk] = shard_planes.reshape(C * bits, wk)
    assert np.array_equal(out, full)


import os

# a repeated device reduces on the host, unless the in-process RCCL branch is forced (test_rccl_stub.py)
_REPEATED = "rccl" if os.environ.get("FHH_GROUP_REDUCE") == "rccl" else "host"


def _pair(L, d, devices=None):
    import fuzzyheavyhitters_amd as fhh
    return fhh.KeyCollection(L, d, devices=devices), fhh.KeyCollection(L, d, devices=devices)


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0], [0, 0], [0, 0, 0]], ids=["1-shard", "2-shards", "3-shards"])
@pytest.mark.parametrize("d", [1, 2])
def test_group_drop_in_path_equals_single(devices, d):
    """tree_init / tree_crawl (share planes) / node_sums_fe / tree_prune level by level, then
    tree_crawl_last / node_sums_fe255 / tree_prune_last / final_shares: the multi-device collection
    returns exactly what the one-GPU collection returns (collect.rs:67-92, 370-505, 775-942)."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    n, L = 64 * 9 + 23, 20
    wl = workload.zipf_workload(n, 32, d, num_sites=6, seed=11)
    left, right = wl.left[:, :, :L].copy(), wl.right[:, :, :L].copy()
    s0, s1 = _pair(L, d)
    g0, g1 = _pair(L, d, devices)
    fhh.gen_keys_pair(s0, s1, left, right, wl.root_seeds)
    fhh.gen_keys_pair(g0, g1, left, right, wl.root_seeds)
    info, red = g0.shard_info()
    assert len(info) == len(devices) and sum(c for _, _, c in info) == n
    assert red == ("none" if len(devices) == 1 else _REPEATED)
    assert g0.num_clients() == n
    for a, b in zip(s1.export_keys(), g1.export_keys()):
        assert np.array_equal(a, b)
    rng = np.random.default_rng(5)
    thr = 3
    for kc in (s0, s1, g0, g1):
        kc.tree_init()
    for lv in range(L):
        last = lv == L - 1
        crawl = (lambda k: k.tree_crawl_last(share_planes=True)) if last else (lambda k: k.tree_crawl(share_planes=True))
        (C, ps0), (_, ps1), (Cg, pg0), (_, pg1) = [crawl(k) for k in (s0, s1, g0, g1)]
        assert C == Cg
        assert np.array_equal(ps0, pg0) and np.array_equal(ps1, pg1), f"share planes level {lv}"
        if lv == L // 2:
            for a, b in zip(s0.export_states(), g0.export_states()):
                assert np.array_equal(a, b), f"states level {lv}"
        # plaintext equality of the two servers' strings -> keep (the GC's output)
        diff = np.zeros((C, ps0.shape[2]), np.uint64)
        for j in range(2 * d):
            diff |= ps0[:, j] ^ ps1[:, j]
        eq = np.unpackbits(diff.view(np.uint8).reshape(C, -1, 8), axis=2, bitorder="little").reshape(C, -1)[:, :n] == 0
        keep = eq.sum(1) >= thr
        if not last:
            vals = rng.integers(0, 1 << 63, (C, n), dtype=np.uint64)
            assert np.array_equal(s0.node_sums_fe(vals), g0.node_sums_fe(vals)), f"FE sums level {lv}"
            for kc in (s0, s1, g0, g1):
                kc.tree_prune(keep)
            if not keep.any():
                break
        else:
            vals = rng.integers(0, 1 << 32, (C, n, 8), dtype=np.uint64).astype(np.uint32)
            us, cs = s0.node_sums_fe255(vals)
            ug, cg = g0.node_sums_fe255(vals)
            assert us == ug and cs == cg, "FieldElm sums"
            for kc in (s0, s1, g0, g1):
                kc.tree_prune_last(keep)
            fs, fg = s0.final_shares(), g0.final_shares()
            assert [(r.path, r.value) for r in fs] == [(r.path, r.value) for r in fg]
    assert s0.frontier_size() == g0.frontier_size()


@pytest.mark.gpu
@pytest.mark.parametrize("devices", [[0, 0], [0, 0, 0, 0]], ids=["2-shards", "4-shards"])
@pytest.mark.parametrize("mode,gc", [("count", False), ("fe", False), ("fe", "ot")], ids=["count", "fe", "gc-ot"])
def test_group_sim_crawl_equals_single(oracle, devices, mode, gc):
    """The device level loop over a multi-device collection (one thread per shard pair, the
    per-level all-reduce over the collection's communicators) gives the one-GPU crawl: every
    level's counts, kept sets and the final heavy hitters with their values."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    n, L = 64 * 13 + 5, 40
    wl = workload.zipf_workload(n, L, 1, num_sites=20, seed=21)
    s0, s1 = _pair(L, 1)
    g0, g1 = _pair(L, 1, devices)
    fhh.gen_keys_pair(s0, s1, wl.left, wl.right, wl.root_seeds)
    fhh.gen_keys_pair(g0, g1, wl.left, wl.right, wl.root_seeds)
    a = fhh.sim_crawl(s0, s1, 0.01, mode=mode, prf_seed=9, gc=gc)
    b = fhh.sim_crawl(g0, g1, 0.01, mode=mode, prf_seed=9, gc=gc)
    assert list(a.level_children) == list(b.level_children)
    assert list(a.level_kept) == list(b.level_kept)
    assert all(np.array_equal(x, y) for x, y in zip(a.counts, b.counts))
    assert [(r.path, r.value) for r in a.final] == [(r.path, r.value) for r in b.final]
    assert len(a.final) > 0
    assert g0.stats()["aes_blocks"] == s0.stats()["aes_blocks"]


@pytest.mark.gpu
def test_group_add_keys_and_bincode_placement(oracle):
    """Keys that arrive by add_key (staged, cut at tree_init) and by the add_keys RPC payload
    (each shard decodes its slice of the records on its GPU, rpc.rs:12-15) land on the shards as
    the one-GPU collection holds them, and crawl the same."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    n, L, d = 64 * 5 + 9, 24, 2
    wl = workload.zipf_workload(n, 32, d, num_sites=5, seed=4)
    k0, k1 = oracle.gen_keys(wl.left[:, :, :L].copy(), wl.right[:, :, :L].copy(), wl.root_seeds)
    s0, s1 = _pair(L, d)
    s0.add_keys(k0.key_idx, k0.root_seed, k0.cw_seed, k0.cw_bits)
    s1.add_keys(k1.key_idx, k1.root_seed, k1.cw_seed, k1.cw_bits)
    g0, _ = _pair(L, d, [0, 0, 0])
    half = n // 2   # two add_keys batches: staging appends in client order
    g0.add_keys(k0.key_idx[:half], k0.root_seed[:half], k0.cw_seed[:half], k0.cw_bits[:half])
    g0.add_keys(k0.key_idx[half:], k0.root_seed[half:], k0.cw_seed[half:], k0.cw_bits[half:])
    g1 = fhh.KeyCollection(L, d, devices=[0, 0, 0])
    g1.add_keys_bincode(workload.add_keys_request_bincode(k1.key_idx, k1.root_seed, k1.cw_seed, k1.cw_bits))
    for kc in (s0, s1, g0, g1):
        kc.tree_init()
    for a, b in zip(s0.export_keys(), g0.export_keys()):
        assert np.array_equal(a, b)
    for a, b in zip(s1.export_keys(), g1.export_keys()):
        assert np.array_equal(a, b)
    for lv in range(6):
        r = [k.tree_crawl(share_planes=True) for k in (s0, s1, g0, g1)]
        assert np.array_equal(r[0][1], r[2][1]) and np.array_equal(r[1][1], r[3][1])
        keep = np.ones(r[0][0], bool)
        keep[::3] = False
        for k in (s0, s1, g0, g1):
            k.tree_prune(keep)


@pytest.mark.gpu
def test_group_node_sums_of_device_values():
    """fhh_node_sums_fe(255)_device: OT outputs already on each shard's GPU (16-B blocks with the
    FE in bytes 0..7, BlockPairs for FieldElm, fastfield.rs:414-431, field.rs:465-492) summed
    without a host round trip equal the sums of the same values passed from the host."""
    import torch
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    from fuzzyheavyhitters_amd._lib import FHH_VALS_FE_BLOCK, FHH_VALS_FE255_BLOCKPAIR
    from fuzzyheavyhitters_amd.fields import FE255_P
    n, L = 64 * 6 + 30, 8
    wl = workload.zipf_workload(n, 32, 1, num_sites=3, seed=8)
    g0, g1 = _pair(L, 1, [0, 0])
    fhh.gen_keys_pair(g0, g1, wl.left[:, :, :L].copy(), wl.right[:, :, :L].copy(), wl.root_seeds)
    g0.tree_init()
    C, _ = g0.tree_crawl()
    info, _ = g0.shard_info()
    rng = np.random.default_rng(2)
    vals = rng.integers(0, 1 << 63, (C, n), dtype=np.uint64)
    blocks = np.zeros((C, n, 2), np.uint64)
    blocks[:, :, 0] = vals
    blocks[:, :, 1] = rng.integers(0, 1 << 63, (C, n), dtype=np.uint64)   # bytes 8..15 are not the value
    dev = [torch.from_numpy(np.ascontiguousarray(blocks[:, b:b + c]).view(np.int64)).cuda() for _, b, c in info]
    torch.cuda.synchronize()
    got = g0.node_sums_fe_device([t.data_ptr() for t in dev], 0, C, FHH_VALS_FE_BLOCK)
    assert np.array_equal(got, g0.node_sums_fe(vals))
    # the last level: FieldElm BlockPairs (32 big-endian bytes)
    g0.tree_prune(np.ones(C, bool))
    C, _ = g0.tree_crawl_last()
    ints = [[int(x) for x in row] for row in rng.integers(0, 1 << 62, (C, n), dtype=np.uint64)]
    ints = [[(v << 190) % FE255_P + v for v in row] for row in ints]
    raw = np.frombuffer(b"".join(v.to_bytes(32, "big") for row in ints for v in row), np.uint8).reshape(C, n, 32)
    limbs = np.frombuffer(b"".join(v.to_bytes(32, "little") for row in ints for v in row), np.uint32).reshape(C, n, 8)
    dev = [torch.from_numpy(np.ascontiguousarray(raw[:, b:b + c])).cuda() for _, b, c in info]
    torch.cuda.synchronize()
    unr, can = g0.node_sums_fe255_device([t.data_ptr() for t in dev], 0, C, FHH_VALS_FE255_BLOCKPAIR)
    unr2, can2 = g0.node_sums_fe255(np.ascontiguousarray(limbs))
    assert unr == unr2 and can == can2
    assert unr == [sum(row) for row in ints]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["count", "fe"])
def test_group_sim_crawl_agrees_on_growth_when_free_memory_differs(monkeypatch, capfd, mode):
    """The device loop grows its tables when a level overflows, choosing the capacity from this GPU's
    free memory (loop_entry_cap). Shards of one crawl must choose the same capacity — the abort level
    of every later batch and each rank's all-reduce sequence and count follow from it — so the choice
    is agreed over the loop's own reduction. FHH_TEST_TABLE_BYTES gives shard 0 ample room and shard 1
    none: the shards grow alike (the debug log shows one capacity sequence) and the crawl equals the
    one-GPU one, with several resumes from capacity 2."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    n, L = 64 * 13 + 5, 40
    wl = workload.zipf_workload(n, L, 1, num_sites=20, seed=21)
    s0, s1 = _pair(L, 1)
    g0, g1 = _pair(L, 1, [0, 0])
    fhh.gen_keys_pair(s0, s1, wl.left, wl.right, wl.root_seeds)
    fhh.gen_keys_pair(g0, g1, wl.left, wl.right, wl.root_seeds)
    a = fhh.sim_crawl(s0, s1, 0.01, mode=mode, prf_seed=9, init_capacity=2)
    monkeypatch.setenv("FHH_TEST_TABLE_BYTES", f"{1 << 40},0")
    monkeypatch.setenv("FHH_DEBUG_LOOP", "1")
    capfd.readouterr()
    b = fhh.sim_crawl(g0, g1, 0.01, mode=mode, prf_seed=9, init_capacity=2)
    err = capfd.readouterr().err
    caps = [ln for ln in err.splitlines() if "[fhh loop] entry cap" in ln]
    seq = lambda lines: [ln.split("need ")[1].split(" (")[0] for ln in lines]   # "need E -> cap" per growth
    roomy = seq(ln for ln in caps if not ln.endswith(" 0.0 GB available)"))
    tight = seq(ln for ln in caps if ln.endswith(" 0.0 GB available)"))
    assert len(tight) >= 2 and roomy == tight, err[-2000:]   # >= 2 growths, the same capacities on both
    assert list(a.level_children) == list(b.level_children)
    assert list(a.level_kept) == list(b.level_kept)
    assert all(np.array_equal(x, y) for x, y in zip(a.counts, b.counts))
    assert [(r.path, r.value) for r in a.final] == [(r.path, r.value) for r in b.final]
    assert len(a.final) > 0
