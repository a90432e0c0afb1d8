"""GPU parity: the HIP path (through the C ABI) against the CPU oracle and the golden
fixtures — bit-exact for keys, seeds, control bits, share bits, counts and field sums."""
import glob
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = sorted(glob.glob(os.path.join(HERE, "golden", "zipf_d*_n*_L*.npz")))   # make_golden.py fixtures


def load(path):
    z = np.load(path, allow_pickle=False)
    return {k: z[k] for k in z.files}


@pytest.fixture(scope="module")
def kc():
    import torch
    assert torch.cuda.is_available(), "GPU tests need a GPU"
    from fuzzyheavyhitters_amd import KeyCollection, gen_keys_pair
    return KeyCollection, gen_keys_pair


def make_pair(kc, left, right, roots):
    KeyCollection, gen_keys_pair = kc
    n, d, L = left.shape
    c0, c1 = KeyCollection(L, d), KeyCollection(L, d)
    gen_keys_pair(c0, c1, left, right, roots)
    return c0, c1


def add_pair(kc, k0, k1):
    KeyCollection, _ = kc
    n, d, _, L = k0.cw_bits.shape
    c0, c1 = KeyCollection(L, d), KeyCollection(L, d)
    c0.add_keys(k0.key_idx, k0.root_seed, k0.cw_seed, k0.cw_bits)
    c1.add_keys(k1.key_idx, k1.root_seed, k1.cw_seed, k1.cw_bits)
    return c0, c1


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(c) for c in CASES])
def test_gpu_keygen_bit_exact(kc, oracle, path):
    g = load(path)
    k0, k1 = oracle.gen_keys(g["left"], g["right"], g["root_seeds"])
    c0, c1 = make_pair(kc, g["left"], g["right"], g["root_seeds"])
    for c, k in ((c0, k0), (c1, k1)):
        ki, rs, cs, cb = c.export_keys()
        assert np.array_equal(ki, k.key_idx)
        assert np.array_equal(rs, k.root_seed)
        assert np.array_equal(cs, k.cw_seed), "cor_words seeds differ"
        assert np.array_equal(cb, k.cw_bits), "cor_words bits differ"
    assert np.array_equal(cs, g["cw_seed"]) and np.array_equal(cb, g["cw_bits"])


def test_keygen_ragged_and_tiny(kc, oracle):
    from fuzzyheavyhitters_amd import workload
    for n in (1, 63, 64, 65, 130):
        wl = workload.zipf_workload(n, 32, 1, num_sites=3, seed=n)
        k0, k1 = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
        c0, c1 = make_pair(kc, wl.left, wl.right, wl.root_seeds)
        _, _, cs, cb = c1.export_keys()
        assert np.array_equal(cs, k1.cw_seed) and np.array_equal(cb, k1.cw_bits)


GENERIC_AES_VARIANT = 33   # T-table k_expand with the generic AES (the default, 52, shares rounds 1-2 of sibling pairs)
# (the r01-r03 A/B forms — bitsliced, hybrid, pair-sliced — were removed in r06; git history at 78c7ebe)


def _need_variant(v):
    """Every variant id the tests name is in the build (52 and 33)."""
    if v is None:
        return
    from fuzzyheavyhitters_amd import lib
    assert lib().fhh_variant_info(v, None, 0, None, None) == 0, f"k_expand variant {v} not in this build"


@pytest.mark.parametrize("variant", [None, GENERIC_AES_VARIANT], ids=["default", "generic-aes"])
@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(c) for c in CASES])
def test_level_states_bit_exact(kc, oracle, path, variant):
    """Every level: EvalState seeds/t/y of all children, share planes and equality counts
    equal the oracle's (reference child order), pruning with the oracle's keep masks."""
    _need_variant(variant)
    g = load(path)
    n, d, L, _, _ = [int(x) for x in g["meta"]]
    k0, k1 = oracle.gen_keys(g["left"], g["right"], g["root_seeds"])
    for build in ("gen", "add"):
        c0, c1 = make_pair(kc, g["left"], g["right"], g["root_seeds"]) if build == "gen" else add_pair(kc, k0, k1)
        if variant is not None:
            c0.set_variant(variant)
            c1.set_variant(variant)
        c0.tree_init()
        c1.tree_init()
        if variant is not None:   # the keys export unchanged after a variant switch
            _, rs, cs, cb = c1.export_keys()
            assert np.array_equal(rs, k1.root_seed) and np.array_equal(cs, k1.cw_seed)
            assert np.array_equal(cb, k1.cw_bits)
        s0, s1 = oracle.tree_init(k0), oracle.tree_init(k1)
        seeds, t, y = c0.export_states()
        assert np.array_equal(seeds, s0.seed) and np.array_equal(t, s0.t) and np.array_equal(y, s0.y)
        parents = np.zeros(1, np.uint64)
        thr = max(1, int(float(g["threshold"][0]) * n))
        from fuzzyheavyhitters_amd.collection import sim_eq_count
        for lvl in range(min(L, 12 if build == "add" else L)):
            o0, _ = oracle.level_expand(k0, s0, parents, lvl)
            o1, _ = oracle.level_expand(k1, s1, parents, lvl)
            C, planes = c0.tree_crawl(share_planes=True)
            C1, _ = c1.tree_crawl()
            assert C == C1 == o0.t.shape[0]
            gs, gt, gy = c0.export_states()
            assert np.array_equal(gt, o0.t), f"t bits level {lvl}"
            assert np.array_equal(gy, o0.y), f"y bits level {lvl}"
            assert np.array_equal(gs, o0.seed), f"seeds level {lvl}"
            gs1, gt1, gy1 = c1.export_states()
            assert np.array_equal(gs1, o1.seed) and np.array_equal(gt1, o1.t) and np.array_equal(gy1, o1.y)
            # share planes: [C][2d][nw] bit (client % 64)
            sb = oracle.share_bits(o0)           # [C][n][2d]
            if C:
                bits = ((planes[:, :, np.arange(n) // 64] >> (np.arange(n, dtype=np.uint64) % 64)) & 1)
                assert np.array_equal(bits.transpose(0, 2, 1).astype(np.uint8), sb)
            cnt = sim_eq_count(c0, c1, C)
            assert np.array_equal(cnt, oracle.eq_counts(o0, o1))
            keep = cnt >= thr
            c0.tree_prune(keep)
            c1.tree_prune(keep)
            parents = np.nonzero(keep)[0].astype(np.uint64)
            s0, s1 = o0, o1
            if parents.size == 0:
                break


@pytest.mark.parametrize("variant", [None, GENERIC_AES_VARIANT], ids=["default-pair-aes", "generic-aes"])
@pytest.mark.parametrize("d", [1, 2])
def test_prg_counter_carry_seeds(kc, oracle, variant, d):
    """Root seeds whose byte 8 is 0xFF: the right child's counter (+1 in the upper u64 lane,
    prg.rs:273-276) carries into byte 9, 11 or wraps bytes 8..15 — the carry fallback of the
    sibling-pair AES — at level 0, every client pattern
    in every wave. Seeds / t / y of the first levels equal the oracle's."""
    _need_variant(variant)
    from fuzzyheavyhitters_amd import workload
    from fuzzyheavyhitters_amd.collection import sim_eq_count
    n, L = 200, 32
    wl = workload.zipf_workload(n, L, d, num_sites=4, seed=99)
    roots = wl.root_seeds.copy()                      # [n][d][side][server][16]
    pat = np.arange(n) % 5
    roots[pat == 1, :, :, :, 8] = 0xFF                 # carry into byte 9
    roots[pat == 2, :, :, :, 8:12] = 0xFF              # carry into byte 12
    roots[pat == 3, :, :, :, 8:16] = 0xFF              # upper lane wraps to 0
    roots[pat == 4, :, 0, :, 8] = 0xFF                 # left keys only
    k0, k1 = oracle.gen_keys(wl.left, wl.right, roots)
    c0, c1 = make_pair(kc, wl.left, wl.right, roots)
    if variant is not None:
        c0.set_variant(variant)
        c1.set_variant(variant)
    c0.tree_init()
    c1.tree_init()
    s0, s1 = oracle.tree_init(k0), oracle.tree_init(k1)
    parents = np.zeros(1, np.uint64)
    for lvl in range(3):
        o0, _ = oracle.level_expand(k0, s0, parents, lvl)
        o1, _ = oracle.level_expand(k1, s1, parents, lvl)
        C, _ = c0.tree_crawl()
        c1.tree_crawl()
        for c, o in ((c0, o0), (c1, o1)):
            gs, gt, gy = c.export_states()
            assert np.array_equal(gs, o.seed), f"seeds level {lvl}"
            assert np.array_equal(gt, o.t) and np.array_equal(gy, o.y), f"t/y level {lvl}"
        cnt = sim_eq_count(c0, c1, C)
        keep = cnt >= 1
        c0.tree_prune(keep)
        c1.tree_prune(keep)
        parents = np.nonzero(keep)[0].astype(np.uint64)
        s0, s1 = o0, o1


@pytest.mark.parametrize("d,ball,thr", [(3, 0, 0.01), (3, 1, 0.03), (4, 0, 0.01), (4, 1, 0.03)])
@pytest.mark.parametrize("mode", ["count", "fe"])
def test_crawl_three_and_four_dims(kc, oracle, d, ball, thr, mode):
    """n_dims 3 and 4 (kMaxDims; the reference takes any n_dims, collect.rs:94-119): every
    level's child counts (or FE sums), the heavy hitters and their values equal the oracle's;
    ball 1 grows the last levels to 2^d x thousands of children."""
    from fuzzyheavyhitters_amd import sim_crawl, workload
    wl = workload.zipf_workload(60, 32, d, num_sites=3, seed=11, ball_size=ball)
    k0, k1 = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
    ref = oracle.crawl(k0, k1, thr, mode=mode, sim_seed=5)
    c0, c1 = make_pair(kc, wl.left, wl.right, wl.root_seeds)
    res = sim_crawl(c0, c1, thr, mode=mode, prf_seed=5)
    assert list(res.level_children) == list(ref.n_children)
    assert np.array_equal(np.concatenate(res.counts), np.concatenate([np.asarray(c, np.uint64) for c in ref.counts]))
    got = [tuple(tuple(int(b) for b in pj) for pj in r.path) for r in res.final]
    assert got == [tuple(tuple(int(x) for x in pj) for pj in p) for p in ref.final_paths]
    assert [int(r.value) for r in res.final] == [int(v) for v in ref.final_values]


@pytest.mark.parametrize("L", [1, 7, 37])
@pytest.mark.parametrize("n", [65, 1000])
def test_add_keys_upload_bit_exact(kc, oracle, L, n):
    """fhh_add_keys (host AoS keys -> device SoA, 8 levels per item): partial level blocks and a
    partial last client word; the uploaded keys export back to the oracle's, and a crawl from them
    equals the oracle's."""
    from fuzzyheavyhitters_amd import sim_crawl, workload
    wl = workload.zipf_workload(n, 40, 2, num_sites=4, seed=n + L, ball_size=2)
    left = np.ascontiguousarray(wl.left[:, :, :L])
    right = np.ascontiguousarray(wl.right[:, :, :L])
    k0, k1 = oracle.gen_keys(left, right, wl.root_seeds)
    c0, c1 = add_pair(kc, k0, k1)
    c0.tree_init()
    c1.tree_init()
    for c, k in ((c0, k0), (c1, k1)):
        ki, rs, cs, cb = c.export_keys()
        assert np.array_equal(ki, k.key_idx) and np.array_equal(rs, k.root_seed)
        assert np.array_equal(cs, k.cw_seed) and np.array_equal(cb, k.cw_bits)
    ref = oracle.crawl(k0, k1, 0.03, mode="count")
    res = sim_crawl(c0, c1, 0.03, mode="count")
    assert list(res.level_children) == list(ref.n_children)


@pytest.mark.parametrize("L", [1, 2, 7, 37])
@pytest.mark.parametrize("d", [1, 2])
@pytest.mark.parametrize("mode", ["count", "fe"])
def test_crawl_odd_data_len(kc, oracle, L, d, mode):
    """data_len 1 (only tree_crawl_last), 2, 7 and 37 (not a multiple of 8 or 32): keys of the
    truncated interval bit strings (l <= r prefixes stay ordered); crawl = oracle."""
    from fuzzyheavyhitters_amd import sim_crawl, workload
    wl = workload.zipf_workload(65, 40, d, num_sites=4, seed=21, ball_size=2)
    left = np.ascontiguousarray(wl.left[:, :, :L])
    right = np.ascontiguousarray(wl.right[:, :, :L])
    k0, k1 = oracle.gen_keys(left, right, wl.root_seeds)
    ref = oracle.crawl(k0, k1, 0.03, mode=mode, sim_seed=3)
    c0, c1 = make_pair(kc, left, right, wl.root_seeds)
    res = sim_crawl(c0, c1, 0.03, mode=mode, prf_seed=3)
    assert list(res.level_children) == list(ref.n_children)
    assert np.array_equal(np.concatenate(res.counts), np.concatenate([np.asarray(c, np.uint64) for c in ref.counts]))
    got = [tuple(tuple(int(b) for b in pj) for pj in r.path) for r in res.final]
    assert got == [tuple(tuple(int(x) for x in pj) for pj in p) for p in ref.final_paths]
    assert [int(r.value) for r in res.final] == [int(v) for v in ref.final_values]


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(c) for c in CASES])
def test_sim_crawl_matches_golden(kc, path):
    from fuzzyheavyhitters_amd import sim_crawl
    g = load(path)
    n, d, L, _, _ = [int(x) for x in g["meta"]]
    mode = str(g["mode"][0])
    c0, c1 = make_pair(kc, g["left"], g["right"], g["root_seeds"])
    res = sim_crawl(c0, c1, float(g["threshold"][0]), mode=mode, prf_seed=77)
    assert np.array_equal(res.level_children, g["level_children"])
    counts = np.concatenate(res.counts) if res.counts else np.zeros(0, np.uint64)
    assert np.array_equal(counts, g["counts"])
    paths = np.array([r.path for r in res.final], np.uint8).reshape(-1, d, L)
    assert np.array_equal(paths, g["final_paths"])
    # count mode: server 0's plaintext counts; fe mode: the leader's final_values of the two
    # servers' FieldElm shares (sim_crawl applies collect.rs:1007-1029)
    assert [r.value for r in res.final] == [int(x) for x in g["final_values"]]
    if mode == "fe":
        from fuzzyheavyhitters_amd import KeyCollection
        fv = KeyCollection.final_values(c0.final_shares(), c1.final_shares())
        assert [r.value for r in fv] == [int(x) for x in g["final_values"]]
    st = c0.stats()
    assert st["levels"] == L


def test_sim_ot_sums_match_oracle(kc, oracle):
    from fuzzyheavyhitters_amd import workload
    from fuzzyheavyhitters_amd.collection import sim_ot_sums
    wl = workload.zipf_workload(150, 40, 1, num_sites=4, seed=3)
    k0, k1 = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
    c0, c1 = make_pair(kc, wl.left, wl.right, wl.root_seeds)
    c0.tree_init(); c1.tree_init()
    s0, s1 = oracle.tree_init(k0), oracle.tree_init(k1)
    parents = np.zeros(1, np.uint64)
    for lvl in range(6):
        o0, _ = oracle.level_expand(k0, s0, parents, lvl)
        o1, _ = oracle.level_expand(k1, s1, parents, lvl)
        C, _ = c0.tree_crawl(); c1.tree_crawl()
        eqm = np.all(oracle.share_bits(o0) == oracle.share_bits(o1), axis=-1)
        a, b = sim_ot_sums(c0, c1, C, 1234, last=False)
        ea, eb = oracle.sim_ot_sums_fe(eqm, 1234, lvl)
        assert a == ea and b == eb
        keep = np.ones(C, bool)
        c0.tree_prune(keep); c1.tree_prune(keep)
        parents = np.arange(C, dtype=np.uint64)
        s0, s1 = o0, o1
    o0, _ = oracle.level_expand(k0, s0, parents, 6)
    o1, _ = oracle.level_expand(k1, s1, parents, 6)
    C, _ = c0.tree_crawl_last(); c1.tree_crawl_last()
    eqm = np.all(oracle.share_bits(o0) == oracle.share_bits(o1), axis=-1)
    a, b = sim_ot_sums(c0, c1, C, 99, last=True)
    ea, eb = oracle.sim_ot_sums_fe255(eqm, 99, 6)
    assert a == ea and b == eb


def test_node_sums_host_values(kc, oracle):
    from fuzzyheavyhitters_amd import workload
    wl = workload.zipf_workload(200, 32, 1, num_sites=3, seed=8)
    c0, c1 = make_pair(kc, wl.left, wl.right, wl.root_seeds)
    c0.tree_init()
    C, _ = c0.tree_crawl()
    rng = np.random.default_rng(5)
    vals = rng.integers(0, 2 ** 64, size=(C, 200), dtype=np.uint64)
    vals[0, :5] = 2 ** 64 - 1
    got = c0.node_sums_fe(vals)
    for c in range(C):
        assert int(got[c]) == oracle.fe_value(oracle.fe_fold_sum(vals[c]))
        assert int(got[c]) == sum(int(x) for x in vals[c]) % oracle.FE_P
    c0.tree_prune(np.ones(C, bool))
    C, _ = c0.tree_crawl_last()
    v8 = rng.integers(0, 2 ** 32, size=(C, 200, 8), dtype=np.uint32)
    v8[:, :, 7] &= 0x7FFFFFFF
    unr, can = c0.node_sums_fe255(v8)
    for c in range(C):
        exact = sum(sum(int(v8[c, i, k]) << (32 * k) for k in range(8)) for i in range(200))
        assert unr[c] == exact
        assert can[c] == exact % oracle.FE255_P
    res = c0.final_shares()
    assert [r.value for r in res] == unr


def test_protocol_edges(kc, oracle):
    """Unpruned double crawl (children become the frontier), crawl_last keeps the frontier,
    prune length mismatches raise, empty frontier yields zero children."""
    from fuzzyheavyhitters_amd import FhhError, workload
    wl = workload.zipf_workload(70, 32, 1, num_sites=3, seed=21)
    k0, k1 = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
    c0, c1 = make_pair(kc, wl.left, wl.right, wl.root_seeds)
    c0.tree_init()
    C1, _ = c0.tree_crawl()
    C2, _ = c0.tree_crawl()          # no prune in between
    assert (C1, C2) == (2, 4)
    s = oracle.tree_init(k0)
    o1, _ = oracle.level_expand(k0, s, np.zeros(1, np.uint64), 0)
    o2, _ = oracle.level_expand(k0, o1, np.arange(2, dtype=np.uint64), 1)
    seeds, t, y = c0.export_states()
    assert np.array_equal(seeds, o2.seed) and np.array_equal(t, o2.t)
    with pytest.raises(FhhError):
        c0.tree_prune(np.ones(3, bool))
    c0.tree_prune(np.array([True, False, False, False]))
    C3, _ = c0.tree_crawl_last()
    assert C3 == 2
    c0.tree_prune_last([False, True])
    assert c0.frontier_size() == (1, 1)
    C4, _ = c0.tree_crawl_last()     # frontier unchanged by crawl_last (collect.rs:909-914)
    assert C4 == 2
    # empty frontier
    c0.tree_prune_last([False, False])
    c0.tree_crawl(); c0.tree_prune([False, False])
    C5, _ = c0.tree_crawl()
    assert C5 == 0
    with pytest.raises(FhhError):
        c1.tree_crawl()              # before tree_init


@pytest.mark.parametrize("d,n,L,sites,thr", [(1, 3000, 512, 40, 0.01), (2, 500, 40, 6, 0.004)])
def test_sim_crawl_matches_oracle_crawl(kc, oracle, d, n, L, sites, thr):
    """Moderate-size end-to-end parity (reference data_len 512 for d = 1)."""
    from fuzzyheavyhitters_amd import sim_crawl, workload
    wl = workload.zipf_workload(n, L, d, num_sites=sites, seed=1000 + n)
    k0, k1 = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
    ores = oracle.crawl(k0, k1, thr, mode="count")
    c0, c1 = make_pair(kc, wl.left, wl.right, wl.root_seeds)
    res = sim_crawl(c0, c1, thr, mode="count")
    assert list(res.level_children) == list(ores.n_children)
    assert np.array_equal(np.concatenate(res.counts), np.concatenate(ores.counts))
    got = sorted(tuple(tuple(p) for p in r.path) for r in res.final)
    exp = sorted(tuple(tuple(p) for p in fp) for fp in ores.final_paths)
    assert got == exp
    st = c0.stats()
    if d == 1:
        assert st["aes_blocks"] * 2 == ores.aes_blocks
    else:
        assert st["aes_blocks"] * 2 <= ores.aes_blocks
        assert st["ref_evals"] * 2 == ores.aes_blocks


def test_every_expand_variant_bit_exact(kc, oracle):
    """Both compiled k_expand variants give the oracle's crawl and the oracle's final-level EvalStates,
    alternated an odd number of times on one ctx pair with refused selections in between: the dynamic
    heads alternate by launch parity, and a refused variant must not advance the launch sequence
    (a sequence step without a launch left the next launch on a used-up head set)."""
    import ctypes
    from fuzzyheavyhitters_amd import lib, sim_crawl, workload
    from fuzzyheavyhitters_amd._lib import FhhError
    wl = workload.zipf_workload(700, 64, 1, num_sites=9, seed=5)
    k0, k1 = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
    ores = oracle.crawl(k0, k1, 0.01, mode="count", keep_levels=[62])
    exp_counts = np.concatenate(ores.counts)
    # tree_crawl_last keeps the frontier (collect.rs:775-796): after the crawl the engines hold the
    # children kept at level L - 2, the parents of the last level
    last0, last1 = ores.level_states[62]
    kept = np.nonzero(ores.keeps[62])[0]
    c0, c1 = make_pair(kc, wl.left, wl.right, wl.root_seeds)
    buf = ctypes.create_string_buffer(64)
    first = None
    built = [v for v in range(64) if lib().fhh_variant_info(v, buf, 64, None, None) == 0]
    assert built == [33, 52]
    for v in (52, 33, 52, 33, 52):
        for bad in (0, 14, 46):
            with pytest.raises(FhhError, match="not in this build"):
                c0.set_variant(bad)
        c0.set_variant(v)
        c1.set_variant(v)
        res = sim_crawl(c0, c1, 0.01, mode="count")
        assert np.array_equal(np.concatenate(res.counts), exp_counts), f"variant {v}"
        # the counts do not depend on the AES (the control bits are constant): the
        # final frontier's seeds must equal the oracle's
        st = [c.export_states() for c in (c0, c1)]
        for (gs, gt, gy), o in zip(st, (last0, last1)):
            assert gs.shape[0] == kept.size, f"variant {v} frontier size"
            assert np.array_equal(gs, o.seed[kept]) and np.array_equal(gt, o.t[kept]) and \
                np.array_equal(gy, o.y[kept]), f"variant {v} states vs oracle"
        if first is None:
            first = st
        for (sa, ta, ya), (sb, tb, yb) in zip(first, st):
            assert np.array_equal(sa, sb) and np.array_equal(ta, tb) and np.array_equal(ya, yb), f"variant {v} states"
