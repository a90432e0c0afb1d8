"""Parity that sees the AES at the timed sizes.

The heavy-hitter output does not depend on any AES block (the PRG's control bits are constant
after the nibble mask, prg.rs:96-105), so full-size count checks cannot catch a
wrong seed. Here the device loop's own k_expand states are read back (the probe of
fhh_sim_config, a gather kernel between k_expand and the count) for a sample of clients that
touches every 64-client word — hence every work item and every wave of the persistent launch —
and compared with the oracle (oracle.replay_states: eval_bit, ibDCF.rs:208-227, with
expand_dir, prg.rs:92-122) evaluated for just those clients along the same surviving paths.

configs[0] (the reference's own CPU configuration, leader.rs:299-443: 1000 Zipf clients,
num_sites 10000, s = 1.03, data_len 512, threshold 0.001) is run exactly, on both sides.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def sample_clients(n: int, word_step: int = 1, seed: int = 7) -> np.ndarray:
    """One client per `word_step`-th 64-client word at a varying lane, plus the edges (first and
    last words, the partial last word)."""
    nw = (n + 63) // 64
    rng = np.random.default_rng(seed)
    w = np.arange(0, nw, word_step)
    c = np.minimum(w * 64 + rng.integers(0, 64, w.size), n - 1)
    edges = [0, 1, 63, 64, 65, n - 1, n - 2, ((n - 1) // 64) * 64, max(0, n - 65)]
    return np.unique(np.concatenate([c, np.array([e for e in edges if 0 <= e < n])])).astype(np.uint64)


def keeps_from_counts(res, thr: int, thr_last: int):
    L = len(res.counts)
    return [np.asarray(res.counts[lv]) >= (thr_last if lv == L - 1 else thr) for lv in range(L)]


def assert_probe_equal(res, ref, clients_sel=None):
    for lv, (seeds, t, y) in res.probe.items():
        o0, o1 = ref[lv]
        for s, o in ((0, o0), (1, o1)):
            os_, ot, oy = o.seed, o.t, o.y
            if clients_sel is not None:
                os_, ot, oy = os_[:, clients_sel], ot[:, clients_sel], oy[:, clients_sel]
            assert seeds[s].shape == os_.shape, f"level {lv} server {s}: {seeds[s].shape} vs {os_.shape}"
            bad = np.nonzero(np.any(seeds[s] != os_, axis=-1))
            assert bad[0].size == 0, (f"level {lv} server {s}: {bad[0].size} seeds differ, first (child, "
                                      f"client, dim, side) = {[int(b[0]) for b in bad]}")
            assert np.array_equal(t[s], ot), f"level {lv} server {s}: t bits differ"
            assert np.array_equal(y[s], oy), f"level {lv} server {s}: y bits differ"


GOLDEN_1M = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "zipf_1m_L512.npz")


def load_golden_1m():
    g = np.load(GOLDEN_1M, allow_pickle=False)
    return {k: g[k] for k in g.files}


def assert_equals_golden_1m(wl, res):
    """The north star's literal target (BASELINE.json): the heavy-hitter output for 1M Zipf
    clients at data_len 512 — every level's child count and counts (leader.rs:417-440), the
    kept set per level, and the final paths with their counts (collect.rs:945-1029) — equal the
    plaintext recount committed as tests/golden/zipf_1m_L512.npz."""
    g = load_golden_1m()
    assert str(g["left_sha256"]) == golden_digest(wl.left), "workload generator changed: regenerate the fixture"
    assert str(g["right_sha256"]) == golden_digest(wl.right), "workload generator changed: regenerate the fixture"
    L = int(g["data_len"])
    lc = g["level_children"].astype(np.int64)
    assert [int(x) for x in res.level_children] == lc.tolist()
    off = np.concatenate([[0], np.cumsum(lc)])
    thr = int(g["thr"])
    for lv in range(L):
        exp = g["counts"][off[lv]:off[lv + 1]].astype(np.uint64)
        got = np.asarray(res.counts[lv], np.uint64)
        assert np.array_equal(got, exp), f"level {lv}: {int(np.sum(got != exp))} of {exp.size} counts differ"
        assert int(res.level_kept[lv]) == int(np.sum(exp >= thr)), f"level {lv}: kept set differs"
    paths = np.unpackbits(g["paths"], axis=1, bitorder="big")[:, :L]
    exp_final = sorted((tuple(int(b) for b in p), int(v)) for p, v in zip(paths, g["values"]))
    got_final = sorted((tuple(int(b) for b in r.path[0]), int(r.value)) for r in res.final)
    assert len(got_final) == len(exp_final) == 206
    assert got_final == exp_final


def golden_digest(a) -> str:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint8).tobytes()).hexdigest()


def crawl_with_probe(n, L, levels, clients, cap, seed=0x5EED, num_sites=10_000, threshold=0.001):
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    wl = workload.zipf_workload(n, L, 1, num_sites=num_sites, zipf_s=1.03, ball_size=1, seed=seed)
    c0, c1 = fhh.KeyCollection(L, 1), fhh.KeyCollection(L, 1)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    res = fhh.sim_crawl(c0, c1, threshold, mode="count",
                        probe={"levels": levels, "clients": clients, "capacity": cap})
    return wl, c0, c1, res


@pytest.mark.parametrize("n,word_step", [(100_000, 1), (1_000_000, 8)], ids=["configs1-100k", "1M"])
def test_sampled_states_bit_exact_full_size(oracle, n, word_step):
    """configs[1] (100k clients) and the metric's 1M clients, data_len 512, seed 0x5EED: the
    default k_expand's seeds / t / y of every child at levels 0, 1, a middle level, L-2 and
    L-1 equal the oracle's for a client in every word (configs[1]) / every 8th word (1M)."""
    L = 512
    clients = sample_clients(n, word_step)
    levels = [0, 1, 256, L - 2, L - 1]
    wl, c0, c1, res = crawl_with_probe(n, L, levels, clients, cap=1024)
    thr = max(1, int(0.001 * n))
    keeps = keeps_from_counts(res, thr, thr)
    k0, k1 = oracle.gen_keys(wl.left[clients.astype(np.int64)], wl.right[clients.astype(np.int64)],
                             wl.root_seeds[clients.astype(np.int64)])
    ref = oracle.replay_states(k0, k1, keeps, levels)
    assert set(res.probe) == set(levels)
    for lv in levels:
        assert res.probe[lv][0].shape[1] == res.level_children[lv] > 0
    assert_probe_equal(res, ref)
    if n > 100_000:
        # 1M: the plaintext recount takes ~2 min in numpy, so its result is the committed golden
        # fixture (tests/golden/make_zipf_1m.py); every level's counts and the heavy hitters
        assert_equals_golden_1m(wl, res)
        return
    # configs[1]: every level's counts, the 222 heavy hitters with their counts and the AES-block
    # total equal the ORACLE's own crawl (tests/golden/oracle_zipf_100k_L512.npz,
    # tests/golden/make_oracle_100k.py)
    from test_oracle_100k import assert_counts_equal_oracle, load_oracle_100k
    g = load_oracle_100k()
    assert_counts_equal_oracle(g, res.level_children, res.counts,
                               [(tuple(int(b) for b in r.path[0]), int(r.value)) for r in res.final])
    assert c0.stats()["aes_blocks"] * 2 == int(g["aes_blocks"])
    # the crawl itself (AES-independent) still matches the plaintext recount
    from fuzzyheavyhitters_amd import workload
    cnt, paths, _ = workload.plaintext_crawl(wl.left, wl.right, thr, thr)
    assert [len(c) for c in cnt] == [int(x) for x in res.level_children]
    assert all(np.array_equal(a, np.asarray(b)) for a, b in zip(cnt, res.counts))
    got = sorted(tuple(tuple(int(b) for b in p) for p in r.path) for r in res.final)
    assert got == sorted(paths)


def test_north_star_1m_fe_shares_equal_golden():
    """The same 1M crawl with the servers' outputs as FE shares (simulated OT: v0 = r1, v1 = eq ?
    r0 : r1, collect.rs:439-472) and the last level over FieldElm: the leader's v0 - v1 per child
    at every level and its final_values (collect.rs:1007-1029) equal the golden counts."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    n, L = 1_000_000, 512
    wl = workload.zipf_workload(n, L, 1, num_sites=10_000, zipf_s=1.03, ball_size=1, seed=0x5EED)
    c0, c1 = fhh.KeyCollection(L, 1), fhh.KeyCollection(L, 1)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    res = fhh.sim_crawl(c0, c1, 0.001, mode="fe", prf_seed=0x1234)
    assert_equals_golden_1m(wl, res)


def test_configs0_gpu_equals_oracle(oracle):
    """configs[0] exactly (leader.rs:299-443, SURVEY §8d Config A): 1000 Zipf clients over
    num_sites 10000 (s = 1.03), data_len 512, d = 1, ball 1, threshold 0.001 -> count threshold
    max(1, 1) = 1, so every non-empty node survives. GPU device loop vs the oracle's crawl
    (reference child order): every level's child count, counts and keep masks, the heavy
    hitters and their counts, and the EvalStates of every client at levels 0, 255 and 511."""
    n, L = 1000, 512
    levels = [0, 255, L - 1]
    clients = np.arange(n, dtype=np.uint64)
    wl, c0, c1, res = crawl_with_probe(n, L, levels, clients, cap=4096)
    k0, k1 = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
    ores = oracle.crawl(k0, k1, 0.001, mode="count", keep_levels=levels)
    assert list(res.level_children) == list(ores.n_children)
    assert sum(ores.n_children) > 100_000            # ~4.9e5 children summed
    for lv in range(L):
        assert np.array_equal(res.counts[lv], ores.counts[lv]), f"counts level {lv}"
        assert int(res.level_kept[lv]) == int(ores.keeps[lv].sum()), f"keep mask level {lv}"
    got = [(tuple(tuple(int(b) for b in p) for p in r.path), int(r.value)) for r in res.final]
    exp = [(tuple(tuple(int(x) for x in p) for p in fp), int(v)) for fp, v in zip(ores.final_paths, ores.final_values)]
    assert got == exp
    assert_probe_equal(res, ores.level_states)
    st = c0.stats()
    assert st["aes_blocks"] * 2 == ores.aes_blocks


@pytest.mark.parametrize("thr_frac,levels,heavy", [(0.075, [0, 5, 9, 13], 0), (0.01, [0, 7, 14, 15], 54),
                                                   (0.001, [0, 9, 15], 1046)],
                         ids=["config-threshold", "deep", "dense"])
def test_configs3_sampled_states_bit_exact(oracle, thr_frac, levels, heavy):
    """configs[3] at its full size (src/bin/config.json: 1M clients, d = 2 lat/lon, data_len 16,
    ball 1, threshold 0.075) on the reference's own county centroids (data/county_centroids.csv,
    Zipf-weighted, 8 km uniform_in_square jitter): the d = 2 path (dim-prefix dedup, per-dim
    entry tables, a node = a pair of entries) at 1M clients. At the config's 0.075 no node
    survives past level 13 (0 heavy hitters: one centidegree cell never holds 7.5 % of the
    clients), so 0.01 (54) and 0.001 (1 046 heavy hitters) crawl to the leaves too. The probe
    reads every child's per-dim states for a client in every 8th word at non-empty levels and the
    oracle replays them; the counts of every level equal the plaintext recount."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    n, L = 1_000_000, 16
    wl = workload.coords_workload(n, ball_size=1, seed=0x5EED)
    c0, c1 = fhh.KeyCollection(L, 2), fhh.KeyCollection(L, 2)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    clients = sample_clients(n, 8)
    res = fhh.sim_crawl(c0, c1, thr_frac, mode="count",
                        probe={"levels": levels, "clients": clients, "capacity": 4096})
    thr = max(1, int(thr_frac * n))
    keeps = keeps_from_counts(res, thr, thr)
    sel = clients.astype(np.int64)
    k0, k1 = oracle.gen_keys(wl.left[sel], wl.right[sel], wl.root_seeds[sel])
    ref = oracle.replay_states(k0, k1, keeps, levels)
    assert set(res.probe) == set(levels)
    assert all(int(res.level_children[lv]) > 0 for lv in levels)
    assert_probe_equal(res, ref)
    cnt, paths, _ = workload.plaintext_crawl(wl.left, wl.right, thr, thr)
    assert [len(c) for c in cnt] == [int(x) for x in res.level_children]
    assert all(np.array_equal(a, np.asarray(b)) for a, b in zip(cnt, res.counts))
    got = sorted(tuple(tuple(int(b) for b in p) for p in r.path) for r in res.final)
    assert got == sorted(paths)
    assert len(got) == heavy
    print("configs[3] children per level:", [int(x) for x in res.level_children], "heavy hitters:", len(got))
