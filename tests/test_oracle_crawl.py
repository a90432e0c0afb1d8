"""Oracle crawl (CPU restatement of collect.rs + leader level loop) against (a) the committed
golden fixtures and (b) a brute-force plaintext recount of every child at every level."""
import glob
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = sorted(glob.glob(os.path.join(HERE, "golden", "zipf_d*_n*_L*.npz")))   # make_golden.py (the 1M fixture: test_golden_1m.py)


def load(path):
    z = np.load(path, allow_pickle=False)
    return {k: z[k] for k in z.files}


def prefix_ints(bits, k):
    """bits [..., L] MSB first -> int of the first k bits (k <= 62)."""
    w = (1 << np.arange(k - 1, -1, -1, dtype=np.int64))
    return (bits[..., :k].astype(np.int64) * w).sum(-1)


def plaintext_counts(left, right, paths_k):
    """paths_k: [C][d] ints of length-k prefixes -> per child number of clients whose
    [l, r] prefix box contains it."""
    k = paths_k["k"]
    lo = prefix_ints(left, k)     # [n][d]
    hi = prefix_ints(right, k)
    p = paths_k["p"]              # [C][d]
    inside = (lo[None] <= p[:, None]) & (p[:, None] <= hi[None])   # [C][n][d]
    return inside.all(-1).sum(-1)


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(c) for c in CASES])
def test_oracle_matches_golden_and_plaintext(oracle, path):
    g = load(path)
    n, d, L, _, _ = [int(x) for x in g["meta"]]
    thr = float(g["threshold"][0])
    mode = str(g["mode"][0])
    k0, k1 = oracle.gen_keys(g["left"], g["right"], g["root_seeds"])
    assert np.array_equal(k0.cw_seed, g["cw_seed"]) and np.array_equal(k0.cw_bits, g["cw_bits"])
    res = oracle.crawl(k0, k1, thr, mode=mode, sim_seed=77)
    assert np.array_equal(np.array(res.n_children, np.uint64), g["level_children"])
    counts = np.concatenate([np.asarray(c, np.uint64) for c in res.counts])
    assert np.array_equal(counts, g["counts"])
    keeps = np.concatenate([np.asarray(k, np.uint8) for k in res.keeps])
    assert np.array_equal(keeps, g["keeps"])

    # brute-force recount, level by level, following the same pruning
    left, right = g["left"], g["right"]
    tcount = max(1, int(thr * n))
    frontier = np.zeros((1, d), np.int64)
    off = 0
    for lvl in range(L):
        kids = []
        for p in frontier:
            for i in range(1 << d):
                kids.append([(p[j] << 1) | ((i >> j) & 1) for j in range(d)])
        kids = np.array(kids, np.int64).reshape(-1, d)
        C = kids.shape[0]
        pc = plaintext_counts(left, right, {"k": lvl + 1, "p": kids})
        assert np.array_equal(pc.astype(np.uint64), counts[off:off + C]), f"level {lvl}"
        keep = pc >= tcount
        assert np.array_equal(keep.astype(np.uint8), keeps[off:off + C])
        off += C
        frontier = kids[keep]
    fp = np.array([[list(map(int, p[j])) for j in range(d)] for p in res.final_paths], np.uint8).reshape(-1, d, L)
    assert np.array_equal(fp, g["final_paths"])
    if mode == "count":
        assert [int(v) for v in res.final_values] == [int(x) for x in g["final_values"]]
    else:
        # FieldElm final values (v0 - v1 mod p) equal the plaintext counts
        assert [int(v) for v in res.final_values] == [int(x) for x in g["final_values"]]
        last_counts = counts[-len(res.keeps[-1]):][res.keeps[-1]]
        assert [int(v) for v in res.final_values] == [int(x) for x in last_counts]


def test_workload_bounds_match_oracle_bitstrings(oracle):
    from fuzzyheavyhitters_amd import workload
    wl = workload.zipf_workload(64, 40, 2, num_sites=7, ball_size=3, seed=5)
    for c in range(64):
        for j in range(2):
            l, r = oracle.l_inf_ball_bounds([bool(b) for b in wl.alpha[c, j]], 3)
            assert list(map(int, l)) == list(wl.left[c, j])
            assert list(map(int, r)) == list(wl.right[c, j])


def test_workload_shard_slices_are_consistent():
    from fuzzyheavyhitters_amd import workload
    full = workload.zipf_workload(300, 64, 1, num_sites=50, seed=11)
    a = workload.zipf_workload(120, 64, 1, num_sites=50, seed=11, client_offset=0)
    b = workload.zipf_workload(180, 64, 1, num_sites=50, seed=11, client_offset=120)
    assert np.array_equal(np.concatenate([a.alpha, b.alpha]), full.alpha)
    assert np.array_equal(np.concatenate([a.root_seeds, b.root_seeds]), full.root_seeds)


@pytest.mark.parametrize("kind", ["zipf_d1", "coords_d2", "zipf_d3_ball1", "zipf_d4_point"])
def test_plaintext_crawl_equals_oracle(oracle, kind):
    """workload.plaintext_crawl (bit-packed, no crypto) reproduces the oracle's per-level
    counts and final heavy hitters — it is then the full-size check of the GPU crawl."""
    from fuzzyheavyhitters_amd import workload
    if kind == "zipf_d1":
        wl = workload.zipf_workload(300, 40, 1, num_sites=8, seed=3)
        thr = 0.02
    elif kind == "zipf_d3_ball1":
        wl = workload.zipf_workload(60, 32, 3, num_sites=3, seed=11, ball_size=1)
        thr = 0.03
    elif kind == "zipf_d4_point":
        wl = workload.zipf_workload(60, 32, 4, num_sites=3, seed=11, ball_size=0)
        thr = 0.01
    else:
        wl = workload.coords_workload(800, ball_size=3, num_centroids=30, side_km=4.0)
        thr = 0.01
    k0, k1 = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
    ref = oracle.crawl(k0, k1, thr, mode="count")
    t, tl = oracle.thresholds(thr, wl.left.shape[0])
    counts, paths, finals = workload.plaintext_crawl(wl.left, wl.right, t, tl)
    assert [c.tolist() for c in counts] == [np.asarray(c, np.uint64).tolist() for c in ref.counts]
    assert paths == [tuple(tuple(int(x) for x in pj) for pj in p) for p in ref.final_paths]
    assert finals == [int(v) for v in ref.final_values]


def test_replay_states_on_client_sample(oracle):
    """oracle.replay_states (the checker of the full-size GPU probe) on a client sample, driven
    by the full crawl's keep masks, reproduces the full crawl's states of those clients."""
    from fuzzyheavyhitters_amd import workload
    wl = workload.zipf_workload(300, 48, 1, num_sites=6, seed=9)
    k0, k1 = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
    levels = [0, 7, 46, 47]
    full = oracle.crawl(k0, k1, 0.02, mode="count", keep_levels=levels)
    sel = np.array([0, 5, 63, 64, 199, 299])
    ref = oracle.replay_states(oracle.subset_keys(k0, sel), oracle.subset_keys(k1, sel), full.keeps, levels)
    for lv in levels:
        for a, b in zip(ref[lv], full.level_states[lv]):
            assert np.array_equal(a.seed, b.seed[:, sel]) and np.array_equal(a.t, b.t[:, sel])
            assert np.array_equal(a.y, b.y[:, sel])


@pytest.mark.gpu
@pytest.mark.parametrize("mode,gc", [("count", False), ("fe", False), ("fe", "ot")],
                         ids=["count", "fe", "fe-gc-ot"])
def test_gpu_full_size_configs1_equals_plaintext(oracle, mode, gc):
    """configs[1] at full size (100 000 Zipf clients, data_len 512, threshold 0.001): every
    level's child counts, the 222 heavy hitters and their counts from the GPU crawl equal the
    plaintext crawl (size-independent check; the CPU oracle would take minutes here) — in count
    mode, in FE mode (simulated OT shares summed in FE, the last level in FieldElm, the leader's
    v0 - v1) and with the real protocol's garbled-circuit equality test + OT extension in every
    level (25.6 M equality tests and 77 M OTs per full level)."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import sim_crawl, workload
    n = 100_000
    wl = workload.zipf_workload(n, 512, 1, num_sites=10_000, zipf_s=1.03, seed=0x5EED)
    c0, c1 = fhh.KeyCollection(512, 1), fhh.KeyCollection(512, 1)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    res = sim_crawl(c0, c1, 0.001, mode=mode, gc=gc)
    t, tl = oracle.thresholds(0.001, n)
    counts, paths, finals = workload.plaintext_crawl(wl.left, wl.right, t, tl)
    assert [c.tolist() for c in res.counts] == [c.tolist() for c in counts]
    assert [tuple(tuple(int(b) for b in pj) for pj in r.path) for r in res.final] == paths
    assert [int(r.value) for r in res.final] == finals
