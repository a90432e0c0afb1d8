"""CPU checks of the north star's golden fixture (tests/golden/zipf_1m_L512.npz, made by
tests/golden/make_zipf_1m.py from workload.plaintext_crawl): it is internally consistent with
the leader's level loop (leader.rs:417-440) — level l + 1 evaluates 2^d children per node kept
at level l (collect.rs:379-391), keep iff count >= threshold (collect.rs:945-989) — and the
final set is the last level's kept children. The GPU suite compares the crawl against it
(tests/test_gpu_fullsize_aes.py)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "zipf_1m_L512.npz")


def test_golden_1m_self_consistent():
    g = np.load(GOLDEN, allow_pickle=False)
    L, thr = int(g["data_len"]), int(g["thr"])
    assert int(g["n"]) == 1_000_000 and L == 512 and thr == 1000
    lc = g["level_children"].astype(np.int64)
    off = np.concatenate([[0], np.cumsum(lc)])
    assert off[-1] == g["counts"].size == 101_998
    assert lc[0] == 2
    kept = []
    for lv in range(L):
        c = g["counts"][off[lv]:off[lv + 1]].astype(np.int64)
        # children of the same parent partition its clients: siblings sum to at most the parent
        assert c.sum() <= 1_000_000 * 2   # ball 1: a client's box may touch two siblings
        kept.append(np.nonzero(c >= thr)[0])
        if lv + 1 < L:
            assert lc[lv + 1] == 2 * kept[-1].size
    last = g["counts"][off[L - 1]:off[L]]
    assert np.array_equal(np.sort(last[kept[-1]]), np.sort(g["values"]))
    assert g["paths"].shape == (206, L // 8)
    paths = np.unpackbits(g["paths"], axis=1, bitorder="big")
    assert len({p.tobytes() for p in paths}) == 206   # distinct heavy hitters


def test_golden_1m_paths_follow_kept_children():
    """Rebuild every kept node's path from the per-level kept indices (child c = parent * 2 + bit)
    and check the final paths are exactly the last level's kept nodes."""
    g = np.load(GOLDEN, allow_pickle=False)
    L, thr = int(g["data_len"]), int(g["thr"])
    lc = g["level_children"].astype(np.int64)
    off = np.concatenate([[0], np.cumsum(lc)])
    paths = [()]
    for lv in range(L):
        c = g["counts"][off[lv]:off[lv + 1]]
        paths = [paths[k >> 1] + (int(k & 1),) for k in np.nonzero(c >= thr)[0]]
    exp = sorted(paths)
    got = sorted(tuple(int(b) for b in p) for p in np.unpackbits(g["paths"], axis=1, bitorder="big")[:, :L])
    assert got == exp
