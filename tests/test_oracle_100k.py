"""configs[1] at full size pinned to the ORACLE (tests/golden/oracle_zipf_100k_L512.npz, made by the
committed tests/golden/make_oracle_100k.py: the oracle's own two-server crawl, keygen ibDCF.rs:84-205,
eval_bit ibDCF.rs:208-227, expand_dir prg.rs:92-122, child order collect.rs:379-391, keep
collect.rs:945-989; 4.16e10 AES blocks, ~17 min on 7 CPU threads).

`workload.plaintext_crawl` — the restatement the 1M golden (tests/golden/zipf_1m_L512.npz) is made with
and that the GPU suite checks configs[1] and 1M against — must equal it at this Zipf-shaped full size:
every level's child count and every child's count, and the 222 heavy hitters with their counts. The
GPU crawl is compared against the same fixture in tests/test_gpu_fullsize_aes.py."""
import hashlib
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "oracle_zipf_100k_L512.npz")


def load_oracle_100k():
    g = np.load(GOLDEN, allow_pickle=False)
    return {k: g[k] for k in g.files}


def _digest(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint8).tobytes()).hexdigest()


def configs1_workload():
    from fuzzyheavyhitters_amd import workload
    g = load_oracle_100k()
    wl = workload.zipf_workload(int(g["n"]), int(g["data_len"]), 1, num_sites=int(g["num_sites"]),
                                zipf_s=float(g["zipf_s"]), ball_size=1, seed=int(g["seed"]))
    assert str(g["left_sha256"]) == _digest(wl.left), "workload generator changed: regenerate the fixture"
    assert str(g["right_sha256"]) == _digest(wl.right), "workload generator changed: regenerate the fixture"
    assert str(g["roots_sha256"]) == _digest(wl.root_seeds), "workload generator changed: regenerate the fixture"
    return wl, g


def assert_counts_equal_oracle(g, level_children, counts, final):
    """level_children [L], counts per level, final [(path bits tuple, value)] vs the oracle fixture."""
    L = int(g["data_len"])
    lc = g["level_children"].astype(np.int64)
    assert [int(x) for x in level_children] == lc.tolist()
    off = np.concatenate([[0], np.cumsum(lc)])
    for lv in range(L):
        exp = g["counts"][off[lv]:off[lv + 1]].astype(np.uint64)
        got = np.asarray(counts[lv], np.uint64)
        assert np.array_equal(got, exp), f"level {lv}: {int(np.sum(got != exp))} of {exp.size} counts differ"
    paths = np.unpackbits(g["paths"], axis=1, bitorder="big")[:, :L]
    exp_final = sorted((tuple(int(b) for b in p), int(v)) for p, v in zip(paths, g["values"]))
    assert sorted(final) == exp_final


def test_oracle_fixture_shape():
    g = load_oracle_100k()
    assert int(g["n"]) == 100_000 and int(g["data_len"]) == 512 and int(g["thr"]) == 100
    assert int(g["level_children"].sum()) == g["counts"].size == 104_020
    assert g["values"].size == 222
    # every child of every level evaluated by both servers' 2 keys: C x n x 2 x 2 AES blocks
    assert int(g["aes_blocks"]) == 104_020 * 100_000 * 4


def test_plaintext_crawl_equals_oracle_at_configs1():
    from fuzzyheavyhitters_amd import workload
    wl, g = configs1_workload()
    thr = int(g["thr"])
    cnt, paths, vals = workload.plaintext_crawl(wl.left, wl.right, thr, thr)
    assert_counts_equal_oracle(g, [len(c) for c in cnt], cnt,
                               [(tuple(int(b) for b in p[0]), int(v)) for p, v in zip(paths, vals)])
