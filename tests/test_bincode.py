"""The add_keys RPC payload (rpc.rs:12-15, bincode 1.x legacy encoding) decoded on the GPU:
the serializer's sizes match the reference's own key size (ibDCFbench.csv: 10 265 B at
512 bits = 1 + 16 + 8 + 20 L), the decoded keys equal the oracle's, a crawl from them matches
the golden fixture, and malformed payloads are rejected."""
import glob
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def test_serialized_key_size_matches_reference(oracle):
    from fuzzyheavyhitters_amd import workload
    wl = workload.zipf_workload(3, 512, 1, num_sites=2, seed=1)
    k0, _ = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
    req = workload.add_keys_request_bincode(k0.key_idx, k0.root_seed, k0.cw_seed, k0.cw_bits)
    # u64 n + per client (u64 d + 2 keys of 10 265 B), ibDCFbench.csv:5
    assert req.size == 8 + 3 * (8 + 2 * 10265)
    assert int(np.frombuffer(req[:8].tobytes(), np.uint64)[0]) == 3


@pytest.mark.gpu
def test_bincode_keys_equal_oracle_and_crawl(oracle):
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    path = sorted(glob.glob(os.path.join(HERE, "golden", "zipf_d2_*.npz")))[0]
    g = np.load(path, allow_pickle=False)
    n, d, L, _, _ = [int(x) for x in g["meta"]]
    k0, k1 = oracle.gen_keys(g["left"], g["right"], g["root_seeds"])
    cs = []
    for k in (k0, k1):
        c = fhh.KeyCollection(L, d)
        c.add_keys_bincode(workload.add_keys_request_bincode(k.key_idx, k.root_seed, k.cw_seed, k.cw_bits))
        ki, rs, cw, cb = c.export_keys()
        assert np.array_equal(ki, k.key_idx) and np.array_equal(rs, k.root_seed)
        assert np.array_equal(cw, k.cw_seed) and np.array_equal(cb, k.cw_bits)
        cs.append(c)
    res = fhh.sim_crawl(cs[0], cs[1], float(g["threshold"][0]), mode=str(g["mode"][0]), prf_seed=77)
    assert np.array_equal(res.level_children, g["level_children"])
    assert np.array_equal(np.concatenate(res.counts), g["counts"])


@pytest.mark.gpu
@pytest.mark.parametrize("n,L,d", [(1000, 104, 2), (129, 40, 1), (64, 32, 1)])
def test_bincode_tiles_equal_oracle(oracle, n, L, d):
    """The tiled decode (64 clients x 32 levels per tile, clients at every byte alignment of the
    20-B CorWords): partial level blocks, a partial last client word, d = 2."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    wl = workload.zipf_workload(n, L, d, num_sites=7, seed=n + L)
    k0, _ = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
    c = fhh.KeyCollection(L, d)
    c.add_keys_bincode(workload.add_keys_request_bincode(k0.key_idx, k0.root_seed, k0.cw_seed, k0.cw_bits))
    ki, rs, cw, cb = c.export_keys()
    assert np.array_equal(ki, k0.key_idx) and np.array_equal(rs, k0.root_seed)
    assert np.array_equal(cw, k0.cw_seed) and np.array_equal(cb, k0.cw_bits)


@pytest.mark.gpu
def test_bincode_malformed_rejected(oracle):
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    wl = workload.zipf_workload(70, 40, 1, num_sites=4, seed=3)
    k0, _ = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
    good = workload.add_keys_request_bincode(k0.key_idx, k0.root_seed, k0.cw_seed, k0.cw_bits)
    KB = 25 + 20 * 40
    R = 8 + 2 * KB
    bad_cases = {
        "truncated": good[:-1],
        "bool2": good.copy(),
        "L": good.copy(),
        "d": good.copy(),
    }
    bad_cases["bool2"][8 + 5 * R + 8 + KB + 25 + 20 * 3 + 17] = 2      # client 5, right key, level 3 bits.1
    bad_cases["L"][8 + 9 * R + 8 + 17] = 39                             # client 9, left key: cor_words len
    bad_cases["d"][8 + 69 * R] = 2                                      # client 69: inner vec len
    for name, buf in bad_cases.items():
        c = fhh.KeyCollection(40, 1)
        with pytest.raises(fhh.FhhError):
            c.add_keys_bincode(buf)
    c = fhh.KeyCollection(40, 1)
    c.add_keys_bincode(good)
    with pytest.raises(fhh.FhhError):   # keys already present
        c.add_keys_bincode(good)
