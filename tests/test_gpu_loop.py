"""Device-resident level loop (keep/prune on the GPU, no per-level host round trip) against
the host-driven loop and the oracle, including forced buffer growth mid-crawl."""
import glob
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
CASES = sorted(glob.glob(os.path.join(HERE, "golden", "zipf_d*_n*_L*.npz")))   # make_golden.py fixtures


def _pair(left, right, roots):
    import fuzzyheavyhitters_amd as fhh
    n, d, L = left.shape
    c0, c1 = fhh.KeyCollection(L, d), fhh.KeyCollection(L, d)
    fhh.gen_keys_pair(c0, c1, left, right, roots)
    return c0, c1


def _sig(res):
    return (res.level_children.tolist(), res.level_kept.tolist(), [c.tolist() for c in res.counts],
            [(r.path, r.value) for r in res.final])


@pytest.mark.parametrize("path", CASES, ids=[os.path.basename(c) for c in CASES])
@pytest.mark.parametrize("cap", [0, 2])
def test_device_loop_equals_host_loop(path, cap):
    from fuzzyheavyhitters_amd import sim_crawl
    z = np.load(path, allow_pickle=False)
    mode = str(z["mode"][0])
    thr = float(z["threshold"][0])
    c0, c1 = _pair(z["left"], z["right"], z["root_seeds"])
    host = sim_crawl(c0, c1, thr, mode=mode, prf_seed=77, host_loop=True)
    dev = sim_crawl(c0, c1, thr, mode=mode, prf_seed=77, host_loop=False, init_capacity=cap)
    assert _sig(dev) == _sig(host)
    assert np.array_equal(np.concatenate(dev.counts), z["counts"])
    # server 1's final shares agree too (leader final_values)
    r1 = c1.final_shares()
    assert [r.path for r in r1] == [r.path for r in dev.final]


@pytest.mark.parametrize("variant", [None, 33], ids=["default", "generic-aes"])
def test_device_loop_large_with_growth(oracle, variant):
    """data_len 512, frontier well past the initial capacity: several grow-and-resume cycles."""
    from fuzzyheavyhitters_amd import sim_crawl, workload
    wl = workload.zipf_workload(4000, 512, 1, num_sites=60, seed=99)
    c0, c1 = _pair(wl.left, wl.right, wl.root_seeds)
    if variant is not None:
        c0.set_variant(variant)
        c1.set_variant(variant)
    host = sim_crawl(c0, c1, 0.002, mode="count", host_loop=True)
    st_host = c0.stats()
    c0.reset_stats()
    dev = sim_crawl(c0, c1, 0.002, mode="count", init_capacity=4)
    st_dev = c0.stats()
    assert _sig(dev) == _sig(host)
    assert st_dev["aes_blocks"] == st_host["aes_blocks"]
    k0, k1 = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
    ores = oracle.crawl(k0, k1, 0.002, mode="count")
    assert dev.level_children.tolist() == list(ores.n_children)
    # the engine state after the loop supports the drop-in API (frontier = pre-last level)
    seeds, t, y = c0.export_states()
    assert seeds.shape[0] == int(dev.level_kept[-2])


def test_device_loop_d2_coords(oracle):
    from fuzzyheavyhitters_amd import sim_crawl, workload
    wl = workload.coords_workload(1500, ball_size=3, num_centroids=40, side_km=4.0)
    c0, c1 = _pair(wl.left, wl.right, wl.root_seeds)
    host = sim_crawl(c0, c1, 0.01, mode="fe", prf_seed=3, host_loop=True)
    dev = sim_crawl(c0, c1, 0.01, mode="fe", prf_seed=3, init_capacity=2)
    assert _sig(dev) == _sig(host)
    k0, k1 = oracle.gen_keys(wl.left, wl.right, wl.root_seeds)
    ores = oracle.crawl(k0, k1, 0.01, mode="count")
    got = sorted(tuple(tuple(p) for p in r.path) for r in dev.final)
    exp = sorted(tuple(tuple(p) for p in fp) for fp in ores.final_paths)
    assert got == exp
