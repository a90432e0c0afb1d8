"""Generate the committed golden fixtures under tests/golden/ with the CPU oracle.

Run:  python tests/golden/make_golden.py
Inputs are the deterministic workloads of fuzzyheavyhitters_amd.workload (seeded), the
expected outputs come from oracle/ (pinned by tests/test_oracle_kat.py). Stored as .npz
(numpy, no pickle) and .json.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from fuzzyheavyhitters_amd import workload  # noqa: E402
from oracle import oracle as O  # noqa: E402

CASES = {
    # name: (n, d, L, num_sites, ball, threshold, mode)
    "zipf_d1_n48_L40": (48, 1, 40, 6, 1, 0.045, "count"),
    "zipf_d2_n70_L32": (70, 2, 32, 5, 1, 0.01, "count"),
    "zipf_d1_n130_L48_fe": (130, 1, 48, 8, 2, 0.02, "fe"),
}


def make_case(name, n, d, L, num_sites, ball, thr, mode):
    wl = workload.zipf_workload(n, L, d, num_sites=num_sites, ball_size=ball, seed=0xC0FFEE + n)
    k0, k1 = O.gen_keys(wl.left, wl.right, wl.root_seeds)
    res = O.crawl(k0, k1, thr, mode=mode, sim_seed=77)
    counts = np.concatenate([np.asarray(c, np.uint64) for c in res.counts]) if res.counts else np.zeros(0, np.uint64)
    keeps = np.concatenate([np.asarray(k, np.uint8) for k in res.keeps]) if res.keeps else np.zeros(0, np.uint8)
    final_paths = np.array([[list(map(int, p[j])) for j in range(d)] for p in res.final_paths], np.uint8).reshape(
        len(res.final_paths), d, L)
    # level-1 states of server 0 (seed/t/y of the 2^d children of the root) for a direct check
    s0 = O.tree_init(k0)
    c1, _ = O.level_expand(k0, s0, np.zeros(1, np.uint64), 0)
    np.savez_compressed(os.path.join(HERE, name + ".npz"),
                        left=wl.left, right=wl.right, root_seeds=wl.root_seeds,
                        cw_seed=k0.cw_seed, cw_bits=k0.cw_bits,
                        level_children=np.array(res.n_children, np.uint64), counts=counts, keeps=keeps,
                        final_paths=final_paths,
                        final_values=np.array([str(v) for v in res.final_values]).astype("U80"),
                        lvl1_seed=c1.seed, lvl1_t=c1.t, lvl1_y=c1.y,
                        meta=np.array([n, d, L, num_sites, ball], np.int64),
                        threshold=np.array([thr]), mode=np.array([mode]))
    return {"n": n, "d": d, "L": L, "levels": len(res.n_children), "final": len(res.final_paths),
            "aes_blocks": res.aes_blocks}


def main():
    kat = {
        "fips197_c1": {"key": bytes(range(16)).hex(), "pt": "00112233445566778899aabbccddeeff",
                       "ct": "69c4e0d86a7b0430d8cdb78070b4c55a"},
        "aes0_zero": {"pt": "00" * 16, "ct": O.aes0(bytes(16)).hex()},
        "mmo_zero_seed": {"left": O.expand_dir(bytes(16), 0)[0].hex(), "right": O.expand_dir(bytes(16), 1)[0].hex()},
        "fe_recip_999": 2885188949795824624,
    }
    rng = np.random.default_rng(9)
    kat["mmo_random"] = []
    for _ in range(16):
        s = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
        kat["mmo_random"].append({"seed": s.hex(), "left": O.expand_dir(s, 0)[0].hex(),
                                  "right": O.expand_dir(s, 1)[0].hex()})
    summary = {}
    for name, args in CASES.items():
        summary[name] = make_case(name, *args)
    kat["cases"] = summary
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
