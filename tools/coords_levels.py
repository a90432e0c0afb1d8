"""Per-level shape of configs[3] (d = 2, data_len 16, 1M clients): AES blocks and children of
each level (crawls cut after 1, 2, ... levels, differenced), then `--reps` full crawls for a
rocprofv3 --kernel-trace to pair each k_expand dispatch with its level.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/coords -- python3 tools/coords_levels.py
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=1_000_000)
    ap.add_argument("--threshold", type=float, default=0.075)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/coords/levels.json")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime: torch's)
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload

    wl = workload.coords_workload(args.clients, ball_size=1, zipf_s=1.03)
    c0 = fhh.KeyCollection(16, 2, device=0)
    c1 = fhh.KeyCollection(16, 2, device=0)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    del wl

    def crawl(levels=0):
        return fhh.sim_crawl(c0, c1, args.threshold, mode="count", record=False, levels=levels)

    crawl()   # warm
    blocks, prev = [], 0
    for lv in range(1, 17):
        c0.reset_stats()
        c1.reset_stats()
        crawl(lv)
        b = c0.stats()["aes_blocks"] + c1.stats()["aes_blocks"]
        blocks.append(b - prev)
        prev = b
    res = crawl()
    for _ in range(args.reps):
        res = crawl()
    out = {"blocks_per_level": blocks, "children_per_level": [int(x) for x in res.level_children],
           "reps_after_cut_crawls": args.reps + 1, "cut_crawls": 16}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(out, f)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
