#!/usr/bin/env python3
"""The drop-in path's per-level phases at a given client count, a few levels only, for rocprofv3:
    python tools/dropin_profile.py [--clients 1000000] [--levels 24] [--mode dropin|fused|crawl]
dropin: two_party_crawl (fhh_tree_crawl per server, the party GC + OT, node sums, keep, prune);
fused: fhh_sim_crawl(gc = 2) over the same levels; crawl: only the two servers' fhh_tree_crawl +
fhh_tree_prune (all children kept) per level, timed per call. Prints one JSON line."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=1_000_000)
    ap.add_argument("--levels", type=int, default=24)
    ap.add_argument("--mode", default="dropin", choices=["dropin", "fused", "crawl"])
    args = ap.parse_args()
    import numpy as np
    import torch
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    n, L = args.clients, 512
    wl = workload.zipf_workload(n, L, 1, num_sites=10_000, zipf_s=1.03, seed=0x5EED)
    c0 = fhh.KeyCollection(L, 1)
    c1 = fhh.KeyCollection(L, 1)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    torch.cuda.synchronize()
    out = {"clients": n, "levels": args.levels, "mode": args.mode}
    t0 = time.perf_counter()
    if args.mode == "dropin":
        tm, log = {}, []
        r = fhh.two_party_crawl(c0, c1, 0.001, prf_seed=7, channel="inplace", timing=tm, record=False,
                                levels=args.levels, level_log=log)
        out["ms_per_level"] = {k: v / args.levels * 1e3 for k, v in tm.items()}
        out["level_log_ms"] = [(lv, C, round(a * 1e3, 3), round(b * 1e3, 3), round(c * 1e3, 3)) for lv, C, a, b, c in log]
        out["children"] = [int(c) for c in r.level_children]
    elif args.mode == "fused":
        r = fhh.sim_crawl(c0, c1, 0.001, mode="fe", prf_seed=7, gc="ot", record=False, levels=args.levels)
        out["children"] = [int(c) for c in r.level_children]
    else:
        c0.tree_init()
        c1.tree_init()
        per = []
        for lv in range(args.levels):
            a = time.perf_counter()
            C, _ = c0.tree_crawl()
            b = time.perf_counter()
            c1.tree_crawl()
            c = time.perf_counter()
            keep = np.ones(C, np.uint8)
            if C > 64:   # keep the frontier bounded like the threshold would
                keep[64:] = 0
            c0.tree_prune(keep)
            c1.tree_prune(keep)
            d = time.perf_counter()
            per.append({"C": C, "crawl0_ms": (b - a) * 1e3, "crawl1_ms": (c - b) * 1e3, "prune_ms": (d - c) * 1e3})
        out["per_level"] = per
    torch.cuda.synchronize()
    out["wall_s"] = time.perf_counter() - t0
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
