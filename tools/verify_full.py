#!/usr/bin/env python3
"""Full-size parity evidence (north star: bit-exact heavy-hitter output for 1M Zipf clients at
data_len 512): GPU keygen + GPU crawl (both servers, count mode) against the bit-packed
plaintext crawl (fuzzyheavyhitters_amd.workload.plaintext_crawl), per-level child counts,
heavy-hitter paths and their counts. Prints one JSON line."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=1_000_000)
    ap.add_argument("--data-len", type=int, default=512)
    ap.add_argument("--threshold", type=float, default=0.001)
    ap.add_argument("--seed", type=int, default=0x5EED)
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import sim_crawl, workload
    from oracle import oracle as O
    t0 = time.perf_counter()
    wl = workload.zipf_workload(args.clients, args.data_len, 1, num_sites=10_000, zipf_s=1.03, seed=args.seed)
    t_gen = time.perf_counter() - t0
    print(f"workload {t_gen:.1f} s", flush=True)
    c0, c1 = fhh.KeyCollection(args.data_len, 1), fhh.KeyCollection(args.data_len, 1)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    sim_crawl(c0, c1, args.threshold, mode="count", record=False)   # warm-up (buffer sizing)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    res = sim_crawl(c0, c1, args.threshold, mode="count")
    t_gpu = time.perf_counter() - t1
    print(f"gpu crawl {t_gpu:.3f} s", flush=True)
    t, tl = O.thresholds(args.threshold, args.clients)
    t2 = time.perf_counter()
    counts, paths, finals = workload.plaintext_crawl(wl.left, wl.right, t, tl)
    t_plain = time.perf_counter() - t2
    got_paths = [tuple(tuple(int(b) for b in pj) for pj in r.path) for r in res.final]
    ok_counts = [c.tolist() for c in res.counts] == [c.tolist() for c in counts]
    ok_paths = got_paths == paths
    ok_values = [int(r.value) for r in res.final] == finals
    print(json.dumps({
        "check": "GPU crawl == plaintext crawl", "clients": args.clients, "data_len": args.data_len,
        "threshold": args.threshold, "heavy_hitters": len(paths), "children_total": int(sum(len(c) for c in counts)),
        "level_counts_equal": ok_counts, "paths_equal": ok_paths, "values_equal": ok_values,
        "gpu_crawl_s": t_gpu, "plaintext_crawl_s": t_plain, "workload_s": t_gen,
    }), flush=True)
    if not (ok_counts and ok_paths and ok_values):
        sys.exit(1)


if __name__ == "__main__":
    main()
