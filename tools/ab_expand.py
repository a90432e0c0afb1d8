#!/usr/bin/env python3
"""A/B the k_expand variants in ONE process, interleaved rounds (cdna_hip_programming.md
§5.4 rule 24), on the bench workload (configs[1]). Checks every variant produces the same
crawl (children per level, per-child counts, heavy hitters) as variant 0.

    python tools/ab_expand.py --clients 100000 --rounds 3 [--variants 0,2,6]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=100_000)
    ap.add_argument("--data-len", type=int, default=512)
    ap.add_argument("--dims", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="")
    ap.add_argument("--threshold", type=float, default=0.001)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import numpy as np
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    lib = fhh.lib()
    nvar = 0
    names = {}
    while True:
        buf = ctypes.create_string_buffer(64)
        thr = ctypes.c_int()
        grid = ctypes.c_int()
        if lib.fhh_variant_info(nvar, buf, 64, ctypes.byref(thr), ctypes.byref(grid)) != 0:
            break
        names[nvar] = (buf.value.decode(), thr.value, grid.value)
        nvar += 1
    variants = [int(v) for v in args.variants.split(",")] if args.variants else list(range(nvar))
    wl = workload.zipf_workload(args.clients, args.data_len, args.dims, seed=0x5EED)
    c0 = fhh.KeyCollection(args.data_len, args.dims)
    c1 = fhh.KeyCollection(args.data_len, args.dims)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    ref = None
    res = {v: {"kernel_ms": [], "wall_ms": []} for v in variants}
    for rnd in range(args.rounds + 1):   # round 0 = warmup
        for v in variants:
            c0.set_variant(v)
            c1.set_variant(v)
            c0.reset_stats()
            t0 = time.perf_counter()
            r = fhh.sim_crawl(c0, c1, args.threshold, record=(rnd == 0))
            wall = (time.perf_counter() - t0) * 1e3
            st = c0.stats()
            if rnd == 0:
                sig = (r.level_children.tolist(), [c.tolist() for c in r.counts],
                       sorted(tuple(tuple(p) for p in x.path) for x in r.final))
                if ref is None:
                    ref = sig
                elif sig != ref:
                    print(f"variant {v}: OUTPUT MISMATCH vs variant {variants[0]}", flush=True)
                    res[v]["mismatch"] = True
                continue
            res[v]["kernel_ms"].append(st["expand_ms"])
            res[v]["wall_ms"].append(wall)
            res[v]["blocks"] = st["expand_blocks_timed"]
        print(f"round {rnd} done", flush=True)
    rows = []
    for v in variants:
        k = statistics.median(res[v]["kernel_ms"])
        w = statistics.median(res[v]["wall_ms"])
        rate = res[v]["blocks"] / (k / 1e3)
        nm, thr, grid = names[v]
        rows.append({"variant": v, "layout": nm, "threads": thr, "grid": grid, "kernel_ms": k, "wall_ms": w,
                     "kernel_blocks_per_s": rate, "kernel_ms_all": res[v]["kernel_ms"],
                     "mismatch": res[v].get("mismatch", False)})
        print(f"v{v:2d} {nm:22s} thr={thr:4d} grid={grid:4d} kernel={k:8.1f} ms wall={w:8.1f} ms "
              f"{rate / 1e9:6.1f} G blocks/s {'MISMATCH' if res[v].get('mismatch') else ''}", flush=True)
    if args.out:
        json.dump(rows, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
