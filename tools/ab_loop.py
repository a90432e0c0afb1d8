#!/usr/bin/env python3
"""A/B the host-driven and the device-resident level loop in one process (configs[1])."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    wl = workload.zipf_workload(n, 512, 1, seed=0x5EED)
    c0, c1 = fhh.KeyCollection(512, 1), fhh.KeyCollection(512, 1)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    res = {"host": [], "device": []}
    kern = {"host": [], "device": []}
    for r in range(rounds + 1):
        for mode in ("host", "device"):
            c0.reset_stats()
            t0 = time.perf_counter()
            fhh.sim_crawl(c0, c1, 0.001, record=False, host_loop=(mode == "host"), init_capacity=1024)
            dt = (time.perf_counter() - t0) * 1e3
            if r:
                res[mode].append(dt)
                kern[mode].append(c0.stats()["expand_ms"])
    for m in res:
        print(f"{m:7s} wall {statistics.median(res[m]):8.1f} ms  k_expand {statistics.median(kern[m]):8.1f} ms  "
              f"all {[round(x, 1) for x in res[m]]}", flush=True)


if __name__ == "__main__":
    main()
