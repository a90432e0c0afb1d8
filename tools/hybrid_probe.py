#!/usr/bin/env python3
"""Feasibility probe for the T-table + bitsliced hybrid: two independent two-server crawls
(disjoint client halves of the configs[1] population), one per k_expand family, run alone
and then concurrently from two host threads (two HIP streams). If the concurrent wall time
beats the sum, the CU's LDS (T-table) and VALU (bitsliced) overlap."""
import argparse
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=100_000)
    ap.add_argument("--frac-tt", type=float, default=0.6)
    ap.add_argument("--vt", type=int, default=27)
    ap.add_argument("--vb", type=int, default=23)
    ap.add_argument("--rounds", type=int, default=2)
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    nA = int(args.clients * args.frac_tt) // 64 * 64
    nB = args.clients - nA
    pairs = []
    for n, v, off in ((nA, args.vt, 0), (nB, args.vb, nA)):
        wl = workload.zipf_workload(n, 512, 1, seed=0x5EED, client_offset=off)
        c0, c1 = fhh.KeyCollection(512, 1), fhh.KeyCollection(512, 1)
        fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
        c0.set_variant(v)
        c1.set_variant(v)
        pairs.append((c0, c1))

    def run(i, out):
        c0, c1 = pairs[i]
        t0 = time.perf_counter()
        fhh.sim_crawl(c0, c1, 0.001, record=False, nclients_total=args.clients)
        out[i] = time.perf_counter() - t0

    out = [0.0, 0.0]
    for p in pairs:
        p[0].reset_stats()
        p[1].reset_stats()
    for i in range(2):
        run(i, out)   # warm
    blocks = []
    for p in pairs:   # executed AES blocks of one crawl (both servers)
        blocks.append(p[0].stats()["aes_blocks"] + p[1].stats()["aes_blocks"])
    for r in range(args.rounds):
        alone = [0.0, 0.0]
        run(0, alone)
        run(1, alone)
        both = [0.0, 0.0]
        t0 = time.perf_counter()
        th = [threading.Thread(target=run, args=(i, both)) for i in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        wall = time.perf_counter() - t0
        print(f"round {r}: T-table v{args.vt} {nA} clients alone {alone[0]*1e3:.1f} ms "
              f"({blocks[0]/alone[0]/1e9:.1f} G/s), bitsliced v{args.vb} {nB} alone {alone[1]*1e3:.1f} ms "
              f"({blocks[1]/alone[1]/1e9:.1f} G/s); sequential {sum(blocks)/sum(alone)/1e9:.1f} G/s; "
              f"concurrent wall {wall*1e3:.1f} ms = {sum(blocks)/wall/1e9:.1f} G/s "
              f"(T {both[0]*1e3:.1f}, B {both[1]*1e3:.1f})", flush=True)


if __name__ == "__main__":
    main()
