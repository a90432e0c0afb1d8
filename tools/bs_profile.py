#!/usr/bin/env python3
"""Phase-cycle breakdown of the bitsliced pair kernel (profiling variant kBsVariant + 6) on the
bench workload: item fetch / seed fetch / LDS->regs / AES / MMO+stores / end barrier."""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=100_000)
    ap.add_argument("--variant", type=int, default=20)
    args = ap.parse_args()
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import workload
    lib = fhh.lib()
    lib.fhh_debug_bs_profile.argtypes = [ctypes.POINTER(ctypes.c_double)]
    wl = workload.zipf_workload(args.clients, 512, 1, seed=0x5EED)
    c0, c1 = fhh.KeyCollection(512, 1), fhh.KeyCollection(512, 1)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    c0.set_variant(args.variant)
    c1.set_variant(args.variant)
    fhh.sim_crawl(c0, c1, 0.001, record=False)
    out = (ctypes.c_double * 6)()
    lib.fhh_debug_bs_profile(out)   # reset after warmup
    c0.reset_stats()
    fhh.sim_crawl(c0, c1, 0.001, record=False)
    lib.fhh_debug_bs_profile(out)
    st = c0.stats()
    tot = sum(out)
    names = ["item fetch", "seed fetch+barrier", "LDS->regs/mask/inc", "AES", "MMO+stores", "end barrier"]
    for n, v in zip(names, out):
        print(f"{n:22s} {v / tot * 100:6.1f} %")
    print(f"kernel {st['expand_ms']:.1f} ms, {st['expand_blocks_timed'] / st['expand_ms'] / 1e6:.1f} G blocks/s")


if __name__ == "__main__":
    main()
