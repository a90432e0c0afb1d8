#!/usr/bin/env python3
"""Debug aid: run the configs[4] level-batched FE verification and report the (level, key)
pairs whose ok bit disagrees with the workload's ground truth, re-checking a few with the oracle."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    keys = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000
    levels = int(sys.argv[2]) if len(sys.argv) > 2 else 1023
    nodes = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import sketch as S
    from oracle import oracle as O
    wl = S.sketch_workload(keys, nodes, seed=0x5EED, bad_fraction=0.01)
    kc = fhh.KeyCollection(8, 1)
    b = S.DeviceSketchBatch(wl)
    S.deal_triples(kc, b, levels=levels, seed=0x5EED)
    S.sim_sketch_verify(kc, b, level=0, n_levels=levels)
    ok = b.ok.cpu().numpy().astype(bool)
    bad = np.argwhere(ok != wl.honest[None, :])
    print("mismatches", len(bad), "levels with any", len(np.unique(bad[:, 0])) if len(bad) else 0, flush=True)
    print("first", bad[:10].tolist(), flush=True)
    if len(bad):
        lv_counts = np.bincount(bad[:, 0], minlength=levels)
        print("per-level counts (first 40 levels)", lv_counts[:40].tolist(), flush=True)
        tr = [t.cpu().numpy().view(np.uint64) for t in b.triples]
        for lv, k in bad[:3]:
            seeds = wl.seeds[k:k + 1].copy()
            seeds[:, 12:16] ^= np.frombuffer(np.uint32(lv).tobytes(), np.uint8)
            ok_e, _ = O.sketch_verify_fe(seeds, wl.x[0][k:k + 1], wl.kx[0][k:k + 1], wl.x[1][k:k + 1],
                                         wl.kx[1][k:k + 1], np.stack(wl.mac)[:, k:k + 1], np.stack(wl.mac2)[:, k:k + 1],
                                         np.stack([tr[0][k:k + 1, lv], tr[1][k:k + 1, lv]]))
            print("level", lv, "key", k, "gpu", ok[lv, k], "oracle", ok_e[0], "honest", wl.honest[k], flush=True)


if __name__ == "__main__":
    main()
