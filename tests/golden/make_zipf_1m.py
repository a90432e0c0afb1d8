#!/usr/bin/env python3
"""Golden fixture of the north star's own output: 1M Zipf clients at data_len 512.

The metric's configuration (BASELINE.json `north_star`, configs[2] = configs[1]'s generator at
1M clients): num_sites 10 000, s = 1.03, ball 1, d = 1, seed 0x5EED, threshold 0.001 -> count
threshold max(1, floor(0.001 * 1e6)) = 1000 at every level (leader.rs:193-194, 245-246).

The expected output is what the two-server protocol recovers, computed without cryptography by
`workload.plaintext_crawl` (a client is inside a node iff l[:k] <= prefix <= r[:k], SURVEY A.3;
child order collect.rs:379-391 / lib.rs:125-129; keep iff count >= threshold,
collect.rs:945-989). That recount equals the oracle's crawl on every small golden workload
(tests/test_oracle_crawl.py::test_plaintext_crawl_equals_oracle). It takes ~110 s on this
container's CPUs, so it is run once here and committed:

  level_children [L]        u32  children evaluated per level (C_l)
  counts         [sum C_l]  u32  every child's count, level after level
  paths          [H][L/8]   u8   the heavy hitters' paths, MSB-first bits packed big-endian
  values         [H]        u64  their final counts
  left_sha256 / right_sha256     digests of the workload's interval bounds, so a test notices a
                                 changed generator instead of comparing against stale counts

Usage: python tests/golden/make_zipf_1m.py   (writes tests/golden/zipf_1m_L512.npz)
"""
import hashlib
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

N, L, NUM_SITES, ZIPF_S, SEED, THRESHOLD = 1_000_000, 512, 10_000, 1.03, 0x5EED, 0.001


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint8).tobytes()).hexdigest()


def main():
    from fuzzyheavyhitters_amd import workload
    t0 = time.time()
    wl = workload.zipf_workload(N, L, 1, num_sites=NUM_SITES, zipf_s=ZIPF_S, ball_size=1, seed=SEED)
    thr = max(1, int(THRESHOLD * N))
    counts, paths, finals = workload.plaintext_crawl(wl.left, wl.right, thr, thr)
    level_children = np.array([len(c) for c in counts], np.uint32)
    flat = np.concatenate([np.asarray(c, np.uint64) for c in counts])
    assert flat.max() < 2**32
    pbits = np.array([p[0] for p in paths], np.uint8).reshape(len(paths), L)
    out = os.path.join(HERE, "zipf_1m_L512.npz")
    np.savez_compressed(out, n=np.uint64(N), data_len=np.uint32(L), num_sites=np.uint32(NUM_SITES),
                        zipf_s=np.float64(ZIPF_S), seed=np.uint64(SEED), threshold=np.float64(THRESHOLD),
                        thr=np.uint64(thr), level_children=level_children, counts=flat.astype(np.uint32),
                        paths=np.packbits(pbits, axis=1, bitorder="big"), values=np.array(finals, np.uint64),
                        left_sha256=np.array(digest(wl.left)), right_sha256=np.array(digest(wl.right)))
    print(f"{out}: {int(level_children.sum())} children over {L} levels, {len(paths)} heavy hitters "
          f"({time.time() - t0:.1f} s)")


if __name__ == "__main__":
    main()
