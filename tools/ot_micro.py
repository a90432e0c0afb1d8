"""OT-extension microbenchmark for kernel-level A/Bs under rocprofv3: m random correlated OTs
through fhh_ot_extend_host (the expand kernels and both transpose-fused hashes), `reps` times.
Usage: python tools/ot_micro.py [m] [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fuzzyheavyhitters_amd as fhh  # noqa: E402
from fuzzyheavyhitters_amd import ot  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 25
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rng = np.random.default_rng(1)
ch = rng.integers(0, 2, m, dtype=np.uint8)
x0 = rng.integers(0, 256, (m, 16), dtype=np.uint8)
delta = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
kc = fhh.KeyCollection(8, 1)
for r in range(reps):
    out = ot.ot_extend(kc, ch, x0, delta=delta, seed=r)
exp = x0.copy()
exp[ch == 1] ^= np.frombuffer(delta, np.uint8)
print("ok" if np.array_equal(out, exp) else "MISMATCH", m, reps)
