"""Dump fhh_debug_aes_ps input / output for offline analysis (gpurun_out/aes_ps_dump.npz)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fuzzyheavyhitters_amd import lib  # noqa: E402

rng = np.random.default_rng(11)
blk = rng.integers(0, 256, (16, 64, 16), dtype=np.uint8)
for u in range(1, 16, 2):
    hi = blk[u - 1, :, 8:].copy().view("<u8")[:, 0] + np.uint64(1)
    blk[u] = blk[u - 1]
    blk[u, :, 8:] = hi.reshape(-1, 1).view(np.uint8)
inp = np.ascontiguousarray(blk.reshape(1024, 16))
out = np.zeros_like(inp)
u8p = ctypes.POINTER(ctypes.c_uint8)
assert lib().fhh_debug_aes_ps(0, inp.ctypes.data_as(u8p), out.ctypes.data_as(u8p)) == 0
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "aes_ps_dump.npz"), inp=inp, out=out)
print("ok")
