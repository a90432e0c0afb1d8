#!/usr/bin/env python3
"""Print the roofline-denominator microbenchmarks (fhh_microbench) of this device."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import fuzzyheavyhitters_amd as fhh  # noqa: E402

names = {0: "v_xor_b32 lane-ops/s (8 waves/SIMD)", 1: "ds_read_b32 bytes/s (k_expand pattern)",
         2: "v_bitop3_b32 lane-ops/s (8 waves/SIMD)", 3: "v_bitop3_b32 lane-ops/s (2 waves/SIMD)",
         4: "v_xor_b32 lane-ops/s (2 waves/SIMD)"}
out = {}
for w, nm in names.items():
    r = ctypes.c_double()
    rc = fhh.lib().fhh_microbench(0, w, ctypes.byref(r))
    out[nm] = r.value if rc == 0 else None
    print(f"{nm:45s} {r.value / 1e12:8.2f} T/s" if rc == 0 else f"{nm}: rc={rc}", flush=True)
for w, nm in {0: "256x1024 thr, 4 KiB LDS", 1: "256x1024 thr, 128 KiB LDS", 2: "alternating 256x1024/128K and 1x1024",
              3: "1x1024 thr", 4: "alternating 64 MiB writer / 1x1024", 5: "alternating 64 MiB nt writer / 1x1024",
              6: "as 2, hipGraph replay", 7: "as 4, hipGraph replay"}.items():
    r = ctypes.c_double()
    rc = fhh.lib().fhh_debug_launch_gaps(0, w, 2000, ctypes.byref(r))
    out["launch_us_" + str(w)] = r.value if rc == 0 else None
    print(f"back-to-back kernels, {nm:40s} {r.value:7.2f} us/kernel" if rc == 0 else f"gaps {w}: rc={rc}", flush=True)
if len(sys.argv) > 1:
    json.dump(out, open(sys.argv[1], "w"), indent=1)
