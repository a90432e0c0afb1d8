#!/usr/bin/env python3
"""Wave timeline of k_expand over one configs[1] crawl (profiling variant 36 = default 34 +
per-wave {start, exit, items} stamps, include/fhh.h fhh_wave_profile_arm). Reports, per launch
and summed over the crawl: kernel span (first start -> last exit), mean wave busy time, the
end-of-launch tail (idle of waves that left before the last one) and the ramp (table fill).

    python tools/tail_profile.py [--clients 100000] [--variant 36]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=100_000)
    ap.add_argument("--variant", type=int, default=36)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import numpy as np
    import torch
    torch.cuda.init()
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import lib, workload
    wl = workload.zipf_workload(args.clients, 512, 1, seed=0x5EED)
    c0, c1 = fhh.KeyCollection(512, 1), fhh.KeyCollection(512, 1)
    fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
    c0.set_variant(args.variant)
    c1.set_variant(args.variant)
    grid = ctypes.c_int()
    thr = ctypes.c_int()
    buf = ctypes.create_string_buffer(64)
    lib().fhh_variant_info(args.variant, buf, 64, ctypes.byref(thr), ctypes.byref(grid))
    nwaves = grid.value * thr.value // 64
    cap = 600
    dev = torch.zeros(cap * nwaves * 3, dtype=torch.int64, device="cuda")
    fhh.sim_crawl(c0, c1, 0.001, record=False)   # warm
    torch.cuda.synchronize()
    lib().fhh_wave_profile_arm(0, ctypes.c_void_p(dev.data_ptr()), cap)
    fhh.sim_crawl(c0, c1, 0.001, record=False)
    torch.cuda.synchronize()
    n = ctypes.c_uint32()
    lib().fhh_wave_profile_launches(0, ctypes.byref(n))
    lib().fhh_wave_profile_arm(0, None, 0)
    L = min(n.value, cap)
    a = dev.cpu().numpy().view(np.uint64).reshape(cap, nwaves, 3)[:L].astype(np.float64)
    start, end, items = a[..., 0], a[..., 1], a[..., 2]
    span = end.max(1) - start.min(1)                  # per launch, 10 ns ticks
    tail = (end.max(1)[:, None] - end).mean(1)        # mean idle after a wave's exit
    ramp = (start - start.min(1)[:, None]).mean(1)    # mean late start (LDS fill / dispatch)
    busy = (end - start).mean(1)
    wpb = thr.value // 64                             # waves of one workgroup (one per CU)
    wg_end = end.reshape(L, -1, wpb).max(2)
    cu_tail = (end.max(1)[:, None] - wg_end).mean(1)  # mean CU idle after its workgroup's last wave
    tot = span.sum()
    res = {"variant": args.variant, "name": buf.value.decode(), "launches": int(L), "waves": int(nwaves),
           "span_ms": tot / 1e5, "busy_ms": busy.sum() / 1e5, "tail_ms": tail.sum() / 1e5,
           "ramp_ms": ramp.sum() / 1e5, "tail_frac": float(tail.sum() / tot),
           "cu_tail_ms": cu_tail.sum() / 1e5, "cu_tail_frac": float(cu_tail.sum() / tot), "ramp_frac": float(ramp.sum() / tot),
           "items_per_wave_mean": float(items.mean()), "items_per_wave_min_median_max":
               [float(np.percentile(items.sum(0), q)) for q in (0, 50, 100)],
           "worst_launches": [{"launch": int(i), "span_us": span[i] / 100, "tail_us": tail[i] / 100}
                              for i in np.argsort(-tail)[:5]]}
    print(json.dumps(res, indent=1))
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
