"""r06: same-process A/B of the FE levels' table shares (FE vs Z_2^32) in the 1M protocol crawl (SoftSpoken k = 2,
CO15 base OTs), alternating, 2 rounds after one warm-up crawl of each."""
import json
import sys
import time

sys.path.insert(0, ".")
import torch  # noqa: E402
import fuzzyheavyhitters_amd as fhh  # noqa: E402
from fuzzyheavyhitters_amd import workload  # noqa: E402

wl = workload.zipf_workload(1_000_000, 512, 1, num_sites=10_000, zipf_s=1.03, ball_size=1, seed=0x5EED)
c0 = fhh.KeyCollection(512, 1)
c1 = fhh.KeyCollection(512, 1)
fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
out = {"fe": [], "ring32": []}
hh = {}
for rnd in range(3):
    for ring in ((True, False) if "ring-first" in sys.argv else (False, True)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = fhh.sim_crawl(c0, c1, 0.001, mode="fe", prf_seed=7, gc="ot", base_ot=True, ot_ss_k=2, table_ring32=ring,
                          record=False)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        key = "ring32" if ring else "fe"
        hh[key] = sorted((tuple(tuple(int(b) for b in p) for p in x.path), int(x.value)) for x in r.final)
        print(f"round {rnd} {key}: {dt:.2f} s, {len(r.final)} heavy hitters", file=sys.stderr, flush=True)
        if rnd > 0:
            out[key].append(dt)
out["same_heavy_hitters"] = hh["fe"] == hh["ring32"]
print(json.dumps(out))
