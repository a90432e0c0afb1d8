"""r06: where the drop-in's cold 1M crawl loses time — per-level (crawl, gcot, node sums) of a cold and a warm
two_party_crawl on the metric's workload, and the levels with the largest cold - warm difference."""
import json
import sys
import time

sys.path.insert(0, ".")
import fuzzyheavyhitters_amd as fhh  # noqa: E402
from fuzzyheavyhitters_amd import workload  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] == "dirty":   # touch and free 120 GB of HBM first (as the bench's fused leg)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    bufs = []
    for _ in range(8):
        q = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(q), ctypes.c_size_t(15 << 30)) == 0
        hip.hipMemset(q, 0x5A, ctypes.c_size_t(15 << 30))
        bufs.append(q)
    hip.hipDeviceSynchronize()
    for q in bufs:
        hip.hipFree(q)
    print("dirtied 120 GB", file=sys.stderr, flush=True)
wl = workload.zipf_workload(1_000_000, 512, 1, num_sites=10_000, zipf_s=1.03, ball_size=1, seed=0x5EED)
if len(sys.argv) > 1 and sys.argv[1] == "fused":   # the bench's order: a fused protocol crawl on its own pair first
    f0 = fhh.KeyCollection(512, 1)
    f1 = fhh.KeyCollection(512, 1)
    fhh.gen_keys_pair(f0, f1, wl.left, wl.right, wl.root_seeds)
    t0 = time.perf_counter()
    fhh.sim_crawl(f0, f1, 0.001, mode="fe", prf_seed=7, gc="ot", record=False, ot_ss_k=2)
    print(f"fused: {time.perf_counter() - t0:.2f} s", file=sys.stderr, flush=True)
    del f0, f1
p0 = fhh.KeyCollection(512, 1)
p1 = fhh.KeyCollection(512, 1)
fhh.gen_keys_pair(p0, p1, wl.left, wl.right, wl.root_seeds)
logs = []
for run in range(2):
    lg = []
    t0 = time.perf_counter()
    fhh.two_party_crawl(p0, p1, 0.001, channel="inplace", record=False, material="fresh", level_log=lg, ot_ss_k=2)
    print(f"run {run}: {time.perf_counter() - t0:.2f} s", file=sys.stderr, flush=True)
    logs.append(lg)
cold, warm = logs
diff = sorted(((c[2] + c[3] + c[4]) - (w[2] + w[3] + w[4]), c[0], c[1], c[2] - w[2], c[3] - w[3], c[4] - w[4])
              for c, w in zip(cold, warm))[::-1]
tot = {k: sum(x[i] for x in cold) - sum(x[i] for x in warm) for k, i in (("crawl", 2), ("gcot", 3), ("sums", 4))}
print(json.dumps({"cold_minus_warm_by_phase_s": tot,
                  "top_levels": [{"level": d[1], "children": d[2], "extra_s": d[0], "crawl": d[3], "gcot": d[4],
                                  "sums": d[5]} for d in diff[:15]]}))
