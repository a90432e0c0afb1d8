"""r06: configs[3] (coords, d = 2, data_len 16) crawls for a kernel trace: prints every level's live entries per
dim (the k_expand work) so the per-dispatch durations can be fitted (fixed cost per launch vs per entry)."""
import json
import sys

sys.path.insert(0, ".")
import fuzzyheavyhitters_amd as fhh  # noqa: E402
from fuzzyheavyhitters_amd import workload  # noqa: E402

wl = workload.coords_workload(1_000_000, ball_size=1, zipf_s=1.03, seed=0x5EED)
c0 = fhh.KeyCollection(16, 2)
c1 = fhh.KeyCollection(16, 2)
fhh.gen_keys_pair(c0, c1, wl.left, wl.right, wl.root_seeds)
res = None
for _ in range(6):
    res = fhh.sim_crawl(c0, c1, 0.075, mode="count")
print(json.dumps({"level_children": [int(x) for x in res.level_children],
                  "level_kept": [int(x) for x in res.level_kept]}))
