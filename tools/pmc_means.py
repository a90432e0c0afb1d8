#!/usr/bin/env python3
"""Per-kernel mean counter values over every pass of a tools/pmc_passes.sh run.

    python tools/pmc_means.py gpurun_out/pmc_<tag> [kernel-substring] [--json out.json]
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    src = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else ""
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in sorted(glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(p)):
            if sub and sub not in r["Kernel_Name"]:
                continue
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, d in agg.items():
        out[k] = {c: {"mean_per_dispatch": sum(v) / len(v), "dispatches": len(v)} for c, v in sorted(d.items())}
        print(k[:100])
        for c, v in sorted(d.items()):
            print(f"  {c:28s} {sum(v) / len(v):18.1f}  (n={len(v)})")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
