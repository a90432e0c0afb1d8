#!/usr/bin/env python3
"""Per-kernel dispatch counts and summed durations from the kernel traces of one tools/pmc_passes.sh
pass (the input of tools/lds_issue.py):

    python tools/pmc_durations.py gpurun_out/pmc_<tag>/p2 out.json
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    agg = collections.defaultdict(lambda: {"dispatches": 0, "total_ns": 0})
    for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            a = agg[r["Kernel_Name"]]
            a["dispatches"] += 1
            a["total_ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    json.dump(agg, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
