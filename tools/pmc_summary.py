#!/usr/bin/env python3
"""Summarise a tools/profile.sh run (gpurun_out/prof_<tag>/) into profiles/<tag>/:
kernel stats, per-kernel PMC means, and profiles/pmc_expand.json for bench.py's
roofline.traffic: HBM bytes per k_expand launch = FETCH_SIZE x 2 (gfx950 reports half of a
16-B/lane streaming read, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both in KiB x 1024.

    python tools/pmc_summary.py <tag> [--config n1000000_L512_d1]
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    config = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "n1000000_L512_d1"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    for f in ("trace/trace_kernel_stats.csv", "trace/trace_domain_stats.csv"):
        p = os.path.join(src, f)
        if os.path.exists(p):
            shutil.copy(p, os.path.join(dst, os.path.basename(f).replace("trace_", "")))
    out = {}
    for name in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_grbm", "pmc_sq2"):
        p = os.path.join(src, name, f"{name}_counter_collection.csv")
        if not os.path.exists(p):
            continue
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(p)):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, d in agg.items():
            for c, v in d.items():
                out.setdefault(k, {})[c] = {"mean_per_dispatch": sum(v) / len(v), "dispatches": len(v)}
    json.dump(out, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
    ex = out.get("k_expand", {})
    # kernel-trace durations of the same passes
    stats = {}
    p = os.path.join(src, "trace", "trace_kernel_stats.csv")
    if os.path.exists(p):
        for r in csv.DictReader(open(p)):
            stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    if "FETCH_SIZE" in ex and "WRITE_SIZE" in ex:
        fetch = ex["FETCH_SIZE"]["mean_per_dispatch"] * 1024 * 2
        write = ex["WRITE_SIZE"]["mean_per_dispatch"] * 1024
        res = {"config": config, "tag": tag, "hbm_bytes_per_launch": fetch + write,
               "fetch_bytes_corrected": fetch, "write_bytes": write,
               "k_expand_avg_ns": stats.get("k_expand", {}).get("avg_ns"),
               "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 counts half of 16-B/lane reads)"}
        if "SQ_INSTS_LDS" in ex:
            res["sq_insts_lds_per_launch"] = ex["SQ_INSTS_LDS"]["mean_per_dispatch"]
            res["sq_insts_valu_per_launch"] = ex["SQ_INSTS_VALU"]["mean_per_dispatch"]
            res["sq_lds_bank_conflict"] = ex["SQ_LDS_BANK_CONFLICT"]["mean_per_dispatch"]
        if "GRBM_GUI_ACTIVE" in ex and res["k_expand_avg_ns"]:
            res["effective_clock_ghz"] = ex["GRBM_GUI_ACTIVE"]["mean_per_dispatch"] / 8 / res["k_expand_avg_ns"]
        # profiles/pmc_expand.json holds one entry per workload (bench.py looks up its own)
        path = os.path.join(ROOT, "profiles", "pmc_expand.json")
        try:
            allp = json.load(open(path))
        except (OSError, ValueError):
            allp = {}
        if "config" in allp:          # the single-entry format of r01
            allp = {allp["config"]: allp}
        allp[config] = res
        json.dump(allp, open(path, "w"), indent=1)
        print(json.dumps(res, indent=1))
    print(json.dumps(stats, indent=1))


if __name__ == "__main__":
    main()
