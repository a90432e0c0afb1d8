#!/usr/bin/env python3
"""Issue fractions of one kernel from a tools/pmc_passes.sh run: VALU (2 cycles per wave64
instruction per SIMD, 1024 SIMDs), LDS issue (ds_read_b32 at 128 B/clk/CU = 2 cycles per wave
instruction, 256 CUs), the waiting fractions of wave cycles, and VALU / LDS instructions per AES
block; clock = GRBM_GUI_ACTIVE / 8 XCDs / the launch's duration in the same pass's kernel trace.

    python tools/sketch_pmc.py gpurun_out/pmc_<tag> <kernel-substring> --blocks B [--json out.json]
"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    src, sub = sys.argv[1], sys.argv[2]
    blocks = float(sys.argv[sys.argv.index("--blocks") + 1])
    cnt = collections.defaultdict(list)
    dur = collections.defaultdict(list)
    name = None
    for p in sorted(glob.glob(os.path.join(src, "p*", "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(p)):
            if sub in r["Kernel_Name"]:
                name = r["Kernel_Name"]
                cnt[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for p in sorted(glob.glob(os.path.join(src, "p*", "**", "*kernel_trace.csv"), recursive=True)):
        for r in csv.DictReader(open(p)):
            if sub in r["Kernel_Name"]:
                dur[os.path.basename(p)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    m = {c: sum(v) / len(v) for c, v in cnt.items()}
    # the clock from the GRBM pass's own launches
    grbm_pass = [k for k in dur if k.startswith("p2")] or list(dur)
    t = sum(dur[grbm_pass[0]]) / len(dur[grbm_pass[0]]) * 1e-9
    clk = m["GRBM_GUI_ACTIVE"] / 8 / t
    out = {
        "kernel": name,
        "launches": len(cnt["SQ_INSTS_VALU"]),
        "us_per_launch_pmc_run": t * 1e6,
        "clock_ghz": clk / 1e9,
        "valu_frac": m["SQ_INSTS_VALU"] * 2 / (1024 * clk * t),
        "lds_issue_frac": m["SQ_INSTS_LDS"] * 2 / (256 * clk * t),
        "wait_inst_any_frac": m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"],
        "wait_any_frac": m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"],
        "valu_per_block": m["SQ_INSTS_VALU"] * 64 / blocks,
        "lds_per_block": m["SQ_INSTS_LDS"] * 64 / blocks,
        "blocks_per_launch": blocks,
    }
    print(json.dumps(out, indent=1))
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
