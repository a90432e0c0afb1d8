#!/usr/bin/env python3
"""Per-kernel LDS issue rate from the PMC means of tools/pmc_passes.sh and the kernel durations:
ds_read_b32-equivalent bytes (SQ_INSTS_LDS x 64 lanes x 4 B) per second, as a fraction of the LDS
array's per-clock limit (128 B / clk / CU x CUs) at the kernel's own clock (GRBM_GUI_ACTIVE / 8 XCDs
/ duration), plus VALU instructions per LDS instruction and the waiting fraction of wave cycles.

    python tools/lds_issue.py means.json durations.json [--cus 256] [--json out.json]
"""
import json
import sys


def main():
    means = json.load(open(sys.argv[1]))
    durs = json.load(open(sys.argv[2]))
    cus = int(sys.argv[sys.argv.index("--cus") + 1]) if "--cus" in sys.argv else 256
    out = {}
    for k, c in means.items():
        short = k.split("(")[0].replace("void ", "").replace("fhh::", "")
        if "<" in short:   # keep a short template tag (k_ot_expand<true> = receiver, <false> = sender)
            base, targs = short.split("<", 1)
            short = base + "<" + targs.split(",")[0][:24].rstrip(">") + ">"
        if short in out:
            short = short + "#" + str(len(out))
        d = durs.get(k)
        if not d or "SQ_INSTS_LDS" not in c or d["dispatches"] == 0:
            continue
        t = d["total_ns"] / d["dispatches"] * 1e-9
        lds = c["SQ_INSTS_LDS"]["mean_per_dispatch"]
        if lds == 0 or t < 20e-6:
            continue
        clk = c["GRBM_GUI_ACTIVE"]["mean_per_dispatch"] / 8 / t
        rate = lds * 64 * 4 / t
        o = {
            "avg_us": round(t * 1e6, 1), "dispatches": d["dispatches"], "total_s": round(d["total_ns"] * 1e-9, 3),
            "lds_TBps_b32eq": round(rate / 1e12, 1), "clk_GHz": round(clk / 1e9, 2),
            "lds_frac_of_clock_limit": round(rate / (128 * cus * clk), 3),
            "valu_per_lds": round(c["SQ_INSTS_VALU"]["mean_per_dispatch"] / lds, 2),
        }
        if "SQ_WAIT_INST_ANY" in c and "SQ_WAVE_CYCLES" in c:
            o["wait_inst_frac"] = round(c["SQ_WAIT_INST_ANY"]["mean_per_dispatch"] /
                                        max(1.0, c["SQ_WAVE_CYCLES"]["mean_per_dispatch"]), 3)
        out[short] = o
    for k, o in sorted(out.items(), key=lambda kv: -kv[1]["total_s"]):
        print(f"{k:24s} {o}")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
