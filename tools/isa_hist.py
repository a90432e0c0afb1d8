#!/usr/bin/env python3
"""Instruction histogram of one kernel in a hipcc --cuda-device-only -S listing:
    python tools/isa_hist.py <file.s> <symbol-substring> [--dump out.s]"""
import collections
import sys


def main():
    path, pat = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    starts = [i for i, l in enumerate(lines) if ":" in l and pat in l.split(":")[0] and not l.startswith((".", "\t", " "))]
    if not starts:
        sys.exit(f"no symbol matching {pat}")
    i = starts[0]
    j = i
    while j < len(lines) and not lines[j].startswith(".Lfunc_end"):
        j += 1
    body = lines[i:j]
    if "--dump" in sys.argv:
        open(sys.argv[sys.argv.index("--dump") + 1], "w").write("\n".join(body))
    c = collections.Counter()
    for l in body:
        t = l.strip().split()
        if t and not t[0].startswith((".", ";")) and not t[0].endswith(":"):
            c[t[0]] += 1
    print(lines[i], "total", sum(c.values()))
    for k, v in c.most_common(60):
        print(f"{k:28s} {v}")
    for l in lines[j:j + 60]:
        if any(k in l for k in ("vgpr_count", "sgpr_count", "scratch", "spill", "Occupancy", "NumVgprs", "LDS")):
            print(l.strip())


if __name__ == "__main__":
    main()
