"""Does the vector-memory (L1) gather path add AES-table lookup throughput beside a
saturated LDS? Runs fhh_microbench_gather for every (LDS chains, global chains) combo and a
few global table spans (tools/gather_probe.py > gpurun_out/gather_probe.log)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import json

from fuzzyheavyhitters_amd import _lib

COMBOS = [(8, 0), (0, 8), (0, 16), (8, 1), (8, 2), (8, 4), (6, 2), (4, 4), (12, 2)]


def main():
    lib = _lib.lib()
    res = []
    for gb in (1024, 4096, 16384):
        for c, (nl, ng) in enumerate(COMBOS):
            if gb != 4096 and nl and ng == 0:
                continue
            r = ctypes.c_double()
            rc = lib.fhh_microbench_gather(0, c, gb, ctypes.byref(r))
            assert rc == 0, rc
            row = {"lds_chains": nl, "global_chains": ng, "gbytes": gb, "G_lookups_per_s": r.value / 1e9,
                   "lds_TBps_equiv": r.value * nl / (nl + ng) * 4 / 1e12}
            res.append(row)
            print(json.dumps(row), flush=True)




def hybrid():
    """fhh_microbench_hybrid: lookups/s of LDS waves beside nb VALU-only waves per workgroup;
    'blocks' converts to AES blocks/s at 144 lookups (T-table) and 520 bitop3 (bitsliced)."""
    lib = _lib.lib()
    for nb in (0, 2, 4, 6, 8):
        r = (ctypes.c_double * 2)()
        assert lib.fhh_microbench_hybrid(0, nb, r) == 0
        print(json.dumps({"valu_waves_per_wg": nb, "T_lookups_per_s": r[0] / 1e12, "T_bitop3_per_s": r[1] / 1e12,
                          "G_blocks_ttable": r[0] / 144 / 1e9, "G_blocks_bitsliced": r[1] / 520 / 1e9,
                          "G_blocks_total": (r[0] / 144 + r[1] / 520) / 1e9}), flush=True)


if __name__ == "__main__":
    if "--hybrid" in sys.argv:
        hybrid()
    else:
        main()
