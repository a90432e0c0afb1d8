"""r06: VALU op rates on the box (fhh_microbench which 0 xor, 7 alignbit, 8 add, 9 / 10 ChaCha double rounds at
8 / 2 waves per SIMD), lane-ops/s."""
import ctypes
import json
import sys

sys.path.insert(0, ".")
from fuzzyheavyhitters_amd._lib import lib  # noqa: E402

out = {}
for which, name in ((0, "v_xor_b32"), (7, "v_alignbit_b32"), (8, "v_add_u32"), (9, "chacha_qr_8w"), (10, "chacha_qr_2w"),
                    (11, "v_perm_b32"), (12, "v_lshl_or_b32")):
    r = ctypes.c_double(0)
    rc = lib().fhh_microbench(0, which, ctypes.byref(r))
    out[name] = r.value / 1e12 if rc == 0 else f"rc {rc}"
print(json.dumps(out))
