"""Field constants and limb conversions used by the host-side mirror.

FE    : p = 2^62 - 2^30 - 1   (src/fastfield.rs:24-28)
FE255 : p = 2^255 - 19        (src/field.rs:19, MODULUS_STR; the comment on :18 is wrong)
"""
from __future__ import annotations

import numpy as np

FE_P = (1 << 62) - (1 << 30) - 1
FE255_P = (1 << 255) - 19


def limbs10_to_int(limbs) -> int:
    return sum(int(x) << (32 * k) for k, x in enumerate(np.asarray(limbs, np.uint64)))


def int_to_limbs(v: int, n: int):
    return [(v >> (32 * k)) & 0xFFFFFFFF for k in range(n)]


def fe255_to_limbs8(v: int):
    """FieldElm value (< 2^256) -> 8 u32 little-endian limbs."""
    return int_to_limbs(v, 8)
