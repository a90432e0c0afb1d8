"""The reference's own end-to-end collection scenarios, with their expected outputs.

`tests/collect_test.rs` (commented out in the reference snapshot, written against the earlier
point-DPF `KeyCollection`) crawls a handful of client strings with threshold 2 and asserts the
recovered heavy hitters and counts:

* `collect_test_eval` (collect_test.rs:6-63): ten 5-character strings; the only strings held by
  at least two clients are "abdef" (4) and "gZ???" (3) — the test fails on any other output;
* `collect_test_eval_full` (collect_test.rs:160-251): four 32-character strings assigned
  round-robin to 10 clients (3, 3, 2, 2 copies);
* `traverse_test_eval_slow` (sketch_test.rs:164-224): the same ten strings, every non-empty node
  followed (threshold 1): all five distinct strings with counts 4, 3, 1, 1, 1.

Here each client submits the interval [x, x] (ball 0) of its string, `string_to_bits` (lib.rs:90-98,
LSB-first per byte), so node counts are exact-match counts and the expected outputs carry over
unchanged. The CPU oracle runs the scenarios in every mode; the GPU runs the same keys through
the device level loop (count, FE with the FieldElm last level, and GC + OT extension in every
level) and must return the same heavy hitters and counts.
"""
import numpy as np
import pytest

EVAL_STRINGS = [b"abdef", b"abdef", b"abdef", b"ghijk", b"gZijk", b"gZ???", b"  ?*g", b"abdef", b"gZ???", b"gZ???"]
EVAL_EXPECTED = {b"abdef": 4, b"gZ???": 3}

FULL_STRINGS = [b"01234567012345670123456701234567", b"z12x45670y2345670123456701234567",
                b"612x45670y2345670123456701234567", b"912x45670y2345670123456701234567"]
FULL_CLIENTS = [FULL_STRINGS[i % 4] for i in range(10)]
FULL_EXPECTED = {FULL_STRINGS[0]: 3, FULL_STRINGS[1]: 3, FULL_STRINGS[2]: 2, FULL_STRINGS[3]: 2}

TRAVERSE_EXPECTED = {b"abdef": 4, b"gZ???": 3, b"ghijk": 1, b"gZijk": 1, b"  ?*g": 1}

# threshold fractions: max(1, floor(0.2 * 10)) = 2 (FieldElm::from(2) in collect_test.rs);
# 0.1 -> 1 (every node with a positive count, traverse_test_eval_slow's `val > 0`)
SCENARIOS = [(EVAL_STRINGS, EVAL_EXPECTED, 0.2), (FULL_CLIENTS, FULL_EXPECTED, 0.2),
             (EVAL_STRINGS, TRAVERSE_EXPECTED, 0.1)]
IDS = ["collect_test_eval", "collect_test_eval_full", "traverse_test_eval_slow"]


def point_keys_inputs(strings, seed=3):
    """left = right = string_to_bits(s): [n][1][L] 0/1, root seeds [n][1][2][2][16]."""
    from oracle import oracle
    bits = np.array([oracle.string_to_bits(s) for s in strings], dtype=np.uint8)[:, None, :]
    rng = np.random.default_rng(seed)
    roots = rng.integers(0, 256, (len(strings), 1, 2, 2, 16), dtype=np.uint8)
    return bits, bits.copy(), roots


def bits_to_string(bits) -> bytes:
    """lib.rs bits_to_string: 8 LSB-first bits per byte."""
    b = [int(x) for x in bits]
    return bytes(sum(b[8 * i + j] << j for j in range(8)) for i in range(len(b) // 8))


def as_dict(paths, values):
    return {bits_to_string(p[0]): int(v) for p, v in zip(paths, values)}


@pytest.mark.parametrize("mode", ["count", "fe"])
@pytest.mark.parametrize("strings,expected,thr", SCENARIOS, ids=IDS)
def test_oracle_reference_scenario(oracle, strings, expected, thr, mode):
    left, right, roots = point_keys_inputs(strings)
    k0, k1 = oracle.gen_keys(left, right, roots)
    res = oracle.crawl(k0, k1, thr, mode=mode)
    assert as_dict(res.final_paths, res.final_values) == expected


@pytest.mark.gpu
@pytest.mark.parametrize("mode,gc", [("count", False), ("fe", False), ("fe", "ot")], ids=["count", "fe", "fe-gc-ot"])
@pytest.mark.parametrize("strings,expected,thr", SCENARIOS, ids=IDS)
def test_gpu_reference_scenario(oracle, strings, expected, thr, mode, gc):
    import fuzzyheavyhitters_amd as fhh
    left, right, roots = point_keys_inputs(strings)
    L = left.shape[2]
    c0, c1 = fhh.KeyCollection(L, 1), fhh.KeyCollection(L, 1)
    fhh.gen_keys_pair(c0, c1, left, right, roots)
    res = fhh.sim_crawl(c0, c1, thr, mode=mode, gc=gc)
    got = {bits_to_string(r.path[0]): int(r.value) for r in res.final}
    assert got == expected
    # and the same as the oracle's crawl on the same keys, level by level
    k0, k1 = oracle.gen_keys(left, right, roots)
    ores = oracle.crawl(k0, k1, thr, mode="count")
    assert list(res.level_children) == list(ores.n_children)
