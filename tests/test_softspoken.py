"""r06: SoftSpoken OT extension (L. Roy, CRYPTO 2022; semi-honest small-field VOLE with the repetition
code) for the protocol's OTs, k = 2 and 4 base OTs per chunk: the receiver's message U shrinks from 128
rows to 128 / k (16 / k bytes per OT). No reference code exists for it (the reference runs ocelot's ALSZ,
which is not vendored): the oracle restatement (oracle/fhh_oracle.c cot_rows / ss_ggm) is pinned by the
functionality — q_j = t_j ^ r_j s, the IKNP correlation every C-OT mode consumes, and the modes' own
identities on top — and by the GGM puncturing (the sender's leaves are the receiver's except the one at
Delta_c, which it never sees); the HIP path is then bit-exact against the oracle on both parties' outputs
and both receiver messages (U and the GGM corrections)."""
import numpy as np
import pytest

FE_P = (1 << 62) - (1 << 30) - 1


def _inputs(m, seed):
    rng = np.random.default_rng(seed)
    ch = rng.integers(0, 2, m, dtype=np.uint8)
    seeds = rng.integers(0, 256, (128, 2, 16), dtype=np.uint8)
    s = bytearray(rng.integers(0, 256, 16, dtype=np.uint8).tobytes())
    s[0] |= 1   # the labels OT uses s as the free-XOR Delta
    delta = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    return ch, seeds, bytes(s), delta


@pytest.mark.parametrize("k", [2, 4])
@pytest.mark.parametrize("m", [1, 511, 513, 3000])
@pytest.mark.parametrize("ctr_off", [0, 256])
def test_oracle_softspoken_correlation(oracle, k, m, ctr_off):
    """t_j = q_j ^ r_j s (FHH_COT_RAW), the U transcript has 128 / k rows, the labels mode delivers
    x0 ^ r Delta and the FE share mode v_g - v_r = [r != mask]."""
    ch, seeds, s, delta = _inputs(m, 31 * m + k + ctr_off)
    q, t, u, _, corr = oracle.cot_extend_ss(k, oracle.COT_RAW, ch, seeds, s, ctr_off=ctr_off)
    S = np.frombuffer(s, np.uint8)
    assert np.array_equal(t, np.where(ch[:, None] == 1, q ^ S, q))
    assert u.shape == (128 // k, (m + 127) // 128, 16) and corr.shape == (128 // k, k, 2, 16)
    x0, out, _, _, _ = oracle.cot_extend_ss(k, oracle.COT_LABELS, ch, seeds, s, delta=delta, ctr_off=ctr_off)
    D = np.frombuffer(delta, np.uint8)
    assert np.array_equal(out, np.where(ch[:, None] == 1, x0 ^ D, x0))
    for mask in (0, 1):
        gv, ev, _, _, _ = oracle.cot_extend_ss(k, oracle.COT_FE, ch, seeds, s, mask=mask, ctr_off=ctr_off)
        diff = (gv.astype(object) - ev.astype(object)) % FE_P
        assert np.array_equal(diff.astype(np.uint64), (ch != mask).astype(np.uint64))


def test_oracle_softspoken_k1_is_iknp(oracle):
    m = 1500
    ch, seeds, s, delta = _inputs(m, 5)
    a = oracle.cot_extend_ss(1, oracle.COT_LABELS, ch, seeds, s, delta=delta, ctr_off=256)
    b = oracle.cot_extend(oracle.COT_LABELS, ch, seeds, s, delta=delta, ctr_off=256)
    for x, y in zip(a[:4], b):
        assert np.array_equal(x, y)


@pytest.mark.parametrize("k", [2, 4])
def test_oracle_softspoken_sender_never_sees_the_punctured_leaf(oracle, k):
    """The sender's output depends on every base key it holds but not on the ones it does not: changing
    the receiver's unchosen keys k_i^{1 - s_i} changes U and the corrections, while the correlation still
    holds; changing only the chosen keys changes q as a whole (the sender's view is re-derived)."""
    m = 700
    ch, seeds, s, _ = _inputs(m, 9 + k)
    q, t, u, _, corr = oracle.cot_extend_ss(k, oracle.COT_RAW, ch, seeds, s)
    sb = np.unpackbits(np.frombuffer(s, np.uint8), bitorder="little")
    seeds2 = seeds.copy()
    for i in range(128):
        seeds2[i, 1 - sb[i]] ^= 0x5A
    q2, t2, u2, _, corr2 = oracle.cot_extend_ss(k, oracle.COT_RAW, ch, seeds2, s)
    S = np.frombuffer(s, np.uint8)
    assert np.array_equal(t2, np.where(ch[:, None] == 1, q2 ^ S, q2))
    assert not np.array_equal(u, u2) and not np.array_equal(corr, corr2)


def test_oracle_softspoken_counter_offset_gives_fresh_pads(oracle):
    m = 600
    ch, seeds, s, _ = _inputs(m, 77)
    a = oracle.cot_extend_ss(4, oracle.COT_RAW, ch, seeds, s, ctr_off=0)
    b = oracle.cot_extend_ss(4, oracle.COT_RAW, ch, seeds, s, ctr_off=256)
    assert not np.array_equal(a[2], b[2]) and not np.array_equal(a[0], b[0])
    assert np.array_equal(a[4], b[4])   # one GGM per base-OT session


@pytest.mark.gpu
@pytest.mark.parametrize("k", [2, 4])
@pytest.mark.parametrize("m", [1, 511, 513, 1000, 8193, 100_000])
def test_gpu_softspoken_bit_exact(oracle, k, m):
    """GPU SoftSpoken C-OT (every mode, two session counters) = the oracle: both parties' outputs, U and the
    GGM corrections, and y where the mode has one."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import ot
    ch, seeds, s, delta = _inputs(m, 7 * m + k)
    kc = fhh.KeyCollection(8, 1)
    for ctr_off in (0, 512):
        got = ot.cot_extend(kc, 4, ch, seeds, s, ctr_off=ctr_off, transcript=True, ss_k=k)
        exp = oracle.cot_extend_ss(k, oracle.COT_RAW, ch, seeds, s, ctr_off=ctr_off)
        for name, g, e in zip(("q", "t", "U", "y", "corr"), got, exp):
            if name != "y":
                assert np.array_equal(g, e), name
        got = ot.cot_extend(kc, 1, ch, seeds, s, delta=delta, ctr_off=ctr_off, transcript=True, ss_k=k)
        exp = oracle.cot_extend_ss(k, oracle.COT_LABELS, ch, seeds, s, delta=delta, ctr_off=ctr_off)
        for g, e in zip(got, exp):
            assert np.array_equal(g, e)
        for mask in (0, 1):
            got = ot.cot_extend(kc, 2, ch, seeds, s, mask=mask, ctr_off=ctr_off, transcript=True, ss_k=k)
            exp = oracle.cot_extend_ss(k, oracle.COT_FE, ch, seeds, s, mask=mask, ctr_off=ctr_off)
            for g, e in zip(got, exp):
                assert np.array_equal(g, e)
