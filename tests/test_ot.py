"""The OT of row f1: IKNP/ALSZ OT extension (ocelot's AlszSender/AlszReceiver at
equalitytest.rs:67-82 and collect.rs:437-471; ocelot is not vendored, so the wire format is
parity-unpinned). The oracle restatement is pinned by the OT functionality (the receiver gets
exactly x^{choice}, for explicit and correlated messages) and by the protocol's algebra (the
sender's rows satisfy q_j = t_j ^ r_j s, checked through the transcript); the HIP path is then
bit-exact against the oracle on the output and both protocol messages (U, Y0, Y1)."""
import numpy as np
import pytest


def _inputs(m, seed):
    rng = np.random.default_rng(seed)
    ch = rng.integers(0, 2, m, dtype=np.uint8)
    x0 = rng.integers(0, 256, (m, 16), dtype=np.uint8)
    x1 = rng.integers(0, 256, (m, 16), dtype=np.uint8)
    seeds = rng.integers(0, 256, (128, 2, 16), dtype=np.uint8)
    s = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    delta = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
    return ch, x0, x1, seeds, s, delta


@pytest.mark.parametrize("m", [1, 127, 128, 129, 1000, 4099])
def test_oracle_ot_functionality(oracle, m):
    ch, x0, x1, seeds, s, delta = _inputs(m, m)
    out = oracle.ot_extend(ch, x0, x1, None, seeds, s, tweak_base=3)
    assert np.array_equal(out, np.where(ch[:, None] == 1, x1, x0))
    out = oracle.ot_extend(ch, x0, None, delta, seeds, s, tweak_base=3)
    assert np.array_equal(out, np.where(ch[:, None] == 1, x0 ^ np.frombuffer(delta, np.uint8), x0))


def test_oracle_ot_transcript_hides_the_unchosen_message(oracle):
    """Y_{1-r} is x_{1-r} masked by H(j, t_j ^ s): a receiver that tries H(j, t_j) on the other
    reply gets garbage, not the other message; and flipping one base choice bit changes U only
    through the sender's side (U is the receiver's message and does not depend on s)."""
    m = 300
    ch, x0, x1, seeds, s, _ = _inputs(m, 7)
    out, u, y0, y1 = oracle.ot_extend(ch, x0, x1, None, seeds, s, transcript=True)
    assert np.array_equal(out, np.where(ch[:, None] == 1, x1, x0))
    s2 = bytes([s[0] ^ 1]) + s[1:]
    out2, u2, _, _ = oracle.ot_extend(ch, x0, x1, None, seeds, s2, transcript=True)
    assert np.array_equal(u, u2) and np.array_equal(out2, out)
    assert not np.array_equal(y0, x0) and not np.array_equal(y1, x1)


@pytest.mark.gpu
@pytest.mark.parametrize("m", [1, 127, 128, 129, 1000, 8192, 8193, 100_000])
def test_gpu_ot_bit_exact(oracle, m):
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import ot
    ch, x0, x1, seeds, s, delta = _inputs(m, m + 1)
    kc = fhh.KeyCollection(8, 1)
    for corr in (False, True):
        args = dict(x1=None, delta=delta) if corr else dict(x1=x1, delta=None)
        got, u, y0, y1 = ot.ot_extend(kc, ch, x0, base_seeds=seeds, base_choice=s, tweak_base=11, transcript=True,
                                      **args)
        exp, eu, ey0, ey1 = oracle.ot_extend(ch, x0, args["x1"], args["delta"], seeds, s, tweak_base=11,
                                             transcript=True)
        assert np.array_equal(got, exp)
        assert np.array_equal(u, eu)
        assert np.array_equal(y0, ey0) and np.array_equal(y1, ey1)
        want = np.where(ch[:, None] == 1, x0 ^ np.frombuffer(delta, np.uint8) if corr else x1, x0)
        assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("m", [33, 1000, 8193])
def test_gpu_ot_extend_device_buffers(oracle, m):
    """fhh_ot_extend_device on device buffers (torch tensors on cuda:0): the choice words carry
    garbage past bit m, which the call clears in stream order; outputs equal the oracle's."""
    import ctypes
    import torch
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd._lib import FhhOtBatch, check, lib
    ch, x0, x1, seeds, s, _ = _inputs(m, 3 * m)
    words = (m + 31) // 32
    cw = np.zeros(words * 32, np.uint8)
    cw[:m] = ch
    cw[m:] = 1                                            # garbage past m
    packed = np.packbits(cw.reshape(words, 32), axis=1, bitorder="little").view(np.uint32).reshape(words)
    kc = fhh.KeyCollection(8, 1)
    d_ch = torch.from_numpy(packed.view(np.int32).copy()).cuda()
    d_x0 = torch.from_numpy(x0.copy()).cuda()
    d_x1 = torch.from_numpy(x1.copy()).cuda()
    d_out = torch.zeros((m, 16), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    b = FhhOtBatch()
    b.m = m
    b.choices_dev = d_ch.data_ptr()
    b.x0_dev = d_x0.data_ptr()
    b.x1_dev = d_x1.data_ptr()
    b.out_dev = d_out.data_ptr()
    ctypes.memmove(b.base_seeds, seeds.tobytes(), 128 * 2 * 16)
    ctypes.memmove(b.base_choice, s, 16)
    check(lib().fhh_ot_extend_device(kc.handle, ctypes.byref(b)), kc.handle)
    got = d_out.cpu().numpy()
    exp = oracle.ot_extend(ch, x0, x1, None, seeds, s)
    assert np.array_equal(got, exp)
    assert np.array_equal(got, np.where(ch[:, None] == 1, x1, x0))


@pytest.mark.gpu
def test_gpu_ot_default_base_material_is_fresh():
    """Without explicit base material every batch draws its own (os.urandom): the receiver's
    message U differs between two batches on the same choices, the outputs are still right."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import ot
    ch, x0, x1, _, _, _ = _inputs(500, 5)
    kc = fhh.KeyCollection(8, 1)
    a, ua, _, _ = ot.ot_extend(kc, ch, x0, x1, transcript=True)
    b, ub, _, _ = ot.ot_extend(kc, ch, x0, x1, transcript=True)
    want = np.where(ch[:, None] == 1, x1, x0)
    assert np.array_equal(a, want) and np.array_equal(b, want)
    assert not np.array_equal(ua, ub)


def _co15(count, choices, seed):
    import ctypes
    from fuzzyheavyhitters_amd._lib import lib, u8p
    ch = np.packbits(np.asarray(choices, np.uint8), bitorder="little")
    sk = np.zeros((count, 2, 16), np.uint8)
    rk = np.zeros((count, 16), np.uint8)
    sd = np.frombuffer(seed, np.uint8).copy()
    rc = lib().fhh_base_ot_co15(count, ch.ctypes.data_as(u8p), sd.ctypes.data_as(u8p), sk.ctypes.data_as(u8p),
                                rk.ctypes.data_as(u8p))
    assert rc == 0, lib().fhh_base_ot_last_error()
    return sk, rk


def test_co15_base_ot_functionality():
    """Chou–Orlandi base OTs (the OT extension's init, collect.rs:454-471; host code in libfhh.so,
    no GPU): the receiver's key is the sender's key of its choice and differs from the other one;
    the split-party entry points give the same keys as the in-process call; a non-point is
    rejected."""
    import ctypes
    from fuzzyheavyhitters_amd._lib import lib, u8p
    rng = np.random.default_rng(9)
    choices = rng.integers(0, 2, 128, dtype=np.uint8)
    seed = bytes(rng.integers(0, 256, 32, dtype=np.uint8))
    sk, rk = _co15(128, choices, seed)
    assert np.array_equal(rk, sk[np.arange(128), choices])
    assert not np.any(np.all(rk == sk[np.arange(128), 1 - choices], axis=1))
    assert len({bytes(k) for k in sk.reshape(-1, 16)}) == 256          # all sender keys distinct
    sk2, rk2 = _co15(128, choices, bytes([seed[0] ^ 1]) + seed[1:])
    assert not np.array_equal(sk, sk2)                                  # fresh seed, fresh keys
    # split parties
    sa = rng.integers(0, 256, 32, dtype=np.uint8)
    sb = rng.integers(0, 256, 32, dtype=np.uint8)
    A = np.zeros(65, np.uint8)
    assert lib().fhh_co15_sender_start(sa.ctypes.data_as(u8p), A.ctypes.data_as(u8p)) == 0
    ch = np.packbits(choices[:40], bitorder="little")
    B = np.zeros((40, 65), np.uint8)
    kr = np.zeros((40, 16), np.uint8)
    assert lib().fhh_co15_receiver(40, A.ctypes.data_as(u8p), ch.ctypes.data_as(u8p), sb.ctypes.data_as(u8p),
                                   B.ctypes.data_as(u8p), kr.ctypes.data_as(u8p)) == 0
    ks = np.zeros((40, 2, 16), np.uint8)
    assert lib().fhh_co15_sender_finish(40, sa.ctypes.data_as(u8p), B.ctypes.data_as(u8p),
                                        ks.ctypes.data_as(u8p)) == 0
    assert np.array_equal(kr, ks[np.arange(40), choices[:40]])
    bad = A.copy()
    bad[1:] ^= 0x5A                                                      # not on the curve
    assert lib().fhh_co15_receiver(1, bad.ctypes.data_as(u8p), ch.ctypes.data_as(u8p), sb.ctypes.data_as(u8p),
                                   B.ctypes.data_as(u8p), kr.ctypes.data_as(u8p)) != 0


# ---- r05: correlated OT extension (the protocol's two OTs as ALSZ C-OT) ------------------------------
FE_P = (1 << 62) - (1 << 30) - 1
P255 = (1 << 255) - 19


def _bp_int(b):
    return int.from_bytes(bytes(b), "big")


@pytest.mark.parametrize("m", [1, 128, 1000, 4099])
@pytest.mark.parametrize("ctr_off", [0, 256, 1 << 20])
def test_oracle_cot_functionality(oracle, m, ctr_off):
    """The three C-OT modes deliver what the reference's plain OTs deliver (collect.rs:437-471,
    equalitytest.rs:67-82): labels out = x0 ^ r Delta with x0 the sender's H(q_j); FE / FieldElm
    shares with v_garbler - v_receiver = 1 iff the choice differs from the garbler's mask (eq = mask ^ o,
    A.5), every value canonical (the receiver's FieldElm unreduced < 2^256, == mod p)."""
    ch, _, _, seeds, s, delta = _inputs(m, m + ctr_off)
    # labels
    x0, out, u, y = oracle.cot_extend(oracle.COT_LABELS, ch, seeds, s, delta=delta, ctr_off=ctr_off)
    D = np.frombuffer(delta, np.uint8)
    assert np.array_equal(out, np.where(ch[:, None] == 1, x0 ^ D, x0))
    # labels as the IKNP correlation (r05b): t_j = q_j ^ r_j s, no reply; the pads are the plain /
    # hashed C-OT's pre-images (the same rows, unhashed)
    q, t, u4, _ = oracle.cot_extend(oracle.COT_RAW, ch, seeds, s, ctr_off=ctr_off)
    S = np.frombuffer(s, np.uint8)
    assert np.array_equal(t, np.where(ch[:, None] == 1, q ^ S, q))
    assert np.array_equal(u4, u)
    # FE share, both masks
    for mask in (0, 1):
        gv, ev, _, _ = oracle.cot_extend(oracle.COT_FE, ch, seeds, s, mask=mask, ctr_off=ctr_off)
        assert int(gv.max()) < FE_P and int(ev.max()) < FE_P
        diff = (gv.astype(object) - ev.astype(object)) % FE_P
        assert np.array_equal(diff.astype(np.uint64), (ch != mask).astype(np.uint64))
    # FieldElm share: pairs (2t, 2t + 1) with one choice
    mm = 2 * ((m + 1) // 2)
    ch2 = np.repeat(ch[: mm // 2], 2)
    for mask in (0, 1):
        gv, ev, _, y2 = oracle.cot_extend(oracle.COT_FE255, ch2, seeds, s, mask=mask, ctr_off=ctr_off)
        for t in range(mm // 2):
            g, e = _bp_int(gv[t]), _bp_int(ev[t])
            assert g < P255 and e < (1 << 256)
            assert (g - e) % P255 == (1 if ch2[2 * t] != mask else 0)


def test_oracle_cot_counter_offset_gives_fresh_pads(oracle):
    """Batches extending one set of base OTs at disjoint row-PRG counters (the party ABI's running
    session counter) get unrelated pads: U and y differ, while each batch stays correct. The same
    counter twice would repeat U ^ choices (the ADVICE r04 hazard)."""
    m = 600
    ch, _, _, seeds, s, delta = _inputs(m, 77)
    a = oracle.cot_extend(oracle.COT_LABELS, ch, seeds, s, delta=delta, ctr_off=0)
    b = oracle.cot_extend(oracle.COT_LABELS, ch, seeds, s, delta=delta, ctr_off=256)
    c = oracle.cot_extend(oracle.COT_LABELS, ch, seeds, s, delta=delta, ctr_off=0)
    assert not np.array_equal(a[2], b[2]) and not np.array_equal(a[0], b[0])
    assert np.array_equal(a[2], c[2])
    # at ctr_off 0 the C-OT's row matrices equal the plain OT's (same base material, same counters)
    _, u_plain, _, _ = oracle.ot_extend(ch, a[0], None, delta, seeds, s, transcript=True)
    assert np.array_equal(a[2], u_plain)


def test_oracle_gc_aes_ni_matches_bytewise(oracle):
    """Row f1's restatement on AES-NI (the CPU baseline's path) equals the byte-wise FIPS-197 path."""
    if not oracle.aes_ni_available():
        pytest.skip("no AES-NI on this CPU")
    m = 700
    ch, x0, x1, seeds, s, delta = _inputs(m, 3)
    try:
        oracle.gc_set_ni(True)
        a = oracle.ot_extend(ch, x0, x1, None, seeds, s, transcript=True)
        ca = oracle.cot_extend(oracle.COT_FE, ch, seeds, s, mask=1, ctr_off=512)
        oracle.gc_set_ni(False)
        b = oracle.ot_extend(ch, x0, x1, None, seeds, s, transcript=True)
        cb = oracle.cot_extend(oracle.COT_FE, ch, seeds, s, mask=1, ctr_off=512)
    finally:
        oracle.gc_set_ni(True)
    for p, q in zip(a, b):
        assert np.array_equal(p, q)
    for p, q in zip(ca, cb):
        assert np.array_equal(p, q)


@pytest.mark.gpu
@pytest.mark.parametrize("m", [1, 127, 1000, 8193, 100_000])
def test_gpu_cot_bit_exact(oracle, m):
    """GPU correlated OT (every mode, at a nonzero session counter) = the oracle: both parties'
    outputs and both protocol messages (U, y; mode 4 has no y)."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import ot
    ch, _, _, seeds, s, delta = _inputs(m, 5 * m + 1)
    kc = fhh.KeyCollection(8, 1)
    for ctr_off in (0, 512):
        got = ot.cot_extend(kc, 1, ch, seeds, s, delta=delta, ctr_off=ctr_off, transcript=True)
        exp = oracle.cot_extend(oracle.COT_LABELS, ch, seeds, s, delta=delta, ctr_off=ctr_off)
        for g, e in zip(got, exp):
            assert np.array_equal(g, e)
        got = ot.cot_extend(kc, 4, ch, seeds, s, ctr_off=ctr_off, transcript=True)
        exp = oracle.cot_extend(oracle.COT_RAW, ch, seeds, s, ctr_off=ctr_off)
        for g, e in zip(got[:3], exp[:3]):   # q, t, U (no y)
            assert np.array_equal(g, e)
        for mask in (0, 1):
            got = ot.cot_extend(kc, 2, ch, seeds, s, mask=mask, ctr_off=ctr_off, transcript=True)
            exp = oracle.cot_extend(oracle.COT_FE, ch, seeds, s, mask=mask, ctr_off=ctr_off)
            for g, e in zip(got, exp):
                assert np.array_equal(g, e)
        mm = 2 * ((m + 1) // 2)
        ch2 = np.repeat(ch[: mm // 2], 2)
        for mask in (0, 1):
            got = ot.cot_extend(kc, 3, ch2, seeds, s, mask=mask, ctr_off=ctr_off, transcript=True)
            exp = oracle.cot_extend(oracle.COT_FE255, ch2, seeds, s, mask=mask, ctr_off=ctr_off)
            for g, e in zip(got, exp):
                assert np.array_equal(g, e)
