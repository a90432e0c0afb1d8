"""Row a9 (sketch.rs / mpc.rs — fully commented out in the reference, so parity is unpinned
beyond what is checked here): pin the oracle's restatement of PrgStream (AES-128-CTR against
OpenSSL), of sketch_at (against an independent pure-Python restatement) and of the MulState
Beaver check (the protocol's own identities: honest keys verify, malformed ones do not —
the property mpc_test.rs:8-69 asserts), then the HIP path against the oracle (-m gpu)."""
import ctypes
import ctypes.util

import numpy as np
import pytest

P = (1 << 62) - (1 << 30) - 1


def _openssl_aes(key: bytes):
    path = ctypes.util.find_library("crypto")
    if not path:
        pytest.skip("libcrypto not present")
    L = ctypes.CDLL(path)
    ks = ctypes.create_string_buffer(512)
    assert L.AES_set_encrypt_key(key, 128, ks) == 0

    def enc(block: bytes) -> bytes:
        out = ctypes.create_string_buffer(16)
        L.AES_encrypt(block, out, ks)
        return out.raw
    return enc


def _py_stream(seed: bytes):
    """PrgSeed::to_rng + next_u64 (prg.rs:82-90,161-182): AES-128-CTR (big-endian 128-bit
    counter from IV 0), keystream consumed 8 bytes per draw, little-endian."""
    enc = _openssl_aes(seed)
    pos = 0
    while True:
        ks = enc((pos // 2).to_bytes(16, "big"))
        yield int.from_bytes(ks[8 * (pos % 2): 8 * (pos % 2) + 8], "little")
        pos += 1


def _py_sketch(seed: bytes, x, kx):
    """sketch_at (sketch.rs:157-200) for T = FE with Python ints; FE::from_rng redraws while
    the low 62 bits are >= p (field.rs:252-264, fastfield.rs:125-139)."""
    st = _py_stream(seed)

    def fe():
        while True:
            v = next(st) & ((1 << 62) - 1)
            if v < P:
                return v
    r1, r2, r3 = fe(), fe(), fe()
    rx = r2x = rkx = 0
    for xi, kxi in zip(x, kx):
        r = fe()
        rx = (rx + int(xi) * r) % P
        r2x = (r2x + int(xi) * r * r) % P
        rkx = (rkx + int(kxi) * r) % P
    return [rx, r2x, rkx, r1, r2, r3]


def test_prg_stream_matches_openssl_ctr(oracle):
    rng = np.random.default_rng(3)
    for _ in range(5):
        seed = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
        st = _py_stream(seed)
        for pos in range(7):
            assert oracle.prg_stream_u64(seed, pos) == next(st)


def test_sketch_oracle_vs_python(oracle):
    from fuzzyheavyhitters_amd import sketch as S
    wl = S.sketch_workload(12, 9, seed=11, bad_fraction=0.3)
    got = oracle.sketch_fe(wl.seeds, wl.x[0], wl.kx[0])
    for i in range(12):
        assert list(map(int, got[i])) == _py_sketch(bytes(wl.seeds[i]), wl.x[0][i], wl.kx[0][i])


def test_beaver_identities(oracle):
    """honest keys verify, malformed vectors / triples / MAC shares do not (mpc_test.rs)."""
    from fuzzyheavyhitters_amd import sketch as S
    wl = S.sketch_workload(300, 21, seed=5, bad_fraction=0.2)
    args = (wl.seeds, wl.x[0], wl.kx[0], wl.x[1], wl.kx[1], np.stack(wl.mac), np.stack(wl.mac2), np.stack(wl.triples))
    ok, outs = oracle.sketch_verify_fe(*args)
    assert ok[wl.honest].all() and not ok[~wl.honest].any()
    # a wrong triple (c off by one) and a wrong MAC share both break the check
    t = np.stack(wl.triples).copy()
    t[0, :, 2] = (t[0, :, 2] + 1) % P
    ok2, _ = oracle.sketch_verify_fe(*args[:7], t)
    assert not ok2.any()
    kx1 = wl.kx[1].copy()
    kx1[:, 0] = (kx1[:, 0] + 1) % P
    ok3, _ = oracle.sketch_verify_fe(wl.seeds, wl.x[0], wl.kx[0], wl.x[1], kx1, np.stack(wl.mac), np.stack(wl.mac2),
                                     np.stack(wl.triples))
    assert not ok3[wl.honest].any()


def test_split_steps_equal_fused(oracle):
    """MulState::cor_share / cor / out_share / verify step by step == the fused batch."""
    from fuzzyheavyhitters_amd import sketch as S
    wl = S.sketch_workload(40, 13, seed=8, bad_fraction=0.25)
    sk = [oracle.sketch_fe(wl.seeds, wl.x[s], wl.kx[s]) for s in range(2)]
    cs = [oracle.mul_cor_share_fe(sk[s], wl.mac[s], wl.mac2[s], wl.triples[s]) for s in range(2)]
    cor = (cs[0] + cs[1]) % np.uint64(P)
    o = [oracle.mul_out_share_fe(s, sk[s], wl.mac[s], wl.mac2[s], wl.triples[s], cor) for s in range(2)]
    ok = ((o[0] + o[1]) % np.uint64(P)) == 0
    ok_f, outs = oracle.sketch_verify_fe(wl.seeds, wl.x[0], wl.kx[0], wl.x[1], wl.kx[1], np.stack(wl.mac),
                                         np.stack(wl.mac2), np.stack(wl.triples))
    assert np.array_equal(ok, ok_f) and np.array_equal(o[0], outs[0]) and np.array_equal(o[1], outs[1])


# ---- HIP path (through the C ABI) against the oracle -----------------------------------------
@pytest.fixture(params=[0, 1, 2, 3, 4], ids=["lds-sched", "r01-256", "otf-1024", "lds-sched-lpk8", "prod-cons"])
def sketch_impl(request):
    """every k_sketch_fe form (fhh_sketch_set_impl): round keys in LDS with the planned lanes per key
    (default: the planned tail launch in the producer / consumer form), r01's, on the fly, round keys
    in LDS at 8 lanes per key throughout, and the producer / consumer form for every key (AES waves and
    product waves paired through LDS, r03)"""
    from fuzzyheavyhitters_amd import lib
    assert lib().fhh_sketch_set_impl(request.param) == 0
    yield request.param
    lib().fhh_sketch_set_impl(0)


@pytest.mark.gpu
@pytest.mark.parametrize("n_keys,n_nodes", [(1, 0), (3, 1), (5, 2), (70, 63), (64, 64), (130, 125), (257, 300),
                                            (2000, 40), (1001, 256), (40000, 256), (300, 700)])
def test_gpu_sketch_at_bit_exact(oracle, n_keys, n_nodes, sketch_impl):
    """(300, 700): 352 keystream blocks per key, so some passes' blocks straddle block 256 and take
    the generic AES instead of the shared-rounds form (aes_ctr_shared needs the counters to differ in
    byte 15 alone)"""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import sketch as S
    wl = S.sketch_workload(n_keys, n_nodes, seed=n_keys * 7 + n_nodes, bad_fraction=0.1)
    kc = fhh.KeyCollection(8, 1)
    for s in range(2):
        got = S.sketch_at(kc, wl.seeds, wl.x[s], wl.kx[s])
        exp = oracle.sketch_fe(wl.seeds, wl.x[s], wl.kx[s])
        assert np.array_equal(got, exp), f"server {s}"


@pytest.mark.gpu
def test_gpu_mul_steps_bit_exact(oracle):
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import sketch as S
    wl = S.sketch_workload(500, 33, seed=21, bad_fraction=0.2)
    kc = fhh.KeyCollection(8, 1)
    sk = [S.sketch_at(kc, wl.seeds, wl.x[s], wl.kx[s]) for s in range(2)]
    cs = [S.mul_cor_share(kc, sk[s], wl.mac[s], wl.mac2[s], wl.triples[s]) for s in range(2)]
    for s in range(2):
        assert np.array_equal(cs[s], oracle.mul_cor_share_fe(sk[s], wl.mac[s], wl.mac2[s], wl.triples[s]))
    cor = S.mul_cor(cs[0], cs[1])
    o = [S.mul_out_share(kc, s, sk[s], wl.mac[s], wl.mac2[s], wl.triples[s], cor) for s in range(2)]
    for s in range(2):
        assert np.array_equal(o[s], oracle.mul_out_share_fe(s, sk[s], wl.mac[s], wl.mac2[s], wl.triples[s], cor))
    ok = S.mul_verify(o[0], o[1])
    assert np.array_equal(ok, wl.honest)


@pytest.mark.gpu
@pytest.mark.parametrize("force_sequential", [False, True], ids=["parallel", "sequential-stream"])
def test_gpu_sim_sketch_verify(oracle, force_sequential, sketch_impl):
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import sketch as S
    wl = S.sketch_workload(3000, 77, seed=99, bad_fraction=0.1)
    kc = fhh.KeyCollection(8, 1)
    b = S.DeviceSketchBatch(wl)
    S.sim_sketch_verify(kc, b, force_sequential=force_sequential)
    ok_exp, outs_exp = oracle.sketch_verify_fe(wl.seeds, wl.x[0], wl.kx[0], wl.x[1], wl.kx[1], np.stack(wl.mac),
                                               np.stack(wl.mac2), np.stack(wl.triples))
    assert np.array_equal(b.ok[0].cpu().numpy().astype(bool), ok_exp)        # [levels][n], one level
    assert np.array_equal(b.out_shares[0].cpu().numpy().view(np.uint64), outs_exp)
    assert np.array_equal(ok_exp, wl.honest)


@pytest.mark.gpu
def test_gpu_sim_sketch_verify_rejects_reused_triples():
    """A batch without per-level triples verifies one level only: MulState::new takes fresh
    triples per level (mpc.rs:94-98), and reusing one across openings leaks input differences.
    Both the Python mirror and the C ABI refuse n_levels > 1 there (nothing is written past the
    one-level ok / out_shares rows)."""
    import ctypes
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import sketch as S
    from fuzzyheavyhitters_amd._lib import FhhError, lib
    wl = S.sketch_workload(200, 9, seed=5, bad_fraction=0.1)
    kc = fhh.KeyCollection(8, 1)
    b = S.DeviceSketchBatch(wl)
    with pytest.raises(FhhError, match="n_levels"):
        S.sim_sketch_verify(kc, b, n_levels=3)
    st = b.struct(level=0, n_levels=3)
    assert lib().fhh_sim_sketch_verify_fe(kc.handle, ctypes.byref(st)) == -1   # FHH_E_ARG
    assert b"fresh triples" in lib().fhh_last_error(kc.handle)


# ---- U = FieldElm: the last level (sketch_at_last, sketch.rs:202-245; MulState<FieldElm>) ------
P255 = (1 << 255) - 19


def _py_stream255(seed: bytes):
    """FieldElm::from_rng = num-bigint 0.3.3 gen_biguint_below(p) on PrgStream (field.rs:367-372):
    each attempt takes the next 32 keystream bytes as 8 little-endian u32 digits, the top digit
    shifted right by 1 (255 bits); redraw while >= p. (num-bigint is not vendored: the digit order
    is the assumption DESIGN.md §5.2 records.)"""
    enc = _openssl_aes(seed)
    blk = 0
    while True:
        raw = enc(blk.to_bytes(16, "big")) + enc((blk + 1).to_bytes(16, "big"))
        blk += 2
        d = [int.from_bytes(raw[4 * k:4 * k + 4], "little") for k in range(8)]
        d[7] >>= 1
        v = sum(x << (32 * k) for k, x in enumerate(d))
        if v < P255:
            yield v


def _py_sketch255(seed: bytes, x, kx):
    st = _py_stream255(seed)
    r1, r2, r3 = next(st), next(st), next(st)
    rx = r2x = rkx = 0
    for xi, kxi in zip(x, kx):
        r = next(st)
        # lazy BigUint ops, one reduce at the end (field.rs:337-349)
        rx += xi * r
        r2x += xi * (r * r)
        rkx += kxi * r
    return [rx % P255, r2x % P255, rkx % P255, r1, r2, r3]


def _ints(a):
    from fuzzyheavyhitters_amd.sketch import fe8_to_int
    a = np.asarray(a)
    return [fe8_to_int(a[idx]) for idx in np.ndindex(a.shape[:-1])]


def test_fe255_oracle_arith_vs_python(oracle):
    rng = np.random.default_rng(17)
    vals = [0, 1, 2, 19, P255 - 1, P255 - 2, (1 << 254), (1 << 255) - 20, (1 << 128) + 7]
    vals += [int.from_bytes(rng.bytes(32), "little") % P255 for _ in range(40)]
    for a in vals:
        assert oracle.fe255_op("neg", a) == (-a) % P255
        for b in vals[::3]:
            assert oracle.fe255_op("mul", a, b) == a * b % P255
            assert oracle.fe255_op("add", a, b) == (a + b) % P255
            assert oracle.fe255_op("sub", a, b) == (a - b) % P255


def test_fe255_stream_matches_openssl_ctr(oracle):
    rng = np.random.default_rng(4)
    for _ in range(4):
        seed = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
        st = _py_stream255(seed)
        for m in range(5):
            assert oracle.fe255_stream_draw(seed, m) == next(st)   # no redraw at these odds (19 / 2^255)


def test_sketch_fe255_oracle_vs_python(oracle):
    from fuzzyheavyhitters_amd import sketch as S
    wl = S.sketch_workload255(10, 7, seed=12, bad_fraction=0.3)
    got = oracle.sketch_fe255(wl.seeds, wl.x[1], wl.kx[1])
    for i in range(10):
        exp = _py_sketch255(bytes(wl.seeds[i]), _ints(wl.x[1][i]), _ints(wl.kx[1][i]))
        assert _ints(got[i]) == exp


def test_beaver_identities_fe255(oracle):
    from fuzzyheavyhitters_amd import sketch as S
    wl = S.sketch_workload255(120, 11, seed=6, bad_fraction=0.25)
    args = (wl.seeds, wl.x[0], wl.kx[0], wl.x[1], wl.kx[1], np.stack(wl.mac), np.stack(wl.mac2), np.stack(wl.triples))
    ok, _ = oracle.sketch_verify_fe255(*args)
    assert ok[wl.honest].all() and not ok[~wl.honest].any()
    t = np.stack(wl.triples).copy()
    t[1, :, 2, 0] ^= 1                       # c of the first triple off by one on server 1
    ok2, _ = oracle.sketch_verify_fe255(*args[:7], t)
    assert not ok2.any()
    mac = np.stack(wl.mac).copy()
    mac[0, :, 0] ^= 4                        # a wrong MAC-key share
    ok3, _ = oracle.sketch_verify_fe255(*args[:5], mac, *args[6:])
    assert not ok3[wl.honest].any()


def test_split_steps_equal_fused_fe255(oracle):
    from fuzzyheavyhitters_amd import sketch as S
    wl = S.sketch_workload255(30, 9, seed=3, bad_fraction=0.3)
    sk = [oracle.sketch_fe255(wl.seeds, wl.x[s], wl.kx[s]) for s in range(2)]
    cs = [oracle.mul_cor_share_fe255(sk[s], wl.mac[s], wl.mac2[s], wl.triples[s]) for s in range(2)]
    cor = np.array([[S.int_to_fe8((a + b) % P255) for a, b in zip(_ints(cs[0][i]), _ints(cs[1][i]))]
                    for i in range(30)], np.uint32)
    o = [oracle.mul_out_share_fe255(s, sk[s], wl.mac[s], wl.mac2[s], wl.triples[s], cor) for s in range(2)]
    ok = np.array([(a + b) % P255 == 0 for a, b in zip(_ints(o[0]), _ints(o[1]))])
    ok_f, outs = oracle.sketch_verify_fe255(wl.seeds, wl.x[0], wl.kx[0], wl.x[1], wl.kx[1], np.stack(wl.mac),
                                            np.stack(wl.mac2), np.stack(wl.triples))
    assert np.array_equal(ok, ok_f) and np.array_equal(ok, wl.honest)
    assert np.array_equal(o[0], outs[0]) and np.array_equal(o[1], outs[1])


@pytest.mark.gpu
@pytest.mark.parametrize("n_keys,n_nodes", [(1, 0), (3, 1), (5, 2), (9, 13), (70, 63), (64, 64), (130, 125),
                                            (600, 40)])
def test_gpu_sketch_at_fe255_bit_exact(oracle, n_keys, n_nodes):
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import sketch as S
    wl = S.sketch_workload255(n_keys, n_nodes, seed=n_keys * 5 + n_nodes, bad_fraction=0.1)
    kc = fhh.KeyCollection(8, 1)
    for s in range(2):
        got = S.sketch_at_fe255(kc, wl.seeds, wl.x[s], wl.kx[s])
        exp = oracle.sketch_fe255(wl.seeds, wl.x[s], wl.kx[s])
        assert np.array_equal(got, exp), f"server {s}"


@pytest.mark.gpu
def test_gpu_mul_steps_fe255_bit_exact(oracle):
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import sketch as S
    wl = S.sketch_workload255(200, 17, seed=23, bad_fraction=0.2)
    kc = fhh.KeyCollection(8, 1)
    sk = [S.sketch_at_fe255(kc, wl.seeds, wl.x[s], wl.kx[s]) for s in range(2)]
    cs = [S.mul_cor_share_fe255(kc, sk[s], wl.mac[s], wl.mac2[s], wl.triples[s]) for s in range(2)]
    for s in range(2):
        assert np.array_equal(cs[s], oracle.mul_cor_share_fe255(sk[s], wl.mac[s], wl.mac2[s], wl.triples[s]))
    cor = S.mul_cor_fe255(cs[0], cs[1])
    o = [S.mul_out_share_fe255(kc, s, sk[s], wl.mac[s], wl.mac2[s], wl.triples[s], cor) for s in range(2)]
    for s in range(2):
        assert np.array_equal(o[s], oracle.mul_out_share_fe255(s, sk[s], wl.mac[s], wl.mac2[s], wl.triples[s], cor))
    assert np.array_equal(S.mul_verify_fe255(o[0], o[1]), wl.honest)


@pytest.mark.gpu
@pytest.mark.parametrize("force_sequential", [False, True], ids=["parallel", "sequential-stream"])
def test_gpu_sim_sketch_verify_fe255(oracle, force_sequential):
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import sketch as S
    wl = S.sketch_workload255(700, 45, seed=98, bad_fraction=0.1)
    kc = fhh.KeyCollection(8, 1)
    b = S.DeviceSketchBatch255(wl)
    S.sim_sketch_verify_fe255(kc, b, force_sequential=force_sequential)
    ok_exp, outs_exp = oracle.sketch_verify_fe255(wl.seeds, wl.x[0], wl.kx[0], wl.x[1], wl.kx[1], np.stack(wl.mac),
                                                  np.stack(wl.mac2), np.stack(wl.triples))
    assert np.array_equal(b.ok.cpu().numpy().astype(bool), ok_exp)
    assert np.array_equal(b.out_shares.cpu().numpy().view(np.uint32), outs_exp)
    assert np.array_equal(ok_exp, wl.honest)


@pytest.mark.gpu
def test_gpu_sketch_verify_level_batch(oracle):
    """Levels [2, 7) in one call (configs[4] runs data_len - 1 = 1023 such levels): level l uses
    the stream of seed ^ l (bytes 12..15) and the dealt triples[l] (TripleShare::new per level,
    MulState::new's triples[3 l ..], mpc.rs:94-98); every level's ok bits and out shares equal
    the oracle's for that level, and the dealt triples satisfy c0 + c1 = (a0 + a1)(b0 + b1)."""
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import sketch as S
    wl = S.sketch_workload(500, 19, seed=41, bad_fraction=0.1)
    kc = fhh.KeyCollection(8, 1)
    b = S.DeviceSketchBatch(wl)
    S.deal_triples(kc, b, levels=8, seed=77)
    S.sim_sketch_verify(kc, b, level=2, n_levels=5)
    tr = [t.cpu().numpy().view(np.uint64) for t in b.triples]           # [n][8][9]
    a = (tr[0][..., 0::3] + tr[1][..., 0::3]) % np.uint64(P)
    bb = (tr[0][..., 1::3] + tr[1][..., 1::3]) % np.uint64(P)
    c = (tr[0][..., 2::3] + tr[1][..., 2::3]) % np.uint64(P)
    for idx in [(0, 0, 0), (3, 5, 2), (499, 7, 1)]:
        assert int(a[idx]) * int(bb[idx]) % P == int(c[idx])
    ok = b.ok.cpu().numpy()
    outs = b.out_shares.cpu().numpy().view(np.uint64)
    for k, lv in enumerate(range(2, 7)):
        seeds = wl.seeds.copy()
        seeds[:, 12:16] ^= np.frombuffer(np.uint32(lv).tobytes(), np.uint8)
        ok_e, outs_e = oracle.sketch_verify_fe(seeds, wl.x[0], wl.kx[0], wl.x[1], wl.kx[1], np.stack(wl.mac),
                                               np.stack(wl.mac2), np.stack([tr[0][:, lv], tr[1][:, lv]]))
        assert np.array_equal(ok[k].astype(bool), ok_e), f"level {lv}"
        assert np.array_equal(outs[k], outs_e), f"level {lv}"
        assert np.array_equal(ok_e, wl.honest)
