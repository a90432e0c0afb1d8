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
@pytest.mark.gpu
@pytest.mark.parametrize("n_keys,n_nodes", [(1, 0), (3, 1), (5, 2), (70, 63), (64, 64), (130, 125), (257, 300),
                                            (2000, 40)])
def test_gpu_sketch_at_bit_exact(oracle, n_keys, n_nodes):
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
def test_gpu_sim_sketch_verify(oracle, force_sequential):
    import fuzzyheavyhitters_amd as fhh
    from fuzzyheavyhitters_amd import sketch as S
    wl = S.sketch_workload(3000, 77, seed=99, bad_fraction=0.1)
    kc = fhh.KeyCollection(8, 1)
    b = S.DeviceSketchBatch(wl)
    S.sim_sketch_verify(kc, b, force_sequential=force_sequential)
    ok_exp, outs_exp = oracle.sketch_verify_fe(wl.seeds, wl.x[0], wl.kx[0], wl.x[1], wl.kx[1], np.stack(wl.mac),
                                               np.stack(wl.mac2), np.stack(wl.triples))
    assert np.array_equal(b.ok.cpu().numpy().astype(bool), ok_exp)
    assert np.array_equal(b.out_shares.cpu().numpy().view(np.uint64), outs_exp)
    assert np.array_equal(ok_exp, wl.honest)
