"""Pin the oracle (CPU restatement) before trusting it: FIPS-197 / OpenSSL AES, the MMO
PRG known answers, fastfield.rs's own known answers, and the ibDCF comparison semantics."""
import ctypes
import ctypes.util
import os

import numpy as np
import pytest


def test_fips197_c1(oracle):
    key = bytes(range(16))
    pt = bytes.fromhex("00112233445566778899aabbccddeeff")
    assert oracle.aes128_encrypt(key, pt).hex() == "69c4e0d86a7b0430d8cdb78070b4c55a"


def test_zero_key_kat(oracle):
    assert oracle.aes0(bytes(16)).hex() == "66e94bd4ef8a2c3b884cfa59ca342b2e"


def _openssl():
    path = ctypes.util.find_library("crypto")
    if not path:
        pytest.skip("libcrypto not present")
    L = ctypes.CDLL(path)
    return L


def test_against_openssl(oracle):
    L = _openssl()
    key = (ctypes.c_uint8 * 16)()
    ks = ctypes.create_string_buffer(512)   # AES_KEY
    assert L.AES_set_encrypt_key(key, 128, ks) == 0
    rng = np.random.default_rng(1)
    for _ in range(200):
        blk = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
        out = ctypes.create_string_buffer(16)
        L.AES_encrypt(blk, out, ks)
        assert oracle.aes0(blk) == out.raw
        if oracle.aes_ni_available():
            assert oracle.aes0(blk, ni=True) == out.raw


def test_chacha20_rfc8439_vector(oracle):
    """The OT row PRG's block function (r06, fhh_oracle.c orc_chacha_block) at 20 rounds: RFC 8439
    2.3.2's test vector (key 00..1f, nonce 00:00:00:09:00:00:00:4a:00:00:00:00, block counter 1) — in the
    64-bit-counter layout: counter word 13 = nonce bytes 0-3, nonce words 14-15 = nonce bytes 4-11."""
    key = bytes(range(32))
    nonce = bytes.fromhex("000000090000004a00000000")
    ctr = 1 | (int.from_bytes(nonce[:4], "little") << 32)
    out = oracle.chacha_block(20, key, ctr, int.from_bytes(nonce[4:], "little"))
    assert out.hex() == ("10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
                         "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")


def test_chacha20_against_openssl(oracle):
    """orc_chacha_block(20, ...) = OpenSSL's EVP_chacha20 keystream (IV = 32-bit counter LE || 96-bit
    nonce) for random keys, counters past 2^32 and the key = seed || seed form the OT rows use."""
    L = _openssl()
    L.EVP_chacha20.restype = ctypes.c_void_p
    L.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p

    def ossl(key, iv):
        ctx = ctypes.c_void_p(L.EVP_CIPHER_CTX_new())
        assert L.EVP_EncryptInit_ex(ctx, ctypes.c_void_p(L.EVP_chacha20()), None, key, iv) == 1
        out, ol = ctypes.create_string_buffer(64), ctypes.c_int()
        assert L.EVP_EncryptUpdate(ctx, out, ctypes.byref(ol), bytes(64), 64) == 1
        L.EVP_CIPHER_CTX_free(ctx)
        return out.raw[:ol.value]

    rng = np.random.default_rng(8439)
    for k in range(64):
        seed = rng.integers(0, 256, 16, dtype=np.uint8).tobytes()
        key = seed + seed if k % 2 else rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        ctr = int(rng.integers(0, 1 << 63)) if k % 3 else k
        iv = (ctr & 0xFFFFFFFF).to_bytes(4, "little") + (ctr >> 32).to_bytes(4, "little") + bytes(8)
        assert oracle.chacha_block(20, key, ctr, 0) == ossl(key, iv)


def test_mmo_prg_kat(oracle):
    # expand of the zero seed; right block uses ctr + 1 in the upper u64 lane
    left, b = oracle.expand_dir(bytes(16), 0)
    right, _ = oracle.expand_dir(bytes(16), 1)
    assert left.hex() == "66e94bd4ef8a2c3b884cfa59ca342b2e"
    assert right.hex() == "0c546f62bf2773cd0e564fceca7ba688"
    assert b == (1, 1, 1, 1)   # control bits read after the nibble mask (prg.rs:96-105)


def test_prg_nibble_mask_and_counter(oracle):
    rng = np.random.default_rng(2)
    for _ in range(100):
        s = bytearray(rng.integers(0, 256, 16, dtype=np.uint8).tobytes())
        k = bytearray(s)
        k[0] &= 0xF0
        left, bits = oracle.expand_dir(bytes(s), 0)
        assert bits == (1, 1, 1, 1)
        assert left == bytes(a ^ b for a, b in zip(oracle.aes0(bytes(k)), k))
        hi = (int.from_bytes(k[8:], "little") + 1) % (1 << 64)
        k2 = k[:8] + hi.to_bytes(8, "little")
        right, _ = oracle.expand_dir(bytes(s), 1)
        assert right == bytes(a ^ b for a, b in zip(oracle.aes0(bytes(k2)), k2))
    # upper-lane wrap does not carry into bytes 0..7
    s = bytes([0x12] + [0xFF] * 15)
    right, _ = oracle.expand_dir(s, 1)
    k2 = bytes([0x10] + [0xFF] * 7 + [0] * 8)
    assert right == bytes(a ^ b for a, b in zip(oracle.aes0(k2), k2))


def test_fastfield_known_answers(oracle):
    """fastfield.rs:459-559 (the reference's own values)."""
    P = oracle.FE_P
    L = oracle.lib()
    fv = lambda x: int(L.orc_fe_value(x))
    new = lambda x: int(L.orc_fe_new(x & (2 ** 64 - 1)))
    assert fv(new(0)) == 0 and fv(new(1337)) == 1337 and fv(new(P)) == 0 and fv(new(P + 1)) == 1
    assert fv(new(P - 1)) == P - 1 and fv(new(P * 2)) == 0
    assert fv(new(2 ** 64 - 1)) == (2 ** 64 - 1) % P
    FE_VAL_MAX = (2 ** 62 - 1) + (3 << 30) + 3
    assert fv(FE_VAL_MAX) == FE_VAL_MAX - P
    sub = lambda a, b: fv(int(L.orc_fe_sub(new(a), new(b))))
    assert sub(0, 100) == P - 100 and sub(100, 105) == P - 5 and sub(300, P + 1) == 299
    mul = lambda a, b: fv(int(L.orc_fe_mul(new(a), new(b))))
    assert mul(999, 1000) == 999000 and mul(P - 1, P - 1) == 1 and mul(P - 2, P - 2) == 4
    # recip(999) == 2885188949795824624 (fastfield.rs:528)
    assert pow(999, P - 2, P) == 2885188949795824624
    assert mul(999, 2885188949795824624) == 1


def test_fe_fold_sum_value(oracle):
    rng = np.random.default_rng(3)
    v = rng.integers(0, 2 ** 63, 5000, dtype=np.uint64) * 2 + 1
    got = oracle.fe_value(oracle.fe_fold_sum(v))
    assert got == sum(int(x) for x in v) % oracle.FE_P


@pytest.mark.parametrize("nbits", [4, 5])
def test_ibdcf_semantics_exhaustive(oracle, nbits):
    """After an MSB-first prefix x[1..k]: E = y0^t0^y1^t1 = [x < a] (left key, side=true)
    and [x > a] (right key, side=false) — derived from ibDCF.rs:84-119,208-227.
    Note: the reference's own test `ibdcf_complete` (tests/ibdcf_tests.rs:4-39) asserts 1 at
    x == a for side=false, which contradicts this algebra."""
    rng = np.random.default_rng(nbits)
    bad = 0
    for a in range(1 << nbits):
        for side in (0, 1):
            al = oracle.msb_u32_to_bits(nbits, a)
            r0 = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
            r1 = bytes(rng.integers(0, 256, 16, dtype=np.uint8))
            cs, cb = oracle.gen_ibdcf(al, side, r0, r1)
            for x in range(1 << nbits):
                xb = oracle.msb_u32_to_bits(nbits, x)
                for k in range(1, nbits + 1):
                    e = oracle.eval_ibdcf(0, r0, cs, cb, xb[:k]) ^ oracle.eval_ibdcf(1, r1, cs, cb, xb[:k])
                    ap, xp = a >> (nbits - k), x >> (nbits - k)
                    bad += e != ((xp < ap) if side else (xp > ap))
    assert bad == 0


def test_bitstring_utils(oracle):
    o = oracle
    assert o.u32_to_bits(5, 21) == [True, False, True, False, True]
    # lib.rs:56-76: u32_to_bits is LSB first, MSB_u32_to_bits MSB first (6 = 0b00110)
    assert o.u32_to_bits(5, 6) == [False, True, True, False, False]
    assert o.msb_u32_to_bits(5, 6) == [False, False, True, True, False]
    assert o.bits_to_u32(o.msb_u32_to_bits(7, 77)) == 77
    assert o.add_bitstrings([True, True], [True]) == [True, False, False]
    assert o.subtract_bitstrings([False, False], [False, True]) == [True, True]
    assert o.all_bit_vectors(2) == [[False, False], [True, False], [False, True], [True, True]]
    assert o.i16_to_bitvec(-1) == [True] * 16
    assert o.string_to_bits(b"A") == o.u32_to_bits(8, 65)
