// Compile-time AES-128 tables for the fixed all-zero key used by the reference PRG
// (src/prg.rs:185-197 `FixedKeyPrgStream::new` keys AES with 16 zero bytes).
//
// Everything here is constexpr: the S-box is derived from GF(2^8) log/antilog tables,
// T0 is the combined SubBytes+MixColumns table, and the zero key's round keys are
// expanded at compile time so they appear as immediates in the device code.
#pragma once
#include <stdint.h>

namespace fhh {

constexpr uint8_t xtime(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

struct ByteTable { uint8_t v[256]; };
struct WordTable { uint32_t v[256]; };
struct RoundKeys { uint32_t w[11][4]; };   // little-endian column words, round 0..10

constexpr ByteTable make_sbox() {
    // antilog (generator 3) / log tables, then S(x) = affine(x^-1), FIPS-197 5.1.1
    uint8_t exp[256] = {};
    uint8_t log[256] = {};
    uint8_t x = 1;
    for (int i = 0; i < 255; i++) {
        exp[i] = x;
        log[x] = (uint8_t)i;
        x = (uint8_t)(x ^ xtime(x));    // multiply by 3
    }
    ByteTable s = {};
    for (int i = 0; i < 256; i++) {
        uint8_t inv = i ? exp[(255 - log[i]) % 255] : 0;
        uint8_t r = inv;
        for (int k = 1; k < 5; k++) r ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
        s.v[i] = (uint8_t)(r ^ 0x63);
    }
    return s;
}

constexpr ByteTable SBOX = make_sbox();

// T0[x] = (2*S[x]) | S[x] << 8 | S[x] << 16 | (3*S[x]) << 24 (little-endian column).
// T_k = rotl(T0, 8k); S[x] is byte 1 (and byte 2) of T0[x].
constexpr WordTable make_t0() {
    WordTable t = {};
    for (int i = 0; i < 256; i++) {
        uint8_t s = SBOX.v[i];
        uint8_t s2 = xtime(s);
        uint8_t s3 = (uint8_t)(s2 ^ s);
        t.v[i] = (uint32_t)s2 | ((uint32_t)s << 8) | ((uint32_t)s << 16) | ((uint32_t)s3 << 24);
    }
    return t;
}

constexpr WordTable T0 = make_t0();

constexpr RoundKeys make_zero_key_schedule() {
    uint8_t rk[176] = {};
    uint8_t rcon = 1;
    for (int i = 4; i < 44; i++) {
        uint8_t t0 = rk[4 * (i - 1) + 0], t1 = rk[4 * (i - 1) + 1], t2 = rk[4 * (i - 1) + 2],
                t3 = rk[4 * (i - 1) + 3];
        if (i % 4 == 0) {
            uint8_t u = t0;
            t0 = (uint8_t)(SBOX.v[t1] ^ rcon);
            t1 = SBOX.v[t2];
            t2 = SBOX.v[t3];
            t3 = SBOX.v[u];
            rcon = xtime(rcon);
        }
        rk[4 * i + 0] = rk[4 * (i - 4) + 0] ^ t0;
        rk[4 * i + 1] = rk[4 * (i - 4) + 1] ^ t1;
        rk[4 * i + 2] = rk[4 * (i - 4) + 2] ^ t2;
        rk[4 * i + 3] = rk[4 * (i - 4) + 3] ^ t3;
    }
    RoundKeys r = {};
    for (int round = 0; round < 11; round++)
        for (int c = 0; c < 4; c++) {
            const uint8_t* p = rk + 16 * round + 4 * c;
            r.w[round][c] = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
        }
    return r;
}

constexpr RoundKeys ZERO_RK = make_zero_key_schedule();

static_assert(SBOX.v[0] == 0x63 && SBOX.v[1] == 0x7c && SBOX.v[0x53] == 0xed, "S-box");
static_assert(ZERO_RK.w[1][0] == 0x63636362u, "zero-key schedule round 1");
static_assert(ZERO_RK.w[10][0] == 0xcb5befb4u, "zero-key schedule round 10");

}  // namespace fhh
