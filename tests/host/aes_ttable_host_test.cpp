// Host-side self-test of the device AES T-table round structure (csrc/aes_ttable.h):
// instantiates fhh::aes0_mmo with emulated v_perm_b32 / LDS-load ops and checks it against
// a byte-oriented FIPS-197 reference computed here, for every replica lane. Catches
// layout/selector mistakes without a GPU. Built with hipcc (host code only) by
// tests/test_host_aes.py; prints "OK" on success.
#include "../../fuzzyheavyhitters_amd/csrc/aes_ttable.h"
#include <cstdio>
#include <cstring>
#include <random>

struct HostOps {
    static uint32_t perm(uint32_t a, uint32_t b, uint32_t sel) {
        uint64_t v = ((uint64_t)a << 32) | b;
        uint32_t out = 0;
        for (int i = 0; i < 4; i++) {
            uint32_t s = (sel >> (8 * i)) & 0xFF;
            uint32_t byte;
            if (s < 8) byte = (uint32_t)(v >> (8 * s)) & 0xFF;
            else if (s == 12) byte = 0;
            else if (s >= 13) byte = 0xFF;
            else { std::fprintf(stderr, "unemulated selector %u\n", s); std::abort(); }
            out |= byte << (8 * i);
        }
        return out;
    }
    static uint32_t load(const uint32_t* tbl, uint32_t byte_addr) {
        if (byte_addr & 3 || byte_addr >= 4u * fhh::kTableWords) { std::fprintf(stderr, "bad addr\n"); std::abort(); }
        return tbl[byte_addr / 4];
    }
};

static uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1b : 0)); }

static void ref_aes0(const uint8_t in[16], uint8_t out[16]) {
    uint8_t rk[176];
    for (int r = 0; r < 11; r++)
        for (int c = 0; c < 4; c++)
            for (int k = 0; k < 4; k++) rk[16 * r + 4 * c + k] = (fhh::ZERO_RK.w[r][c] >> (8 * k)) & 0xFF;
    uint8_t s[16];
    for (int i = 0; i < 16; i++) s[i] = in[i] ^ rk[i];
    for (int round = 1; round <= 10; round++) {
        uint8_t t[16];
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 4; r++) t[4 * c + r] = fhh::SBOX.v[s[4 * ((c + r) & 3) + r]];
        if (round < 10) {
            for (int c = 0; c < 4; c++) {
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                s[4 * c + 0] = xt(a0) ^ (xt(a1) ^ a1) ^ a2 ^ a3;
                s[4 * c + 1] = a0 ^ xt(a1) ^ (xt(a2) ^ a2) ^ a3;
                s[4 * c + 2] = a0 ^ a1 ^ xt(a2) ^ (xt(a3) ^ a3);
                s[4 * c + 3] = (xt(a0) ^ a0) ^ a1 ^ a2 ^ xt(a3);
            }
        } else {
            std::memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; i++) s[i] ^= rk[16 * round + i];
    }
    std::memcpy(out, s, 16);
}

int main() {
    static uint32_t tbl[fhh::kTableWords];
    for (int i = 0; i < fhh::kTableWords; i++) tbl[i] = fhh::T0.v[i / fhh::kTableReplicas];
    // FIPS-197 zero-key KAT
    {
        uint8_t z[16] = {0}, o[16];
        ref_aes0(z, o);
        const uint8_t kat[16] = {0x66, 0xe9, 0x4b, 0xd4, 0xef, 0x8a, 0x2c, 0x3b,
                                 0x88, 0x4c, 0xfa, 0x59, 0xca, 0x34, 0x2b, 0x2e};
        if (std::memcmp(o, kat, 16)) { std::printf("FAIL ref KAT\n"); return 1; }
    }
    std::mt19937_64 rng(12345);
    int fails = 0;
    for (int it = 0; it < 2000; it++) {
        uint32_t lane = it % 64;
        uint32_t s[2][4];
        uint8_t in[2][16];
        for (int b = 0; b < 2; b++) {
            for (int c = 0; c < 4; c++) s[b][c] = (uint32_t)rng();
            std::memcpy(in[b], s[b], 16);
        }
        fhh::aes0_mmo<HostOps, 2>(s, tbl, lane * 4);
        for (int b = 0; b < 2; b++) {
            uint8_t e[16];
            ref_aes0(in[b], e);
            for (int i = 0; i < 16; i++) e[i] ^= in[b][i];
            if (std::memcmp(e, s[b], 16)) fails++;
        }
    }
    // prg counter: dir 1 increments the upper u64 lane with wrap, no carry into low half
    {
        uint32_t seed[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu}, c[4];
        fhh::prg_ctr(seed, 1, c);
        if (!(c[0] == 0xFFFFFFF0u && c[1] == 0xFFFFFFFFu && c[2] == 0 && c[3] == 0)) fails++;
        uint32_t seed2[4] = {0x12345678u, 0, 0xFFFFFFFFu, 7}, c2[4];
        fhh::prg_ctr(seed2, 1, c2);
        if (!(c2[0] == 0x12345670u && c2[2] == 0 && c2[3] == 8)) fails++;
        uint32_t bit, ybit;
        fhh::prg_ctrl_bits(c2[0], 0, bit, ybit);
        if (bit != 1 || ybit != 1) fails++;
        fhh::prg_ctrl_bits(c2[0], 1, bit, ybit);
        if (bit != 1 || ybit != 1) fails++;
    }
    if (fails) { std::printf("FAIL %d\n", fails); return 1; }
    std::printf("OK\n");
    return 0;
}
