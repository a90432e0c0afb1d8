// Host-side self-test of the device AES T-table round structure (csrc/aes_ttable.h):
// instantiates fhh::aes0_mmo with emulated v_perm_b32 / LDS-load ops and checks it against
// a byte-oriented FIPS-197 reference computed here, for every replica lane. Catches
// layout/selector mistakes without a GPU. Built with hipcc (host code only) by
// tests/test_host_aes.py; prints "OK" on success.
#include "../../fuzzyheavyhitters_amd/csrc/expand_kernel.h"
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
        if (byte_addr & 3 || byte_addr >= 4u * 2 * 256 * 64) { std::fprintf(stderr, "bad addr\n"); std::abort(); }
        return tbl[byte_addr / 4];
    }
    static uint32_t bfe(uint32_t x, uint32_t off, uint32_t w) { return (x >> off) & ((1u << w) - 1u); }
    static uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return a ^ b ^ c; }
    static bool any(bool p) { return p; }
};

// as HostOps, but every wave-uniform "any" of aes0_mmo_pair answers (no full redo, byte-9
// fix-up taken): on the device the fix-up runs for all lanes of a wave, carry or not
struct HostOpsMedium : HostOps {
    static bool any(bool) {
        static unsigned calls = 0;
        return (calls++ & 1u) == 1u;
    }
};

template <class Tab>
static int check_pair_medium(std::mt19937_64& rng) {
    static uint32_t tbl[2 * 256 * 64];
    for (int i = 0; i < Tab::kWords; i++) tbl[i] = Tab::word(fhh::T0.v, i);
    int fails = 0;
    for (int it = 0; it < 4096; it++) {
        uint32_t b0, b1;
        Tab::bases(it % 64, b0, b1);
        uint32_t seed[2][4];
        for (int q = 0; q < 2; q++)
            for (int c = 0; c < 4; c++) seed[q][c] = (uint32_t)rng();
        if (it & 1) seed[it & 2 ? 1 : 0][2] |= 0xFFu;   // carry into byte 9 (byte 9 random)
        for (int q = 0; q < 2; q++)
            if ((seed[q][2] & 0xFFFFu) == 0xFFFFu) seed[q][2] ^= 0x100u;   // no carry past byte 9
        uint32_t s1[4][4], s2[4][4];
        for (int q = 0; q < 2; q++)
            for (int dir = 0; dir < 2; dir++) {
                fhh::prg_ctr(seed[q], dir, s1[2 * q + dir]);
                fhh::prg_ctr(seed[q], dir, s2[2 * q + dir]);
            }
        fhh::aes0_mmo_tab<HostOps, Tab, 4>(s1, tbl, b0, b1);
        fhh::aes0_mmo_pair<HostOpsMedium, Tab, 4>(s2, tbl, b0, b1);
        if (std::memcmp(s1, s2, sizeof s1)) fails++;
    }
    if (fails) std::printf("pair (byte-9 fix-up for every lane) %s: %d failures\n", Tab::kName, fails);
    return fails;
}

// aes0_mmo_pair (sibling counters k, k + 2^64 sharing rounds 1-2) == aes0_mmo_tab, including
// the carry fallback (byte 8 = 0xFF, with longer carry chains into bytes 9..15 and the wrap)
template <class Tab>
static int check_pair(std::mt19937_64& rng) {
    static uint32_t tbl[2 * 256 * 64];
    for (int i = 0; i < Tab::kWords; i++) tbl[i] = Tab::word(fhh::T0.v, i);
    int fails = 0;
    for (int it = 0; it < 4096; it++) {
        const uint32_t lane = it % 64;
        uint32_t b0, b1;
        Tab::bases(lane, b0, b1);
        uint32_t seed[2][4];
        for (int q = 0; q < 2; q++)
            for (int c = 0; c < 4; c++) seed[q][c] = (uint32_t)rng();
        const int mode = it % 8;   // 0..3 random, 4: byte 8 = FF, 5: bytes 8..11 FF, 6: all upper FF, 7: 8..12 FF
        if (mode == 4) seed[it & 1][2] |= 0xFFu;
        if (mode == 5) seed[it & 1][2] = 0xFFFFFFFFu;
        if (mode == 6) { seed[0][2] = seed[0][3] = 0xFFFFFFFFu; }
        if (mode == 7) { seed[1][2] = 0xFFFFFFFFu; seed[1][3] |= 0xFFu; }
        uint32_t s1[4][4], s2[4][4];
        for (int q = 0; q < 2; q++)
            for (int dir = 0; dir < 2; dir++) {
                fhh::prg_ctr(seed[q], dir, s1[2 * q + dir]);
                fhh::prg_ctr(seed[q], dir, s2[2 * q + dir]);
            }
        fhh::aes0_mmo_tab<HostOps, Tab, 4>(s1, tbl, b0, b1);
        fhh::aes0_mmo_pair<HostOps, Tab, 4>(s2, tbl, b0, b1);
        if (std::memcmp(s1, s2, sizeof s1)) fails++;
    }
    if (fails) std::printf("pair %s: %d failures\n", Tab::kName, fails);
    return fails;
}

// every LDS layout of expand_kernel.h: same outputs as the byte-oriented reference, every lane,
// and lanes that share a ds_read_b32 lane group (32 lanes) hit distinct banks
template <class Tab>
static int check_layout(std::mt19937_64& rng, void (*ref)(const uint8_t*, uint8_t*)) {
    static uint32_t tbl[2 * 256 * 64];
    for (int i = 0; i < Tab::kWords; i++) tbl[i] = Tab::word(fhh::T0.v, i);
    int fails = 0;
    for (int it = 0; it < 512; it++) {
        const uint32_t lane = it % 64;
        uint32_t b0, b1;
        Tab::bases(lane, b0, b1);
        uint32_t s[2][4];
        uint8_t in[2][16];
        for (int b = 0; b < 2; b++) {
            for (int c = 0; c < 4; c++) s[b][c] = (uint32_t)rng();
            std::memcpy(in[b], s[b], 16);
        }
        fhh::aes0_mmo_tab<HostOps, Tab, 2>(s, tbl, b0, b1);
        for (int b = 0; b < 2; b++) {
            uint8_t e[16];
            ref(in[b], e);
            for (int i = 0; i < 16; i++) e[i] ^= in[b][i];
            if (std::memcmp(e, s[b], 16)) fails++;
        }
    }
    // bank check: for a fixed looked-up word, the 32 lanes of a group use 32 distinct banks
    for (int k = 0; k < 4; k++) {
        for (int trial = 0; trial < 64; trial++) {
            const uint32_t x = (uint32_t)rng();
            bool used[32] = {false};
            for (uint32_t lane = 0; lane < 32; lane++) {
                uint32_t b0, b1;
                Tab::bases(lane, b0, b1);
                // address of term<k>: recompute via a table whose words encode their own address
                (void)b1;
                uint32_t addr = 0;
                static uint32_t ident[2 * 256 * 64];
                static bool init = false;
                if (!init) { for (int i = 0; i < 2 * 256 * 64; i++) ident[i] = (uint32_t)i * 4; init = true; }
                if (k == 0) addr = Tab::template last<0>(ident, b0, b1, x);
                if (k == 1) addr = Tab::template last<1>(ident, b0, b1, x);
                if (k == 2) addr = Tab::template last<2>(ident, b0, b1, x);
                if (k == 3) addr = Tab::template last<3>(ident, b0, b1, x);
                const uint32_t bank = (addr / 4) % 32;
                if (used[bank]) fails++;
                used[bank] = true;
            }
        }
    }
    if (fails) std::printf("layout %s: %d failures\n", Tab::kName, fails);
    return fails;
}

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
    fails += check_layout<fhh::TabT0R64<HostOps>>(rng, ref_aes0);
    fails += check_layout<fhh::Tab4T32<HostOps>>(rng, ref_aes0);
    fails += check_layout<fhh::TabT0R32<HostOps>>(rng, ref_aes0);
    fails += check_layout<fhh::TabT01R32<HostOps>>(rng, ref_aes0);
    fails += check_pair<fhh::Tab4T32<HostOps>>(rng);
    fails += check_pair<fhh::TabT0R64<HostOps>>(rng);
    fails += check_pair_medium<fhh::Tab4T32<HostOps>>(rng);
    if (fails) { std::printf("FAIL %d\n", fails); return 1; }
    std::printf("OK\n");
    return 0;
}
