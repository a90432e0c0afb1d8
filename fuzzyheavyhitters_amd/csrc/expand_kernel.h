// k_expand — the hot path: ibDCFKey::eval_bit (ibDCF.rs:208-227) for every
// (dim-prefix entry, client, side, direction), with the PRG expand_dir (prg.rs:92-122) as an
// LDS T-table AES-128 and the MMO feed-forward.
//
// The kernel is a template over
//   Tab   — the LDS T-table layout (how a byte of state becomes a conflict-free ds_read_b32),
//   NB    — AES blocks per lane kept in flight (4: both sides x both dirs; 2: one side),
//   THR   — workgroup size,
// plus a runtime choice of static (grid-stride) or dynamic (atomic work counter) item
// distribution. fhh_kernels.hip instantiates the variants; fhh_set_variant selects one.
//
// Every Tab is generic over Ops (perm/load/bfe) so tests/host/aes_ttable_host_test.cpp can
// instantiate the exact same lookup code on the CPU with emulated v_perm_b32.
#pragma once
#include "aes_ttable.h"
#include "fhh_internal.h"

namespace fhh {

template <int k> __host__ __device__ __forceinline__ uint32_t rotk(uint32_t v) {
    if constexpr (k == 0) return v;
    else return rotl32(v, 8 * k);
}

// ---- layouts ----------------------------------------------------------------------------
// A: T0 only, one replica per lane (64), entry stride 256 B (64 KiB). addr = 1 v_perm.
template <class Ops> struct TabT0R64 {
    static constexpr int kWords = 256 * 64;
    static constexpr const char* kName = "T0/64rep/64KiB";
    __host__ __device__ static uint32_t word(const uint32_t* t0, int i) { return t0[i >> 6]; }
    __host__ __device__ static void bases(uint32_t lane, uint32_t& b0, uint32_t& b1) { b0 = lane * 4; b1 = 0; }
    template <int k>
    __host__ __device__ static uint32_t term(const uint32_t* t, uint32_t b0, uint32_t, uint32_t x) {
        return rotk<k>(Ops::load(t, Ops::perm(b0, x, lookup_sel(k))));
    }
    template <int k>
    __host__ __device__ static uint32_t last(const uint32_t* t, uint32_t b0, uint32_t, uint32_t x) {
        return Ops::load(t, Ops::perm(b0, x, lookup_sel(k)));
    }
    static constexpr int spos(int) { return 1; }
};

// B: four tables T0..T3, 32 replicas each (lanes l and l+32 share a replica: they are in
// different ds_read_b32 lane groups), 128 KiB. Region m (64 KiB) holds T_{2m} in bytes
// [0,128) and T_{2m+1} in [128,256) of each 256-B entry row. No rotations.
template <class Ops> struct Tab4T32 {
    static constexpr int kWords = 2 * 256 * 64;
    static constexpr const char* kName = "T0..T3/32rep/128KiB";
    __host__ __device__ static uint32_t word(const uint32_t* t0, int i) {
        const int region = i >> 14, within = i & 16383, x = within >> 6, slot = within & 63;
        const int tab = 2 * region + (slot >= 32 ? 1 : 0);
        const uint32_t v = t0[x];
        return tab == 0 ? v : rotl32(v, 8 * tab);
    }
    __host__ __device__ static void bases(uint32_t lane, uint32_t& b0, uint32_t& b1) {
        b0 = (lane & 31) * 4;
        b1 = b0 | (1u << 16);
    }
    template <int tab>
    __host__ __device__ static uint32_t look(const uint32_t* t, uint32_t b0, uint32_t b1, uint32_t x, int k) {
        // {lb.byte0, x.byte[k], lb.byte2, 0}
        const uint32_t sel = 0x0C060004u | ((uint32_t)k << 8);
        const uint32_t a = Ops::perm((tab >> 1) ? b1 : b0, x, sel) + 128u * (tab & 1);
        return Ops::load(t, a);
    }
    template <int k>
    __host__ __device__ static uint32_t term(const uint32_t* t, uint32_t b0, uint32_t b1, uint32_t x) {
        return look<k>(t, b0, b1, x, k);
    }
    // final round: take S[x] at byte k from T_{(k+3)&3}
    template <int k>
    __host__ __device__ static uint32_t last(const uint32_t* t, uint32_t b0, uint32_t b1, uint32_t x) {
        return look<(k + 3) & 3>(t, b0, b1, x, k);
    }
    static constexpr int spos(int k) { return k; }
};

// C: T0 only, 32 replicas, entry stride 128 B (32 KiB). addr = bfe + lshl_or (2 VALU).
template <class Ops> struct TabT0R32 {
    static constexpr int kWords = 256 * 32;
    static constexpr const char* kName = "T0/32rep/32KiB";
    __host__ __device__ static uint32_t word(const uint32_t* t0, int i) { return t0[i >> 5]; }
    __host__ __device__ static void bases(uint32_t lane, uint32_t& b0, uint32_t& b1) { b0 = (lane & 31) * 4; b1 = 0; }
    template <int k>
    __host__ __device__ static uint32_t addr(uint32_t b0, uint32_t x) {
        return (Ops::bfe(x, 8 * k, 8) << 7) | b0;
    }
    template <int k>
    __host__ __device__ static uint32_t term(const uint32_t* t, uint32_t b0, uint32_t, uint32_t x) {
        return rotk<k>(Ops::load(t, addr<k>(b0, x)));
    }
    template <int k>
    __host__ __device__ static uint32_t last(const uint32_t* t, uint32_t b0, uint32_t, uint32_t x) {
        return Ops::load(t, addr<k>(b0, x));
    }
    static constexpr int spos(int) { return 1; }
};

// D: T0 and T1 interleaved (32 replicas each, 64 KiB); T2 = rotl16(T0), T3 = rotl16(T1).
template <class Ops> struct TabT01R32 {
    static constexpr int kWords = 256 * 64;
    static constexpr const char* kName = "T0,T1/32rep/64KiB";
    __host__ __device__ static uint32_t word(const uint32_t* t0, int i) {
        const uint32_t v = t0[i >> 6];
        return (i & 63) >= 32 ? rotl32(v, 8) : v;
    }
    __host__ __device__ static void bases(uint32_t lane, uint32_t& b0, uint32_t& b1) { b0 = (lane & 31) * 4; b1 = 0; }
    template <int k>
    __host__ __device__ static uint32_t term(const uint32_t* t, uint32_t b0, uint32_t, uint32_t x) {
        const uint32_t v = Ops::load(t, Ops::perm(b0, x, lookup_sel(k)) + 128u * (k & 1));
        return (k >= 2) ? rotl32(v, 16) : v;
    }
    template <int k>
    __host__ __device__ static uint32_t last(const uint32_t* t, uint32_t b0, uint32_t, uint32_t x) {
        return Ops::load(t, Ops::perm(b0, x, lookup_sel(k)));
    }
    static constexpr int spos(int) { return 1; }
};

// ---- AES-128 (zero key) + MMO over a table layout ----------------------------------------
template <class Ops, class Tab, int NB>
__host__ __device__ __forceinline__ void aes0_mmo_tab(uint32_t (&s)[NB][4], const uint32_t* tbl, uint32_t b0,
                                                      uint32_t b1) {
    uint32_t x[NB][4];
#pragma unroll
    for (int b = 0; b < NB; b++)
#pragma unroll
        for (int c = 0; c < 4; c++) x[b][c] = s[b][c];   // rk0 = 0
#pragma unroll
    for (int r = 1; r < 10; r++) {
        uint32_t y[NB][4];
#pragma unroll
        for (int b = 0; b < NB; b++)
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const uint32_t t0 = Tab::template term<0>(tbl, b0, b1, x[b][c]);
                const uint32_t t1 = Tab::template term<1>(tbl, b0, b1, x[b][(c + 1) & 3]);
                const uint32_t t2 = Tab::template term<2>(tbl, b0, b1, x[b][(c + 2) & 3]);
                const uint32_t t3 = Tab::template term<3>(tbl, b0, b1, x[b][(c + 3) & 3]);
                // two v_bitop3_b32 (3-input XOR) instead of four v_xor_b32
                y[b][c] = Ops::xor3(Ops::xor3(t0, t1, t2), t3, ZERO_RK.w[r][c]);
            }
#pragma unroll
        for (int b = 0; b < NB; b++)
#pragma unroll
            for (int c = 0; c < 4; c++) x[b][c] = y[b][c];
    }
    constexpr uint32_t sel_lo = 0x0C0C0000u | ((uint32_t)(4 + Tab::spos(1)) << 8) | (uint32_t)Tab::spos(0);
    constexpr uint32_t sel_hi = ((uint32_t)(4 + Tab::spos(3)) << 24) | ((uint32_t)Tab::spos(2) << 16) | 0x0C0Cu;
#pragma unroll
    for (int b = 0; b < NB; b++) {
        uint32_t o[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t a0 = Tab::template last<0>(tbl, b0, b1, x[b][c]);
            const uint32_t a1 = Tab::template last<1>(tbl, b0, b1, x[b][(c + 1) & 3]);
            const uint32_t a2 = Tab::template last<2>(tbl, b0, b1, x[b][(c + 2) & 3]);
            const uint32_t a3 = Tab::template last<3>(tbl, b0, b1, x[b][(c + 3) & 3]);
            o[c] = Ops::xor3(Ops::perm(a1, a0, sel_lo), Ops::perm(a3, a2, sel_hi), ZERO_RK.w[10][c]);
        }
#pragma unroll
        for (int c = 0; c < 4; c++) s[b][c] ^= o[c];   // MMO feed-forward (prg.rs:227-230)
    }
}

// ---- AES-128 (zero key) + MMO for sibling counter PAIRS ---------------------------------
// expand_dir evaluates a seed in both directions at every level: block 2q uses ctr = k
// (dir 0, left child), block 2q+1 uses ctr = k + 2^64 (dir 1, prg.rs:273-276). Unless byte 8
// of k is 0xFF (a carry into byte 9), the two counters differ in byte 8 alone, i.e. in one
// byte of column 2. After round 1 only column 2 differs (MixColumns stays inside the
// column), and in round 2 each output column takes exactly one byte of column 2
// (ShiftRows). So the dir-1 block needs 1 table lookup in round 1 and 4 in round 2 instead of
// 16 + 16; rounds 3..10 are independent. Per pair: 293 lookups instead of 320 (the generic
// function's compiler CSE reaches 312).
// A carry in any lane of the wave (probability 1 - (255/256)^64 = 22 % per pair) makes the
// whole wave recompute the dir-1 block's rounds 1-2 in full (a wave-uniform branch; it is
// exact for every lane, carry or not), so the output is bit-identical to aes0_mmo_tab.
template <class Ops, class Tab, int NB>
__host__ __device__ __forceinline__ void aes0_mmo_pair(uint32_t (&s)[NB][4], const uint32_t* tbl, uint32_t b0,
                                                       uint32_t b1) {
    static_assert(NB % 2 == 0, "blocks come in (dir 0, dir 1) pairs");
    uint32_t x[NB][4];
#pragma unroll
    for (int q = 0; q < NB / 2; q++) {
        const uint32_t* a = s[2 * q];
        const uint32_t* bb = s[2 * q + 1];
        // round 1: generic for block A, only the column-2 row-0 term differs for block B
        uint32_t ya[4], yb2;
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t t0 = Tab::template term<0>(tbl, b0, b1, a[c]);
            const uint32_t t1 = Tab::template term<1>(tbl, b0, b1, a[(c + 1) & 3]);
            const uint32_t t2 = Tab::template term<2>(tbl, b0, b1, a[(c + 2) & 3]);
            const uint32_t t3 = Tab::template term<3>(tbl, b0, b1, a[(c + 3) & 3]);
            const uint32_t p = Ops::xor3(t1, t2, t3);
            ya[c] = Ops::xor3(p, t0, ZERO_RK.w[1][c]);
            if (c == 2) yb2 = Ops::xor3(p, Tab::template term<0>(tbl, b0, b1, bb[2]), ZERO_RK.w[1][2]);
        }
        // round 2: each output column c takes row k = (2 - c) & 3 of column 2
        uint32_t za[4], zb[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            uint32_t t[4];
            t[0] = Tab::template term<0>(tbl, b0, b1, ya[c]);
            t[1] = Tab::template term<1>(tbl, b0, b1, ya[(c + 1) & 3]);
            t[2] = Tab::template term<2>(tbl, b0, b1, ya[(c + 2) & 3]);
            t[3] = Tab::template term<3>(tbl, b0, b1, ya[(c + 3) & 3]);
            const int k = (2 - c) & 3;
            uint32_t tb;
            if (k == 0) tb = Tab::template term<0>(tbl, b0, b1, yb2);
            else if (k == 1) tb = Tab::template term<1>(tbl, b0, b1, yb2);
            else if (k == 2) tb = Tab::template term<2>(tbl, b0, b1, yb2);
            else tb = Tab::template term<3>(tbl, b0, b1, yb2);
            const uint32_t p = Ops::xor3(t[(k + 1) & 3], t[(k + 2) & 3], t[(k + 3) & 3]);
            za[c] = Ops::xor3(p, t[k], ZERO_RK.w[2][c]);
            zb[c] = Ops::xor3(p, tb, ZERO_RK.w[2][c]);
        }
        // carry into byte 9 somewhere in the wave (byte 8 = 0xFF): B's counter also differs in
        // byte 9 = row 1 of column 2, which round 1 sends to output column 1. Fix-up exact for
        // every lane whose carry stops at byte 9 (lanes without a carry cancel to zero): round 1
        // column 1 gains one lookup pair, round 2 one row-(1 - c) term of column 1 per column.
        // A carry past byte 9 (bytes 8-9 = 0xFFFF, 1/65536 per lane) redoes rounds 1-2 in full.
        if (Ops::any((a[2] & 0xFFFFu) == 0xFFFFu)) {
            uint32_t u[4];
#pragma unroll
            for (int c = 0; c < 4; c++) u[c] = bb[c];
#pragma unroll
            for (int r = 1; r <= 2; r++) {
                uint32_t v[4];
#pragma unroll
                for (int c = 0; c < 4; c++)
                    v[c] = Ops::xor3(Ops::xor3(Tab::template term<0>(tbl, b0, b1, u[c]),
                                               Tab::template term<1>(tbl, b0, b1, u[(c + 1) & 3]),
                                               Tab::template term<2>(tbl, b0, b1, u[(c + 2) & 3])),
                                     Tab::template term<3>(tbl, b0, b1, u[(c + 3) & 3]), ZERO_RK.w[r][c]);
#pragma unroll
                for (int c = 0; c < 4; c++) u[c] = v[c];
            }
#pragma unroll
            for (int c = 0; c < 4; c++) zb[c] = u[c];
        } else if (Ops::any((a[2] & 0xFFu) == 0xFFu)) {
            const uint32_t yb1 = Ops::xor3(ya[1], Tab::template term<1>(tbl, b0, b1, a[2]),
                                           Tab::template term<1>(tbl, b0, b1, bb[2]));
            // output column c takes row k = (1 - c) & 3 of column 1: c = 0 k 1, c = 1 k 0, c = 2 k 3, c = 3 k 2
            zb[0] = Ops::xor3(zb[0], Tab::template term<1>(tbl, b0, b1, ya[1]), Tab::template term<1>(tbl, b0, b1, yb1));
            zb[1] = Ops::xor3(zb[1], Tab::template term<0>(tbl, b0, b1, ya[1]), Tab::template term<0>(tbl, b0, b1, yb1));
            zb[2] = Ops::xor3(zb[2], Tab::template term<3>(tbl, b0, b1, ya[1]), Tab::template term<3>(tbl, b0, b1, yb1));
            zb[3] = Ops::xor3(zb[3], Tab::template term<2>(tbl, b0, b1, ya[1]), Tab::template term<2>(tbl, b0, b1, yb1));
        }
#pragma unroll
        for (int c = 0; c < 4; c++) {
            x[2 * q][c] = za[c];
            x[2 * q + 1][c] = zb[c];
        }
    }
#pragma unroll
    for (int r = 3; r < 10; r++) {
        uint32_t y[NB][4];
#pragma unroll
        for (int b = 0; b < NB; b++)
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const uint32_t t0 = Tab::template term<0>(tbl, b0, b1, x[b][c]);
                const uint32_t t1 = Tab::template term<1>(tbl, b0, b1, x[b][(c + 1) & 3]);
                const uint32_t t2 = Tab::template term<2>(tbl, b0, b1, x[b][(c + 2) & 3]);
                const uint32_t t3 = Tab::template term<3>(tbl, b0, b1, x[b][(c + 3) & 3]);
                y[b][c] = Ops::xor3(Ops::xor3(t0, t1, t2), t3, ZERO_RK.w[r][c]);
            }
#pragma unroll
        for (int b = 0; b < NB; b++)
#pragma unroll
            for (int c = 0; c < 4; c++) x[b][c] = y[b][c];
    }
    constexpr uint32_t sel_lo = 0x0C0C0000u | ((uint32_t)(4 + Tab::spos(1)) << 8) | (uint32_t)Tab::spos(0);
    constexpr uint32_t sel_hi = ((uint32_t)(4 + Tab::spos(3)) << 24) | ((uint32_t)Tab::spos(2) << 16) | 0x0C0Cu;
#pragma unroll
    for (int b = 0; b < NB; b++) {
        uint32_t o[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t a0 = Tab::template last<0>(tbl, b0, b1, x[b][c]);
            const uint32_t a1 = Tab::template last<1>(tbl, b0, b1, x[b][(c + 1) & 3]);
            const uint32_t a2 = Tab::template last<2>(tbl, b0, b1, x[b][(c + 2) & 3]);
            const uint32_t a3 = Tab::template last<3>(tbl, b0, b1, x[b][(c + 3) & 3]);
            o[c] = Ops::xor3(Ops::perm(a1, a0, sel_lo), Ops::perm(a3, a2, sel_hi), ZERO_RK.w[10][c]);
        }
#pragma unroll
        for (int c = 0; c < 4; c++) s[b][c] ^= o[c];   // MMO feed-forward (prg.rs:227-230)
    }
}

struct DevOpsX : DevOps {
    // wave-uniform "any lane": the carry fallback of aes0_mmo_pair is a scalar branch
    static __device__ __forceinline__ bool any(bool p) { return __ballot(p) != 0; }
    static __device__ __forceinline__ uint32_t bfe(uint32_t x, uint32_t off, uint32_t w) {
        return (x >> off) & ((1u << w) - 1u);
    }
    // gfx950 v_bitop3_b32, truth table 0x96 = a ^ b ^ c (hipcc does not form it from ^ chains)
    static __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
        return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
    }
};

}  // namespace fhh
