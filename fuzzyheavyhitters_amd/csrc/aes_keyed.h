// AES-128 T-table rounds with runtime round keys (any table layout of expand_kernel.h), shared
// by the sketch PrgStream (fhh_sketch.hip) and the garbled-circuit kernels (fhh_gc.hip).
#pragma once
#include "expand_kernel.h"

namespace fhh {

// s <- AES_rk(s) for NB independent blocks (little-endian column words)
template <class Tab, int NB>
__device__ __forceinline__ void aes_rk(uint32_t (&s)[NB][4], const uint32_t* tbl, uint32_t b0, uint32_t b1,
                                       const uint32_t (&rk)[11][4]) {
    uint32_t x[NB][4];
#pragma unroll
    for (int q = 0; q < NB; q++)
#pragma unroll
        for (int c = 0; c < 4; c++) x[q][c] = s[q][c] ^ rk[0][c];
#pragma unroll
    for (int r = 1; r < 10; r++) {
        uint32_t y[NB][4];
#pragma unroll
        for (int q = 0; q < NB; q++)
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const uint32_t t0 = Tab::template term<0>(tbl, b0, b1, x[q][c]);
                const uint32_t t1 = Tab::template term<1>(tbl, b0, b1, x[q][(c + 1) & 3]);
                const uint32_t t2 = Tab::template term<2>(tbl, b0, b1, x[q][(c + 2) & 3]);
                const uint32_t t3 = Tab::template term<3>(tbl, b0, b1, x[q][(c + 3) & 3]);
                y[q][c] = DevOpsX::xor3(DevOpsX::xor3(t0, t1, t2), t3, rk[r][c]);
            }
#pragma unroll
        for (int q = 0; q < NB; q++)
#pragma unroll
            for (int c = 0; c < 4; c++) x[q][c] = y[q][c];
    }
    constexpr uint32_t sel_lo = 0x0C0C0000u | ((uint32_t)(4 + Tab::spos(1)) << 8) | (uint32_t)Tab::spos(0);
    constexpr uint32_t sel_hi = ((uint32_t)(4 + Tab::spos(3)) << 24) | ((uint32_t)Tab::spos(2) << 16) | 0x0C0Cu;
#pragma unroll
    for (int q = 0; q < NB; q++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t a0 = Tab::template last<0>(tbl, b0, b1, x[q][c]);
            const uint32_t a1 = Tab::template last<1>(tbl, b0, b1, x[q][(c + 1) & 3]);
            const uint32_t a2 = Tab::template last<2>(tbl, b0, b1, x[q][(c + 2) & 3]);
            const uint32_t a3 = Tab::template last<3>(tbl, b0, b1, x[q][(c + 3) & 3]);
            s[q][c] = DevOpsX::xor3(DevOpsX::perm(a1, a0, sel_lo), DevOpsX::perm(a3, a2, sel_hi), rk[10][c]);
        }
}

// s <- AES_rk0(s) for blocks [0, Q) and AES_rk1(s) for blocks [Q, 2Q): two uniform key
// schedules (the OT receiver's row keys k_i^0, k_i^1) with all 2Q blocks in lockstep
template <class Tab, int Q>
__device__ __forceinline__ void aes_rk2(uint32_t (&s)[2 * Q][4], const uint32_t* tbl, uint32_t b0, uint32_t b1,
                                        const uint32_t (&rk0)[11][4], const uint32_t (&rk1)[11][4]) {
    constexpr int NB = 2 * Q;
    uint32_t x[NB][4];
#pragma unroll
    for (int q = 0; q < NB; q++)
#pragma unroll
        for (int c = 0; c < 4; c++) x[q][c] = s[q][c] ^ (q < Q ? rk0[0][c] : rk1[0][c]);
#pragma unroll
    for (int r = 1; r < 10; r++) {
        uint32_t y[NB][4];
#pragma unroll
        for (int q = 0; q < NB; q++)
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const uint32_t t0 = Tab::template term<0>(tbl, b0, b1, x[q][c]);
                const uint32_t t1 = Tab::template term<1>(tbl, b0, b1, x[q][(c + 1) & 3]);
                const uint32_t t2 = Tab::template term<2>(tbl, b0, b1, x[q][(c + 2) & 3]);
                const uint32_t t3 = Tab::template term<3>(tbl, b0, b1, x[q][(c + 3) & 3]);
                y[q][c] = DevOpsX::xor3(DevOpsX::xor3(t0, t1, t2), t3, q < Q ? rk0[r][c] : rk1[r][c]);
            }
#pragma unroll
        for (int q = 0; q < NB; q++)
#pragma unroll
            for (int c = 0; c < 4; c++) x[q][c] = y[q][c];
    }
    constexpr uint32_t sel_lo = 0x0C0C0000u | ((uint32_t)(4 + Tab::spos(1)) << 8) | (uint32_t)Tab::spos(0);
    constexpr uint32_t sel_hi = ((uint32_t)(4 + Tab::spos(3)) << 24) | ((uint32_t)Tab::spos(2) << 16) | 0x0C0Cu;
#pragma unroll
    for (int q = 0; q < NB; q++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t a0 = Tab::template last<0>(tbl, b0, b1, x[q][c]);
            const uint32_t a1 = Tab::template last<1>(tbl, b0, b1, x[q][(c + 1) & 3]);
            const uint32_t a2 = Tab::template last<2>(tbl, b0, b1, x[q][(c + 2) & 3]);
            const uint32_t a3 = Tab::template last<3>(tbl, b0, b1, x[q][(c + 3) & 3]);
            s[q][c] = DevOpsX::xor3(DevOpsX::perm(a1, a0, sel_lo), DevOpsX::perm(a3, a2, sel_hi),
                                    q < Q ? rk0[10][c] : rk1[10][c]);
        }
}

// s <- AES_key(s) for NB blocks under ONE per-lane key, the schedule expanded on the fly (one
// round key live instead of 44 words: the sketch kernels' per-key PrgStream, where a lane's key
// differs from its neighbours' and a stored schedule would cost 44 VGPRs). Per round: SubWord of
// RotWord(w3) through the same tables (4 lookups), rcon, the w0..w3 chain (FIPS-197 5.2).
template <class Tab>
__device__ __forceinline__ uint32_t sub_rot_word(uint32_t w3, const uint32_t* tbl, uint32_t b0, uint32_t b1) {
    constexpr uint32_t sel_lo = 0x0C0C0000u | ((uint32_t)(4 + Tab::spos(1)) << 8) | (uint32_t)Tab::spos(0);
    constexpr uint32_t sel_hi = ((uint32_t)(4 + Tab::spos(3)) << 24) | ((uint32_t)Tab::spos(2) << 16) | 0x0C0Cu;
    const uint32_t r = (w3 >> 8) | (w3 << 24);   // RotWord on the little-endian column word
    const uint32_t a0 = Tab::template last<0>(tbl, b0, b1, r);
    const uint32_t a1 = Tab::template last<1>(tbl, b0, b1, r);
    const uint32_t a2 = Tab::template last<2>(tbl, b0, b1, r);
    const uint32_t a3 = Tab::template last<3>(tbl, b0, b1, r);
    return DevOpsX::perm(a1, a0, sel_lo) | DevOpsX::perm(a3, a2, sel_hi);
}

template <class Tab, int NB>
__device__ __forceinline__ void aes_otf(uint32_t (&s)[NB][4], const uint32_t* tbl, uint32_t b0, uint32_t b1,
                                        const uint32_t (&key)[4]) {
    uint32_t k[4] = {key[0], key[1], key[2], key[3]};
    uint32_t x[NB][4];
#pragma unroll
    for (int q = 0; q < NB; q++)
#pragma unroll
        for (int c = 0; c < 4; c++) x[q][c] = s[q][c] ^ k[c];
    uint32_t rcon = 1;
#pragma unroll
    for (int r = 1; r < 10; r++) {
        k[0] ^= sub_rot_word<Tab>(k[3], tbl, b0, b1) ^ rcon;
        k[1] ^= k[0];
        k[2] ^= k[1];
        k[3] ^= k[2];
        rcon = (rcon << 1) ^ ((rcon & 0x80) ? 0x11Bu : 0u);
        uint32_t y[NB][4];
#pragma unroll
        for (int q = 0; q < NB; q++)
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const uint32_t t0 = Tab::template term<0>(tbl, b0, b1, x[q][c]);
                const uint32_t t1 = Tab::template term<1>(tbl, b0, b1, x[q][(c + 1) & 3]);
                const uint32_t t2 = Tab::template term<2>(tbl, b0, b1, x[q][(c + 2) & 3]);
                const uint32_t t3 = Tab::template term<3>(tbl, b0, b1, x[q][(c + 3) & 3]);
                y[q][c] = DevOpsX::xor3(DevOpsX::xor3(t0, t1, t2), t3, k[c]);
            }
#pragma unroll
        for (int q = 0; q < NB; q++)
#pragma unroll
            for (int c = 0; c < 4; c++) x[q][c] = y[q][c];
    }
    k[0] ^= sub_rot_word<Tab>(k[3], tbl, b0, b1) ^ rcon;   // rcon(10) = 0x36
    k[1] ^= k[0];
    k[2] ^= k[1];
    k[3] ^= k[2];
    constexpr uint32_t sel_lo = 0x0C0C0000u | ((uint32_t)(4 + Tab::spos(1)) << 8) | (uint32_t)Tab::spos(0);
    constexpr uint32_t sel_hi = ((uint32_t)(4 + Tab::spos(3)) << 24) | ((uint32_t)Tab::spos(2) << 16) | 0x0C0Cu;
#pragma unroll
    for (int q = 0; q < NB; q++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t a0 = Tab::template last<0>(tbl, b0, b1, x[q][c]);
            const uint32_t a1 = Tab::template last<1>(tbl, b0, b1, x[q][(c + 1) & 3]);
            const uint32_t a2 = Tab::template last<2>(tbl, b0, b1, x[q][(c + 2) & 3]);
            const uint32_t a3 = Tab::template last<3>(tbl, b0, b1, x[q][(c + 3) & 3]);
            s[q][c] = DevOpsX::xor3(DevOpsX::perm(a1, a0, sel_lo), DevOpsX::perm(a3, a2, sel_hi), k[c]);
        }
}

// s <- AES(s) for NB blocks with the 11 round keys read from LDS (rkl: 44 words, 16-B aligned,
// the same address for every lane of a key's segment: a broadcast ds_read_b128 per round)
template <class Tab, int NB>
__device__ __forceinline__ void aes_lds_rk(uint32_t (&s)[NB][4], const uint32_t* tbl, uint32_t b0, uint32_t b1,
                                           const uint4* rkl) {
    uint32_t x[NB][4];
    {
        const uint4 k = rkl[0];
        const uint32_t kw[4] = {k.x, k.y, k.z, k.w};
#pragma unroll
        for (int q = 0; q < NB; q++)
#pragma unroll
            for (int c = 0; c < 4; c++) x[q][c] = s[q][c] ^ kw[c];
    }
#pragma unroll
    for (int r = 1; r < 10; r++) {
        const uint4 k = rkl[r];
        const uint32_t kw[4] = {k.x, k.y, k.z, k.w};
        uint32_t y[NB][4];
#pragma unroll
        for (int q = 0; q < NB; q++)
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const uint32_t t0 = Tab::template term<0>(tbl, b0, b1, x[q][c]);
                const uint32_t t1 = Tab::template term<1>(tbl, b0, b1, x[q][(c + 1) & 3]);
                const uint32_t t2 = Tab::template term<2>(tbl, b0, b1, x[q][(c + 2) & 3]);
                const uint32_t t3 = Tab::template term<3>(tbl, b0, b1, x[q][(c + 3) & 3]);
                y[q][c] = DevOpsX::xor3(DevOpsX::xor3(t0, t1, t2), t3, kw[c]);
            }
#pragma unroll
        for (int q = 0; q < NB; q++)
#pragma unroll
            for (int c = 0; c < 4; c++) x[q][c] = y[q][c];
    }
    const uint4 k = rkl[10];
    const uint32_t kw[4] = {k.x, k.y, k.z, k.w};
    constexpr uint32_t sel_lo = 0x0C0C0000u | ((uint32_t)(4 + Tab::spos(1)) << 8) | (uint32_t)Tab::spos(0);
    constexpr uint32_t sel_hi = ((uint32_t)(4 + Tab::spos(3)) << 24) | ((uint32_t)Tab::spos(2) << 16) | 0x0C0Cu;
#pragma unroll
    for (int q = 0; q < NB; q++)
#pragma unroll
        for (int c = 0; c < 4; c++) {
            const uint32_t a0 = Tab::template last<0>(tbl, b0, b1, x[q][c]);
            const uint32_t a1 = Tab::template last<1>(tbl, b0, b1, x[q][(c + 1) & 3]);
            const uint32_t a2 = Tab::template last<2>(tbl, b0, b1, x[q][(c + 2) & 3]);
            const uint32_t a3 = Tab::template last<3>(tbl, b0, b1, x[q][(c + 3) & 3]);
            s[q][c] = DevOpsX::xor3(DevOpsX::perm(a1, a0, sel_lo), DevOpsX::perm(a3, a2, sel_hi), kw[c]);
        }
}

// the 11 round keys of `key` (FIPS-197 5.2) through the tables (for writing to LDS)
template <class Tab>
__device__ __forceinline__ void key_schedule_tab(const uint32_t (&key)[4], uint32_t (&rk)[11][4],
                                                 const uint32_t* tbl, uint32_t b0, uint32_t b1) {
#pragma unroll
    for (int c = 0; c < 4; c++) rk[0][c] = key[c];
    uint32_t rcon = 1;
#pragma unroll
    for (int r = 1; r < 11; r++) {
        rk[r][0] = rk[r - 1][0] ^ sub_rot_word<Tab>(rk[r - 1][3], tbl, b0, b1) ^ rcon;
        rk[r][1] = rk[r - 1][1] ^ rk[r][0];
        rk[r][2] = rk[r - 1][2] ^ rk[r][1];
        rk[r][3] = rk[r - 1][3] ^ rk[r][2];
        rcon = (rcon << 1) ^ ((rcon & 0x80) ? 0x11Bu : 0u);
    }
}

}  // namespace fhh
