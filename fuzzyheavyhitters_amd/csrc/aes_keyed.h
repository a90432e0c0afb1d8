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

// T_k lookup with k known only after unrolling (folds to one term<k>)
template <class Tab>
__device__ __forceinline__ uint32_t term_k(int k, const uint32_t* tbl, uint32_t b0, uint32_t b1, uint32_t x) {
    switch (k & 3) {
        case 0: return Tab::template term<0>(tbl, b0, b1, x);
        case 1: return Tab::template term<1>(tbl, b0, b1, x);
        case 2: return Tab::template term<2>(tbl, b0, b1, x);
        default: return Tab::template term<3>(tbl, b0, b1, x);
    }
}

// s <- AES_rk(s) for NB blocks that differ from block 0 only in the byte at row R of column C
// (one lane's AES-CTR blocks whose counters share every other byte, e.g. the OT expand's blocks
// c0 + 64 q + lane with c0 a multiple of 256). The key addition keeps the difference in that byte;
// round 1 sends it through T_R into output column D = (C - R) & 3 alone (MixColumns stays in its
// column), and in round 2 each output column takes exactly one byte of column D (ShiftRows). So
// blocks 1.. cost 1 + 4 lookups in rounds 1-2 instead of 32 (k_expand's sibling pairs, variant 34,
// use the same structure for the zero key): 133 instead of 160 per block. Exact for any inputs
// that meet the precondition; the caller guarantees it.
// Round keys come from a source: RkRegs (registers / SGPRs) or RkLds (one ds_read_b128 per round).
struct RkRegs {
    const uint32_t (&rk)[11][4];
    __device__ __forceinline__ void get(int r, uint32_t (&w)[4]) const {
#pragma unroll
        for (int c = 0; c < 4; c++) w[c] = rk[r][c];
    }
};
struct RkLds {
    const uint4* rkl;
    __device__ __forceinline__ void get(int r, uint32_t (&w)[4]) const {
        const uint4 k = rkl[r];
        w[0] = k.x;
        w[1] = k.y;
        w[2] = k.z;
        w[3] = k.w;
    }
};

template <class Tab, int NB, int R, int C, class Rk>
__device__ __forceinline__ void aes_ctr_shared(uint32_t (&s)[NB][4], const uint32_t* tbl, uint32_t b0, uint32_t b1,
                                               const Rk& src) {
    constexpr int D = (C - R + 4) & 3;
    uint32_t rk[4];
    src.get(0, rk);
    uint32_t a[4], d[NB];
#pragma unroll
    for (int c = 0; c < 4; c++) a[c] = s[0][c] ^ rk[c];
#pragma unroll
    for (int q = 0; q < NB; q++) d[q] = s[q][C] ^ rk[C];
    src.get(1, rk);
    // round 1 (block 0 in full; the others differ only in column D's term R)
    uint32_t y[4], pd = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) {
        uint32_t t[4];
#pragma unroll
        for (int k = 0; k < 4; k++) t[k] = term_k<Tab>(k, tbl, b0, b1, a[(c + k) & 3]);
        if (c == D) {
            pd = DevOpsX::xor3(t[(R + 1) & 3], t[(R + 2) & 3], t[(R + 3) & 3]);
            y[c] = DevOpsX::xor3(pd, t[R], rk[c]);
        } else {
            y[c] = DevOpsX::xor3(DevOpsX::xor3(t[0], t[1], t[2]), t[3], rk[c]);
        }
    }
    uint32_t yd[NB];
    yd[0] = y[D];
#pragma unroll
    for (int q = 1; q < NB; q++) yd[q] = DevOpsX::xor3(pd, term_k<Tab>(R, tbl, b0, b1, d[q]), rk[D]);
    src.get(2, rk);
    // round 2: output column c takes row k = (D - c) & 3 of column D
    uint32_t x[NB][4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
        uint32_t t[4];
#pragma unroll
        for (int k = 0; k < 4; k++) t[k] = term_k<Tab>(k, tbl, b0, b1, y[(c + k) & 3]);
        const int k = (D - c + 4) & 3;
        const uint32_t pex = DevOpsX::xor3(t[(k + 1) & 3], t[(k + 2) & 3], t[(k + 3) & 3]);
        x[0][c] = DevOpsX::xor3(pex, t[k], rk[c]);
#pragma unroll
        for (int q = 1; q < NB; q++) x[q][c] = DevOpsX::xor3(pex, term_k<Tab>(k, tbl, b0, b1, yd[q]), rk[c]);
    }
#pragma unroll
    for (int r = 3; r < 10; r++) {
        src.get(r, rk);
        uint32_t z[NB][4];
#pragma unroll
        for (int q = 0; q < NB; q++)
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const uint32_t t0 = Tab::template term<0>(tbl, b0, b1, x[q][c]);
                const uint32_t t1 = Tab::template term<1>(tbl, b0, b1, x[q][(c + 1) & 3]);
                const uint32_t t2 = Tab::template term<2>(tbl, b0, b1, x[q][(c + 2) & 3]);
                const uint32_t t3 = Tab::template term<3>(tbl, b0, b1, x[q][(c + 3) & 3]);
                z[q][c] = DevOpsX::xor3(DevOpsX::xor3(t0, t1, t2), t3, rk[c]);
            }
#pragma unroll
        for (int q = 0; q < NB; q++)
#pragma unroll
            for (int c = 0; c < 4; c++) x[q][c] = z[q][c];
    }
    src.get(10, rk);
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
            s[q][c] = DevOpsX::xor3(DevOpsX::perm(a1, a0, sel_lo), DevOpsX::perm(a3, a2, sel_hi), rk[c]);
        }
}

// r05: the per-key constant part of rounds 1-2 for AES-CTR blocks that ALL differ from s0 only in
// the byte at row R of column C (the sketch keystream: big-endian counters b < 256 differ in byte 15
// alone, for every block of the key). aes_ctr_shared pays block 0's rounds 1-2 in full on every
// call; here they are paid once per key: pre[0] = round 1's column-D terms other than T_R, with
// rk1[D]; pre[1 + c] = round 2's column-c terms other than the one fed by column D, with rk2[c];
// pre[5] = rk0[C]. Every block then costs 1 + 4 lookups in rounds 1-2 (133 per block, aes_ctr_pre).
template <class Tab, int R, int C, class Rk>
__device__ __forceinline__ void aes_ctr_pre_init(const uint32_t (&s0)[4], const uint32_t* tbl, uint32_t b0,
                                                 uint32_t b1, const Rk& src, uint32_t (&pre)[6]) {
    constexpr int D = (C - R + 4) & 3;
    uint32_t rk[4], a[4], y[4];
    src.get(0, rk);
    pre[5] = rk[C];
#pragma unroll
    for (int c = 0; c < 4; c++) a[c] = s0[c] ^ rk[c];
    src.get(1, rk);
#pragma unroll
    for (int c = 0; c < 4; c++) {
        uint32_t t[4];
#pragma unroll
        for (int k = 0; k < 4; k++) t[k] = term_k<Tab>(k, tbl, b0, b1, a[(c + k) & 3]);
        y[c] = DevOpsX::xor3(DevOpsX::xor3(t[0], t[1], t[2]), t[3], rk[c]);
        if (c == D) pre[0] = DevOpsX::xor3(t[(R + 1) & 3], t[(R + 2) & 3], t[(R + 3) & 3]) ^ rk[c];
    }
    src.get(2, rk);
#pragma unroll
    for (int c = 0; c < 4; c++) {
        const int k = (D - c + 4) & 3;   // the row of column D that output column c takes
        uint32_t t[4];
#pragma unroll
        for (int j = 1; j < 4; j++) t[j] = term_k<Tab>((k + j) & 3, tbl, b0, b1, y[(c + ((k + j) & 3)) & 3]);
        pre[1 + c] = DevOpsX::xor3(t[1], t[2], t[3]) ^ rk[c];
    }
}

template <class Tab, int NB, int R, int C, class Rk>
__device__ __forceinline__ void aes_ctr_pre(uint32_t (&s)[NB][4], const uint32_t* tbl, uint32_t b0, uint32_t b1,
                                            const Rk& src, const uint32_t (&pre)[6]) {
    constexpr int D = (C - R + 4) & 3;
    uint32_t x[NB][4];
#pragma unroll
    for (int q = 0; q < NB; q++) {
        const uint32_t yd = pre[0] ^ term_k<Tab>(R, tbl, b0, b1, s[q][C] ^ pre[5]);   // round 1, column D
#pragma unroll
        for (int c = 0; c < 4; c++) x[q][c] = pre[1 + c] ^ term_k<Tab>((D - c + 4) & 3, tbl, b0, b1, yd);   // round 2
    }
    uint32_t rk[4];
#pragma unroll
    for (int r = 3; r < 10; r++) {
        src.get(r, rk);
        uint32_t z[NB][4];
#pragma unroll
        for (int q = 0; q < NB; q++)
#pragma unroll
            for (int c = 0; c < 4; c++) {
                const uint32_t t0 = Tab::template term<0>(tbl, b0, b1, x[q][c]);
                const uint32_t t1 = Tab::template term<1>(tbl, b0, b1, x[q][(c + 1) & 3]);
                const uint32_t t2 = Tab::template term<2>(tbl, b0, b1, x[q][(c + 2) & 3]);
                const uint32_t t3 = Tab::template term<3>(tbl, b0, b1, x[q][(c + 3) & 3]);
                z[q][c] = DevOpsX::xor3(DevOpsX::xor3(t0, t1, t2), t3, rk[c]);
            }
#pragma unroll
        for (int q = 0; q < NB; q++)
#pragma unroll
            for (int c = 0; c < 4; c++) x[q][c] = z[q][c];
    }
    src.get(10, rk);
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
            s[q][c] = DevOpsX::xor3(DevOpsX::perm(a1, a0, sel_lo), DevOpsX::perm(a3, a2, sel_hi), rk[c]);
        }
}

template <class Tab, int NB, int R, int C>
__device__ __forceinline__ void aes_rk_ctr(uint32_t (&s)[NB][4], const uint32_t* tbl, uint32_t b0, uint32_t b1,
                                           const uint32_t (&rk)[11][4]) {
    aes_ctr_shared<Tab, NB, R, C>(s, tbl, b0, b1, RkRegs{rk});
}

template <class Tab, int NB, int R, int C>
__device__ __forceinline__ void aes_lds_rk_ctr(uint32_t (&s)[NB][4], const uint32_t* tbl, uint32_t b0, uint32_t b1,
                                               const uint4* rkl) {
    aes_ctr_shared<Tab, NB, R, C>(s, tbl, b0, b1, RkLds{rkl});
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
