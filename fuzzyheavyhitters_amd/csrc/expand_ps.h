// VALU waves of the hybrid k_expand (variants 45-48): the same work items as
// the T-table waves (64 clients of one word x up to 16 prefix entries x 2 sides x 2 dirs, from
// the same counter, in the same client-major layout), but the AES runs pair-sliced on the VALU
// (aes_ps_gen.h) instead of through the LDS T-tables, so these waves add blocks without
// touching the LDS array the T-table waves saturate.
//
// One batch = 4 entries x 2 sides x 2 dirs = 16 units of 64 clients = 1024 blocks. Lane
// 4u + 2h + p holds unit u's clients 32h .. 32h + 31, part p (p = 0: block bytes 0..7, 1: 8..15).
//   in:  each lane loads its 8-byte half of its 32 clients' parent seeds, forms the PRG counter
//        (prg.rs:96, 273-276) and bit-transposes them (two 32x32 in-register transposes); the
//        t / y planes come from word 0 of the seeds with lanes = clients, as in expand_item.
//   AES: aes0_ps (the zero-key AES-128, 517 lane-ops per block).
//   out: two 32x32 in-register transposes give each lane the u32 words 2p, 2p + 1 of its 32
//        clients; feed-forward (the counter, reloaded from L2), correction word under t
//        (ibDCF.rs:215-217), 8-byte stores into the child rows. t / y planes as expand_item.
#pragma once
#include "aes_ps_gen.h"
#include "aes_ttable.h"
#include "fhh_internal.h"

namespace fhh {

struct PsDevOps {
    template <int imm>
    static __device__ __forceinline__ uint32_t b3(uint32_t a, uint32_t b, uint32_t c) {
        return __builtin_amdgcn_bitop3_b32(a, b, c, imm);
    }
    static __device__ __forceinline__ void fence() { __builtin_amdgcn_sched_barrier(0); }
    // the partner lane's value (DPP quad_perm [1,0,3,2]: lanes 2k <-> 2k + 1)
    static __device__ __forceinline__ uint32_t swap(uint32_t x) {
        return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, false);
    }
};

// 32x32 bit transpose of a[O .. O + 31] (out[b] bit j = in[j] bit b, = transpose32): v_perm for
// the 16- and 8-bit stages (2 ops per word pair), a shift + v_bitop3 select for 4, 2, 1 (4 ops)
template <int O, int S>
__device__ __forceinline__ void transpose_stage_dev(uint32_t (&a)[64]) {
    constexpr uint32_t m = S == 4 ? 0x0F0F0F0Fu : S == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
    for (int hi = 0; hi < 32; hi += 2 * S)
#pragma unroll
        for (int lo = 0; lo < S; lo++) {
            const int j = O + hi + lo;
            const uint32_t A = a[j], B = a[j + S];
            if constexpr (S == 16) {
                a[j] = __builtin_amdgcn_perm(B, A, 0x05040100u);
                a[j + S] = __builtin_amdgcn_perm(B, A, 0x07060302u);
            } else if constexpr (S == 8) {
                a[j] = __builtin_amdgcn_perm(B, A, 0x06020400u);
                a[j + S] = __builtin_amdgcn_perm(B, A, 0x07030501u);
            } else {
                a[j] = __builtin_amdgcn_bitop3_b32(m, A, B << S, 0xCA);        // m ? A : B << S
                a[j + S] = __builtin_amdgcn_bitop3_b32(m, A >> S, B, 0xCA);    // m ? A >> S : B
            }
        }
}

// an empty asm per word ends a stage: the compiler may neither merge permutes across stages
// (perm o perm = perm, which stretches live ranges past the 128-VGPR budget) nor reorder them
template <int O>
__device__ __forceinline__ void stage_fence(uint32_t (&a)[64]) {
#pragma unroll
    for (int j = O; j < O + 32; j++) asm volatile("" : "+v"(a[j]));
}

template <int O>
__device__ __forceinline__ void transpose32_dev(uint32_t (&a)[64]) {
    stage_fence<O>(a);
    transpose_stage_dev<O, 16>(a);
    stage_fence<O>(a);
    transpose_stage_dev<O, 8>(a);
    stage_fence<O>(a);
    transpose_stage_dev<O, 4>(a);
    stage_fence<O>(a);
    transpose_stage_dev<O, 2>(a);
    stage_fence<O>(a);
    transpose_stage_dev<O, 1>(a);
    stage_fence<O>(a);
}

// Lane-parallel bit transpose in: the lane's 8-byte part p of 32 consecutive client blocks
// (row = the row at client 32h, offset by p uint2; client m at row[2m]) -> pair-sliced state.
// CTR: the PRG counter of the block (prg.rs:96, 273-276): p = 0 masks the low nibble of byte 0,
// p = 1 adds `cadd` (the direction) to the upper u64.
template <bool CTR>
__device__ __forceinline__ void ps_gather_in(uint32_t (&st)[64], const uint2* row, uint64_t cmask, uint64_t cadd) {
#pragma unroll
    for (int m = 0; m < 32; m++) {
        const uint2 v = row[2 * m];
        uint64_t x = ((uint64_t)v.y << 32) | v.x;
        if constexpr (CTR) x = (x & cmask) + cadd;
        st[m] = (uint32_t)x;
        st[32 + m] = (uint32_t)(x >> 32);
    }
    __builtin_amdgcn_sched_barrier(0);
    transpose32_dev<0>(st);
    transpose32_dev<32>(st);
}

__device__ __forceinline__ void expand_item_ps(const ExpandJob& J, uint64_t local, uint32_t lane) {
    const uint32_t w = (uint32_t)(local % J.nw);
    const uint32_t g = (uint32_t)(local / J.nw);
    const size_t npad = J.npad, nw = J.nw;
    const size_t krow = (size_t)J.level * J.K + 2 * J.dim;
    const uint32_t c = w * 64 + lane;
    // this lane's unit u = 4 ei + 2 s + dir, client half h, part p
    const uint32_t p = lane & 1, h = (lane >> 1) & 1, u = lane >> 2;
    const uint32_t ei_l = u >> 2, s_l = (u >> 1) & 1, dir_l = u & 1;
    const uint32_t isb = 0u - p;
    const uint64_t cmask = p ? ~0ull : ~0xFull;   // prg_ctr on this lane's half of the block
    const uint64_t cadd = p ? dir_l : 0;
    const size_t col = (size_t)w * 64 + 32 * h;
    uint64_t cwp[2][4];
#pragma unroll
    for (int s = 0; s < 2; s++)
#pragma unroll
        for (int b = 0; b < 4; b++) cwp[s][b] = J.cw_bits[((krow + s) * 4 + b) * nw + w];

    const uint32_t e_begin = J.e_base + g * J.group;
    const uint32_t e_end = min(e_begin + J.group, J.n_live);
    for (uint32_t eb = e_begin; eb < e_end; eb += 4) {
        const uint32_t ne = min(4u, e_end - eb);
        // t / y planes of the batch's children (ibDCF.rs:211-219, as expand_item): lanes = clients
        for (uint32_t ei = 0; ei < ne; ei++) {
            const uint32_t src = J.live[eb + ei];
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const uint32_t w0 = reinterpret_cast<const uint32_t*>(J.src_seed + ((size_t)src * 2 + s) * npad + c)[0];
                const uint64_t tw = J.src_t[((size_t)src * 2 + s) * nw + w];
                const uint64_t yw = J.src_y[((size_t)src * 2 + s) * nw + w];
#pragma unroll
                for (int dir = 0; dir < 2; dir++) {
                    uint32_t bit, ybit;
                    prg_ctrl_bits(w0 & 0xFFFFFFF0u, dir, bit, ybit);
                    const uint64_t pb = __ballot(bit), py = __ballot(ybit);
                    if (lane == 0) {
                        const size_t de = (size_t)(2 * (eb + ei) + dir) * 2 + s;
                        J.dst_t[de * nw + w] = pb ^ (tw & cwp[s][dir]);
                        J.dst_y[de * nw + w] = py ^ (tw & cwp[s][2 + dir]) ^ yw;
                    }
                }
            }
        }
        // every lane runs its unit (lanes of absent units take the batch's last entry and store
        // nothing), so no branch pulls the AES into a divergent block
        const bool act = ei_l < ne;
        const uint32_t e = eb + (act ? ei_l : ne - 1);
        const uint32_t src = J.live[e];
        const uint2* srow = reinterpret_cast<const uint2*>(J.src_seed + ((size_t)src * 2 + s_l) * npad + col) + p;
        uint32_t st[64];
        ps_gather_in<true>(st, srow, cmask, cadd);
        aes0_ps<PsDevOps>(st, isb);
        __builtin_amdgcn_sched_barrier(0);
        transpose32_dev<0>(st);
        transpose32_dev<32>(st);
        // feed-forward (the counter again, from L1/L2), correction word under t, store
        const uint2* crow = reinterpret_cast<const uint2*>(J.cw_seed + (krow + s_l) * npad + col) + p;
        uint2* drow = reinterpret_cast<uint2*>(J.dst_seed + ((size_t)(2 * e + dir_l) * 2 + s_l) * npad + col) + p;
        const uint32_t th = (uint32_t)(J.src_t[((size_t)src * 2 + s_l) * nw + w] >> (32 * h));
#pragma unroll
        for (int m = 0; m < 32; m++) {
            const uint2 sv = srow[2 * m];
            const uint2 cv = crow[2 * m];
            const uint64_t ctr = ((((uint64_t)sv.y << 32) | sv.x) & cmask) + cadd;
            const uint32_t tm = (uint32_t)__builtin_amdgcn_sbfe((int)th, m, 1);   // state.bit ? ~0 : 0
            uint2 o;
            o.x = st[m] ^ (uint32_t)ctr ^ (cv.x & tm);
            o.y = st[32 + m] ^ (uint32_t)(ctr >> 32) ^ (cv.y & tm);
            if (act) drow[2 * m] = o;
            if ((m & 7) == 7) __builtin_amdgcn_sched_barrier(0);   // <= 8 clients' loads in flight
        }
    }
}

// Debug / test kernel (fhh_debug_aes_ps): one wave, 16 units x 64 blocks; in[u * 64 + j] is
// unit u's block j; out = AES_0 of each block through the expand_item_ps data path (gather +
// transpose in, aes0_ps, transposes out), without feed-forward.
__global__ __launch_bounds__(64) void k_debug_aes_ps(const uint4* __restrict__ in, uint4* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t p = lane & 1, h = (lane >> 1) & 1, u = lane >> 2;
    uint32_t st[64];
    ps_gather_in<false>(st, reinterpret_cast<const uint2*>(in + u * 64 + 32 * h) + p, 0, 0);
    aes0_ps<PsDevOps>(st, 0u - p);
    __builtin_amdgcn_sched_barrier(0);
    transpose32_dev<0>(st);
    transpose32_dev<32>(st);
    uint2* o = reinterpret_cast<uint2*>(out + u * 64 + 32 * h) + p;
#pragma unroll
    for (int m = 0; m < 32; m++) o[2 * m] = make_uint2(st[m], st[32 + m]);
}

}  // namespace fhh
