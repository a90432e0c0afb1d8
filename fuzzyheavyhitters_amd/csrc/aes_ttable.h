// AES-128 (fixed all-zero key) + Matyas-Meyer-Oseas feed-forward, T-table form for CDNA4.
//
// Restates `FixedKeyPrgStream::refill` (src/prg.rs:212-234): out = AES_0(ctr) XOR ctr,
// one block per `eval_bit` (ibDCF.rs:208-227 -> prg.rs:92-122).
//
// Table layout in LDS (64 KiB per workgroup): T0 entry x, replica r at byte address
// x*256 + r*4, one replica per lane of the wave (r = lane). A `ds_read_b32` services a
// wave64 in two 32-lane groups and banks on (addr/4) mod 32 = lane mod 32, so every
// lookup is bank-conflict free whatever the looked-up bytes are. The address of byte k of
// a state word is ONE `v_perm_b32`: {0, 0, x.byte[k], lane*4}.
// T1..T3 are rotations of T0 (`v_alignbit_b32`); the last round extracts S[x] = byte 1 of
// T0[x] with two `v_perm_b32` per column.
//
// The code is generic over the primitive ops (Ops::perm, Ops::load) so the identical round
// structure can be instantiated on the host with emulated ops for a CPU self-test
// (tests/host/aes_ttable_host_test.cpp); the product only instantiates DevOps.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "aes_tables.h"

namespace fhh {

constexpr int kTableReplicas = 64;                        // one per lane
constexpr int kTableWords = 256 * kTableReplicas;         // 16384 u32 = 64 KiB

__host__ __device__ constexpr uint32_t rotl32(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

// v_perm_b32 selector: {lanebase.byte0, x.byte[k], 0, 0}
__host__ __device__ constexpr uint32_t lookup_sel(int k) { return 0x0C0C0004u | ((uint32_t)k << 8); }

template <class Ops>
__host__ __device__ __forceinline__ uint32_t tlook(const uint32_t* tbl, uint32_t lanebase, uint32_t x, int k) {
    return Ops::load(tbl, Ops::perm(lanebase, x, lookup_sel(k)));
}

// s[b][0..3]: counter blocks as little-endian column words; replaced by AES_0(s) ^ s.
template <class Ops, int NB>
__host__ __device__ __forceinline__ void aes0_mmo(uint32_t (&s)[NB][4], const uint32_t* tbl, uint32_t lanebase) {
    uint32_t x[NB][4];
#pragma unroll
    for (int b = 0; b < NB; b++)
#pragma unroll
        for (int c = 0; c < 4; c++) x[b][c] = s[b][c];   // AddRoundKey(rk0 = 0) is the identity

#pragma unroll
    for (int r = 1; r < 10; r++) {
        uint32_t y[NB][4];
#pragma unroll
        for (int b = 0; b < NB; b++) {
#pragma unroll
            for (int c = 0; c < 4; c++) {
                // column c of SubBytes∘ShiftRows takes row k from column c+k
                uint32_t a0 = tlook<Ops>(tbl, lanebase, x[b][c], 0);
                uint32_t a1 = tlook<Ops>(tbl, lanebase, x[b][(c + 1) & 3], 1);
                uint32_t a2 = tlook<Ops>(tbl, lanebase, x[b][(c + 2) & 3], 2);
                uint32_t a3 = tlook<Ops>(tbl, lanebase, x[b][(c + 3) & 3], 3);
                y[b][c] = a0 ^ rotl32(a1, 8) ^ rotl32(a2, 16) ^ rotl32(a3, 24) ^ ZERO_RK.w[r][c];
            }
        }
#pragma unroll
        for (int b = 0; b < NB; b++)
#pragma unroll
            for (int c = 0; c < 4; c++) x[b][c] = y[b][c];
    }

    // final round: SubBytes∘ShiftRows, no MixColumns; S[v] = byte 1 of T0[v]
#pragma unroll
    for (int b = 0; b < NB; b++) {
        uint32_t o[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            uint32_t a0 = tlook<Ops>(tbl, lanebase, x[b][c], 0);
            uint32_t a1 = tlook<Ops>(tbl, lanebase, x[b][(c + 1) & 3], 1);
            uint32_t a2 = tlook<Ops>(tbl, lanebase, x[b][(c + 2) & 3], 2);
            uint32_t a3 = tlook<Ops>(tbl, lanebase, x[b][(c + 3) & 3], 3);
            uint32_t lo = Ops::perm(a1, a0, 0x0C0C0501u);   // {a0.b1, a1.b1, 0, 0}
            uint32_t hi = Ops::perm(a3, a2, 0x05010C0Cu);   // {0, 0, a2.b1, a3.b1}
            o[c] = lo ^ hi ^ ZERO_RK.w[10][c];
        }
#pragma unroll
        for (int c = 0; c < 4; c++) s[b][c] ^= o[c];         // MMO feed-forward (prg.rs:227-230)
    }
}

// The PRG counter for `expand_dir` (prg.rs:92-122): key byte 0 masked to its high nibble
// (prg.rs:96); the right child's block uses ctr + 1 in the UPPER u64 lane (bytes 8..15,
// little-endian, no carry into bytes 0..7: `_mm_add_epi64(v, _mm_set_epi64x(1, 0))`,
// prg.rs:273-276).
__host__ __device__ __forceinline__ void prg_ctr(const uint32_t seed[4], int dir, uint32_t out[4]) {
    out[0] = seed[0] & 0xFFFFFFF0u;
    out[1] = seed[1];
    uint64_t hi = ((uint64_t)seed[3] << 32) | seed[2];
    hi += (uint64_t)dir;
    out[2] = (uint32_t)hi;
    out[3] = (uint32_t)(hi >> 32);
}

// Control bits of `expand_dir` read from the MASKED byte 0 (prg.rs:101-104): after
// `key_short[0] &= 0xF0` they are always (true, true) — returned as (bits, y_bits) words
// computed from the masked byte, exactly as the reference does.
__host__ __device__ __forceinline__ void prg_ctrl_bits(uint32_t masked_w0, int dir, uint32_t& bit, uint32_t& ybit) {
    uint32_t b0 = masked_w0 & 0xFFu;
    bit = ((b0 >> dir) & 1u) ^ 1u;          // (k[0] & (1 << dir)) == 0
    ybit = ((b0 >> (2 + dir)) & 1u) ^ 1u;   // (k[0] & (4 << dir)) == 0
}

struct DevOps {
    static __device__ __forceinline__ uint32_t perm(uint32_t a, uint32_t b, uint32_t sel) {
        return __builtin_amdgcn_perm(a, b, sel);
    }
    static __device__ __forceinline__ uint32_t load(const uint32_t* tbl, uint32_t byte_addr) {
        return *(const uint32_t*)((const char*)tbl + byte_addr);
    }
};

}  // namespace fhh
