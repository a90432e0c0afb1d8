// Field arithmetic shared by the host engine and the device-resident level loop.
//   FE    : p = 2^62 - 2^30 - 1   (src/fastfield.rs:24-28)
//   FE255 : p = 2^255 - 19        (src/field.rs:19)
// Sums arrive as u64 partials of 32-bit limbs (limb k has weight 2^(32k)), so 2^32 summands
// per limb cannot overflow; one reduction at the end gives the canonical value.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fhh {

constexpr uint64_t kFieldFeP = (1ull << 62) - (1ull << 30) - 1;

// (lo + hi * 2^32) mod p_FE
__host__ __device__ inline uint64_t fe_canon_from_limbs(uint64_t lo, uint64_t hi) {
    const unsigned __int128 v = (unsigned __int128)lo + ((unsigned __int128)hi << 32);
    return (uint64_t)(v % kFieldFeP);
}

// (a - b) mod p_FE on canonical values — keep_values (collect.rs:950-953)
__host__ __device__ inline uint64_t fe_sub_canon(uint64_t a, uint64_t b) { return a >= b ? a - b : a + (kFieldFeP - b); }

// carry-propagate 8 u64 limb sums into 10 u32 limbs (the exact unreduced integer)
__host__ __device__ inline void limbs10_from_partials(const uint64_t* p8, uint32_t* out10) {
    unsigned __int128 carry = 0;
    for (int k = 0; k < 10; k++) {
        const unsigned __int128 acc = carry + (k < 8 ? p8[k] : 0);
        out10[k] = (uint32_t)acc;
        carry = acc >> 32;
    }
}

// x mod (2^255 - 19) for x = 10 u32 limbs (< 2^320) -> 8 u32 limbs
__host__ __device__ inline void fe255_reduce(const uint32_t* x10, uint32_t* out8) {
    uint64_t w[5] = {0, 0, 0, 0, 0};
    for (int k = 0; k < 10; k++) w[k / 2] |= (uint64_t)x10[k] << (32 * (k % 2));
    for (int iter = 0; iter < 3; iter++) {   // x = hi * 2^255 + lo -> lo + 19 * hi
        const uint64_t hi0 = (w[3] >> 63) | (w[4] << 1), hi1 = w[4] >> 63;
        const uint64_t lo3 = w[3] & 0x7FFFFFFFFFFFFFFFull;
        unsigned __int128 acc = (unsigned __int128)w[0] + (unsigned __int128)hi0 * 19;
        w[0] = (uint64_t)acc;
        acc = (acc >> 64) + w[1] + (unsigned __int128)hi1 * 19;
        w[1] = (uint64_t)acc;
        acc = (acc >> 64) + w[2];
        w[2] = (uint64_t)acc;
        acc = (acc >> 64) + lo3;
        w[3] = (uint64_t)acc;
        w[4] = (uint64_t)(acc >> 64);
    }
    for (int iter = 0; iter < 2; iter++) {   // conditional subtract p
        uint64_t t[4];
        unsigned __int128 acc = (unsigned __int128)w[0] + 19;
        t[0] = (uint64_t)acc;
        for (int k = 1; k < 4; k++) {
            acc = (acc >> 64) + w[k];
            t[k] = (uint64_t)acc;
        }
        if (t[3] >> 63) {
            w[0] = t[0];
            w[1] = t[1];
            w[2] = t[2];
            w[3] = t[3] & 0x7FFFFFFFFFFFFFFFull;
        }
    }
    for (int k = 0; k < 8; k++) out8[k] = (uint32_t)(w[k / 2] >> (32 * (k % 2)));
}

// (a - b) mod p255 on canonical 8-limb values (field.rs:352-359 after reduce())
__host__ __device__ inline void fe255_sub(const uint32_t* a8, const uint32_t* b8, uint32_t* out8) {
    const uint32_t P[8] = {0xFFFFFFEDu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                           0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};
    uint32_t x[10];
    int64_t carry = 0;
    for (int k = 0; k < 8; k++) {
        const int64_t v = (int64_t)a8[k] + (int64_t)P[k] - (int64_t)b8[k] + carry;
        x[k] = (uint32_t)((uint64_t)v & 0xFFFFFFFFull);
        carry = (v - (int64_t)x[k]) / ((int64_t)1 << 32);
    }
    x[8] = (uint32_t)carry;
    x[9] = 0;
    fe255_reduce(x, out8);
}

__host__ __device__ inline bool fe255_ge_u32(const uint32_t* v8, uint32_t t) {
    for (int k = 7; k >= 1; k--)
        if (v8[k]) return true;
    return v8[0] >= t;
}

// ---- canonical GF(2^255 - 19) arithmetic on 8 x u32 little-endian limbs (FieldElm's lazy ops
// are exact BigUint add / mul then one reduce, field.rs:337-349: the same value mod p) --------
__host__ __device__ inline bool fe255_geq_p(const uint32_t (&a)[8]) {
    if (a[7] != 0x7FFFFFFFu) return a[7] > 0x7FFFFFFFu;
    for (int k = 6; k >= 1; k--)
        if (a[k] != 0xFFFFFFFFu) return false;
    return a[0] >= 0xFFFFFFEDu;
}

// r < 2^256 (= 2 p + 38) -> r mod p
__host__ __device__ inline void fe255_sub_p_twice(uint32_t (&r)[8]) {
    const uint32_t P[8] = {0xFFFFFFEDu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                           0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};
#pragma unroll
    for (int it = 0; it < 2; it++) {
        if (!fe255_geq_p(r)) break;
        uint64_t borrow = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint64_t v = (uint64_t)r[k] - P[k] - borrow;
            r[k] = (uint32_t)v;
            borrow = (v >> 63) & 1;
        }
    }
}

// x = lo + 2^256 hi (16 limbs) -> x mod p, folding 2^256 = 38 (mod p)
__host__ __device__ inline void fe255_fold16(const uint32_t (&x)[16], uint32_t (&out)[8]) {
    uint64_t c = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint64_t v = (uint64_t)x[k] + (uint64_t)x[8 + k] * 38u + c;
        out[k] = (uint32_t)v;
        c = v >> 32;
    }
    c *= 38u;   // < 39 * 38
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint64_t v = (uint64_t)out[k] + c;
        out[k] = (uint32_t)v;
        c = v >> 32;
    }
    if (c) {    // wrapped past 2^256 once more: the remainder is tiny, add 38
        uint64_t cc = 38;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint64_t v = (uint64_t)out[k] + cc;
            out[k] = (uint32_t)v;
            cc = v >> 32;
        }
    }
    fe255_sub_p_twice(out);
}

__host__ __device__ inline void fe255_mulm(const uint32_t (&a)[8], const uint32_t (&b)[8], uint32_t (&out)[8]) {
    uint32_t x[16];
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        uint64_t c = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint64_t v = (uint64_t)a[i] * b[j] + x[i + j] + c;
            x[i + j] = (uint32_t)v;
            c = v >> 32;
        }
        x[i + 8] = (uint32_t)c;
    }
    fe255_fold16(x, out);
}

__host__ __device__ inline void fe255_addm(const uint32_t (&a)[8], const uint32_t (&b)[8], uint32_t (&out)[8]) {
    uint64_t c = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint64_t v = (uint64_t)a[k] + b[k] + c;
        out[k] = (uint32_t)v;
        c = v >> 32;
    }
    // a, b < p: the sum < 2 p < 2^256, no carry out
    fe255_sub_p_twice(out);
}

__host__ __device__ inline void fe255_negm(const uint32_t (&a)[8], uint32_t (&out)[8]) {
    const uint32_t P[8] = {0xFFFFFFEDu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                           0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};
    uint64_t borrow = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        const uint64_t v = (uint64_t)P[k] - a[k] - borrow;
        out[k] = (uint32_t)v;
        borrow = (v >> 63) & 1;
    }
    fe255_sub_p_twice(out);   // a = 0 gives p -> 0
}

__host__ __device__ inline void fe255_subm(const uint32_t (&a)[8], const uint32_t (&b)[8], uint32_t (&out)[8]) {
    uint32_t nb[8];
    fe255_negm(b, nb);
    fe255_addm(a, nb, out);
}

// any value < 2^256 -> canonical
__host__ __device__ inline void fe255_canonm(uint32_t (&a)[8]) { fe255_sub_p_twice(a); }

}  // namespace fhh
