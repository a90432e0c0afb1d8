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

}  // namespace fhh
