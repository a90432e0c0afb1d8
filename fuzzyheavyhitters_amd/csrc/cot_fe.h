// The correlated OTs' FE value of a 16-B hash output (fhh_ot.hip mode 2, and since r05c the share the
// garbled circuit's output labels carry, fhh_gc.hip): the block as a little-endian u128 mod
// p_FE = 2^62 - 2^30 - 1 (fastfield.rs), oracle/fhh_oracle.c cot_fe_of_block.
#pragma once
#include <cstdint>

#include <hip/hip_runtime.h>

namespace fhh {

constexpr uint64_t kOtFeP = (1ull << 62) - (1ull << 30) - 1;

// 2^64 = 2^32 + 4 and 2^62 = 2^30 + 1 mod p (statistically 2^-66 from uniform)
__device__ __forceinline__ uint64_t ot_fe_of_u128(uint64_t lo, uint64_t hi) {
    constexpr uint64_t M62 = (1ull << 62) - 1;
    const unsigned __int128 x = (unsigned __int128)hi * ((1ull << 32) + 4) + lo;     // < 2^98
    const unsigned __int128 y = (unsigned __int128)(uint64_t)(x >> 62) * ((1ull << 30) + 1) + ((uint64_t)x & M62);
    uint64_t z = ((uint64_t)y & M62) + (uint64_t)(y >> 62) * ((1ull << 30) + 1);       // < 2^62 + 2^36
    return z >= kOtFeP ? z - kOtFeP : z;
}

}  // namespace fhh
