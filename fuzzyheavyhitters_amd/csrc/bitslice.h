// The 32 x 32 bit transpose of the OT kernels (fhh_ot.hip) and the garbled-table kernels (fhh_gc.hip),
// which read the tile-major IKNP matrices as row words; host self-test tests/host/transpose_host_test.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fhh {

// 32x32 bit transpose in registers: out[b] bit j = in[j] bit b (an involution). Stage S swaps
// the off-diagonal SxS blocks of every 2Sx2S block.
template <int S>
__host__ __device__ __forceinline__ void transpose_stage(uint32_t (&a)[32]) {
    constexpr uint32_t m = S == 16 ? 0x0000FFFFu : S == 8 ? 0x00FF00FFu : S == 4 ? 0x0F0F0F0Fu
                         : S == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
    for (int hi = 0; hi < 32; hi += 2 * S)
#pragma unroll
        for (int lo = 0; lo < S; lo++) {
            const int j = hi + lo;
            const uint32_t t = ((a[j] >> S) ^ a[j + S]) & m;
            a[j + S] ^= t;
            a[j] ^= t << S;
        }
}

__host__ __device__ __forceinline__ void transpose32(uint32_t (&a)[32]) {
    transpose_stage<16>(a);
    transpose_stage<8>(a);
    transpose_stage<4>(a);
    transpose_stage<2>(a);
    transpose_stage<1>(a);
}

}  // namespace fhh
