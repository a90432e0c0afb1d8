// Host self-test of the 32 x 32 bit transpose (csrc/bitslice.h) the OT hashes and the garbled-table
// kernels use on the tile-major IKNP matrices: out[b] bit j = in[j] bit b, and an involution.
#include <cstdio>
#include <random>

#include "../../fuzzyheavyhitters_amd/csrc/bitslice.h"

int main() {
    std::mt19937 rng(7);
    for (int it = 0; it < 2000; it++) {
        uint32_t a[32], b[32];
        for (int i = 0; i < 32; i++) a[i] = b[i] = rng();
        if (it == 0)
            for (int i = 0; i < 32; i++) a[i] = b[i] = 1u << i;   // identity
        fhh::transpose32(b);
        for (int i = 0; i < 32; i++)
            for (int j = 0; j < 32; j++)
                if (((b[i] >> j) & 1u) != ((a[j] >> i) & 1u)) {
                    std::printf("FAIL transpose it %d (%d, %d)\n", it, i, j);
                    return 1;
                }
        fhh::transpose32(b);
        for (int i = 0; i < 32; i++)
            if (b[i] != a[i]) {
                std::printf("FAIL involution it %d\n", it);
                return 1;
            }
    }
    std::printf("OK\n");
    return 0;
}
