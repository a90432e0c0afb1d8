// Host check of the k_expand work decomposition (fhh_internal.h item_layout) and of the
// kernel's item -> (job, entry range, word range) decode (fhh_kernels.hip k_expand, including
// the multi-word bulk items of variant 51): for random job sizes, every (job, entry, word) is
// covered exactly once, no item reaches past n_live or nw, and a multi-word layout still gives
// every wave at least kMwItemsPerWave items.
// Built with hipcc (host code only) by tests/test_host_aes.py; prints "OK" on success.
#include "../../fuzzyheavyhitters_amd/csrc/fhh_internal.h"
#include <cstdio>
#include <random>
#include <vector>

int main() {
    std::mt19937_64 rng(7);
    int fails = 0;
    for (int it = 0; it < 3000; it++) {
        const uint32_t njobs = 1 + rng() % fhh::kMaxJobs;
        const uint32_t unit = 1 + rng() % 64;
        const uint32_t max_group = 1 + rng() % 16;
        const uint64_t waves = 1 + rng() % 512;
        const bool tail = rng() & 1;
        const uint32_t max_wpi = (rng() & 1) ? 1u : 1u + (uint32_t)(rng() % 16);
        uint32_t n_live[fhh::kMaxJobs] = {};
        for (uint32_t k = 0; k < njobs; k++) n_live[k] = (it % 7 == 0) ? (uint32_t)(rng() % 3) : (uint32_t)(rng() % 700);
        fhh::ItemLayout L;
        fhh::item_layout(n_live, njobs, unit, max_group, waves, tail, L, max_wpi);
        std::vector<std::vector<uint8_t>> seen(njobs);
        for (uint32_t k = 0; k < njobs; k++) seen[k].assign((size_t)n_live[k] * unit, 0);
        if (L.items_a > L.total) fails++;
        if (L.wpi < 1 || L.wpi > max_wpi || (tail && L.wpi != 1)) fails++;
        if (L.wpi > 1 && L.total < fhh::kMwItemsPerWave * waves) fails++;
        const uint32_t nwi = (unit + L.wpi - 1) / L.wpi;   // bulk items per entry group
        for (uint64_t item = 0; item < L.total; item++) {
            const bool tl = item >= L.items_a;
            uint32_t ji = 0;
            const uint64_t* beg = tl ? L.begin_b : L.begin_a;
            while (ji + 1 < njobs && item >= beg[ji + 1]) ji++;
            const uint64_t local = item - beg[ji];
            const uint32_t per = tl ? unit : nwi, wpi = tl ? 1u : L.wpi;
            const uint32_t wc = (uint32_t)(local % per), g = (uint32_t)(local / per);
            const uint32_t w0 = wc * wpi, w1 = w0 + wpi < unit ? w0 + wpi : unit;
            const uint32_t base = tl ? L.split[ji] : 0, grp = tl ? L.g_b : L.g;
            const uint32_t end_lim = tl ? n_live[ji] : L.split[ji];
            const uint32_t e0 = base + g * grp;
            uint32_t e1 = e0 + grp;
            if (e1 > end_lim) e1 = end_lim;
            if (e0 >= e1) { fails++; continue; }   // an item with no work
            if (w0 >= w1) { fails++; continue; }
            for (uint32_t e = e0; e < e1; e++)
                for (uint32_t w = w0; w < w1; w++) seen[ji][(size_t)e * unit + w]++;
        }
        for (uint32_t k = 0; k < njobs; k++)
            for (uint8_t v : seen[k])
                if (v != 1) { fails++; break; }
        if (L.split[0] > n_live[0]) fails++;
    }
    // the narrow / wide cases of DESIGN.md §5 at 1M clients (nw 15 625, 4 096 waves)
    {
        const uint32_t narrow[4] = {1, 1, 1, 1};   // configs[3]: ~1 entry per (server, dim)
        fhh::ItemLayout L;
        fhh::item_layout(narrow, 4, 15625, 16, 4096, false, L, 16);
        if (L.wpi != 3 || L.total != 4 * 5209) fails++;   // lowered until 4 items per wave
        const uint32_t wide[2] = {200, 200};                // a deep d = 1 level
        fhh::item_layout(wide, 2, 15625, 16, 4096, false, L, 16);
        if (L.g != 16) fails++;
        if (L.wpi != 1) fails++;
    }
    if (fails) { std::printf("FAIL %d\n", fails); return 1; }
    std::printf("OK\n");
    return 0;
}
