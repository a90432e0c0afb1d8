// Garbled-circuit equality test on the GPU: the circuit of
// `multiple_gb_equality_test` / `multiple_ev_equality_test` (src/equalitytest.rs:25-219) —
// per test, z_j = NOT(x_j XOR y_j) over the 2d share bits (`bin_eq_bundles`, :128-147),
// eq = AND of the z_j folded left to right (`and_many`), out = eq XOR mask
// (`multi_bin_eq_bundles_shared`, :165-189) — garbled with free-XOR + half-gates (Zahur, Rosulek,
// Evans 2015) and the TCCR hash H(x, i) = pi(pi(x) ^ i) ^ pi(x) (Guo, Katz, Wang, Yu 2020), as
// the swanky `fancy-garbling` garbler the reference links (@553ede0, not vendored: its fixed AES
// key and wire format cannot be restated, so pi here is AES-128 with the all-zero key, the same
// fixed-key permutation as the ibDCF PRG).
//
//   k_gc_garble  one lane per test: the garbler's zero labels from AES-128-CTR under its key,
//                2 ciphertexts per AND gate (4 TCCR = 8 AES), its active input labels, the
//                evaluator's active labels (ideal OT: the labels an OT extension would deliver)
//                and the output decoding bit
//   k_gc_eval    one lane per test: 2 TCCR (4 AES) per AND gate, output bit = colour ^ decode,
//                optionally also ballot-packed as the FE-share OT's choice words
//
// Both use the 4-table / 32-replica LDS T-table (conflict-free, as k_expand) and SoA outputs, so
// a wave's 64 lanes read and write 64 consecutive 16-B blocks.
#include "fhh_internal.h"
#include "aes_keyed.h"
#include "cot_fe.h"
#include "bitslice.h"

namespace fhh {

__constant__ WordTable c_T0_gc = T0;
using GcTab = Tab4T32<DevOpsX>;
constexpr int kGcThreads = 1024;

__device__ __forceinline__ void gc_fill(uint32_t* tbl) {
    for (int i = threadIdx.x; i < GcTab::kWords; i += blockDim.x) tbl[i] = GcTab::word(c_T0_gc.v, i);
    __syncthreads();
}

__device__ __forceinline__ void zero_rk(uint32_t (&rk)[11][4]) {
#pragma unroll
    for (int r = 0; r < 11; r++)
#pragma unroll
        for (int c = 0; c < 4; c++) rk[r][c] = ZERO_RK.w[r][c];
}

// TCCR on NB blocks: x <- pi(pi(x) ^ tweak) ^ pi(x), tweak in the low 64 bits
template <int NB>
__device__ __forceinline__ void tccr(uint32_t (&x)[NB][4], const uint64_t (&tw)[NB], const uint32_t* tbl,
                                     uint32_t b0, uint32_t b1, const uint32_t (&zrk)[11][4]) {
    uint32_t p[NB][4], q[NB][4];
#pragma unroll
    for (int k = 0; k < NB; k++)
#pragma unroll
        for (int c = 0; c < 4; c++) p[k][c] = x[k][c];
    aes_rk<GcTab, NB>(p, tbl, b0, b1, zrk);
#pragma unroll
    for (int k = 0; k < NB; k++) {
        q[k][0] = p[k][0] ^ (uint32_t)tw[k];
        q[k][1] = p[k][1] ^ (uint32_t)(tw[k] >> 32);
        q[k][2] = p[k][2];
        q[k][3] = p[k][3];
    }
    aes_rk<GcTab, NB>(q, tbl, b0, b1, zrk);
#pragma unroll
    for (int k = 0; k < NB; k++)
#pragma unroll
        for (int c = 0; c < 4; c++) x[k][c] = q[k][c] ^ p[k][c];
}

__device__ __forceinline__ uint32_t plane_bit(const uint64_t* planes, uint64_t g, uint32_t bits, uint32_t j,
                                              uint32_t nw, uint32_t i) {
    return (uint32_t)(planes[((size_t)g * bits + j) * nw + (i >> 6)] >> (i & 63)) & 1u;
}

// tests to run: G * N, or, inside the level loop, those of the chunk's groups [g_off, g_off + G)
// that the previous prune left (C children)
__device__ __forceinline__ uint64_t gc_active(const GcArgs& a) {
    if (!a.ctl) return a.G * a.N;
    if (a.ctl->abort) return 0;
    const uint64_t C = a.ctl->C;
    if (C <= a.g_off) return 0;
    const uint64_t g = C - a.g_off;
    return (g < a.G ? g : a.G) * a.N;
}

__device__ __forceinline__ void st_blk(uint4* base, uint64_t row, uint64_t n, uint64_t t, const uint32_t (&v)[4]) {
    base[row * n + t] = make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ void ld_blk(const uint4* base, uint64_t row, uint64_t n, uint64_t t, uint32_t (&v)[4]) {
    const uint4 q = base[row * n + t];
    v[0] = q.x;
    v[1] = q.y;
    v[2] = q.z;
    v[3] = q.w;
}

// The ideal-OT garbler (fhh_gc_equality_*, fhh_sim_config.gc = 1): every label drawn by the garbler,
// the evaluator's active ones written to ev_labels as an ideal OT would deliver them.
template <int B>
__global__ __launch_bounds__(kGcThreads) void k_gc_garble(GcArgs a) {
    __shared__ uint32_t tbl_gc[GcTab::kWords];   // static: a dynamic base costs an add per lookup
    // a workgroup without tests leaves before filling 128 KiB of tables (the level loop enqueues a
    // level's chunks up to its capacity, and chunks past the level's children run empty: r03 measured
    // 31 us per empty launch with the fill); the test is uniform over the workgroup
    if ((uint64_t)blockIdx.x * kGcThreads >= gc_active(a)) return;
    gc_fill(tbl_gc);
    uint32_t b0, b1;
    GcTab::bases(threadIdx.x & 63, b0, b1);
    uint32_t zrk[11][4];
    zero_rk(zrk);
    const uint64_t n = a.G * a.N;
    const uint32_t D[4] = {a.delta[0], a.delta[1], a.delta[2], a.delta[3]};
    uint32_t lrk[11][4];   // uniform: the label key schedule stays in SGPRs
#pragma unroll
    for (int r = 0; r < 11; r++)
#pragma unroll
        for (int c = 0; c < 4; c++) lrk[r][c] = a.rk_label[r][c];
    constexpr int W = 2 * B + 1;
    // label counter stride: the power of two >= W, so with label_nonce a multiple of it (the level
    // loop and the party ABI use 0) a test's W counters differ in byte 0 alone and a pass of its
    // label blocks shares AES rounds 1-2 (aes_rk_ctr: 133 instead of 160 lookups per extra block)
    constexpr int WS = W <= 4 ? 4 : W <= 8 ? 8 : W <= 16 ? 16 : 32;
    const uint64_t n_act = gc_active(a);
    for (uint64_t t = (uint64_t)blockIdx.x * kGcThreads + threadIdx.x; t < n_act; t += (uint64_t)gridDim.x * kGcThreads) {
        const uint64_t g = t / a.N;                  // group within the chunk
        const uint32_t i = (uint32_t)(t - g * a.N);
        const uint64_t tg = a.g_off * a.N + t;       // the test's index in the whole level
        // zero labels, generated per wire pair as the gates consume them (registers do not
        // grow with B): garbler string 0..B-1, mask B, evaluator string B+1..2B
        const uint64_t ctr0 = a.label_nonce + tg * WS;
        // wave-uniform: no lane's counters ctr0 .. ctr0 + W - 1 carry out of byte 0 (always, for an
        // aligned label_nonce; otherwise the pass runs every round in full)
        const bool shared = __ballot(((uint32_t)ctr0 & 0xFFu) + (W - 1) > 0xFFu) == 0;
        auto ctr_blk = [&](uint32_t (&b)[4], uint64_t c) {
            b[0] = (uint32_t)c;
            b[1] = (uint32_t)(c >> 32);
            b[2] = 0u;
            b[3] = 0u;
        };
        // B <= 2 (d = 1: the metric's configuration): all W <= 5 label blocks in one pass up front, 4
        // sharing rounds 1-2 with the first, instead of a 2-block pass then a 3-block one (692 instead of
        // 719 lookups, and 5 independent blocks in flight per lane)
        constexpr bool kOnePass = W <= 5;
        uint32_t L[kOnePass ? W : 1][4];
        if constexpr (kOnePass) {
#pragma unroll
            for (int w = 0; w < W; w++) ctr_blk(L[w], ctr0 + w);
            if (shared) aes_rk_ctr<GcTab, W, 0, 0>(L, tbl_gc, b0, b1, lrk);
            else aes_rk<GcTab, W>(L, tbl_gc, b0, b1, lrk);
        }
        uint32_t acc[4], m[1][4];
#pragma unroll
        for (int k = 0; k < B; k++) {
            // wires k (garbler) and B + 1 + k (evaluator); the last pair also takes the mask wire B
            uint32_t s[2][4];
            if constexpr (kOnePass) {
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    s[0][c] = L[k][c];
                    s[1][c] = L[B + 1 + k][c];
                    if (k == B - 1) m[0][c] = L[B][c];
                }
            } else if (k == B - 1) {
                uint32_t s3[3][4];
                ctr_blk(s3[0], ctr0 + k);
                ctr_blk(s3[1], ctr0 + B + 1 + k);
                ctr_blk(s3[2], ctr0 + B);
                if (shared) aes_rk_ctr<GcTab, 3, 0, 0>(s3, tbl_gc, b0, b1, lrk);
                else aes_rk<GcTab, 3>(s3, tbl_gc, b0, b1, lrk);
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    s[0][c] = s3[0][c];
                    s[1][c] = s3[1][c];
                    m[0][c] = s3[2][c];
                }
            } else {
                ctr_blk(s[0], ctr0 + k);
                ctr_blk(s[1], ctr0 + B + 1 + k);
                if (shared) aes_rk_ctr<GcTab, 2, 0, 0>(s, tbl_gc, b0, b1, lrk);
                else aes_rk<GcTab, 2>(s, tbl_gc, b0, b1, lrk);
            }
            // active labels: the garbler's bit (sent in the clear), the evaluator's (via OT)
            const uint32_t gb = plane_bit(a.gb_planes, a.g_off + g, B, k, a.nw, i);
            uint32_t x[4], bz[4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                x[c] = s[0][c] ^ (gb ? D[c] : 0u);
                bz[c] = s[0][c] ^ s[1][c] ^ D[c];   // z_k = NOT(x_k ^ y_k): free XOR, NOT = ^Delta
            }
            st_blk(a.gb_labels, k, n, t, x);
            {   // ideal OT: the evaluator's active label (what an OT would deliver)
                const uint32_t eb = plane_bit(a.ev_planes, a.g_off + g, B, k, a.nw, i);
                uint32_t y[4];
#pragma unroll
                for (int c = 0; c < 4; c++) y[c] = s[1][c] ^ (eb ? D[c] : 0u);
                st_blk(a.ev_labels, k, n, t, y);
            }
            if (k == 0) {
#pragma unroll
                for (int c = 0; c < 4; c++) acc[c] = bz[c];
                continue;
            }
            // half-gates AND(acc, z_k), gate index gate_base + t (B - 1) + k - 1
            uint32_t h[4][4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                h[0][c] = acc[c];
                h[1][c] = acc[c] ^ D[c];
                h[2][c] = bz[c];
                h[3][c] = bz[c] ^ D[c];
            }
            const uint32_t pa = acc[0] & 1u, pb = bz[0] & 1u;
            const uint64_t j = 2 * (a.gate_base + tg * (B - 1) + (k - 1));
            const uint64_t tw[4] = {j, j, j + 1, j + 1};
            tccr<4>(h, tw, tbl_gc, b0, b1, zrk);
            uint32_t TG[4], TE[4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                TG[c] = h[0][c] ^ h[1][c] ^ (pb ? D[c] : 0u);
                TE[c] = h[2][c] ^ h[3][c] ^ acc[c];
                const uint32_t wg = h[0][c] ^ (pa ? TG[c] : 0u);
                const uint32_t we = h[2][c] ^ (pb ? (TE[c] ^ acc[c]) : 0u);
                acc[c] = wg ^ we;
            }
            st_blk(a.tables, 2 * (k - 1), n, t, TG);
            st_blk(a.tables, 2 * (k - 1) + 1, n, t, TE);
        }
        // mask wire (labelled with the last pair); out = eq ^ mask has zero label acc ^ M0, decoding
        // bit = its colour
        a.decode[t] = (uint8_t)((acc[0] ^ m[0][0]) & 1u);
#pragma unroll
        for (int c = 0; c < 4; c++) m[0][c] ^= a.mask ? D[c] : 0u;
        st_blk(a.gb_labels, B, n, t, m[0]);
    }
}

// The r05 garbler (ev_ot = 1): the evaluator's input labels arrive by correlated OT — its zero label
// of share bit k is the C-OT's sender message E_k = H(q_j) at OT index (g B + k) Npad + i — and the
// garbler's own string is folded into the circuit instead of being encoded as input wires: for the
// input z_k = NOT(x_k ^ y_k) the garbler knows x_k, so it takes Z_k^0 = E_k ^ (x_k ? 0 : Delta), which
// makes the evaluator's OT'd label E_k ^ y_k Delta exactly Z_k's active label (XOR with a constant
// the garbler knows is free under free-XOR and hidden like any free gate). The mask folds into the
// decoding bit the same way: d = colour(out^0) ^ mask, so out = colour(acc) ^ d = eq ^ mask. No label
// is drawn at all (0 instead of 2 bits + 1 AES blocks per test) and no garbler label is sent: the gc
// message is the tables and the decoding bit (33 B per test at d = 1 instead of 81).
template <int B>
__global__ __launch_bounds__(kGcThreads) void k_gc_garble_cot(GcArgs a) {
    __shared__ uint32_t tbl_gc[GcTab::kWords];
    if ((uint64_t)blockIdx.x * kGcThreads >= gc_active(a)) return;   // no tests: skip the table fill
    gc_fill(tbl_gc);
    uint32_t b0, b1;
    GcTab::bases(threadIdx.x & 63, b0, b1);
    uint32_t zrk[11][4];
    zero_rk(zrk);
    const uint64_t n = a.G * a.N;
    const uint64_t Npad = (uint64_t)a.nw * 64;
    const uint32_t D[4] = {a.delta[0], a.delta[1], a.delta[2], a.delta[3]};
    const uint64_t n_act = gc_active(a);
    for (uint64_t t = (uint64_t)blockIdx.x * kGcThreads + threadIdx.x; t < n_act; t += (uint64_t)gridDim.x * kGcThreads) {
        const uint64_t g = t / a.N;                  // group within the chunk
        const uint32_t i = (uint32_t)(t - g * a.N);
        const uint64_t tg = a.g_off * a.N + t;       // the test's index in the whole level (gate tweaks)
        uint32_t acc[4];
#pragma unroll
        for (int k = 0; k < B; k++) {
            uint32_t bz[4];
            ld_blk(a.ev_labels, g * B + k, Npad, i, bz);   // E_k, the C-OT's zero label
            const uint32_t xb = plane_bit(a.gb_planes, a.g_off + g, B, k, a.nw, i);
#pragma unroll
            for (int c = 0; c < 4; c++) bz[c] ^= xb ? 0u : D[c];   // Z_k^0 = E_k ^ (x_k ? 0 : Delta)
            if (k == 0) {
#pragma unroll
                for (int c = 0; c < 4; c++) acc[c] = bz[c];
                continue;
            }
            // half-gates AND(acc, z_k), gate index gate_base + t (B - 1) + k - 1
            uint32_t h[4][4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                h[0][c] = acc[c];
                h[1][c] = acc[c] ^ D[c];
                h[2][c] = bz[c];
                h[3][c] = bz[c] ^ D[c];
            }
            const uint32_t pa = acc[0] & 1u, pb = bz[0] & 1u;
            const uint64_t j = 2 * (a.gate_base + tg * (B - 1) + (k - 1));
            const uint64_t tw[4] = {j, j, j + 1, j + 1};
            tccr<4>(h, tw, tbl_gc, b0, b1, zrk);
            uint32_t TG[4], TE[4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                TG[c] = h[0][c] ^ h[1][c] ^ (pb ? D[c] : 0u);
                TE[c] = h[2][c] ^ h[3][c] ^ acc[c];
                const uint32_t wg = h[0][c] ^ (pa ? TG[c] : 0u);
                const uint32_t we = h[2][c] ^ (pb ? (TE[c] ^ acc[c]) : 0u);
                acc[c] = wg ^ we;
            }
            st_blk(a.tables, 2 * (k - 1), n, t, TG);
            st_blk(a.tables, 2 * (k - 1) + 1, n, t, TE);
        }
        a.decode[t] = (uint8_t)((acc[0] ^ a.mask) & 1u);   // colour of eq's zero label, mask folded in
        if (a.sh_gb) {
            // r05c: the FE share from the output labels (oracle gc_share_garbler). W_0 = the label of
            // o = eq ^ mask = 0, W_1 = W_0 ^ Delta; (W_0, Delta) play the share C-OT's (q_j, s):
            // v = H(W_0) mod p, pair[1] = mask ? v + 1 : v - 1, node value r1 = v + mask,
            // y = lo64(H(W_1)) ^ pair[1]; H = cr_hash (2 AES blocks per test instead of the C-OT's 6)
            uint32_t h[2][4];
#pragma unroll
            for (int c = 0; c < 4; c++) {
                h[0][c] = acc[c] ^ (a.mask ? D[c] : 0u);
                h[1][c] = h[0][c] ^ D[c];
            }
            aes0_mmo_tab<DevOpsX, GcTab, 2>(h, tbl_gc, b0, b1);
            const uint64_t v = ot_fe_of_u128((uint64_t)h[0][0] | ((uint64_t)h[0][1] << 32),
                                             (uint64_t)h[0][2] | ((uint64_t)h[0][3] << 32));
            const uint64_t vp = v + 1 == kOtFeP ? 0 : v + 1, vm = v ? v - 1 : kOtFeP - 1;
            a.sh_gb[t] = a.mask ? vp : v;
            a.sh_y[t] = ((uint64_t)h[1][0] | ((uint64_t)h[1][1] << 32)) ^ (a.mask ? vp : vm);
        }
    }
}

// spread 32 bits to 64: bit k -> bits 2k and 2k + 1 (the doubled choices of a BlockPair OT)
__device__ __forceinline__ uint64_t spread2(uint32_t x) {
    uint64_t v = x;
    v = (v | (v << 16)) & 0x0000FFFF0000FFFFull;
    v = (v | (v << 8)) & 0x00FF00FF00FF00FFull;
    v = (v | (v << 4)) & 0x0F0F0F0F0F0F0F0Full;
    v = (v | (v << 2)) & 0x3333333333333333ull;
    v = (v | (v << 1)) & 0x5555555555555555ull;
    return v | (v << 1);
}

// Waves step over aligned 64-test slices (t0 wave-uniform), so with out_packed set the wave's
// ballot of its output bits is directly the OT choice words of tests t0 .. t0 + 63 (dup = 2:
// each bit twice, collect.rs:868) — no separate byte-to-bit pass.
// FOLD (ev_ot, r05): the garbler's string and the mask are folded into the circuit (k_gc_garble_cot),
// so the evaluator's OT'd label of bit k IS input z_k's active label, and the message has no garbler
// labels; otherwise (ideal OT) z_k = garbler label ^ evaluator label and the mask is a wire.
template <int B, bool FOLD>
__global__ __launch_bounds__(kGcThreads) void k_gc_eval(GcArgs a) {
    __shared__ uint32_t tbl_gc[GcTab::kWords];   // static: a dynamic base costs an add per lookup
    if ((uint64_t)blockIdx.x * kGcThreads >= gc_active(a)) return;   // no tests: skip the table fill
    gc_fill(tbl_gc);
    const uint32_t lane = threadIdx.x & 63;
    uint32_t b0, b1;
    GcTab::bases(lane, b0, b1);
    uint32_t zrk[11][4];
    zero_rk(zrk);
    const uint64_t n = a.G * a.N;
    const uint64_t n_act = gc_active(a);
    const uint64_t Npad = (uint64_t)a.nw * 64;
    for (uint64_t t0 = (uint64_t)blockIdx.x * kGcThreads + (threadIdx.x & ~63u); t0 < n_act;
         t0 += (uint64_t)gridDim.x * kGcThreads) {
        const uint64_t t = t0 + lane;
        uint32_t bit = 0;
        if (t < n_act) {
            const uint64_t g = t / a.N;
            const uint32_t i = (uint32_t)(t - g * a.N);
            uint32_t acc[4], x[4] = {0, 0, 0, 0}, y[4];
            if constexpr (FOLD) {
                ld_blk(a.ev_labels, g * B, Npad, i, y);
            } else {
                ld_blk(a.gb_labels, 0, n, t, x);
                ld_blk(a.ev_labels, 0, n, t, y);
            }
#pragma unroll
            for (int c = 0; c < 4; c++) acc[c] = x[c] ^ y[c];   // NOT is free for the evaluator
#pragma unroll
            for (int k = 1; k < B; k++) {
                uint32_t h[2][4], TG[4], TE[4];
                if constexpr (FOLD) {
                    ld_blk(a.ev_labels, g * B + k, Npad, i, y);
                } else {
                    ld_blk(a.gb_labels, k, n, t, x);
                    ld_blk(a.ev_labels, k, n, t, y);
                }
                ld_blk(a.tables, 2 * (k - 1), n, t, TG);
                ld_blk(a.tables, 2 * (k - 1) + 1, n, t, TE);
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    h[0][c] = acc[c];
                    h[1][c] = x[c] ^ y[c];
                }
                const uint32_t sa = acc[0] & 1u, sb = h[1][0] & 1u;
                const uint64_t j = 2 * (a.gate_base + (a.g_off * a.N + t) * (B - 1) + (k - 1));
                const uint64_t tw[2] = {j, j + 1};
                tccr<2>(h, tw, tbl_gc, b0, b1, zrk);
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const uint32_t wg = h[0][c] ^ (sa ? TG[c] : 0u);
                    const uint32_t we = h[1][c] ^ (sb ? (TE[c] ^ acc[c]) : 0u);
                    acc[c] = wg ^ we;
                }
            }
            if constexpr (!FOLD) ld_blk(a.gb_labels, B, n, t, x);   // mask wire (FOLD: in the decoding bit)
            bit = ((acc[0] ^ x[0]) & 1u) ^ a.decode[t];
            if (a.out) a.out[t] = (uint8_t)bit;
            if (FOLD && a.sh_ev) {
                // r05c: acc is W_o, o = bit (oracle gc_share_evaluator): o = 0 -> H(W_0) mod p = pair[0],
                // o = 1 -> lo64(H(W_1)) ^ y = pair[1]
                uint32_t h[1][4] = {{acc[0], acc[1], acc[2], acc[3]}};
                aes0_mmo_tab<DevOpsX, GcTab, 1>(h, tbl_gc, b0, b1);
                const uint64_t hl = (uint64_t)h[0][0] | ((uint64_t)h[0][1] << 32);
                a.sh_ev[t] = bit ? (hl ^ a.sh_y[t]) : ot_fe_of_u128(hl, (uint64_t)h[0][2] | ((uint64_t)h[0][3] << 32));
            }
        }
        if (a.out_packed) {
            const uint64_t v = __ballot(bit);
            if (a.out_dup == 1) {
                if (lane < 2) a.out_packed[t0 / 32 + lane] = (uint32_t)(v >> (32 * lane));
            } else if (lane < 4) {
                const uint64_t w = spread2((uint32_t)(v >> (32 * (lane >> 1))));
                a.out_packed[t0 / 16 + lane] = (uint32_t)(w >> (32 * (lane & 1)));
            }
        }
    }
}

// ---- r05d: the FE levels' equality test + share as one garbled table ----------------------------
// Yao's garbled gate with point-and-permute for the b-input gate "the share of eq ^ mask" (oracle
// orc_gt_garble / orc_gt_eval): the inputs are the folded garbler's Z_k (as
// k_gc_garble_cot), the evaluator's OT'd t_k is z_k's active label and its colours name its row r.
// Row r's key H(K_r), K_r = XOR_k sigma^k(label of z_k in row r) ^ tweak (sigma = doubling in
// GF(2^128)), H = cr_hash; row 0 carries no message (its value is H(K_0) mod p), rows 1 .. 2^b - 1
// send lo64(H(K_r)) ^ pair[o_r]. Garbler 2^b AES per test (4 at d = 1, against 8 + 2 for half-gates +
// the output-label share), evaluator 1 (against 4 + 1).
__device__ __forceinline__ void gf_dbl(uint32_t (&x)[4]) {
    const uint32_t carry = x[3] >> 31;
    x[3] = (x[3] << 1) | (x[2] >> 31);
    x[2] = (x[2] << 1) | (x[1] >> 31);
    x[1] = (x[1] << 1) | (x[0] >> 31);
    x[0] = (x[0] << 1) ^ (carry ? 0x87u : 0u);
}

__device__ __forceinline__ uint64_t fe_inc(uint64_t v) { return v + 1 == kOtFeP ? 0 : v + 1; }
__device__ __forceinline__ uint64_t fe_dec(uint64_t v) { return v ? v - 1 : kOtFeP - 1; }

#ifndef FHH_GT_GARBLE_U
#define FHH_GT_GARBLE_U 1   // tests per lane per pass (A/B knob)
#endif
#ifndef FHH_GT_EVAL_U
#define FHH_GT_EVAL_U 2
#endif


template <int B>
__global__ __launch_bounds__(kGcThreads) void k_gt_garble(GcArgs a) {
    __shared__ uint32_t tbl_gc[GcTab::kWords];
    if ((uint64_t)blockIdx.x * kGcThreads >= gc_active(a)) return;   // no tests: skip the table fill
    gc_fill(tbl_gc);
    uint32_t b0, b1;
    GcTab::bases(threadIdx.x & 63, b0, b1);
    constexpr uint32_t R = 1u << B;
    constexpr int NB = R < 4 ? (int)R : 4;   // rows per AES pass and test
    constexpr int U = FHH_GT_GARBLE_U;       // tests per lane per pass
    const uint64_t n = a.G * a.N;
    const uint64_t Npad = (uint64_t)a.nw * 64;
    uint32_t Dk[B][4];   // sigma^k(Delta)
#pragma unroll
    for (int c = 0; c < 4; c++) Dk[0][c] = a.delta[c];
#pragma unroll
    for (int k = 1; k < B; k++) {
#pragma unroll
        for (int c = 0; c < 4; c++) Dk[k][c] = Dk[k - 1][c];
        gf_dbl(Dk[k]);
    }
    const uint64_t n_act = gc_active(a);
    const uint64_t stride = (uint64_t)gridDim.x * kGcThreads;
    // the raw inputs of a lane's U tests (labels E_k, the garbler's bits x_k as a mask)
    auto fetch = [&](uint64_t t0f, uint32_t (&zr)[U][B][4], uint32_t (&xr)[U]) {
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t t = t0f + u * stride;
            const uint64_t tc = t < n_act ? t : (t0f < n_act ? t0f : 0);   // a valid test for padding lanes
            const uint64_t g = tc / a.N;
            const uint32_t i = (uint32_t)(tc - g * a.N);
            xr[u] = 0;
#pragma unroll
            for (int k = 0; k < B; k++) {
                ld_blk(a.ev_labels, g * B + k, Npad, i, zr[u][k]);   // E_k, the labels OT's q
                xr[u] |= plane_bit(a.gb_planes, a.g_off + g, B, k, a.nw, i) << k;
            }
        }
    };
    // (fetching the next pass's inputs during this pass's AES measured +1 %: the kernel waits on LDS
    // issue, not on these loads; profiles/r05/table/ab_gt_prefetch.json)
    for (uint64_t t0 = (uint64_t)blockIdx.x * kGcThreads + threadIdx.x; t0 < n_act; t0 += U * stride) {
        uint32_t zc[U][B][4], xc[U];
        fetch(t0, zc, xc);
        uint32_t S[U][4], col[U];
        uint64_t tt[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t t = t0 + u * stride;
            tt[u] = t;
            const uint64_t tc = t < n_act ? t : t0;
            const uint64_t tw = a.gate_base + a.g_off * a.N + tc;   // the test's index in the whole level
#pragma unroll
            for (int c = 0; c < 4; c++) S[u][c] = 0u;
            col[u] = 0;
#pragma unroll
            for (int k = B - 1; k >= 0; k--) {   // Horner: S = sigma(S) ^ Z_k
                gf_dbl(S[u]);
                const uint32_t xb = (xc[u] >> k) & 1u;
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    const uint32_t z = zc[u][k][c] ^ (xb ? 0u : a.delta[c]);   // Z_k = E_k ^ (x_k ? 0 : Delta)
                    S[u][c] ^= z;
                    if (c == 0) col[u] |= (z & 1u) << k;
                }
            }
            S[u][0] ^= (uint32_t)tw;
            S[u][1] ^= (uint32_t)(tw >> 32);
        }
        uint64_t p0[U], p1[U];
#pragma unroll
        for (uint32_t pass = 0; pass < R / NB; pass++) {
            uint32_t h[U * NB][4];
#pragma unroll
            for (int u = 0; u < U; u++)
#pragma unroll
                for (int j = 0; j < NB; j++) {
                    const uint32_t flip = (pass * NB + j) ^ col[u];   // z_k of the row = bit k of r ^ col
#pragma unroll
                    for (int c = 0; c < 4; c++) {
                        uint32_t w = S[u][c];
#pragma unroll
                        for (int k = 0; k < B; k++) w ^= ((flip >> k) & 1u) ? Dk[k][c] : 0u;
                        h[u * NB + j][c] = w;
                    }
                }
            aes0_mmo_tab<DevOpsX, GcTab, U * NB>(h, tbl_gc, b0, b1);   // cr_hash: pi(K) ^ K
#pragma unroll
            for (int u = 0; u < U; u++) {
                const uint64_t t = tt[u];
                const uint32_t rstar = ~col[u] & (R - 1);   // the row whose z are all 1 (eq = 1)
#pragma unroll
                for (int j = 0; j < NB; j++) {
                    const uint32_t r = pass * NB + j;
                    const uint32_t o = (uint32_t)(r == rstar) ^ a.mask;
                    const uint32_t* hj = h[u * NB + j];
                    const uint64_t hl = (uint64_t)hj[0] | ((uint64_t)hj[1] << 32);
                    if (r == 0) {   // row 0's value pair[o_0] is H(K_0) mod p: it fixes v
                        const uint64_t hv = ot_fe_of_u128(hl, (uint64_t)hj[2] | ((uint64_t)hj[3] << 32));
                        const uint64_t v = o == 0 ? hv : (a.mask ? fe_dec(hv) : fe_inc(hv));
                        p0[u] = v;
                        p1[u] = a.mask ? fe_inc(v) : fe_dec(v);
                        if (t < n_act) a.sh_gb[t] = a.mask ? fe_inc(v) : v;   // r1 = v + mask
                    } else if (t < n_act) {
                        a.gt_msgs[(uint64_t)(r - 1) * n + t] = hl ^ (o ? p1[u] : p0[u]);
                    }
                }
            }
        }
    }
}

template <int B>
__global__ __launch_bounds__(kGcThreads) void k_gt_eval(GcArgs a) {
    __shared__ uint32_t tbl_gc[GcTab::kWords];
    if ((uint64_t)blockIdx.x * kGcThreads >= gc_active(a)) return;
    gc_fill(tbl_gc);
    uint32_t b0, b1;
    GcTab::bases(threadIdx.x & 63, b0, b1);
    const uint64_t n = a.G * a.N;
    const uint64_t Npad = (uint64_t)a.nw * 64;
    const uint64_t n_act = gc_active(a);
    // U tests per lane per pass (U AES blocks in flight)
    constexpr int U = FHH_GT_EVAL_U;
    const uint64_t stride = (uint64_t)gridDim.x * kGcThreads;
    for (uint64_t t0 = (uint64_t)blockIdx.x * kGcThreads + threadIdx.x; t0 < n_act; t0 += U * stride) {
        uint32_t h[U][4], row[U];
        uint64_t tt[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t t = t0 + u * stride;
            tt[u] = t;
            const uint64_t tc = t < n_act ? t : t0;   // a valid test for the padding block
            const uint64_t g = tc / a.N;
            const uint32_t i = (uint32_t)(tc - g * a.N);
            const uint64_t tw = a.gate_base + a.g_off * a.N + tc;
            uint32_t S[4] = {0u, 0u, 0u, 0u}, r = 0;
#pragma unroll
            for (int k = B - 1; k >= 0; k--) {
                uint32_t z[4];
                ld_blk(a.ev_labels, g * B + k, Npad, i, z);   // t_k, z_k's active label
                gf_dbl(S);
#pragma unroll
                for (int c = 0; c < 4; c++) S[c] ^= z[c];
                r |= (z[0] & 1u) << k;
            }
            S[0] ^= (uint32_t)tw;
            S[1] ^= (uint32_t)(tw >> 32);
#pragma unroll
            for (int c = 0; c < 4; c++) h[u][c] = S[c];
            row[u] = r;
        }
        aes0_mmo_tab<DevOpsX, GcTab, U>(h, tbl_gc, b0, b1);
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint64_t t = tt[u];
            if (t >= n_act) continue;
            const uint64_t hl = (uint64_t)h[u][0] | ((uint64_t)h[u][1] << 32);
            a.sh_ev[t] = row[u] ? (hl ^ a.gt_msgs[(uint64_t)(row[u] - 1) * n + t])
                                : ot_fe_of_u128(hl, (uint64_t)h[u][2] | ((uint64_t)h[u][3] << 32));
        }
    }
}

// ---- r06: the garbled table on the labels OT's tile-major matrices ------------------------------
// k_gt_garble / k_gt_eval read one row-major 16-B label per (test, bit), which k_ot_rows_out produced
// from the tile-major Q / T the OT expands write: 32 B of HBM per OT and party (read + write) and a
// launch, ~12 % of the 1M protocol crawl. Here the table kernels read Q / T tile-major
// themselves. With the OT index (g b + k) Npad + i and Npad a multiple of 512 (the level loop pads the
// share planes to 8-word rows), test i's b labels sit at the same position p = i % 512 of the b tiles
// ((g b + k) Npad / 512 + i / 512), so a wave takes one 512-test tile: its lanes load the b tiles' row
// words (whole 128-B lines), fold the labels into the tests' row keys in the row domain (gt_tile_rows), make
// ONE in-register transpose (transpose32) and deal the keys to the lanes through 2 KiB of LDS, as the OT
// hashes do (ot_tile_load / ot_tile_round) — no label is stored. Lane l takes tests p = 256 u + 32 (l >> 3) +
// 8 r + (l & 7) (u < 2, exchange round r < 4): 8 consecutive lanes hold 8 consecutive tests, so the
// messages and node values move in 64-B runs. Each round's two tests go to the AES at once (garbler: the
// 2^b rows of one test per pass, as k_gt_garble; evaluator: two rounds' 4 tests per pass). Identical
// outputs to k_ot_rows_out + k_gt_garble / k_gt_eval (oracle orc_gt_garble / orc_gt_eval).
constexpr int kGtWaves = kGcThreads / 64;
constexpr uint32_t kGtTileWords = 128 * 16;   // one 512-OT tile of Q / T: 128 rows x 16 words

// exchange round r (x[0..7] = the tile's x[8 r .. 8 r + 7]): lane l receives OTs 32 qq + 8 r + (l & 7),
// qq = (l >> 3) + 8 u, u < 2; then x moves down by 8 (a rolled round loop keeps x in registers). Stage
// word of (kk, writer lane l') = 64 kk + (l' ^ 8 kk): the writes are lane-linear per kk, and the 16 lanes
// of a ds_read_b128 group hit 16 distinct bank quads (4 qq ^ 8 kk = 8 (kk ^ (qq >> 1)) + 4 (qq & 1)).
__device__ __forceinline__ void gt_tile_round(uint32_t* st, uint32_t (&x)[32], uint32_t lane, uint32_t (&o)[2][4]) {
#pragma unroll
    for (int kk = 0; kk < 8; kk++) st[64 * kk + (lane ^ (8 * kk))] = x[kk];
    __builtin_amdgcn_wave_barrier();
    const uint32_t kk = lane & 7;
#pragma unroll
    for (int u = 0; u < 2; u++) {
        const uint32_t qq = (lane >> 3) + 8 * u;
        const uint4 v = *reinterpret_cast<const uint4*>(st + 64 * kk + ((4 * qq) ^ (8 * kk)));
        o[u][0] = v.x;
        o[u][1] = v.y;
        o[u][2] = v.z;
        o[u][3] = v.w;
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < 24; i++) x[i] = x[i + 8];
}

// the wave's sum of lo / hi 32-bit limbs of its live values, added to node_partials[child][k0], [k0 + 1]
__device__ __forceinline__ void gt_add_partials(uint64_t* partials, uint64_t child, int k0, uint64_t lo, uint64_t hi,
                                                uint32_t lane) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        lo += __shfl_xor(lo, off, 64);
        hi += __shfl_xor(hi, off, 64);
    }
    if (lane == 0) {
        atomicAdd(reinterpret_cast<unsigned long long*>(partials + child * 4 + k0), (unsigned long long)lo);
        atomicAdd(reinterpret_cast<unsigned long long*>(partials + child * 4 + k0 + 1), (unsigned long long)hi);
    }
}

// the lane's test of round r, u within its 512-test tile
__device__ __forceinline__ uint32_t gt_tile_test(uint32_t lane, int r, int u) {
    return 256 * u + 32 * (lane >> 3) + 8 * r + (lane & 7);
}

// The tile's raw row keys, S = e_0 ^ sigma(e_1) over the labels OT's matrix (Horner at b = 2; b = 1:
// S = e_0), built in the ROW domain before the one transpose: row r of sigma(e) is row r - 1 of e, plus
// row 127 into rows 0, 1, 2, 7 (x^128 = x^7 + x^2 + x + 1; row r = bit r of the LE u128 label), so lane
// (q, rg) loads e_1's rows shifted by one — its first load is row 32 rg - 1, or for rg = 0 row 127, which
// is also the reduction term. One transpose per tile instead of one per label. (The garbler's labels are
// Z_k = E_k ^ (x_k ? 0 : Delta); being linear, its Delta terms are added per test after the exchange.)
// On return x[k] = word rg of S for test 32 q + k, lane (q, rg) = (lane >> 2, lane & 3).
template <int B>
__device__ __forceinline__ void gt_tile_rows(const GcArgs& a, uint64_t g, uint32_t iw, uint32_t Npt, uint32_t lane,
                                             uint32_t (&x)[32]) {
    static_assert(B == 1 || B == 2, "gt_tile_rows: b <= 2");
    const uint32_t q = lane >> 2, rg = lane & 3;
    const uint32_t* t0 = reinterpret_cast<const uint32_t*>(a.ev_labels) + (((uint64_t)g * B) * Npt + iw) * kGtTileWords + q;
#pragma unroll
    for (int i = 0; i < 32; i++) x[i] = __builtin_nontemporal_load(t0 + (32 * rg + i) * 16);
    if constexpr (B == 2) {
        const uint32_t* t1 = t0 + (uint64_t)Npt * kGtTileWords;   // bit 1's tile
        const uint32_t y0 = __builtin_nontemporal_load(t1 + (rg ? 32 * rg - 1 : 127) * 16);
        x[0] ^= y0;
#pragma unroll
        for (int i = 1; i < 32; i++) x[i] ^= __builtin_nontemporal_load(t1 + (32 * rg + i - 1) * 16);
        if (rg == 0) {   // e_1's row 127: the reduction into rows 1, 2, 7 (row 0 took it above)
            x[1] ^= y0;
            x[2] ^= y0;
            x[7] ^= y0;
        }
    }
    transpose32(x);
}

// the colours of the lane's tests (r, u): bit 8 r + (lane & 7) of cw[u] = row 0 word (lane >> 3) + 8 u of
// the tile, packed as the test's row index bits (b = 2: colour of z_1 << 1 | colour of z_0)
template <int B>
__device__ __forceinline__ void gt_tile_colours(const GcArgs& a, uint64_t g, uint32_t iw, uint32_t Npt, uint32_t lane,
                                                uint32_t (&cw)[B][2]) {
    const uint32_t* lab = reinterpret_cast<const uint32_t*>(a.ev_labels);
#pragma unroll
    for (int k = 0; k < B; k++)
#pragma unroll
        for (int u = 0; u < 2; u++)   // row 0 (cached: the tile was just read)
            cw[k][u] = lab[(((uint64_t)g * B + k) * Npt + iw) * kGtTileWords + (lane >> 3) + 8 * u];
}

template <int B>
__device__ __forceinline__ uint32_t gt_row_of(const uint32_t (&cw)[B][2], int r, int u, uint32_t lane) {
    const uint32_t sh = 8 * r + (lane & 7);
    uint32_t row = 0;
#pragma unroll
    for (int k = 0; k < B; k++) row |= ((cw[k][u] >> sh) & 1u) << k;
    return row;
}

// the lane's 8 tests' row keys S[j] (j = 2 r + u, without the tweak) and row indices (4 bits per test, test
// j at bits 4 j of col): gt_tile_rows, then the 4 exchange rounds; each round's two keys rotate to the end
// of S (a rolled round loop keeps S and x in registers), so after 4 rounds S is in order. The tile's words
// are dead before the AES phase starts (live beside the AES they spilled the 128-VGPR budget).
template <int B, bool GARBLER>
__device__ __forceinline__ void gt_tile_keys(const GcArgs& a, uint64_t g, uint32_t iw, uint32_t Npt, uint32_t* st,
                                             uint32_t lane, const uint32_t (&Dk)[B][4], uint32_t (&S)[8][4],
                                             uint32_t& col) {
    uint32_t x[32], cw[B][2], nx[B][2];
    gt_tile_rows<B>(a, g, iw, Npt, lane, x);
    gt_tile_colours<B>(a, g, iw, Npt, lane, cw);
    if constexpr (GARBLER) {   // ~x_k of the lane's tests (plane words (lane >> 3) + 8 u of the tile)
#pragma unroll
        for (int k = 0; k < B; k++)
#pragma unroll
            for (int u = 0; u < 2; u++) {
                nx[k][u] = ~reinterpret_cast<const uint32_t*>(a.gb_planes)[((a.g_off + g) * B + k) * (2 * (uint64_t)a.nw) +
                                                                          16 * iw + (lane >> 3) + 8 * u];
                cw[k][u] ^= nx[k][u];   // Z_k's colour: Delta's colour bit is 1
            }
    }
    col = 0;
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
        for (int u = 0; u < 2; u++) col |= gt_row_of<B>(cw, r, u, lane) << (4 * (2 * r + u));
#pragma unroll 1
    for (int r = 0; r < 4; r++) {
        uint32_t o[2][4];
        gt_tile_round(st, x, lane, o);
        if constexpr (GARBLER) {   // S ^= XOR_k (x_k ? 0 : sigma^k(Delta))
#pragma unroll
            for (int u = 0; u < 2; u++)
#pragma unroll
                for (int k = 0; k < B; k++) {
                    const uint32_t f = (nx[k][u] >> (8 * r + (lane & 7))) & 1u;
#pragma unroll
                    for (int c = 0; c < 4; c++) o[u][c] ^= f ? Dk[k][c] : 0u;
                }
        }
#pragma unroll
        for (int j = 0; j < 6; j++)
#pragma unroll
            for (int c = 0; c < 4; c++) S[j][c] = S[j + 2][c];
#pragma unroll
        for (int c = 0; c < 4; c++) {
            S[6][c] = o[0][c];
            S[7][c] = o[1][c];
        }
    }
}

// (b <= 2, the d = 1 tests of the metric's configuration; d = 2 keeps k_ot_rows_out + the row-major kernels)
template <int B, bool RING = false>   // RING: GcArgs::ring32 (a separate instantiation: no FE code beside it)
__global__ __launch_bounds__(kGcThreads) void k_gt_garble_tm(GcArgs a) {
    static_assert(B <= 2, "the tile-major garbler takes b <= 2");
    __shared__ uint32_t tbl_gc[GcTab::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t stage[kGtWaves][512];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t n_act = gc_active(a);
    const uint32_t Npt = a.nw / 8;   // 512-test tiles per group
    const uint64_t tiles = (n_act / a.N) * Npt;
    if ((uint64_t)blockIdx.x * kGtWaves >= tiles) return;   // no tiles for this workgroup: skip the table fill
    gc_fill(tbl_gc);
    uint32_t b0, b1;
    GcTab::bases(lane, b0, b1);
    constexpr uint32_t R = 1u << B;   // rows per test: one AES pass
    const uint64_t n = a.G * a.N;
    uint32_t Dk[B][4];   // sigma^k(Delta)
#pragma unroll
    for (int c = 0; c < 4; c++) Dk[0][c] = a.delta[c];
#pragma unroll
    for (int k = 1; k < B; k++) {
#pragma unroll
        for (int c = 0; c < 4; c++) Dk[k][c] = Dk[k - 1][c];
        gf_dbl(Dk[k]);
    }
    for (uint64_t wt = (uint64_t)blockIdx.x * kGtWaves + wv; wt < tiles; wt += (uint64_t)gridDim.x * kGtWaves) {
        const uint64_t g = wt / Npt;
        const uint32_t iw = (uint32_t)(wt - g * Npt);
        uint32_t S[8][4], col;
        gt_tile_keys<B, true>(a, g, iw, Npt, stage[wv], lane, Dk, S, col);
        uint64_t acc_lo = 0, acc_hi = 0;   // node_partials: this lane's live node values' limbs
#pragma unroll 1
        for (int j = 0; j < 8; j++) {   // test j = (r, u) = (j >> 1, j & 1); S and col rotate by one test
            const uint32_t i = 512 * iw + gt_tile_test(lane, j >> 1, j & 1);
            const bool live = i < a.N;
            const uint64_t t = g * a.N + i;
            const uint64_t tw = a.gate_base + a.g_off * a.N + t;   // the test's index in the whole level
            const uint32_t K[4] = {S[0][0] ^ (uint32_t)tw, S[0][1] ^ (uint32_t)(tw >> 32), S[0][2], S[0][3]};
            const uint32_t cl = col & (R - 1);
            const uint32_t rstar = ~cl & (R - 1);   // the row whose z are all 1 (eq = 1)
            uint32_t h[R][4];
#pragma unroll
            for (uint32_t q = 0; q < R; q++) {
                const uint32_t flip = q ^ cl;   // z_k of the row = bit k of r ^ col
#pragma unroll
                for (int c = 0; c < 4; c++) {
                    uint32_t w = K[c];
#pragma unroll
                    for (int k = 0; k < B; k++) w ^= ((flip >> k) & 1u) ? Dk[k][c] : 0u;
                    h[q][c] = w;
                }
            }
            aes0_mmo_tab<DevOpsX, GcTab, R>(h, tbl_gc, b0, b1);   // cr_hash: pi(K) ^ K
            uint64_t p0 = 0, p1 = 0;
#pragma unroll
            for (uint32_t q = 0; q < R; q++) {
                const uint32_t o_r = (uint32_t)(q == rstar) ^ a.mask;
                const uint64_t hl = (uint64_t)h[q][0] | ((uint64_t)h[q][1] << 32);
                // r06: the same table over Z_2^32 (lo32 of the hash, 4-B messages). RING = false folds the branch
                // away (the FE form alone, no spill); RING = true keeps it a runtime test beside the FE code:
                // compiled that way the Z_2^32 garbler ran ~10 % faster than as a Z_2^32-only body
                // (profiles/r06/ring32/)
                if (RING && a.ring32) {
                    if (q == 0) {
                        const uint32_t h32 = h[0][0];
                        const uint32_t v = o_r == 0 ? h32 : (a.mask ? h32 - 1u : h32 + 1u);
                        p0 = v;
                        p1 = (uint32_t)(a.mask ? v + 1u : v - 1u);
                        const uint32_t r1 = a.mask ? v + 1u : v;   // r1 = v + mask
                        if (live && a.node_partials) acc_lo += r1;
                        else if (live) a.sh_gb[t] = r1;
                    } else if (live) {
                        reinterpret_cast<uint32_t*>(a.gt_msgs)[(uint64_t)(q - 1) * n + t] =
                            h[q][0] ^ (uint32_t)(o_r ? p1 : p0);
                    }
                    continue;
                }
                if (q == 0) {   // row 0's value pair[o_0] is H(K_0) mod p: it fixes v
                    const uint64_t hv = ot_fe_of_u128(hl, (uint64_t)h[q][2] | ((uint64_t)h[q][3] << 32));
                    const uint64_t v = o_r == 0 ? hv : (a.mask ? fe_dec(hv) : fe_inc(hv));
                    p0 = v;
                    p1 = a.mask ? fe_inc(v) : fe_dec(v);
                    const uint64_t r1 = a.mask ? fe_inc(v) : v;   // r1 = v + mask
                    if (live && a.node_partials) {
                        acc_lo += r1 & 0xFFFFFFFFull;
                        acc_hi += r1 >> 32;
                    } else if (live) {
                        a.sh_gb[t] = r1;
                    }
                } else if (live) {
                    a.gt_msgs[(uint64_t)(q - 1) * n + t] = hl ^ (o_r ? p1 : p0);
                }
            }
#pragma unroll
            for (int jj = 0; jj < 7; jj++)
#pragma unroll
                for (int c = 0; c < 4; c++) S[jj][c] = S[jj + 1][c];
            col >>= 4;
        }
        if (a.node_partials) gt_add_partials(a.node_partials, a.node_off + a.g_off + g, 0, acc_lo, acc_hi, lane);
    }
}

// (the Z_2^32 form is a runtime branch here: as its own instantiation the evaluator ran ~20 % slower,
// profiles/r06/ring32/)
template <int B>
__global__ __launch_bounds__(kGcThreads) void k_gt_eval_tm(GcArgs a) {
    static_assert(B <= 2, "the tile-major evaluator takes b <= 2");
    __shared__ uint32_t tbl_gc[GcTab::kWords];
    __shared__ __attribute__((aligned(16))) uint32_t stage[kGtWaves][512];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t n_act = gc_active(a);
    const uint32_t Npt = a.nw / 8;
    const uint64_t tiles = (n_act / a.N) * Npt;
    if ((uint64_t)blockIdx.x * kGtWaves >= tiles) return;
    gc_fill(tbl_gc);
    uint32_t b0, b1;
    GcTab::bases(lane, b0, b1);
    const uint64_t n = a.G * a.N;
    for (uint64_t wt = (uint64_t)blockIdx.x * kGtWaves + wv; wt < tiles; wt += (uint64_t)gridDim.x * kGtWaves) {
        const uint64_t g = wt / Npt;
        const uint32_t iw = (uint32_t)(wt - g * Npt);
        uint32_t S[8][4], col;
        const uint32_t nod[B][4] = {};
        gt_tile_keys<B, false>(a, g, iw, Npt, stage[wv], lane, nod, S, col);
        uint64_t acc_lo = 0, acc_hi = 0;
#pragma unroll 1
        for (int r = 0; r < 4; r++) {   // round r's 2 tests: 2 AES blocks in lockstep (4 spilled 6 VGPRs)
            uint32_t h[2][4];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const uint32_t i = 512 * iw + gt_tile_test(lane, r, u);
                const uint64_t tw = a.gate_base + a.g_off * a.N + g * a.N + i;
                h[u][0] = S[u][0] ^ (uint32_t)tw;
                h[u][1] = S[u][1] ^ (uint32_t)(tw >> 32);
                h[u][2] = S[u][2];
                h[u][3] = S[u][3];
            }
            aes0_mmo_tab<DevOpsX, GcTab, 2>(h, tbl_gc, b0, b1);
            // (the row messages are loaded after the AES: r05 measured the early load neutral,
            // profiles/r05/table/ab_gt_eval_msg.json)
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const uint32_t i = 512 * iw + gt_tile_test(lane, r, u);
                if (i >= a.N) continue;
                const uint64_t t = g * a.N + i;
                const uint32_t row = (col >> (4 * u)) & 0xFu;
                const uint64_t hl = (uint64_t)h[u][0] | ((uint64_t)h[u][1] << 32);
                uint64_t val;
                if (a.ring32)   // r06: Z_2^32 shares, 4-B messages
                    val = row ? (h[u][0] ^ reinterpret_cast<const uint32_t*>(a.gt_msgs)[(uint64_t)(row - 1) * n + t]) : h[u][0];
                else
                    val = row ? (hl ^ a.gt_msgs[(uint64_t)(row - 1) * n + t])
                              : ot_fe_of_u128(hl, (uint64_t)h[u][2] | ((uint64_t)h[u][3] << 32));
                if (a.node_partials) {
                    acc_lo += val & 0xFFFFFFFFull;
                    acc_hi += val >> 32;
                } else {
                    a.sh_ev[t] = val;
                }
            }
#pragma unroll
            for (int jj = 0; jj < 6; jj++)
#pragma unroll
                for (int c = 0; c < 4; c++) S[jj][c] = S[jj + 2][c];
            col >>= 8;
        }
        if (a.node_partials) gt_add_partials(a.node_partials, a.node_off + a.g_off + g, 2, acc_lo, acc_hi, lane);
    }
}

template <int B>
static hipError_t gt_launch(const GcArgs& a, bool garble, hipStream_t stream) {
    int dev = 0, cus = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    const uint64_t n = a.G * a.N;
    if constexpr (B <= 2) if (a.lab_tm) {   // r06: one wave per 512-test tile, one 160 KiB workgroup per CU
        const uint64_t tiles = a.G * (a.nw / 8), need = (tiles + kGtWaves - 1) / kGtWaves;
        const int grid = (int)(need < (uint64_t)cus ? (need ? need : 1) : (uint64_t)cus);
        if (garble && a.ring32) hipLaunchKernelGGL((k_gt_garble_tm<B, true>), dim3(grid), dim3(kGcThreads), 0, stream, a);
        else if (garble) hipLaunchKernelGGL((k_gt_garble_tm<B, false>), dim3(grid), dim3(kGcThreads), 0, stream, a);
        else hipLaunchKernelGGL(k_gt_eval_tm<B>, dim3(grid), dim3(kGcThreads), 0, stream, a);
        return hipGetLastError();
    }
    const uint64_t need = (n + kGcThreads - 1) / kGcThreads;
    const int grid = (int)(need < (uint64_t)cus * 8 ? (need ? need : 1) : (uint64_t)cus * 8);
    if (garble) hipLaunchKernelGGL(k_gt_garble<B>, dim3(grid), dim3(kGcThreads), 0, stream, a);
    else hipLaunchKernelGGL(k_gt_eval<B>, dim3(grid), dim3(kGcThreads), 0, stream, a);
    return hipGetLastError();
}

static hipError_t gt_dispatch(const GcArgs& a, bool garble, hipStream_t stream) {
    if (a.G * a.N == 0) return hipSuccess;
    if (!a.gt_msgs || (!(garble ? a.sh_gb : a.sh_ev) && !(a.lab_tm && a.node_partials)) || !a.ev_labels)
        return hipErrorInvalidValue;
    // r06 tile-major labels: 512-test tiles per group, b <= 2 (gt_tm_bits)
    if (a.lab_tm && (a.nw % 8 != 0 || a.bits > (uint32_t)kGtTmMaxBits)) return hipErrorInvalidValue;
    if (a.ring32 && !a.lab_tm) return hipErrorInvalidValue;   // Z_2^32: the tile-major kernels only
    switch (a.bits) {
        case 1: return gt_launch<1>(a, garble, stream);
        case 2: return gt_launch<2>(a, garble, stream);
        case 3: return gt_launch<3>(a, garble, stream);
        case 4: return gt_launch<4>(a, garble, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_gt_garble(const GcArgs& a, hipStream_t stream) { return gt_dispatch(a, true, stream); }

hipError_t launch_gt_eval(const GcArgs& a, hipStream_t stream) { return gt_dispatch(a, false, stream); }

template <int B>
static hipError_t gc_launch(const GcArgs& a, bool garble, hipStream_t stream) {
    int dev = 0, cus = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e != hipSuccess) return e;
    const uint64_t n = a.G * a.N;
    const uint64_t need = (n + kGcThreads - 1) / kGcThreads;
    // 8 workgroups per CU (one resident per CU, each filling its tables once, measured -5.6 % for
    // evaluate at configs[1] but +3.2 % for evaluate and +0.7 % for the whole GC + OT crawl at 1M
    // clients, alternated twice; r03)
    const int grid = (int)(need < (uint64_t)cus * 8 ? (need ? need : 1) : (uint64_t)cus * 8);
    if (garble && a.ev_ot) hipLaunchKernelGGL(k_gc_garble_cot<B>, dim3(grid), dim3(kGcThreads), 0, stream, a);
    else if (garble) hipLaunchKernelGGL(k_gc_garble<B>, dim3(grid), dim3(kGcThreads), 0, stream, a);
    else if (a.ev_ot) hipLaunchKernelGGL((k_gc_eval<B, true>), dim3(grid), dim3(kGcThreads), 0, stream, a);
    else hipLaunchKernelGGL((k_gc_eval<B, false>), dim3(grid), dim3(kGcThreads), 0, stream, a);
    return hipGetLastError();
}

static hipError_t gc_dispatch(const GcArgs& a, bool garble, hipStream_t stream) {
    if (a.G * a.N == 0) return hipSuccess;
    switch (a.bits) {
        case 1: return gc_launch<1>(a, garble, stream);
        case 2: return gc_launch<2>(a, garble, stream);
        case 3: return gc_launch<3>(a, garble, stream);
        case 4: return gc_launch<4>(a, garble, stream);
        case 5: return gc_launch<5>(a, garble, stream);
        case 6: return gc_launch<6>(a, garble, stream);
        case 7: return gc_launch<7>(a, garble, stream);
        case 8: return gc_launch<8>(a, garble, stream);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_gc_garble(const GcArgs& a, hipStream_t stream) { return gc_dispatch(a, true, stream); }

hipError_t launch_gc_eval(const GcArgs& a, hipStream_t stream) { return gc_dispatch(a, false, stream); }

}  // namespace fhh
