// OT extension on the GPU (the OT half): IKNP in the ALSZ form, the protocol
// of `ocelot::ot::{AlszSender, AlszReceiver}` that the reference runs for the evaluator's input
// labels (equalitytest.rs:67-82) and for the FE share conversion (collect.rs:437-471). ocelot is
// not vendored; the published scheme is restated (oracle/fhh_oracle.c orc_ot_extend):
//
//   receiver (choice bits r):  t_i = G(k_i^0),  u_i = t_i ^ G(k_i^1) ^ r        i < 128
//   sender   (base choice s):  q_i = G(k_i^{s_i}) ^ s_i u_i  =>  q_j = t_j ^ r_j s (columns)
//   sender:    y_j^b = x_j^b ^ H(j, q_j ^ b s)        receiver:  x_j^{r_j} = y_j^{r_j} ^ H(j, t_j)
//
// G = ChaCha12 under the row key since r06 (one 64-B block -> OTs 512 j .. 512 j + 511 of a row; AES-128-CTR,
// block c -> OTs 128 c .. 128 c + 127, in r01-r05 as ocelot's AesRng), H(j, x) = scuttlebutt's
// AesHash::cr_hash(j, x) = pi(x) ^ x (the correlation-robust hash ocelot's ALSZ applies to q_j,
// q_j ^ s and t_j; j is not an input), pi = AES-128 under the zero key (as fhh_gc.hip): the
// fixed-key AES + feed-forward of k_expand (aes0_mmo_tab, round keys as immediates). The 128 base OTs are
// ideal (the host hands the sender k_i^{s_i}).
//
//   k_ot_recv_expand_cc / k_ot_send_expand_cc  one lane per (row, 512-OT tile): 2 / 1 ChaCha12 blocks
//   k_ot_send_hash_rows / k_ot_recv_hash_rows  one wave per 512 OTs, the 128 x 512 bit tile of T / Q
//                                              transposed in registers + LDS: 2 / 1 cr_hash per OT
#include "fhh_internal.h"

#include <atomic>

#include "aes_keyed.h"
#include "bitslice.h"
#include "cot_fe.h"


namespace fhh {

__constant__ WordTable c_T0_ot = T0;
using OtTab = Tab4T32<DevOpsX>;

__device__ __forceinline__ void ot_fill(uint32_t* tbl) {
    for (int i = threadIdx.x; i < OtTab::kWords; i += blockDim.x) tbl[i] = OtTab::word(c_T0_ot.v, i);
    __syncthreads();
}

// OTs to run: m, or inside the level loop per_group * min(groups, ctl->C - g_off)
__device__ __forceinline__ uint64_t ot_active(const OtArgs& a) {
    if (!a.ctl) return a.m;
    if (a.ctl->abort) return 0;
    const uint64_t C = a.ctl->C;
    if (C <= a.g_off) return 0;
    const uint64_t v = a.per_group * (C - a.g_off);   // the chunk's groups from g_off on
    return v < a.m ? v : a.m;
}

// T and Q (internal to the parties, never on the wire) are stored tile-major: a hash's 512-OT tile
// (4 blocks x 128 rows = 8 KiB) is one contiguous run, row r at words 16 r .. 16 r + 15, so its 32
// row loads per lane read whole 128 B lines (rows r, r + 1) instead of 64 B from each of 128 rows
// mp / 8 bytes apart. U, the receiver's message to the sender, was in row form [128][mp / 128] until r06;
// the ChaCha expands write (and read) it tile-major as well (the transcript exports convert it back).
// Same-box A/B at configs[1] (profiles/r04/ab_ot_tmaj/): receive hash -11 %, send hash -3 %, the
// sender's expand +12 % (one row per wave: its Q stores are 64 B runs), all kernels -0.9 / -1.6 %;
// T alone tile-major -0.2 %; 8-block (128 B per row) runs: hashes as before.
__device__ __forceinline__ uint64_t ot_tmaj(uint32_t i, uint64_t c) {
    return (c >> 2) * 512 + (uint64_t)i * 4 + (c & 3);
}

// ---- r06: the row PRG G = ChaCha12 (VALU only) ------------------------------------------------
// The expands were T-table AES-CTR under the row keys (r01-r05: k_ot_expand<true> 2 blocks per OT
// and row, k_ot_send_expand_pair 1, both bound by LDS issue beside the garbled table's AES). G is now
// the ChaCha block function with 12 rounds (rand_chacha's StdRng; fhh_oracle.c orc_chacha_block /
// ot_prg_block, pinned for 20 rounds against RFC 8439 and OpenSSL), key = row seed || row seed, 64-bit
// block counter = ctr_off / 4 + tile, nonce 0: one 64-byte block is exactly one row of a 512-OT tile of
// the tile-major T / Q (ot_tmaj), so a lane stores 64 contiguous bytes. 4 adds + 4 xors + 4 rotates
// (v_alignbit) per quarter round, ~600 VALU per 64 B against ~250 VALU + 144-160 ds_read_b32 per 16 B of
// AES: no LDS at all, so the expands leave the LDS to the table kernels' cr_hash. The row seed is words
// 0..3 of the row's key schedule in rk (the schedules the AES form used; unchanged on the host).
constexpr int kOtChachaRounds = 12;

#ifndef FHH_CC_PERM
#define FHH_CC_PERM 0   // A/B knob: 1 = the byte rotations (16, 8) as v_perm_b32
#endif
#ifndef FHH_CC_TPI
#define FHH_CC_TPI 2    // tiles per receiver work item (2 TPI ChaCha blocks per lane in lockstep; 1: +4 %, profiles/r06/ab_ot_cc/)
#endif
#ifndef FHH_CC_THREADS
#define FHH_CC_THREADS 256
#endif
__device__ __forceinline__ uint32_t cc_rotl(uint32_t x, int n) {
    if (FHH_CC_PERM && n == 16) return __builtin_amdgcn_perm(x, x, 0x01000302u);
    if (FHH_CC_PERM && n == 8) return __builtin_amdgcn_perm(x, x, 0x02010003u);
    return __builtin_amdgcn_alignbit(x, x, 32 - n);
}

__device__ __forceinline__ void cc_qr(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
    a += b; d ^= a; d = cc_rotl(d, 16);
    c += d; b ^= c; b = cc_rotl(b, 12);
    a += b; d ^= a; d = cc_rotl(d, 8);
    c += d; b ^= c; b = cc_rotl(b, 7);
}

// NB independent ChaCha blocks (key k[q] = seed || seed, counter ctr[q], nonce 0) in lockstep
template <int NB>
__device__ __forceinline__ void cc_blocks(const uint32_t (&k)[NB][4], const uint64_t (&ctr)[NB], uint32_t (&x)[NB][16]) {
#pragma unroll
    for (int q = 0; q < NB; q++) {
        x[q][0] = 0x61707865u; x[q][1] = 0x3320646eu; x[q][2] = 0x79622d32u; x[q][3] = 0x6b206574u;
#pragma unroll
        for (int w = 0; w < 4; w++) x[q][4 + w] = x[q][8 + w] = k[q][w];
        x[q][12] = (uint32_t)ctr[q];
        x[q][13] = (uint32_t)(ctr[q] >> 32);
        x[q][14] = 0u;
        x[q][15] = 0u;
    }
#pragma unroll
    for (int r = 0; r < kOtChachaRounds; r += 2) {
#pragma unroll
        for (int q = 0; q < NB; q++) {
            cc_qr(x[q][0], x[q][4], x[q][8], x[q][12]);
            cc_qr(x[q][1], x[q][5], x[q][9], x[q][13]);
            cc_qr(x[q][2], x[q][6], x[q][10], x[q][14]);
            cc_qr(x[q][3], x[q][7], x[q][11], x[q][15]);
            cc_qr(x[q][0], x[q][5], x[q][10], x[q][15]);
            cc_qr(x[q][1], x[q][6], x[q][11], x[q][12]);
            cc_qr(x[q][2], x[q][7], x[q][8], x[q][13]);
            cc_qr(x[q][3], x[q][4], x[q][9], x[q][14]);
        }
    }
#pragma unroll
    for (int q = 0; q < NB; q++) {   // feed-forward
        x[q][0] += 0x61707865u; x[q][1] += 0x3320646eu; x[q][2] += 0x79622d32u; x[q][3] += 0x6b206574u;
#pragma unroll
        for (int w = 0; w < 4; w++) {
            x[q][4 + w] += k[q][w];
            x[q][8 + w] += k[q][w];
        }
        x[q][12] += (uint32_t)ctr[q];
        x[q][13] += (uint32_t)(ctr[q] >> 32);
    }
}

__device__ __forceinline__ void ld_seed(const uint32_t* rk, uint32_t row, uint32_t (&k)[4]) {
    const uint4 v = *reinterpret_cast<const uint4*>(rk + (size_t)row * 44);   // words 0..3 of the schedule = the key
    k[0] = v.x;
    k[1] = v.y;
    k[2] = v.z;
    k[3] = v.w;
}

constexpr int kOtCcThreads = FHH_CC_THREADS;
constexpr int kOtCcWaves = kOtCcThreads / 64;
constexpr int kOtCcRowWords = 20;   // LDS words per staged 64-B row (80 B: 16 lanes of a b128 access hit distinct banks)

// A wave's 64 rows x 64 B of one tile — rows 64 h .. 64 h + 63 of tile j, one contiguous 4 KiB run of a
// tile-major matrix (ot_tmaj) — moved through LDS so that every store instruction writes 1 KiB of whole
// 128-B lines: lane l stages its row at 80 l, then store k writes bytes 1024 k + 16 l (row 16 k + l / 4,
// chunk l % 4). Lane-row stores (16 B into each of 64 rows per instruction) left partial lines in the L2
// and cost 2.2-2.5x the algorithmic bytes in HBM writes (WRITE_SIZE, profiles/r06/ot_pmc/).
typedef uint32_t cc_v4 __attribute__((ext_vector_type(4)));   // for the nontemporal builtins

__device__ __forceinline__ void cc_store_rows(uint32_t* st, uint32_t lane, const uint32_t (&v)[16], uint4* run) {
#pragma unroll
    for (int w = 0; w < 4; w++)
        *reinterpret_cast<uint4*>(st + kOtCcRowWords * lane + 4 * w) = make_uint4(v[4 * w], v[4 * w + 1], v[4 * w + 2], v[4 * w + 3]);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t r = 16 * k + (lane >> 2), w = lane & 3;
        __builtin_nontemporal_store(*reinterpret_cast<const cc_v4*>(st + kOtCcRowWords * r + 4 * w),
                                    reinterpret_cast<cc_v4*>(run + 64 * k + lane));
    }
    __builtin_amdgcn_wave_barrier();   // the reads precede the next item's stage writes
}

// the inverse: the 4 KiB run read by whole lines (load k = bytes 1024 k + 16 l) and dealt to the lanes by row
__device__ __forceinline__ void cc_load_rows(uint32_t* st, uint32_t lane, const uint4* run, uint32_t (&v)[16]) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t r = 16 * k + (lane >> 2), w = lane & 3;
        *reinterpret_cast<cc_v4*>(st + kOtCcRowWords * r + 4 * w) =
            __builtin_nontemporal_load(reinterpret_cast<const cc_v4*>(run + 64 * k + lane));
    }
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const uint4 x = *reinterpret_cast<const uint4*>(st + kOtCcRowWords * lane + 4 * w);
        v[4 * w] = x.x;
        v[4 * w + 1] = x.y;
        v[4 * w + 2] = x.z;
        v[4 * w + 3] = x.w;
    }
    __builtin_amdgcn_wave_barrier();
}

// The receiver: work item = (512-OT tile j, row half h); lane l = row i = 64 h + l computes G(k_i^0) and
// G(k_i^1) for tile j (2 ChaCha blocks in lockstep); T = G(k_i^0) and U = T ^ G(k_i^1) ^ r are both stored
// tile-major (r06: U, the message to the sender, in the same layout as T — row i's 64 B of tile j at
// ot_tmaj(i, 4 j)), each as the wave's contiguous 4 KiB run. The tile's choice words r are the same for
// every lane (a broadcast load); 128-OT blocks past the active OTs get no choice bits.
__global__ __launch_bounds__(kOtCcThreads) void k_ot_recv_expand_cc(OtArgs a) {
    constexpr int TPI = FHH_CC_TPI;
    __shared__ __attribute__((aligned(16))) uint32_t stage[kOtCcWaves][64 * kOtCcRowWords];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t nblk_act = (ot_active(a) + 127) / 128;
    const uint64_t tiles = (nblk_act + 3) / 4;
    const uint64_t items = 2 * ((tiles + TPI - 1) / TPI);
    const uint64_t nwaves = (uint64_t)gridDim.x * kOtCcWaves;
    for (uint64_t it = (uint64_t)blockIdx.x * kOtCcWaves + wv; it < items; it += nwaves) {
        const uint64_t j0 = TPI * (it >> 1);
        const uint32_t h = (uint32_t)(it & 1), i = 64 * h + lane;
        uint32_t k[2 * TPI][4];
        ld_seed(a.rk, i, k[0]);
        ld_seed(a.rk, 128 + i, k[1]);
        uint64_t ctr[2 * TPI];
#pragma unroll
        for (int q = 0; q < TPI; q++) {
#pragma unroll
            for (int w = 0; w < 4; w++) {
                k[2 * q][w] = k[0][w];
                k[2 * q + 1][w] = k[1][w];
            }
            ctr[2 * q] = ctr[2 * q + 1] = a.ctr_off / 4 + j0 + q;
        }
        uint32_t g[2 * TPI][16];
        cc_blocks<2 * TPI>(k, ctr, g);
        const uint4* ch = reinterpret_cast<const uint4*>(a.choices);
#pragma unroll
        for (int q = 0; q < TPI; q++) {
            const uint64_t j = j0 + q;
            if (j >= tiles) break;   // wave-uniform
#pragma unroll
            for (int w = 0; w < 4; w++) {
                const uint64_t c = 4 * j + w;
                const uint4 r = c < nblk_act ? ch[c] : make_uint4(0, 0, 0, 0);
                g[2 * q + 1][4 * w] ^= g[2 * q][4 * w] ^ r.x;
                g[2 * q + 1][4 * w + 1] ^= g[2 * q][4 * w + 1] ^ r.y;
                g[2 * q + 1][4 * w + 2] ^= g[2 * q][4 * w + 2] ^ r.z;
                g[2 * q + 1][4 * w + 3] ^= g[2 * q][4 * w + 3] ^ r.w;
            }
            const uint64_t run = ot_tmaj(64 * h, 4 * j);   // the wave's 4 KiB of tile j
            cc_store_rows(stage[wv], lane, g[2 * q], a.T + run);
            cc_store_rows(stage[wv], lane, g[2 * q + 1], a.U + run);
        }
    }
}

// The sender: work item = (2 tiles j, j + 1, row half h); lane row i computes G(k_i^{s_i}) for both tiles
// (2 ChaCha blocks in lockstep) and stores Q = G ^ s_i U tile-major (U read, Q written as whole-line runs).
__global__ __launch_bounds__(kOtCcThreads) void k_ot_send_expand_cc(OtArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t stage[kOtCcWaves][64 * kOtCcRowWords];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t nblk_act = (ot_active(a) + 127) / 128;
    const uint64_t tiles = (nblk_act + 3) / 4;
    const uint64_t items = 2 * ((tiles + 1) / 2);
    const uint64_t nwaves = (uint64_t)gridDim.x * kOtCcWaves;
    for (uint64_t it = (uint64_t)blockIdx.x * kOtCcWaves + wv; it < items; it += nwaves) {
        const uint64_t j0 = 2 * (it >> 1);
        const uint32_t h = (uint32_t)(it & 1), i = 64 * h + lane;
        const uint32_t si = (a.s[i >> 5] >> (i & 31)) & 1u;
        uint32_t k[2][4];
        ld_seed(a.rk, 256 + i, k[0]);
#pragma unroll
        for (int w = 0; w < 4; w++) k[1][w] = k[0][w];
        const uint64_t ctr[2] = {a.ctr_off / 4 + j0, a.ctr_off / 4 + j0 + 1};
        uint32_t g[2][16];
        cc_blocks<2>(k, ctr, g);
#pragma unroll
        for (int q = 0; q < 2; q++) {
            if (j0 + q >= tiles) break;   // wave-uniform
            const uint64_t run = ot_tmaj(64 * h, 4 * (j0 + q));
            uint32_t u[16];
            cc_load_rows(stage[wv], lane, a.U + run, u);
#pragma unroll
            for (int w = 0; w < 16; w++) g[q][w] ^= si ? u[w] : 0u;
            cc_store_rows(stage[wv], lane, g[q], a.Q + run);
        }
    }
}

// ---- r06: SoftSpoken OT extension (OtArgs::ss_k = 2, 4; oracle/fhh_oracle.c cot_rows / ss_ggm) ---------
// L. Roy, "SoftSpoken OT" (CRYPTO 2022), semi-honest small-field VOLE with the repetition code: the 128 base
// OTs in n_c = 128 / k chunks of k; chunk c's GGM tree gives the receiver 2^k leaf seeds and the sender every
// leaf but x = Delta_c (Delta_c bit b = s bit b n_c + c). Receiver: u_c = XOR_x G(leaf_x), t row b n_c + c =
// XOR_{x_b = 1} G(leaf_x), U_c = u_c ^ r on the wire; sender: q row b n_c + c = XOR_{y != 0, y_b = 1}
// G(leaf_{y ^ Delta_c}) ^ (Delta_c)_b U_c. Then q_j = t_j ^ r_j s exactly as IKNP, so every mode after the
// expands is unchanged — and U is 128 / k rows: 16 / k bytes per OT on the wire instead of 16. The price is
// ChaCha work: 2^k blocks per (chunk, tile) at the receiver (2 per row at k = 1: k = 2 the same, k = 4 2x) and
// 2^k - 1 at the sender (1 per row at k = 1: k = 2 1.5x, k = 4 3.75x). G is the IKNP row PRG (ChaCha12, key
// leaf || leaf, counter ctr_off / 4 + tile, nonce 0); the GGM tree's PRG and masks use nonces 1, 2, its root 3.

// one ChaCha12 block of a general 256-bit key, 64-bit counter and nonce (the GGM tree: one thread per chunk)
__device__ void cc_block_key8(const uint32_t (&key)[8], uint64_t ctr, uint32_t nonce, uint32_t (&x)[16]) {
    uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                       key[4], key[5], key[6], key[7], (uint32_t)ctr, (uint32_t)(ctr >> 32), nonce, 0u};
#pragma unroll
    for (int w = 0; w < 16; w++) x[w] = st[w];
    for (int r = 0; r < kOtChachaRounds; r += 2) {
        cc_qr(x[0], x[4], x[8], x[12]);
        cc_qr(x[1], x[5], x[9], x[13]);
        cc_qr(x[2], x[6], x[10], x[14]);
        cc_qr(x[3], x[7], x[11], x[15]);
        cc_qr(x[0], x[5], x[10], x[15]);
        cc_qr(x[1], x[6], x[11], x[12]);
        cc_qr(x[2], x[7], x[8], x[13]);
        cc_qr(x[3], x[4], x[9], x[14]);
    }
#pragma unroll
    for (int w = 0; w < 16; w++) x[w] += st[w];
}

__device__ __forceinline__ uint4 ss_key_row(const uint32_t* rk, uint32_t row) {
    return *reinterpret_cast<const uint4*>(rk + (size_t)row * 44);
}

// ChaCha12(a || b, ctr, nonce): the first 8 words (two 16-B seeds)
__device__ __forceinline__ void ss_cc(uint4 a, uint4 b, uint64_t ctr, uint32_t nonce, uint4& o0, uint4& o1) {
    const uint32_t key[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t x[16];
    cc_block_key8(key, ctr, nonce, x);
    o0 = make_uint4(x[0], x[1], x[2], x[3]);
    o1 = make_uint4(x[4], x[5], x[6], x[7]);
}

__device__ __forceinline__ uint4 x4(uint4 a, uint4 b) { return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w); }

// Both parties' GGM trees (the level loop runs both servers): thread c = chunk c. Receiver: the root from its
// pair k_c^0 || k_c^1, every level's two side sums masked under k_i^{1 - beta} (ss_corr [n_c][K][2], the
// wire); sender: unmasks side 1 - s_i with k_i^{s_i} and rebuilds every leaf but Delta_c. ss_leaf = receiver
// [n_c][2^K] then sender [n_c][2^K] (its x = Delta_c entry zero).
template <int K>
__global__ __launch_bounds__(64) void k_ss_ggm(OtArgs a) {
    constexpr uint32_t NC = 128 / K, NL = 1u << K;
    const uint32_t c = threadIdx.x;
    if (c >= NC) return;
    // every loop is unrolled (K is a template argument) so node / nxt stay in registers (no scratch)
    uint4 node[NL], nxt[NL];
    uint4 dummy;
    uint4* corr = a.ss_corr + (size_t)c * K * 2;
    if (a.ss_role != 2) {   // the receiver
        ss_cc(ss_key_row(a.rk, c), ss_key_row(a.rk, 128 + c), c, 3, node[0], dummy);
#pragma unroll
        for (uint32_t l = 1; l <= K; l++) {
            const uint32_t half = 1u << (l - 1), i = (l - 1) * NC + c;
            uint4 ks[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
#pragma unroll
            for (uint32_t z = 0; z < half; z++) {
                uint4 lft, rgt;
                ss_cc(node[z], node[z], 0, 1, lft, rgt);
                nxt[z] = lft;
                nxt[z | half] = rgt;
                ks[0] = x4(ks[0], lft);
                ks[1] = x4(ks[1], rgt);
            }
#pragma unroll
            for (uint32_t beta = 0; beta < 2; beta++) {
                const uint4 kk = ss_key_row(a.rk, (1 - beta) * 128 + i);
                uint4 msk;
                ss_cc(kk, kk, 0, 2, msk, dummy);
                corr[(l - 1) * 2 + beta] = x4(ks[beta], msk);
            }
#pragma unroll
            for (uint32_t z = 0; z < 2 * half; z++) node[z] = nxt[z];
        }
        uint4* leaf_r = a.ss_leaf + (size_t)c * NL;
#pragma unroll
        for (uint32_t x = 0; x < NL; x++) leaf_r[x] = node[x];
    }
    if (a.ss_role == 1) return;
    // the sender
    uint32_t dc = 0;
    for (uint32_t b = 0; b < (uint32_t)K; b++) {
        const uint32_t i = b * NC + c;
        dc |= ((a.s[i >> 5] >> (i & 31)) & 1u) << b;
    }
#pragma unroll
    for (uint32_t x = 0; x < NL; x++) node[x] = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t l = 1; l <= K; l++) {
        const uint32_t half = 1u << (l - 1), i = (l - 1) * NC + c, db = (dc >> (l - 1)) & 1u;
        const uint32_t path = dc & (half - 1);
        const uint4 kk = ss_key_row(a.rk, 256 + i);   // k_i^{s_i}
        uint4 msk;
        ss_cc(kk, kk, 0, 2, msk, dummy);
        uint4 sib = x4(corr[(l - 1) * 2 + (1 - db)], msk);
#pragma unroll
        for (uint32_t x = 0; x < NL; x++) nxt[x] = make_uint4(0, 0, 0, 0);
        if (l > 1) {
#pragma unroll
            for (uint32_t z = 0; z < half; z++) {
                if (z == path) continue;   // the unknown node on the path (its children stay zero)
                uint4 lft, rgt;
                ss_cc(node[z], node[z], 0, 1, lft, rgt);
                nxt[z] = lft;
                nxt[z | half] = rgt;
                sib = x4(sib, db ? lft : rgt);
            }
        }
        const uint32_t at = path | ((1 - db) << (l - 1));   // the path's sibling
#pragma unroll
        for (uint32_t z = 0; z < 2 * half; z++)
            if (z == at) nxt[z] = sib;
#pragma unroll
        for (uint32_t z = 0; z < 2 * half; z++) node[z] = nxt[z];
    }
    uint4* leaf_s = a.ss_leaf + (size_t)(NC + c) * NL;
#pragma unroll
    for (uint32_t x = 0; x < NL; x++) leaf_s[x] = x == dc ? make_uint4(0, 0, 0, 0) : node[x];
}

// the staging store of cc_store_rows with the wave's 64 rows in two runs: stage rows 0..31 -> run_lo, 32..63
// -> run_hi (k = 4: two tiles per wave), the high half skipped when hi_ok is false
__device__ __forceinline__ void cc_store_rows2(uint32_t* st, uint32_t lane, const uint32_t (&v)[16], uint4* run_lo,
                                               uint4* run_hi, bool hi_ok) {
#pragma unroll
    for (int w = 0; w < 4; w++)
        *reinterpret_cast<uint4*>(st + kOtCcRowWords * lane + 4 * w) = make_uint4(v[4 * w], v[4 * w + 1], v[4 * w + 2], v[4 * w + 3]);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uint32_t r = 16 * k + (lane >> 2), w = lane & 3;
        if (k >= 2 && !hi_ok) break;   // wave-uniform
        uint4* dst = (k < 2 ? run_lo + 64 * k : run_hi + 64 * (k - 2)) + lane;
        __builtin_nontemporal_store(*reinterpret_cast<const cc_v4*>(st + kOtCcRowWords * r + 4 * w),
                                    reinterpret_cast<cc_v4*>(dst));
    }
    __builtin_amdgcn_wave_barrier();
}

// Receiver: one wave = 64 (chunk, tile) lanes — k = 2: tile j, lane = chunk; k = 4: tiles j0, j0 + 1, lane =
// 32 (tile - j0) + chunk. 2^K blocks per lane, 2 in lockstep; t rows b n_c + c and U row c stored tile-major
// through the LDS stage (the wave's rows are whole-line runs: T rows b n_c .. b n_c + n_c - 1 of its tiles,
// U rows 0 .. n_c - 1 of its tiles — one contiguous 4 KiB, U's tile stride being n_c rows).
template <int K>
__global__ __launch_bounds__(kOtCcThreads) void k_ss_recv_expand(OtArgs a) {
    constexpr uint32_t NC = 128 / K, NL = 1u << K, TPW = 64 / NC;   // tiles per wave
    __shared__ __attribute__((aligned(16))) uint32_t stage[kOtCcWaves][64 * kOtCcRowWords];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t c = lane % NC, tq = lane / NC;
    const uint64_t nblk_act = (ot_active(a) + 127) / 128;
    const uint64_t tiles = (nblk_act + 3) / 4;
    const uint64_t items = (tiles + TPW - 1) / TPW;
    const uint64_t nwaves = (uint64_t)gridDim.x * kOtCcWaves;
    const uint4* leaf = a.ss_leaf + (size_t)c * NL;
    for (uint64_t it = (uint64_t)blockIdx.x * kOtCcWaves + wv; it < items; it += nwaves) {
        const uint64_t j0 = TPW * it, j = j0 + tq;
        const bool hi_ok = TPW == 1 || j0 + 1 < tiles;
        uint32_t u[16], v[K][16];
#pragma unroll
        for (int w = 0; w < 16; w++) {
            u[w] = 0;
#pragma unroll
            for (int b = 0; b < K; b++) v[b][w] = 0;
        }
#pragma unroll
        for (uint32_t x = 0; x < NL; x += 2) {
            uint32_t kk[2][4];
            const uint4 l0 = leaf[x], l1 = leaf[x + 1];
            kk[0][0] = l0.x; kk[0][1] = l0.y; kk[0][2] = l0.z; kk[0][3] = l0.w;
            kk[1][0] = l1.x; kk[1][1] = l1.y; kk[1][2] = l1.z; kk[1][3] = l1.w;
            const uint64_t ctr[2] = {a.ctr_off / 4 + j, a.ctr_off / 4 + j};
            uint32_t g[2][16];
            cc_blocks<2>(kk, ctr, g);
#pragma unroll
            for (int q = 0; q < 2; q++) {
#pragma unroll
                for (int w = 0; w < 16; w++) {
                    u[w] ^= g[q][w];
#pragma unroll
                    for (int b = 0; b < K; b++)
                        if (((x + q) >> b) & 1) v[b][w] ^= g[q][w];
                }
            }
        }
        const uint4* ch = reinterpret_cast<const uint4*>(a.choices);
#pragma unroll
        for (int w = 0; w < 4; w++) {
            const uint64_t cb = 4 * j + w;
            const uint4 r = cb < nblk_act ? ch[cb] : make_uint4(0, 0, 0, 0);
            u[4 * w] ^= r.x;
            u[4 * w + 1] ^= r.y;
            u[4 * w + 2] ^= r.z;
            u[4 * w + 3] ^= r.w;
        }
        // U: tile j0's rows 0 .. n_c - 1 onwards, contiguous for the wave (tile stride 4 n_c uint4)
        uint4* urun = a.U + j0 * (4 * NC);
        cc_store_rows2(stage[wv], lane, u, urun, urun + 128, hi_ok);
#pragma unroll
        for (int b = 0; b < K; b++)
            cc_store_rows2(stage[wv], lane, v[b], a.T + ot_tmaj(b * NC, 4 * j0),
                           a.T + ot_tmaj(b * NC + (TPW == 1 ? 32 : 0), 4 * (j0 + TPW - 1)), hi_ok);
    }
}

// Sender: the same lanes; y = 1 .. 2^K - 1 walks the leaves x = y ^ Delta_c (the coefficient (x ^ Delta_c)_b
// = y_b is the same for every lane), then q rows = w_b ^ (Delta_c)_b U_c.
template <int K>
__global__ __launch_bounds__(kOtCcThreads) void k_ss_send_expand(OtArgs a) {
    constexpr uint32_t NC = 128 / K, NL = 1u << K, TPW = 64 / NC;
    __shared__ __attribute__((aligned(16))) uint32_t stage[kOtCcWaves][64 * kOtCcRowWords];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t c = lane % NC, tq = lane / NC;
    const uint64_t nblk_act = (ot_active(a) + 127) / 128;
    const uint64_t tiles = (nblk_act + 3) / 4;
    const uint64_t items = (tiles + TPW - 1) / TPW;
    const uint64_t nwaves = (uint64_t)gridDim.x * kOtCcWaves;
    uint32_t dc = 0;
#pragma unroll
    for (int b = 0; b < K; b++) {
        const uint32_t i = b * NC + c;
        dc |= ((a.s[i >> 5] >> (i & 31)) & 1u) << b;
    }
    const uint4* leaf = a.ss_leaf + (size_t)(NC + c) * NL;
    for (uint64_t it = (uint64_t)blockIdx.x * kOtCcWaves + wv; it < items; it += nwaves) {
        const uint64_t j0 = TPW * it, j = j0 + tq;
        const bool hi_ok = TPW == 1 || j0 + 1 < tiles;
        uint32_t wr[K][16];
#pragma unroll
        for (int w = 0; w < 16; w++)
#pragma unroll
            for (int b = 0; b < K; b++) wr[b][w] = 0;
#pragma unroll
        for (uint32_t y = 1; y < NL; y += 2) {   // pairs (y, y + 1); y = NL - 1 alone
            const bool two = y + 1 < NL;
            uint32_t kk[2][4];
            const uint4 l0 = leaf[y ^ dc], l1 = two ? leaf[(y + 1) ^ dc] : l0;
            kk[0][0] = l0.x; kk[0][1] = l0.y; kk[0][2] = l0.z; kk[0][3] = l0.w;
            kk[1][0] = l1.x; kk[1][1] = l1.y; kk[1][2] = l1.z; kk[1][3] = l1.w;
            const uint64_t ctr[2] = {a.ctr_off / 4 + j, a.ctr_off / 4 + j};
            uint32_t g[2][16];
            if (two) {
                cc_blocks<2>(kk, ctr, g);
            } else {
                uint32_t k1[1][4] = {{kk[0][0], kk[0][1], kk[0][2], kk[0][3]}};
                const uint64_t c1[1] = {ctr[0]};
                uint32_t g1[1][16];
                cc_blocks<1>(k1, c1, g1);
#pragma unroll
                for (int w = 0; w < 16; w++) g[0][w] = g1[0][w];
            }
#pragma unroll
            for (int q = 0; q < 2; q++) {
                if (q == 1 && !two) break;
#pragma unroll
                for (int w = 0; w < 16; w++)
#pragma unroll
                    for (int b = 0; b < K; b++)
                        if (((y + q) >> b) & 1) wr[b][w] ^= g[q][w];
            }
        }
        uint32_t u[16];
        {   // U rows of the wave's tiles (contiguous), dealt to the lanes through the stage
            const uint4* urun = a.U + j0 * (4 * NC);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t r = 16 * k + (lane >> 2), w = lane & 3;
                if (k >= 2 && !hi_ok) break;
                *reinterpret_cast<cc_v4*>(stage[wv] + kOtCcRowWords * r + 4 * w) =
                    __builtin_nontemporal_load(reinterpret_cast<const cc_v4*>(urun + 64 * k + lane));
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int w = 0; w < 4; w++) {
                const uint4 x = *reinterpret_cast<const uint4*>(stage[wv] + kOtCcRowWords * lane + 4 * w);
                u[4 * w] = x.x;
                u[4 * w + 1] = x.y;
                u[4 * w + 2] = x.z;
                u[4 * w + 3] = x.w;
            }
            __builtin_amdgcn_wave_barrier();
        }
#pragma unroll
        for (int b = 0; b < K; b++) {
            const uint32_t db = (dc >> b) & 1u;
#pragma unroll
            for (int w = 0; w < 16; w++) wr[b][w] ^= db ? u[w] : 0u;
            cc_store_rows2(stage[wv], lane, wr[b], a.Q + ot_tmaj(b * NC, 4 * j0),
                           a.Q + ot_tmaj(b * NC + (TPW == 1 ? 32 : 0), 4 * (j0 + TPW - 1)), hi_ok);
        }
    }
}

// ---- transpose-fused hashes (r02) ------------------------------------------------------------
// The hashes read the 128 x m bit matrices (T, Q; tile-major) as row words and transpose on the fly, so
// the separate transpose pass of r01 (k_ot_transpose: an HBM round trip of 32 B per OT, 7 % of the
// GC + OT crawl) is gone.
// One wave = one tile of 16 words x 128 rows = 512 OTs. Lane l = 4 q + g loads rows 32 g .. 32 g + 31
// of word w = 16 tile + q (4 rows x 64 B per load instruction) and transposes them in registers:
// x[k] = word g of OT 32 w + k. The OTs then reach their lanes through 2 KB of LDS per wave, in
// four rounds of 8 k's: round r writes x[8 r + kk] to word kk * 64 + l (lane-linear ds_write_b32)
// and lane l reads OTs kk = (l >> 4) + 4 u, q = l & 15 (u < 2) as ds_read_b128 at kk * 64 + 4 q —
// 16 distinct q per b128 lane group, banks 4 q .. 4 q + 3 of 64: conflict-free. The staging rides
// beside the 128 KiB of T-tables (160 KiB per workgroup, one workgroup per CU). LDS accesses of one
// wave retire in order, so the exchange needs no barrier. The exchange rounds run as a rolled loop
// (x moves down by 8 words per round): unrolled, the scheduler interleaved the rounds and spilled
// ~90 VGPRs. The receiver hashes 4 OTs (two rounds) per AES pass, the sender one OT (2 blocks) per
// pass: its 4-block form still spilled 9 VGPRs beside the tile's 32 words.
constexpr int kOtTileWords = 16;
constexpr int kOtRowsThreads = 1024;
constexpr int kOtWaves = kOtRowsThreads / 64;

__device__ __forceinline__ uint64_t ot_tile_ot(uint64_t tile, uint32_t lane, int r, int u) {
    return 32 * (tile * kOtTileWords + (lane & 15)) + 8 * r + (lane >> 4) + 4 * u;
}

__device__ __forceinline__ void ot_tile_load(const uint32_t* rows, uint64_t tile, uint32_t lane, uint32_t (&x)[32]) {
    const uint32_t q = lane >> 2, g = lane & 3;
    const uint32_t* p = rows + tile * (128 * kOtTileWords) + (32 * g) * kOtTileWords + q;   // ot_tmaj
#pragma unroll
    for (int i = 0; i < 32; i++) x[i] = __builtin_nontemporal_load(p + i * kOtTileWords);
    transpose32(x);   // x[k] bit i = row 32 g + i of OT 32 w + k
}

// one round of the exchange: this lane's OTs ot_tile_ot(tile, lane, r, 0 / 1) as uint4 {word 0..3}
// from x[0..7] = x[8 r .. 8 r + 7] of the tile, then x moves down by 8 (a rolled round loop keeps
// the 32 words in registers; indexing x by the round would put them in scratch)
__device__ __forceinline__ void ot_tile_round(uint32_t* st, uint32_t (&x)[32], uint32_t lane, uint4 (&o)[2]) {
#pragma unroll
    for (int kk = 0; kk < 8; kk++) st[kk * 64 + lane] = x[kk];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < 2; u++) o[u] = *reinterpret_cast<const uint4*>(st + ((lane >> 4) + 4 * u) * 64 + 4 * (lane & 15));
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < 24; i++) x[i] = x[i + 8];
}

__device__ __forceinline__ uint64_t ot_mix64(uint64_t z) {   // SplitMix64's finaliser (ideal base OTs only)
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// The send hash: one wave per 512-OT tile (transposed in registers + LDS), one OT (2 blocks: q, q ^ s)
// per pass. MODE (OtArgs::mode): 0 plain OT (y^b = x^b ^ H(q ^ b s)), 1 C-OT labels (sx = H(q),
// y = H(q) ^ delta ^ H(q ^ s)), 2 C-OT FE share (sx = v + mask, y = lo64(H(q ^ s)) ^ pair[1], 8 B),
// 3 C-OT raw (sx = H(q), y = H(q ^ s); k_cot_fe255_finish completes the FieldElm share)
template <int MODE>
__global__ __launch_bounds__(kOtRowsThreads) void k_ot_send_hash_rows(OtArgs a) {
    __shared__ uint32_t tbl_ot[OtTab::kWords];
    __shared__ uint32_t stage[kOtWaves][512];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t m = ot_active(a);
    const uint64_t tiles = (m + 32 * kOtTileWords - 1) / (32 * kOtTileWords);
    if ((uint64_t)blockIdx.x * kOtWaves >= tiles) return;   // no tiles for this workgroup: skip the fill
    ot_fill(tbl_ot);
    uint32_t b0, b1;
    OtTab::bases(lane, b0, b1);
    const uint64_t nwaves = (uint64_t)gridDim.x * kOtWaves;
    const uint32_t* rows = reinterpret_cast<const uint32_t*>(a.Q);
    for (uint64_t t = (uint64_t)blockIdx.x * kOtWaves + wv; t < tiles; t += nwaves) {
        uint32_t x[32];
        ot_tile_load(rows, t, lane, x);
#pragma unroll 1
        for (int r = 0; r < 4; r++) {
            uint4 q[2];
            ot_tile_round(stage[wv], x, lane, q);
#pragma unroll
            for (int u = 0; u < 2; u++) {
                uint32_t h[2][4] = {{q[u].x, q[u].y, q[u].z, q[u].w},
                                    {q[u].x ^ a.s[0], q[u].y ^ a.s[1], q[u].z ^ a.s[2], q[u].w ^ a.s[3]}};
                aes0_mmo_tab<DevOpsX, OtTab, 2>(h, tbl_ot, b0, b1);   // cr_hash: pi(x) ^ x
                const uint64_t j = ot_tile_ot(t, lane, r, u);
                if (j >= m) continue;
                if constexpr (MODE == 0) {
                    const uint4 x0 = a.x0[j];
                    const uint4 x1 = a.x1 ? a.x1[j]
                                          : make_uint4(x0.x ^ a.delta[0], x0.y ^ a.delta[1], x0.z ^ a.delta[2],
                                                       x0.w ^ a.delta[3]);
                    a.Y0[j] = make_uint4(x0.x ^ h[0][0], x0.y ^ h[0][1], x0.z ^ h[0][2], x0.w ^ h[0][3]);
                    a.Y1[j] = make_uint4(x1.x ^ h[1][0], x1.y ^ h[1][1], x1.z ^ h[1][2], x1.w ^ h[1][3]);
                } else if constexpr (MODE == 1) {
                    static_cast<uint4*>(a.sx)[j] = make_uint4(h[0][0], h[0][1], h[0][2], h[0][3]);
                    a.Y0[j] = make_uint4(h[0][0] ^ a.delta[0] ^ h[1][0], h[0][1] ^ a.delta[1] ^ h[1][1],
                                         h[0][2] ^ a.delta[2] ^ h[1][2], h[0][3] ^ a.delta[3] ^ h[1][3]);
                } else if constexpr (MODE == 2) {
                    const uint64_t v = ot_fe_of_u128((uint64_t)h[0][0] | ((uint64_t)h[0][1] << 32),
                                                     (uint64_t)h[0][2] | ((uint64_t)h[0][3] << 32));
                    const uint64_t vp = v + 1 == kOtFeP ? 0 : v + 1, vm = v ? v - 1 : kOtFeP - 1;
                    const uint64_t gv = a.mask ? vp : v, p1 = a.mask ? vp : vm;   // r1 = v + mask; pair[1]
                    static_cast<uint64_t*>(a.sx)[j] = gv;
                    reinterpret_cast<uint2*>(a.Y0)[j] = make_uint2(h[1][0] ^ (uint32_t)p1, h[1][1] ^ (uint32_t)(p1 >> 32));
                } else {
                    static_cast<uint4*>(a.sx)[j] = make_uint4(h[0][0], h[0][1], h[0][2], h[0][3]);
                    a.Y0[j] = make_uint4(h[1][0], h[1][1], h[1][2], h[1][3]);
                }
            }
        }
    }
}

// The receive hash: one wave per 512-OT tile, 4 OTs (4 blocks) per AES pass. MODE 0: out = y^{r} ^
// H(t); 1 / 3: out = r ? y ^ H(t) : H(t); 2: out (u64) = r ? lo64(y ^ H(t)) : H(t) mod p.
template <int MODE>
__global__ __launch_bounds__(kOtRowsThreads) void k_ot_recv_hash_rows(OtArgs a) {
    __shared__ uint32_t tbl_ot[OtTab::kWords];
    __shared__ uint32_t stage[kOtWaves][512];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t m = ot_active(a);
    const uint64_t tiles = (m + 32 * kOtTileWords - 1) / (32 * kOtTileWords);
    if ((uint64_t)blockIdx.x * kOtWaves >= tiles) return;   // no tiles for this workgroup: skip the fill
    ot_fill(tbl_ot);
    uint32_t b0, b1;
    OtTab::bases(lane, b0, b1);
    const uint64_t nwaves = (uint64_t)gridDim.x * kOtWaves;
    const uint32_t* rows = reinterpret_cast<const uint32_t*>(a.T);
    for (uint64_t t = (uint64_t)blockIdx.x * kOtWaves + wv; t < tiles; t += nwaves) {
        uint32_t x[32];
        ot_tile_load(rows, t, lane, x);
        // the lane's 8 OTs of the tile share one choice word (ot_tile_ot: j >> 5 = 16 t + (lane & 15));
        // read once per tile, and only if the word holds an active OT (the buffer may end at m bits)
        const uint64_t cwi = t * kOtTileWords + (lane & 15);
        const uint32_t cw = 32 * cwi < m ? a.choices[cwi] : 0u;
#pragma unroll 1
        for (int r = 0; r < 4; r += 2) {   // two rounds = 4 OTs = 4 blocks in lockstep
            uint32_t h[4][4];
#pragma unroll
            for (int rr = 0; rr < 2; rr++) {
                uint4 tv[2];
                ot_tile_round(stage[wv], x, lane, tv);
#pragma unroll
                for (int u = 0; u < 2; u++) {
                    h[2 * rr + u][0] = tv[u].x; h[2 * rr + u][1] = tv[u].y;
                    h[2 * rr + u][2] = tv[u].z; h[2 * rr + u][3] = tv[u].w;
                }
            }
            auto otj = [&](int b) -> uint64_t { return ot_tile_ot(t, lane, r + (b >> 1), b & 1); };
            auto chosen = [&](int b) -> uint32_t {   // the OT is active and its choice bit is set
                const uint64_t j = otj(b);
                return j < m ? (cw >> (j & 31)) & 1u : 0u;
            };
            // the Y blocks the pass needs are in flight while its AES runs (r03: without the Y loads the
            // plain kernel was 18 % faster, `profiles/r03/ot_diag/`): straight into the exchange stage,
            // idle until the next pass (global_load_lds, lane-linear). Plain OT: OTs 0, 1 of the pass
            // (16 B each; 2, 3 load after the AES). C-OT: a lane loads only when its choice bit is set
            // (modes 1 / 3: 16 B for OTs 0, 1; mode 2: 8 B for all four OTs as two dwords)
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the exchange's stage reads are done
            if constexpr (MODE == 0) {
                auto ysrc = [&](int b) -> const uint4* {   // the OT's chosen Y (inactive OTs: a valid block)
                    const uint64_t j = otj(b);
                    return j < m ? (((cw >> (j & 31)) & 1u) ? a.Y1 : a.Y0) + j : a.Y0;
                };
#pragma unroll
                for (int b = 0; b < 2; b++)
                    __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(ysrc(b)), &stage[wv][256 * b], 16, 0, 0);
                aes0_mmo_tab<DevOpsX, OtTab, 4>(h, tbl_ot, b0, b1);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the stage's Y blocks have landed
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const uint4 y = b < 2 ? *reinterpret_cast<const uint4*>(&stage[wv][256 * b + 4 * lane]) : *ysrc(b);
                    const uint64_t j = otj(b);
                    if (j >= m) continue;
                    a.out[j] = make_uint4(y.x ^ h[b][0], y.y ^ h[b][1], y.z ^ h[b][2], y.w ^ h[b][3]);
                }
            } else if constexpr (MODE == 2) {
                const uint32_t* y32 = reinterpret_cast<const uint32_t*>(a.Y0);
#pragma unroll
                for (int b = 0; b < 4; b++)
                    if (chosen(b)) {
                        const uint64_t j = otj(b);
                        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(y32 + 2 * j), &stage[wv][128 * b], 4, 0, 0);
                        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(y32 + 2 * j + 1), &stage[wv][128 * b + 64], 4, 0, 0);
                    }
                aes0_mmo_tab<DevOpsX, OtTab, 4>(h, tbl_ot, b0, b1);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                uint64_t* o = reinterpret_cast<uint64_t*>(a.out);
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const uint64_t j = otj(b);
                    if (j >= m) continue;
                    const uint64_t hl = (uint64_t)h[b][0] | ((uint64_t)h[b][1] << 32);
                    if (chosen(b)) {
                        const uint64_t y = (uint64_t)stage[wv][128 * b + lane] | ((uint64_t)stage[wv][128 * b + 64 + lane] << 32);
                        o[j] = y ^ hl;
                    } else {
                        o[j] = ot_fe_of_u128(hl, (uint64_t)h[b][2] | ((uint64_t)h[b][3] << 32));
                    }
                }
            } else {   // modes 1, 3
#pragma unroll
                for (int b = 0; b < 2; b++)
                    if (chosen(b))
                        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(a.Y0 + otj(b)), &stage[wv][256 * b], 16, 0, 0);
                aes0_mmo_tab<DevOpsX, OtTab, 4>(h, tbl_ot, b0, b1);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const uint64_t j = otj(b);
                    if (j >= m) continue;
                    uint4 y = make_uint4(0, 0, 0, 0);
                    if (chosen(b)) y = b < 2 ? *reinterpret_cast<const uint4*>(&stage[wv][256 * b + 4 * lane]) : a.Y0[j];
                    a.out[j] = make_uint4(y.x ^ h[b][0], y.y ^ h[b][1], y.z ^ h[b][2], y.w ^ h[b][3]);
                }
            }
            __builtin_amdgcn_wave_barrier();   // the Y reads precede the next pass's stage writes
        }
    }
}

// Mode 4 (r05b): the labels OT as the IKNP correlation itself. With the sender's s as the free-XOR
// offset, q_j (sender) and t_j = q_j ^ r_j s (receiver) already are the zero label and the active label
// of the evaluator's input wire j — the random correlated OT that free-XOR garbling consumes — so no
// hash and no message y is needed: this kernel only transposes the tile-major matrix into one 16-B row
// per OT. One wave per 512-OT tile: the hashes' row loads + in-register 32 x 32 transposes, then the
// whole tile goes through LDS once so that every store writes 64 consecutive OTs (1 KiB): lane (q, g)
// writes word g of OTs 32 q + k at 132 q + 4 k + g (banks 4 q + g + 4 k: conflict-free), lane l reads
// OT 64 r + l as one ds_read_b128. No T-tables: 8.25 KiB of stage per wave.
constexpr int kOtOutThreads = 256;
constexpr int kOtOutStride = 132;   // words per 32-OT group in the stage (128 + 4: bank spread)
__global__ __launch_bounds__(kOtOutThreads) void k_ot_rows_out(OtArgs a, int sender) {
    __shared__ __attribute__((aligned(16))) uint32_t stage[kOtOutThreads / 64][kOtTileWords * kOtOutStride];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t m = ot_active(a);
    const uint64_t tiles = (m + 32 * kOtTileWords - 1) / (32 * kOtTileWords);
    const uint64_t nwaves = (uint64_t)gridDim.x * (kOtOutThreads / 64);
    const uint32_t* rows = reinterpret_cast<const uint32_t*>(sender ? a.Q : a.T);
    uint4* out = sender ? static_cast<uint4*>(a.sx) : a.out;
    uint32_t* st = stage[wv];
    const uint32_t q = lane >> 2, g = lane & 3;
    for (uint64_t t = (uint64_t)blockIdx.x * (kOtOutThreads / 64) + wv; t < tiles; t += nwaves) {
        uint32_t x[32];
        {   // the tile as ot_tile_load reads it, by cached loads: rows r, r + 1 share a 128-B line (the
            // non-temporal form measured 2.40-2.48 s per 1M crawl against 2.29-2.33 s, profiles/r05/table/)
            const uint32_t* p = rows + t * (128 * kOtTileWords) + (32 * g) * kOtTileWords + q;
#pragma unroll
            for (int i = 0; i < 32; i++) x[i] = p[i * kOtTileWords];
            transpose32(x);   // x[k] = word g of OT 32 (16 t + q) + k
        }
#pragma unroll
        for (int k = 0; k < 32; k++) st[kOtOutStride * q + 4 * k + g] = x[k];
        __builtin_amdgcn_wave_barrier();
        const uint64_t j0 = 512 * t;
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const uint32_t o = 64 * r + lane;
            const uint4 v = *reinterpret_cast<const uint4*>(st + kOtOutStride * (o >> 5) + 4 * (o & 31));
            if (j0 + o < m) out[j0 + o] = v;
        }
        __builtin_amdgcn_wave_barrier();   // the reads precede the next tile's stage writes
    }
}

// mode 3's second pass (the garbler's FieldElm share, collect.rs:846-876): test t = OT pair (2t, 2t + 1).
// V = H(q_2t) || H(q_2t+1) read as 32 big-endian bytes (the BlockPair convention, field.rs:466-492),
// reduced mod p255; the garbler's node value r1 = V + mask replaces the H(q) pair in sx (canonical
// BlockPair), pair[1] = mask ? V + 1 : V - 1 is XORed into y = H(q ^ s). One lane per test.
__device__ __forceinline__ void ot_bp_to_limbs(uint4 b0, uint4 b1, uint64_t (&r)[4]) {
    r[3] = ((uint64_t)__builtin_bswap32(b0.x) << 32) | __builtin_bswap32(b0.y);
    r[2] = ((uint64_t)__builtin_bswap32(b0.z) << 32) | __builtin_bswap32(b0.w);
    r[1] = ((uint64_t)__builtin_bswap32(b1.x) << 32) | __builtin_bswap32(b1.y);
    r[0] = ((uint64_t)__builtin_bswap32(b1.z) << 32) | __builtin_bswap32(b1.w);
}
__device__ __forceinline__ uint4 ot_limbs_to_block(uint64_t hi, uint64_t lo) {
    return make_uint4(__builtin_bswap32((uint32_t)(hi >> 32)), __builtin_bswap32((uint32_t)hi),
                      __builtin_bswap32((uint32_t)(lo >> 32)), __builtin_bswap32((uint32_t)lo));
}
// x (< 2^256) - p255 when x >= p255, at most twice (2^256 = 2 p + 38)
__device__ __forceinline__ void ot_fe255_canon(uint64_t (&x)[4]) {
    constexpr uint64_t P[4] = {0xFFFFFFFFFFFFFFEDull, ~0ull, ~0ull, 0x7FFFFFFFFFFFFFFFull};
#pragma unroll
    for (int it = 0; it < 2; it++) {
        uint64_t t[4], borrow = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const unsigned __int128 v = (unsigned __int128)x[k] - P[k] - borrow;
            t[k] = (uint64_t)v;
            borrow = (uint64_t)(v >> 64) & 1;
        }
        if (!borrow) {
#pragma unroll
            for (int k = 0; k < 4; k++) x[k] = t[k];
        }
    }
}
// x +- 1 mod p255 for canonical x
__device__ __forceinline__ void ot_fe255_inc(const uint64_t (&x)[4], uint64_t (&o)[4]) {
    unsigned __int128 acc = (unsigned __int128)x[0] + 1;
    o[0] = (uint64_t)acc;
#pragma unroll
    for (int k = 1; k < 4; k++) {
        acc = (unsigned __int128)x[k] + (uint64_t)(acc >> 64);
        o[k] = (uint64_t)acc;
    }
    ot_fe255_canon(o);
}
__device__ __forceinline__ void ot_fe255_dec(const uint64_t (&x)[4], uint64_t (&o)[4]) {
    if ((x[0] | x[1] | x[2] | x[3]) == 0) {   // 0 - 1 = p - 1
        o[0] = 0xFFFFFFFFFFFFFFECull;
        o[1] = o[2] = ~0ull;
        o[3] = 0x7FFFFFFFFFFFFFFFull;
        return;
    }
    uint64_t borrow = 1;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        o[k] = x[k] - borrow;
        borrow = (x[k] < borrow) ? 1 : 0;
    }
}

__global__ __launch_bounds__(256) void k_cot_fe255_finish(OtArgs a) {
    const uint64_t tests = ot_active(a) / 2;
    uint4* sx = static_cast<uint4*>(a.sx);
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < tests; t += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t V[4], G[4], P1[4];
        ot_bp_to_limbs(sx[2 * t], sx[2 * t + 1], V);
        ot_fe255_canon(V);
        if (a.mask) {
            ot_fe255_inc(V, G);
#pragma unroll
            for (int k = 0; k < 4; k++) P1[k] = G[k];
        } else {
#pragma unroll
            for (int k = 0; k < 4; k++) G[k] = V[k];
            ot_fe255_dec(V, P1);
        }
        sx[2 * t] = ot_limbs_to_block(G[3], G[2]);
        sx[2 * t + 1] = ot_limbs_to_block(G[1], G[0]);
        const uint4 e0 = ot_limbs_to_block(P1[3], P1[2]), e1 = ot_limbs_to_block(P1[1], P1[0]);
        const uint4 y0 = a.Y0[2 * t], y1 = a.Y0[2 * t + 1];
        a.Y0[2 * t] = make_uint4(y0.x ^ e0.x, y0.y ^ e0.y, y0.z ^ e0.z, y0.w ^ e0.w);
        a.Y0[2 * t + 1] = make_uint4(y1.x ^ e1.x, y1.y ^ e1.y, y1.z ^ e1.z, y1.w ^ e1.w);
    }
}

// Level-loop base OTs (ideal): the 128 seed pairs derived from (prf_seed, level, salt) on the
// device, so an enqueued level needs no host data; key schedules [3][128][44] (k_i^0, k_i^1,
// k_i^{s_i}). One thread per key.
__constant__ ByteTable c_sbox_ot = SBOX;

__device__ __forceinline__ uint64_t ot_seed_word(uint64_t prf, uint32_t level, uint32_t salt, uint32_t i, uint32_t b,
                                                 int h) {
    const uint64_t z = ot_mix64(prf ^ 0x6f745f62617365ull ^ ((uint64_t)level << 24) ^ ((uint64_t)salt << 20) ^
                                ((uint64_t)i << 2) ^ b);
    return h ? ot_mix64(z) : z;
}

__global__ void k_ot_level_keys(uint64_t prf, uint32_t level, uint32_t salt, uint32_t s0, uint32_t s1, uint32_t s2,
                                uint32_t s3, uint32_t* rk) {
    const uint32_t k = threadIdx.x;
    if (k >= 384) return;
    const uint32_t which = k / 128, i = k % 128;
    const uint32_t sw[4] = {s0, s1, s2, s3};
    const uint32_t b = which < 2 ? which : (sw[i >> 5] >> (i & 31)) & 1u;
    const uint64_t lo = ot_seed_word(prf, level, salt, i, b, 0), hi = ot_seed_word(prf, level, salt, i, b, 1);
    uint32_t w[44] = {(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
    uint32_t rcon = 1;
    for (int j = 4; j < 44; j++) {
        uint32_t t = w[j - 1];
        if (j % 4 == 0) {
            t = (t >> 8) | (t << 24);
            t = (uint32_t)c_sbox_ot.v[t & 0xFF] | ((uint32_t)c_sbox_ot.v[(t >> 8) & 0xFF] << 8) |
                ((uint32_t)c_sbox_ot.v[(t >> 16) & 0xFF] << 16) | ((uint32_t)c_sbox_ot.v[t >> 24] << 24);
            t ^= rcon;
            rcon = ((rcon << 1) ^ ((rcon & 0x80) ? 0x1B : 0)) & 0xFF;
        }
        w[j] = w[j - 4] ^ t;
    }
    for (int j = 0; j < 44; j++) rk[((size_t)which * 128 + i) * 44 + j] = w[j];
}

hipError_t launch_ot_level_keys(uint64_t prf, uint32_t level, uint32_t salt, const uint32_t s[4], uint32_t* rk,
                                hipStream_t stream) {
    hipLaunchKernelGGL(k_ot_level_keys, dim3(1), dim3(384), 0, stream, prf, level, salt, s[0], s[1], s[2], s[3], rk);
    return hipGetLastError();
}

// CU count of the current device, queried once per device (the level loop launches these
// kernels thousands of times per crawl)
static int device_cus() {
    static std::atomic<int> cache[64] = {};   // shard threads of a multi-device ctx share it
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int cus = cache[dev].load(std::memory_order_relaxed);
    if (!cus) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
        cache[dev].store(cus, std::memory_order_relaxed);
    }
    return cus;
}


// the ChaCha expands: 256-thread workgroups (20 KiB of LDS staging, ~70 VGPRs), 8 per CU, waves stride over the items
static int ot_cc_grid(uint64_t items) {
    const uint64_t wpb = kOtCcThreads / 64, need = (items + wpb - 1) / wpb, cap = (uint64_t)device_cus() * 8;
    return (int)(need < cap ? (need ? need : 1) : cap);
}

hipError_t launch_ot_recv_expand(const OtArgs& a, hipStream_t stream) {
    if (a.ctr_off % 4) return hipErrorInvalidValue;   // ChaCha counters per 512-OT tile
    if (a.ss_k == 2 || a.ss_k == 4) {   // SoftSpoken: one wave per tile (k = 2) or tile pair (k = 4)
        const uint64_t tiles = a.mp / 512;
        if (a.ss_k == 2) hipLaunchKernelGGL(k_ss_recv_expand<2>, dim3(ot_cc_grid(tiles)), dim3(kOtCcThreads), 0, stream, a);
        else hipLaunchKernelGGL(k_ss_recv_expand<4>, dim3(ot_cc_grid((tiles + 1) / 2)), dim3(kOtCcThreads), 0, stream, a);
        return hipGetLastError();
    }
    if (a.ss_k > 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ot_recv_expand_cc, dim3(ot_cc_grid(2 * (a.mp / 512))), dim3(kOtCcThreads), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_ot_send_expand(const OtArgs& a, hipStream_t stream) {
    if (a.ctr_off % 4) return hipErrorInvalidValue;
    if (a.ss_k == 2 || a.ss_k == 4) {
        const uint64_t tiles = a.mp / 512;
        if (a.ss_k == 2) hipLaunchKernelGGL(k_ss_send_expand<2>, dim3(ot_cc_grid(tiles)), dim3(kOtCcThreads), 0, stream, a);
        else hipLaunchKernelGGL(k_ss_send_expand<4>, dim3(ot_cc_grid((tiles + 1) / 2)), dim3(kOtCcThreads), 0, stream, a);
        return hipGetLastError();
    }
    if (a.ss_k > 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_ot_send_expand_cc, dim3(ot_cc_grid(a.mp / 512)), dim3(kOtCcThreads), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_ss_ggm(const OtArgs& a, hipStream_t stream) {
    switch (a.ss_k) {
        case 2: hipLaunchKernelGGL(k_ss_ggm<2>, dim3(1), dim3(64), 0, stream, a); break;
        case 4: hipLaunchKernelGGL(k_ss_ggm<4>, dim3(1), dim3(64), 0, stream, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

__global__ void k_mask_word(uint32_t* word, uint32_t mask) {
    if (threadIdx.x == 0) *word &= mask;
}

hipError_t launch_mask_word(uint32_t* word, uint32_t mask, hipStream_t stream) {
    hipLaunchKernelGGL(k_mask_word, dim3(1), dim3(64), 0, stream, word, mask);
    return hipGetLastError();
}

// the hashes: one 1024-thread workgroup per CU (160 KiB of LDS), waves stride over the tiles
static int ot_rows_grid(const OtArgs& a) {
    const uint64_t tiles = (a.m + 32 * kOtTileWords - 1) / (32 * kOtTileWords);
    const uint64_t need = (tiles + kOtWaves - 1) / kOtWaves, cap = (uint64_t)device_cus();
    return (int)(need < cap ? (need ? need : 1) : cap);
}

hipError_t launch_ot_send_hash_rows(const OtArgs& a, hipStream_t stream) {
    if (a.mp % 8192 != 0) return hipErrorInvalidValue;   // tiles of 16 words stay inside a row
    const dim3 g(ot_rows_grid(a)), b(kOtRowsThreads);
    switch (a.mode) {
        case 0: hipLaunchKernelGGL(k_ot_send_hash_rows<0>, g, b, 0, stream, a); break;
        case 1: hipLaunchKernelGGL(k_ot_send_hash_rows<1>, g, b, 0, stream, a); break;
        case 2: hipLaunchKernelGGL(k_ot_send_hash_rows<2>, g, b, 0, stream, a); break;
        case 3: hipLaunchKernelGGL(k_ot_send_hash_rows<3>, g, b, 0, stream, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_ot_recv_hash_rows(const OtArgs& a, hipStream_t stream) {
    if (a.mp % 8192 != 0) return hipErrorInvalidValue;
    const dim3 g(ot_rows_grid(a)), b(kOtRowsThreads);
    switch (a.mode) {
        case 0: hipLaunchKernelGGL(k_ot_recv_hash_rows<0>, g, b, 0, stream, a); break;
        case 1: hipLaunchKernelGGL(k_ot_recv_hash_rows<1>, g, b, 0, stream, a); break;
        case 2: hipLaunchKernelGGL(k_ot_recv_hash_rows<2>, g, b, 0, stream, a); break;
        case 3: hipLaunchKernelGGL(k_ot_recv_hash_rows<3>, g, b, 0, stream, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_ot_rows_out(const OtArgs& a, bool sender, hipStream_t stream) {
    if (a.mp % 8192 != 0) return hipErrorInvalidValue;   // tiles of 16 words stay inside a row
    const uint64_t tiles = (a.m + 32 * kOtTileWords - 1) / (32 * kOtTileWords);
    const uint64_t wpb = kOtOutThreads / 64, need = (tiles + wpb - 1) / wpb, cap = (uint64_t)device_cus() * 8;
    hipLaunchKernelGGL(k_ot_rows_out, dim3((int)(need < cap ? (need ? need : 1) : cap)), dim3(kOtOutThreads), 0, stream,
                       a, sender ? 1 : 0);
    return hipGetLastError();
}

hipError_t launch_cot_fe255_finish(const OtArgs& a, hipStream_t stream) {
    if (a.mode != 3 || a.m % 2) return hipErrorInvalidValue;
    const uint64_t tests = a.m / 2;
    const uint64_t need = (tests + 255) / 256, cap = (uint64_t)device_cus() * 8;
    hipLaunchKernelGGL(k_cot_fe255_finish, dim3((int)(need < cap ? (need ? need : 1) : cap)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace fhh
