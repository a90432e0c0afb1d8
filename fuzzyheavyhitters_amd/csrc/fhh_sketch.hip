// Sketch + Beaver-triple verification: SketchDPFKey::sketch_at
// (src/sketch.rs:157-200) and MulState (src/mpc.rs:83-220), both fully commented out in the
// reference; restated from the commented text for T = FE (GF(2^62 - 2^30 - 1)).
//
//   k_sketch_fe   one wave per key: the key's PrgStream (AES-128-CTR, key = the key's sketch
//                 seed, IV 0, prg.rs:82-90) is random-access, so lane l produces keystream
//                 blocks l, l+64, ... (two u64 draws each: rand1..3, then r_j for node j),
//                 reads its nodes' (x, kx) coalesced, accumulates <r,x>, <r^2,x>, <r,kx> mod p
//                 and the wave reduces. FE::from_rng redraws on a draw >= p (P ~ 2^-32): a
//                 wave that sees one falls back to the sequential stream for that key.
//   k_mul_fe      MulState::cor_share / out_share per key (one lane per key).
//   k_verify_fe   MulState::cor + out shares of both servers + verify, fused (in-process).
//   k_sketch_fe255 / k_mul_fe255 / k_verify_fe255: the same for U = FieldElm (GF(2^255 - 19)),
//                 the last level's sketch_at_last (sketch.rs:202-245).
#include "fhh_internal.h"

#include <atomic>
#include <type_traits>
#include "expand_kernel.h"
#include "aes_tables.h"
#include "field_arith.h"
#include "aes_keyed.h"
#include "../../include/fhh.h"

namespace fhh {

constexpr uint64_t kFeP_ = kFieldFeP;

__constant__ WordTable c_T0_sk = T0;

// ---- FE, canonical representatives in [0, p) ---------------------------------------------
__device__ __forceinline__ uint64_t fe_addc(uint64_t a, uint64_t b) {
    const uint64_t s = a + b;
    return s >= kFeP_ ? s - kFeP_ : s;
}
__device__ __forceinline__ uint64_t fe_negc(uint64_t a) { return a ? kFeP_ - a : 0; }
__device__ __forceinline__ uint64_t fe_subc(uint64_t a, uint64_t b) { return fe_addc(a, fe_negc(b)); }
// a * b mod p, a, b < 2^63: 2^62 = 2^30 + 1 (mod p) folds the product twice (fastfield.rs:299-328)
__device__ __forceinline__ uint64_t fe_mulc(uint64_t a, uint64_t b) {
    const unsigned __int128 v = (unsigned __int128)a * b;
    const uint64_t mask = (1ull << 62) - 1;
    const unsigned __int128 h = v >> 62;
    const unsigned __int128 t = (v & mask) + h + (h << 30);
    const uint64_t h2 = (uint64_t)(t >> 62);
    uint64_t r = ((uint64_t)t & mask) + h2 + (h2 << 30);
    if (r >= kFeP_) r -= kFeP_;
    if (r >= kFeP_) r -= kFeP_;
    return r;
}
__device__ __forceinline__ uint64_t fe_canon_dev(uint64_t v) {   // any u64 val -> value()
    const uint64_t mask = (1ull << 62) - 1;
    uint64_t r = (v & mask) + (v >> 62) + ((v >> 62) << 30);
    if (r >= kFeP_) r -= kFeP_;
    if (r >= kFeP_) r -= kFeP_;
    return r;
}

// ---- AES-128 with a per-key schedule (the PrgStream cipher) -------------------------------
// Key schedule on little-endian column words (FIPS-197 5.2): RotWord = rotr 8, rcon in byte 0.
// SubWord reads S[x] = byte 1 of T0[x] from the LDS table (TabT0R32: entry x, replica lane % 32
// at word 32 x + lane % 32) — 4 independent ds_read_b32 per round instead of dependent scalar
// loads from constant memory.
__device__ __forceinline__ uint32_t sub_word(uint32_t w, const uint32_t* tbl, uint32_t rep) {
    uint32_t o = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) o |= ((tbl[(((w >> (8 * k)) & 0xFF) << 5) + rep] >> 8) & 0xFF) << (8 * k);
    return o;
}

__device__ __forceinline__ void key_schedule(const uint32_t key[4], uint32_t (&rk)[11][4], const uint32_t* tbl,
                                             uint32_t rep) {
    uint32_t w[44];
#pragma unroll
    for (int i = 0; i < 4; i++) w[i] = key[i];
    uint32_t rcon = 1;
#pragma unroll
    for (int i = 4; i < 44; i++) {
        uint32_t t = w[i - 1];
        if (i % 4 == 0) {
            t = sub_word((t >> 8) | (t << 24), tbl, rep) ^ rcon;
            rcon = ((rcon << 1) ^ ((rcon & 0x80) ? 0x1B : 0)) & 0xFF;
        }
        w[i] = w[i - 4] ^ t;
    }
#pragma unroll
    for (int r = 0; r < 11; r++)
#pragma unroll
        for (int c = 0; c < 4; c++) rk[r][c] = w[4 * r + c];
}

using SkTab = TabT0R32<DevOpsX>;
constexpr int kSketchThreads = 256;

// keystream block b (< 2^32): AES_seed(BE128(b)) -> two LE u64 draws (positions 2b, 2b+1)
__device__ __forceinline__ void ks_block(uint64_t b, const uint32_t* tbl, uint32_t b0, uint32_t b1,
                                         const uint32_t (&rk)[11][4], uint64_t& d0, uint64_t& d1) {
    uint32_t s[1][4] = {{0u, 0u, __builtin_bswap32((uint32_t)(b >> 32)), __builtin_bswap32((uint32_t)b)}};
    aes_rk<SkTab, 1>(s, tbl, b0, b1, rk);
    d0 = (uint64_t)s[0][0] | ((uint64_t)s[0][1] << 32);
    d1 = (uint64_t)s[0][2] | ((uint64_t)s[0][3] << 32);
}

// the same with the schedule expanded on the fly (k_sketch_fe's default form)
template <class Tab>
__device__ __forceinline__ void ks_block_otf(uint64_t b, const uint32_t* tbl, uint32_t b0, uint32_t b1,
                                             const uint32_t (&key)[4], uint64_t& d0, uint64_t& d1) {
    uint32_t s[1][4] = {{0u, 0u, __builtin_bswap32((uint32_t)(b >> 32)), __builtin_bswap32((uint32_t)b)}};
    aes_otf<Tab, 1>(s, tbl, b0, b1, key);
    d0 = (uint64_t)s[0][0] | ((uint64_t)s[0][1] << 32);
    d1 = (uint64_t)s[0][2] | ((uint64_t)s[0][3] << 32);
}

// draw `pos` of the key's stream (value v = low 62 bits): rand1..3 or node j = pos - 3
__device__ __forceinline__ void sketch_draw(uint64_t pos, uint64_t v, uint64_t xv, uint64_t kxv, uint64_t F,
                                            int h, bool& rej, uint64_t& rnd0, uint64_t& rnd1, uint64_t& rx,
                                            uint64_t& r2x, uint64_t& rkx) {
    if (pos < 3) {
        // lane 0 holds rand1, rand2 (block 0); lane 1 holds rand3 (block 1, draw 0)
        rej |= v >= kFeP_;
        if (h == 0) rnd0 = v;
        else rnd1 = v;
    } else if (pos < F + 3) {
        rej |= v >= kFeP_;
        const uint64_t r2 = fe_mulc(v, v);
        xv = fe_canon_dev(xv);
        rx = fe_addc(rx, fe_mulc(xv, v));
        r2x = fe_addc(r2x, fe_mulc(xv, r2));
        rkx = fe_addc(rkx, fe_mulc(fe_canon_dev(kxv), v));
    }
}

// v mod p for any v < 2^128 (three folds of 2^62 = 2^30 + 1, then canonical)
__device__ __forceinline__ uint64_t fe_red128(unsigned __int128 v) {
    const uint64_t mask = (1ull << 62) - 1;
#pragma unroll
    for (int i = 0; i < 2; i++) {
        const unsigned __int128 h = v >> 62;
        v = (v & mask) + h + (h << 30);
    }
    const uint64_t h = (uint64_t)(v >> 62);
    uint64_t r = ((uint64_t)v & mask) + h + (h << 30);
    if (r >= kFeP_) r -= kFeP_;
    if (r >= kFeP_) r -= kFeP_;
    return r;
}

// v^2 mod p for v < 2^62 (a masked draw): after the two folds r < 1.5 * 2^62 + 2^31, so one
// conditional subtraction makes it canonical (fe_mulc's second one is for operands up to 2^63)
__device__ __forceinline__ uint64_t fe_sqr62(uint64_t v) {
    const unsigned __int128 w = (unsigned __int128)v * v;
    const uint64_t mask = (1ull << 62) - 1;
    const unsigned __int128 h = w >> 62;
    const unsigned __int128 t = (w & mask) + h + (h << 30);
    const uint64_t h2 = (uint64_t)(t >> 62);
    const uint64_t r = ((uint64_t)t & mask) + h2 + (h2 << 30);
    return r >= kFeP_ ? r - kFeP_ : r;
}

// w mod p up to a multiple of p for w < 2^126: two folds of 2^62 = 2^30 + 1 leave
// r < 2^62 + 2^33 + 2^63 < 2^64, no subtraction (the caller only multiplies or adds it)
__device__ __forceinline__ uint64_t fe_fold126(unsigned __int128 w) {
    const uint64_t mask = (1ull << 62) - 1;
    const unsigned __int128 h = w >> 62;
    const unsigned __int128 t = (w & mask) + h + (h << 30);
    const uint64_t h2 = (uint64_t)(t >> 62);
    return ((uint64_t)t & mask) + h2 + (h2 << 30);
}

// sketch_draw with the three inner-product terms accumulated unreduced, one fe_red128 per
// accumulator per pass instead of a reduction per product.
// CANON = false (the fused kernel, at most 4 draws per pass) multiplies the stored x / kx words as
// they are (x = x' mod p gives the same sums mod p) and forms x r^2 as (x r) r: t = fold(x r) < 2^64
// is added to <r, x> and multiplied by r for <r^2, x> — 12 instead of 15 32-bit partial products
// per draw, no squaring. Every accumulator takes at most 4 products of a u64 word and a draw below
// 2^62 (plus a start below 2^62), so it stays below 2^128:
// 4 (2^64 - 1)(2^62 - 1) + 2^62 = 2^128 - 2^66 - 2^64 + 2^62 + 4.
// CANON = true (the producer / consumer form, 6 draws per phase) reduces x and kx first and squares
// the draw (products below 2^124).
template <bool CANON = true>
__device__ __forceinline__ void sketch_draw_lazy(uint64_t pos, uint64_t v, uint64_t xv, uint64_t kxv, uint64_t F,
                                                 int h, bool& rej, uint64_t& rnd0, uint64_t& rnd1,
                                                 unsigned __int128& ax, unsigned __int128& a2x,
                                                 unsigned __int128& akx) {
    // branch-free (pos depends on the lane): out-of-range positions carry x = kx = 0 (the loads
    // are skipped), so their products vanish; a divergent branch here would keep the compiler from
    // interleaving the pass's four independent draws
    const bool is_rand = pos < 3, live = pos < F + 3;
    rej |= live && v >= kFeP_;
    rnd0 = (is_rand && h == 0) ? v : rnd0;
    rnd1 = (is_rand && h == 1) ? v : rnd1;
    if constexpr (CANON) {
        const uint64_t r2 = fe_sqr62(v);
        xv = fe_canon_dev(xv);
        kxv = fe_canon_dev(kxv);
        ax += (unsigned __int128)xv * v;
        a2x += (unsigned __int128)xv * r2;
    } else {
        const uint64_t t = fe_fold126((unsigned __int128)xv * v);   // x r (mod p), < 2^64
        ax += t;
        a2x += (unsigned __int128)t * v;                            // x r^2 (mod p)
    }
    akx += (unsigned __int128)kxv * v;
}

__device__ __forceinline__ uint64_t wave_fe_sum(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fe_addc(v, __shfl_xor(v, off, 64));
    return v;
}

// segment (LPK lanes = one key) reductions
template <int LPK>
__device__ __forceinline__ uint64_t seg_fe_sum(uint64_t v) {
#pragma unroll
    for (int off = LPK / 2; off > 0; off >>= 1) v = fe_addc(v, __shfl_xor(v, off, 64));
    return v;
}

// The sequential PrgStream with FE::from_rng redraws (field.rs:252-264) for one key, one lane:
// the path of a key whose parallel draws hit a value >= p (P ~ 2^-32 per draw) and of the
// force_sequential tests. Out of line so its registers do not weigh on the parallel loop.
template <class Tab>
__device__ __noinline__ void sketch_sequential_otf(const uint32_t* tbl, uint32_t b0, uint32_t b1,
                                                   const uint32_t (&seed)[4], const uint64_t* x, const uint64_t* kx,
                                                   uint64_t F, uint64_t* o) {
    const uint64_t mask = (1ull << 62) - 1;
    uint64_t pos = 0, cur_b = ~0ull, d[2] = {0, 0};
    auto draw = [&]() -> uint64_t {
        for (;;) {
            const uint64_t b = pos >> 1;
            if (b != cur_b) {
                ks_block_otf<Tab>(b, tbl, b0, b1, seed, d[0], d[1]);
                cur_b = b;
            }
            const uint64_t v = d[pos & 1] & mask;
            pos++;
            if (v < kFeP_) return v;
        }
    };
    const uint64_t q1 = draw(), q2 = draw(), q3 = draw();
    uint64_t sx = 0, s2x = 0, skx = 0;
    for (uint64_t j = 0; j < F; j++) {
        const uint64_t r = draw();
        const uint64_t r2 = fe_mulc(r, r);
        const uint64_t xv = fe_canon_dev(x[j]), kxv = fe_canon_dev(kx[j]);
        sx = fe_addc(sx, fe_mulc(xv, r));
        s2x = fe_addc(s2x, fe_mulc(xv, r2));
        skx = fe_addc(skx, fe_mulc(kxv, r));
    }
    o[0] = sx;
    o[1] = s2x;
    o[2] = skx;
    o[3] = q1;
    o[4] = q2;
    o[5] = q3;
}

// KPW keys per wave, LPK = 64 / KPW lanes per key: lane l of a key's segment produces keystream
// blocks l, l + LPK, ... two per pass in lockstep, with the pass's (x, kx) loads issued first.
// The key differs per segment, so the schedule is per lane: OTF = false keeps all 11 round keys
// in VGPRs (r01: T0 + rotations, 256 threads, 157 VGPRs, 3 waves/SIMD); OTF = true expands it on
// the fly per pass (4 extra lookups per round, shared by the pass's two blocks), which with the
// four-table LDS layout (one v_perm per lookup) fits 1024 threads x <= 128 VGPRs.
// SCHED 2: the schedule is computed once per key (every lane of the segment, through the tables)
// and kept in LDS beside the tables (16 waves x KPW keys x 176 B = 22.5 KiB at KPW 8); a round
// reads it with one broadcast ds_read_b128 instead of 4 lookups + the SubWord chain per pass.
template <int KPW, class Tab = SkTab, int THR = kSketchThreads, int SCHED = 0, int NBP = 2>
__global__ __launch_bounds__(THR) void k_sketch_fe(SketchArgs a) {
    constexpr bool OTF = SCHED >= 1;   // lazy sums, out-of-line fallback, key expanded through Tab
    constexpr int LPK = 64 / KPW;
    __shared__ uint32_t tbl[Tab::kWords];
    __shared__ uint4 rks_lds[SCHED == 2 ? THR / 64 : 1][SCHED == 2 ? KPW : 1][11];
    for (int i = threadIdx.x; i < Tab::kWords; i += THR) tbl[i] = Tab::word(c_T0_sk.v, i);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t seg = lane / LPK, sl = lane % LPK;
    uint32_t b0, b1;
    Tab::bases(lane, b0, b1);
    const uint64_t mask = (1ull << 62) - 1;
    const uint64_t nwaves = (uint64_t)gridDim.x * (THR / 64);
    const uint64_t F = a.n_nodes;
    const uint64_t nb = (F + 3 + 1) / 2;   // draws 0..F+2
    const uint64_t wave = (uint64_t)blockIdx.x * (THR / 64) + (threadIdx.x >> 6);
    for (uint64_t kbase = wave * KPW; kbase < a.n_keys; kbase += nwaves * KPW) {
        const uint64_t k_all = kbase + seg;
        const bool kact = k_all < a.n_keys;
        // the two-server form: keys past n_srv are server 1's (same seeds, its own vectors and outputs)
        const bool srv1 = a.n_srv && (kact ? k_all : kbase) >= a.n_srv;
        const uint64_t k = srv1 ? k_all - a.n_srv : k_all;
        const uint64_t kk = kact ? k : (srv1 ? kbase - a.n_srv : kbase);
        const uint64_t* const xs = srv1 ? a.x1 : a.x;
        const uint64_t* const kxs = srv1 ? a.kx1 : a.kx;
        uint64_t* const outs = srv1 ? a.out1 : a.out;
        uint32_t seed[4];
#pragma unroll
        for (int c = 0; c < 4; c++) seed[c] = reinterpret_cast<const uint32_t*>(a.seeds)[4 * kk + c];
        seed[3] ^= a.level;   // the level's stream (bytes 12..15; level 0 = the seed itself)
        uint32_t rk[OTF ? 1 : 11][4];
        if constexpr (!OTF) key_schedule(seed, rk, tbl, lane & 31);
        const uint4* rkl = rks_lds[SCHED == 2 ? (threadIdx.x >> 6) : 0][SCHED == 2 ? seg : 0];
        if constexpr (SCHED == 2) {
            uint32_t full[11][4];
            key_schedule_tab<Tab>(seed, full, tbl, b0, b1);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // the previous key's reads are done
            if (sl == 0) {
                uint4* w = rks_lds[threadIdx.x >> 6][seg];
#pragma unroll
                for (int r = 0; r < 11; r++) w[r] = make_uint4(full[r][0], full[r][1], full[r][2], full[r][3]);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            __builtin_amdgcn_wave_barrier();
        }
        // r05: when every block of the key's stream (and the passes' overrun) has a counter below 256,
        // all of them differ only in byte 15, so rounds 1-2 keep a per-key constant part: paid here once
        // (aes_ctr_pre_init), then 5 instead of 32 lookups per block in rounds 1-2 (aes_ctr_pre: 133
        // lookups per block against 146.5 for aes_ctr_shared's pairs)
        const bool pre_ok = SCHED == 2 && nb + (uint64_t)NBP * LPK <= 256;   // wave-uniform
        uint32_t pre[6] = {0, 0, 0, 0, 0, 0};
        if constexpr (SCHED == 2) {
            if (pre_ok) {
                const uint32_t z[4] = {0u, 0u, 0u, 0u};   // counter 0: BE128(0)
                aes_ctr_pre_init<Tab, 3, 3>(z, tbl, b0, b1, RkLds{rkl}, pre);
            }
        }
        const uint64_t* x = xs + kk * F;
        const uint64_t* kx = kxs + kk * F;
        uint64_t rx = 0, r2x = 0, rkx = 0, rnd0 = 0, rnd1 = 0;
        bool rej = false;
        // one pass: NB keystream blocks per lane (bb, bb + LPK, ...) and their draws' products
        auto pass = [&](uint64_t bb, auto nbc) {
            constexpr int NB = decltype(nbc)::value;
            // the pass's (x, kx) loads go ahead of the AES at 2 blocks per pass; at 4 their 32
            // registers would be live across it, so they follow it (other waves hide the latency)
            uint64_t xv[2 * NB] = {}, kxv[2 * NB] = {};
            auto load_xkx = [&]() {
#pragma unroll
                for (int q = 0; q < NB; q++)
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const uint64_t pos = 2 * (bb + LPK * q) + h;
                        if (pos >= 3 && pos < F + 3) {
                            xv[2 * q + h] = x[pos - 3];
                            kxv[2 * q + h] = kx[pos - 3];
                        }
                    }
            };
            if constexpr (NB <= 2) load_xkx();
            uint32_t st[NB][4];
#pragma unroll
            for (int q = 0; q < NB; q++) {
                const uint64_t b = bb + LPK * q;
                st[q][0] = 0u;
                st[q][1] = 0u;
                st[q][2] = __builtin_bswap32((uint32_t)(b >> 32));
                st[q][3] = __builtin_bswap32((uint32_t)b);
            }
            if constexpr (SCHED == 2) {
                // the pass's counters differ only in byte 15 (the low byte of the big-endian
                // block index) unless a lane's blocks straddle a multiple of 256: then rounds 1-2
                // of the second block reuse the first's terms (aes_ctr_shared, 293 vs 320 lookups)
                const bool same_hi = (bb >> 8) == ((bb + LPK * (NB - 1)) >> 8);
                if (pre_ok) aes_ctr_pre<Tab, NB, 3, 3>(st, tbl, b0, b1, RkLds{rkl}, pre);
                else if (NB == 1 || __ballot(!same_hi) == 0) aes_lds_rk_ctr<Tab, NB, 3, 3>(st, tbl, b0, b1, rkl);
                else aes_lds_rk<Tab, NB>(st, tbl, b0, b1, rkl);
            } else if constexpr (OTF) aes_otf<Tab, NB>(st, tbl, b0, b1, seed);
            else aes_rk<Tab, NB>(st, tbl, b0, b1, rk);
            if constexpr (NB > 2) load_xkx();
            unsigned __int128 ax = rx, a2x = r2x, akx = rkx;
#pragma unroll
            for (int q = 0; q < NB; q++) {
                const uint64_t b = bb + LPK * q;
                if (!OTF && b >= nb) break;   // OTF: positions past the stream are no-ops
                const uint64_t dr[2] = {(uint64_t)st[q][0] | ((uint64_t)st[q][1] << 32),
                                        (uint64_t)st[q][2] | ((uint64_t)st[q][3] << 32)};
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    if constexpr (OTF)
                        sketch_draw_lazy<(2 * NB > 4)>(2 * b + h, dr[h] & mask, xv[2 * q + h], kxv[2 * q + h], F, h,
                                                       rej, rnd0, rnd1, ax, a2x, akx);
                    else
                        sketch_draw(2 * b + h, dr[h] & mask, xv[2 * q + h], kxv[2 * q + h], F, h, rej, rnd0, rnd1,
                                    rx, r2x, rkx);
                }
            }
            if constexpr (OTF) {
                rx = fe_red128(ax);
                r2x = fe_red128(a2x);
                rkx = fe_red128(akx);
            }
        };
        if (!a.force_sequential) {
            for (uint64_t bb = sl; bb < nb; bb += NBP * LPK) {
                // a pass whose blocks past the first are beyond the stream on every lane (the last
                // pass of a 130-block key at LPK 8: blocks 128, 129) runs one block per lane: about
                // half the AES and products of a full pass (OTF: past-the-stream positions are no-ops)
                if (OTF && NBP > 1 && __ballot(bb + LPK < nb) == 0) pass(bb, std::integral_constant<int, 1>{});
                else pass(bb, std::integral_constant<int, NBP>{});
            }
        }
        // per-key rejection flag over the key's segment
        const uint64_t rej_mask = __ballot(rej);
        const uint64_t seg_bits = (LPK == 64 ? ~0ull : ((1ull << LPK) - 1)) << (seg * LPK);
        const bool key_rej = a.force_sequential || (rej_mask & seg_bits) != 0;
        rx = seg_fe_sum<LPK>(rx);
        r2x = seg_fe_sum<LPK>(r2x);
        rkx = seg_fe_sum<LPK>(rkx);
        const uint64_t rand1 = __shfl(rnd0, seg * LPK, 64);
        const uint64_t rand2 = __shfl(rnd1, seg * LPK, 64);
        const uint64_t rand3 = __shfl(rnd0, seg * LPK + 1, 64);
        if (kact && !key_rej && sl == 0) {
            uint64_t* o = outs + 6 * k;
            o[0] = rx;
            o[1] = r2x;
            o[2] = rkx;
            o[3] = rand1;
            o[4] = rand2;
            o[5] = rand3;
        } else if (kact && key_rej && sl == 0 && OTF) {
            sketch_sequential_otf<Tab>(tbl, b0, b1, seed, x, kx, F, outs + 6 * k);
        } else if (kact && key_rej && sl == 0) {
            // sequential PrgStream with FE::from_rng redraws (field.rs:252-264) for this key
            uint64_t pos = 0, cur_b = ~0ull, d[2] = {0, 0};
            auto draw = [&]() -> uint64_t {
                for (;;) {
                    const uint64_t b = pos >> 1;
                    if (b != cur_b) {
                        if constexpr (!OTF) ks_block(b, tbl, b0, b1, rk, d[0], d[1]);
                        cur_b = b;
                    }
                    const uint64_t v = d[pos & 1] & mask;
                    pos++;
                    if (v < kFeP_) return v;
                }
            };
            const uint64_t q1 = draw(), q2 = draw(), q3 = draw();
            uint64_t sx = 0, s2x = 0, skx = 0;
            for (uint64_t j = 0; j < F; j++) {
                const uint64_t r = draw();
                const uint64_t r2 = fe_mulc(r, r);
                const uint64_t xv = fe_canon_dev(x[j]), kxv = fe_canon_dev(kx[j]);
                sx = fe_addc(sx, fe_mulc(xv, r));
                s2x = fe_addc(s2x, fe_mulc(xv, r2));
                skx = fe_addc(skx, fe_mulc(kxv, r));
            }
            uint64_t* o = outs + 6 * k;
            o[0] = sx;
            o[1] = s2x;
            o[2] = skx;
            o[3] = q1;
            o[4] = q2;
            o[5] = q3;
        }
    }
}

// ---- producer / consumer form (r03) --------------------------------------------------------
// PMC put the fused kernel at 0.33 of VALU and 0.35 of LDS issue: every wave runs a pass's AES
// (LDS-bound) and then its FE products (VALU-bound, ~63 % of the VALU instructions), and the waves
// of a workgroup stay in step, so the two phases add instead of overlapping. Here the roles are
// split: waves 0..7 of the 1024-thread workgroup only run the keystream AES and waves 8..15 only the
// draws' products; wave w and wave w + 8 form a pair that hands over a phase's blocks (PCB per lane)
// through LDS. A phase: the producers run the AES of pass g into registers while the consumers
// multiply out pass g - 1 from the buffer; barrier; the producers store pass g; barrier. Waves are
// dealt to SIMDs round-robin, so every SIMD holds two producers and two consumers, and the consumers'
// VALU work fills the slots the producers leave while they wait on the LDS.
// A pair task = KPW keys at LPK = 64 / KPW lanes per key; lane l of a key's segment takes keystream
// blocks (PCB p + q) LPK + l, q < PCB, in pass p, so a task is ceil(nb / (PCB LPK)) phases, and the
// pairs of the grid run the tasks in rounds (uniform across the grid, so every wave meets every
// barrier). The consumer issues its next pass's (x, kx) loads one phase ahead. LDS: 128 KiB tables +
// the hand-over buffer, 8 pairs x PCB x 64 lanes x 16 B = 24 KiB at PCB = 3 (152 KiB; the producers
// keep their keys' schedules in VGPRs).
constexpr int kPcPairs = 8;
constexpr int kPcThreads = 1024;
// keystream blocks per producer lane per phase: 3, with the key's schedule kept in VGPRs (4 with the
// schedule expanded on the fly spilled in the consumer and ran 287.6 vs 235.6 us per launch, r03)
constexpr int kPcBlocks = 3;

template <int KPW, int PCB = kPcBlocks>
__global__ __launch_bounds__(kPcThreads) void k_sketch_fe_pc(SketchArgs a) {
    constexpr int LPK = 64 / KPW;
    using Tab = Tab4T32<DevOpsX>;
    __shared__ uint32_t tbl[Tab::kWords];
    __shared__ uint4 buf[kPcPairs][PCB][64];
    static_assert(sizeof(tbl) + sizeof(buf) <= 160 * 1024, "k_sketch_fe_pc: static LDS above the CU's 160 KiB");
    for (int i = threadIdx.x; i < Tab::kWords; i += kPcThreads) tbl[i] = Tab::word(c_T0_sk.v, i);
    __syncthreads();
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const bool prod = wv < kPcPairs;
    const uint32_t pair = prod ? wv : wv - kPcPairs;
    const uint32_t seg = lane / LPK, sl = lane % LPK;
    uint32_t b0, b1;
    Tab::bases(lane, b0, b1);
    const uint64_t mask = (1ull << 62) - 1;
    const uint64_t F = a.n_nodes;
    const uint64_t nb = (F + 3 + 1) / 2;   // keystream blocks per key: draws 0..F+2
    const uint64_t passes = (nb + PCB * LPK - 1) / (PCB * LPK);
    const uint64_t ntasks = (a.n_keys + KPW - 1) / KPW;
    const uint64_t pairs_total = (uint64_t)gridDim.x * kPcPairs;
    const uint64_t rounds = (ntasks + pairs_total - 1) / pairs_total;
    const uint64_t steps = rounds * passes;   // producer phases; the consumer trails by one
    auto task_of = [&](uint64_t step, uint64_t& p) -> uint64_t {   // step -> (task, pass p)
        const uint64_t round = step / passes;
        p = step - round * passes;
        return round * pairs_total + (uint64_t)blockIdx.x * kPcPairs + pair;
    };
    // the two roles run separate loops (so neither's loop-carried registers weigh on the other)
    // with the same two barriers per phase
    if (prod) {
        uint32_t rk[11][4];   // the lane's key's schedule (its segment's key), kept for the task
        for (uint64_t g = 0; g <= steps; g++) {
            uint32_t st[PCB][4];
            uint64_t p;
            const uint64_t task = g < steps ? task_of(g, p) : ntasks;
            const bool produced = task < ntasks;   // wave-uniform
            if (produced) {
                const uint64_t k = task * KPW + seg;
                const uint64_t kk = k < a.n_keys ? k : task * KPW;
                if (p == 0) {   // the task's key schedules, once per key, through the tables
                    uint32_t seed[4];
#pragma unroll
                    for (int c = 0; c < 4; c++) seed[c] = reinterpret_cast<const uint32_t*>(a.seeds)[4 * kk + c];
                    seed[3] ^= a.level;   // the level's stream (bytes 12..15)
                    key_schedule_tab<Tab>(seed, rk, tbl, b0, b1);
                }
#pragma unroll
                for (int q = 0; q < PCB; q++) {
                    const uint64_t b = (PCB * p + q) * LPK + sl;
                    st[q][0] = 0u;
                    st[q][1] = 0u;
                    st[q][2] = __builtin_bswap32((uint32_t)(b >> 32));
                    st[q][3] = __builtin_bswap32((uint32_t)b);
                }
                {   // counters differing only in byte 15 (see k_sketch_fe): shared rounds 1-2
                    const uint64_t bf = PCB * p * LPK + sl, bl = (PCB * p + PCB - 1) * LPK + sl;
                    if (__ballot((bf >> 8) != (bl >> 8)) == 0) aes_rk_ctr<Tab, PCB, 3, 3>(st, tbl, b0, b1, rk);
                    else aes_rk<Tab, PCB>(st, tbl, b0, b1, rk);
                }
            }
            __syncthreads();   // the consumers are done with the buffer
            if (produced) {
#pragma unroll
                for (int q = 0; q < PCB; q++) buf[pair][q][lane] = make_uint4(st[q][0], st[q][1], st[q][2], st[q][3]);
            }
            __syncthreads();   // pass g is in the buffer
        }
        return;
    }
    unsigned __int128 ax = 0, a2x = 0, akx = 0;
    uint64_t rnd0 = 0, rnd1 = 0, xv_n[2 * PCB] = {}, kxv_n[2 * PCB] = {};
    bool rej = false;
    auto load_xkx = [&](uint64_t step) {   // the (x, kx) of the lane's 2 PCB draws of `step`
        uint64_t p;
        const uint64_t task = task_of(step, p);
#pragma unroll
        for (int i = 0; i < 2 * PCB; i++) xv_n[i] = kxv_n[i] = 0;
        if (task >= ntasks) return;
        const uint64_t k = task * KPW + seg;
        if (k >= a.n_keys) return;
#pragma unroll
        for (int q = 0; q < PCB; q++)
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const uint64_t pos = 2 * ((PCB * p + q) * LPK + sl) + h;
                if (pos >= 3 && pos < F + 3) {
                    xv_n[2 * q + h] = a.x[k * F + pos - 3];
                    kxv_n[2 * q + h] = a.kx[k * F + pos - 3];
                }
            }
    };
    if (steps > 0) load_xkx(0);
    for (uint64_t g = 0; g <= steps; g++) {
        if (g > 0) {
            const uint64_t step = g - 1;
            uint64_t p;
            const uint64_t task = task_of(step, p);
            const uint64_t* xv = xv_n;
            const uint64_t* kxv = kxv_n;
            if (task < ntasks) {   // wave-uniform
                const uint64_t k = task * KPW + seg;
                const bool kact = k < a.n_keys;
                if (p == 0) {
                    ax = a2x = akx = 0;
                    rnd0 = rnd1 = 0;
                    rej = false;
                }
#pragma unroll
                for (int q = 0; q < PCB; q++) {
                    const uint4 s = buf[pair][q][lane];
                    const uint64_t b = (PCB * p + q) * LPK + sl;
                    const uint64_t dr[2] = {(uint64_t)s.x | ((uint64_t)s.y << 32), (uint64_t)s.z | ((uint64_t)s.w << 32)};
#pragma unroll
                    for (int h = 0; h < 2; h++)   // positions past the stream carry x = kx = 0: no-ops
                        sketch_draw_lazy<(2 * PCB > 4)>(2 * b + h, dr[h] & mask, xv[2 * q + h], kxv[2 * q + h], F, h,
                                                        rej, rnd0, rnd1,
                                         ax, a2x, akx);
                }
                ax = fe_red128(ax);
                a2x = fe_red128(a2x);
                akx = fe_red128(akx);
                if (step + 1 < steps) load_xkx(step + 1);   // a phase ahead: they land during the barriers
                if (p == passes - 1) {
                    const uint64_t rej_mask = __ballot(rej);
                    const uint64_t seg_bits = (LPK == 64 ? ~0ull : ((1ull << LPK) - 1)) << (seg * LPK);
                    const bool key_rej = a.force_sequential || (rej_mask & seg_bits) != 0;
                    const uint64_t rx = seg_fe_sum<LPK>((uint64_t)ax), r2x = seg_fe_sum<LPK>((uint64_t)a2x),
                                   rkx = seg_fe_sum<LPK>((uint64_t)akx);
                    const uint64_t rand1 = __shfl(rnd0, seg * LPK, 64);
                    const uint64_t rand2 = __shfl(rnd1, seg * LPK, 64);
                    const uint64_t rand3 = __shfl(rnd0, seg * LPK + 1, 64);
                    if (kact && sl == 0) {
                        if (!key_rej) {
                            uint64_t* o = a.out + 6 * k;
                            o[0] = rx;
                            o[1] = r2x;
                            o[2] = rkx;
                            o[3] = rand1;
                            o[4] = rand2;
                            o[5] = rand3;
                        } else {
                            // a from_rng redraw (P ~ 2^-32 per draw) or force_sequential: this lane
                            // replays the key's sequential stream; the workgroup's other waves wait
                            // for it at the phase barrier (correct, and rare outside the tests)
                            uint32_t seed[4];
#pragma unroll
                            for (int c = 0; c < 4; c++) seed[c] = reinterpret_cast<const uint32_t*>(a.seeds)[4 * k + c];
                            seed[3] ^= a.level;
                            sketch_sequential_otf<Tab>(tbl, b0, b1, seed, a.x + k * F, a.kx + k * F, F, a.out + 6 * k);
                        }
                    }
                }
            }
        }
        __syncthreads();   // the producers may overwrite the buffer
        __syncthreads();   // the next pass is in the buffer
    }
}

constexpr int kSketchKeysPerWave = 4;
// default form: 8 keys per wave (8 lanes per key: at 256 nodes 130 blocks fill 9 passes of 16
// slots, 90 % of the slots), four-table LDS layout, 1024 threads, round keys in LDS
constexpr int kSketchKpwOtf = 8;
constexpr int kSketchThreadsOtf = 1024;
constexpr int kSketchNbpOtf = 2;   // 4 blocks per pass (16 keys per wave) spills at 128 VGPRs: 0.88 vs 0.66 ms/level
using SkTab4 = Tab4T32<DevOpsX>;

template <class K>
static hipError_t launch_sketch_kernel(K kern, int thr, int kpw, const SketchArgs& a, hipStream_t stream) {
    int cus = 256, dev = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern), thr, 0) !=
            hipSuccess || per_cu < 1)
        per_cu = 1;
    const uint64_t wpb = thr / 64;
    const uint64_t waves_needed = (a.n_keys + kpw - 1) / kpw;
    uint64_t blocks = (waves_needed + wpb - 1) / wpb;
    const uint64_t cap = (uint64_t)cus * per_cu;   // one resident wave set; keys are strided over it
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(thr), 0, stream, a);
    return hipGetLastError();
}

// The default form with the key-to-wave granularity chosen per launch. Keys are strided over one
// resident wave set (W = CUs x 16 waves), a task = KPW keys of LPK = 64 / KPW lanes each, so a
// launch takes ceil(tasks / W) rounds of ceil(ceil(nb / LPK) / NBP) passes. At configs[4] (100k
// keys, 256 nodes, nb = 130) LPK 8 alone needs 3.05 rounds: the fourth runs 212 of 4096 waves for
// as long as a full round (the kernel is latency-bound, a lone wave is not faster), 36 passes where
// 24.8 would do. plan_sketch splits such a launch: R full LPK-8 rounds, then the remaining keys in
// one launch with the LPK that needs the fewest passes (LPK 64: 1 round of 2 passes), 29 in all.
template <int KPW>
static hipError_t launch_sketch_lds(const SketchArgs& a, hipStream_t stream) {
    return launch_sketch_kernel(k_sketch_fe<KPW, SkTab4, kSketchThreadsOtf, 2, kSketchNbpOtf>, kSketchThreadsOtf, KPW,
                                a, stream);
}

static hipError_t launch_sketch_lpk(int lpk, const SketchArgs& a, hipStream_t stream) {
    if (a.n_keys == 0) return hipSuccess;
    switch (lpk) {
        case 8: return launch_sketch_lds<8>(a, stream);
        case 16: return launch_sketch_lds<4>(a, stream);
        case 32: return launch_sketch_lds<2>(a, stream);
        default: return launch_sketch_lds<1>(a, stream);
    }
}

// resident waves of the LDS-schedule kernel on the current device (cached per device)
static uint64_t sketch_resident_waves() {
    static std::atomic<uint64_t> cache[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
    uint64_t w = cache[dev].load(std::memory_order_relaxed);
    if (!w) {
        int cus = 256, per_cu = 0;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &per_cu, reinterpret_cast<const void*>(k_sketch_fe<8, SkTab4, kSketchThreadsOtf, 2, kSketchNbpOtf>),
                kSketchThreadsOtf, 0) != hipSuccess || per_cu < 1)
            per_cu = 1;
        w = (uint64_t)(cus > 0 ? cus : 256) * per_cu * (kSketchThreadsOtf / 64);
        cache[dev].store(w, std::memory_order_relaxed);
    }
    return w;
}

// cost in passes of one launch of n keys at LPK lanes per key (+ half a pass per round for the key
// schedule, the reductions and the stores)
static double sketch_launch_cost(uint64_t n, uint64_t nb, int lpk, uint64_t W, int nbp = kSketchNbpOtf) {
    if (n == 0) return 0.0;
    const uint64_t kpw = 64 / lpk, tasks = (n + kpw - 1) / kpw, rounds = (tasks + W - 1) / W;
    const uint64_t passes = ((nb + lpk - 1) / lpk + nbp - 1) / nbp;
    return (double)rounds * ((double)passes + 0.5);
}

// W = resident waves (fused form, nbp = 2 blocks per lane per pass) or resident producer / consumer
// pairs (nbp = kPcBlocks = 3 blocks per producer lane per phase)
SketchPlan plan_sketch_nbp(uint64_t n_keys, uint32_t n_nodes, uint64_t W, int nbp);
SketchPlan plan_sketch(uint64_t n_keys, uint32_t n_nodes, uint64_t W) {
    return plan_sketch_nbp(n_keys, n_nodes, W, kSketchNbpOtf);
}

SketchPlan plan_sketch_nbp(uint64_t n_keys, uint32_t n_nodes, uint64_t W, int nbp) {
    static const int kLpk[4] = {8, 16, 32, 64};
    const uint64_t nb = ((uint64_t)n_nodes + 4) / 2;
    SketchPlan best{n_keys, 8, 8};
    double best_cost = sketch_launch_cost(n_keys, nb, 8, W, nbp);
    for (int L : kLpk) {   // one launch (ties keep the smaller LPK: less redundant schedule work)
        const double c = sketch_launch_cost(n_keys, nb, L, W, nbp);
        if (c < best_cost) best_cost = c, best = SketchPlan{n_keys, L, L};
    }
    for (int Lm : kLpk) {   // R full rounds at Lm, the rest at Lt (+ half a pass for the second launch)
        const uint64_t kpw = 64 / Lm, R = n_keys / kpw / W;
        if (R == 0) continue;
        const uint64_t n_main = R * W * kpw;
        if (n_main >= n_keys) continue;
        for (int Lt : kLpk) {
            const double c = sketch_launch_cost(n_main, nb, Lm, W, nbp) + sketch_launch_cost(n_keys - n_main, nb, Lt, W, nbp) + 0.5;
            if (c < best_cost) best_cost = c, best = SketchPlan{n_main, Lm, Lt};
        }
    }
    return best;
}

extern "C" int fhh_sketch_plan(uint64_t n_keys, uint32_t n_nodes, uint64_t resident_waves, uint64_t* n_main,
                               int* lpk_main, int* lpk_tail) {
    if (!n_main || !lpk_main || !lpk_tail || resident_waves == 0) return FHH_E_ARG;
    const SketchPlan p = plan_sketch(n_keys, n_nodes, resident_waves);
    *n_main = p.n_main;
    *lpk_main = p.lpk_main;
    *lpk_tail = p.lpk_tail;
    return FHH_OK;
}

// impl (fhh_sketch_set_impl): 0 = default (schedule once per key in LDS, 1024 threads, planned
// key granularity), 1 = the r01 kernel, 2 = the schedule expanded on the fly per pass, 3 = the
// default kernel at LPK 8 for every key (the form before plan_sketch)
static int g_sketch_impl = 0;
extern "C" int fhh_sketch_set_impl(int impl) {
    if (impl < 0 || impl > 4) return FHH_E_ARG;
    g_sketch_impl = impl;
    return FHH_OK;
}

// the producer / consumer form: one 1024-thread workgroup per CU (155 KiB of LDS), the same
// planned split of the keys over lanes-per-key as the fused form, priced at kPcBlocks per phase
template <int KPW>
static hipError_t launch_sketch_pc_kpw(const SketchArgs& a, int cus, hipStream_t stream) {
    const uint64_t tasks = (a.n_keys + KPW - 1) / KPW;
    uint64_t blocks = (tasks + kPcPairs - 1) / kPcPairs;
    if (blocks > (uint64_t)cus) blocks = (uint64_t)cus;
    hipLaunchKernelGGL(k_sketch_fe_pc<KPW>, dim3((unsigned)blocks), dim3(kPcThreads), 0, stream, a);
    return hipGetLastError();
}

static hipError_t launch_sketch_pc_lpk(int lpk, const SketchArgs& a, int cus, hipStream_t stream) {
    if (a.n_keys == 0) return hipSuccess;
    switch (lpk) {
        case 8: return launch_sketch_pc_kpw<8>(a, cus, stream);
        case 16: return launch_sketch_pc_kpw<4>(a, cus, stream);
        case 32: return launch_sketch_pc_kpw<2>(a, cus, stream);
        default: return launch_sketch_pc_kpw<1>(a, cus, stream);
    }
}

// CU count of the current device, queried once per device (the sketch launches run per level; the
// shard threads of a multi-device ctx may fill the cache concurrently, hence the atomics)
static int sketch_cus() {
    static std::atomic<int> cache[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int cus = cache[dev].load(std::memory_order_relaxed);
    if (!cus) {
        if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
        cache[dev].store(cus, std::memory_order_relaxed);
    }
    return cus;
}

static hipError_t launch_sketch_pc(const SketchArgs& a, hipStream_t stream) {
    const int cus = sketch_cus();
    const SketchPlan p = plan_sketch_nbp(a.n_keys, a.n_nodes, (uint64_t)cus * kPcPairs, kPcBlocks);
    SketchArgs m = a;
    m.n_keys = p.n_main;
    hipError_t e = launch_sketch_pc_lpk(p.lpk_main, m, cus, stream);
    if (e != hipSuccess || p.n_main == a.n_keys) return e;
    SketchArgs t = a;
    t.seeds = a.seeds + 16 * p.n_main;
    t.x = a.x ? a.x + p.n_main * a.n_nodes : nullptr;
    t.kx = a.kx ? a.kx + p.n_main * a.n_nodes : nullptr;
    t.out = a.out + 6 * p.n_main;
    t.n_keys = a.n_keys - p.n_main;
    return launch_sketch_pc_lpk(p.lpk_tail, t, cus, stream);
}

hipError_t launch_sketch_fe(const SketchArgs& a, hipStream_t stream) { return launch_sketch_fe2(a, stream, stream); }

// the default form's main launch on `stream`, its tail launch (the keys past n_main, disjoint outputs)
// on `tail_stream`: a caller with a second stream lets the tail fill the main launch's ragged end
hipError_t launch_sketch_fe2(const SketchArgs& a, hipStream_t stream, hipStream_t tail_stream) {
    if (a.n_keys == 0) return hipSuccess;
    if (g_sketch_impl == 4 && a.n_srv) {   // the producer / consumer kernel takes one server at a time
        for (int srv = 0; srv < 2; srv++) {
            SketchArgs o = a;
            o.n_srv = 0;
            o.n_keys = srv ? a.n_keys - a.n_srv : a.n_srv;
            if (srv) {
                o.x = a.x1;
                o.kx = a.kx1;
                o.out = a.out1;
            }
            const hipError_t e = launch_sketch_pc(o, stream);
            if (e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    if (g_sketch_impl == 4) return launch_sketch_pc(a, stream);
    if (g_sketch_impl == 1)
        return launch_sketch_kernel(k_sketch_fe<kSketchKeysPerWave>, kSketchThreads, kSketchKeysPerWave, a, stream);
    if (g_sketch_impl == 2)
        return launch_sketch_kernel(k_sketch_fe<kSketchKpwOtf, SkTab4, kSketchThreadsOtf, 1, kSketchNbpOtf>,
                                    kSketchThreadsOtf, kSketchKpwOtf, a, stream);
    if (g_sketch_impl == 3) return launch_sketch_lpk(8, a, stream);
    const SketchPlan p = plan_sketch(a.n_keys, a.n_nodes, sketch_resident_waves());
    SketchArgs m = a;
    m.n_keys = p.n_main;
    hipError_t e = launch_sketch_lpk(p.lpk_main, m, stream);
    if (e != hipSuccess || p.n_main == a.n_keys) return e;
    // the tail: the keys past n_main, in one round of the producer / consumer form (r03, configs[4]: its
    // 3 blocks per lane cover a 130-block key at LPK 64 in one pass where the fused form takes two: 16.2
    // vs 28.8 us; the main launch stays fused, 227 vs 236 us); one launch per server the tail touches
    const uint64_t ns = a.n_srv ? a.n_srv : a.n_keys;
    for (int srv = 0; srv < (a.n_srv ? 2 : 1); srv++) {
        const uint64_t lo = std::max<uint64_t>(p.n_main, srv * ns), hi = srv ? a.n_keys : std::min(a.n_keys, ns);
        if (lo >= hi) continue;
        const uint64_t off = lo - srv * ns;   // the server's first tail key
        SketchArgs t = a;
        t.n_srv = 0;
        t.seeds = a.seeds + 16 * off;
        const uint64_t* xs = srv ? a.x1 : a.x;
        const uint64_t* kxs = srv ? a.kx1 : a.kx;
        t.x = xs ? xs + off * a.n_nodes : nullptr;
        t.kx = kxs ? kxs + off * a.n_nodes : nullptr;
        t.out = (srv ? a.out1 : a.out) + 6 * off;
        t.n_keys = hi - lo;
        e = launch_sketch_pc_lpk(p.lpk_tail, t, sketch_cus(), tail_stream);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// ---- MulState (mpc.rs:83-220), FE, one lane per key ---------------------------------------
// MulState::new: xs = [r_x, k, r_x], ys = [r_x, k, k], zs = [-r2_x, -k2, -r_kx],
// rs = [rand1, rand2, rand3] (sketch6 = {r_x, r2_x, r_kx, rand1, rand2, rand3}).
struct MulView {
    uint64_t xs[3], ys[3], zs[3], rs[3];
};

__device__ __forceinline__ MulView mul_view(const uint64_t* sk, uint64_t mac, uint64_t mac2) {
    MulView m;
    const uint64_t rx = fe_canon_dev(sk[0]), r2x = fe_canon_dev(sk[1]), rkx = fe_canon_dev(sk[2]);
    mac = fe_canon_dev(mac);
    mac2 = fe_canon_dev(mac2);
    m.xs[0] = rx;  m.ys[0] = rx;  m.zs[0] = fe_negc(r2x);
    m.xs[1] = mac; m.ys[1] = mac; m.zs[1] = fe_negc(mac2);
    m.xs[2] = rx;  m.ys[2] = mac; m.zs[2] = fe_negc(rkx);
    for (int i = 0; i < 3; i++) m.rs[i] = fe_canon_dev(sk[3 + i]);
    return m;
}

// out_share term sum: sum_i r_i * ([server 1] d*e + d*b + e*a + c + z)
__device__ __forceinline__ uint64_t out_share_fe(const MulView& m, int server_idx, const uint64_t* tr,
                                                 const uint64_t* cor) {
    uint64_t out = 0;
    for (int i = 0; i < 3; i++) {
        const uint64_t d = fe_canon_dev(cor[i]), e = fe_canon_dev(cor[3 + i]);
        const uint64_t ta = fe_canon_dev(tr[3 * i]), tb = fe_canon_dev(tr[3 * i + 1]), tc = fe_canon_dev(tr[3 * i + 2]);
        uint64_t term = server_idx ? fe_mulc(d, e) : 0;
        term = fe_addc(term, fe_mulc(d, tb));
        term = fe_addc(term, fe_mulc(e, ta));
        term = fe_addc(term, tc);
        term = fe_addc(term, m.zs[i]);
        out = fe_addc(out, fe_mulc(term, m.rs[i]));
    }
    return out;
}

// mode 0: cor_share (mpc.rs:142-158) -> out [n][6] {d0,d1,d2,e0,e1,e2}
// mode 1: out_share (mpc.rs:182-212) -> out [n]
__global__ __launch_bounds__(256) void k_mul_fe(MulArgs a) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * blockDim.x) {
        const MulView m = mul_view(a.sketch + 6 * i, a.mac[i], a.mac2[i]);
        const uint64_t* tr = a.triples + 9 * (i * a.triples_levels + a.level);
        if (a.mode == 0) {
            for (int t = 0; t < 3; t++) {
                a.out[6 * i + t] = fe_subc(m.xs[t], fe_canon_dev(tr[3 * t]));
                a.out[6 * i + 3 + t] = fe_subc(m.ys[t], fe_canon_dev(tr[3 * t + 1]));
            }
        } else {
            a.out[i] = out_share_fe(m, a.server_idx, tr, a.cor + 6 * i);
        }
    }
}

// both servers in one process: cor shares, cor = share0 + share1, out shares, verify
__global__ __launch_bounds__(256) void k_verify_fe(VerifyArgs a) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * blockDim.x) {
        MulView m[2];
        uint64_t cor[6] = {0, 0, 0, 0, 0, 0};
        for (int s = 0; s < 2; s++) {
            m[s] = mul_view(a.sketch[s] + 6 * i, a.mac[s][i], a.mac2[s][i]);
            const uint64_t* tr = a.triples[s] + 9 * (i * a.triples_levels + a.level);
            for (int t = 0; t < 3; t++) {
                cor[t] = fe_addc(cor[t], fe_subc(m[s].xs[t], fe_canon_dev(tr[3 * t])));
                cor[3 + t] = fe_addc(cor[3 + t], fe_subc(m[s].ys[t], fe_canon_dev(tr[3 * t + 1])));
            }
        }
        const uint64_t o0 = out_share_fe(m[0], 0, a.triples[0] + 9 * (i * a.triples_levels + a.level), cor);
        const uint64_t o1 = out_share_fe(m[1], 1, a.triples[1] + 9 * (i * a.triples_levels + a.level), cor);
        if (a.out_shares) {
            a.out_shares[i] = o0;
            a.out_shares[a.n + i] = o1;
        }
        a.ok[i] = fe_addc(o0, o1) == 0 ? 1 : 0;   // MulState::verify (mpc.rs:214-220)
    }
}

static unsigned grid_for(uint64_t n) {
    const uint64_t b = (n + 255) / 256;
    return (unsigned)(b < 65535 ? (b ? b : 1) : 65535);
}

hipError_t launch_mul_fe(const MulArgs& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mul_fe, dim3(grid_for(a.n)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_verify_fe(const VerifyArgs& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_verify_fe, dim3(grid_for(a.n)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

// ---- dealer (harness): TripleShare::new (mpc.rs:18-45) for n keys x levels x 3 triples ------
// a = a0 + a1, b = b0 + b1 with random shares, c = a b shared as c0 random, c1 = c - c0; the
// randomness is a mix64 PRF of (seed, key, level, triple, word) (the reference: thread_rng).
__device__ __forceinline__ uint64_t deal_mix(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void k_deal_triples_fe(uint64_t n, uint32_t levels, uint64_t seed, uint64_t* t0,
                                                         uint64_t* t1) {
    const uint64_t total = n * levels * 3;
    for (uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; q < total; q += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t base = deal_mix(seed ^ deal_mix(q));
        uint64_t w[5];
#pragma unroll
        for (int k = 0; k < 5; k++) w[k] = fe_canon_dev(deal_mix(base ^ (uint64_t)k) & ((1ull << 62) - 1));
        const uint64_t a = fe_addc(w[0], w[1]), b = fe_addc(w[2], w[3]);
        const uint64_t c = fe_mulc(a, b);
        t0[3 * q] = w[0];
        t0[3 * q + 1] = w[2];
        t0[3 * q + 2] = w[4];
        t1[3 * q] = w[1];
        t1[3 * q + 1] = w[3];
        t1[3 * q + 2] = fe_subc(c, w[4]);
    }
}

hipError_t launch_deal_triples_fe(uint64_t n, uint32_t levels, uint64_t seed, uint64_t* t0, uint64_t* t1,
                                  hipStream_t stream) {
    const uint64_t total = n * levels * 3;
    if (total == 0) return hipSuccess;
    const uint64_t b = (total + 255) / 256;
    hipLaunchKernelGGL(k_deal_triples_fe, dim3((unsigned)(b < 65535 ? b : 65535)), dim3(256), 0, stream, n, levels,
                       seed, t0, t1);
    return hipGetLastError();
}

// ---- U = FieldElm (the last level, sketch_at_last, sketch.rs:202-245) ----------------------
// FieldElm::from_rng = num-bigint gen_biguint_below(p) (field.rs:367-372): 32 keystream bytes
// per attempt as 8 little-endian u32 digits, top digit >> 1, redraw while >= p (probability
// 19 / 2^255). Draw m is keystream blocks 2m, 2m + 1 while nothing was redrawn (the stream is
// byte-continuous). Segment lane l of a key produces draws l, l + LPK, ... (rand1..3 for m < 3,
// then node m - 3), both blocks of a draw in lockstep; a segment that sees a draw >= p falls
// back to the sequential stream for its key.
using Fe8 = uint32_t[8];

__device__ __forceinline__ void ld8(const uint32_t* p, uint32_t (&v)[8]) {
    const uint4 a = reinterpret_cast<const uint4*>(p)[0], b = reinterpret_cast<const uint4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void st8(uint32_t* p, const uint32_t (&v)[8]) {
    reinterpret_cast<uint4*>(p)[0] = make_uint4(v[0], v[1], v[2], v[3]);
    reinterpret_cast<uint4*>(p)[1] = make_uint4(v[4], v[5], v[6], v[7]);
}

template <int LPK>
__device__ __forceinline__ void seg_fe255_sum(uint32_t (&v)[8]) {
#pragma unroll
    for (int off = LPK / 2; off > 0; off >>= 1) {
        uint32_t o[8];
#pragma unroll
        for (int k = 0; k < 8; k++) o[k] = __shfl_xor(v[k], off, 64);
        fe255_addm(v, o, v);
    }
}

// draw m (two blocks) of a key's stream: the 8 digits, top one shifted
__device__ __forceinline__ void fe255_draw_blocks(uint64_t m, const uint32_t* tbl, uint32_t b0, uint32_t b1,
                                                  const uint32_t (&rk)[11][4], uint32_t (&d)[8]) {
    uint32_t st[2][4];
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint64_t b = 2 * m + h;
        st[h][0] = 0u;
        st[h][1] = 0u;
        st[h][2] = __builtin_bswap32((uint32_t)(b >> 32));
        st[h][3] = __builtin_bswap32((uint32_t)b);
    }
    aes_rk<SkTab, 2>(st, tbl, b0, b1, rk);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        d[k] = st[0][k];
        d[4 + k] = st[1][k];
    }
    d[7] >>= 1;
}

template <int KPW>
__global__ __launch_bounds__(kSketchThreads) void k_sketch_fe255(Sketch255Args a) {
    constexpr int LPK = 64 / KPW;
    __shared__ uint32_t tbl[SkTab::kWords];
    for (int i = threadIdx.x; i < SkTab::kWords; i += kSketchThreads) tbl[i] = SkTab::word(c_T0_sk.v, i);
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t seg = lane / LPK, sl = lane % LPK;
    uint32_t b0, b1;
    SkTab::bases(lane, b0, b1);
    const uint64_t nwaves = (uint64_t)gridDim.x * (kSketchThreads / 64);
    const uint64_t F = a.n_nodes;
    const uint64_t wave = (uint64_t)blockIdx.x * (kSketchThreads / 64) + (threadIdx.x >> 6);
    for (uint64_t kbase = wave * KPW; kbase < a.n_keys; kbase += nwaves * KPW) {
        const uint64_t k = kbase + seg;
        const bool kact = k < a.n_keys;
        const uint64_t kk = kact ? k : kbase;
        uint32_t seed[4];
#pragma unroll
        for (int c = 0; c < 4; c++) seed[c] = reinterpret_cast<const uint32_t*>(a.seeds)[4 * kk + c];
        seed[3] ^= a.level;
        uint32_t rk[11][4];
        key_schedule(seed, rk, tbl, lane & 31);
        const uint32_t* x = a.x + kk * F * 8;
        const uint32_t* kx = a.kx + kk * F * 8;
        uint32_t acc[3][8], rnd[8];
#pragma unroll
        for (int q = 0; q < 8; q++) acc[0][q] = acc[1][q] = acc[2][q] = rnd[q] = 0;
        bool rej = false;
        if (!a.force_sequential) {
            for (uint64_t m = sl; m < F + 3; m += LPK) {
                uint32_t xv[8], kxv[8], r[8];
                if (m >= 3) {
                    ld8(x + 8 * (m - 3), xv);
                    ld8(kx + 8 * (m - 3), kxv);
                }
                fe255_draw_blocks(m, tbl, b0, b1, rk, r);
                rej |= fe255_geq_p(r);
                if (m < 3) {   // rand1..3 live on segment lanes 0..2 (LPK >= 4)
#pragma unroll
                    for (int q = 0; q < 8; q++) rnd[q] = r[q];
                    continue;
                }
                fe255_canonm(xv);
                fe255_canonm(kxv);
                uint32_t r2[8], t[8];
                fe255_mulm(r, r, r2);
                fe255_mulm(xv, r, t);
                fe255_addm(acc[0], t, acc[0]);
                fe255_mulm(xv, r2, t);
                fe255_addm(acc[1], t, acc[1]);
                fe255_mulm(kxv, r, t);
                fe255_addm(acc[2], t, acc[2]);
            }
        }
        const uint64_t rej_mask = __ballot(rej);
        const uint64_t seg_bits = (LPK == 64 ? ~0ull : ((1ull << LPK) - 1)) << (seg * LPK);
        const bool key_rej = a.force_sequential || (rej_mask & seg_bits) != 0;
#pragma unroll
        for (int i = 0; i < 3; i++) seg_fe255_sum<LPK>(acc[i]);
        uint32_t r3[3][8];
#pragma unroll
        for (int i = 0; i < 3; i++)
#pragma unroll
            for (int q = 0; q < 8; q++) r3[i][q] = __shfl(rnd[q], seg * LPK + i, 64);
        if (kact && sl == 0) {
            uint32_t* o = a.out + 48 * k;
            if (!key_rej) {
#pragma unroll
                for (int i = 0; i < 3; i++) st8(o + 8 * i, acc[i]);
#pragma unroll
                for (int i = 0; i < 3; i++) st8(o + 8 * (3 + i), r3[i]);
            } else {
                // sequential stream with redraws (field.rs:367-372) for this key
                uint64_t m = 0;
                auto draw = [&](uint32_t (&v)[8]) {
                    for (;;) {
                        fe255_draw_blocks(m++, tbl, b0, b1, rk, v);
                        if (!fe255_geq_p(v)) return;
                    }
                };
                uint32_t q[3][8], s[3][8];
#pragma unroll
                for (int i = 0; i < 3; i++) draw(q[i]);
#pragma unroll
                for (int i = 0; i < 3; i++)
#pragma unroll
                    for (int w = 0; w < 8; w++) s[i][w] = 0;
                for (uint64_t j = 0; j < F; j++) {
                    uint32_t r[8], r2[8], t[8], xv[8], kxv[8];
                    draw(r);
                    ld8(x + 8 * j, xv);
                    ld8(kx + 8 * j, kxv);
                    fe255_canonm(xv);
                    fe255_canonm(kxv);
                    fe255_mulm(r, r, r2);
                    fe255_mulm(xv, r, t);
                    fe255_addm(s[0], t, s[0]);
                    fe255_mulm(xv, r2, t);
                    fe255_addm(s[1], t, s[1]);
                    fe255_mulm(kxv, r, t);
                    fe255_addm(s[2], t, s[2]);
                }
#pragma unroll
                for (int i = 0; i < 3; i++) st8(o + 8 * i, s[i]);
#pragma unroll
                for (int i = 0; i < 3; i++) st8(o + 8 * (3 + i), q[i]);
            }
        }
    }
}

constexpr int kSketch255KeysPerWave = 4;   // 16 lanes per key

hipError_t launch_sketch_fe255(const Sketch255Args& a, hipStream_t stream) {
    if (a.n_keys == 0) return hipSuccess;
    int cus = 256, dev = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const void* fn = reinterpret_cast<const void*>(&k_sketch_fe255<kSketch255KeysPerWave>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kSketchThreads, 0) != hipSuccess || per_cu < 1)
        per_cu = 1;
    const uint64_t waves_needed = (a.n_keys + kSketch255KeysPerWave - 1) / kSketch255KeysPerWave;
    uint64_t blocks = (waves_needed + 3) / 4;
    const uint64_t cap = (uint64_t)cus * per_cu;
    if (blocks > cap) blocks = cap;
    hipLaunchKernelGGL(k_sketch_fe255<kSketch255KeysPerWave>, dim3((unsigned)blocks), dim3(kSketchThreads), 0, stream,
                       a);
    return hipGetLastError();
}

// MulState (mpc.rs:83-220) for U: xs = [r_x, k, r_x], ys = [r_x, k, k], zs = [-r2_x, -k2, -r_kx]
struct MulView255 {
    uint32_t xs[3][8], ys[3][8], zs[3][8], rs[3][8];
};

__device__ __forceinline__ void mul_view255(const uint32_t* sk, const uint32_t* mac_p, const uint32_t* mac2_p,
                                            MulView255& m) {
    uint32_t rx[8], r2x[8], rkx[8], mac[8], mac2[8];
    ld8(sk, rx);
    ld8(sk + 8, r2x);
    ld8(sk + 16, rkx);
    ld8(mac_p, mac);
    ld8(mac2_p, mac2);
    fe255_canonm(rx); fe255_canonm(r2x); fe255_canonm(rkx); fe255_canonm(mac); fe255_canonm(mac2);
#pragma unroll
    for (int q = 0; q < 8; q++) {
        m.xs[0][q] = rx[q];  m.ys[0][q] = rx[q];
        m.xs[1][q] = mac[q]; m.ys[1][q] = mac[q];
        m.xs[2][q] = rx[q];  m.ys[2][q] = mac[q];
    }
    fe255_negm(r2x, m.zs[0]);
    fe255_negm(mac2, m.zs[1]);
    fe255_negm(rkx, m.zs[2]);
#pragma unroll
    for (int i = 0; i < 3; i++) {
        ld8(sk + 8 * (3 + i), m.rs[i]);
        fe255_canonm(m.rs[i]);
    }
}

__device__ __forceinline__ void out_share_fe255(const MulView255& m, int server_idx, const uint32_t* tr,
                                                const uint32_t (&cor)[6][8], uint32_t (&out)[8]) {
#pragma unroll
    for (int q = 0; q < 8; q++) out[q] = 0;
    for (int i = 0; i < 3; i++) {
        uint32_t ta[8], tb[8], tc[8], term[8], t[8];
        ld8(tr + 8 * (3 * i), ta);
        ld8(tr + 8 * (3 * i + 1), tb);
        ld8(tr + 8 * (3 * i + 2), tc);
        fe255_canonm(ta); fe255_canonm(tb); fe255_canonm(tc);
        if (server_idx) {
            fe255_mulm(cor[i], cor[3 + i], term);
        } else {
#pragma unroll
            for (int q = 0; q < 8; q++) term[q] = 0;
        }
        fe255_mulm(cor[i], tb, t);
        fe255_addm(term, t, term);
        fe255_mulm(cor[3 + i], ta, t);
        fe255_addm(term, t, term);
        fe255_addm(term, tc, term);
        fe255_addm(term, m.zs[i], term);
        fe255_mulm(term, m.rs[i], t);
        fe255_addm(out, t, out);
    }
}

__device__ __forceinline__ void cor_share255(const MulView255& m, const uint32_t* tr, uint32_t (&d)[6][8]) {
    for (int i = 0; i < 3; i++) {
        uint32_t ta[8], tb[8];
        ld8(tr + 8 * (3 * i), ta);
        ld8(tr + 8 * (3 * i + 1), tb);
        fe255_canonm(ta);
        fe255_canonm(tb);
        fe255_subm(m.xs[i], ta, d[i]);
        fe255_subm(m.ys[i], tb, d[3 + i]);
    }
}

// mode 0: cor_share -> out [n][6][8]; mode 1: out_share -> out [n][8]
__global__ __launch_bounds__(256) void k_mul_fe255(Mul255Args a) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * blockDim.x) {
        MulView255 m;
        mul_view255(a.sketch + 48 * i, a.mac + 8 * i, a.mac2 + 8 * i, m);
        const uint32_t* tr = a.triples + 72 * i;
        if (a.mode == 0) {
            uint32_t d[6][8];
            cor_share255(m, tr, d);
            for (int q = 0; q < 6; q++) st8(a.out + 48 * i + 8 * q, d[q]);
        } else {
            uint32_t cor[6][8], o[8];
            for (int q = 0; q < 6; q++) {
                ld8(a.cor + 48 * i + 8 * q, cor[q]);
                fe255_canonm(cor[q]);
            }
            out_share_fe255(m, a.server_idx, tr, cor, o);
            st8(a.out + 8 * i, o);
        }
    }
}

// both servers in one process (main.rs:14-70 at the last level): cor shares, cor, out shares, verify
__global__ __launch_bounds__(256) void k_verify_fe255(Verify255Args a) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * blockDim.x) {
        MulView255 m[2];
        uint32_t cor[6][8];
        for (int s = 0; s < 2; s++) {
            mul_view255(a.sketch[s] + 48 * i, a.mac[s] + 8 * i, a.mac2[s] + 8 * i, m[s]);
            uint32_t d[6][8];
            cor_share255(m[s], a.triples[s] + 72 * i, d);
            for (int q = 0; q < 6; q++) {
                if (s == 0) {
                    for (int w = 0; w < 8; w++) cor[q][w] = d[q][w];
                } else {
                    fe255_addm(cor[q], d[q], cor[q]);   // MulState::cor (mpc.rs:160-180)
                }
            }
        }
        uint32_t o0[8], o1[8], sum[8];
        out_share_fe255(m[0], 0, a.triples[0] + 72 * i, cor, o0);
        out_share_fe255(m[1], 1, a.triples[1] + 72 * i, cor, o1);
        if (a.out_shares) {
            st8(a.out_shares + 8 * i, o0);
            st8(a.out_shares + 8 * (a.n + i), o1);
        }
        fe255_addm(o0, o1, sum);   // MulState::verify (mpc.rs:214-220)
        uint32_t nz = 0;
        for (int w = 0; w < 8; w++) nz |= sum[w];
        a.ok[i] = nz == 0 ? 1 : 0;
    }
}

hipError_t launch_mul_fe255(const Mul255Args& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mul_fe255, dim3(grid_for(a.n)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_verify_fe255(const Verify255Args& a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_verify_fe255, dim3(grid_for(a.n)), dim3(256), 0, stream, a);
    return hipGetLastError();
}

}  // namespace fhh
