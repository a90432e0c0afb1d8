// Host side of row f1: the garbled-circuit equality test and the OT extension of tree_crawl
// (src/equalitytest.rs:25-219, src/collect.rs:419-482) — key schedules and per-level material,
// the OT-extension runner the device level loop and the C ABI share, the one-process C ABI
// (fhh_gc_equality_*, fhh_ot_extend_*), and the two-party split (fhh_gb_* / fhh_ev_*: each server
// runs its half on its own ctx, only the protocol messages cross).
#include "fhh_engine.h"
#include "aes_tables.h"
#include "field_arith.h"

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

namespace fhh {
namespace eng {

// ---- garbled-circuit equality test helpers (row f1) ------------------------------------------
// FIPS-197 key expansion on little-endian column words (RotWord = rotr 8, rcon in byte 0), the
// convention of the device T-table rounds (aes_keyed.h)
void host_key_schedule(const uint8_t key[16], uint32_t (&rk)[11][4]) {
    uint32_t w[44];
    for (int i = 0; i < 4; i++)
        w[i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) | ((uint32_t)key[4 * i + 2] << 16) |
               ((uint32_t)key[4 * i + 3] << 24);
    uint32_t rcon = 1;
    for (int i = 4; i < 44; i++) {
        uint32_t t = w[i - 1];
        if (i % 4 == 0) {
            t = (t >> 8) | (t << 24);
            t = (uint32_t)SBOX.v[t & 0xFF] | ((uint32_t)SBOX.v[(t >> 8) & 0xFF] << 8) |
                ((uint32_t)SBOX.v[(t >> 16) & 0xFF] << 16) | ((uint32_t)SBOX.v[t >> 24] << 24);
            t ^= rcon;
            rcon = ((rcon << 1) ^ ((rcon & 0x80) ? 0x1B : 0)) & 0xFF;
        }
        w[i] = w[i - 4] ^ t;
    }
    for (int r = 0; r < 11; r++)
        for (int c = 0; c < 4; c++) rk[r][c] = w[4 * r + c];
}

void words_from_bytes(const uint8_t b[16], uint32_t (&w)[4]) {
    for (int c = 0; c < 4; c++)
        w[c] = (uint32_t)b[4 * c] | ((uint32_t)b[4 * c + 1] << 8) | ((uint32_t)b[4 * c + 2] << 16) |
               ((uint32_t)b[4 * c + 3] << 24);
}

uint64_t host_mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// the level loop's per-level garbler secrets (a fresh key, Delta and mask per tree_crawl call)
void gc_level_material(uint64_t prf_seed, uint32_t level, uint8_t key[16], uint8_t delta[16], uint32_t* mask) {
    uint64_t z = host_mix64(prf_seed ^ 0x67635f6c6576656cull ^ ((uint64_t)level << 20));
    for (int h = 0; h < 2; h++) {
        z = host_mix64(z);
        std::memcpy(key + 8 * h, &z, 8);
    }
    for (int h = 0; h < 2; h++) {
        z = host_mix64(z);
        std::memcpy(delta + 8 * h, &z, 8);
    }
    *mask = (uint32_t)(host_mix64(z) & 1);
}

// chunk k of a level's GC (the in-process loop splits a level's tests in chunks of children, each a
// fresh protocol instance, as the reference's channels are, collect.rs:423-430); chunk 0 = the
// level's material
void gc_chunk_material(uint64_t prf_seed, uint32_t level, uint64_t chunk, uint8_t key[16], uint8_t delta[16],
                       uint32_t* mask) {
    gc_level_material(chunk ? host_mix64(prf_seed ^ (0x6368756e6b000000ull + chunk)) : prf_seed, level, key, delta,
                      mask);
}

// validated GcArgs from a batch (device pointers)
int gc_args(fhh_ctx* ctx, const fhh_gc_batch* b, GcArgs& a) {
    if (!b) return ctx->fail(FHH_E_ARG, "gc: NULL batch");
    if (b->bits < 1 || b->bits > (uint32_t)kGcMaxBits) return ctx->fail(FHH_E_ARG, "gc: bits must be in [1, 8]");
    if ((uint64_t)b->words * 64 < b->clients) return ctx->fail(FHH_E_ARG, "gc: words < ceil(clients / 64)");
    const uint64_t n = b->groups * b->clients;
    if (n && (!b->gb_planes_dev || !b->ev_planes_dev || !b->gb_labels_dev || !b->ev_labels_dev || !b->decode_dev ||
              !b->out_dev || (b->bits > 1 && !b->tables_dev)))
        return ctx->fail(FHH_E_ARG, "gc: NULL device buffer");
    a = GcArgs{};
    a.gb_planes = b->gb_planes_dev;
    a.ev_planes = b->ev_planes_dev;
    a.G = b->groups;
    a.N = b->clients;
    a.nw = b->words;
    a.bits = b->bits;
    a.mask = b->mask & 1u;
    host_key_schedule(b->label_key, a.rk_label);
    words_from_bytes(b->delta, a.delta);
    a.delta[0] |= 1u;   // colour bit of Delta = 1 (point-and-permute)
    a.label_nonce = b->label_nonce;
    a.gate_base = b->gate_base;
    a.tables = reinterpret_cast<uint4*>(b->tables_dev);
    a.gb_labels = reinterpret_cast<uint4*>(b->gb_labels_dev);
    a.ev_labels = reinterpret_cast<uint4*>(b->ev_labels_dev);
    a.decode = b->decode_dev;
    a.out = b->out_dev;
    a.ctl = nullptr;
    return FHH_OK;
}

// ---- OT extension runner (row f1's OT) --------------------------------------------------------
uint64_t ot_padded(uint64_t m) { return (m + 8191) / 8192 * 8192; }

// the sender's base-OT choice bits of a level-loop OT (ideal base OTs; k_ot_level_keys derives
// the seeds from the same material on the device)
void ot_level_choice(uint64_t prf, uint32_t level, uint32_t salt, uint32_t s[4]) {
    const uint64_t z0 = host_mix64(prf ^ 0x6f745f63686f6963ull ^ ((uint64_t)level << 24) ^ ((uint64_t)salt << 20));
    const uint64_t z1 = host_mix64(z0);
    s[0] = (uint32_t)z0;
    s[1] = (uint32_t)(z0 >> 32);
    s[2] = (uint32_t)z1;
    s[3] = (uint32_t)(z1 >> 32);
    if (salt == 0) s[0] |= 1u;   // the labels session's s is the circuit's free-XOR Delta: colour bit 1
}

// padded choice-bit buffer of the ctx's OT scratch (mp / 32 words, zero past m)
hipError_t ot_choices_buffer(fhh_ctx* ctx, uint64_t m, uint32_t** out) {
    const uint64_t mp = ot_padded(m);
    hipError_t e = ctx->ot_buf[7].ensure(mp / 8);
    if (e != hipSuccess) return e;
    *out = ctx->ot_buf[7].as<uint32_t>();
    return hipSuccess;
}

// the 3 x 128 base-OT key schedules from host seeds (receiver k_i^0, k_i^1; sender k_i^{s_i}),
// uploaded and synchronised (the staging vector is reused by the next call)
int ot_host_keys(fhh_ctx* ctx, const uint8_t seeds[128 * 2 * 16], const uint8_t s[16], const uint32_t** rk_dev) {
    ctx->ot_rk_host.assign((size_t)3 * 128 * 44, 0);
    for (int i = 0; i < 128; i++) {
        const int si = (s[i / 8] >> (i % 8)) & 1;
        uint32_t rk[11][4];
        for (int b = 0; b < 3; b++) {
            host_key_schedule(seeds + (size_t)(i * 2 + (b < 2 ? b : si)) * 16, rk);
            std::memcpy(ctx->ot_rk_host.data() + ((size_t)b * 128 + i) * 44, rk, 44 * 4);
        }
    }
    HIP_TRY(ctx, ctx->ot_rk.ensure(ctx->ot_rk_host.size() * 4));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->ot_rk.p, ctx->ot_rk_host.data(), ctx->ot_rk_host.size() * 4,
                                hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *rk_dev = ctx->ot_rk.as<uint32_t>();
    return FHH_OK;
}

// m OTs on ctx's stream (OtArgs in include fhh_internal.h): the caller fills the mode's fields of
// `a` (mode, choices from ot_choices_buffer or a padded buffer of its own, x0 / x1 / delta, mask, sx,
// out, rk, s, ctr_off, ctl / per_group / g_off); ot_run sets the sizes and the scratch matrices and
// messages, then launches receiver expand -> sender expand -> send hash (-> the FieldElm finish) ->
// receive hash (mode 4: the two row transposes instead). Mode 0 keeps Y0 | Y1 in ot_buf[5 / 6]; modes
// 1-3 one y buffer in ot_buf[5]; mode 4 has no y.
int ot_run(fhh_ctx* ctx, OtArgs a, uint64_t m, OtOut* tr) {
    if (m == 0) return FHH_OK;
    if (a.ctr_off % 256) return ctx->fail(FHH_E_ARG, "ot: the row PRG offset must be a multiple of 256 blocks");
    const uint64_t mp = ot_padded(m);
    const size_t rows = (size_t)128 * (mp / 128) * 16;   // = 16 mp bytes
    for (int k = 0; k < 3; k++) HIP_TRY(ctx, ctx->ot_buf[k].ensure(rows));
    if (a.mode < 4) HIP_TRY(ctx, ctx->ot_buf[5].ensure(m * 16));
    if (a.mode == 0) HIP_TRY(ctx, ctx->ot_buf[6].ensure(m * 16));
    a.m = m;
    a.mp = mp;
    a.T = ctx->ot_buf[0].as<uint4>();
    a.U = ctx->ot_buf[1].as<uint4>();
    a.Q = ctx->ot_buf[2].as<uint4>();
    a.Y0 = a.mode < 4 ? ctx->ot_buf[5].as<uint4>() : nullptr;
    a.Y1 = a.mode == 0 ? ctx->ot_buf[6].as<uint4>() : nullptr;
    if (a.ss_k > 1) {   // SoftSpoken: both GGM trees (the receiver's corrections are its first message)
        if (a.ss_k != 2 && a.ss_k != 4) return ctx->fail(FHH_E_ARG, "ot: SoftSpoken k must be 2 or 4");
        HIP_TRY(ctx, ctx->ot_buf[3].ensure((size_t)2 * 128 * 16 * 16 / a.ss_k));
        HIP_TRY(ctx, ctx->ot_buf[4].ensure((size_t)128 * 2 * 16));
        a.ss_leaf = ctx->ot_buf[3].as<uint4>();
        a.ss_corr = ctx->ot_buf[4].as<uint4>();
        HIP_TRY(ctx, launch_ss_ggm(a, ctx->stream));
    }
    HIP_TRY(ctx, launch_ot_recv_expand(a, ctx->stream));     // receiver -> sender: U
    HIP_TRY(ctx, launch_ot_send_expand(a, ctx->stream));     // sender: Q
    if (a.mode == 5) {   // the correlation, left tile-major in Q / T for the r06 garbled table
    } else if (a.mode == 4) {   // the correlation itself: q_j, t_j (no hash, no y)
        HIP_TRY(ctx, launch_ot_rows_out(a, true, ctx->stream));
        HIP_TRY(ctx, launch_ot_rows_out(a, false, ctx->stream));
    } else {
        HIP_TRY(ctx, launch_ot_send_hash_rows(a, ctx->stream));  // sender -> receiver: y (Y0 | Y1)
        if (a.mode == 3) HIP_TRY(ctx, launch_cot_fe255_finish(a, ctx->stream));
        HIP_TRY(ctx, launch_ot_recv_hash_rows(a, ctx->stream));
    }
    if (tr) {
        tr->U = a.U;
        tr->Y0 = a.Y0;
        tr->Y1 = a.Y1;
        tr->nblk = mp / 128;
        tr->u_rows = a.ss_k > 1 ? 128 / a.ss_k : 128;
        tr->corr = a.ss_k > 1 ? a.ss_corr : nullptr;
    }
    return FHH_OK;
}

// the transcript's U [128][ceil(m / 128)][16] (row form) from the device's tile-major U (r06, fhh_ot.hip ot_tmaj:
// 128-OT block c of row i at uint4 (c / 4) 512 + 4 i + c % 4)
int u_transcript(fhh_ctx* ctx, const OtOut& tr, uint64_t m, uint8_t* u_out) {
    const uint64_t nb = (m + 127) / 128, R = tr.u_rows;   // SoftSpoken: R = 128 / k rows, tile stride R rows
    std::vector<uint8_t> h(tr.nblk * R * 16);
    HIP_TRY(ctx, hipMemcpy(h.data(), tr.U, h.size(), hipMemcpyDeviceToHost));
    for (uint64_t i = 0; i < R; i++)
        for (uint64_t c = 0; c < nb; c++)
            std::memcpy(u_out + (i * nb + c) * 16, h.data() + ((c / 4) * 4 * R + 4 * i + c % 4) * 16, 16);
    return FHH_OK;
}

// row-PRG blocks one batch of m OTs takes from its base-OT session (a multiple of 256, the expand
// kernels' shared-rounds alignment)
uint64_t ot_session_blocks(uint64_t m) { return (ot_padded(m) / 128 + 255) / 256 * 256; }

}  // namespace eng
}  // namespace fhh

extern "C" {

// ---- garbled-circuit equality test (row f1) ------------------------------------------------
int fhh_gc_equality_device(fhh_ctx* ctx, const fhh_gc_batch* b) {
    CTX_CHECK(ctx);
    int rc = ctx_set_device(ctx);
    if (rc) return rc;
    GcArgs a;
    rc = gc_args(ctx, b, a);
    if (rc) return rc;
    HIP_TRY(ctx, launch_gc_garble(a, ctx->stream));
    HIP_TRY(ctx, launch_gc_eval(a, ctx->stream));
    return ctx_sync(ctx);
}

int fhh_gc_equality_host(fhh_ctx* ctx, uint64_t n, uint32_t bits, const uint8_t* gb_bits, const uint8_t* ev_bits,
                         uint32_t mask, const uint8_t label_key[16], const uint8_t delta[16], uint64_t label_nonce,
                         uint64_t gate_base, uint8_t* tables, uint8_t* gb_labels, uint8_t* ev_labels,
                         uint8_t* decode, uint8_t* out) {
    CTX_CHECK(ctx);
    int rc = ctx_set_device(ctx);
    if (rc) return rc;
    if (bits < 1 || bits > (uint32_t)kGcMaxBits) return ctx->fail(FHH_E_ARG, "gc: bits must be in [1, 8]");
    if (n == 0) return FHH_OK;
    if (!gb_bits || !ev_bits || !label_key || !delta || !out) return ctx->fail(FHH_E_ARG, "gc: NULL argument");
    if (n > 0xFFFFFFFFull) return ctx->fail(FHH_E_ARG, "gc: n must fit 32 bits");
    const uint64_t nw = (n + 63) / 64;
    std::vector<uint64_t> planes[2];
    const uint8_t* src[2] = {gb_bits, ev_bits};
    for (int s = 0; s < 2; s++) {
        planes[s].assign((size_t)bits * nw, 0);
        for (uint64_t t = 0; t < n; t++)
            for (uint32_t j = 0; j < bits; j++)
                if (src[s][t * bits + j] & 1) planes[s][(size_t)j * nw + t / 64] |= 1ull << (t % 64);
    }
    DevBuf dp[2], dt, dg, de, dd, dout;
    for (int s = 0; s < 2; s++) {
        HIP_TRY(ctx, dp[s].ensure(planes[s].size() * 8));
        HIP_TRY(ctx, hipMemcpyAsync(dp[s].p, planes[s].data(), planes[s].size() * 8, hipMemcpyHostToDevice, ctx->stream));
    }
    HIP_TRY(ctx, dt.ensure((size_t)std::max(bits - 1, 1u) * 2 * n * 16));
    HIP_TRY(ctx, dg.ensure((size_t)(bits + 1) * n * 16));
    HIP_TRY(ctx, de.ensure((size_t)bits * n * 16));
    HIP_TRY(ctx, dd.ensure(n));
    HIP_TRY(ctx, dout.ensure(n));
    fhh_gc_batch b{};
    b.groups = 1;
    b.clients = (uint32_t)n;
    b.words = (uint32_t)nw;
    b.bits = bits;
    b.mask = mask;
    std::memcpy(b.label_key, label_key, 16);
    std::memcpy(b.delta, delta, 16);
    b.label_nonce = label_nonce;
    b.gate_base = gate_base;
    b.gb_planes_dev = dp[0].as<uint64_t>();
    b.ev_planes_dev = dp[1].as<uint64_t>();
    b.tables_dev = dt.as<uint8_t>();
    b.gb_labels_dev = dg.as<uint8_t>();
    b.ev_labels_dev = de.as<uint8_t>();
    b.decode_dev = dd.as<uint8_t>();
    b.out_dev = dout.as<uint8_t>();
    rc = fhh_gc_equality_device(ctx, &b);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(out, dout.p, n, hipMemcpyDeviceToHost));
    if (decode) HIP_TRY(ctx, hipMemcpy(decode, dd.p, n, hipMemcpyDeviceToHost));
    // SoA [row][t][16] -> AoS [t][row][16]
    auto soa_to_aos = [&](const DevBuf& d, uint32_t rows, uint8_t* dst) -> int {
        if (!dst || rows == 0) return FHH_OK;
        std::vector<uint8_t> h((size_t)rows * n * 16);
        HIP_TRY(ctx, hipMemcpy(h.data(), d.p, h.size(), hipMemcpyDeviceToHost));
        for (uint32_t r = 0; r < rows; r++)
            for (uint64_t t = 0; t < n; t++)
                std::memcpy(dst + (t * rows + r) * 16, h.data() + ((size_t)r * n + t) * 16, 16);
        return FHH_OK;
    };
    rc = soa_to_aos(dt, 2 * (bits - 1), tables);
    if (rc) return rc;
    rc = soa_to_aos(dg, bits + 1, gb_labels);
    if (rc) return rc;
    return soa_to_aos(de, bits, ev_labels);
}

// ---- OT extension (row f1's OT) ---------------------------------------------------------------
int fhh_ot_extend_device(fhh_ctx* ctx, const fhh_ot_batch* b) {
    CTX_CHECK(ctx);
    int rc = ctx_set_device(ctx);
    if (rc) return rc;
    if (!b) return ctx->fail(FHH_E_ARG, "ot_extend: NULL batch");
    if (b->m == 0) return FHH_OK;
    if (!b->choices_dev || !b->x0_dev || !b->out_dev) return ctx->fail(FHH_E_ARG, "ot_extend: NULL device buffer");
    uint32_t* ch = nullptr;
    HIP_TRY(ctx, ot_choices_buffer(ctx, b->m, &ch));
    const uint64_t mp = ot_padded(b->m), words = (b->m + 31) / 32;
    HIP_TRY(ctx, hipMemsetAsync(ch, 0, mp / 8, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(ch, b->choices_dev, words * 4, hipMemcpyDeviceToDevice, ctx->stream));
    // clear the bits past m in the last word, in stream order on the device
    if (b->m % 32) HIP_TRY(ctx, launch_mask_word(ch + words - 1, (1u << (b->m % 32)) - 1, ctx->stream));
    const uint32_t* rk = nullptr;
    rc = ot_host_keys(ctx, &b->base_seeds[0][0][0], b->base_choice, &rk);
    if (rc) return rc;
    OtArgs a{};
    a.rk = rk;
    words_from_bytes(b->base_choice, a.s);
    a.choices = ch;
    a.x0 = reinterpret_cast<const uint4*>(b->x0_dev);
    a.x1 = reinterpret_cast<const uint4*>(b->x1_dev);
    words_from_bytes(b->delta, a.delta);
    a.out = reinterpret_cast<uint4*>(b->out_dev);
    a.tweak_base = b->tweak_base;
    rc = ot_run(ctx, a, b->m, nullptr);
    if (rc) return rc;
    return ctx_sync(ctx);
}

int fhh_ot_extend_host(fhh_ctx* ctx, uint64_t m, const uint8_t* choices, const uint8_t* x0, const uint8_t* x1,
                       const uint8_t delta[16], const uint8_t base_seeds[128 * 2 * 16], const uint8_t base_choice[16],
                       uint64_t tweak_base, uint8_t* out, uint8_t* u_out, uint8_t* y0_out, uint8_t* y1_out) {
    CTX_CHECK(ctx);
    int rc = ctx_set_device(ctx);
    if (rc) return rc;
    if (m == 0) return FHH_OK;
    if (!choices || !x0 || !out || !base_seeds || !base_choice || (!x1 && !delta))
        return ctx->fail(FHH_E_ARG, "ot_extend: NULL argument");
    const uint64_t mp = ot_padded(m);
    std::vector<uint32_t> bits(mp / 32, 0);
    for (uint64_t j = 0; j < m; j++)
        if (choices[j] & 1) bits[j / 32] |= 1u << (j % 32);
    uint32_t* ch = nullptr;
    HIP_TRY(ctx, ot_choices_buffer(ctx, m, &ch));
    HIP_TRY(ctx, hipMemcpyAsync(ch, bits.data(), mp / 8, hipMemcpyHostToDevice, ctx->stream));
    DevBuf d0, d1, dout;
    HIP_TRY(ctx, d0.ensure(m * 16));
    HIP_TRY(ctx, dout.ensure(m * 16));
    HIP_TRY(ctx, hipMemcpyAsync(d0.p, x0, m * 16, hipMemcpyHostToDevice, ctx->stream));
    if (x1) {
        HIP_TRY(ctx, d1.ensure(m * 16));
        HIP_TRY(ctx, hipMemcpyAsync(d1.p, x1, m * 16, hipMemcpyHostToDevice, ctx->stream));
    }
    OtOut tr;
    const uint32_t* rk = nullptr;
    rc = ot_host_keys(ctx, base_seeds, base_choice, &rk);
    if (rc) return rc;
    OtArgs a{};
    a.rk = rk;
    words_from_bytes(base_choice, a.s);
    a.choices = ch;
    a.x0 = d0.as<uint4>();
    a.x1 = x1 ? d1.as<uint4>() : nullptr;
    if (!x1) words_from_bytes(delta, a.delta);
    a.out = dout.as<uint4>();
    a.tweak_base = tweak_base;
    rc = ot_run(ctx, a, m, &tr);
    if (rc) return rc;
    rc = ctx_sync(ctx);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(out, dout.p, m * 16, hipMemcpyDeviceToHost));
    if (y0_out) HIP_TRY(ctx, hipMemcpy(y0_out, tr.Y0, m * 16, hipMemcpyDeviceToHost));
    if (y1_out) HIP_TRY(ctx, hipMemcpy(y1_out, tr.Y1, m * 16, hipMemcpyDeviceToHost));
    if (u_out) {   // rows [128][ceil(m / 128)] of the padded tile-major matrix
        rc = u_transcript(ctx, tr, m, u_out);
        if (rc) return rc;
    }
    return FHH_OK;
}

int fhh_cot_extend_ss_host(fhh_ctx* ctx, uint32_t ss_k, uint64_t m, uint32_t mode, const uint8_t* choices,
                           const uint8_t delta[16], uint32_t mask, const uint8_t base_seeds[128 * 2 * 16],
                           const uint8_t base_choice[16], uint64_t ctr_off, uint8_t* sender_out, uint8_t* out,
                           uint8_t* u_out, uint8_t* y_out, uint8_t* corr_out) {
    CTX_CHECK(ctx);
    int rc = ctx_set_device(ctx);
    if (rc) return rc;
    if (ss_k != 1 && ss_k != 2 && ss_k != 4) return ctx->fail(FHH_E_ARG, "cot_extend: ss_k must be 1, 2 or 4");
    if (mode < FHH_COT_LABELS || mode > FHH_COT_RAW) return ctx->fail(FHH_E_ARG, "cot_extend: mode must be 1..4");
    if (m == 0) return FHH_OK;
    if (!choices || !out || !base_seeds || !base_choice || (mode == FHH_COT_LABELS && !delta))
        return ctx->fail(FHH_E_ARG, "cot_extend: NULL argument");
    if (mode == FHH_COT_FE255 && (m % 2)) return ctx->fail(FHH_E_ARG, "cot_extend: FieldElm shares take OT pairs (m even)");
    const uint64_t mp = ot_padded(m);
    std::vector<uint32_t> bits(mp / 32, 0);
    for (uint64_t j = 0; j < m; j++)
        if (choices[j] & 1) bits[j / 32] |= 1u << (j % 32);
    if (mode == FHH_COT_FE255)
        for (uint64_t t = 0; 2 * t < m; t++)
            if (((bits[(2 * t) / 32] >> ((2 * t) % 32)) & 1u) != ((bits[(2 * t + 1) / 32] >> ((2 * t + 1) % 32)) & 1u))
                return ctx->fail(FHH_E_ARG, "cot_extend: a FieldElm OT pair needs one choice for both halves");
    uint32_t* ch = nullptr;
    HIP_TRY(ctx, ot_choices_buffer(ctx, m, &ch));
    HIP_TRY(ctx, hipMemcpyAsync(ch, bits.data(), mp / 8, hipMemcpyHostToDevice, ctx->stream));
    const size_t per = mode == FHH_COT_FE ? 8 : 16;   // bytes per OT of out / sender values / y
    DevBuf dsx, dout;
    HIP_TRY(ctx, dsx.ensure(m * per));
    HIP_TRY(ctx, dout.ensure(m * per));
    const uint32_t* rk = nullptr;
    rc = ot_host_keys(ctx, base_seeds, base_choice, &rk);
    if (rc) return rc;
    OtArgs a{};
    a.mode = mode;
    a.mask = mask & 1u;
    a.rk = rk;
    words_from_bytes(base_choice, a.s);
    a.choices = ch;
    if (delta) words_from_bytes(delta, a.delta);
    a.ctr_off = ctr_off;
    a.sx = dsx.p;
    a.out = dout.as<uint4>();
    a.ss_k = ss_k;
    OtOut tr;
    rc = ot_run(ctx, a, m, &tr);
    if (rc) return rc;
    rc = ctx_sync(ctx);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(out, dout.p, m * per, hipMemcpyDeviceToHost));
    if (sender_out) HIP_TRY(ctx, hipMemcpy(sender_out, dsx.p, m * per, hipMemcpyDeviceToHost));
    if (y_out && mode != FHH_COT_RAW) HIP_TRY(ctx, hipMemcpy(y_out, tr.Y0, m * per, hipMemcpyDeviceToHost));
    if (u_out) {
        rc = u_transcript(ctx, tr, m, u_out);
        if (rc) return rc;
    }
    if (corr_out && ss_k > 1) HIP_TRY(ctx, hipMemcpy(corr_out, tr.corr, (size_t)128 * 2 * 16, hipMemcpyDeviceToHost));
    return FHH_OK;
}

int fhh_cot_extend_host(fhh_ctx* ctx, uint64_t m, uint32_t mode, const uint8_t* choices, const uint8_t delta[16],
                        uint32_t mask, const uint8_t base_seeds[128 * 2 * 16], const uint8_t base_choice[16],
                        uint64_t ctr_off, uint8_t* sender_out, uint8_t* out, uint8_t* u_out, uint8_t* y_out) {
    return fhh_cot_extend_ss_host(ctx, 1, m, mode, choices, delta, mask, base_seeds, base_choice, ctr_off, sender_out,
                                  out, u_out, y_out, nullptr);
}

int fhh_gc_cot_host(fhh_ctx* ctx, uint64_t n, uint32_t bits, const uint8_t* gb_bits, const uint8_t* ev_bits,
                    uint32_t mask, uint64_t gate_base, const uint8_t base_seeds[128 * 2 * 16],
                    const uint8_t base_choice[16], uint64_t ctr_off, uint8_t* tables, uint8_t* ev_zero,
                    uint8_t* ev_active, uint8_t* decode, uint8_t* out, uint64_t* gb_share, uint64_t* ev_share,
                    uint64_t* share_y) {
    CTX_CHECK(ctx);
    int rc = ctx_set_device(ctx);
    if (rc) return rc;
    if (bits < 1 || bits > (uint32_t)kGcMaxBits) return ctx->fail(FHH_E_ARG, "gc_cot: bits must be in [1, 8]");
    if (n == 0) return FHH_OK;
    if (!gb_bits || !ev_bits || !base_seeds || !base_choice || !out) return ctx->fail(FHH_E_ARG, "gc_cot: NULL argument");
    if (!(base_choice[0] & 1)) return ctx->fail(FHH_E_ARG, "gc_cot: s is the free-XOR Delta: its bit 0 must be 1");
    if (n > 0xFFFFFFFFull) return ctx->fail(FHH_E_ARG, "gc_cot: n must fit 32 bits");
    const bool share = gb_share || ev_share || share_y;
    if (share && !(gb_share && ev_share && share_y))
        return ctx->fail(FHH_E_ARG, "gc_cot: gb_share, ev_share and share_y go together");
    const uint64_t nw = (n + 63) / 64, npad = 64 * nw, m = (uint64_t)bits * npad;
    std::vector<uint64_t> planes[2];
    const uint8_t* src[2] = {gb_bits, ev_bits};
    for (int s = 0; s < 2; s++) {
        planes[s].assign((size_t)bits * nw + ot_padded(m) / 64, 0);   // the evaluator's: OT choice words, padded
        for (uint64_t t = 0; t < n; t++)
            for (uint32_t j = 0; j < bits; j++)
                if (src[s][t * bits + j] & 1) planes[s][(size_t)j * nw + t / 64] |= 1ull << (t % 64);
    }
    DevBuf dp[2], dt, dg, de, da, dd, dout, dsh;
    for (int s = 0; s < 2; s++) {
        HIP_TRY(ctx, dp[s].ensure(planes[s].size() * 8));
        HIP_TRY(ctx, hipMemcpyAsync(dp[s].p, planes[s].data(), planes[s].size() * 8, hipMemcpyHostToDevice, ctx->stream));
    }
    HIP_TRY(ctx, dt.ensure((size_t)std::max(bits - 1, 1u) * 2 * n * 16));
    HIP_TRY(ctx, dg.ensure(16));   // no garbler labels in this protocol (gc_args wants a pointer)
    HIP_TRY(ctx, de.ensure(m * 16));
    HIP_TRY(ctx, da.ensure(m * 16));
    HIP_TRY(ctx, dd.ensure(n));
    HIP_TRY(ctx, dout.ensure(n));
    if (share) HIP_TRY(ctx, dsh.ensure(3 * n * 8));   // [gb | y | ev]
    // 1. the labels OT (OtArgs mode 4): choice bits = the evaluator's planes at OT index j npad + i;
    // the garbler's zero labels q_j, the evaluator's active labels t_j = q_j ^ r_j s
    const uint32_t* rk = nullptr;
    rc = ot_host_keys(ctx, base_seeds, base_choice, &rk);
    if (rc) return rc;
    fhh_gc_batch gb{};
    gb.groups = 1;
    gb.clients = (uint32_t)n;
    gb.words = (uint32_t)nw;
    gb.bits = bits;
    gb.mask = mask;
    std::memcpy(gb.delta, base_choice, 16);   // Delta = s; no label key: the garbler draws no labels
    gb.gate_base = gate_base;
    gb.gb_planes_dev = dp[0].as<uint64_t>();
    gb.ev_planes_dev = dp[1].as<uint64_t>();
    gb.tables_dev = dt.as<uint8_t>();
    gb.gb_labels_dev = dg.as<uint8_t>();
    gb.ev_labels_dev = de.as<uint8_t>();
    gb.decode_dev = dd.as<uint8_t>();
    gb.out_dev = dout.as<uint8_t>();
    GcArgs g;
    rc = gc_args(ctx, &gb, g);
    if (rc) return rc;
    OtArgs a{};
    a.mode = 4;
    a.rk = rk;
    words_from_bytes(base_choice, a.s);
    a.choices = dp[1].as<uint32_t>();
    a.ctr_off = ctr_off;
    a.sx = de.p;
    a.out = da.as<uint4>();
    rc = ot_run(ctx, a, m, nullptr);
    if (rc) return rc;
    // 2. garble on the C-OT's zero labels with the garbler's string and mask folded in, 3. evaluate on the
    // OT'd active labels
    g.ev_ot = 1;
    if (share) {
        g.sh_gb = dsh.as<uint64_t>();
        g.sh_y = g.sh_gb + n;
    }
    HIP_TRY(ctx, launch_gc_garble(g, ctx->stream));
    g.ev_labels = da.as<uint4>();
    g.sh_gb = nullptr;
    if (share) g.sh_ev = dsh.as<uint64_t>() + 2 * n;
    HIP_TRY(ctx, launch_gc_eval(g, ctx->stream));
    rc = ctx_sync(ctx);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(out, dout.p, n, hipMemcpyDeviceToHost));
    if (share) {
        HIP_TRY(ctx, hipMemcpy(gb_share, dsh.p, n * 8, hipMemcpyDeviceToHost));
        HIP_TRY(ctx, hipMemcpy(share_y, dsh.as<uint64_t>() + n, n * 8, hipMemcpyDeviceToHost));
        HIP_TRY(ctx, hipMemcpy(ev_share, dsh.as<uint64_t>() + 2 * n, n * 8, hipMemcpyDeviceToHost));
    }
    if (decode) HIP_TRY(ctx, hipMemcpy(decode, dd.p, n, hipMemcpyDeviceToHost));
    auto soa_to_aos = [&](const DevBuf& d, uint32_t rows_, uint64_t stride, uint8_t* dst) -> int {
        if (!dst || rows_ == 0) return FHH_OK;
        std::vector<uint8_t> h((size_t)rows_ * stride * 16);
        HIP_TRY(ctx, hipMemcpy(h.data(), d.p, h.size(), hipMemcpyDeviceToHost));
        for (uint32_t r = 0; r < rows_; r++)
            for (uint64_t t = 0; t < n; t++)
                std::memcpy(dst + (t * rows_ + r) * 16, h.data() + ((size_t)r * stride + t) * 16, 16);
        return FHH_OK;
    };
    rc = soa_to_aos(dt, 2 * (bits - 1), n, tables);
    if (!rc) rc = soa_to_aos(de, bits, npad, ev_zero);
    if (!rc) rc = soa_to_aos(da, bits, npad, ev_active);
    return rc;
}

static int gt_cot_host(fhh_ctx* ctx, uint64_t n, uint32_t bits, const uint8_t* gb_bits, const uint8_t* ev_bits,
                       uint32_t mask, uint64_t gate_base, const uint8_t base_seeds[128 * 2 * 16],
                       const uint8_t base_choice[16], uint64_t ctr_off, uint8_t* ev_zero, uint8_t* ev_active,
                       uint64_t* msgs, uint64_t* gb_share, uint64_t* ev_share, bool ring32) {
    CTX_CHECK(ctx);
    int rc = ctx_set_device(ctx);
    if (rc) return rc;
    if (bits < 1 || bits > (uint32_t)kGtMaxBits) return ctx->fail(FHH_E_ARG, "gt_cot: bits must be in [1, 4]");
    if (ring32 && bits > (uint32_t)kGtTmMaxBits)
        return ctx->fail(FHH_E_ARG, "gt_cot: the Z_2^32 table runs on the tile-major kernels (bits <= 2)");
    if (n == 0) return FHH_OK;
    if (!gb_bits || !ev_bits || !base_seeds || !base_choice || !gb_share || !ev_share)
        return ctx->fail(FHH_E_ARG, "gt_cot: NULL argument");
    if (!(base_choice[0] & 1)) return ctx->fail(FHH_E_ARG, "gt_cot: s is the free-XOR Delta: its bit 0 must be 1");
    if (n > 0xFFFFFFFFull) return ctx->fail(FHH_E_ARG, "gt_cot: n must fit 32 bits");
    // r06: b <= 2 runs the tile-major table kernels on Q / T (the level loop's form), whose OT index wants
    // plane rows of whole 512-client tiles; b = 3, 4 the row-major labels of k_ot_rows_out
    const bool tm = bits <= (uint32_t)kGtTmMaxBits;
    const uint64_t nw = tm ? (n + 511) / 512 * 8 : (n + 63) / 64, npad = 64 * nw, m = (uint64_t)bits * npad;
    const uint64_t R = 1ull << bits;
    std::vector<uint64_t> planes[2];
    const uint8_t* src[2] = {gb_bits, ev_bits};
    for (int s = 0; s < 2; s++) {
        planes[s].assign((size_t)bits * nw + ot_padded(m) / 64, 0);
        for (uint64_t t = 0; t < n; t++)
            for (uint32_t j = 0; j < bits; j++)
                if (src[s][t * bits + j] & 1) planes[s][(size_t)j * nw + t / 64] |= 1ull << (t % 64);
    }
    DevBuf dp[2], de, da, dm, dsh;
    for (int s = 0; s < 2; s++) {
        HIP_TRY(ctx, dp[s].ensure(planes[s].size() * 8));
        HIP_TRY(ctx, hipMemcpyAsync(dp[s].p, planes[s].data(), planes[s].size() * 8, hipMemcpyHostToDevice, ctx->stream));
    }
    HIP_TRY(ctx, de.ensure(m * 16));
    HIP_TRY(ctx, da.ensure(m * 16));
    HIP_TRY(ctx, dm.ensure(std::max<uint64_t>(R - 1, 1) * n * 8));
    HIP_TRY(ctx, dsh.ensure(2 * n * 8));
    const uint32_t* rk = nullptr;
    rc = ot_host_keys(ctx, base_seeds, base_choice, &rk);
    if (rc) return rc;
    // 1. the labels OT (mode 4, as fhh_gc_cot_host; b <= 2: mode 5, Q / T left tile-major)
    OtArgs a{};
    a.mode = tm ? 5 : 4;
    a.rk = rk;
    words_from_bytes(base_choice, a.s);
    a.choices = dp[1].as<uint32_t>();
    a.ctr_off = ctr_off;
    a.sx = de.p;
    a.out = da.as<uint4>();
    rc = ot_run(ctx, a, m, nullptr);
    if (rc) return rc;
    // 2. the garbled table on the zero labels, 3. its row on the OT'd labels
    GcArgs g{};
    g.gb_planes = dp[0].as<uint64_t>();
    g.ev_planes = dp[1].as<uint64_t>();
    g.G = 1;
    g.N = (uint32_t)n;
    g.nw = (uint32_t)nw;
    g.bits = bits;
    g.mask = mask & 1u;
    words_from_bytes(base_choice, g.delta);
    g.gate_base = gate_base;
    g.ev_labels = tm ? ctx->ot_buf[2].as<uint4>() : de.as<uint4>();
    g.lab_tm = tm ? 1u : 0u;
    g.ev_ot = 1;
    g.gt_msgs = dm.as<uint64_t>();
    g.ring32 = ring32 ? 1u : 0u;
    g.sh_gb = dsh.as<uint64_t>();
    HIP_TRY(ctx, launch_gt_garble(g, ctx->stream));
    g.ev_labels = tm ? ctx->ot_buf[0].as<uint4>() : da.as<uint4>();
    g.sh_gb = nullptr;
    g.sh_ev = dsh.as<uint64_t>() + n;
    HIP_TRY(ctx, launch_gt_eval(g, ctx->stream));
    if (tm && (ev_zero || ev_active)) {   // the transcript's row-major labels, after the fact (tests only)
        a.m = m;
        a.mp = ot_padded(m);
        a.T = ctx->ot_buf[0].as<uint4>();
        a.Q = ctx->ot_buf[2].as<uint4>();
        HIP_TRY(ctx, launch_ot_rows_out(a, true, ctx->stream));
        HIP_TRY(ctx, launch_ot_rows_out(a, false, ctx->stream));
    }
    rc = ctx_sync(ctx);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpy(gb_share, dsh.p, n * 8, hipMemcpyDeviceToHost));
    HIP_TRY(ctx, hipMemcpy(ev_share, dsh.as<uint64_t>() + n, n * 8, hipMemcpyDeviceToHost));
    if (msgs && R > 1 && ring32) {   // SoA [R-1][n] u32 on the device -> [n][R-1] (zero-extended)
        std::vector<uint32_t> h((R - 1) * n);
        HIP_TRY(ctx, hipMemcpy(h.data(), dm.p, h.size() * 4, hipMemcpyDeviceToHost));
        for (uint64_t r = 0; r + 1 < R; r++)
            for (uint64_t t = 0; t < n; t++) msgs[t * (R - 1) + r] = h[r * n + t];
    } else if (msgs && R > 1) {   // SoA [R-1][n] on the device -> [n][R-1]
        std::vector<uint64_t> h((R - 1) * n);
        HIP_TRY(ctx, hipMemcpy(h.data(), dm.p, h.size() * 8, hipMemcpyDeviceToHost));
        for (uint64_t r = 0; r + 1 < R; r++)
            for (uint64_t t = 0; t < n; t++) msgs[t * (R - 1) + r] = h[r * n + t];
    }
    auto soa_to_aos = [&](const DevBuf& d, uint8_t* dst) -> int {
        if (!dst) return FHH_OK;
        std::vector<uint8_t> h((size_t)bits * npad * 16);
        HIP_TRY(ctx, hipMemcpy(h.data(), d.p, h.size(), hipMemcpyDeviceToHost));
        for (uint32_t r = 0; r < bits; r++)
            for (uint64_t t = 0; t < n; t++)
                std::memcpy(dst + (t * bits + r) * 16, h.data() + ((size_t)r * npad + t) * 16, 16);
        return FHH_OK;
    };
    rc = soa_to_aos(de, ev_zero);
    if (!rc) rc = soa_to_aos(da, ev_active);
    return rc;
}

int fhh_gt_cot_host(fhh_ctx* ctx, uint64_t n, uint32_t bits, const uint8_t* gb_bits, const uint8_t* ev_bits,
                    uint32_t mask, uint64_t gate_base, const uint8_t base_seeds[128 * 2 * 16],
                    const uint8_t base_choice[16], uint64_t ctr_off, uint8_t* ev_zero, uint8_t* ev_active,
                    uint64_t* msgs, uint64_t* gb_share, uint64_t* ev_share) {
    return gt_cot_host(ctx, n, bits, gb_bits, ev_bits, mask, gate_base, base_seeds, base_choice, ctr_off, ev_zero,
                       ev_active, msgs, gb_share, ev_share, false);
}

int fhh_gt_cot_ring32_host(fhh_ctx* ctx, uint64_t n, uint32_t bits, const uint8_t* gb_bits, const uint8_t* ev_bits,
                           uint32_t mask, uint64_t gate_base, const uint8_t base_seeds[128 * 2 * 16],
                           const uint8_t base_choice[16], uint64_t ctr_off, uint8_t* ev_zero, uint8_t* ev_active,
                           uint64_t* msgs, uint64_t* gb_share, uint64_t* ev_share) {
    return gt_cot_host(ctx, n, bits, gb_bits, ev_bits, mask, gate_base, base_seeds, base_choice, ctr_off, ev_zero,
                       ev_active, msgs, gb_share, ev_share, true);
}

}  // extern "C"

// ================================================================================================
// Two-party split of a level's GC equality test + OT (collect.rs:419-482 with gc_sender = true on
// server 0 and false on server 1; equalitytest.rs:25-106). Each server's ctx runs only its own half
// and holds only its own secrets: the garbler's fhh_gb_cfg (label key, Delta, mask, its base-OT
// outputs) never reaches the evaluator's ctx, the evaluator's fhh_ev_cfg (its base-OT key pairs)
// never the garbler's. Four buffers cross per chunk, in protocol order (r05: both OTs correlated; y1
// is empty since r05b):
//   E -> G  u1      labels OT: U (the evaluator's share planes are its choice bits); the IKNP
//                   correlation itself is the label pair: zero label q_j, active label t_j = q_j ^ r_j s,
//                   with the garbler's labels-kind s as the circuit's Delta — no reply
//   G -> E  gc      the garbled tables and decoding bits (the garbler's string and mask are folded
//                   into the circuit, k_gc_garble_cot: no garbler labels cross)
//   E -> G  u2      share C-OT (collect.rs:437-471 / 846-876): U
//   G -> E  y2      share C-OT: 8 B per OT (FE), 16 B per OT (FieldElm: 2 OTs per test)
// Buffers are device memory owned by the producing ctx (valid until its next party call); the
// caller moves them (a network in a deployment, a device copy in the in-process tests).
// Counters: each OT kind's base-OT session (the cfg's base material) keeps a running row-PRG
// counter per ctx, so chunks and levels that extend the same base OTs never repeat pads (ocelot's
// AlszSender keeps its PRG across `send` calls the same way); a new set of base OTs starts at 0. The
// gate tweaks use the test's index in the whole level (child_begin x n + t).
// ================================================================================================
namespace fhh {
namespace eng {

struct PartyState {
    int role = -1;              // 0 garbler / OT sender (server 0), 1 evaluator / OT receiver (server 1)
    int step = 0;               // protocol position (calls must come in order)
    bool last = false;          // tree_crawl_last: FieldElm shares (BlockPair = 2 OTs per test)
    bool lshare = false;        // r05c (FE levels): the share from the GC output labels, no OT 2
    bool ltable = false;        // r05d (FE levels, bits <= kGtMaxBits): one garbled table per test
    bool ltm = false;           // r06 (ltable, bits <= kGtTmMaxBits): the table kernels read the labels OT's
                                // tile-major Q / T (no row transposes); npad / nw = whole 512-client tiles
    // C = this instance's children: the chunk [c_off, c_off + C) of the level's level_C children
    // (child_begin / child_count); covered = children whose OTs are finished
    uint64_t c_off = 0, level_C = 0, covered = 0;
    uint32_t level_id = 0;
    bool level_last = false;
    uint64_t C = 0, n = 0, npad = 0, nw = 0, tests = 0, m1 = 0, m2 = 0;
    uint32_t bits = 0, mask = 0, per2 = 1;
    uint32_t s[2][4] = {};      // garbler: the OT-extension sender's base choice words per OT kind
    uint64_t ctr[2] = {0, 0};   // this chunk's row-PRG offsets per OT kind (blocks)
    // per OT kind: the base material of the running session and its next free counter
    std::vector<uint8_t> sess[2];
    uint64_t sess_next[2] = {0, 0};
    GcArgs g{};                 // garbler: the chunk's garbling arguments
    DevBuf planes;              // own share planes [C][bits][nw] (+ padding: OT 1's choice words)
    DevBuf gc;                  // garbler: the gc message
    DevBuf labels;              // garbler: the evaluator's zero labels (C-OT 1 sender messages); evaluator: its active labels
    DevBuf rk[2];               // base-OT key schedules [3][128][44] per OT kind, own rows only
    DevBuf T, U, Q, Y;          // OT matrices (T / Q private) and messages (U or y)
    DevBuf choices2;            // evaluator: the GC outputs packed as OT 2's choice words
    DevBuf out;                 // evaluator: GC output bytes (eq ^ mask)
    DevBuf vals;                // the level's node values [level_C][n] (u64, or a BlockPair at the last level)
    std::vector<uint32_t> rk_host;
    uint64_t bytes_sent = 0;    // this ctx's outgoing message bytes for the level
    uint32_t ss_k = 1;          // r06: 1 IKNP, 2 / 4 SoftSpoken (both OT kinds; fhh_ev_cfg / fhh_gb_cfg.ot_ss_k)
    DevBuf ss_leaf;             // SoftSpoken: this party's GGM leaves
    // r06 (ltm): the table kernels add this party's node values per child into partials [level_C][4] (the
    // level loop's layout: garbler slots 0, 1, evaluator 2, 3) instead of storing them in vals, and the
    // garble / evaluate calls copy the partials to the host before they return: fhh_party_node_sums then
    // needs no device work (no sums kernel, no values round trip, no extra synchronisation)
    bool lfused = false;
    DevBuf partials;
    std::vector<uint64_t> partials_host;
};

void party_destroy(fhh_ctx* ctx) {
    delete ctx->party;
    ctx->party = nullptr;
}

namespace {

PartyState& party_of(fhh_ctx* ctx) {
    if (!ctx->party) ctx->party = new PartyState();
    return *ctx->party;
}

int party_begin(fhh_ctx* ctx, int role, uint64_t child_begin, uint64_t child_count, uint32_t form) {
    int rc = ctx_set_device(ctx);
    if (rc) return rc;
    if (ctx->group) return ctx->fail(FHH_E_ARG, "party: run the GC + OT per shard (fhh_shard_ctx)");
    if (ctx->phase != Phase::kPending && ctx->phase != Phase::kPendingLast)
        return ctx->fail(FHH_E_STATE, "party: needs a pending tree_crawl / tree_crawl_last");
    if (2 * ctx->d > (uint32_t)kGcMaxBits) return ctx->fail(FHH_E_ARG, "party: d <= 4");
    PartyState& P = party_of(ctx);
    const bool last = ctx->phase == Phase::kPendingLast;
    // the chunk of children (collect.rs:423-430: a level's tests split over channels), in order
    const uint64_t LC = ctx->pending_C, b = child_begin;
    if (child_count == 0 && b != 0) return ctx->fail(FHH_E_ARG, "party: child_begin without child_count");
    if (b > LC || (child_count && b == LC && LC))
        return ctx->fail(FHH_E_ARG, "party: child_begin " + std::to_string(b) + " past the level's " +
                                        std::to_string(LC) + " children");
    if (b != 0 && (P.role != role || P.level_id != ctx->level || P.level_last != last || P.level_C != LC ||
                   P.covered != b))
        return ctx->fail(FHH_E_STATE, "party: chunk at child " + std::to_string(b) + " does not follow the level's " +
                                          "finished children (" + std::to_string(P.covered) + ")");
    P.role = role;
    P.step = 0;
    P.last = last;
    P.level_id = ctx->level;
    P.level_last = last;
    P.level_C = LC;
    if (b == 0) P.covered = 0;
    P.c_off = b;
    P.C = child_count ? std::min<uint64_t>(child_count, LC - b) : LC;
    P.n = ctx->n;
    P.npad = ctx->npad;   // (r06 tile-major table: whole 512-client tiles, set below)
    P.nw = ctx->nw;
    P.bits = 2 * ctx->d;
    P.tests = P.C * P.n;
    P.per2 = P.last ? 2 : 1;
    P.lshare = !P.last;
    P.ltable = P.lshare && P.bits <= (uint32_t)kGtMaxBits && form == 0;   // form 1: the circuit (r05c)
    P.ltm = P.ltable && P.bits <= (uint32_t)kGtTmMaxBits;
    if (P.ltm) {   // plane rows and the OT index over whole 512-client tiles (both parties alike: n is public)
        P.nw = (ctx->nw + 7) / 8 * 8;
        P.npad = 64 * P.nw;
    }
    P.m1 = P.C * P.bits * P.npad;   // OT index (g bits + j) npad + i: the share planes as choice bits
    P.m2 = P.lshare ? 0 : P.tests * P.per2;   // OT 2 (the share OT) at the FieldElm level only
    if (b == 0) P.bytes_sent = 0;   // the level's outgoing bytes, over its chunks
    // this server's share planes [C][bits][nw] of the chunk (collect.rs:393-418), zero-padded to the
    // OT's whole choice words (ot_padded(m1) bits)
    const uint64_t plane_words = P.C * P.bits * P.nw, pad_words = ot_padded(std::max<uint64_t>(P.m1, 1)) / 64;
    HIP_TRY(ctx, P.planes.ensure(std::max(plane_words, pad_words) * 8));
    HIP_TRY(ctx, hipMemsetAsync(P.planes.p, 0, std::max(plane_words, pad_words) * 8, ctx->stream));
    if (P.C) {
        ChildArgs a = ctx_child_args(ctx);
        a.c_off = P.c_off;
        a.c_cnt = P.C;
        a.plane_nw = (uint32_t)P.nw;
        HIP_TRY(ctx, launch_share_planes(a, P.planes.as<uint64_t>(), ctx->stream));
    }
    // the level's node values, one row of n per child (u64 FE, or a BlockPair at the last level); with the
    // fused sums (ltm) only the per-child partials, zeroed at the level's first chunk
    P.lfused = P.ltm;
    if (b == 0 && P.lfused) {
        HIP_TRY(ctx, P.partials.ensure(std::max<uint64_t>(LC, 1) * 4 * 8));
        HIP_TRY(ctx, hipMemsetAsync(P.partials.p, 0, std::max<uint64_t>(LC, 1) * 4 * 8, ctx->stream));
        P.partials_host.assign(std::max<uint64_t>(LC, 1) * 4, 0);
    } else if (b == 0) {
        HIP_TRY(ctx, P.vals.ensure(std::max<uint64_t>(LC * P.n * P.per2, 1) * (P.last ? 16 : 8)));
    }
    return FHH_OK;
}

// the fused partials of the level so far, to the host (each chunk's call copies the whole accumulating
// array; after the level's last chunk the host copy is complete)
int party_partials_to_host(fhh_ctx* ctx, PartyState& P) {
    if (!P.lfused || P.level_C == 0) return FHH_OK;
    HIP_TRY(ctx, hipMemcpyAsync(P.partials_host.data(), P.partials.p, P.level_C * 4 * 8, hipMemcpyDeviceToHost,
                                ctx->stream));
    return FHH_OK;
}

// base-OT session of OT kind w: the same material as the running session continues its counter,
// new material starts a session at 0; the chunk's m OTs take the next blocks
void party_session(PartyState& P, int w, const uint8_t* mat, size_t bytes, uint64_t m) {
    if (P.sess[w].size() != bytes || std::memcmp(P.sess[w].data(), mat, bytes) != 0) {
        P.sess[w].assign(mat, mat + bytes);
        P.sess_next[w] = 0;
    }
    P.ctr[w] = P.sess_next[w];
    P.sess_next[w] += m ? ot_session_blocks(m) : 0;
}

// key schedules of OT kind w's base OTs into P.rk[w]: receiver rows 0 / 1 from both seeds of each
// base OT, sender row 2 from its chosen seeds (the other party's rows stay zero: never read)
int party_keys(fhh_ctx* ctx, PartyState& P, int w, const uint8_t* pairs /*[128][2][16] or null*/,
               const uint8_t* chosen /*[128][16] or null*/) {
    P.rk_host.assign((size_t)3 * 128 * 44, 0);
    for (int i = 0; i < 128; i++) {
        uint32_t k[11][4];
        for (int b = 0; b < 2 && pairs; b++) {
            host_key_schedule(pairs + ((size_t)i * 2 + b) * 16, k);
            std::memcpy(P.rk_host.data() + ((size_t)b * 128 + i) * 44, k, 44 * 4);
        }
        if (chosen) {
            host_key_schedule(chosen + (size_t)i * 16, k);
            std::memcpy(P.rk_host.data() + ((size_t)2 * 128 + i) * 44, k, 44 * 4);
        }
    }
    HIP_TRY(ctx, P.rk[w].ensure(P.rk_host.size() * 4));
    HIP_TRY(ctx, hipMemcpyAsync(P.rk[w].p, P.rk_host.data(), P.rk_host.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    // the staging vector is rewritten by the next call: finish the copy now
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return FHH_OK;
}

OtArgs party_ot(PartyState& P, int w, uint64_t m) {
    OtArgs a{};
    a.m = m;
    a.mp = ot_padded(m);
    a.rk = P.rk[w].as<uint32_t>();
    a.T = P.T.as<uint4>();
    a.U = P.U.as<uint4>();
    a.Q = P.Q.as<uint4>();
    a.ctr_off = P.ctr[w];
    a.ss_k = P.ss_k > 1 ? P.ss_k : 0;
    return a;
}

// SoftSpoken (P.ss_k > 1): this party's half of the GGM trees before its expand — the receiver's corrections
// go after U in its message, the sender reads them there (a.U = the received message)
hipError_t party_ggm(PartyState& P, OtArgs& a, bool receiver, hipStream_t stream) {
    if (P.ss_k < 2) return hipSuccess;
    a.ss_leaf = P.ss_leaf.as<uint4>();
    a.ss_corr = reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(a.U) + 16 * a.mp / P.ss_k);
    a.ss_role = receiver ? 1 : 2;
    return launch_ss_ggm(a, stream);
}

// message sizes: U = 128 / k rows of the padded OTs (+ SoftSpoken's GGM corrections, 4 KiB)
uint64_t u_bytes(uint64_t m, uint32_t k) { return 16 * ot_padded(m) / k + (k > 1 ? 128 * 2 * 16 : 0); }

int party_ot_buffers(fhh_ctx* ctx, PartyState& P, uint64_t m, bool receiver, bool reply = true) {
    const uint64_t rows = 16 * ot_padded(m);   // [128][mp / 128] blocks
    HIP_TRY(ctx, (receiver ? P.T : P.Q).ensure(rows));
    if (receiver) HIP_TRY(ctx, P.U.ensure(u_bytes(m, P.ss_k)));
    else if (reply) HIP_TRY(ctx, P.Y.ensure(std::max<uint64_t>(m, 1) * 16));
    if (P.ss_k > 1) HIP_TRY(ctx, P.ss_leaf.ensure((size_t)2 * 128 * 16 * 16 / P.ss_k));
    return FHH_OK;
}

uint64_t gc_bytes(const PartyState& P) {
    if (P.ltable) return P.tests * (((uint64_t)1 << P.bits) - 1) * 8;   // rows 1 .. 2^bits - 1, 8 B each
    return P.tests * ((uint64_t)2 * (P.bits - 1) * 16 + 1 + (P.lshare ? 8 : 0));
}
uint64_t y2_bytes(const PartyState& P) { return P.m2 * (P.last ? 16 : 8); }

int check_in(fhh_ctx* ctx, const void* p, uint64_t got, uint64_t want, const char* what) {
    if (want && !p) return ctx->fail(FHH_E_ARG, std::string("party: NULL ") + what);
    if (got != want)
        return ctx->fail(FHH_E_ARG, std::string("party: ") + what + " is " + std::to_string(got) + " bytes, expected " +
                                        std::to_string(want));
    return FHH_OK;
}

// carve the gc message [tables | y | decode] (the garbler's string and mask are folded into the circuit:
// no garbler labels cross, k_gc_garble_cot; y = the FE share's 8 B per test at the FE levels, r05c)
void gc_layout(const PartyState& P, uint8_t* base, GcArgs& g) {
    const uint64_t t = P.tests, tb = (uint64_t)2 * (P.bits - 1) * t * 16;
    g.tables = reinterpret_cast<uint4*>(base);
    g.gb_labels = nullptr;
    g.sh_y = P.lshare ? reinterpret_cast<uint64_t*>(base + tb) : nullptr;
    g.decode = base + tb + (P.lshare ? 8 * t : 0);
    if (P.ltable) {   // r05d: the gc message is the garbled table's rows 1 .. 2^bits - 1 (SoA, u64)
        g.tables = nullptr;
        g.sh_y = nullptr;
        g.decode = nullptr;
        g.gt_msgs = reinterpret_cast<uint64_t*>(base);
    }
}

// this chunk's rows of the level's node values (u64 FE, or a BlockPair at the last level)
uint8_t* party_vals(PartyState& P) { return P.vals.as<uint8_t>() + P.c_off * P.n * P.per2 * (P.last ? 16 : 8); }

// the chunk's gate tweaks: the level in bits 40+ (Delta = the labels session's s may serve several levels
// when base OTs are reused), then the test's index in the whole level (c_off n + t)
uint64_t party_gate_base(const PartyState& P) { return ((uint64_t)P.level_id << 40) + P.c_off * P.n * (P.bits - 1); }

}  // namespace
}  // namespace eng
}  // namespace fhh

extern "C" {

int fhh_ev_ot_labels(fhh_ctx* ctx, const fhh_ev_cfg* cfg, const uint8_t** u_dev, uint64_t* u_len) {
    CTX_CHECK(ctx);
    if (!cfg || !u_dev || !u_len) return ctx->fail(FHH_E_ARG, "ev_ot_labels: NULL argument");
    if (cfg->form > 1) return ctx->fail(FHH_E_ARG, "ev_ot_labels: form must be 0 (table) or 1 (circuit)");
    if (cfg->ot_ss_k > 1 && cfg->ot_ss_k != 2 && cfg->ot_ss_k != 4)
        return ctx->fail(FHH_E_ARG, "ev_ot_labels: ot_ss_k must be 0 / 1 (IKNP), 2 or 4 (SoftSpoken)");
    int rc = party_begin(ctx, 1, cfg->child_begin, cfg->child_count, cfg->form);
    if (rc) return rc;
    PartyState& P = *ctx->party;
    P.ss_k = cfg->ot_ss_k > 1 ? cfg->ot_ss_k : 1;
    // both OT kinds' receiver schedules and session counters (OtReceiver::init, collect.rs:460)
    // (kind 1, the share OT, at the FieldElm level only: the FE levels' share rides on the GC, r05c)
    party_session(P, 0, &cfg->base_pairs[0][0][0][0], 128 * 32, P.m1);
    rc = party_keys(ctx, P, 0, &cfg->base_pairs[0][0][0][0], nullptr);
    if (!rc && !P.lshare) {
        party_session(P, 1, &cfg->base_pairs[1][0][0][0], 128 * 32, P.m2);
        rc = party_keys(ctx, P, 1, &cfg->base_pairs[1][0][0][0], nullptr);
    }
    if (rc) return rc;
    rc = party_ot_buffers(ctx, P, P.m1, true);
    if (rc) return rc;
    if (!P.ltm) HIP_TRY(ctx, P.labels.ensure(std::max<uint64_t>(P.m1, 1) * 16));
    if (P.m1) {   // OT 1's receiver: choice bits = this server's share planes as they stand
        OtArgs a = party_ot(P, 0, P.m1);
        a.mode = P.ltm ? 5 : 4;
        a.choices = P.planes.as<uint32_t>();
        a.out = P.ltm ? nullptr : P.labels.as<uint4>();
        HIP_TRY(ctx, party_ggm(P, a, true, ctx->stream));
        HIP_TRY(ctx, launch_ot_recv_expand(a, ctx->stream));        // T, U
        // its active labels t_j: row-major for the circuit; the r06 table reads T tile-major
        if (!P.ltm) HIP_TRY(ctx, launch_ot_rows_out(a, false, ctx->stream));
    }
    rc = ctx_sync(ctx);
    if (rc) return rc;
    P.step = 1;
    *u_dev = P.U.as<uint8_t>();
    *u_len = P.m1 ? u_bytes(P.m1, P.ss_k) : 0;
    P.bytes_sent += *u_len;
    return FHH_OK;
}

int fhh_gb_ot_labels(fhh_ctx* ctx, const fhh_gb_cfg* cfg, const uint8_t* u_dev, uint64_t u_len, const uint8_t** y_dev,
                     uint64_t* y_len) {
    CTX_CHECK(ctx);
    if (!cfg || !y_dev || !y_len) return ctx->fail(FHH_E_ARG, "gb_ot_labels: NULL argument");
    if (cfg->form > 1) return ctx->fail(FHH_E_ARG, "gb_ot_labels: form must be 0 (table) or 1 (circuit)");
    if (cfg->ot_ss_k > 1 && cfg->ot_ss_k != 2 && cfg->ot_ss_k != 4)
        return ctx->fail(FHH_E_ARG, "gb_ot_labels: ot_ss_k must be 0 / 1 (IKNP), 2 or 4 (SoftSpoken)");
    int rc = party_begin(ctx, 0, cfg->child_begin, cfg->child_count, cfg->form);
    if (rc) return rc;
    PartyState& P = *ctx->party;
    P.ss_k = cfg->ot_ss_k > 1 ? cfg->ot_ss_k : 1;
    rc = check_in(ctx, u_dev, u_len, P.m1 ? u_bytes(P.m1, P.ss_k) : 0, "U (labels OT)");
    if (rc) return rc;
    P.mask = cfg->mask & 1u;
    if (!(cfg->base_choice[0][0] & 1))
        return ctx->fail(FHH_E_ARG, "gb_ot_labels: the labels base OTs' s is the free-XOR Delta: its bit 0 must be 1");
    // the OT kinds' sender schedules and session counters (OtSender::init, collect.rs:454): kind 1 (the
    // share OT) at the FieldElm level only (r05c)
    for (int w = 0; w < (P.lshare ? 1 : 2); w++) {
        std::vector<uint8_t> mat((size_t)128 * 16 + 16);
        std::memcpy(mat.data(), &cfg->base_chosen[w][0][0], 128 * 16);
        std::memcpy(mat.data() + 128 * 16, cfg->base_choice[w], 16);
        party_session(P, w, mat.data(), mat.size(), w ? P.m2 : P.m1);
        words_from_bytes(cfg->base_choice[w], P.s[w]);
        rc = party_keys(ctx, P, w, nullptr, &cfg->base_chosen[w][0][0]);
        if (rc) return rc;
    }
    // the garbling arguments of the chunk (multiple_gb_equality_test, equalitytest.rs:25-65); the
    // evaluator's zero labels are OT 1's sender messages, at the OT index of its choice bits
    HIP_TRY(ctx, P.gc.ensure(std::max<uint64_t>(gc_bytes(P), 1)));
    if (!P.ltm) HIP_TRY(ctx, P.labels.ensure(std::max<uint64_t>(P.m1, 1) * 16));
    rc = party_ot_buffers(ctx, P, P.m1, false, false);
    if (rc) return rc;
    fhh_gc_batch gb{};
    gb.groups = P.C;
    gb.clients = (uint32_t)P.n;
    gb.words = (uint32_t)P.nw;
    gb.bits = P.bits;
    gb.mask = P.mask;
    std::memcpy(gb.delta, cfg->base_choice[0], 16);   // Delta = the labels session's s
    gb.gate_base = party_gate_base(P);
    gb.gb_planes_dev = P.planes.as<uint64_t>();
    gb.ev_planes_dev = P.planes.as<uint64_t>();   // not read: the evaluator's labels go by OT
    gb.tables_dev = P.gc.as<uint8_t>();
    gb.gb_labels_dev = P.gc.as<uint8_t>();
    gb.ev_labels_dev = P.ltm ? P.Q.as<uint8_t>() : P.labels.as<uint8_t>();   // r06: the tile-major Q itself
    gb.decode_dev = P.gc.as<uint8_t>();
    gb.out_dev = P.gc.as<uint8_t>();
    rc = gc_args(ctx, &gb, P.g);
    if (rc) return rc;
    gc_layout(P, P.gc.as<uint8_t>(), P.g);
    P.g.ev_ot = 1;
    P.g.lab_tm = P.ltm ? 1u : 0u;
    P.g.out = nullptr;
    // r05c: the garbler's node values r1 straight into the level's rows (the y it forms travels in gc);
    // r06 (ltm): added per child into the partials instead
    P.g.sh_gb = P.lshare && !P.lfused ? reinterpret_cast<uint64_t*>(party_vals(P)) : nullptr;
    P.g.node_partials = P.lfused ? P.partials.as<uint64_t>() : nullptr;
    P.g.node_off = P.c_off;
    // OT 1 as the IKNP correlation (gb_set_fancy_inputs, equalitytest.rs:67-82): q_j is the evaluator's
    // zero label of its share bit j, q_j ^ s its one label, and s = Delta: nothing to send back
    if (P.m1) {
        OtArgs a = party_ot(P, 0, P.m1);
        a.mode = P.ltm ? 5 : 4;
        a.U = const_cast<uint4*>(reinterpret_cast<const uint4*>(u_dev));
        for (int c = 0; c < 4; c++) a.s[c] = P.s[0][c];
        a.sx = P.ltm ? nullptr : P.labels.p;
        HIP_TRY(ctx, party_ggm(P, a, false, ctx->stream));
        HIP_TRY(ctx, launch_ot_send_expand(a, ctx->stream));      // Q from U
        if (!P.ltm) HIP_TRY(ctx, launch_ot_rows_out(a, true, ctx->stream));   // the zero labels q_j (the circuit)
    }
    rc = ctx_sync(ctx);
    if (rc) return rc;
    P.step = 1;
    *y_dev = nullptr;
    *y_len = 0;   // the labels OT has no reply
    return FHH_OK;
}

int fhh_gb_garble(fhh_ctx* ctx, const uint8_t** gc_msg_dev, uint64_t* gc_msg_bytes) {
    CTX_CHECK(ctx);
    if (!gc_msg_dev || !gc_msg_bytes) return ctx->fail(FHH_E_ARG, "gb_garble: NULL argument");
    int rc = ctx_set_device(ctx);
    if (rc) return rc;
    PartyState* Pp = ctx->party;
    if (!Pp || Pp->role != 0 || Pp->step != 1) return ctx->fail(FHH_E_STATE, "gb_garble: call after fhh_gb_ot_labels");
    PartyState& P = *Pp;
    if (P.tests) HIP_TRY(ctx, P.ltable ? launch_gt_garble(P.g, ctx->stream) : launch_gc_garble(P.g, ctx->stream));
    rc = party_partials_to_host(ctx, P);
    if (rc) return rc;
    rc = ctx_sync(ctx);
    if (rc) return rc;
    P.step = 2;
    *gc_msg_dev = P.gc.as<uint8_t>();
    *gc_msg_bytes = gc_bytes(P);
    P.bytes_sent += *gc_msg_bytes;
    return FHH_OK;
}

int fhh_ev_evaluate(fhh_ctx* ctx, const uint8_t* gc_msg_dev, uint64_t gc_len, const uint8_t* y_dev, uint64_t y_len,
                    const uint8_t** u_dev, uint64_t* u_len) {
    CTX_CHECK(ctx);
    if (!u_dev || !u_len) return ctx->fail(FHH_E_ARG, "ev_evaluate: NULL output");
    int rc = ctx_set_device(ctx);
    if (rc) return rc;
    PartyState* Pp = ctx->party;
    if (!Pp || Pp->role != 1 || Pp->step != 1) return ctx->fail(FHH_E_STATE, "ev_evaluate: call after fhh_ev_ot_labels");
    PartyState& P = *Pp;
    rc = check_in(ctx, gc_msg_dev, gc_len, gc_bytes(P), "gc message");
    if (rc) return rc;
    rc = check_in(ctx, y_dev, y_len, 0, "y (labels OT: empty since r05b)");
    if (rc) return rc;
    // 1. OT 1's output, the evaluator's active input labels t_j (ev_set_fancy_inputs,
    // equalitytest.rs:108-119), is in P.labels since fhh_ev_ot_labels
    // 2. evaluate (multiple_ev_equality_test); the outputs are packed as OT 2's choice words
    const uint64_t mp2 = ot_padded(std::max<uint64_t>(P.m2, 1));
    HIP_TRY(ctx, P.choices2.ensure(mp2 / 8 + 64));
    HIP_TRY(ctx, hipMemsetAsync(P.choices2.p, 0, mp2 / 8 + 64, ctx->stream));
    HIP_TRY(ctx, P.out.ensure(std::max<uint64_t>(P.tests, 1)));
    GcArgs g{};
    g.G = P.C;
    g.N = (uint32_t)P.n;
    g.nw = (uint32_t)P.nw;
    g.bits = P.bits;
    g.gate_base = party_gate_base(P);
    gc_layout(P, const_cast<uint8_t*>(gc_msg_dev), g);
    g.ev_labels = P.ltm ? P.T.as<uint4>() : P.labels.as<uint4>();   // r06: the tile-major T itself
    g.lab_tm = P.ltm ? 1u : 0u;
    g.ev_ot = 1;
    g.out = P.out.as<uint8_t>();
    if (P.lfused) {   // r06: added per child into the partials
        g.node_partials = P.partials.as<uint64_t>();
        g.node_off = P.c_off;
    } else if (P.lshare) {
        // r05c: its node value from its output label and the gc message's y, straight into the rows
        g.sh_ev = reinterpret_cast<uint64_t*>(party_vals(P));
    } else {
        g.out_packed = P.choices2.as<uint32_t>();
        g.out_dup = P.per2;
    }
    if (P.tests) HIP_TRY(ctx, P.ltable ? launch_gt_eval(g, ctx->stream) : launch_gc_eval(g, ctx->stream));
    rc = party_partials_to_host(ctx, P);
    if (rc) return rc;
    // 3. OT 2's receiver: choice = the GC output (collect.rs:461-471); T and U reused
    rc = party_ot_buffers(ctx, P, P.m2, true);
    if (rc) return rc;
    if (P.m2) {
        OtArgs a = party_ot(P, 1, P.m2);
        a.choices = P.choices2.as<uint32_t>();
        HIP_TRY(ctx, party_ggm(P, a, true, ctx->stream));
        HIP_TRY(ctx, launch_ot_recv_expand(a, ctx->stream));
    }
    rc = ctx_sync(ctx);
    if (rc) return rc;
    P.step = 2;
    *u_dev = P.U.as<uint8_t>();
    *u_len = P.m2 ? u_bytes(P.m2, P.ss_k) : 0;
    P.bytes_sent += *u_len;
    return FHH_OK;
}

int fhh_gb_ot_shares(fhh_ctx* ctx, const uint8_t* u_dev, uint64_t u_len, const uint8_t** y_dev, uint64_t* y_len) {
    CTX_CHECK(ctx);
    if (!y_dev || !y_len) return ctx->fail(FHH_E_ARG, "gb_ot_shares: NULL output");
    int rc = ctx_set_device(ctx);
    if (rc) return rc;
    PartyState* Pp = ctx->party;
    if (!Pp || Pp->role != 0 || Pp->step != 2) return ctx->fail(FHH_E_STATE, "gb_ot_shares: call after fhh_gb_garble");
    PartyState& P = *Pp;
    rc = check_in(ctx, u_dev, u_len, P.m2 ? u_bytes(P.m2, P.ss_k) : 0, "U (shares OT)");
    if (rc) return rc;
    rc = party_ot_buffers(ctx, P, P.m2, false);
    if (rc) return rc;
    if (P.m2) {
        // OT 2 as a correlated OT (collect.rs:439-471): pair[0] = H(q_j) read as the share (FE: a LE u128
        // mod p; FieldElm: the OT pair's 32 big-endian bytes mod p), pair[1] = pair[0] +- 1 as the mask
        // orders (r0, r1); this server's node value r1 goes straight into the level's rows
        OtArgs a = party_ot(P, 1, P.m2);
        a.mode = P.last ? 3 : 2;
        a.mask = P.mask;
        a.U = const_cast<uint4*>(reinterpret_cast<const uint4*>(u_dev));
        for (int c = 0; c < 4; c++) a.s[c] = P.s[1][c];
        a.sx = party_vals(P);
        a.Y0 = P.Y.as<uint4>();
        HIP_TRY(ctx, party_ggm(P, a, false, ctx->stream));
        HIP_TRY(ctx, launch_ot_send_expand(a, ctx->stream));
        HIP_TRY(ctx, launch_ot_send_hash_rows(a, ctx->stream));
        if (P.last) HIP_TRY(ctx, launch_cot_fe255_finish(a, ctx->stream));
    }
    P.covered = P.c_off + P.C;
    rc = ctx_sync(ctx);
    if (rc) return rc;
    P.step = 3;
    *y_dev = P.Y.as<uint8_t>();
    *y_len = y2_bytes(P);
    P.bytes_sent += *y_len;
    return FHH_OK;
}

int fhh_ev_ot_shares(fhh_ctx* ctx, const uint8_t* y_dev, uint64_t y_len) {
    CTX_CHECK(ctx);
    int rc = ctx_set_device(ctx);
    if (rc) return rc;
    PartyState* Pp = ctx->party;
    if (!Pp || Pp->role != 1 || Pp->step != 2) return ctx->fail(FHH_E_STATE, "ev_ot_shares: call after fhh_ev_evaluate");
    PartyState& P = *Pp;
    rc = check_in(ctx, y_dev, y_len, y2_bytes(P), "y (shares OT)");
    if (rc) return rc;
    if (P.m2) {   // the OT outputs are this server's node values, straight into the level's rows
        OtArgs a = party_ot(P, 1, P.m2);
        a.mode = P.last ? 3 : 2;
        a.choices = P.choices2.as<uint32_t>();
        a.Y0 = const_cast<uint4*>(reinterpret_cast<const uint4*>(y_dev));
        a.out = reinterpret_cast<uint4*>(party_vals(P));
        HIP_TRY(ctx, launch_ot_recv_hash_rows(a, ctx->stream));
    }
    P.covered = P.c_off + P.C;
    rc = ctx_sync(ctx);
    if (rc) return rc;
    P.step = 3;
    return FHH_OK;
}

int fhh_party_node_sums(fhh_ctx* ctx, void* sums_a, void* sums_b) {
    CTX_CHECK(ctx);
    if (ctx->group) {
        // every shard ran its own channel (fhh_shard_ctx); sum the shards' device values
        int S = 0;
        int rc = fhh_shard_info(ctx, 0, &S, nullptr, nullptr, nullptr, nullptr);
        if (rc) return rc;
        std::vector<const void*> v((size_t)S, nullptr);
        std::vector<PartyState*> fused_shards;
        int last = -1;
        for (int k = 0; k < S; k++) {
            fhh_ctx* sh = nullptr;
            uint64_t nk = 0;
            rc = fhh_shard_ctx(ctx, k, &sh);
            if (!rc) rc = fhh_shard_info(ctx, k, nullptr, nullptr, nullptr, &nk, nullptr);
            if (rc) return rc;
            if (!nk) continue;
            PartyState* P = sh->party;
            if (!P || P->step != 3 || P->covered != P->level_C)
                return ctx->fail(FHH_E_STATE, "party_node_sums: shard " + std::to_string(k) +
                                                  "'s OTs are not finished for every child of the level");
            if (last >= 0 && last != (int)P->last) return ctx->fail(FHH_E_STATE, "party_node_sums: shards disagree");
            last = P->last;
            v[(size_t)k] = P->vals.p;
            fused_shards.push_back(P);
        }
        if (last < 0) return ctx->fail(FHH_E_STATE, "party_node_sums: no shard holds clients");
        if (!fused_shards.empty() && fused_shards[0]->lfused) {   // r06: the shards' host partials, summed
            const uint64_t LC = fused_shards[0]->level_C;
            std::vector<uint64_t> h(LC * 2, 0);
            for (PartyState* P : fused_shards) {
                if (!P->lfused || P->level_C != LC) return ctx->fail(FHH_E_STATE, "party_node_sums: shards disagree");
                const int k0 = P->role == 0 ? 0 : 2;
                for (uint64_t c = 0; c < LC; c++) {
                    h[2 * c] += P->partials_host[4 * c + k0];
                    h[2 * c + 1] += P->partials_host[4 * c + k0 + 1];
                }
            }
            uint64_t* sums = static_cast<uint64_t*>(sums_a);
            if (sums)
                for (uint64_t c = 0; c < LC; c++) sums[c] = fhh::fe_canon_from_limbs(h[2 * c], h[2 * c + 1]);
            return FHH_OK;
        }
        const uint32_t fmt = last ? FHH_VALS_FE255_BLOCKPAIR : FHH_VALS_FE_U64;
        return group_node_sums(ctx, v.data(), false, 0, fmt, sums_a, sums_b);   // ld 0: each shard's n
    }
    PartyState* Pp = ctx->party;
    if (!Pp || Pp->step != 3 || Pp->covered != Pp->level_C)
        return ctx->fail(FHH_E_STATE, "party_node_sums: the level's OTs are not finished for every child");
    PartyState& P = *Pp;
    if (P.lfused) {   // r06: the partials the garble / evaluate calls copied to the host
        const int k0 = P.role == 0 ? 0 : 2;
        uint64_t* sums = static_cast<uint64_t*>(sums_a);
        if (sums)
            for (uint64_t c = 0; c < P.level_C; c++)
                sums[c] = fhh::fe_canon_from_limbs(P.partials_host[4 * c + k0], P.partials_host[4 * c + k0 + 1]);
        return FHH_OK;
    }
    // the garbler's value is r1 = v + mask, the evaluator's its C-OT output (written per chunk into
    // P.vals); rows of n values: FE as u64, FieldElm as a BlockPair (2 blocks)
    const void* vv[1] = {P.vals.p};
    if (P.last)
        return fhh_node_sums_fe255_device(ctx, vv, P.n, FHH_VALS_FE255_BLOCKPAIR, static_cast<uint32_t*>(sums_a),
                                          static_cast<uint32_t*>(sums_b));
    return fhh_node_sums_fe_device(ctx, vv, P.n, FHH_VALS_FE_U64, static_cast<uint64_t*>(sums_a));
}

int fhh_party_bytes_sent(const fhh_ctx* ctx, uint64_t* bytes) {
    CTX_CHECK(ctx);
    if (bytes) *bytes = ctx->party ? ctx->party->bytes_sent : 0;
    return FHH_OK;
}

// TEST MODE: the in-process level loop's material (fhh_sim_crawl gc = 2 with ideal base OTs) for
// prf_seed and level, split into the two parties' configs. Deterministic from one seed, so NOT private:
// a deployment draws each party's material on its own side (fuzzyheavyhitters_amd.party).
int fhh_gc_party_test_cfgs(uint64_t prf_seed, uint32_t level, fhh_gb_cfg* gb, fhh_ev_cfg* ev) {
    if (!gb || !ev) {
        g_err = "gc_party_test_cfgs: NULL output";
        return FHH_E_ARG;
    }
    std::memset(gb, 0, sizeof(*gb));
    std::memset(ev, 0, sizeof(*ev));
    uint8_t label_key[16], delta[16];   // the ideal-OT loop's; the r05 garbler draws no labels, Delta = s
    gc_level_material(prf_seed, level, label_key, delta, &gb->mask);
    for (uint32_t salt = 0; salt < 2; salt++) {
        uint32_t sw[4];
        ot_level_choice(prf_seed, level, salt, sw);
        std::memcpy(gb->base_choice[salt], sw, 16);
        for (uint32_t i = 0; i < 128; i++) {
            const uint32_t si = (sw[i >> 5] >> (i & 31)) & 1u;
            for (uint32_t b = 0; b < 2; b++) {
                // k_ot_level_keys' seeds (fhh_ot.hip ot_seed_word): the level loop's ideal base OTs
                const uint64_t z = host_mix64(prf_seed ^ 0x6f745f62617365ull ^ ((uint64_t)level << 24) ^
                                              ((uint64_t)salt << 20) ^ ((uint64_t)i << 2) ^ b);
                const uint64_t lo = z, hi = host_mix64(z);
                std::memcpy(ev->base_pairs[salt][i][b], &lo, 8);
                std::memcpy(ev->base_pairs[salt][i][b] + 8, &hi, 8);
            }
            std::memcpy(gb->base_chosen[salt][i], ev->base_pairs[salt][i][si], 16);
        }
    }
    return FHH_OK;
}

}  // extern "C"
