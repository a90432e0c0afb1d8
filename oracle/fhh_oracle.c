/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the per-level client-key evaluation of
 * sks-codes/fuzzyheavyhitters (Rust crate `counttree`, read-only at /root/reference).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library; the product library (fuzzyheavyhitters_amd/libfhh.so) never links it.
 *
 * The reference cannot be compiled here (Rust: no cargo/rustc, crates not vendored), so
 * this file restates it. Parity is pinned by:
 *   - FIPS-197 AES-128 known answers and OpenSSL's AES_encrypt (tests/test_oracle_kat.py),
 *   - the ibDCF comparison semantics derived from the algebra, checked exhaustively,
 *   - fastfield.rs's own known answers (FE tests, recip(999)).
 * Every function cites the reference file:line it follows.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

#if defined(__x86_64__)
#include <immintrin.h>
#include <cpuid.h>
#endif

/* ------------------------------------------------------------------ */
/* AES-128, portable byte-oriented FIPS-197 implementation.           */
/* Third-party algorithm: crate `aes 0.4.0` / `aesni 0.7.0`           */
/* (Cargo.lock:17-70), called at src/prg.rs:224 `encrypt_block`.      */
/* ------------------------------------------------------------------ */

static uint8_t g_sbox[256];
static uint8_t g_rk0[176];          /* expanded zero key, src/prg.rs:185-197 */
static int g_init = 0;

static uint8_t gf_mul(uint8_t a, uint8_t b) {
    uint8_t p = 0;
    for (int i = 0; i < 8; i++) {
        if (b & 1) p ^= a;
        uint8_t hi = a & 0x80;
        a <<= 1;
        if (hi) a ^= 0x1b;
        b >>= 1;
    }
    return p;
}

static uint8_t rotl8(uint8_t x, int s) { return (uint8_t)((x << s) | (x >> (8 - s))); }

static void build_sbox(void) {
    /* S(x) = affine(inverse(x)), FIPS-197 5.1.1 */
    for (int x = 0; x < 256; x++) {
        uint8_t inv = 0;
        if (x) {
            for (int y = 1; y < 256; y++)
                if (gf_mul((uint8_t)x, (uint8_t)y) == 1) { inv = (uint8_t)y; break; }
        }
        uint8_t s = inv ^ rotl8(inv, 1) ^ rotl8(inv, 2) ^ rotl8(inv, 3) ^ rotl8(inv, 4) ^ 0x63;
        g_sbox[x] = s;
    }
}

static void key_expand(const uint8_t key[16], uint8_t rk[176]) {
    memcpy(rk, key, 16);
    uint8_t rcon = 1;
    for (int i = 4; i < 44; i++) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 4 == 0) {
            uint8_t u = t[0];
            t[0] = g_sbox[t[1]] ^ rcon;
            t[1] = g_sbox[t[2]];
            t[2] = g_sbox[t[3]];
            t[3] = g_sbox[u];
            rcon = gf_mul(rcon, 2);
        }
        for (int k = 0; k < 4; k++) rk[4 * i + k] = rk[4 * (i - 4) + k] ^ t[k];
    }
}

static void oracle_init(void) {
    if (g_init) return;
#pragma omp critical(fhh_oracle_init)
    {
        if (!g_init) {
            uint8_t zero[16] = {0};
            build_sbox();
            key_expand(zero, g_rk0);
            __atomic_store_n(&g_init, 1, __ATOMIC_RELEASE);
        }
    }
}

static void aes128_encrypt_rk(const uint8_t rk[176], const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16];
    for (int i = 0; i < 16; i++) s[i] = in[i] ^ rk[i];
    for (int round = 1; round <= 10; round++) {
        uint8_t t[16];
        /* SubBytes + ShiftRows: state byte (r,c) lives at s[4c+r] */
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 4; r++)
                t[4 * c + r] = g_sbox[s[4 * ((c + r) & 3) + r]];
        if (round != 10) {
            for (int c = 0; c < 4; c++) {
                uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
                s[4 * c + 0] = gf_mul(a0, 2) ^ gf_mul(a1, 3) ^ a2 ^ a3;
                s[4 * c + 1] = a0 ^ gf_mul(a1, 2) ^ gf_mul(a2, 3) ^ a3;
                s[4 * c + 2] = a0 ^ a1 ^ gf_mul(a2, 2) ^ gf_mul(a3, 3);
                s[4 * c + 3] = gf_mul(a0, 3) ^ a1 ^ a2 ^ gf_mul(a3, 2);
            }
        } else {
            memcpy(s, t, 16);
        }
        for (int i = 0; i < 16; i++) s[i] ^= rk[16 * round + i];
    }
    memcpy(out, s, 16);
}

void orc_aes128_encrypt(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
    oracle_init();
    uint8_t rk[176];
    key_expand(key, rk);
    aes128_encrypt_rk(rk, in, out);
}

/* AES-128 with the fixed all-zero key (src/prg.rs:185-197 `FixedKeyPrgStream::new`). */
void orc_aes128_zero_encrypt(const uint8_t in[16], uint8_t out[16]) {
    oracle_init();
    aes128_encrypt_rk(g_rk0, in, out);
}

void orc_sbox(uint8_t out[256]) {
    oracle_init();
    memcpy(out, g_sbox, 256);
}

void orc_zero_round_keys(uint8_t out[176]) {
    oracle_init();
    memcpy(out, g_rk0, 176);
}

/* ---------------- AES-NI path (CPU baseline speed) ---------------- */
#if defined(__x86_64__)
static __m128i g_ni_rk[11];
static int g_ni_ready = 0;

int orc_aes_ni_available(void) {
    unsigned a, b, c, d;
    if (!__get_cpuid(1, &a, &b, &c, &d)) return 0;
    return (c & bit_AES) ? 1 : 0;
}

__attribute__((target("aes,sse4.1"))) static void ni_prepare(void) {
    oracle_init();
    for (int i = 0; i < 11; i++) g_ni_rk[i] = _mm_loadu_si128((const __m128i*)(g_rk0 + 16 * i));
    g_ni_ready = 1;
}

/* One non-pipelined AES-NI block, like the reference's single-block `encrypt_block`. */
__attribute__((target("aes,sse4.1"))) static inline __m128i ni_aes0(__m128i x) {
    x = _mm_xor_si128(x, g_ni_rk[0]);
    x = _mm_aesenc_si128(x, g_ni_rk[1]);
    x = _mm_aesenc_si128(x, g_ni_rk[2]);
    x = _mm_aesenc_si128(x, g_ni_rk[3]);
    x = _mm_aesenc_si128(x, g_ni_rk[4]);
    x = _mm_aesenc_si128(x, g_ni_rk[5]);
    x = _mm_aesenc_si128(x, g_ni_rk[6]);
    x = _mm_aesenc_si128(x, g_ni_rk[7]);
    x = _mm_aesenc_si128(x, g_ni_rk[8]);
    x = _mm_aesenc_si128(x, g_ni_rk[9]);
    return _mm_aesenclast_si128(x, g_ni_rk[10]);
}

__attribute__((target("aes,sse4.1"))) void orc_aes128_zero_encrypt_ni(const uint8_t in[16], uint8_t out[16]) {
    if (!g_ni_ready) ni_prepare();
    __m128i x = _mm_loadu_si128((const __m128i*)in);
    _mm_storeu_si128((__m128i*)out, ni_aes0(x));
}

/* Keyed AES-NI block under an expanded key (the GC label PRG and the OT extension's row PRG:
 * swanky's AesRng / scuttlebutt Aes128 run on AES-NI, as the reference builds with
 * target-cpu=native, README.md:43). */
__attribute__((target("aes,sse4.1"))) static void ni_aes_rk(const uint8_t rk[176], const uint8_t in[16],
                                                            uint8_t out[16]) {
    __m128i x = _mm_xor_si128(_mm_loadu_si128((const __m128i*)in), _mm_loadu_si128((const __m128i*)rk));
    for (int r = 1; r < 10; r++) x = _mm_aesenc_si128(x, _mm_loadu_si128((const __m128i*)(rk + 16 * r)));
    _mm_storeu_si128((__m128i*)out, _mm_aesenclast_si128(x, _mm_loadu_si128((const __m128i*)(rk + 160))));
}
#else
int orc_aes_ni_available(void) { return 0; }
void orc_aes128_zero_encrypt_ni(const uint8_t in[16], uint8_t out[16]) { orc_aes128_zero_encrypt(in, out); }
static void ni_aes_rk(const uint8_t rk[176], const uint8_t in[16], uint8_t out[16]) { aes128_encrypt_rk(rk, in, out); }
#endif

/* The GC / OT restatement (row f1) runs its AES on AES-NI when the CPU has it (-1: not yet
 * decided), the byte-wise FIPS-197 path otherwise; orc_gc_set_ni(0) forces the byte-wise path (the
 * tests compare both). */
static int g_gc_ni = -1;
void orc_gc_set_ni(int on) { g_gc_ni = on ? orc_aes_ni_available() : 0; }
int orc_gc_get_ni(void) {
    if (g_gc_ni < 0) g_gc_ni = orc_aes_ni_available();
    return g_gc_ni;
}
static void gc_aes_rk(const uint8_t rk[176], const uint8_t in[16], uint8_t out[16]) {
    if (orc_gc_get_ni()) ni_aes_rk(rk, in, out);
    else aes128_encrypt_rk(rk, in, out);
}
static void gc_aes0(const uint8_t in[16], uint8_t out[16]) {
    if (orc_gc_get_ni()) orc_aes128_zero_encrypt_ni(in, out);
    else orc_aes128_zero_encrypt(in, out);
}

/* ------------------------------------------------------------------ */
/* Fixed-key PRG (src/prg.rs)                                          */
/* ------------------------------------------------------------------ */

/* `inc_be` (src/prg.rs:273-276): _mm_add_epi64(v, _mm_set_epi64x(1, 0)) adds 1 to the
 * UPPER 64-bit lane (bytes 8..15 as a little-endian u64), no carry into bytes 0..7. */
static void ctr_inc(uint8_t k[16]) {
    uint64_t hi;
    memcpy(&hi, k + 8, 8);
    hi += 1;
    memcpy(k + 8, &hi, 8);
}

/* MMO block: `refill` (src/prg.rs:212-234) = AES_0(ctr) XOR ctr. */
static void mmo(const uint8_t ctr[16], uint8_t out[16], int use_ni) {
    uint8_t e[16];
    if (use_ni) orc_aes128_zero_encrypt_ni(ctr, e);
    else aes128_encrypt_rk(g_rk0, ctr, e);
    for (int i = 0; i < 16; i++) out[i] = e[i] ^ ctr[i];
}

/* `PrgSeed::expand_dir(!dir, dir)` (src/prg.rs:92-122) as called by eval_bit: only the
 * requested side is encrypted, the other is `skip_block`ed. bits4 receives
 * (bits.0, bits.1, y_bits.0, y_bits.1) read from the MASKED byte 0 (prg.rs:96-105). */
static void expand_dir_impl(const uint8_t seed[16], int dir, uint8_t out[16], uint8_t bits4[4], int use_ni) {
    uint8_t k[16];
    memcpy(k, seed, 16);
    k[0] &= 0xF0;                               /* prg.rs:96 */
    bits4[0] = (k[0] & 0x1) == 0;               /* prg.rs:102 */
    bits4[1] = (k[0] & 0x2) == 0;
    bits4[2] = (k[0] & 0x4) == 0;               /* prg.rs:103 */
    bits4[3] = (k[0] & 0x8) == 0;
    if (dir) ctr_inc(k);                        /* left block skipped: skip_block, prg.rs:205-210 */
    mmo(k, out, use_ni);
}

void orc_expand_dir(const uint8_t seed[16], int dir, uint8_t out[16], uint8_t bits4[4]) {
    oracle_init();
    expand_dir_impl(seed, dir, out, bits4, 0);
}

/* `PrgSeed::expand` (src/prg.rs:124-126): both children. */
static void expand_both(const uint8_t seed[16], uint8_t left[16], uint8_t right[16], uint8_t bits4[4], int use_ni) {
    expand_dir_impl(seed, 0, left, bits4, use_ni);
    expand_dir_impl(seed, 1, right, bits4, use_ni);
}

/* ------------------------------------------------------------------ */
/* ibDCF (src/ibDCF.rs)                                                */
/* cw_bits nibble: bit0 = bits.0, bit1 = bits.1, bit2 = y_bits.0, bit3 = y_bits.1    */
/* ------------------------------------------------------------------ */

/* `gen_ibDCF` (ibDCF.rs:138-164) with `gen_cor_word` (ibDCF.rs:84-119). Root seeds are
 * caller-provided (the reference draws them from thread_rng, prg.rs:153-158). */
static void gen_ibdcf_impl(const uint8_t* alpha, uint32_t L, int side, const uint8_t root0[16],
                           const uint8_t root1[16], uint8_t* cw_seed, uint8_t* cw_bits, int use_ni) {
    uint8_t seeds[2][16];
    int bits[2] = {0, 1};                       /* root_bits = (false, true), ibDCF.rs:140 */
    memcpy(seeds[0], root0, 16);
    memcpy(seeds[1], root1, 16);
    for (uint32_t l = 0; l < L; l++) {
        int bit = alpha[l] ? 1 : 0;
        uint8_t ds[2][2][16];                   /* data[b].seeds.{0,1} */
        uint8_t db[2][4];                       /* data[b].bits / y_bits */
        for (int b = 0; b < 2; b++) expand_both(seeds[b], ds[b][0], ds[b][1], db[b], use_ni);
        int keep = bit, lose = !bit;
        uint8_t cws[16];
        for (int i = 0; i < 16; i++) cws[i] = ds[0][lose][i] ^ ds[1][lose][i];          /* :91 */
        int cb0 = db[0][0] ^ db[1][0] ^ bit ^ 1;                                          /* :93 */
        int cb1 = db[0][1] ^ db[1][1] ^ bit;                                              /* :94 */
        int cy0 = db[0][2] ^ db[1][2] ^ (bit & !side);                                    /* :97 */
        int cy1 = db[0][3] ^ db[1][3] ^ ((!bit) & side);                                  /* :98 */
        int cwb[2] = {cb0, cb1};
        for (int b = 0; b < 2; b++) {                                                     /* :103-116 */
            memcpy(seeds[b], ds[b][keep], 16);
            if (bits[b])
                for (int i = 0; i < 16; i++) seeds[b][i] ^= cws[i];
            int nb = db[b][keep];
            if (bits[b]) nb ^= cwb[keep];
            bits[b] = nb;
        }
        memcpy(cw_seed + 16 * (size_t)l, cws, 16);
        cw_bits[l] = (uint8_t)(cb0 | (cb1 << 1) | (cy0 << 2) | (cy1 << 3));
    }
}

void orc_gen_ibdcf(const uint8_t* alpha, uint32_t L, int side, const uint8_t root0[16],
                   const uint8_t root1[16], uint8_t* cw_seed, uint8_t* cw_bits) {
    oracle_init();
    gen_ibdcf_impl(alpha, L, side, root0, root1, cw_seed, cw_bits, 0);
}

/* Batched interval keygen, `gen_interval` (ibDCF.rs:166-173) per dim: left key =
 * gen_ibDCF(l, side=true), right key = gen_ibDCF(r, side=false); both servers' keys share
 * cor_words (ibDCF.rs:152-163), so cw arrays are produced once.
 *   left_bits/right_bits: [n][d][L] (0/1)
 *   root_seeds: [n][d][2 side][2 server][16]
 *   cw_seed out: [n][d][2 side][L][16], cw_bits out: [n][d][2 side][L]            */
void orc_gen_keys(uint64_t n, uint32_t d, uint32_t L, const uint8_t* left_bits, const uint8_t* right_bits,
                  const uint8_t* root_seeds, uint8_t* cw_seed, uint8_t* cw_bits, int nthreads) {
    oracle_init();
    int ni = orc_aes_ni_available();
#if defined(__x86_64__)
    if (ni && !g_ni_ready) ni_prepare();
#endif
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads)
    for (int64_t c = 0; c < (int64_t)n; c++) {
        for (uint32_t j = 0; j < d; j++) {
            for (int s = 0; s < 2; s++) {
                const uint8_t* alpha = (s == 0 ? left_bits : right_bits) + ((size_t)c * d + j) * L;
                const uint8_t* rs = root_seeds + (((size_t)c * d + j) * 2 + s) * 32;
                size_t key = ((size_t)c * d + j) * 2 + s;
                gen_ibdcf_impl(alpha, L, s == 0 ? 1 : 0, rs, rs + 16, cw_seed + key * L * 16,
                               cw_bits + key * L, ni);
            }
        }
    }
}

/* `eval_bit` (ibDCF.rs:208-227). */
static inline void eval_bit_impl(const uint8_t seed[16], int t, int y, const uint8_t cws[16], uint8_t cwb,
                                 int dir, uint8_t out[16], uint8_t* t_out, uint8_t* y_out, int use_ni) {
    uint8_t b4[4];
    expand_dir_impl(seed, dir, out, b4, use_ni);   /* tau = expand_dir(!dir, dir) */
    int nb = b4[dir];                              /* tau.bits.get(dir) */
    int ny = b4[2 + dir];                          /* tau.y_bits.get(dir) */
    if (t) {
        for (int i = 0; i < 16; i++) out[i] ^= cws[i];
        nb ^= (cwb >> dir) & 1;
        ny ^= (cwb >> (2 + dir)) & 1;
    }
    ny ^= y;
    *t_out = (uint8_t)nb;
    *y_out = (uint8_t)ny;
}

void orc_eval_bit(const uint8_t seed[16], int t, int y, const uint8_t cw_seed[16], uint8_t cw_bits, int dir,
                  uint8_t out_seed[16], uint8_t* t_out, uint8_t* y_out) {
    oracle_init();
    eval_bit_impl(seed, t, y, cw_seed, cw_bits, dir, out_seed, t_out, y_out, 0);
}

/* ------------------------------------------------------------------ */
/* Collection engine (src/collect.rs), reference child order.          */
/* State arrays are node-major: [node][client][dim][side] -> seed(16), t, y.        */
/* ------------------------------------------------------------------ */

/* `tree_init` (collect.rs:67-92) + `eval_init` (ibDCF.rs:229-236):
 * key_idx [n][d][2], root_seed [n][d][2][16]. Output node 0. */
void orc_tree_init(uint64_t n, uint32_t d, const uint8_t* key_idx, const uint8_t* root_seed,
                   uint8_t* seeds, uint8_t* t, uint8_t* y) {
    size_t K = (size_t)n * d * 2;
    memcpy(seeds, root_seed, K * 16);
    for (size_t k = 0; k < K; k++) {
        t[k] = key_idx[k] ? 1 : 0;
        y[k] = key_idx[k] ? 1 : 0;
    }
}

/* One crawl level, `tree_crawl` frontier expansion (collect.rs:379-391) +
 * `make_tree_node` (collect.rs:94-119) + `eval_str` (ibDCF.rs:120-131).
 * Children are ordered by parent, then by i in `all_bit_vectors(d)` (lib.rs:125-129):
 * child i takes direction (i >> j) & 1 in dim j.
 *   cw_seed [n][d][2][L][16], cw_bits [n][d][2][L]
 *   parent_idx[F]: rows of the input state arrays that form the frontier (after prune)
 *   out arrays hold F * 2^d nodes.  Returns the number of AES blocks executed. */
uint64_t orc_level_expand(uint64_t n, uint32_t d, uint32_t L, uint32_t level, const uint8_t* cw_seed,
                          const uint8_t* cw_bits, uint64_t F, const uint64_t* parent_idx,
                          const uint8_t* in_seed, const uint8_t* in_t, const uint8_t* in_y,
                          uint8_t* out_seed, uint8_t* out_t, uint8_t* out_y, int nthreads, int use_ni) {
    oracle_init();
#if defined(__x86_64__)
    if (use_ni && !orc_aes_ni_available()) use_ni = 0;
    if (use_ni && !g_ni_ready) ni_prepare();
#else
    use_ni = 0;
#endif
    if (nthreads <= 0) nthreads = omp_get_max_threads();
    const uint32_t nch = 1u << d;
    const size_t per_node = (size_t)n * d * 2;
    for (uint64_t p = 0; p < F; p++) {
        const size_t src = (size_t)parent_idx[p];
        for (uint32_t i = 0; i < nch; i++) {
            const size_t dst = (size_t)p * nch + i;
#pragma omp parallel for schedule(static) num_threads(nthreads)
            for (int64_t c = 0; c < (int64_t)n; c++) {
                for (uint32_t j = 0; j < d; j++) {
                    int dir = (i >> j) & 1;
                    for (int s = 0; s < 2; s++) {
                        size_t key = ((size_t)c * d + j) * 2 + s;
                        size_t si = src * per_node + key, di = dst * per_node + key;
                        eval_bit_impl(in_seed + si * 16, in_t[si], in_y[si], cw_seed + (key * L + level) * 16,
                                      cw_bits[key * L + level], dir, out_seed + di * 16, out_t + di, out_y + di,
                                      use_ni);
                    }
                }
            }
        }
    }
    return (uint64_t)F * nch * n * d * 2;
}

/* Share strings (collect.rs:393-418): per (child, client), [left.y^left.t for each dim]
 * then [right.y^right.t for each dim]. out [C][n][2d]. */
void orc_share_bits(uint64_t C, uint64_t n, uint32_t d, const uint8_t* t, const uint8_t* y, uint8_t* out) {
    for (uint64_t c = 0; c < C; c++)
        for (uint64_t i = 0; i < n; i++)
            for (int s = 0; s < 2; s++)
                for (uint32_t j = 0; j < d; j++) {
                    size_t k = ((c * n + i) * d + j) * 2 + s;
                    out[(c * n + i) * 2 * d + (size_t)s * d + j] = t[k] ^ y[k];
                }
}

/* Plaintext stand-in for the GC equality test (equalitytest.rs:25-106): count, per child,
 * the clients whose two servers' share strings are equal (eq = mask ^ out, collect.rs:439-472). */
void orc_eq_count(uint64_t C, uint64_t n, uint32_t d, const uint8_t* t0, const uint8_t* y0, const uint8_t* t1,
                  const uint8_t* y1, uint64_t* counts) {
    const size_t per = (size_t)n * d * 2;
    for (uint64_t c = 0; c < C; c++) {
        uint64_t cnt = 0;
        for (uint64_t i = 0; i < n; i++) {
            int eq = 1;
            for (size_t k = 0; k < (size_t)d * 2; k++) {
                size_t idx = c * per + i * d * 2 + k;
                if ((t0[idx] ^ y0[idx]) != (t1[idx] ^ y1[idx])) { eq = 0; break; }
            }
            cnt += (uint64_t)eq;
        }
        counts[c] = cnt;
    }
}

/* ------------------------------------------------------------------ */
/* FE, p = 2^62 - 2^30 - 1 (src/fastfield.rs)                          */
/* ------------------------------------------------------------------ */
#define FE_NBITS 62
#define FE_OFFSET 30
#define FE_P ((((uint64_t)1) << FE_NBITS) - (((uint64_t)1) << FE_OFFSET) - 1)
#define FE_MASK ((((uint64_t)1) << FE_NBITS) - 1)

uint64_t orc_fe_bit_reduce_once(uint64_t v) {       /* fastfield.rs:86-95 */
    uint64_t excess = v >> FE_NBITS;
    uint64_t low = v & FE_MASK;
    return low + excess + (excess << FE_OFFSET);
}
static uint64_t fe_reduce_by_p(uint64_t v) {        /* fastfield.rs:100-107 */
    uint64_t diff = v - FE_P;
    uint64_t mask = (uint64_t)(((int64_t)(diff & ((uint64_t)1 << 63))) >> 63);
    return (mask & v) | (~mask & diff);
}
uint64_t orc_fe_new(uint64_t v) { return orc_fe_bit_reduce_once(v); }                       /* :112-118 */
uint64_t orc_fe_value(uint64_t val) { return fe_reduce_by_p(orc_fe_bit_reduce_once(val)); } /* :147-152 */
uint64_t orc_fe_add(uint64_t a, uint64_t b) { return orc_fe_new(a + b); }                   /* :226-233 */
uint64_t orc_fe_neg(uint64_t a) { return orc_fe_new(FE_P * 2 - a); }                        /* :235-242 */
uint64_t orc_fe_sub(uint64_t a, uint64_t b) { return orc_fe_add(a, orc_fe_neg(b)); }        /* :244-249 */
uint64_t orc_fe_mul(uint64_t a, uint64_t b) {                                               /* :299-328 */
    unsigned __int128 prod = (unsigned __int128)a * b;
    for (int r = 0; r < 2; r++) {
        unsigned __int128 low = prod & FE_MASK;
        unsigned __int128 high = prod >> FE_NBITS;
        prod = low + (high << FE_OFFSET) + high;
    }
    return orc_fe_new((uint64_t)prod);
}

/* Node sum with `add_lazy` = `add` for FE (field.rs:219-222; collect.rs:487-501), folded
 * in client order. Returns the internal (bit-reduced-once) val; compare value(). */
uint64_t orc_fe_fold_sum(const uint64_t* vals, uint64_t n) {
    uint64_t acc = 0;
    for (uint64_t i = 0; i < n; i++) acc = orc_fe_add(acc, orc_fe_new(vals[i]));
    return acc;
}

/* ------------------------------------------------------------------ */
/* Simulated OT share values (harness-defined).         */
/* The real values come from ALSZ OT (collect.rs:439-472); the        */
/* reference draws r0 from thread_rng, so any fixed PRF is as faithful. */
/* ------------------------------------------------------------------ */
static inline uint64_t mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ULL;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
uint64_t orc_sim_prf(uint64_t seed, uint64_t level, uint64_t child, uint64_t client, uint32_t word) {
    return mix64(mix64(mix64(mix64(seed ^ level) ^ child) ^ client) ^ word);
}

/* ------------------------------------------------------------------ */
/* Sketch + Beaver-triple verification (row a9; DEAD in the reference: */
/* src/sketch.rs and src/mpc.rs are fully commented out, so this      */
/* restates the commented text — parity unpinned beyond the protocol's */
/* own identities, see tests/test_sketch.py).                          */
/* ------------------------------------------------------------------ */

/* PrgSeed::to_rng (prg.rs:82-90): AES-128-CTR, key = seed, IV = 0. Crate `aes-ctr 0.4`
 * (Cargo.lock) counts the whole 128-bit block big-endian from the IV, so keystream block b is
 * AES_seed(BE128(b)). PrgStream::next_u64 = next_u64_via_fill (prg.rs:166-168, rand_core):
 * the next 8 keystream bytes, little-endian. Draw number `pos` = bytes [8 pos, 8 pos + 8). */
uint64_t orc_prg_stream_u64(const uint8_t seed[16], uint64_t pos) {
    oracle_init();
    uint8_t rk[176], ctr[16] = {0}, ks[16];
    key_expand(seed, rk);
    const uint64_t b = pos >> 1;
    for (int i = 0; i < 8; i++) ctr[15 - i] = (uint8_t)(b >> (8 * i));
    aes128_encrypt_rk(rk, ctr, ks);
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v |= (uint64_t)ks[8 * (pos & 1) + i] << (8 * i);
    return v;
}

/* FE::from_rng (field.rs:252-264 + fastfield.rs:125-139): redraw until the low 62 bits are
 * below p. Returns the FE val; *pos advances past the draws used. */
static uint64_t fe_from_stream(const uint8_t rk[176], uint64_t* pos, uint8_t ks[16], uint64_t* ks_block) {
    for (;;) {
        const uint64_t b = *pos >> 1;
        if (*ks_block != b) {
            uint8_t ctr[16] = {0};
            for (int i = 0; i < 8; i++) ctr[15 - i] = (uint8_t)(b >> (8 * i));
            aes128_encrypt_rk(rk, ctr, ks);
            *ks_block = b;
        }
        uint64_t v = 0;
        for (int i = 0; i < 8; i++) v |= (uint64_t)ks[8 * (*pos & 1) + i] << (8 * i);
        (*pos)++;
        v &= FE_MASK;
        if (v < FE_P) return v;
    }
}

/* SketchDPFKey::sketch_at (sketch.rs:157-200) for T = FE, one key:
 *   rand1..3 = from_rng, then per (x, kx): r = from_rng; r2 = r*r;
 *   r_x += x*r; r2_x += x*r2; r_kx += kx*r   (mul_lazy = mul, add_lazy = add for FE).
 * out6 = canonical {r_x, r2_x, r_kx, rand1, rand2, rand3}; x / kx as FE vals. */
void orc_sketch_fe(const uint8_t seed[16], uint32_t n_nodes, const uint64_t* x, const uint64_t* kx, uint64_t* out6) {
    oracle_init();
    uint8_t rk[176], ks[16];
    key_expand(seed, rk);
    uint64_t pos = 0, blk = ~(uint64_t)0;
    const uint64_t rand1 = fe_from_stream(rk, &pos, ks, &blk);
    const uint64_t rand2 = fe_from_stream(rk, &pos, ks, &blk);
    const uint64_t rand3 = fe_from_stream(rk, &pos, ks, &blk);
    uint64_t r_x = 0, r2_x = 0, r_kx = 0;
    for (uint32_t j = 0; j < n_nodes; j++) {
        const uint64_t r = fe_from_stream(rk, &pos, ks, &blk);
        const uint64_t r2 = orc_fe_mul(r, r);
        r_x = orc_fe_add(r_x, orc_fe_mul(x[j], r));
        r2_x = orc_fe_add(r2_x, orc_fe_mul(x[j], r2));
        r_kx = orc_fe_add(r_kx, orc_fe_mul(kx[j], r));
    }
    out6[0] = orc_fe_value(r_x);
    out6[1] = orc_fe_value(r2_x);
    out6[2] = orc_fe_value(r_kx);
    out6[3] = orc_fe_value(rand1);
    out6[4] = orc_fe_value(rand2);
    out6[5] = orc_fe_value(rand3);
}

void orc_sketch_fe_batch(uint64_t n_keys, uint32_t n_nodes, const uint8_t* seeds, const uint64_t* x,
                         const uint64_t* kx, uint64_t* out6, int nthreads) {
    oracle_init();
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t i = 0; i < (int64_t)n_keys; i++)
        orc_sketch_fe(seeds + 16 * i, n_nodes, x + (uint64_t)i * n_nodes, kx + (uint64_t)i * n_nodes, out6 + 6 * i);
}

/* MulState::new (mpc.rs:83-140) for T = FE: xs = [r_x, k, r_x], ys = [r_x, k, k],
 * zs = [-r2_x, -k2, -r_kx], rs = [rand1, rand2, rand3]. */
static void mul_state(const uint64_t* sk6, uint64_t mac, uint64_t mac2, uint64_t xs[3], uint64_t ys[3],
                      uint64_t zs[3], uint64_t rs[3]) {
    xs[0] = sk6[0]; ys[0] = sk6[0]; zs[0] = orc_fe_neg(sk6[1]);
    xs[1] = mac;    ys[1] = mac;    zs[1] = orc_fe_neg(mac2);
    xs[2] = sk6[0]; ys[2] = mac;    zs[2] = orc_fe_neg(sk6[2]);
    rs[0] = sk6[3]; rs[1] = sk6[4]; rs[2] = sk6[5];
}

/* MulState::cor_share (mpc.rs:142-158): d_i = x_i - a_i, e_i = y_i - b_i.
 * triples9 = {a0,b0,c0, a1,b1,c1, a2,b2,c2}; out6 = canonical {d0,d1,d2,e0,e1,e2}. */
void orc_mul_cor_share_fe(const uint64_t* sk6, uint64_t mac, uint64_t mac2, const uint64_t* triples9,
                          uint64_t* out6) {
    uint64_t xs[3], ys[3], zs[3], rs[3];
    mul_state(sk6, mac, mac2, xs, ys, zs, rs);
    for (int i = 0; i < 3; i++) {
        out6[i] = orc_fe_value(orc_fe_sub(xs[i], triples9[3 * i]));
        out6[3 + i] = orc_fe_value(orc_fe_sub(ys[i], triples9[3 * i + 1]));
    }
}

/* MulState::cor (mpc.rs:160-180): d = d0 + d1, e = e0 + e1. */
void orc_mul_cor_fe(const uint64_t* s0, const uint64_t* s1, uint64_t* cor6) {
    for (int k = 0; k < 6; k++) cor6[k] = orc_fe_value(orc_fe_add(orc_fe_add(0, s0[k]), s1[k]));
}

/* MulState::out_share (mpc.rs:182-212): sum_i r_i * ([server 1] d*e + d*b + e*a + c + z). */
uint64_t orc_mul_out_share_fe(int server_idx, const uint64_t* sk6, uint64_t mac, uint64_t mac2,
                              const uint64_t* triples9, const uint64_t* cor6) {
    uint64_t xs[3], ys[3], zs[3], rs[3];
    mul_state(sk6, mac, mac2, xs, ys, zs, rs);
    uint64_t out = 0;
    for (int i = 0; i < 3; i++) {
        const uint64_t d = cor6[i], e = cor6[3 + i];
        const uint64_t a = triples9[3 * i], b = triples9[3 * i + 1], c = triples9[3 * i + 2];
        uint64_t term = 0;
        if (server_idx) term = orc_fe_add(term, orc_fe_mul(d, e));
        term = orc_fe_add(term, orc_fe_mul(d, b));
        term = orc_fe_add(term, orc_fe_mul(e, a));
        term = orc_fe_add(term, c);
        term = orc_fe_add(term, zs[i]);
        term = orc_fe_mul(term, rs[i]);
        out = orc_fe_add(out, term);
    }
    return orc_fe_value(out);
}

/* MulState::verify (mpc.rs:214-220): out0 + out1 == 0. */
int orc_mul_verify_fe(uint64_t out0, uint64_t out1) { return orc_fe_value(orc_fe_add(out0, out1)) == 0; }

/* The whole per-level check of main.rs:14-70 (verify_sketches) for a batch of keys, both
 * servers in one process: sketch, cor shares, cor, out shares, verify -> ok[n]. */
void orc_sketch_verify_fe_batch(uint64_t n_keys, uint32_t n_nodes, const uint8_t* seeds, const uint64_t* x0,
                                const uint64_t* kx0, const uint64_t* x1, const uint64_t* kx1,
                                const uint64_t* mac /*[2][n]*/, const uint64_t* mac2 /*[2][n]*/,
                                const uint64_t* triples /*[2][n][9]*/, uint8_t* ok, uint64_t* out_shares /*[2][n]*/,
                                int nthreads) {
    oracle_init();
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 64)
    for (int64_t i = 0; i < (int64_t)n_keys; i++) {
        uint64_t sk[2][6], cs[2][6], cor[6], o[2];
        const uint64_t* xs[2] = {x0, x1};
        const uint64_t* kxs[2] = {kx0, kx1};
        for (int s = 0; s < 2; s++)
            orc_sketch_fe(seeds + 16 * i, n_nodes, xs[s] + (uint64_t)i * n_nodes, kxs[s] + (uint64_t)i * n_nodes,
                          sk[s]);
        for (int s = 0; s < 2; s++)
            orc_mul_cor_share_fe(sk[s], mac[s * n_keys + i], mac2[s * n_keys + i], triples + (s * n_keys + i) * 9,
                                 cs[s]);
        orc_mul_cor_fe(cs[0], cs[1], cor);
        for (int s = 0; s < 2; s++)
            o[s] = orc_mul_out_share_fe(s, sk[s], mac[s * n_keys + i], mac2[s * n_keys + i],
                                        triples + (s * n_keys + i) * 9, cor);
        ok[i] = (uint8_t)orc_mul_verify_fe(o[0], o[1]);
        if (out_shares) {
            out_shares[i] = o[0];
            out_shares[n_keys + i] = o[1];
        }
    }
}

/* ------------------------------------------------------------------ */
/* Row a9, last level: sketch_at_last (sketch.rs:202-245) and MulState  */
/* (mpc.rs:83-222) for U = FieldElm (BigUint mod p = 2^255 - 19,       */
/* field.rs:14-30,312-372). Values: 8 x u32 little-endian limbs.       */
/* FieldElm's lazy ops are exact BigUint add / mul followed by one     */
/* reduce (field.rs:337-349), so every result equals the same          */
/* expression computed mod p — which is how it is computed here.       */
/* ------------------------------------------------------------------ */
static const uint32_t P255[8] = {0xFFFFFFEDu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu,
                                 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0x7FFFFFFFu};

static int fe255_geq_p(const uint32_t a[8]) {
    for (int k = 7; k >= 0; k--) {
        if (a[k] > P255[k]) return 1;
        if (a[k] < P255[k]) return 0;
    }
    return 1;
}

/* a (< 2^256) -> a mod p, assuming a < 2 p + 2^255 (one or two subtractions) */
static void fe255_canon(uint32_t a[8]) {
    for (int it = 0; it < 3 && fe255_geq_p(a); it++) {
        uint64_t borrow = 0;
        for (int k = 0; k < 8; k++) {
            const uint64_t v = (uint64_t)a[k] - P255[k] - borrow;
            a[k] = (uint32_t)v;
            borrow = (v >> 63) & 1;
        }
    }
}

/* 16-limb product -> mod p: x = lo + 2^256 hi == lo + 38 hi (2^256 = 38 mod p) */
static void fe255_reduce16(const uint32_t x[16], uint32_t out[8]) {
    uint64_t t[9];
    uint64_t c = 0;
    for (int k = 0; k < 8; k++) {
        const uint64_t v = (uint64_t)x[k] + (uint64_t)x[8 + k] * 38u + c;
        t[k] = v & 0xFFFFFFFFu;
        c = v >> 32;
    }
    t[8] = c;   /* < 39 */
    /* fold t[8] * 2^256 again */
    uint32_t r[8];
    c = t[8] * 38u;
    for (int k = 0; k < 8; k++) {
        const uint64_t v = t[k] + c;
        r[k] = (uint32_t)v;
        c = v >> 32;
    }
    if (c) {   /* a carry out of 2^256 once more (only for r near 2^256) */
        uint64_t cc = 38;
        for (int k = 0; k < 8 && cc; k++) {
            const uint64_t v = (uint64_t)r[k] + cc;
            r[k] = (uint32_t)v;
            cc = v >> 32;
        }
    }
    /* r < 2^256 = 2 p + 38: at most two subtractions of p (the top bit may be set) */
    for (int it = 0; it < 2; it++) {
        if (!fe255_geq_p(r)) break;
        uint64_t borrow = 0;
        for (int k = 0; k < 8; k++) {
            const uint64_t v = (uint64_t)r[k] - P255[k] - borrow;
            r[k] = (uint32_t)v;
            borrow = (v >> 63) & 1;
        }
    }
    memcpy(out, r, 32);
}

void orc_fe255_mul(const uint32_t a[8], const uint32_t b[8], uint32_t out[8]) {
    uint32_t x[16] = {0};
    for (int i = 0; i < 8; i++) {
        uint64_t c = 0;
        for (int j = 0; j < 8; j++) {
            const uint64_t v = (uint64_t)a[i] * b[j] + x[i + j] + c;
            x[i + j] = (uint32_t)v;
            c = v >> 32;
        }
        x[i + 8] = (uint32_t)c;
    }
    fe255_reduce16(x, out);
}

void orc_fe255_add(const uint32_t a[8], const uint32_t b[8], uint32_t out[8]) {
    uint32_t x[16] = {0};
    uint64_t c = 0;
    for (int k = 0; k < 8; k++) {
        const uint64_t v = (uint64_t)a[k] + b[k] + c;
        x[k] = (uint32_t)v;
        c = v >> 32;
    }
    x[8] = (uint32_t)c;
    fe255_reduce16(x, out);
}

/* p - a for canonical a (the Group::negate of field.rs:361-364 gives p for a = 0: equal mod p) */
void orc_fe255_neg(const uint32_t a[8], uint32_t out[8]) {
    uint32_t r[8];
    uint64_t borrow = 0;
    for (int k = 0; k < 8; k++) {
        const uint64_t v = (uint64_t)P255[k] - a[k] - borrow;
        r[k] = (uint32_t)v;
        borrow = (v >> 63) & 1;
    }
    fe255_canon(r);
    memcpy(out, r, 32);
}

void orc_fe255_sub(const uint32_t a[8], const uint32_t b[8], uint32_t out[8]) {   /* field.rs:352-359 */
    uint32_t nb[8];
    orc_fe255_neg(b, nb);
    orc_fe255_add(a, nb, out);
}

/* FieldElm::from_rng (field.rs:367-372) = num-bigint 0.3.3 `gen_biguint_below(p)` (not vendored;
 * its published algorithm): loop { n = gen_biguint(bits(p) = 255); if n < p { return n } }, with
 * gen_biguint = ceil(255 / 32) = 8 u32 digits filled by `Rng::fill` (rand 0.7: fill_bytes of the
 * digits' 32 bytes, each digit little-endian), then the top digit >>= 32 - 255 % 32 = 1
 * (`gen_bits`). ASSUMPTION (parity unpinned): that digit fill order and the shift — num-bigint
 * is absent here, so no reference output pins them. The PrgStream is byte-continuous
 * (apply_keystream), so a draw is keystream bytes [32 m, 32 m + 32) = blocks 2 m, 2 m + 1. */
static void fe255_from_stream(const uint8_t rk[176], uint64_t* pos /* in 32-B draws */, uint32_t out[8]) {
    for (;;) {
        uint8_t bytes[32];
        for (int h = 0; h < 2; h++) {
            const uint64_t b = 2 * *pos + h;
            uint8_t ctr[16] = {0};
            for (int i = 0; i < 8; i++) ctr[15 - i] = (uint8_t)(b >> (8 * i));
            aes128_encrypt_rk(rk, ctr, bytes + 16 * h);
        }
        (*pos)++;
        uint32_t d[8];
        for (int k = 0; k < 8; k++)
            d[k] = (uint32_t)bytes[4 * k] | ((uint32_t)bytes[4 * k + 1] << 8) | ((uint32_t)bytes[4 * k + 2] << 16) |
                   ((uint32_t)bytes[4 * k + 3] << 24);
        d[7] >>= 1;
        if (!fe255_geq_p(d)) {
            memcpy(out, d, 32);
            return;
        }
    }
}

/* one draw of the FieldElm stream for tests: draw number m (no redraw applied) */
void orc_fe255_stream_draw(const uint8_t seed[16], uint64_t m, uint32_t out[8]) {
    oracle_init();
    uint8_t rk[176];
    key_expand(seed, rk);
    uint8_t bytes[32];
    for (int h = 0; h < 2; h++) {
        const uint64_t b = 2 * m + h;
        uint8_t ctr[16] = {0};
        for (int i = 0; i < 8; i++) ctr[15 - i] = (uint8_t)(b >> (8 * i));
        aes128_encrypt_rk(rk, ctr, bytes + 16 * h);
    }
    for (int k = 0; k < 8; k++)
        out[k] = (uint32_t)bytes[4 * k] | ((uint32_t)bytes[4 * k + 1] << 8) | ((uint32_t)bytes[4 * k + 2] << 16) |
                 ((uint32_t)bytes[4 * k + 3] << 24);
    out[7] >>= 1;
}

/* sketch_at_last (sketch.rs:202-245), one key: rand1..3 = from_rng, then per (x, kx):
 * r = from_rng; r2 = r * r; r_x += x r; r2_x += x r2; r_kx += kx r; reduce.
 * x, kx [n_nodes][8]; out6 [6][8] canonical {r_x, r2_x, r_kx, rand1, rand2, rand3}. */
void orc_sketch_fe255(const uint8_t seed[16], uint32_t n_nodes, const uint32_t* x, const uint32_t* kx, uint32_t* out6) {
    oracle_init();
    uint8_t rk[176];
    key_expand(seed, rk);
    uint64_t pos = 0;
    uint32_t rnd[3][8], acc[3][8];
    memset(acc, 0, sizeof acc);
    for (int i = 0; i < 3; i++) fe255_from_stream(rk, &pos, rnd[i]);
    for (uint32_t j = 0; j < n_nodes; j++) {
        uint32_t r[8], r2[8], t[8], xj[8], kxj[8];
        fe255_from_stream(rk, &pos, r);
        orc_fe255_mul(r, r, r2);
        memcpy(xj, x + 8 * (size_t)j, 32);
        memcpy(kxj, kx + 8 * (size_t)j, 32);
        orc_fe255_mul(xj, r, t);
        orc_fe255_add(acc[0], t, acc[0]);
        orc_fe255_mul(xj, r2, t);
        orc_fe255_add(acc[1], t, acc[1]);
        orc_fe255_mul(kxj, r, t);
        orc_fe255_add(acc[2], t, acc[2]);
    }
    memcpy(out6, acc, 96);
    memcpy(out6 + 24, rnd, 96);
}

void orc_sketch_fe255_batch(uint64_t n_keys, uint32_t n_nodes, const uint8_t* seeds, const uint32_t* x,
                            const uint32_t* kx, uint32_t* out6, int nthreads) {
    oracle_init();
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t i = 0; i < (int64_t)n_keys; i++)
        orc_sketch_fe255(seeds + 16 * i, n_nodes, x + (uint64_t)i * n_nodes * 8, kx + (uint64_t)i * n_nodes * 8,
                         out6 + 48 * i);
}

/* MulState::new (mpc.rs:83-140) for U: xs = [r_x, k, r_x], ys = [r_x, k, k],
 * zs = [-r2_x, -k2, -r_kx], rs = [rand1, rand2, rand3]. */
static void mul_state255(const uint32_t* sk6, const uint32_t* mac, const uint32_t* mac2, uint32_t xs[3][8],
                         uint32_t ys[3][8], uint32_t zs[3][8], uint32_t rs[3][8]) {
    memcpy(xs[0], sk6, 32);     memcpy(ys[0], sk6, 32);     orc_fe255_neg(sk6 + 8, zs[0]);
    memcpy(xs[1], mac, 32);     memcpy(ys[1], mac, 32);     orc_fe255_neg(mac2, zs[1]);
    memcpy(xs[2], sk6, 32);     memcpy(ys[2], mac, 32);     orc_fe255_neg(sk6 + 16, zs[2]);
    for (int i = 0; i < 3; i++) memcpy(rs[i], sk6 + 8 * (3 + i), 32);
}

/* MulState::cor_share (mpc.rs:142-158): triples9 [3 triples][a, b, c][8]; out6 [d0 d1 d2 e0 e1 e2][8] */
void orc_mul_cor_share_fe255(const uint32_t* sk6, const uint32_t* mac, const uint32_t* mac2, const uint32_t* triples9,
                             uint32_t* out6) {
    uint32_t xs[3][8], ys[3][8], zs[3][8], rs[3][8];
    mul_state255(sk6, mac, mac2, xs, ys, zs, rs);
    for (int i = 0; i < 3; i++) {
        orc_fe255_sub(xs[i], triples9 + 8 * (3 * i), out6 + 8 * i);
        orc_fe255_sub(ys[i], triples9 + 8 * (3 * i + 1), out6 + 8 * (3 + i));
    }
}

/* MulState::out_share (mpc.rs:182-212): sum_i r_i ([server 1] d e + d b + e a + c + z) */
void orc_mul_out_share_fe255(int server_idx, const uint32_t* sk6, const uint32_t* mac, const uint32_t* mac2,
                             const uint32_t* triples9, const uint32_t* cor6, uint32_t* out) {
    uint32_t xs[3][8], ys[3][8], zs[3][8], rs[3][8];
    mul_state255(sk6, mac, mac2, xs, ys, zs, rs);
    uint32_t acc[8] = {0};
    for (int i = 0; i < 3; i++) {
        const uint32_t* d = cor6 + 8 * i;
        const uint32_t* e = cor6 + 8 * (3 + i);
        const uint32_t* a = triples9 + 8 * (3 * i);
        const uint32_t* b = triples9 + 8 * (3 * i + 1);
        const uint32_t* c = triples9 + 8 * (3 * i + 2);
        uint32_t term[8] = {0}, t[8];
        if (server_idx) orc_fe255_mul(d, e, term);
        orc_fe255_mul(d, b, t);
        orc_fe255_add(term, t, term);
        orc_fe255_mul(e, a, t);
        orc_fe255_add(term, t, term);
        orc_fe255_add(term, c, term);
        orc_fe255_add(term, zs[i], term);
        orc_fe255_mul(term, rs[i], t);
        orc_fe255_add(acc, t, acc);
    }
    memcpy(out, acc, 32);
}

/* main.rs:14-70 verify_sketches at the last level, both servers: ok[n] (and out_shares [2][n][8]) */
void orc_sketch_verify_fe255_batch(uint64_t n_keys, uint32_t n_nodes, const uint8_t* seeds, const uint32_t* x0,
                                   const uint32_t* kx0, const uint32_t* x1, const uint32_t* kx1,
                                   const uint32_t* mac /*[2][n][8]*/, const uint32_t* mac2 /*[2][n][8]*/,
                                   const uint32_t* triples /*[2][n][9][8]*/, uint8_t* ok,
                                   uint32_t* out_shares /*[2][n][8]*/, int nthreads) {
    oracle_init();
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16)
    for (int64_t i = 0; i < (int64_t)n_keys; i++) {
        uint32_t sk[2][48], cs[2][48], cor[48], o[2][8], sum[8];
        const uint32_t* xs[2] = {x0, x1};
        const uint32_t* kxs[2] = {kx0, kx1};
        for (int s = 0; s < 2; s++)
            orc_sketch_fe255(seeds + 16 * i, n_nodes, xs[s] + (uint64_t)i * n_nodes * 8,
                             kxs[s] + (uint64_t)i * n_nodes * 8, sk[s]);
        for (int s = 0; s < 2; s++)
            orc_mul_cor_share_fe255(sk[s], mac + (s * n_keys + i) * 8, mac2 + (s * n_keys + i) * 8,
                                    triples + (s * n_keys + i) * 72, cs[s]);
        for (int k = 0; k < 6; k++) orc_fe255_add(cs[0] + 8 * k, cs[1] + 8 * k, cor + 8 * k);   /* MulState::cor */
        for (int s = 0; s < 2; s++)
            orc_mul_out_share_fe255(s, sk[s], mac + (s * n_keys + i) * 8, mac2 + (s * n_keys + i) * 8,
                                    triples + (s * n_keys + i) * 72, cor, o[s]);
        orc_fe255_add(o[0], o[1], sum);   /* MulState::verify (mpc.rs:214-220) */
        int zero = 1;
        for (int k = 0; k < 8; k++) zero &= sum[k] == 0;
        ok[i] = (uint8_t)zero;
        if (out_shares) {
            memcpy(out_shares + 8 * i, o[0], 32);
            memcpy(out_shares + 8 * (n_keys + i), o[1], 32);
        }
    }
}

/* ------------------------------------------------------------------ */
/* Row f1: garbled-circuit equality test (equalitytest.rs:25-219).    */
/* Third-party algorithm: swanky `fancy-garbling` @553ede0 (not       */
/* vendored). Restated from the published schemes it implements:     */
/* free-XOR + half-gates (Zahur, Rosulek, Evans, EUROCRYPT 2015) with */
/* the TCCR hash H(x, i) = pi(pi(x) ^ i) ^ pi(x) (Guo, Katz, Wang, Yu,*/
/* S&P 2020), pi = AES-128 under the all-zero key (swanky's fixed key */
/* is not restatable). Circuit: bin_eq_bundles (:128-147) = and_many  */
/* of NOT(x_j ^ y_j), folded left; XOR the garbler's mask (:165-189). */
/* Parity: functional (eq_gc, :222-266) — wire format unpinned.       */
/* ------------------------------------------------------------------ */
static void gc_tccr(const uint8_t x[16], uint64_t tweak, uint8_t out[16]) {
    uint8_t px[16], q[16], y[16];
    gc_aes0(x, px);
    memcpy(q, px, 16);
    for (int k = 0; k < 8; k++) q[k] ^= (uint8_t)(tweak >> (8 * k));
    gc_aes0(q, y);
    for (int k = 0; k < 16; k++) out[k] = y[k] ^ px[k];
}

static void gc_xor(uint8_t* d, const uint8_t* a, const uint8_t* b) {
    for (int k = 0; k < 16; k++) d[k] = a[k] ^ b[k];
}

static void ot_cr_hash(const uint8_t x[16], uint8_t out[16]);
static uint64_t cot_fe_of_block(const uint8_t b[16]);

/* r05c: the FE share from the circuit's output labels instead of a second OT. The output wire
 * o = eq ^ mask has the labels W_0 (o = 0) and W_1 = W_0 ^ D; the evaluator holds W_o and knows o.
 * That is the correlated-OT situation of orc_cot_extend mode 2 with (q_j, s) = (W_0, D) and the
 * evaluator's GC output as its choice, so the same pair is formed from the same hash: v = H(W_0) as a
 * little-endian u128 mod p, pair[0] = v, pair[1] = mask ? v + 1 : v - 1, the garbler's node value
 * r1 = v + mask, y = lo64(H(W_1)) ^ pair[1] (8 B); the evaluator's value = o ? lo64(H(W_o)) ^ y : H(W_o)
 * mod p. H = cr_hash (pi(x) ^ x), as the OT's. collect.rs:437-452 (the pair and its order). */
static void gc_share_garbler(const uint8_t eq0[16], const uint8_t D[16], uint32_t mask, uint64_t* gv_out,
                             uint64_t* y_out) {
    uint8_t w0[16], w1[16], h0[16], h1[16];
    memcpy(w0, eq0, 16);
    if (mask & 1) gc_xor(w0, w0, D);          /* o = 0 <=> eq = mask */
    gc_xor(w1, w0, D);
    ot_cr_hash(w0, h0);
    ot_cr_hash(w1, h1);
    const uint64_t v = cot_fe_of_block(h0);
    const uint64_t gv = (mask & 1) ? (v + 1 == FE_P ? 0 : v + 1) : v;     /* r1 = v + mask */
    const uint64_t p1 = (mask & 1) ? gv : (v == 0 ? FE_P - 1 : v - 1);     /* pair[1] */
    uint64_t hl;
    memcpy(&hl, h1, 8);
    *gv_out = gv;
    *y_out = hl ^ p1;
}

static uint64_t gc_share_evaluator(const uint8_t w[16], int o, uint64_t y) {
    uint8_t h[16];
    ot_cr_hash(w, h);
    uint64_t hl;
    memcpy(&hl, h, 8);
    return o ? (hl ^ y) : cot_fe_of_block(h);
}

/* Garbler (multiple_gb_equality_test, :25-64) for n tests of `bits` bits with an ideal OT for the
 * evaluator's labels. Layouts: tables [n][bits-1][2][16], gb_labels [n][bits+1][16] (mask last),
 * ev_labels [n][bits][16]. Every zero label is AES_key(LE128(nonce + t S + w)), S = the power of two
 * >= 2 bits + 1 (w < bits: the garbler's string, w = bits: the mask, w > bits: the evaluator's
 * string); the evaluator's ACTIVE labels (what an OT would deliver, gb_set_fancy_inputs :67-82) are
 * written to ev_labels. */
static void gc_garble_impl(uint64_t n, uint32_t bits, const uint8_t* gb_bits, const uint8_t* ev_bits,
                           uint32_t mask, const uint8_t key[16], const uint8_t delta_in[16], uint64_t label_nonce,
                           uint64_t gate_base, uint8_t* tables, uint8_t* gb_labels, uint8_t* ev_labels,
                           uint8_t* decode) {
    oracle_init();
    uint8_t rk[176], D[16];
    key_expand(key, rk);
    memcpy(D, delta_in, 16);
    D[0] |= 1;
    const uint64_t W = 2 * (uint64_t)bits + 1;
    uint64_t WS = 4;                                 /* label counter stride: the power of two >= W */
    while (WS < W) WS *= 2;
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < (int64_t)n; t++) {
        uint8_t L[17][16], acc[16];
        for (uint64_t w = 0; w < W; w++) {           /* zero labels: AES_key(LE128(nonce + t WS + w)) */
            uint8_t ctr[16] = {0};
            const uint64_t c = label_nonce + (uint64_t)t * WS + w;
            for (int k = 0; k < 8; k++) ctr[k] = (uint8_t)(c >> (8 * k));
            gc_aes_rk(rk, ctr, L[w]);
        }
        for (uint32_t j = 0; j < bits; j++) {        /* active input labels */
            uint8_t* g = gb_labels + ((uint64_t)t * (bits + 1) + j) * 16;
            memcpy(g, L[j], 16);
            if (gb_bits[(uint64_t)t * bits + j] & 1) gc_xor(g, g, D);
            uint8_t* e = ev_labels + ((uint64_t)t * bits + j) * 16;
            memcpy(e, L[bits + 1 + j], 16);
            if (ev_bits[(uint64_t)t * bits + j] & 1) gc_xor(e, e, D);
        }
        uint8_t* m = gb_labels + ((uint64_t)t * (bits + 1) + bits) * 16;
        memcpy(m, L[bits], 16);
        if (mask & 1) gc_xor(m, m, D);
        /* z_0 = NOT(x_0 ^ y_0): zero label X0 ^ Y0 ^ D */
        gc_xor(acc, L[0], L[bits + 1]);
        gc_xor(acc, acc, D);
        for (uint32_t k = 1; k < bits; k++) {         /* and_many: acc = AND(acc, z_k) */
            uint8_t bz[16], a1[16], b1[16], hA0[16], hA1[16], hB0[16], hB1[16], TG[16], TE[16], WG[16], WE[16];
            gc_xor(bz, L[k], L[bits + 1 + k]);
            gc_xor(bz, bz, D);
            gc_xor(a1, acc, D);
            gc_xor(b1, bz, D);
            const int pa = acc[0] & 1, pb = bz[0] & 1;
            const uint64_t j = 2 * (gate_base + (uint64_t)t * (bits - 1) + (k - 1));
            gc_tccr(acc, j, hA0);
            gc_tccr(a1, j, hA1);
            gc_tccr(bz, j + 1, hB0);
            gc_tccr(b1, j + 1, hB1);
            gc_xor(TG, hA0, hA1);                     /* T_G = H(A0) ^ H(A1) ^ pb D */
            if (pb) gc_xor(TG, TG, D);
            memcpy(WG, hA0, 16);                      /* W_G0 = H(A0) ^ pa T_G */
            if (pa) gc_xor(WG, WG, TG);
            gc_xor(TE, hB0, hB1);                     /* T_E = H(B0) ^ H(B1) ^ A0 */
            gc_xor(TE, TE, acc);
            memcpy(WE, hB0, 16);                      /* W_E0 = H(B0) ^ pb (T_E ^ A0) */
            if (pb) {
                uint8_t te_a[16];
                gc_xor(te_a, TE, acc);
                gc_xor(WE, WE, te_a);
            }
            uint8_t* tb = tables + ((uint64_t)t * (bits - 1) + (k - 1)) * 32;
            memcpy(tb, TG, 16);
            memcpy(tb + 16, TE, 16);
            gc_xor(acc, WG, WE);
        }
        decode[t] = (uint8_t)((acc[0] ^ L[bits][0]) & 1);   /* colour of out's zero label */
    }
}

void orc_gc_garble_eq(uint64_t n, uint32_t bits, const uint8_t* gb_bits, const uint8_t* ev_bits, uint32_t mask,
                      const uint8_t key[16], const uint8_t delta_in[16], uint64_t label_nonce, uint64_t gate_base,
                      uint8_t* tables, uint8_t* gb_labels, uint8_t* ev_labels, uint8_t* decode) {
    gc_garble_impl(n, bits, gb_bits, ev_bits, mask, key, delta_in, label_nonce, gate_base, tables, gb_labels,
                   ev_labels, decode);
}

/* The garbler of the r05 protocol (k_gc_garble_cot): the evaluator's zero labels ev_zero [n][bits][16]
 * come from the labels C-OT (orc_cot_extend mode 1), and the garbler's own string and mask are FOLDED
 * into the circuit instead of encoded as input wires — it knows x_j, so the input z_j = NOT(x_j ^ y_j)
 * gets the zero label Z_j = E_j ^ (x_j ? 0 : D), which makes the evaluator's OT'd label E_j ^ y_j D
 * exactly z_j's active label (XOR with a garbler-known constant is free under free-XOR), and the mask
 * goes into the decoding bit: decode = colour(out^0) ^ mask. No label is drawn (no label key) and no
 * garbler label is sent. Same circuit as bin_eq_bundles / and_many (:128-189). Layouts: tables
 * [n][bits-1][2][16], decode [n]. */
/* gb_share / share_y (r05c, both or neither): the garbler's node value and the 8-B message per test
 * (gc_share_garbler). */
void orc_gc_garble_eq_cot_share(uint64_t n, uint32_t bits, const uint8_t* gb_bits, const uint8_t* ev_zero,
                                uint32_t mask, const uint8_t delta_in[16], uint64_t gate_base, uint8_t* tables,
                                uint8_t* decode, uint64_t* gb_share, uint64_t* share_y) {
    oracle_init();
    uint8_t D[16];
    memcpy(D, delta_in, 16);
    D[0] |= 1;
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < (int64_t)n; t++) {
        uint8_t acc[16];
        for (uint32_t k = 0; k < bits; k++) {
            uint8_t bz[16];
            memcpy(bz, ev_zero + ((uint64_t)t * bits + k) * 16, 16);
            if (!(gb_bits[(uint64_t)t * bits + k] & 1)) gc_xor(bz, bz, D);   /* Z_k = E_k ^ (x_k ? 0 : D) */
            if (k == 0) {
                memcpy(acc, bz, 16);
                continue;
            }
            uint8_t a1[16], b1[16], hA0[16], hA1[16], hB0[16], hB1[16], TG[16], TE[16], WG[16], WE[16];
            gc_xor(a1, acc, D);
            gc_xor(b1, bz, D);
            const int pa = acc[0] & 1, pb = bz[0] & 1;
            const uint64_t j = 2 * (gate_base + (uint64_t)t * (bits - 1) + (k - 1));
            gc_tccr(acc, j, hA0);
            gc_tccr(a1, j, hA1);
            gc_tccr(bz, j + 1, hB0);
            gc_tccr(b1, j + 1, hB1);
            gc_xor(TG, hA0, hA1);
            if (pb) gc_xor(TG, TG, D);
            memcpy(WG, hA0, 16);
            if (pa) gc_xor(WG, WG, TG);
            gc_xor(TE, hB0, hB1);
            gc_xor(TE, TE, acc);
            memcpy(WE, hB0, 16);
            if (pb) {
                uint8_t te_a[16];
                gc_xor(te_a, TE, acc);
                gc_xor(WE, WE, te_a);
            }
            uint8_t* tb = tables + ((uint64_t)t * (bits - 1) + (k - 1)) * 32;
            memcpy(tb, TG, 16);
            memcpy(tb + 16, TE, 16);
            gc_xor(acc, WG, WE);
        }
        decode[t] = (uint8_t)((acc[0] ^ mask) & 1);   /* colour of eq's zero label, mask folded in */
        if (gb_share) gc_share_garbler(acc, D, mask, gb_share + t, share_y + t);
    }
}

void orc_gc_garble_eq_cot(uint64_t n, uint32_t bits, const uint8_t* gb_bits, const uint8_t* ev_zero, uint32_t mask,
                          const uint8_t delta_in[16], uint64_t gate_base, uint8_t* tables, uint8_t* decode) {
    orc_gc_garble_eq_cot_share(n, bits, gb_bits, ev_zero, mask, delta_in, gate_base, tables, decode, NULL, NULL);
}

/* The r05 evaluator: its OT'd labels ev_active [n][bits][16] are the inputs' active labels;
 * out[t] = colour(acc) ^ decode[t] = eq ^ mask. */
/* share_y / ev_share (r05c, both or neither): the evaluator's node value from its output label
 * (gc_share_evaluator). */
void orc_gc_eval_eq_cot_share(uint64_t n, uint32_t bits, const uint8_t* tables, const uint8_t* ev_active,
                              const uint8_t* decode, uint64_t gate_base, uint8_t* out, const uint64_t* share_y,
                              uint64_t* ev_share) {
    oracle_init();
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < (int64_t)n; t++) {
        uint8_t acc[16];
        memcpy(acc, ev_active + (uint64_t)t * bits * 16, 16);
        for (uint32_t k = 1; k < bits; k++) {
            uint8_t b[16], hA[16], hB[16];
            memcpy(b, ev_active + ((uint64_t)t * bits + k) * 16, 16);
            const int sa = acc[0] & 1, sb = b[0] & 1;
            const uint64_t j = 2 * (gate_base + (uint64_t)t * (bits - 1) + (k - 1));
            const uint8_t* tb = tables + ((uint64_t)t * (bits - 1) + (k - 1)) * 32;
            gc_tccr(acc, j, hA);
            gc_tccr(b, j + 1, hB);
            if (sa) gc_xor(hA, hA, tb);
            if (sb) {
                uint8_t te_a[16];
                gc_xor(te_a, tb + 16, acc);
                gc_xor(hB, hB, te_a);
            }
            gc_xor(acc, hA, hB);
        }
        out[t] = (uint8_t)((acc[0] & 1) ^ decode[t]);
        if (ev_share) ev_share[t] = gc_share_evaluator(acc, out[t], share_y[t]);
    }
}

void orc_gc_eval_eq_cot(uint64_t n, uint32_t bits, const uint8_t* tables, const uint8_t* ev_active,
                        const uint8_t* decode, uint64_t gate_base, uint8_t* out) {
    orc_gc_eval_eq_cot_share(n, bits, tables, ev_active, decode, gate_base, out, NULL, NULL);
}

/* r05d: the FE levels' equality test + share as ONE garbled table (Yao's garbled gate with
 * point-and-permute, generalised to the b-input gate "share of eq ^ mask") instead of the half-gates
 * chain + the output-label share. Inputs are the folded-garbler zero labels Z_k = E_k ^ (x_k ? 0 : D)
 * (E_k the labels OT's q, as orc_gc_garble_eq_cot), so the evaluator's OT'd label t_k is z_k's active
 * label and its colour p_k = lsb(t_k) = lsb(Z_k) ^ z_k names its row r = sum p_k 2^k. Row r's key is
 * H(K_r), K_r = XOR_k sigma^k(label of z_k in row r) ^ tweak, sigma = doubling in GF(2^128) (x^128 +
 * x^7 + x^2 + x + 1 on the block as a little-endian u128), tweak = gate_base + t in the low 64 bits,
 * H = cr_hash. Any other row's K differs from the evaluator's by (sum_{k in S} x^k) D for a nonempty
 * S — a nonzero field element times the unknown D — so its key is hidden as H(q ^ s) hides the
 * unchosen message in the correlated OT. eq = 1 in exactly the row r* whose z are all 1; o_r =
 * eq_r ^ mask; the values are the C-OT share pair (collect.rs:447-451): pair[0] = v, pair[1] = mask ?
 * v + 1 : v - 1, node value r1 = v + mask. Row 0 carries no message: its value pair[o_0] IS H(K_0) mod
 * p (which fixes v); rows 1 .. 2^b - 1 send m_r = lo64(H(K_r)) ^ pair[o_r] (8 B each). The evaluator:
 * value = r ? lo64(H(K)) ^ m_r : H(K) mod p. msgs [n][2^b - 1] u64, gb_share / ev_share [n]. */
static void gf128_dbl(uint8_t b[16]) {
    const int carry = b[15] >> 7;
    for (int k = 15; k > 0; k--) b[k] = (uint8_t)((b[k] << 1) | (b[k - 1] >> 7));
    b[0] = (uint8_t)(b[0] << 1);
    if (carry) b[0] ^= 0x87;
}

/* XOR_k sigma^k(L_k) ^ tweak */
static void gt_key(const uint8_t* labels /* [bits][16] */, uint32_t bits, uint64_t tweak, uint8_t K[16]) {
    uint8_t acc[16] = {0};
    for (int k = (int)bits - 1; k >= 0; k--) {   /* Horner: acc = sigma(acc) ^ L_k */
        gf128_dbl(acc);
        gc_xor(acc, acc, labels + (uint64_t)k * 16);
    }
    for (int k = 0; k < 8; k++) acc[k] ^= (uint8_t)(tweak >> (8 * k));
    memcpy(K, acc, 16);
}

static uint64_t fe_add1(uint64_t v) { return v + 1 == FE_P ? 0 : v + 1; }
static uint64_t fe_sub1(uint64_t v) { return v == 0 ? FE_P - 1 : v - 1; }

void orc_gt_garble(uint64_t n, uint32_t bits, const uint8_t* gb_bits, const uint8_t* ev_zero, uint32_t mask,
                   const uint8_t delta_in[16], uint64_t gate_base, uint64_t* msgs, uint64_t* gb_share) {
    oracle_init();
    uint8_t D[16];
    memcpy(D, delta_in, 16);
    D[0] |= 1;
    mask &= 1;
    const uint32_t R = 1u << bits;
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < (int64_t)n; t++) {
        uint8_t Z[8][16], L[8][16], K[16], H[16];
        uint32_t c = 0;
        for (uint32_t k = 0; k < bits; k++) {
            memcpy(Z[k], ev_zero + ((uint64_t)t * bits + k) * 16, 16);
            if (!(gb_bits[(uint64_t)t * bits + k] & 1)) gc_xor(Z[k], Z[k], D);   /* Z_k = E_k ^ (x_k ? 0 : D) */
            c |= (uint32_t)(Z[k][0] & 1) << k;
        }
        const uint32_t rstar = (~c) & (R - 1);   /* the row whose z are all 1 */
        uint64_t v = 0, p0 = 0, p1 = 0;
        for (uint32_t r = 0; r < R; r++) {
            for (uint32_t k = 0; k < bits; k++) {   /* label of z_k = ((r >> k) ^ c_k) & 1 */
                memcpy(L[k], Z[k], 16);
                if ((((r ^ c) >> k) & 1)) gc_xor(L[k], L[k], D);
            }
            gt_key(&L[0][0], bits, gate_base + (uint64_t)t, K);
            ot_cr_hash(K, H);
            const uint32_t o = (uint32_t)(r == rstar) ^ mask;
            if (r == 0) {
                const uint64_t h = cot_fe_of_block(H);   /* = pair[o_0] */
                v = o == 0 ? h : (mask ? fe_sub1(h) : fe_add1(h));
                p0 = v;
                p1 = mask ? fe_add1(v) : fe_sub1(v);
                gb_share[t] = mask ? fe_add1(v) : v;     /* r1 = v + mask */
            } else {
                uint64_t hl;
                memcpy(&hl, H, 8);
                msgs[(uint64_t)t * (R - 1) + (r - 1)] = hl ^ (o ? p1 : p0);
            }
        }
    }
}

void orc_gt_eval(uint64_t n, uint32_t bits, const uint8_t* ev_active, const uint64_t* msgs, uint64_t gate_base,
                 uint64_t* ev_share) {
    oracle_init();
    const uint32_t R = 1u << bits;
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < (int64_t)n; t++) {
        const uint8_t* Lt = ev_active + (uint64_t)t * bits * 16;
        uint8_t K[16], H[16];
        uint32_t r = 0;
        for (uint32_t k = 0; k < bits; k++) r |= (uint32_t)(Lt[k * 16] & 1) << k;   /* colours name the row */
        gt_key(Lt, bits, gate_base + (uint64_t)t, K);
        ot_cr_hash(K, H);
        uint64_t hl;
        memcpy(&hl, H, 8);
        ev_share[t] = r ? (hl ^ msgs[(uint64_t)t * (R - 1) + (r - 1)]) : cot_fe_of_block(H);
    }
}

/* r06: the same table with its shares in Z_2^32 (fhh_sim_config.table_ring32; GcArgs::ring32): row 0's value
 * pair[o_0] = lo32(H(K_0)), pair = (v, v +- 1 mod 2^32), rows 1 .. 2^b - 1 send m_r = lo32(H(K_r)) ^ pair[o_r]
 * (4 B), the evaluator's value = r ? lo32(H(K)) ^ m_r : lo32(H(K)). gb - ev = [eq ^ mask ... ] as the FE form,
 * mod 2^32: the per-child count v0 - v1 (< 2^32) is the same integer. msgs [n][2^b - 1] u32. */
void orc_gt_garble_ring32(uint64_t n, uint32_t bits, const uint8_t* gb_bits, const uint8_t* ev_zero, uint32_t mask,
                          const uint8_t delta_in[16], uint64_t gate_base, uint32_t* msgs, uint32_t* gb_share) {
    oracle_init();
    uint8_t D[16];
    memcpy(D, delta_in, 16);
    D[0] |= 1;
    mask &= 1;
    const uint32_t R = 1u << bits;
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < (int64_t)n; t++) {
        uint8_t Z[8][16], L[8][16], K[16], H[16];
        uint32_t c = 0;
        for (uint32_t k = 0; k < bits; k++) {
            memcpy(Z[k], ev_zero + ((uint64_t)t * bits + k) * 16, 16);
            if (!(gb_bits[(uint64_t)t * bits + k] & 1)) gc_xor(Z[k], Z[k], D);
            c |= (uint32_t)(Z[k][0] & 1) << k;
        }
        const uint32_t rstar = (~c) & (R - 1);
        uint32_t v = 0, p0 = 0, p1 = 0;
        for (uint32_t r = 0; r < R; r++) {
            for (uint32_t k = 0; k < bits; k++) {
                memcpy(L[k], Z[k], 16);
                if ((((r ^ c) >> k) & 1)) gc_xor(L[k], L[k], D);
            }
            gt_key(&L[0][0], bits, gate_base + (uint64_t)t, K);
            ot_cr_hash(K, H);
            const uint32_t o = (uint32_t)(r == rstar) ^ mask;
            uint32_t h32;
            memcpy(&h32, H, 4);
            if (r == 0) {
                v = o == 0 ? h32 : (mask ? h32 - 1u : h32 + 1u);
                p0 = v;
                p1 = mask ? v + 1u : v - 1u;
                gb_share[t] = mask ? v + 1u : v;
            } else {
                msgs[(uint64_t)t * (R - 1) + (r - 1)] = h32 ^ (o ? p1 : p0);
            }
        }
    }
}

void orc_gt_eval_ring32(uint64_t n, uint32_t bits, const uint8_t* ev_active, const uint32_t* msgs, uint64_t gate_base,
                        uint32_t* ev_share) {
    oracle_init();
    const uint32_t R = 1u << bits;
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < (int64_t)n; t++) {
        const uint8_t* Lt = ev_active + (uint64_t)t * bits * 16;
        uint8_t K[16], H[16];
        uint32_t r = 0;
        for (uint32_t k = 0; k < bits; k++) r |= (uint32_t)(Lt[k * 16] & 1) << k;
        gt_key(Lt, bits, gate_base + (uint64_t)t, K);
        ot_cr_hash(K, H);
        uint32_t h32;
        memcpy(&h32, H, 4);
        ev_share[t] = r ? (h32 ^ msgs[(uint64_t)t * (R - 1) + (r - 1)]) : h32;
    }
}

/* Evaluator (multiple_ev_equality_test, :85-105): out[t] = eq ^ mask. */
void orc_gc_eval_eq(uint64_t n, uint32_t bits, const uint8_t* tables, const uint8_t* gb_labels,
                    const uint8_t* ev_labels, const uint8_t* decode, uint64_t gate_base, uint8_t* out) {
    oracle_init();
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < (int64_t)n; t++) {
        uint8_t acc[16];
        gc_xor(acc, gb_labels + (uint64_t)t * (bits + 1) * 16, ev_labels + (uint64_t)t * bits * 16);
        for (uint32_t k = 1; k < bits; k++) {
            uint8_t b[16], hA[16], hB[16];
            gc_xor(b, gb_labels + ((uint64_t)t * (bits + 1) + k) * 16, ev_labels + ((uint64_t)t * bits + k) * 16);
            const int sa = acc[0] & 1, sb = b[0] & 1;
            const uint64_t j = 2 * (gate_base + (uint64_t)t * (bits - 1) + (k - 1));
            const uint8_t* tb = tables + ((uint64_t)t * (bits - 1) + (k - 1)) * 32;
            gc_tccr(acc, j, hA);
            gc_tccr(b, j + 1, hB);
            if (sa) gc_xor(hA, hA, tb);                /* W_G = H(A) ^ sa T_G */
            if (sb) {                                  /* W_E = H(B) ^ sb (T_E ^ A) */
                uint8_t te_a[16];
                gc_xor(te_a, tb + 16, acc);
                gc_xor(hB, hB, te_a);
            }
            gc_xor(acc, hA, hB);
        }
        const uint8_t* m = gb_labels + ((uint64_t)t * (bits + 1) + bits) * 16;
        out[t] = (uint8_t)(((acc[0] ^ m[0]) & 1) ^ decode[t]);
    }
}

/* ------------------------------------------------------------------ */
/* Row f1's OT: IKNP OT extension in the ALSZ form (u_i = G(k_i^0) ^  */
/* G(k_i^1) ^ r), as `ocelot::ot::Alsz{Sender,Receiver}` (@553ede0,   */
/* not vendored) used at equalitytest.rs:67-82 (evaluator labels) and */
/* collect.rs:437-471 (FE shares). Published scheme restated: kappa = */
/* 128 base OTs (ideal here: the sender is handed k_i^{s_i}), G =     */
/* ChaCha12 under k (r06; prg 0: AES-128-CTR, block c = LE128(c) gives */
/* OT bits 128c..+127 — ot_prg_block),                                 */
/* H(j, x) = cr_hash(j, x) = pi(x) ^ x (ot_cr_hash; tweak_base is    */
/* not an input of it). Parity: functional (out_j = x_j^{r_j}); wire  */
/* format unpinned.                                                   */
/* ------------------------------------------------------------------ */
static void ot_prg_block_aes(const uint8_t rk[176], uint64_t c, uint8_t out[16]) {
    uint8_t ctr[16] = {0};
    for (int k = 0; k < 8; k++) ctr[k] = (uint8_t)(c >> (8 * k));
    gc_aes_rk(rk, ctr, out);
}

/* ChaCha block function (RFC 8439 2.3 with the original 64-bit block counter in state words 12-13 and a
 * 64-bit nonce in 14-15; "expand 32-byte k"), `rounds` = 20 / 12 / 8: out = the 64-byte block. Pinned for
 * rounds = 20 against RFC 8439 2.3.2's vector and OpenSSL's EVP_chacha20 (tests/test_oracle_kat.py). */
static inline uint32_t cc_rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
#define CC_QR(a, b, c, d)                                                                             \
    a += b; d ^= a; d = cc_rotl(d, 16); c += d; b ^= c; b = cc_rotl(b, 12);                            \
    a += b; d ^= a; d = cc_rotl(d, 8); c += d; b ^= c; b = cc_rotl(b, 7);
void orc_chacha_block(uint32_t rounds, const uint8_t key[32], uint64_t ctr, uint64_t nonce, uint8_t out[64]) {
    uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
    for (int k = 0; k < 8; k++)
        st[4 + k] = (uint32_t)key[4 * k] | ((uint32_t)key[4 * k + 1] << 8) | ((uint32_t)key[4 * k + 2] << 16) |
                    ((uint32_t)key[4 * k + 3] << 24);
    st[12] = (uint32_t)ctr;
    st[13] = (uint32_t)(ctr >> 32);
    st[14] = (uint32_t)nonce;
    st[15] = (uint32_t)(nonce >> 32);
    uint32_t x[16];
    memcpy(x, st, sizeof x);
    for (uint32_t r = 0; r < rounds; r += 2) {
        CC_QR(x[0], x[4], x[8], x[12]) CC_QR(x[1], x[5], x[9], x[13]) CC_QR(x[2], x[6], x[10], x[14])
        CC_QR(x[3], x[7], x[11], x[15])
        CC_QR(x[0], x[5], x[10], x[15]) CC_QR(x[1], x[6], x[11], x[12]) CC_QR(x[2], x[7], x[8], x[13])
        CC_QR(x[3], x[4], x[9], x[14])
    }
    for (int k = 0; k < 16; k++) {
        const uint32_t v = x[k] + st[k];
        for (int b = 0; b < 4; b++) out[4 * k + b] = (uint8_t)(v >> (8 * b));
    }
}

/* r06: the OT extension's row PRG G is ChaCha12 (the block function above, 12 rounds — rand_chacha's
 * StdRng) keyed by the row's base-OT seed k (key = k || k, nonce 0): 128-OT block c (the row's bits
 * 128 c .. 128 c + 127) = bytes 16 (c % 4) .. 16 (c % 4) + 15 of the ChaCha block at counter c / 4 — one
 * ChaCha block = one row of a 512-OT tile of the GPU's tile-major matrices. It replaces AES-128-CTR
 * (r01-r05, ocelot's AesRng): a VALU-only PRG, no T-table lookups. prg 0 keeps the
 * AES-CTR form (the reference-form CPU baseline, bench.py cpu_protocol_baseline). */
#define OT_CHACHA_ROUNDS 12
typedef struct {   /* the last ChaCha block of one row key (the row loops walk c upwards) */
    uint64_t ctr;
    int valid;
    uint8_t blk[64];
} ot_cc_cache;
static void ot_prg_block(int prg, const uint8_t seed[16], const uint8_t rk[176], uint64_t c, uint8_t out[16],
                         ot_cc_cache* cache) {
    if (prg == 0) {
        ot_prg_block_aes(rk, c, out);
        return;
    }
    if (!cache->valid || cache->ctr != c / 4) {
        uint8_t key[32];
        memcpy(key, seed, 16);
        memcpy(key + 16, seed, 16);
        orc_chacha_block(OT_CHACHA_ROUNDS, key, c / 4, 0, cache->blk);
        cache->ctr = c / 4;
        cache->valid = 1;
    }
    memcpy(out, cache->blk + 16 * (c % 4), 16);
}

/* Correlation-robust hash of the OT extension: scuttlebutt AesHash::cr_hash(i, x) = pi(x) ^ x,
 * the index i is not an input (ocelot's ALSZ sender/receiver hash q_j, q_j ^ s, t_j with it);
 * pi = AES-128 under the all-zero key (swanky's fixed AesHash key is not restatable). */
static void ot_cr_hash(const uint8_t x[16], uint8_t out[16]) {
    uint8_t px[16];
    gc_aes0(x, px);
    for (int k = 0; k < 16; k++) out[k] = px[k] ^ x[k];
}

/* choices: m bits (bit j of byte j/8); x1 NULL -> x1 = x0 ^ delta. Optional transcript:
 * u_out [128][nblk][16] (nblk = ceil(m / 128)), y0_out / y1_out [m][16]. */
void orc_ot_extend(uint64_t m, const uint8_t* choices, const uint8_t* x0, const uint8_t* x1, const uint8_t delta[16],
                   const uint8_t seeds[128 * 2 * 16], const uint8_t s[16], uint64_t tweak_base, uint8_t* out,
                   uint8_t* u_out, uint8_t* y0_out, uint8_t* y1_out, int prg) {
    oracle_init();
    const uint64_t nblk = (m + 127) / 128;
    uint8_t* T = (uint8_t*)calloc(128 * nblk * 16, 1);
    uint8_t* Q = (uint8_t*)calloc(128 * nblk * 16, 1);
    uint8_t* U = (uint8_t*)calloc(128 * nblk * 16, 1);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < 128; i++) {
        uint8_t rk0[176], rk1[176], rks[176];
        key_expand(seeds + (i * 2 + 0) * 16, rk0);
        key_expand(seeds + (i * 2 + 1) * 16, rk1);
        const int si = (s[i / 8] >> (i % 8)) & 1;
        key_expand(seeds + (i * 2 + si) * 16, rks);   /* ideal base OT: the sender holds k_i^{s_i} */
        ot_cc_cache cc[3] = {{0, 0, {0}}, {0, 0, {0}}, {0, 0, {0}}};
        for (uint64_t c = 0; c < nblk; c++) {
            uint8_t g0[16], g1[16], gs[16];
            ot_prg_block(prg, seeds + (i * 2 + 0) * 16, rk0, c, g0, &cc[0]);
            ot_prg_block(prg, seeds + (i * 2 + 1) * 16, rk1, c, g1, &cc[1]);
            uint8_t* t = T + ((uint64_t)i * nblk + c) * 16;
            uint8_t* u = U + ((uint64_t)i * nblk + c) * 16;
            for (int k = 0; k < 16; k++) {
                uint8_t r = 0;
                for (int b = 0; b < 8; b++) {
                    const uint64_t j = c * 128 + (uint64_t)k * 8 + b;
                    if (j < m && ((choices[j / 8] >> (j % 8)) & 1)) r |= (uint8_t)(1u << b);
                }
                t[k] = g0[k];
                u[k] = g0[k] ^ g1[k] ^ r;                 /* receiver -> sender */
            }
            ot_prg_block(prg, seeds + (i * 2 + si) * 16, rks, c, gs, &cc[2]);   /* sender: q_i = G(k_i^{s_i}) ^ s_i u_i */
            uint8_t* q = Q + ((uint64_t)i * nblk + c) * 16;
            for (int k = 0; k < 16; k++) q[k] = gs[k] ^ (si ? u[k] : 0);
        }
    }
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < (int64_t)m; j++) {
        uint8_t qj[16] = {0}, tj[16] = {0}, qs[16], h0[16], h1[16], ht[16], y0[16], y1[16];
        const uint64_t c = (uint64_t)j / 128, bit = (uint64_t)j % 128;
        for (int i = 0; i < 128; i++) {                   /* column j of Q and T */
            const uint8_t* q = Q + ((uint64_t)i * nblk + c) * 16;
            const uint8_t* t = T + ((uint64_t)i * nblk + c) * 16;
            if ((q[bit / 8] >> (bit % 8)) & 1) qj[i / 8] |= (uint8_t)(1u << (i % 8));
            if ((t[bit / 8] >> (bit % 8)) & 1) tj[i / 8] |= (uint8_t)(1u << (i % 8));
        }
        for (int k = 0; k < 16; k++) qs[k] = qj[k] ^ s[k];
        ot_cr_hash(qj, h0);
        ot_cr_hash(qs, h1);
        for (int k = 0; k < 16; k++) {
            const uint8_t a = x0[j * 16 + k];
            const uint8_t b = x1 ? x1[j * 16 + k] : (uint8_t)(a ^ delta[k]);
            y0[k] = a ^ h0[k];                            /* sender -> receiver */
            y1[k] = b ^ h1[k];
        }
        if (y0_out) memcpy(y0_out + j * 16, y0, 16);
        if (y1_out) memcpy(y1_out + j * 16, y1, 16);
        const int rj = (choices[j / 8] >> (j % 8)) & 1;
        ot_cr_hash(tj, ht);
        for (int k = 0; k < 16; k++) out[j * 16 + k] = (rj ? y1[k] : y0[k]) ^ ht[k];
    }
    if (u_out) memcpy(u_out, U, 128 * nblk * 16);
    free(T);
    free(Q);
    free(U);
}

/* ------------------------------------------------------------------ */
/* r05: the protocol's two OTs as CORRELATED OT extension (ALSZ13     */
/* C-OT: the sender's first message of OT j is the hash H(q_j) itself */
/* and only y_j = f(H(q_j)) ^ H(q_j ^ s) crosses; ocelot's AlszSender */
/* offers the same as `send_correlated`). Fewer AES blocks per test   */
/* than the reference's plain OTs (collect.rs:454-471,                */
/* equalitytest.rs:67-82), same functionality:                        */
/*  mode 1  labels (XOR correlation, the evaluator's input labels):   */
/*          x0_j = H(q_j) = the evaluator's zero label, x1 = x0 ^ D;  */
/*          y_j = x0_j ^ D ^ H(q_j ^ s) (16 B);                       */
/*          receiver out_j = r_j ? y_j ^ H(t_j) : H(t_j).             */
/*  mode 2  the FE share (collect.rs:437-452): v_j = H(q_j) as a      */
/*          little-endian u128 mod p; the garbler's pair is           */
/*          (r0, r1) = mask ? (v, v + 1) : (v - 1, v) ordered         */
/*          (r0, r1) if mask else (r1, r0) — so pair[0] = v and       */
/*          pair[1] = mask ? v + 1 : v - 1; its node value r1 =       */
/*          v + mask; y_j = lo64(H(q_j ^ s)) ^ pair[1] (8 B); the     */
/*          receiver's value = r_j ? lo64(y_j ^ H(t_j)) : v.          */
/*  mode 3  the FieldElm share (collect.rs:846-876): a test is the    */
/*          OT pair (2t, 2t + 1) with the same choice; V = the        */
/*          32 big-endian bytes H(q_2t) || H(q_2t+1) mod p255, pair   */
/*          [1] = mask ? V + 1 : V - 1 as a BlockPair (field.rs:      */
/*          478-492), node value V + mask; y = H(q ^ s) ^ pair[1]     */
/*          (16 B per OT); the receiver's BlockPair = r ? y ^ H(t) :  */
/*          H(t), read unreduced as FieldElm::try_from(BlockPair)     */
/*          does (field.rs:466-476).                                  */
/*  mode 4  r05b, labels as the IKNP correlation itself (random COT   */
/*          with the global offset s): no hash and no message after   */
/*          U — sender_out_j = q_j, out_j = t_j = q_j ^ r_j s. Used   */
/*          with s as the free-XOR Delta (bit 0 of byte 0 set by the  */
/*          garbler), q_j is the zero label of input wire j and t_j   */
/*          the evaluator's active label: the correlated OT free-XOR  */
/*          garbling consumes. y_out is not written.                  */
/* H = cr_hash (ot_cr_hash). ctr_off: the row PRG G starts at block   */
/* ctr_off — the running counter of a base-OT session, so several     */
/* batches can extend one set of base OTs without repeating pads (as  */
/* ocelot's AlszSender keeps its PRG across `send` calls).            */
/* Parity: functional (the tests check the OT identities); wire       */
/* format unpinned like the rest of row f1.                           */
/* ------------------------------------------------------------------ */
static uint64_t cot_fe_of_block(const uint8_t b[16]) {
    unsigned __int128 x = 0;
    for (int k = 15; k >= 0; k--) x = (x << 8) | b[k];
    return (uint64_t)(x % (unsigned __int128)FE_P);
}

/* 32 big-endian bytes <-> 8 little-endian u32 limbs */
static void be32_to_limbs(const uint8_t* be, uint32_t v[8]) {
    for (int k = 0; k < 8; k++) {
        const uint8_t* q = be + 4 * (7 - k);
        v[k] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
    }
}
static void limbs_to_be32(const uint32_t v[8], uint8_t* be) {
    for (int k = 0; k < 8; k++) {
        uint8_t* q = be + 4 * (7 - k);
        q[0] = (uint8_t)(v[k] >> 24);
        q[1] = (uint8_t)(v[k] >> 16);
        q[2] = (uint8_t)(v[k] >> 8);
        q[3] = (uint8_t)v[k];
    }
}

/* ------------------------------------------------------------------ */
/* r06: SoftSpoken OT extension (L. Roy, "SoftSpoken OT", CRYPTO     */
/* 2022: small-field subspace VOLE with the repetition code, the      */
/* semi-honest form, no consistency check). The 128 base OTs are cut  */
/* into n_c = 128 / k chunks of k; chunk c turns its k OTs into a     */
/* (2^k - 1)-out-of-2^k OT of leaf seeds by a GGM tree, and the row   */
/* matrices come from the 2^k leaves:                                 */
/*   receiver: u_c = XOR_x G(leaf_x),  v_c[b] = XOR_{x: x_b = 1}      */
/*             G(leaf_x) (b < k);  U_c = u_c ^ r on the wire          */
/*   sender (Delta_c, every leaf but x = Delta_c):                    */
/*             w_c[b] = XOR_{x != Delta_c} (x ^ Delta_c)_b G(leaf_x)  */
/*                      ^ (Delta_c)_b U_c  =  v_c[b] ^ (Delta_c)_b r  */
/* so with t row i = v_c[b], q row i = w_c[b] for i = b n_c + c (row  */
/* order bit-major) and s bit i = (Delta_c)_b, q_j = t_j ^ r_j s: the */
/* IKNP correlation every mode below consumes, for 128 / k rows of U  */
/* (16 / k bytes per OT on the wire instead of 16). k = 1 is IKNP.    */
/* GGM (one per chunk): root = ChaCha12(k_c^0 || k_c^1, ctr c, nonce  */
/* 3)[0..15] (the receiver holds both, the sender one); node -> (left, */
/* right) = ChaCha12(node || node, ctr 0, nonce 1)[0..31]; the leaf   */
/* index x takes bit l - 1 at level l. Level l's correction of side   */
/* beta = XOR of the level's nodes with bit l - 1 = beta, masked with */
/* ChaCha12(k || k, 0, nonce 2)[0..15] of k = k_i^{1 - beta},         */
/* i = (l - 1) n_c + c: the sender (k_i^{s_i}) unmasks side 1 - s_i,  */
/* the sibling of its path, and rebuilds every leaf but Delta_c.      */
/* Rows: G(leaf) = ChaCha12 as IKNP's row PRG (key leaf || leaf,      */
/* counter ctr_off / 4 + tile, nonce 0). corr [n_c][k][2][16].        */
/* Parity: functional (q = t ^ r s; the GPU's matrices bit-exact);    */
/* the scheme is restated from the paper, no reference code.          */
/* ------------------------------------------------------------------ */
static void ss_cc16(const uint8_t a[16], const uint8_t b[16], uint64_t ctr, uint64_t nonce, uint8_t* out, size_t n) {
    uint8_t key[32], blk[64];
    memcpy(key, a, 16);
    memcpy(key + 16, b, 16);
    orc_chacha_block(OT_CHACHA_ROUNDS, key, ctr, nonce, blk);
    memcpy(out, blk, n);
}

/* chunk c's GGM: leaf_r [2^k][16] (receiver), leaf_s [2^k][16] (sender; x = Delta_c zero), corr [k][2][16] */
static void ss_ggm(uint32_t k, uint32_t c, const uint8_t seeds[128 * 2 * 16], const uint8_t s[16], uint8_t* leaf_r,
                   uint8_t* leaf_s, uint8_t* corr) {
    const uint32_t nc = 128 / k, nl = 1u << k;
    uint8_t node[16 * 16], nxt[16 * 16];
    ss_cc16(seeds + (c * 2 + 0) * 16, seeds + (c * 2 + 1) * 16, c, 3, node, 16);
    for (uint32_t l = 1; l <= k; l++) {
        const uint32_t half = 1u << (l - 1), i = (l - 1) * nc + c;
        uint8_t K[2][16] = {{0}};
        for (uint32_t z = 0; z < half; z++) {
            uint8_t lr[32];
            ss_cc16(node + 16 * z, node + 16 * z, 0, 1, lr, 32);
            memcpy(nxt + 16 * z, lr, 16);
            memcpy(nxt + 16 * (z | half), lr + 16, 16);
            for (int q = 0; q < 16; q++) {
                K[0][q] ^= lr[q];
                K[1][q] ^= lr[16 + q];
            }
        }
        for (int beta = 0; beta < 2; beta++) {
            uint8_t msk[16];
            ss_cc16(seeds + (i * 2 + (1 - beta)) * 16, seeds + (i * 2 + (1 - beta)) * 16, 0, 2, msk, 16);
            for (int q = 0; q < 16; q++) corr[((l - 1) * 2 + beta) * 16 + q] = K[beta][q] ^ msk[q];
        }
        memcpy(node, nxt, 16 * 2 * half);
    }
    memcpy(leaf_r, node, 16 * nl);
    /* the sender: path Delta_c, knows k_i^{s_i} of every level */
    uint32_t dc = 0;
    for (uint32_t b = 0; b < k; b++) dc |= (uint32_t)((s[(b * nc + c) / 8] >> ((b * nc + c) % 8)) & 1) << b;
    uint8_t kn[16 * 16];
    memset(kn, 0, sizeof kn);
    for (uint32_t l = 1; l <= k; l++) {
        const uint32_t half = 1u << (l - 1), i = (l - 1) * nc + c, db = (dc >> (l - 1)) & 1;
        const uint32_t path = dc & (half - 1);   /* the level-(l-1) node on the path (unknown) */
        uint8_t nk[16 * 16];
        memset(nk, 0, sizeof nk);
        uint8_t K[16], msk[16];
        const uint8_t* ks = seeds + (i * 2 + db) * 16;   /* k_i^{s_i} */
        ss_cc16(ks, ks, 0, 2, msk, 16);
        for (int q = 0; q < 16; q++) K[q] = corr[((l - 1) * 2 + (1 - db)) * 16 + q] ^ msk[q];
        for (uint32_t z = 0; z < half; z++) {
            if (l > 1 && z == path) continue;
            uint8_t lr[32];
            if (l == 1) continue;
            ss_cc16(kn + 16 * z, kn + 16 * z, 0, 1, lr, 32);
            memcpy(nk + 16 * z, lr, 16);
            memcpy(nk + 16 * (z | half), lr + 16, 16);
            const uint8_t* side = (1 - db) ? lr + 16 : lr;
            for (int q = 0; q < 16; q++) K[q] ^= side[q];
        }
        memcpy(nk + 16 * (path | ((1 - db) << (l - 1))), K, 16);   /* the sibling of the path */
        memcpy(kn, nk, 16 * 2 * half);
    }
    memcpy(leaf_s, kn, 16 * nl);
    memset(leaf_s + 16 * dc, 0, 16);
}

/* the row matrices T, Q [128][nblk][16] and U [128 / k][nblk][16] (row form) of m OTs; corr (k > 1)
 * [n_c][k][2][16] */
static void cot_rows(uint32_t k, uint64_t m, const uint8_t* choices, const uint8_t seeds[128 * 2 * 16],
                     const uint8_t s[16], uint64_t ctr_off, uint8_t* T, uint8_t* Q, uint8_t* U, uint8_t* corr) {
    const uint64_t nblk = (m + 127) / 128;
    if (k > 1) {
        const uint32_t nc = 128 / k, nl = 1u << k;
        const uint64_t tiles = (nblk + 3) / 4;
#pragma omp parallel for schedule(static)
        for (int c = 0; c < (int)nc; c++) {
            uint8_t leaf_r[16 * 16], leaf_s[16 * 16];
            ss_ggm(k, (uint32_t)c, seeds, s, leaf_r, leaf_s, corr + (size_t)c * k * 32);
            uint32_t dc = 0;
            for (uint32_t b = 0; b < k; b++) dc |= (uint32_t)((s[(b * nc + c) / 8] >> ((b * nc + c) % 8)) & 1) << b;
            for (uint64_t J = 0; J < tiles; J++) {
                uint8_t g[64], u[64] = {0}, v[4][64], w[4][64];
                memset(v, 0, sizeof v);
                memset(w, 0, sizeof w);
                for (uint32_t x = 0; x < nl; x++) {
                    ss_cc16(leaf_r + 16 * x, leaf_r + 16 * x, ctr_off / 4 + J, 0, g, 64);
                    for (int q = 0; q < 64; q++) u[q] ^= g[q];
                    for (uint32_t b = 0; b < k; b++)
                        if ((x >> b) & 1)
                            for (int q = 0; q < 64; q++) v[b][q] ^= g[q];
                    if (x == dc) continue;
                    ss_cc16(leaf_s + 16 * x, leaf_s + 16 * x, ctr_off / 4 + J, 0, g, 64);
                    for (uint32_t b = 0; b < k; b++)
                        if (((x ^ dc) >> b) & 1)
                            for (int q = 0; q < 64; q++) w[b][q] ^= g[q];
                }
                for (uint32_t wd = 0; wd < 4; wd++) {
                    const uint64_t cb = 4 * J + wd;
                    if (cb >= nblk) break;
                    uint8_t r[16];
                    for (int q = 0; q < 16; q++) {
                        r[q] = 0;
                        for (int bt = 0; bt < 8; bt++) {
                            const uint64_t j = cb * 128 + (uint64_t)q * 8 + bt;
                            if (j < m && ((choices[j / 8] >> (j % 8)) & 1)) r[q] |= (uint8_t)(1u << bt);
                        }
                    }
                    uint8_t* uc = U + ((uint64_t)c * nblk + cb) * 16;
                    for (int q = 0; q < 16; q++) uc[q] = u[16 * wd + q] ^ r[q];
                    for (uint32_t b = 0; b < k; b++) {
                        const uint64_t i = (uint64_t)b * nc + c;
                        uint8_t* t = T + (i * nblk + cb) * 16;
                        uint8_t* qq = Q + (i * nblk + cb) * 16;
                        for (int q = 0; q < 16; q++) {
                            t[q] = v[b][16 * wd + q];
                            qq[q] = w[b][16 * wd + q] ^ (((dc >> b) & 1) ? uc[q] : 0);
                        }
                    }
                }
            }
        }
        return;
    }
#pragma omp parallel for schedule(static)
    for (int i = 0; i < 128; i++) {
        uint8_t rk0[176], rk1[176], rks[176];
        key_expand(seeds + (i * 2 + 0) * 16, rk0);
        key_expand(seeds + (i * 2 + 1) * 16, rk1);
        const int si = (s[i / 8] >> (i % 8)) & 1;
        key_expand(seeds + (i * 2 + si) * 16, rks);
        ot_cc_cache cc[3] = {{0, 0, {0}}, {0, 0, {0}}, {0, 0, {0}}};
        for (uint64_t c = 0; c < nblk; c++) {
            uint8_t g0[16], g1[16], gs[16];
            ot_prg_block(1, seeds + (i * 2 + 0) * 16, rk0, ctr_off + c, g0, &cc[0]);
            ot_prg_block(1, seeds + (i * 2 + 1) * 16, rk1, ctr_off + c, g1, &cc[1]);
            uint8_t* t = T + ((uint64_t)i * nblk + c) * 16;
            uint8_t* u = U + ((uint64_t)i * nblk + c) * 16;
            for (int k = 0; k < 16; k++) {
                uint8_t r = 0;
                for (int b = 0; b < 8; b++) {
                    const uint64_t j = c * 128 + (uint64_t)k * 8 + b;
                    if (j < m && ((choices[j / 8] >> (j % 8)) & 1)) r |= (uint8_t)(1u << b);
                }
                t[k] = g0[k];
                u[k] = g0[k] ^ g1[k] ^ r;
            }
            ot_prg_block(1, seeds + (i * 2 + si) * 16, rks, ctr_off + c, gs, &cc[2]);
            uint8_t* q = Q + ((uint64_t)i * nblk + c) * 16;
            for (int kk = 0; kk < 16; kk++) q[kk] = gs[kk] ^ (si ? u[kk] : 0);
        }
    }
}

/* ss_k = 1: IKNP (orc_cot_extend); 2 / 4: SoftSpoken (cot_rows), u_out [128 / ss_k][nblk][16], corr_out
 * [128 / ss_k][ss_k][2][16] (ss_k > 1) */
void orc_cot_extend_ss(uint32_t ss_k, uint64_t m, uint32_t mode, const uint8_t* choices, const uint8_t delta[16],
                       uint32_t mask, const uint8_t seeds[128 * 2 * 16], const uint8_t s[16], uint64_t ctr_off,
                       uint8_t* sender_out, uint8_t* out, uint8_t* u_out, uint8_t* y_out, uint8_t* corr_out) {
    oracle_init();
    mask &= 1;
    const uint64_t nblk = (m + 127) / 128;
    uint8_t* T = (uint8_t*)calloc(128 * nblk * 16 + 16, 1);
    uint8_t* Q = (uint8_t*)calloc(128 * nblk * 16 + 16, 1);
    uint8_t* U = (uint8_t*)calloc(128 * nblk * 16 + 16, 1);
    uint8_t* H0 = (uint8_t*)calloc(m * 16 + 16, 1);   /* H(q_j) */
    uint8_t* H1 = (uint8_t*)calloc(m * 16 + 16, 1);   /* H(q_j ^ s) */
    uint8_t* HT = (uint8_t*)calloc(m * 16 + 16, 1);   /* H(t_j) */
    uint8_t corr[128 * 2 * 16];
    cot_rows(ss_k, m, choices, seeds, s, ctr_off, T, Q, U, corr);
    if (corr_out && ss_k > 1) memcpy(corr_out, corr, (size_t)128 * 2 * 16);
#pragma omp parallel for schedule(static)
    for (int64_t j = 0; j < (int64_t)m; j++) {
        uint8_t qj[16] = {0}, tj[16] = {0}, qs[16];
        const uint64_t c = (uint64_t)j / 128, bit = (uint64_t)j % 128;
        for (int i = 0; i < 128; i++) {
            const uint8_t* q = Q + ((uint64_t)i * nblk + c) * 16;
            const uint8_t* t = T + ((uint64_t)i * nblk + c) * 16;
            if ((q[bit / 8] >> (bit % 8)) & 1) qj[i / 8] |= (uint8_t)(1u << (i % 8));
            if ((t[bit / 8] >> (bit % 8)) & 1) tj[i / 8] |= (uint8_t)(1u << (i % 8));
        }
        if (mode == 4) {   /* the correlation itself, unhashed */
            if (sender_out) memcpy(sender_out + j * 16, qj, 16);
            memcpy(out + j * 16, tj, 16);
            continue;
        }
        for (int k = 0; k < 16; k++) qs[k] = qj[k] ^ s[k];
        ot_cr_hash(qj, H0 + j * 16);
        ot_cr_hash(qs, H1 + j * 16);
        ot_cr_hash(tj, HT + j * 16);
    }
    if (mode == 1) {
        for (uint64_t j = 0; j < m; j++) {
            const int rj = (choices[j / 8] >> (j % 8)) & 1;
            uint8_t y[16];
            for (int k = 0; k < 16; k++) y[k] = H0[j * 16 + k] ^ delta[k] ^ H1[j * 16 + k];
            if (sender_out) memcpy(sender_out + j * 16, H0 + j * 16, 16);
            if (y_out) memcpy(y_out + j * 16, y, 16);
            for (int k = 0; k < 16; k++) out[j * 16 + k] = (rj ? y[k] : 0) ^ HT[j * 16 + k];
        }
    } else if (mode == 2) {
        for (uint64_t j = 0; j < m; j++) {
            const int rj = (choices[j / 8] >> (j % 8)) & 1;
            const uint64_t v = cot_fe_of_block(H0 + j * 16);
            const uint64_t gv = mask ? (v + 1 == FE_P ? 0 : v + 1) : v;          /* r1 = v + mask */
            const uint64_t p1 = mask ? gv : (v == 0 ? FE_P - 1 : v - 1);         /* pair[1] */
            uint64_t h1, ht;
            memcpy(&h1, H1 + j * 16, 8);
            memcpy(&ht, HT + j * 16, 8);
            const uint64_t y = h1 ^ p1;
            if (sender_out) memcpy(sender_out + j * 8, &gv, 8);
            if (y_out) memcpy(y_out + j * 8, &y, 8);
            const uint64_t got = rj ? (y ^ ht) : cot_fe_of_block(HT + j * 16);
            memcpy(out + j * 8, &got, 8);
        }
    } else if (mode == 3) {
        for (uint64_t t = 0; 2 * t + 1 < m; t++) {
            uint32_t V[8], one[8] = {1, 0, 0, 0, 0, 0, 0, 0}, gv[8], p1[8];
            be32_to_limbs(H0 + 2 * t * 16, V);   /* H(q_2t) || H(q_2t+1): 32 big-endian bytes */
            fe255_canon(V);
            if (mask) {
                orc_fe255_add(V, one, gv);
                memcpy(p1, gv, 32);
            } else {
                memcpy(gv, V, 32);
                orc_fe255_sub(V, one, p1);
            }
            uint8_t pb[32], y[32];
            limbs_to_be32(p1, pb);
            for (int k = 0; k < 32; k++) y[k] = H1[2 * t * 16 + k] ^ pb[k];
            if (sender_out) limbs_to_be32(gv, sender_out + t * 32);
            if (y_out) memcpy(y_out + t * 32, y, 32);
            const int rj = (choices[(2 * t) / 8] >> ((2 * t) % 8)) & 1;
            for (int k = 0; k < 32; k++) out[t * 32 + k] = (rj ? y[k] : 0) ^ HT[2 * t * 16 + k];
        }
    }
    if (u_out) memcpy(u_out, U, (128 / ss_k) * nblk * 16);
    free(T);
    free(Q);
    free(U);
    free(H0);
    free(H1);
    free(HT);
}

void orc_cot_extend(uint64_t m, uint32_t mode, const uint8_t* choices, const uint8_t delta[16], uint32_t mask,
                    const uint8_t seeds[128 * 2 * 16], const uint8_t s[16], uint64_t ctr_off, uint8_t* sender_out,
                    uint8_t* out, uint8_t* u_out, uint8_t* y_out) {
    orc_cot_extend_ss(1, m, mode, choices, delta, mask, seeds, s, ctr_off, sender_out, out, u_out, y_out, NULL);
}
