// Base OTs of the OT extension (row f1's OT): Chou–Orlandi "simplest OT" (CO15), host side.
//
// The reference re-initialises ocelot's AlszSender / AlszReceiver for every channel of every
// level (collect.rs:454-471, equalitytest.rs:67-82); `init` runs kappa = 128 base OTs, which in
// ocelot are Chou–Orlandi over the Ristretto group (curve25519-dalek). Neither crate is vendored,
// so the published protocol is restated here over NIST P-256 (OpenSSL's EC arithmetic — the
// image has no Ristretto implementation): the group, the point encoding and the key hash differ,
// so the wire format is parity-unpinned; the functionality (the receiver learns k_{c_i}, the
// sender k_i^0 and k_i^1, and nothing else) is what tests/test_ot.py checks.
//
//   sender:    a <- Z_q,  A = a G,  T = a A                                  -> A
//   receiver:  b_i <- Z_q,  B_i = b_i G  (c_i = 0)  or  A + b_i G  (c_i = 1) -> B_i
//              k_i = H(i, A, B_i, b_i A)
//   sender:    k_i^0 = H(i, A, B_i, a B_i),  k_i^1 = H(i, A, B_i, a B_i - T)
//
// H = SHA-256 over (i as 8-byte LE, A, B_i, P), uncompressed 65-byte points, truncated to 16
// bytes. Scalars come from SHA-256 of a caller seed (deterministic for tests and the harness;
// a deployment passes fresh OS randomness per batch).
#include "../../include/fhh.h"

#include <openssl/bn.h>
#include <openssl/ec.h>
#include <openssl/evp.h>
#include <openssl/obj_mac.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_bot_err;

int bot_fail(const char* msg) {
    g_bot_err = msg;
    return FHH_E_ARG;
}

struct Ctx {
    EC_GROUP* g = nullptr;
    BN_CTX* bn = nullptr;
    BIGNUM* q = nullptr;
    Ctx() {
        g = EC_GROUP_new_by_curve_name(NID_X9_62_prime256v1);
        bn = BN_CTX_new();
        q = BN_new();
        if (g && bn && q) EC_GROUP_get_order(g, q, bn);
    }
    ~Ctx() {
        BN_free(q);
        BN_CTX_free(bn);
        EC_GROUP_free(g);
    }
    bool ok() const { return g && bn && q; }
};

struct Pt {
    EC_POINT* p;
    explicit Pt(const EC_GROUP* g) : p(EC_POINT_new(g)) {}
    ~Pt() { EC_POINT_free(p); }
};
struct Bn {
    BIGNUM* b = BN_new();
    ~Bn() { BN_free(b); }
};

void sha256(const void* data, size_t len, uint8_t out[32]) {
    unsigned int olen = 32;
    EVP_Digest(data, len, out, &olen, EVP_sha256(), nullptr);
}

// scalar = SHA-256(tag || seed || index) mod q, never zero
bool derive_scalar(Ctx& c, const char tag, const uint8_t seed[32], uint64_t index, BIGNUM* out) {
    uint8_t buf[41], h[32];
    buf[0] = (uint8_t)tag;
    std::memcpy(buf + 1, seed, 32);
    for (int k = 0; k < 8; k++) buf[33 + k] = (uint8_t)(index >> (8 * k));
    sha256(buf, sizeof buf, h);
    if (!BN_bin2bn(h, 32, out) || !BN_nnmod(out, out, c.q, c.bn)) return false;
    if (BN_is_zero(out)) BN_one(out);
    return true;
}

bool enc(Ctx& c, const EC_POINT* p, uint8_t out[65]) {
    return EC_POINT_point2oct(c.g, p, POINT_CONVERSION_UNCOMPRESSED, out, 65, c.bn) == 65;
}

bool dec(Ctx& c, const uint8_t in[65], EC_POINT* p) { return EC_POINT_oct2point(c.g, p, in, 65, c.bn) == 1; }

void kdf(uint64_t i, const uint8_t A[65], const uint8_t B[65], const uint8_t P[65], uint8_t key[16]) {
    uint8_t buf[8 + 65 * 3], h[32];
    for (int k = 0; k < 8; k++) buf[k] = (uint8_t)(i >> (8 * k));
    std::memcpy(buf + 8, A, 65);
    std::memcpy(buf + 73, B, 65);
    std::memcpy(buf + 138, P, 65);
    sha256(buf, sizeof buf, h);
    std::memcpy(key, h, 16);
}

}  // namespace

extern "C" {

const char* fhh_base_ot_last_error(void) { return g_bot_err.c_str(); }

int fhh_co15_sender_start(const uint8_t seed[32], uint8_t A_out[65]) {
    if (!seed || !A_out) return bot_fail("co15_sender_start: NULL argument");
    Ctx c;
    if (!c.ok()) return bot_fail("co15: EC setup failed");
    Bn a;
    Pt A(c.g);
    if (!derive_scalar(c, 'a', seed, 0, a.b) || !EC_POINT_mul(c.g, A.p, a.b, nullptr, nullptr, c.bn) ||
        !enc(c, A.p, A_out))
        return bot_fail("co15_sender_start: EC failure");
    return FHH_OK;
}

int fhh_co15_receiver(uint32_t count, const uint8_t A_in[65], const uint8_t* choices, const uint8_t seed[32],
                      uint8_t* B_out, uint8_t* keys) {
    if (!A_in || (count && (!choices || !seed || !B_out || !keys))) return bot_fail("co15_receiver: NULL argument");
    Ctx c;
    if (!c.ok()) return bot_fail("co15: EC setup failed");
    Pt A(c.g), B(c.g), P(c.g);
    Bn b;
    if (!dec(c, A_in, A.p)) return bot_fail("co15_receiver: A is not a P-256 point");
    for (uint32_t i = 0; i < count; i++) {
        const int ci = (choices[i / 8] >> (i % 8)) & 1;
        uint8_t Pe[65];
        if (!derive_scalar(c, 'b', seed, i, b.b) || !EC_POINT_mul(c.g, B.p, b.b, nullptr, nullptr, c.bn) ||
            (ci && !EC_POINT_add(c.g, B.p, B.p, A.p, c.bn)) || !enc(c, B.p, B_out + 65 * (size_t)i) ||
            !EC_POINT_mul(c.g, P.p, nullptr, A.p, b.b, c.bn) || !enc(c, P.p, Pe))
            return bot_fail("co15_receiver: EC failure");
        kdf(i, A_in, B_out + 65 * (size_t)i, Pe, keys + 16 * (size_t)i);
    }
    return FHH_OK;
}

int fhh_co15_sender_finish(uint32_t count, const uint8_t seed[32], const uint8_t* B_in, uint8_t* keys) {
    if (!seed || (count && (!B_in || !keys))) return bot_fail("co15_sender_finish: NULL argument");
    Ctx c;
    if (!c.ok()) return bot_fail("co15: EC setup failed");
    Bn a;
    Pt A(c.g), T(c.g), B(c.g), P(c.g);
    uint8_t Ae[65];
    if (!derive_scalar(c, 'a', seed, 0, a.b) || !EC_POINT_mul(c.g, A.p, a.b, nullptr, nullptr, c.bn) ||
        !EC_POINT_mul(c.g, T.p, nullptr, A.p, a.b, c.bn) || !enc(c, A.p, Ae))
        return bot_fail("co15_sender_finish: EC failure");
    if (!EC_POINT_invert(c.g, T.p, c.bn)) return bot_fail("co15_sender_finish: EC failure");
    for (uint32_t i = 0; i < count; i++) {
        uint8_t P0[65], P1[65];
        if (!dec(c, B_in + 65 * (size_t)i, B.p)) return bot_fail("co15_sender_finish: B_i is not a P-256 point");
        if (!EC_POINT_mul(c.g, P.p, nullptr, B.p, a.b, c.bn) || !enc(c, P.p, P0) ||
            !EC_POINT_add(c.g, P.p, P.p, T.p, c.bn) || !enc(c, P.p, P1))
            return bot_fail("co15_sender_finish: EC failure");
        kdf(i, Ae, B_in + 65 * (size_t)i, P0, keys + 32 * (size_t)i);
        kdf(i, Ae, B_in + 65 * (size_t)i, P1, keys + 32 * (size_t)i + 16);
    }
    return FHH_OK;
}

int fhh_base_ot_co15(uint32_t count, const uint8_t* choices, const uint8_t seed[32], uint8_t* sender_keys,
                     uint8_t* receiver_keys) {
    if (!seed || (count && (!choices || !sender_keys || !receiver_keys))) return bot_fail("base_ot_co15: NULL argument");
    uint8_t sa[32], sb[32], A[65];
    uint8_t t[33];
    std::memcpy(t + 1, seed, 32);
    t[0] = 'S';
    sha256(t, sizeof t, sa);
    t[0] = 'R';
    sha256(t, sizeof t, sb);
    std::vector<uint8_t> B((size_t)count * 65);
    int rc = fhh_co15_sender_start(sa, A);
    if (rc) return rc;
    rc = fhh_co15_receiver(count, A, choices, sb, B.data(), receiver_keys);
    if (rc) return rc;
    return fhh_co15_sender_finish(count, sa, B.data(), sender_keys);
}

}  // extern "C"

namespace fhh {

// Per-instance worker of BaseOtProducer: 128 base OTs of OT extension k (seed SHA-256(seed || k),
// the OT-extension sender's choice bits choices[16]) -> pairs [128][2][16] (the OT-extension
// receiver's seed pairs) and chosen [128][16] (the sender's k_i^{s_i}).
int base_ot_instance(uint64_t k, const uint8_t seed[32], const uint8_t choices[16], uint8_t* pairs, uint8_t* chosen,
                     std::string* err) {
    uint8_t s[40], sk[32];
    std::memcpy(s, seed, 32);
    for (int b = 0; b < 8; b++) s[32 + b] = (uint8_t)(k >> (8 * b));
    sha256(s, sizeof s, sk);
    const int rc = fhh_base_ot_co15(128, choices, sk, pairs, chosen);
    if (rc && err) *err = fhh_base_ot_last_error();
    return rc;
}

}  // namespace fhh
