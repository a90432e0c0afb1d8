// Engine state shared by the host sources — not part of the public C ABI (include/fhh.h):
//   fhh_host.cpp   one server's KeyCollection on one GPU (engine, device level loop, C ABI)
//   fhh_group.cpp  one KeyCollection over several GPUs: clients sharded in 64-client words,
//                  per-child partials reduced over an in-process RCCL communicator
//   fhh_gcot.cpp   the GC equality test + OT extension of tree_crawl and their two-party split
//                  (each server's half on its own ctx; only byte buffers cross)
#pragma once
#include "fhh_internal.h"
#include "field_arith.h"
#include "../../include/fhh.h"

#include <hip/hip_runtime.h>

#include <array>
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

struct fhh_ctx;

namespace fhh {
namespace eng {

extern thread_local std::string g_err;   // message of the last failure (fhh_host.cpp)

constexpr uint64_t kFeP = (1ull << 62) - (1ull << 30) - 1;   // fastfield.rs:24-28

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    ~DevBuf() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    // grow-only; contents are NOT preserved
    hipError_t ensure(size_t nbytes) {
        if (nbytes <= bytes && p) return hipSuccess;
        release();
        if (nbytes == 0) nbytes = 256;
        hipError_t e = hipMalloc(&p, nbytes);
        if (e != hipSuccess) {
            p = nullptr;
            return e;
        }
        bytes = nbytes;
        return hipSuccess;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

struct PinnedBuf {
    void* p = nullptr;
    size_t bytes = 0;
    ~PinnedBuf() {
        if (p) (void)hipHostFree(p);
    }
    hipError_t ensure(size_t nbytes) {
        if (nbytes <= bytes && p) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
        if (nbytes == 0) nbytes = 256;
        hipError_t e = hipHostMalloc(&p, nbytes, hipHostMallocDefault);
        if (e != hipSuccess) {
            p = nullptr;
            return e;
        }
        bytes = nbytes;
        return hipSuccess;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
};

struct DimTable {
    DevBuf seed[2], t[2], y[2];
    size_t cap[2] = {0, 0};       // entries
    int cur = 0;                  // buffer that holds the frontier's entries
    std::vector<uint32_t> live;   // frontier entries (indices into buffer `cur`), ordered
};

struct Node {
    uint32_t pos[kMaxDims];       // position of the node's dim-j entry in tab[j].live
};

enum class Phase { kNoInit, kFrontier, kPending, kPendingLast };

// 320-bit little-endian u32 helpers for FE255 (field.rs)
using Limbs10 = std::array<uint32_t, 10>;

struct Group;       // fhh_group.cpp: shards of a multi-device ctx
struct PartyState;  // fhh_party.cpp: one server's half of a level's GC + OT

}  // namespace eng
}  // namespace fhh

using namespace fhh;
using namespace fhh::eng;

struct fhh_ctx {
    int device = 0;
    hipStream_t stream = nullptr;       // execution stream (own_stream, or the peer's in pair mode)
    hipStream_t own_stream = nullptr;
    fhh_ctx* peer = nullptr;            // pair mode: ctx whose staging/timing this ctx's syncs also retire
    uint32_t L = 0, d = 0, K = 0;
    uint64_t n = 0, npad = 0, nw = 0;
    uint64_t client_base = 0;
    int variant = 0;              // k_expand variant (fhh_set_variant)
    int grid = 0;
    uint32_t loop_cap_hint = 0;   // device loop: capacity the previous crawl grew to
    DevBuf work_counter;          // dynamic item distribution
    uint32_t expand_seq = 0;      // k_expand launches on work_counter (its counter slot alternates)

    // host-staged keys (add_key); uploaded at tree_init
    std::vector<uint8_t> h_key_idx, h_root, h_cws, h_cwb;
    uint64_t h_n = 0;
    bool dev_keys = false;        // keys resident on the device (uploaded or generated)

    DevBuf cw_seed, cw_bits, root_seed, key_idx, valid;
    DimTable tab[kMaxDims];

    Phase phase = Phase::kNoInit;
    uint32_t level = 0;           // depth of the frontier (= CorWord index of next crawl)
    std::vector<Node> frontier;
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> hist;   // per depth: (parent, i)
    uint64_t pending_C = 0;
    int child_buf[kMaxDims] = {0};
    DevBuf lists;                 // per crawl: live lists of every dim + parent_pos, one upload
    const uint32_t* live_ptr[kMaxDims] = {nullptr};
    const uint32_t* parent_pos_ptr = nullptr;   // [F][d] u32 for pending children

    // frontier_last (collect.rs:33, 909-914): surviving (parent, i) + values
    std::vector<std::pair<uint32_t, uint32_t>> last_nodes;
    std::vector<Limbs10> last_values;
    uint32_t last_depth = 0;
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> last_hist;

    DevBuf scratch, scratch2;
    // level-batched sketch verification (fhh_sim_sketch_verify_fe): a second stream for the sketch
    // tails and the verify, its events, and the odd levels' sketch outputs
    hipStream_t side_stream = nullptr;
    hipEvent_t side_ev[4] = {nullptr, nullptr, nullptr, nullptr};
    DevBuf sketch_alt;
    DevBuf ot_buf[8], ot_rk;                     // OT extension scratch (T U Q - - Y0 Y1 choices)
    std::vector<uint32_t> ot_rk_host;            // key schedules staged for ot_rk
    std::vector<PinnedBuf*> stage;   // pinned staging for async H2D, recycled at every sync
    size_t stage_used = 0;

    fhh_stats stats{};
    bool timing = true;
    uint32_t timing_every = 1;   // device level loop: time every K-th k_expand launch
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
    std::vector<std::pair<size_t, uint64_t>> ev_pending;   // (pool index, blocks)
    size_t ev_next = 0;

    // multi-device ctx (fhh_create_multi): the shards hold the keys and the frontier; this ctx
    // only routes the KeyCollection calls (fhh_group.cpp)
    Group* group = nullptr;
    // this server's half of the current level's GC + OT when the two servers run on separate ctxs
    // (fhh_gb_* / fhh_ev_*, fhh_gcot.cpp)
    PartyState* party = nullptr;

    std::string err;

    int fail(int code, const std::string& msg) {
        err = msg;
        g_err = msg;
        return code;
    }
};

#define CTX_CHECK(ctx)                                              \
    do {                                                            \
        if (!(ctx)) {                                               \
            g_err = "null fhh_ctx";                                 \
            return FHH_E_ARG;                                       \
        }                                                           \
    } while (0)

#define HIP_TRY(ctx, expr)                                                                   \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess)                                                                \
            return (ctx)->fail(e_ == hipErrorOutOfMemory ? FHH_E_NOMEM : FHH_E_HIP,          \
                               std::string(#expr) + ": " + hipGetErrorString(e_));          \
    } while (0)

namespace fhh {
namespace eng {

// ---- fhh_host.cpp ----------------------------------------------------------------------------
int ctx_sync(fhh_ctx* ctx);         // drain the ctx stream, retire its timing events and staging
int ctx_set_device(fhh_ctx* ctx);   // hipSetDevice(ctx->device)
ChildArgs ctx_child_args(fhh_ctx* ctx);   // the pending crawl's children as k_share_planes reads them

// tree_crawl(_last)'s expansion; the share planes [C][2d][nw] (NULL: none) go to a host buffer
// whose rows are pitch_words u64 wide, this ctx's words starting at word_off (a shard of a
// multi-device ctx writes its 64-client words into the group's planes in place)
int crawl_level(fhh_ctx* ctx, bool last, uint64_t* n_children, uint64_t* planes, uint64_t pitch_words,
                uint64_t word_off);
// per-child 32-bit-limb partials of this ctx's OT outputs, enqueued on its stream (no sync):
// [C][2] (FE formats) or [C][8] (FE255); vals [C][ld] in format fmt, on the host (this ctx's
// clients at columns col0 .. col0 + n) or on the ctx's device (columns 0 .. n)
int node_partials(fhh_ctx* ctx, const void* vals, uint32_t fmt, uint64_t ld, uint64_t col0, bool host,
                  uint64_t** partials_dev);
// canonical FE sums [C] / unreduced [C][10] + canonical [C][8] FE255 sums from reduced partials;
// FE255 sums of a pending crawl_last become the frontier_last values (collect.rs:909-914)
int node_sums_finish(fhh_ctx* ctx, const uint64_t* partials, uint32_t fmt, void* out_a, void* out_b);
// the add_keys RPC payload's n client records (without the leading u64), decoded on the device
int add_keys_bincode_records(fhh_ctx* ctx, uint64_t n, const uint8_t* recs);
bool fmt_is_fe255(uint32_t fmt);

// ---- fhh_group.cpp (multi-device ctx) --------------------------------------------------------
void group_destroy(fhh_ctx* g);
int group_reset(fhh_ctx* g);
int group_set_client_base(fhh_ctx* g, uint64_t base);
int group_add_keys_bincode(fhh_ctx* g, const uint8_t* req, uint64_t len);
int group_gen_keys_pair(fhh_ctx* g0, fhh_ctx* g1, uint64_t n, const uint8_t* left, const uint8_t* right,
                        const uint8_t* roots);
int group_num_clients(const fhh_ctx* g, uint64_t* n);
int group_export_keys(fhh_ctx* g, uint8_t* key_idx, uint8_t* root_seed, uint8_t* cw_seed, uint8_t* cw_bits);
int group_tree_init(fhh_ctx* g);
int group_tree_crawl(fhh_ctx* g, bool last, uint64_t* n_children, uint64_t* planes);
int group_node_sums(fhh_ctx* g, const void* const* vals, bool host, uint64_t ld, uint32_t fmt, void* out_a,
                    void* out_b);
int group_tree_prune(fhh_ctx* g, const uint8_t* keep, uint64_t n, bool last);
fhh_ctx* group_lead(const fhh_ctx* g);   // first shard with clients (frontier / final shares)
int group_export_states(fhh_ctx* g, uint64_t* n_nodes, uint8_t* seeds, uint8_t* t, uint8_t* y);
int group_sim_crawl(fhh_ctx* g0, fhh_ctx* g1, const fhh_sim_config* cfg);
int group_get_stats(const fhh_ctx* g, fhh_stats* out);
int group_each(fhh_ctx* g, int (*fn)(fhh_ctx*, int), int arg);   // set_variant / set_timing / reset_stats

void party_destroy(fhh_ctx* ctx);   // fhh_gcot.cpp

// ---- fhh_gcot.cpp (row f1) -------------------------------------------------------------------
void host_key_schedule(const uint8_t key[16], uint32_t (&rk)[11][4]);
void words_from_bytes(const uint8_t b[16], uint32_t (&w)[4]);
uint64_t host_mix64(uint64_t z);
void gc_level_material(uint64_t prf_seed, uint32_t level, uint8_t key[16], uint8_t delta[16], uint32_t* mask);
void gc_chunk_material(uint64_t prf_seed, uint32_t level, uint64_t chunk, uint8_t key[16], uint8_t delta[16],
                       uint32_t* mask);
int gc_args(fhh_ctx* ctx, const fhh_gc_batch* b, GcArgs& a);
uint64_t ot_padded(uint64_t m);
void ot_level_choice(uint64_t prf, uint32_t level, uint32_t salt, uint32_t s[4]);
hipError_t ot_choices_buffer(fhh_ctx* ctx, uint64_t m, uint32_t** out);
struct OtOut {            // optional transcript (device pointers into the scratch)
    const uint4* U = nullptr;
    const uint4* Y0 = nullptr;
    const uint4* Y1 = nullptr;
    uint64_t nblk = 0;
    uint32_t u_rows = 128;            // 128 / ss_k (SoftSpoken)
    const uint4* corr = nullptr;      // SoftSpoken: the GGM corrections [u_rows][ss_k][2]
};
int ot_host_keys(fhh_ctx* ctx, const uint8_t seeds[128 * 2 * 16], const uint8_t s[16], const uint32_t** rk_dev);
// m OTs of OtArgs a's mode on ctx's stream (fhh_gcot.cpp): sizes, scratch matrices and messages are
// set here; tr (optional) receives the transcript's device pointers
int ot_run(fhh_ctx* ctx, OtArgs a, uint64_t m, OtOut* tr);
// row-PRG blocks a batch of m OTs takes from its base-OT session (a multiple of 256)
uint64_t ot_session_blocks(uint64_t m);

}  // namespace eng
}  // namespace fhh
