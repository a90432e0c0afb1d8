// Host engine of the MI355X evaluator: one fhh_ctx = one server's
// `KeyCollection<FE, FieldElm>` (src/collect.rs:28-1030) bound to one GPU, exposed through
// the C ABI declared in include/fhh.h.
//
// The frontier of the reference is a Vec<TreeNode> whose nodes carry every client's d
// (left, right) EvalStates (collect.rs:18-22). Here a node is a tuple of d indices into
// per-dim prefix tables that live on the GPU (fhh_internal.h); pruning edits index lists
// on the host and never moves state (the reference does O(F) Vec::remove of whole nodes,
// collect.rs:918-929).
#include "fhh_engine.h"

#ifndef FHH_GT_FUSED_SUMS
#define FHH_GT_FUSED_SUMS 1   // r06: the tile-major table kernels add the node values per child themselves
#endif
#include "aes_tables.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

thread_local std::string fhh::eng::g_err;

namespace {

constexpr int kDefaultVariant = 52;  // 4 tables, 128 KiB, 1024 thr, dynamic items (first one static, multi-word on narrow levels), <= 16 entries per item, nontemporal parent-seed loads and child-seed stores, sibling-pair AES (r02b A/Bs vs 34, 51)


// ---- timing -------------------------------------------------------------------------------
hipError_t timing_begin(fhh_ctx* ctx, size_t* slot) {
    if (ctx->ev_next >= ctx->ev_pool.size()) {
        hipEvent_t a, b;
        hipError_t e = hipEventCreate(&a);
        if (e != hipSuccess) return e;
        e = hipEventCreate(&b);
        if (e != hipSuccess) return e;
        ctx->ev_pool.emplace_back(a, b);
    }
    *slot = ctx->ev_next++;
    return hipEventRecord(ctx->ev_pool[*slot].first, ctx->stream);
}

hipError_t timing_end(fhh_ctx* ctx, size_t slot, uint64_t blocks) {
    ctx->ev_pending.emplace_back(slot, blocks);
    return hipEventRecord(ctx->ev_pool[slot].second, ctx->stream);
}

// `blocks` tags of the event pairs that bracket the level loop's cross-rank all-reduce and its
// GC + OT step (share planes to the last chunk's sums)
constexpr uint64_t kAllreduceTag = ~0ull;
constexpr uint64_t kGcotTag = ~1ull;

// call after the stream is synchronised
void timing_resolve(fhh_ctx* ctx) {
    for (auto& pr : ctx->ev_pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, ctx->ev_pool[pr.first].first, ctx->ev_pool[pr.first].second) != hipSuccess)
            continue;
        if (pr.second == kAllreduceTag) {
            ctx->stats.allreduce_ms += ms;
            ctx->stats.allreduce_timed++;
        } else if (pr.second == kGcotTag) {
            ctx->stats.gcot_ms += ms;
            ctx->stats.gcot_timed++;
        } else {
            ctx->stats.expand_ms += ms;
            ctx->stats.expand_blocks_timed += pr.second;
            ctx->stats.expand_launches_timed++;
        }
    }
    ctx->ev_pending.clear();
    ctx->ev_next = 0;
}

int sync(fhh_ctx* ctx) {
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    timing_resolve(ctx);
    ctx->stage_used = 0;
    if (ctx->peer) {
        timing_resolve(ctx->peer);
        ctx->peer->stage_used = 0;
    }
    return FHH_OK;
}

// Pair mode (in-process two-server harness): c1 runs on c0's stream, so one stream carries
// both servers' work in order and the level loop needs a single host sync.
struct PairScope {
    fhh_ctx *c0, *c1;
    PairScope(fhh_ctx* a, fhh_ctx* b) : c0(a), c1(b) {
        c1->stream = c0->stream;
        c0->peer = c1;
    }
    ~PairScope() {
        (void)hipStreamSynchronize(c0->stream);
        c1->stream = c1->own_stream;
        c0->peer = nullptr;
    }
};

// pinned host staging that stays valid until the next sync(ctx)
void* stage_bytes(fhh_ctx* ctx, size_t bytes) {
    if (ctx->stage_used >= ctx->stage.size()) ctx->stage.push_back(new PinnedBuf());
    PinnedBuf* b = ctx->stage[ctx->stage_used];
    if (b->ensure(bytes) != hipSuccess) return nullptr;
    ctx->stage_used++;
    return b->p;
}

// ---- FE / FE255 host arithmetic --------------------------------------------------------------
uint64_t fe_canon_from_limbs(uint64_t lo, uint64_t hi) { return fhh::fe_canon_from_limbs(lo, hi); }

uint64_t fe_canon(uint64_t v) { return v % kFeP; }

// carry-propagate 8 u64 limb sums (limb k weight 2^(32k)) into 10 u32 limbs
Limbs10 limbs_from_partials(const uint64_t* p8) {
    Limbs10 out{};
    fhh::limbs10_from_partials(p8, out.data());
    return out;
}

std::array<uint32_t, 8> fe255_reduce(const Limbs10& x) {
    std::array<uint32_t, 8> out{};
    fhh::fe255_reduce(x.data(), out.data());
    return out;
}

std::array<uint32_t, 8> fe255_sub(const std::array<uint32_t, 8>& a, const std::array<uint32_t, 8>& b) {
    std::array<uint32_t, 8> out{};
    fhh::fe255_sub(a.data(), b.data(), out.data());
    return out;
}

bool fe255_ge_u32(const std::array<uint32_t, 8>& v, uint32_t t) { return fhh::fe255_ge_u32(v.data(), t); }

// ---- device key / table management -----------------------------------------------------------
int alloc_keys(fhh_ctx* ctx, uint64_t n) {
    ctx->n = n;
    ctx->nw = (n + 63) / 64;
    if (ctx->nw == 0) ctx->nw = 1;
    ctx->npad = ctx->nw * 64;
    const size_t K = ctx->K, L = ctx->L;
    HIP_TRY(ctx, ctx->cw_seed.ensure(L * K * ctx->npad * 16));
    HIP_TRY(ctx, ctx->cw_bits.ensure(L * K * 4 * ctx->nw * 8));
    HIP_TRY(ctx, ctx->root_seed.ensure(K * ctx->npad * 16));
    HIP_TRY(ctx, ctx->key_idx.ensure(K * ctx->nw * 8));
    HIP_TRY(ctx, ctx->valid.ensure(ctx->nw * 8));
    std::vector<uint64_t> v(ctx->nw, ~0ull);
    if (n % 64) v[ctx->nw - 1] = (1ull << (n % 64)) - 1;
    if (n == 0) v[0] = 0;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->valid.p, v.data(), ctx->nw * 8, hipMemcpyHostToDevice, ctx->stream));
    return sync(ctx);
}

int upload_staged_keys(fhh_ctx* ctx) {
    if (ctx->h_n == 0) return FHH_OK;
    if (ctx->dev_keys) return ctx->fail(FHH_E_STATE, "cannot mix add_keys with device-generated keys");
    int rc = alloc_keys(ctx, ctx->h_n);
    if (rc) return rc;
    const size_t K = ctx->K, L = ctx->L, n = ctx->h_n;
    DevBuf a, b, c, dd;
    HIP_TRY(ctx, a.ensure(n * K));
    HIP_TRY(ctx, b.ensure(n * K * 16));
    HIP_TRY(ctx, c.ensure(n * K * L * 16));
    HIP_TRY(ctx, dd.ensure(n * K * L));
    HIP_TRY(ctx, hipMemcpyAsync(a.p, ctx->h_key_idx.data(), n * K, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(b.p, ctx->h_root.data(), n * K * 16, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(c.p, ctx->h_cws.data(), n * K * L * 16, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(dd.p, ctx->h_cwb.data(), n * K * L, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, launch_keys_from_aos(a.as<uint8_t>(), b.as<uint8_t>(), c.as<uint8_t>(), dd.as<uint8_t>(), n,
                                      ctx->K, ctx->L, (uint32_t)ctx->npad, (uint32_t)ctx->nw, ctx->cw_seed.as<uint4>(),
                                      ctx->cw_bits.as<uint64_t>(), ctx->root_seed.as<uint4>(),
                                      ctx->key_idx.as<uint64_t>(), ctx->stream));
    rc = sync(ctx);
    if (rc) return rc;
    ctx->dev_keys = true;
    ctx->h_key_idx.clear();
    ctx->h_root.clear();
    ctx->h_cws.clear();
    ctx->h_cwb.clear();
    ctx->h_key_idx.shrink_to_fit();
    ctx->h_root.shrink_to_fit();
    ctx->h_cws.shrink_to_fit();
    ctx->h_cwb.shrink_to_fit();
    ctx->h_n = 0;
    return FHH_OK;
}

int table_ensure(fhh_ctx* ctx, DimTable& T, int buf, size_t entries) {
    if (entries <= T.cap[buf] && T.seed[buf].p) return FHH_OK;
    size_t cap = std::max<size_t>(entries, T.cap[buf] * 2);
    cap = std::max<size_t>(cap, 4);
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (T.seed[buf].ensure(cap * 2 * ctx->npad * 16) != hipSuccess) {
        // the doubling does not fit (32 MB per entry at 1M clients): exactly what is needed
        (void)hipGetLastError();
        cap = std::max<size_t>(entries, 4);
        HIP_TRY(ctx, T.seed[buf].ensure(cap * 2 * ctx->npad * 16));
    }
    HIP_TRY(ctx, T.t[buf].ensure(cap * 2 * ctx->nw * 8));
    HIP_TRY(ctx, T.y[buf].ensure(cap * 2 * ctx->nw * 8));
    T.cap[buf] = cap;
    return FHH_OK;
}

int upload_u32(fhh_ctx* ctx, DevBuf& dst, const std::vector<uint32_t>& v) {
    const size_t bytes = std::max<size_t>(v.size() * 4, 4);
    if (dst.bytes < bytes) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        HIP_TRY(ctx, dst.ensure(bytes * 2));
    }
    if (!v.empty()) {
        void* h = stage_bytes(ctx, v.size() * 4);
        if (!h) return ctx->fail(FHH_E_NOMEM, "pinned staging allocation failed");
        std::memcpy(h, v.data(), v.size() * 4);
        HIP_TRY(ctx, hipMemcpyAsync(dst.p, h, v.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    }
    return FHH_OK;
}

// One H2D copy per crawl: [live_0 | ... | live_{d-1} | parent_pos[F][d]] (u32).
int upload_lists(fhh_ctx* ctx) {
    std::vector<uint32_t> v;
    size_t off[kMaxDims + 1];
    for (uint32_t j = 0; j < ctx->d; j++) {
        off[j] = v.size();
        v.insert(v.end(), ctx->tab[j].live.begin(), ctx->tab[j].live.end());
    }
    off[ctx->d] = v.size();
    for (const Node& nd : ctx->frontier)
        for (uint32_t j = 0; j < ctx->d; j++) v.push_back(nd.pos[j]);
    int rc = upload_u32(ctx, ctx->lists, v);
    if (rc) return rc;
    const uint32_t* base = ctx->lists.as<uint32_t>();
    for (uint32_t j = 0; j < ctx->d; j++) ctx->live_ptr[j] = base + off[j];
    ctx->parent_pos_ptr = base + off[ctx->d];
    return FHH_OK;
}

// Prepare expansion jobs for one ctx (dst buffers sized; lists already on the device).
int prepare_expand(fhh_ctx* ctx, ExpandJob* jobs, uint32_t* njobs) {
    for (uint32_t j = 0; j < ctx->d; j++) {
        DimTable& T = ctx->tab[j];
        const int src = T.cur, dst = 1 - T.cur;
        int rc = table_ensure(ctx, T, dst, 2 * T.live.size());
        if (rc) return rc;
        ExpandJob& J = jobs[(*njobs)++];
        J.cw_seed = ctx->cw_seed.as<uint4>();
        J.cw_bits = ctx->cw_bits.as<uint64_t>();
        J.src_seed = T.seed[src].as<uint4>();
        J.src_t = T.t[src].as<uint64_t>();
        J.src_y = T.y[src].as<uint64_t>();
        J.dst_seed = T.seed[dst].as<uint4>();
        J.dst_t = T.t[dst].as<uint64_t>();
        J.dst_y = T.y[dst].as<uint64_t>();
        J.live = ctx->live_ptr[j];
        J.n_live = (uint32_t)T.live.size();
        J.level = ctx->level;
        J.dim = j;
        J.K = ctx->K;
        J.npad = (uint32_t)ctx->npad;
        J.nw = (uint32_t)ctx->nw;
        J.group = 1;
        J.wpi = 1;
        J.item_begin = 0;
        J.split = J.n_live;
        J.group_b = 1;
        J.e_base = 0;
        J.pad2_ = 0;
        J.item_begin_b = 0;
    }
    return FHH_OK;
}

void finalize_launch(ExpandLaunch& L, int grid, int variant) {
    // every job of a launch has the same client count (both servers hold the same clients)
    const uint64_t waves = (uint64_t)grid * (expand_threads(variant) / 64);
    uint32_t n_live[kMaxJobs] = {};
    for (uint32_t k = 0; k < L.njobs; k++) n_live[k] = L.job[k].n_live;
    ItemLayout lay;
    item_layout(n_live, L.njobs, L.job[0].nw, expand_max_group(variant), waves,
                expand_tail_split(variant), lay, expand_max_wpi(variant));
    L.wpi = lay.wpi;
    for (uint32_t k = 0; k < L.njobs; k++) {
        ExpandJob& J = L.job[k];
        J.wpi = lay.wpi;
        J.group = lay.g;
        J.group_b = lay.g_b;
        J.split = lay.split[k];
        J.item_begin = lay.begin_a[k];
        J.item_begin_b = lay.begin_b[k];
    }
    L.items_a = lay.items_a;
    L.total_items = lay.total;
}

uint64_t launch_blocks(const fhh_ctx* ctx) {
    uint64_t b = 0;
    for (uint32_t j = 0; j < ctx->d; j++) b += (uint64_t)ctx->tab[j].live.size() * 4 * ctx->n;
    return b;
}

// Record the children created by an expansion of ctx's frontier.
int post_expand(fhh_ctx* ctx, bool last) {
    const uint64_t F = ctx->frontier.size();
    ctx->pending_C = F << ctx->d;
    for (uint32_t j = 0; j < ctx->d; j++) {
        DimTable& T = ctx->tab[j];
        ctx->child_buf[j] = 1 - T.cur;
        if (!last) T.cur = 1 - T.cur;     // tree_crawl: next_frontier replaces frontier
    }
    ctx->stats.aes_blocks += launch_blocks(ctx);
    ctx->stats.ref_evals += ctx->pending_C * ctx->n * 2 * ctx->d;
    ctx->stats.levels += 1;
    if (last) {
        ctx->phase = Phase::kPendingLast;
        ctx->last_nodes.clear();
        for (uint64_t c = 0; c < ctx->pending_C; c++)
            ctx->last_nodes.emplace_back((uint32_t)(c >> ctx->d), (uint32_t)(c & ((1u << ctx->d) - 1)));
        ctx->last_values.assign(ctx->pending_C, Limbs10{});
        ctx->last_depth = ctx->level + 1;
        ctx->last_hist = ctx->hist;
    } else {
        ctx->phase = Phase::kPending;
    }
    return FHH_OK;
}

int prune_impl(fhh_ctx* ctx, const uint8_t* keep, uint64_t n);

int check_can_crawl(fhh_ctx* ctx) {
    if (ctx->phase == Phase::kNoInit) return ctx->fail(FHH_E_STATE, "tree_crawl before tree_init");
    if (ctx->phase == Phase::kPending) {
        // the unpruned children become the frontier (collect.rs:505 `self.frontier = next_frontier`)
        std::vector<uint8_t> all(ctx->pending_C, 1);
        int rc = prune_impl(ctx, all.data(), ctx->pending_C);
        if (rc) return rc;
    }
    if (ctx->level >= ctx->L) return ctx->fail(FHH_E_STATE, "crawl past data_len (cor_words index out of bounds)");
    return FHH_OK;
}

int crawl_one(fhh_ctx* ctx, bool last) {
    int rc = check_can_crawl(ctx);
    if (rc) return rc;
    rc = upload_lists(ctx);
    if (rc) return rc;
    ExpandLaunch La{};
    La.njobs = 0;
    rc = prepare_expand(ctx, La.job, &La.njobs);
    if (rc) return rc;
    finalize_launch(La, ctx->grid, ctx->variant);
    size_t slot = 0;
    if (ctx->timing) HIP_TRY(ctx, timing_begin(ctx, &slot));
    HIP_TRY(ctx, launch_expand(La, ctx->variant, ctx->grid, ctx->work_counter.as<uint32_t>(), &ctx->expand_seq, ctx->stream));
    if (ctx->timing) HIP_TRY(ctx, timing_end(ctx, slot, launch_blocks(ctx)));
    ctx->stats.expand_launches++;
    return post_expand(ctx, last);
}

// Both servers' expansions in ONE launch (same device): the in-process harness path.
int crawl_pair(fhh_ctx* c0, fhh_ctx* c1, bool last) {
    int rc = check_can_crawl(c0);
    if (rc) return rc;
    rc = check_can_crawl(c1);
    if (rc) return rc;
    if (c1->stream != c0->stream) HIP_TRY(c1, hipStreamSynchronize(c1->stream));
    // both servers prune with the same keep masks, so their frontiers and live lists are
    // identical: upload once and let server 1's jobs read server 0's copy
    if (c0->frontier.size() != c1->frontier.size()) return c0->fail(FHH_E_ARG, "pair: frontiers differ");
    for (uint32_t j = 0; j < c0->d; j++)
        if (c0->tab[j].live != c1->tab[j].live) return c0->fail(FHH_E_ARG, "pair: live lists differ");
    rc = upload_lists(c0);
    if (rc) return rc;
    for (uint32_t j = 0; j < c0->d; j++) c1->live_ptr[j] = c0->live_ptr[j];
    c1->parent_pos_ptr = c0->parent_pos_ptr;
    ExpandLaunch La{};
    La.njobs = 0;
    rc = prepare_expand(c0, La.job, &La.njobs);
    if (rc) return rc;
    rc = prepare_expand(c1, La.job, &La.njobs);
    if (rc) return rc;
    finalize_launch(La, c0->grid, c0->variant);
    size_t slot = 0;
    const uint64_t blocks = launch_blocks(c0) + launch_blocks(c1);
    if (c0->timing) HIP_TRY(c0, timing_begin(c0, &slot));
    HIP_TRY(c0, launch_expand(La, c0->variant, c0->grid, c0->work_counter.as<uint32_t>(), &c0->expand_seq, c0->stream));
    if (c0->timing) HIP_TRY(c0, timing_end(c0, slot, blocks));
    c0->stats.expand_launches++;
    rc = post_expand(c0, last);
    if (rc) return rc;
    return post_expand(c1, last);
}

ChildArgs child_args(fhh_ctx* c0, fhh_ctx* c1) {
    ChildArgs a{};
    for (uint32_t j = 0; j < c0->d; j++) {
        a.s0.t[j] = c0->tab[j].t[c0->child_buf[j]].as<uint64_t>();
        a.s0.y[j] = c0->tab[j].y[c0->child_buf[j]].as<uint64_t>();
        fhh_ctx* o = c1 ? c1 : c0;
        a.s1.t[j] = o->tab[j].t[o->child_buf[j]].as<uint64_t>();
        a.s1.y[j] = o->tab[j].y[o->child_buf[j]].as<uint64_t>();
    }
    a.parent_pos = c0->parent_pos_ptr;
    a.valid = c0->valid.as<uint64_t>();
    a.C = c0->pending_C;
    a.d = c0->d;
    a.nw = (uint32_t)c0->nw;
    a.client_base = c0->client_base;
    a.level = c0->level;
    a.n = (uint32_t)c0->n;
    return a;
}

int prune_impl(fhh_ctx* ctx, const uint8_t* keep, uint64_t n) {
    if (ctx->phase != Phase::kPending) return ctx->fail(FHH_E_STATE, "tree_prune without a pending tree_crawl");
    if (n != ctx->pending_C)
        return ctx->fail(FHH_E_ARG, "tree_prune: keep.len() != frontier.len() (collect.rs:919)");
    const uint32_t d = ctx->d;
    std::vector<Node> nf;
    std::vector<std::pair<uint32_t, uint32_t>> h;
    std::vector<std::vector<uint32_t>> new_live(d);
    // child entry e of dim j lies in [0, 2 * |live_j|): flat remap, first reference wins
    thread_local std::vector<int32_t> remap[kMaxDims];
    for (uint32_t j = 0; j < d; j++) remap[j].assign(2 * ctx->tab[j].live.size(), -1);
    nf.reserve(n);
    h.reserve(n);
    for (uint64_t c = 0; c < n; c++) {
        if (!keep[c]) continue;
        const uint32_t p = (uint32_t)(c >> d), i = (uint32_t)(c & ((1u << d) - 1));
        Node node{};
        for (uint32_t j = 0; j < d; j++) {
            const uint32_t e = 2 * ctx->frontier[p].pos[j] + ((i >> j) & 1);
            int32_t& r = remap[j][e];
            if (r < 0) {
                r = (int32_t)new_live[j].size();
                new_live[j].push_back(e);
            }
            node.pos[j] = (uint32_t)r;
        }
        nf.push_back(node);
        h.emplace_back(p, i);
    }
    for (uint32_t j = 0; j < d; j++) ctx->tab[j].live = std::move(new_live[j]);
    ctx->frontier = std::move(nf);
    ctx->hist.push_back(std::move(h));
    ctx->level += 1;
    ctx->pending_C = 0;
    ctx->phase = Phase::kFrontier;
    return FHH_OK;
}

// path of a frontier node at depth `depth` (hist[0..depth-1]) followed by (p, i)
void node_path(const std::vector<std::vector<std::pair<uint32_t, uint32_t>>>& hist, uint32_t depth, uint32_t p,
               uint32_t i, uint32_t d, uint8_t* out /*[d][depth+1]*/) {
    const uint32_t len = depth + 1;
    for (uint32_t j = 0; j < d; j++) out[j * len + depth] = (uint8_t)((i >> j) & 1);
    uint32_t node = p;
    for (int64_t lv = (int64_t)depth - 1; lv >= 0; lv--) {
        const auto& pr = hist[(size_t)lv][node];
        for (uint32_t j = 0; j < d; j++) out[j * len + (uint32_t)lv] = (uint8_t)((pr.second >> j) & 1);
        node = pr.first;
    }
}

int check_pair(fhh_ctx* c0, fhh_ctx* c1) {
    if (!c0 || !c1) {
        g_err = "null fhh_ctx";
        return FHH_E_ARG;
    }
    if (c0->device != c1->device) return c0->fail(FHH_E_ARG, "sim: ctxs on different devices");
    if (c0->d != c1->d || c0->n != c1->n || c0->L != c1->L)
        return c0->fail(FHH_E_ARG, "sim: ctx shapes differ");
    if (c0->phase != c1->phase || (c0->phase != Phase::kPending && c0->phase != Phase::kPendingLast))
        return c0->fail(FHH_E_STATE, "sim: both ctxs need a pending crawl");
    if (c0->pending_C != c1->pending_C || c0->frontier.size() != c1->frontier.size())
        return c0->fail(FHH_E_ARG, "sim: frontiers differ");
    for (size_t k = 0; k < c0->frontier.size(); k++)
        for (uint32_t j = 0; j < c0->d; j++)
            if (c0->frontier[k].pos[j] != c1->frontier[k].pos[j]) return c0->fail(FHH_E_ARG, "sim: frontiers differ");
    if (c1->stream != c0->stream) HIP_TRY(c1, hipStreamSynchronize(c1->stream));
    return FHH_OK;
}

// partials on device -> (optional all-reduce) -> host
int fetch_partials(fhh_ctx* ctx, const fhh_sim_config* cfg, uint64_t* dev, uint64_t count, uint64_t* host) {
    if (count == 0) return FHH_OK;
    if (cfg && cfg->comm) {
        std::string err;
        if (comm_allreduce(cfg->comm, dev, dev, count, ctx->stream, &err)) return ctx->fail(FHH_E_COMM, err);
        HIP_TRY(ctx, hipMemcpyAsync(host, dev, count * 8, hipMemcpyDeviceToHost, ctx->stream));
    } else if (cfg && cfg->allreduce) {
        if (!cfg->xchg_dev || cfg->xchg_capacity < count)
            return ctx->fail(FHH_E_ARG, "sim: all-reduce exchange buffer too small");
        HIP_TRY(ctx, hipMemcpyAsync(cfg->xchg_dev, dev, count * 8, hipMemcpyDeviceToDevice, ctx->stream));
        int rc = sync(ctx);
        if (rc) return rc;
        if (cfg->allreduce(cfg->xchg_dev, count, cfg->allreduce_user) != 0)
            return ctx->fail(FHH_E_CALLBACK, "all-reduce callback failed");
        HIP_TRY(ctx, hipMemcpyAsync(host, cfg->xchg_dev, count * 8, hipMemcpyDeviceToHost, ctx->stream));
    } else {
        HIP_TRY(ctx, hipMemcpyAsync(host, dev, count * 8, hipMemcpyDeviceToHost, ctx->stream));
    }
    return sync(ctx);
}

int sim_eq_count_impl(fhh_ctx* c0, fhh_ctx* c1, const fhh_sim_config* cfg, uint64_t* counts) {
    int rc = check_pair(c0, c1);
    if (rc) return rc;
    const uint64_t C = c0->pending_C;
    HIP_TRY(c0, c0->scratch2.ensure(std::max<uint64_t>(C, 1) * 8 * 16));
    ChildArgs a = child_args(c0, c1);
    HIP_TRY(c0, launch_eq_count(a, c0->scratch2.as<uint64_t>(), c0->stream));
    return fetch_partials(c0, cfg, c0->scratch2.as<uint64_t>(), C, counts);
}

// mode FE (non-last): sums0/sums1 [C] canonical; FE255 (last): [C][10] unreduced
int sim_ot_sums_impl(fhh_ctx* c0, fhh_ctx* c1, const fhh_sim_config* cfg, uint64_t seed, void* s0, void* s1) {
    int rc = check_pair(c0, c1);
    if (rc) return rc;
    const uint64_t C = c0->pending_C;
    const bool last = c0->phase == Phase::kPendingLast;
    const uint64_t per = last ? 16 : 4;
    HIP_TRY(c0, c0->scratch2.ensure(std::max<uint64_t>(C, 1) * 8 * 16));
    ChildArgs a = child_args(c0, c1);
    a.prf_seed = seed;
    if (last) HIP_TRY(c0, launch_child_sums_fe255(a, c0->scratch2.as<uint64_t>(), c0->stream));
    else HIP_TRY(c0, launch_child_sums_fe(a, c0->scratch2.as<uint64_t>(), c0->stream, true));
    std::vector<uint64_t> h(C * per);
    rc = fetch_partials(c0, cfg, c0->scratch2.as<uint64_t>(), C * per, h.data());
    if (rc) return rc;
    for (uint64_t c = 0; c < C; c++) {
        if (!last) {
            static_cast<uint64_t*>(s0)[c] = fe_canon_from_limbs(h[c * 4 + 0], h[c * 4 + 1]);
            static_cast<uint64_t*>(s1)[c] = fe_canon_from_limbs(h[c * 4 + 2], h[c * 4 + 3]);
        } else {
            Limbs10 v0 = limbs_from_partials(&h[c * 16]);
            Limbs10 v1 = limbs_from_partials(&h[c * 16 + 8]);
            std::memcpy(static_cast<uint32_t*>(s0) + c * 10, v0.data(), 40);
            std::memcpy(static_cast<uint32_t*>(s1) + c * 10, v1.data(), 40);
            c0->last_values[c] = v0;
            c1->last_values[c] = v1;
        }
    }
    return FHH_OK;
}

int set_device(fhh_ctx* ctx) {
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    return FHH_OK;
}

}  // namespace

namespace fhh {
namespace eng {
int ctx_sync(fhh_ctx* ctx) { return sync(ctx); }
int ctx_set_device(fhh_ctx* ctx) { return set_device(ctx); }
ChildArgs ctx_child_args(fhh_ctx* ctx) { return child_args(ctx, nullptr); }

int crawl_level(fhh_ctx* ctx, bool last, uint64_t* n_children, uint64_t* planes, uint64_t pitch_words,
                uint64_t word_off) {
    int rc = crawl_one(ctx, last);
    if (rc) return rc;
    if (n_children) *n_children = ctx->pending_C;
    if (planes && ctx->pending_C) {
        // k_share_planes writes [C][2d][nw] on the device; one strided copy lands this ctx's words
        // in the caller's rows (the gather of a multi-device ctx costs no host pass)
        const size_t rows = ctx->pending_C * 2 * ctx->d;
        HIP_TRY(ctx, ctx->scratch.ensure(rows * ctx->nw * 8));
        ChildArgs a = child_args(ctx, nullptr);
        HIP_TRY(ctx, launch_share_planes(a, ctx->scratch.as<uint64_t>(), ctx->stream));
        HIP_TRY(ctx, hipMemcpy2DAsync(planes + word_off, pitch_words * 8, ctx->scratch.p, ctx->nw * 8, ctx->nw * 8, rows,
                                      hipMemcpyDeviceToHost, ctx->stream));
    }
    return sync(ctx);
}

bool fmt_is_fe255(uint32_t fmt) { return fmt == FHH_VALS_FE255_LIMBS || fmt == FHH_VALS_FE255_BLOCKPAIR; }

static size_t fmt_bytes(uint32_t fmt) {
    return fmt == FHH_VALS_FE_U64 ? 8 : fmt == FHH_VALS_FE_BLOCK ? 16 : 32;
}

int node_partials(fhh_ctx* ctx, const void* vals, uint32_t fmt, uint64_t ld, uint64_t col0, bool host,
                  uint64_t** partials_dev) {
    if (ctx->phase != Phase::kPending && ctx->phase != Phase::kPendingLast)
        return ctx->fail(FHH_E_STATE, "node_sums without a pending crawl");
    if (fmt > FHH_VALS_FE255_BLOCKPAIR) return ctx->fail(FHH_E_ARG, "node_sums: unknown value format");
    const uint64_t C = ctx->pending_C, n = ctx->n;
    const size_t eb = fmt_bytes(fmt), per = fmt_is_fe255(fmt) ? 8 : 2;
    HIP_TRY(ctx, ctx->scratch2.ensure(std::max<uint64_t>(C, 1) * per * 8));
    *partials_dev = ctx->scratch2.as<uint64_t>();
    if (C == 0) return FHH_OK;
    if (!vals) return ctx->fail(FHH_E_ARG, "node_sums: NULL values");
    if (ld < col0 + n) return ctx->fail(FHH_E_ARG, "node_sums: row pitch shorter than the client count");
    const void* src = vals;
    uint64_t pitch = ld;
    if (host) {
        // this ctx's column block of the caller's [C][ld] rows, one strided host-to-device copy
        HIP_TRY(ctx, ctx->scratch.ensure(C * n * eb));
        HIP_TRY(ctx, hipMemcpy2DAsync(ctx->scratch.p, n * eb, static_cast<const uint8_t*>(vals) + col0 * eb, ld * eb,
                                      n * eb, C, hipMemcpyHostToDevice, ctx->stream));
        src = ctx->scratch.p;
        pitch = n;
    }
    HIP_TRY(ctx, launch_sum_vals(src, fmt, C, n, pitch, *partials_dev, ctx->stream));
    return FHH_OK;
}

int node_sums_finish(fhh_ctx* ctx, const uint64_t* h, uint32_t fmt, void* out_a, void* out_b) {
    const uint64_t C = ctx->pending_C;
    if (!fmt_is_fe255(fmt)) {
        uint64_t* sums = static_cast<uint64_t*>(out_a);   // NULL: a shard that only takes part
        if (!sums) return FHH_OK;
        for (uint64_t c = 0; c < C; c++) sums[c] = fe_canon_from_limbs(h[2 * c], h[2 * c + 1]);
        return FHH_OK;
    }
    uint32_t* unr = static_cast<uint32_t*>(out_a);
    uint32_t* can = static_cast<uint32_t*>(out_b);
    for (uint64_t c = 0; c < C; c++) {
        Limbs10 v = limbs_from_partials(&h[c * 8]);
        if (unr) std::memcpy(unr + c * 10, v.data(), 40);
        if (can) {
            auto r = ::fe255_reduce(v);
            std::memcpy(can + c * 8, r.data(), 32);
        }
        if (ctx->phase == Phase::kPendingLast) ctx->last_values[c] = v;
    }
    return FHH_OK;
}

int add_keys_bincode_records(fhh_ctx* ctx, uint64_t n, const uint8_t* recs) {
    int rc = set_device(ctx);
    if (rc) return rc;
    if (ctx->dev_keys || ctx->h_n) return ctx->fail(FHH_E_STATE, "add_keys_bincode: ctx already holds keys");
    const uint64_t KB = 25 + 20ull * ctx->L, R = 8 + (uint64_t)ctx->K * KB, len = 8 + n * R;
    rc = alloc_keys(ctx, n);
    if (rc) return rc;
    DevBuf buf, err;
    HIP_TRY(ctx, buf.ensure(len + 4));   // k_bincode_cw_tiles reads whole dwords: up to 3 B past len
    HIP_TRY(ctx, err.ensure(4));
    HIP_TRY(ctx, hipMemsetAsync(err.p, 0, 4, ctx->stream));
    // the u64 client count, then the records (a shard of a multi-device ctx uploads its slice)
    HIP_TRY(ctx, hipMemcpyAsync(buf.p, &n, 8, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(buf.as<uint8_t>() + 8, recs, n * R, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, launch_keys_from_bincode(buf.as<uint8_t>(), n, ctx->d, ctx->L, (uint32_t)ctx->npad, (uint32_t)ctx->nw,
                                          ctx->cw_seed.as<uint4>(), ctx->cw_bits.as<uint64_t>(),
                                          ctx->root_seed.as<uint4>(), ctx->key_idx.as<uint64_t>(), err.as<uint32_t>(),
                                          ctx->stream));
    uint32_t herr = 0;
    HIP_TRY(ctx, hipMemcpyAsync(&herr, err.p, 4, hipMemcpyDeviceToHost, ctx->stream));
    rc = sync(ctx);
    if (rc) return rc;
    if (herr) {
        ctx->n = 0;
        return ctx->fail(FHH_E_ARG, std::string("add_keys_bincode: malformed request (") +
                                        ((herr & 1) ? "bool byte > 1 " : "") + ((herr & 2) ? "cor_words length " : "") +
                                        ((herr & 4) ? "dims per client" : "") + ")");
    }
    ctx->dev_keys = true;
    return FHH_OK;
}
}  // namespace eng
}  // namespace fhh

// ---- device-resident level loop (fhh_sim_crawl, host_loop = 0) ---------------------------------
// FHH_DEBUG_PHASES=1 prints host wall-clock per crawl phase to stderr (setup / loop / readback)
struct PhaseClock {
    bool on = std::getenv("FHH_DEBUG_PHASES") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(const char* what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[fhh phase] %-10s %9.3f ms\n", what,
                     std::chrono::duration<double, std::milli>(now - t).count());
        t = now;
    }
};

// Host producer of the real base OTs (fhh_sim_config.base_ot). Each level's two OT extensions — kind
// 0 the evaluator's labels, kind 1 the share conversion — start from their own 128 Chou–Orlandi OTs
// (AlszSender/AlszReceiver::init per channel and level, collect.rs:454-471); the level's chunks extend
// them from disjoint row-PRG counters. The level loop requests instances (lv, kind) a few levels ahead
// of the level it enqueues; worker threads compute them in request order with their key schedules
// [3][128][44] (receiver k_i^0, k_i^1; sender k_i^{s_i}); wait(i) blocks until request i is done.
// Accounting (fhh_stats): compute_ms sums every instance's own CO15 + key-schedule time over the
// workers (the host CPU the base OTs cost), stall_ms is the time the enqueueing thread spent blocked
// in wait() — the base OTs' share of the crawl's critical path. An instance's schedules are released
// once uploaded (release()); a resumed level re-requests and recomputes them.
struct BaseOtProducer {
    struct Inst {
        uint32_t lv, salt;
        std::vector<uint32_t> rk;
        bool done = false;
    };
    uint64_t prf;
    uint8_t seed[32];
    std::deque<Inst> insts;                          // stable addresses under push_back
    std::map<uint64_t, size_t> index;                // (lv << 32 | salt) -> request (until released)
    size_t next_work = 0;
    bool stop = false;
    std::mutex mu;
    std::condition_variable cv_done, cv_work;
    int rc = FHH_OK;
    std::string err;
    std::vector<std::thread> workers;
    double compute_ms = 0;                           // summed per-instance compute (all workers)
    double stall_ms = 0;                             // enqueueing thread blocked in wait()
    uint64_t computed = 0;                           // instances finished
    BaseOtProducer(uint64_t prf_seed, const uint8_t s[32]) : prf(prf_seed) {
        std::memcpy(seed, s, 32);
        unsigned nt = std::thread::hardware_concurrency();
        if (const char* e = std::getenv("OMP_NUM_THREADS")) nt = (unsigned)std::atoi(e);
        nt = std::max(1u, std::min(nt ? nt : 1u, 64u));
        for (unsigned w = 0; w < nt; w++) workers.emplace_back([this] { work(); });
    }
    ~BaseOtProducer() {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv_work.notify_all();
        for (auto& t : workers) t.join();
    }
    size_t request(uint32_t lv, uint32_t salt) {
        std::lock_guard<std::mutex> lk(mu);
        const uint64_t key = (uint64_t)lv << 32 | salt;
        auto it = index.find(key);
        if (it != index.end()) return it->second;
        insts.push_back(Inst{lv, salt, {}, false});
        index.emplace(key, insts.size() - 1);
        cv_work.notify_one();
        return insts.size() - 1;
    }
    void work() {
        std::vector<uint8_t> pairs(128 * 32), chosen(128 * 16);
        for (;;) {
            Inst* in = nullptr;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv_work.wait(lk, [&] { return stop || next_work < insts.size(); });
                if (stop) return;
                in = &insts[next_work++];
            }
            const auto t_begin = std::chrono::steady_clock::now();
            // the OT-extension sender's base choice bits: the words the ideal mode uses (ot_level_choice)
            uint32_t sw[4];
            ot_level_choice(prf, in->lv, in->salt, sw);
            uint8_t ch[16];
            std::memcpy(ch, sw, 16);
            std::string e;
            const int r = base_ot_instance((uint64_t)in->lv << 32 | in->salt, seed, ch, pairs.data(), chosen.data(), &e);
            std::vector<uint32_t> rk;
            if (!r) {
                rk.resize((size_t)3 * 128 * 44);
                for (int i = 0; i < 128; i++) {
                    uint32_t w[11][4];
                    for (int b = 0; b < 3; b++) {
                        host_key_schedule(b < 2 ? &pairs[((size_t)i * 2 + b) * 16] : &chosen[(size_t)i * 16], w);
                        std::memcpy(&rk[((size_t)b * 128 + i) * 44], w, 44 * 4);
                    }
                }
            }
            const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_begin).count();
            std::lock_guard<std::mutex> lk(mu);
            if (r && !rc) {
                rc = r;
                err = e;
            }
            in->rk.swap(rk);
            in->done = true;
            compute_ms += ms;
            computed++;
            cv_done.notify_all();
        }
    }
    int wait(size_t i) {
        std::unique_lock<std::mutex> lk(mu);
        if (insts[i].done || rc != FHH_OK) return rc;
        const auto t_begin = std::chrono::steady_clock::now();
        cv_done.wait(lk, [&] { return insts[i].done || rc != FHH_OK; });
        stall_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_begin).count();
        return rc;
    }
    const uint32_t* schedules(size_t i) {
        std::lock_guard<std::mutex> lk(mu);
        return insts[i].rk.data();
    }
    // the schedules have left the host (their upload returned): free them, and let a later request for
    // the same (lv, salt) compute a fresh instance
    void release(size_t i) {
        std::lock_guard<std::mutex> lk(mu);
        std::vector<uint32_t>().swap(insts[i].rk);
        index.erase((uint64_t)insts[i].lv << 32 | insts[i].salt);
    }
};

struct LoopBuffers {
    DevBuf ctl, live[2], pos[2], mark, partials, sizes, final_vals;
    DevBuf hist_rows, hist_packed;               // end-of-crawl readback (k_gather_hist)
    DevBuf gc_planes[2], gc_tables, gc_gbl, gc_evl, gc_decode, gc_out;   // cfg->gc (row f1)
    DevBuf gc_evact, gc_val[2], gc_y, gc_msgs;                            // cfg->gc = 2: OT / share / table buffers
    // multi-rank: kernels write this rank's partials, k_prune reads the cross-rank sum in
    // `reduced` (out of place, so re-reducing an aborted level's stale partials is idempotent)
    DevBuf reduced;
    DevBuf agree;                                // multi-rank: the growth decision's flags (loop_entry_cap)
    bool distributed = false;
    uint64_t* red() const { return distributed ? reduced.as<uint64_t>() : partials.as<uint64_t>(); }
    // parity probe (cfg->probe_*): per probed level, the gathered states at stride probe_stride
    static constexpr uint32_t kMaxProbe = 16;
    DevBuf probe_seed[kMaxProbe], probe_ty[kMaxProbe];
    uint64_t probe_stride[kMaxProbe] = {};
    DevBuf probe_C, probe_clients;
    // cfg->base_ot: the key schedules [3][128][44] of the real base OTs, uploaded into a ring of
    // kBaseRing slots on the engine stream (stream order: a slot is rewritten only after the OT
    // kernels enqueued before the copy have read it)
    static constexpr uint32_t kBaseRing = 8;
    bool base_ot = false;
    DevBuf base_rk;
    uint32_t base_slot = 0;
    std::unique_ptr<BaseOtProducer> bot;
    std::vector<DevBuf*> hist_epochs;            // hist rows; a new epoch per F_cap growth
    std::vector<uint32_t*> hist_ptr;             // per level
    uint32_t E_cap = 0, F_cap = 0;
    PinnedBuf ctl_host, rec;                     // ctl readback; per-level partial records
    std::vector<size_t> rec_off;                 // per level offset (u64) into rec
    std::vector<uint32_t> rec_stride;            // per level C_cap at that time
    ~LoopBuffers() {
        for (auto* b : hist_epochs) delete b;
    }
};

// wait for the base OTs of OT extension (lv, salt) and copy their key schedules to the next ring
// slot; returns the slot's device address. The copy is from pageable memory, so it has left the host
// buffer on return, and the instance is released.
int upload_base_ot(fhh_ctx* c0, LoopBuffers& B, uint32_t lv, uint32_t salt, const uint32_t** rk_dev) {
    const size_t i = B.bot->request(lv, salt);
    const int rc = B.bot->wait(i);
    if (rc) return c0->fail(rc, "base OTs: " + B.bot->err);
    const size_t words = (size_t)3 * 128 * 44;
    uint32_t* dst = B.base_rk.as<uint32_t>() + (size_t)(B.base_slot++ % LoopBuffers::kBaseRing) * words;
    HIP_TRY(c0, hipMemcpyAsync(dst, B.bot->schedules(i), words * 4, hipMemcpyHostToDevice, c0->stream));
    B.bot->release(i);   // a pageable copy has left the host buffer on return
    *rk_dev = dst;
    return FHH_OK;
}

uint32_t next_pow2(uint32_t v) {
    uint32_t p = 1;
    while (p < v) p <<= 1;
    return p;
}

// grow one buffer of a dim table, preserving the first `keep` entries
int table_grow(fhh_ctx* ctx, DimTable& T, int buf, size_t cap, size_t keep) {
    if (cap <= T.cap[buf] && T.seed[buf].p) return FHH_OK;
    DevBuf ns, nt, ny;
    HIP_TRY(ctx, ns.ensure(cap * 2 * ctx->npad * 16));
    HIP_TRY(ctx, nt.ensure(cap * 2 * ctx->nw * 8));
    HIP_TRY(ctx, ny.ensure(cap * 2 * ctx->nw * 8));
    if (keep) {
        HIP_TRY(ctx, hipMemcpyAsync(ns.p, T.seed[buf].p, keep * 2 * ctx->npad * 16, hipMemcpyDeviceToDevice, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(nt.p, T.t[buf].p, keep * 2 * ctx->nw * 8, hipMemcpyDeviceToDevice, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(ny.p, T.y[buf].p, keep * 2 * ctx->nw * 8, hipMemcpyDeviceToDevice, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    std::swap(T.seed[buf].p, ns.p);
    std::swap(T.seed[buf].bytes, ns.bytes);
    std::swap(T.t[buf].p, nt.p);
    std::swap(T.t[buf].bytes, nt.bytes);
    std::swap(T.y[buf].p, ny.p);
    std::swap(T.y[buf].bytes, ny.bytes);
    T.cap[buf] = cap;
    return FHH_OK;
}

void table_release(DimTable& T, int buf) {
    T.seed[buf].release();
    T.t[buf].release();
    T.y[buf].release();
    T.cap[buf] = 0;
}

size_t table_entry_bytes(const fhh_ctx* c) { return 2 * c->npad * 16 + 2 * 2 * c->nw * 8; }

// Entry capacity of every dim table after a device-loop abort that needs `need` entries. 2x the
// next power of two (few resumes) when the tables of the servers on this device fit beside what
// else is allocated; else 1.25x the need in 64-entry steps; else the need itself. At 1M clients an
// entry is 32 MB (both sides' seeds), so the doubling alone overshot 288 GB at configs[3]'s dense
// thresholds (2 servers x d dims x 2 parities of tables on one GPU).
//
// Ranks of a sharded crawl (cfg->comm / cfg->allreduce) must pick the SAME capacity: the abort level
// of every later batch, the loop's all-reduce sequence and count (C_cap x per) and the next crawl's
// loop_cap_hint all follow from it, and their free memory differs. So each rank's "does candidate k
// fit here" flags are summed over the ranks through the loop's own reduction and the first candidate
// that fits on every rank is taken. FHH_TEST_TABLE_BYTES="a0,a1,..." replaces the available bytes of
// rank r by a_r (the last entry for higher ranks): r = the communicator's rank, or FHH_TEST_RANK on the
// cfg->allreduce callback path (0 if unset): tests force different free memory per rank with it.
int loop_entry_cap(fhh_ctx* const (&cs)[2], const fhh_sim_config* cfg, LoopBuffers& B, uint32_t d, uint32_t E_cap,
                   uint32_t need, uint32_t la, uint32_t& out) {
    size_t free_b = 0, total_b = 0;
    HIP_TRY(cs[0], hipMemGetInfo(&free_b, &total_b));
    size_t held = 0, old_pres = 0, n_tab = 0;   // bytes the tables hold now; largest preserved one
    for (fhh_ctx* c : cs) {
        if (c->device != cs[0]->device) continue;
        const size_t bpe = table_entry_bytes(c);
        for (uint32_t j = 0; j < d; j++) {
            held += (c->tab[j].cap[0] + c->tab[j].cap[1]) * bpe;
            old_pres = std::max(old_pres, c->tab[j].cap[1 - (la & 1)] * bpe);
            n_tab += 2;
        }
    }
    const size_t bpe = table_entry_bytes(cs[0]);
    const size_t margin = (size_t)2 << 30;
    size_t avail = free_b + held > margin ? free_b + held - margin : 0;
    if (const char* e = std::getenv("FHH_TEST_TABLE_BYTES")) {
        const char* tr = std::getenv("FHH_TEST_RANK");
        const int r = cfg->comm ? comm_rank(cfg->comm) : (tr ? std::atoi(tr) : 0);
        std::string s(e);
        size_t pos = 0;
        for (int k = 0;; k++) {
            const size_t comma = s.find(',', pos);
            avail = (size_t)std::strtoull(s.substr(pos, comma - pos).c_str(), nullptr, 10);
            if (k == r || comma == std::string::npos) break;
            pos = comma + 1;
        }
    }
    const uint64_t cand[3] = {(uint64_t)next_pow2(need) * 2, ((uint64_t)need * 5 / 4 + 63) / 64 * 64, need};
    uint64_t nofit[3];
    for (int k = 0; k < 3; k++) {
        const uint64_t e = std::max<uint64_t>(cand[k], E_cap);
        nofit[k] = e * bpe * n_tab + old_pres <= avail ? 0 : 1;
    }
    if (cfg->comm || cfg->allreduce) {
        // every rank reaches this abort at the same level (the frontier is replicated and the
        // capacities agree), so the extra collective pairs up across ranks
        fhh_ctx* c0 = cs[0];
        HIP_TRY(c0, B.agree.ensure(2 * 3 * 8));
        uint64_t* dv = B.agree.as<uint64_t>();
        HIP_TRY(c0, hipMemcpyAsync(dv, nofit, sizeof nofit, hipMemcpyHostToDevice, c0->stream));
        if (cfg->comm) {
            std::string err;
            if (comm_allreduce(cfg->comm, dv, dv + 3, 3, c0->stream, &err)) return c0->fail(FHH_E_COMM, err);
        } else {
            if (!cfg->xchg_dev || cfg->xchg_capacity < 3)
                return c0->fail(FHH_E_ARG, "sim: all-reduce exchange buffer too small");
            HIP_TRY(c0, hipMemcpyAsync(cfg->xchg_dev, dv, sizeof nofit, hipMemcpyDeviceToDevice, c0->stream));
            HIP_TRY(c0, hipStreamSynchronize(c0->stream));
            if (cfg->allreduce(cfg->xchg_dev, 3, cfg->allreduce_user) != 0)
                return c0->fail(FHH_E_CALLBACK, "all-reduce callback failed");
            HIP_TRY(c0, hipMemcpyAsync(dv + 3, cfg->xchg_dev, sizeof nofit, hipMemcpyDeviceToDevice, c0->stream));
        }
        HIP_TRY(c0, hipMemcpyAsync(nofit, dv + 3, sizeof nofit, hipMemcpyDeviceToHost, c0->stream));
        HIP_TRY(c0, hipStreamSynchronize(c0->stream));
    }
    out = std::max<uint32_t>(E_cap, need);
    for (int k = 0; k < 3; k++)
        if (!nofit[k]) {
            out = (uint32_t)std::max<uint64_t>(cand[k], E_cap);
            break;
        }
    if (std::getenv("FHH_DEBUG_LOOP"))
        std::fprintf(stderr, "[fhh loop] entry cap: need %u -> %u (%.1f GB of tables, %.1f GB available)\n", need,
                     out, (double)out * bpe * n_tab / 1e9, (double)avail / 1e9);
    return FHH_OK;
}

// (re)size the loop buffers; preserve what a resumed prune of `level` still reads
int loop_resize(fhh_ctx* c0, LoopBuffers& B, uint32_t E_cap, uint32_t F_cap, uint32_t levels, uint32_t level,
                bool preserve, uint32_t keep_nodes, uint32_t keep_children, uint32_t per) {
    const uint32_t d = c0->d;
    const size_t C_old = (size_t)B.F_cap << d, C_new = (size_t)F_cap << d;
    HIP_TRY(c0, hipStreamSynchronize(c0->stream));
    for (int b = 0; b < 2; b++) {
        DevBuf nl;
        HIP_TRY(c0, nl.ensure((size_t)d * E_cap * 4));
        std::swap(B.live[b].p, nl.p);
        std::swap(B.live[b].bytes, nl.bytes);
        DevBuf np;
        HIP_TRY(c0, np.ensure((size_t)F_cap * d * 4));
        const int keep_par = level & 1;
        if (preserve && b == keep_par && keep_nodes) {
            // stream-ordered (the engine streams do not wait for the null stream), and finished
            // before the old buffer is released
            HIP_TRY(c0, hipMemcpyAsync(np.p, B.pos[b].p, (size_t)keep_nodes * d * 4, hipMemcpyDeviceToDevice, c0->stream));
            HIP_TRY(c0, hipStreamSynchronize(c0->stream));
        }
        std::swap(B.pos[b].p, np.p);
        std::swap(B.pos[b].bytes, np.bytes);
    }
    HIP_TRY(c0, B.mark.ensure((size_t)d * E_cap * 4));
    {
        // a resumed prune reads the (reduced) partials of `level`
        DevBuf npart, nred;
        HIP_TRY(c0, npart.ensure(C_new * 16 * 8));
        // FE levels add into the partials (k_child_sums_fe client chunks); k_prune re-zeroes them
        HIP_TRY(c0, hipMemsetAsync(npart.p, 0, C_new * 16 * 8, c0->stream));
        if (B.distributed) HIP_TRY(c0, nred.ensure(C_new * 16 * 8));
        // ... and, multi-rank, the local partials too: the all-reduces of the no-op levels
        // after an abort re-reduce them, which must reproduce the same sums
        if (preserve && keep_children) {
            HIP_TRY(c0, hipMemcpyAsync(npart.p, B.partials.p, (size_t)keep_children * per * 8, hipMemcpyDeviceToDevice, c0->stream));
            if (B.distributed)
                HIP_TRY(c0, hipMemcpyAsync(nred.p, B.reduced.p, (size_t)keep_children * per * 8, hipMemcpyDeviceToDevice, c0->stream));
        }
        HIP_TRY(c0, hipStreamSynchronize(c0->stream));
        std::swap(B.partials.p, npart.p);
        std::swap(B.partials.bytes, npart.bytes);
        if (B.distributed) {
            std::swap(B.reduced.p, nred.p);
            std::swap(B.reduced.bytes, nred.bytes);
        }
    }
    (void)C_old;
    // hist rows for levels >= level live in a new epoch of stride F_cap
    DevBuf* ep = new DevBuf();
    if (ep->ensure((size_t)(levels - level) * F_cap * 4) != hipSuccess) {
        delete ep;
        return c0->fail(FHH_E_NOMEM, "loop: hist allocation failed");
    }
    B.hist_epochs.push_back(ep);
    B.hist_ptr.resize(levels, nullptr);
    for (uint32_t lv = level; lv < levels; lv++) B.hist_ptr[lv] = ep->as<uint32_t>() + (size_t)(lv - level) * F_cap;
    B.E_cap = E_cap;
    B.F_cap = F_cap;
    return FHH_OK;
}

int sim_crawl_device_loop(fhh_ctx* c0, fhh_ctx* c1, const fhh_sim_config* cfg, uint32_t levels, uint64_t thr,
                          uint32_t thr_last) {
    const uint32_t d = c0->d;
    const int variant = c0->variant;
    const uint64_t grid_waves = (uint64_t)c0->grid * (expand_threads(variant) / 64);
    const uint32_t per_level_per = cfg->mode == 0 ? 1 : 4;   // partial u64 per child (non-last)
    // GC + OT chunk: children per protocol instance, so the level's GC and OT buffers (~400 B per
    // test at d = 1) stay within FHH_GC_CHUNK_BYTES (default 64 GiB): one chunk per level at
    // configs[1], ~160 children per chunk at 1M clients
    uint64_t gc_groups = ~0ull, gc_groups_last = ~0ull;
    if (cfg->gc) {
        uint64_t budget = 64ull << 30;
        if (const char* e = std::getenv("FHH_GC_CHUNK_BYTES")) budget = std::strtoull(e, nullptr, 10);
        // r06: the d = 1 garbled table on the tile-major labels holds ~140 B per test (T, U, Q 96, rows 24,
        // node values 16), not the circuit's ~400: larger chunks, one per level at 1M clients
        const bool tm_table = cfg->gc == 2 && 2 * d <= (uint32_t)kGtTmMaxBits;
        const uint64_t per_test = tm_table ? 150ull : 200ull * 2 * d + 2;
        gc_groups = std::max<uint64_t>(1, budget / (per_test * std::max<uint64_t>(c0->npad, 1)));
        // the FieldElm level runs the circuit + share C-OT whatever the FE levels run
        gc_groups_last = std::max<uint64_t>(1, budget / ((200ull * 2 * d + 2) * std::max<uint64_t>(c0->npad, 1)));
    }
    // r06: Z_2^32 table shares at the FE levels (the tile-major table with fused sums, d = 1)
    const bool ring32 = cfg->table_ring32 && cfg->gc == 2 && cfg->mode == 1 && 2 * d <= (uint32_t)kGtTmMaxBits &&
                        FHH_GT_FUSED_SUMS;
    PhaseClock pc;
    LoopBuffers B;
    B.distributed = cfg->comm || cfg->allreduce;
    uint32_t cap0 = std::max(cfg->init_capacity ? next_pow2(cfg->init_capacity) : 256u, c0->loop_cap_hint);
    // tables: both buffers of every dim of both servers hold >= E_cap entries
    fhh_ctx* cs[2] = {c0, c1};
    for (fhh_ctx* c : cs)
        for (uint32_t j = 0; j < d; j++)
            for (int b = 0; b < 2; b++) {
                int rc = table_grow(c, c->tab[j], b, std::max<size_t>(cap0, c->tab[j].cap[b]), 0);
                if (rc) return rc;
            }
    int rc = fhh_tree_init(c0);   // fills buffer 0 with the roots (after the growth above)
    if (rc) return rc;
    rc = fhh_tree_init(c1);
    if (rc) return rc;
    PairScope pair(c0, c1);
    HIP_TRY(c0, B.ctl.ensure(sizeof(LoopCtl)));
    HIP_TRY(c0, B.sizes.ensure((size_t)levels * (4 + kMaxDims) * 4));
    HIP_TRY(c0, hipMemsetAsync(B.sizes.p, 0, (size_t)levels * (4 + kMaxDims) * 4, c0->stream));
    HIP_TRY(c0, B.ctl_host.ensure(sizeof(LoopCtl)));
    rc = loop_resize(c0, B, cap0, cap0, levels, 0, false, 0, 0, 1);
    if (rc) return rc;
    if (cfg->gc >= 2 && cfg->base_ot) {
        // the OT extensions of every level and chunk each start with 128 Chou–Orlandi base OTs
        // (AlszSender/AlszReceiver::init, collect.rs:454-471): host threads produce them a few levels
        // ahead of this thread's enqueueing, which waits only for the chunk it is about to enqueue
        uint8_t seed[32];
        for (int k = 0; k < 4; k++) {
            const uint64_t z = host_mix64(cfg->prf_seed ^ (0x626173655f6f74ull + (uint64_t)k));
            std::memcpy(seed + 8 * k, &z, 8);
        }
        HIP_TRY(c0, B.base_rk.ensure((size_t)LoopBuffers::kBaseRing * 3 * 128 * 44 * 4));
        B.bot = std::make_unique<BaseOtProducer>(cfg->prf_seed, seed);
        B.base_ot = true;
    }
    if (cfg->probe_n_levels) {
        if (cfg->probe_n_levels > LoopBuffers::kMaxProbe || !cfg->probe_levels || !cfg->probe_n_clients ||
            !cfg->probe_clients || !cfg->probe_seeds || !cfg->probe_ty || !cfg->probe_children)
            return c0->fail(FHH_E_ARG, "sim_crawl: bad probe arguments");
        for (uint32_t i = 0; i < cfg->probe_n_clients; i++)
            if (cfg->probe_clients[i] >= c0->n) return c0->fail(FHH_E_ARG, "sim_crawl: probe client out of range");
        HIP_TRY(c0, B.probe_C.ensure((size_t)cfg->probe_n_levels * 4));
        HIP_TRY(c0, hipMemsetAsync(B.probe_C.p, 0, (size_t)cfg->probe_n_levels * 4, c0->stream));
        HIP_TRY(c0, B.probe_clients.ensure((size_t)cfg->probe_n_clients * 8));
        HIP_TRY(c0, hipMemcpyAsync(B.probe_clients.p, cfg->probe_clients, (size_t)cfg->probe_n_clients * 8,
                                   hipMemcpyHostToDevice, c0->stream));
        HIP_TRY(c0, hipStreamSynchronize(c0->stream));
    }
    {
        uint32_t* l0[kMaxDims] = {nullptr, nullptr, nullptr, nullptr};
        for (uint32_t j = 0; j < d; j++) l0[j] = B.live[0].as<uint32_t>() + (size_t)j * B.E_cap;
        for (uint32_t j = d; j < kMaxDims; j++) l0[j] = l0[0];
        HIP_TRY(c0, launch_loop_init(B.ctl.as<LoopCtl>(), d, (uint32_t)c0->nw, expand_max_group(variant),
                                     expand_max_wpi(variant),
                                     d, 2, grid_waves, B.pos[0].as<uint32_t>(), l0, c0->stream));
    }
    pc.mark("setup");
    const bool record = cfg->counts != nullptr;
    const uint32_t kBatch = 32;
    bool prune_only = false;           // resume after growth: prune of this level only
    for (uint32_t lv = 0; lv < levels;) {
        const bool last = lv + 1 == levels;
        const int par = lv & 1;
        const uint32_t pmode = cfg->mode == 0 ? 0 : (last ? 2 : 1);
        const uint32_t per = pmode == 0 ? 1 : (pmode == 1 ? 4 : 16);
        const uint64_t C_cap = (uint64_t)B.F_cap << d;
        if (!prune_only) {
            // -- k_expand, both servers, sizes from LoopCtl
            ExpandLaunch La{};
            La.njobs = 2 * d;
            La.jobs_per_ctx = d;
            La.ctl = B.ctl.as<LoopCtl>();
            for (int s = 0; s < 2; s++)
                for (uint32_t j = 0; j < d; j++) {
                    fhh_ctx* c = cs[s];
                    DimTable& T = c->tab[j];
                    ExpandJob& J = La.job[s * d + j];
                    J.cw_seed = c->cw_seed.as<uint4>();
                    J.cw_bits = c->cw_bits.as<uint64_t>();
                    J.src_seed = T.seed[par].as<uint4>();
                    J.src_t = T.t[par].as<uint64_t>();
                    J.src_y = T.y[par].as<uint64_t>();
                    J.dst_seed = T.seed[1 - par].as<uint4>();
                    J.dst_t = T.t[1 - par].as<uint64_t>();
                    J.dst_y = T.y[1 - par].as<uint64_t>();
                    J.live = B.live[par].as<uint32_t>() + (size_t)j * B.E_cap;
                    J.level = lv;
                    J.dim = j;
                    J.K = c->K;
                    J.npad = (uint32_t)c->npad;
                    J.nw = (uint32_t)c->nw;
                }
            size_t slot = 0;
            const bool timed = c0->timing && lv % c0->timing_every == 0;
            if (timed) HIP_TRY(c0, timing_begin(c0, &slot));
            La.total_items = 1;   // non-zero: the real count comes from LoopCtl
            HIP_TRY(c0, launch_expand(La, variant, c0->grid, c0->work_counter.as<uint32_t>(), &c0->expand_seq, c0->stream));
            if (timed) HIP_TRY(c0, timing_end(c0, slot, 0));
            c0->stats.expand_launches++;
            for (uint32_t k = 0; k < cfg->probe_n_levels; k++) {
                if (cfg->probe_levels[k] != lv) continue;
                const size_t per = (size_t)C_cap * cfg->probe_n_clients * d * 2;
                HIP_TRY(c0, B.probe_seed[k].ensure(2 * per * 16));
                HIP_TRY(c0, B.probe_ty[k].ensure(2 * per));
                B.probe_stride[k] = C_cap;
                ProbeArgs pr{};
                for (int s = 0; s < 2; s++)
                    for (uint32_t j = 0; j < d; j++) {
                        pr.seed[s][j] = cs[s]->tab[j].seed[1 - par].as<uint4>();
                        pr.t[s][j] = cs[s]->tab[j].t[1 - par].as<uint64_t>();
                        pr.y[s][j] = cs[s]->tab[j].y[1 - par].as<uint64_t>();
                    }
                pr.parent_pos = B.pos[par].as<uint32_t>();
                pr.clients = B.probe_clients.as<uint64_t>();
                pr.ctl = B.ctl.as<LoopCtl>();
                pr.out_seed = B.probe_seed[k].as<uint4>();
                pr.out_ty = B.probe_ty[k].as<uint8_t>();
                pr.out_C = B.probe_C.as<uint32_t>() + k;
                pr.C_cap = C_cap;
                pr.npad = c0->npad;
                pr.nw = c0->nw;
                pr.n_probe = cfg->probe_n_clients;
                pr.d = d;
                HIP_TRY(c0, launch_probe_states(pr, c0->stream));
            }
            // -- equality count / simulated OT sums per child
            ChildArgs a{};
            for (uint32_t j = 0; j < d; j++) {
                a.s0.t[j] = c0->tab[j].t[1 - par].as<uint64_t>();
                a.s0.y[j] = c0->tab[j].y[1 - par].as<uint64_t>();
                a.s1.t[j] = c1->tab[j].t[1 - par].as<uint64_t>();
                a.s1.y[j] = c1->tab[j].y[1 - par].as<uint64_t>();
            }
            a.parent_pos = B.pos[par].as<uint32_t>();
            a.valid = c0->valid.as<uint64_t>();
            a.C = C_cap;   // grid hint; the real C comes from LoopCtl
            a.d = d;
            a.nw = (uint32_t)c0->nw;
            a.client_base = c0->client_base;
            a.prf_seed = cfg->prf_seed;
            a.level = lv;
            a.n = (uint32_t)c0->n;
            a.ctl = B.ctl.as<LoopCtl>();
            uint64_t* part = B.partials.as<uint64_t>();
            if (cfg->gc && pmode != 0) {
                // garbled-circuit equality (tree_crawl with gc_sender, collect.rs:419-482): both
                // servers' share planes, server 0 garbles, server 1 evaluates. The level's tests
                // run in chunks of gc_groups children (bounded memory at 1M clients; the reference
                // splits a level's tests over its channels the same way, collect.rs:423-430), each
                // chunk a fresh protocol instance: its own garbler key / Delta / mask, and its own
                // row-PRG range of the level's base-OT sessions
                const uint32_t bits = 2 * d;
                const bool real_ot = cfg->gc >= 2;
                // r05c / r05d: at the FE levels the share comes from the circuit's output labels, or (d <= 2,
                // gc 2) from ONE garbled table per test; r06: for b <= 2 (d = 1) the table kernels read the
                // labels OT's tile-major Q / T themselves (no k_ot_rows_out), which wants plane rows of
                // whole 512-client tiles: the planes and the OT index take nw_gc = nw rounded up to 8 words
                const bool lshare = real_ot && pmode == 1;
                const bool ltable = lshare && bits <= (uint32_t)kGtMaxBits && cfg->gc == 2;   // gc 3: the circuit
                const bool ltm = ltable && bits <= (uint32_t)kGtTmMaxBits;
                const uint64_t nw_gc = ltm ? (c0->nw + 7) / 8 * 8 : c0->nw, npad_gc = 64 * nw_gc;
                const size_t plane_bytes = (size_t)C_cap * bits * nw_gc * 8;
                for (int s = 0; s < 2; s++) HIP_TRY(c0, B.gc_planes[s].ensure(plane_bytes));
                size_t gc_slot = 0;
                if (timed) HIP_TRY(c0, timing_begin(c0, &gc_slot));
                ChildArgs pa = a;
                pa.plane_nw = (uint32_t)nw_gc;
                HIP_TRY(c0, launch_share_planes(pa, B.gc_planes[0].as<uint64_t>(), c0->stream));
                pa.s0 = a.s1;
                HIP_TRY(c0, launch_share_planes(pa, B.gc_planes[1].as<uint64_t>(), c0->stream));
                const uint64_t Gc = std::min<uint64_t>(C_cap, pmode == 2 ? gc_groups_last : gc_groups);
                const uint64_t chunks = (C_cap + Gc - 1) / Gc;
                const uint64_t tests = Gc * c0->n;
                const uint32_t per2 = pmode == 1 ? 1 : 2;   // OTs per test of the share conversion
                const uint64_t m1 = Gc * bits * npad_gc, m2 = tests * per2;
                // the level's two base-OT sessions (OtSender / OtReceiver::init per level and kind,
                // collect.rs:454,460): kind 0 the labels OT, kind 1 the share OT; chunk k extends them
                // from row-PRG block k x (the chunk's blocks), so no two chunks share a pad
                const uint32_t* rk_ot[2] = {nullptr, nullptr};
                uint32_t sw_ot[2][4];
                if (real_ot) {
                    HIP_TRY(c0, c0->ot_rk.ensure((size_t)2 * 3 * 128 * 44 * 4));
                    if (B.base_ot) {
                        // keep the producer well ahead of the enqueueing: the first levels take ~1 ms of
                        // GPU time against ~9 ms per CO15 instance, so at 4 levels ahead the loop waited
                        // 0.56-0.59 s per 1M crawl (base_ot_stall_ms); 32 levels = 64 instances, 4.3 MB
                        // (kind 1, the share OT, runs at the FieldElm level only: the FE levels take their
                        // share from the circuit's output labels, r05c)
                        constexpr uint32_t kAhead = 32;
                        for (uint32_t l = lv; l < std::min(levels, lv + kAhead); l++)
                            for (uint32_t w = 0; w < (l + 1 == levels ? 2u : 1u); w++) (void)B.bot->request(l, w);
                    }
                    for (uint32_t w = 0; w < (pmode == 2 ? 2u : 1u); w++) {
                        ot_level_choice(cfg->prf_seed, lv, w, sw_ot[w]);
                        if (B.base_ot) {
                            rc = upload_base_ot(c0, B, lv, w, &rk_ot[w]);
                            if (rc) return rc;
                        } else {
                            uint32_t* rk = c0->ot_rk.as<uint32_t>() + (size_t)w * 3 * 128 * 44;
                            HIP_TRY(c0, launch_ot_level_keys(cfg->prf_seed, lv, w, sw_ot[w], rk, c0->stream));
                            rk_ot[w] = rk;
                        }
                    }
                }
                // (the garbled table writes no half-gate tables, decoding bits or output bytes)
                HIP_TRY(c0, B.gc_tables.ensure(ltable ? 16 : (size_t)std::max(bits - 1, 1u) * 2 * tests * 16));
                // garbler labels: the ideal-OT garbler's only (the r05 garbler folds its string in)
                HIP_TRY(c0, B.gc_gbl.ensure(real_ot ? 16 : (size_t)(bits + 1) * tests * 16));
                // ideal OT: the evaluator's active labels [bits][tests]; OT mode: its zero labels (the
                // labels C-OT's sender messages) at OT index (g bits + j) npad + i (r06 tile-major table: none,
                // the kernels read Q / T)
                HIP_TRY(c0, B.gc_evl.ensure(std::max<size_t>((size_t)bits * tests, real_ot && !ltm ? m1 : 0) * 16));
                HIP_TRY(c0, B.gc_decode.ensure(ltable ? 1 : tests));
                HIP_TRY(c0, B.gc_out.ensure(ltable ? 1 : tests));
                for (uint64_t k = 0; k < chunks; k++) {
                    const uint64_t g_off = k * Gc;
                    fhh_gc_batch gb{};
                    gb.groups = Gc;
                    gb.clients = (uint32_t)c0->n;
                    gb.words = (uint32_t)nw_gc;
                    gb.bits = bits;
                    gc_chunk_material(cfg->prf_seed, lv, k, gb.label_key, gb.delta, &gb.mask);
                    gb.gate_base = (uint64_t)lv << 40;   // the level in the gate tweaks (party_gate_base)
                    gb.gb_planes_dev = B.gc_planes[0].as<uint64_t>();
                    gb.ev_planes_dev = B.gc_planes[1].as<uint64_t>();
                    gb.tables_dev = B.gc_tables.as<uint8_t>();
                    gb.gb_labels_dev = B.gc_gbl.as<uint8_t>();
                    gb.ev_labels_dev = B.gc_evl.as<uint8_t>();
                    gb.decode_dev = B.gc_decode.as<uint8_t>();
                    gb.out_dev = B.gc_out.as<uint8_t>();
                    GcArgs g{};
                    rc = gc_args(c0, &gb, g);
                    if (rc) return rc;
                    g.ctl = B.ctl.as<LoopCtl>();
                    g.g_off = g_off;
                    if (real_ot) {
                        // 1. the evaluator's input labels by correlated OT (gb_set_fancy_inputs /
                        // ev_set_fancy_inputs, equalitytest.rs:67-82,108-119): server 1's choice bits are
                        // its share planes [C][bits][nw] from the chunk's first group on, as they stand
                        // (m1 a multiple of 128: npad of 64, bits even). The IKNP correlation is the label
                        // pair (r05b, OtArgs mode 4): server 0's q_j is the zero label, server 1's t_j =
                        // q_j ^ r_j s the active one, with the labels session's s (colour bit set) as the
                        // circuit's Delta; server 0's string and mask fold into the circuit
                        // (k_gc_garble_cot: no label is drawn, no reply is sent)
                        if (!ltm) HIP_TRY(c0, B.gc_evact.ensure(m1 * 16));
                        for (int c = 0; c < 4; c++) g.delta[c] = sw_ot[0][c];
                        OtArgs a1{};
                        a1.mode = ltm ? 5 : 4;
                        a1.rk = rk_ot[0];
                        for (int c = 0; c < 4; c++) a1.s[c] = sw_ot[0][c];
                        a1.choices = B.gc_planes[1].as<uint32_t>() + g_off * bits * nw_gc * 2;
                        a1.ctr_off = k * ot_session_blocks(m1);
                        a1.sx = ltm ? nullptr : B.gc_evl.p;
                        a1.out = ltm ? nullptr : B.gc_evact.as<uint4>();
                        a1.ctl = B.ctl.as<LoopCtl>();
                        a1.per_group = npad_gc * bits;
                        a1.g_off = g_off;
                        a1.ss_k = cfg->ot_ss_k;
                        rc = ot_run(c0, a1, m1, nullptr);
                        if (rc) return rc;
                        g.ev_ot = 1;
                        if (ltm) {   // the table kernels on the tile-major Q (garbler) / T (evaluator)
                            g.lab_tm = 1;
                            g.ev_labels = c0->ot_buf[2].as<uint4>();
                        }
                    }
                    // r05c: at the FE levels the share comes from the circuit's output labels (W_0 and
                    // W_0 ^ Delta of o = eq ^ mask in the share C-OT's roles): server 0's node value r1 and
                    // the 8-B y from k_gc_garble_cot, server 1's value from k_gc_eval — no second OT.
                    // r05d: tests of <= kGtMaxBits bits (d <= 2) take the share from ONE garbled table per
                    // test (k_gt_garble / k_gt_eval: 2^bits + 1 AES instead of the half-gates chain's)
                    if (ltable) {
                        // r06 (tile-major table): the kernels add the node values per child into the level's
                        // partials themselves (no stored values, no k_child_sums_fe pass)
                        const bool fused = ltm && FHH_GT_FUSED_SUMS;
                        if (!fused) for (int sv = 0; sv < 2; sv++) HIP_TRY(c0, B.gc_val[sv].ensure(tests * 8));
                        HIP_TRY(c0, B.gc_msgs.ensure(tests * (((size_t)1 << bits) - 1) * 8));
                        g.gt_msgs = B.gc_msgs.as<uint64_t>();
                        g.node_partials = ltm && FHH_GT_FUSED_SUMS ? part : nullptr;
                        g.node_off = 0;
                        g.ring32 = ring32 && ltm ? 1u : 0u;
                        g.sh_gb = fused ? nullptr : B.gc_val[0].as<uint64_t>();
                        HIP_TRY(c0, launch_gt_garble(g, c0->stream));
                        g.ev_labels = ltm ? c0->ot_buf[0].as<uint4>() : B.gc_evact.as<uint4>();
                        g.sh_gb = nullptr;
                        g.sh_ev = fused ? nullptr : B.gc_val[1].as<uint64_t>();
                        HIP_TRY(c0, launch_gt_eval(g, c0->stream));
                    } else if (lshare) {
                        for (int sv = 0; sv < 2; sv++) HIP_TRY(c0, B.gc_val[sv].ensure(tests * 8));
                        HIP_TRY(c0, B.gc_y.ensure(tests * 8));
                        g.sh_gb = B.gc_val[0].as<uint64_t>();
                        g.sh_y = B.gc_y.as<uint64_t>();
                    }
                    if (!ltable) {
                        HIP_TRY(c0, launch_gc_garble(g, c0->stream));
                        if (real_ot) {
                            g.ev_labels = B.gc_evact.as<uint4>();
                            g.sh_gb = nullptr;
                            if (lshare) {
                                g.sh_ev = B.gc_val[1].as<uint64_t>();
                            } else {
                                // k_gc_eval ballot-packs its outputs as the share-conversion OT's choice words
                                uint32_t* och = nullptr;
                                HIP_TRY(c0, ot_choices_buffer(c0, m2, &och));
                                g.out_packed = och;
                                g.out_dup = per2;
                            }
                        }
                        HIP_TRY(c0, launch_gc_eval(g, c0->stream));
                    }
                    ChildArgs ca = a;   // this chunk's children
                    ca.c_off = g_off;
                    ca.c_cnt = Gc;
                    ca.gc_out = g.out;
                    ca.gc_N = g.N;
                    ca.gc_mask = g.mask;
                    if (lshare) {
                        ca.ot_val[0] = B.gc_val[0].p;
                        ca.ot_val[1] = B.gc_val[1].p;
                    } else if (real_ot) {
                        // 2. the share conversion by correlated OT (collect.rs:846-876 at the last level,
                        // where a FieldElm travels as a BlockPair = 2 OTs): server 0's pair is
                        // (H(q_j), H(q_j) +- 1) ordered by its mask, its node value r1 = H(q_j) + mask;
                        // server 1 chooses with its GC output bit
                        const size_t vb = pmode == 1 ? 8 : 16;
                        for (int sv = 0; sv < 2; sv++) HIP_TRY(c0, B.gc_val[sv].ensure(m2 * vb));
                        OtArgs a2{};
                        a2.mode = pmode == 1 ? 2 : 3;
                        a2.mask = g.mask;
                        a2.rk = rk_ot[1];
                        for (int c = 0; c < 4; c++) a2.s[c] = sw_ot[1][c];
                        a2.choices = g.out_packed;
                        a2.ctr_off = k * ot_session_blocks(m2);
                        a2.sx = B.gc_val[0].p;
                        a2.out = B.gc_val[1].as<uint4>();
                        a2.ctl = B.ctl.as<LoopCtl>();
                        a2.per_group = (uint64_t)c0->n * per2;
                        a2.g_off = g_off;
                        a2.ss_k = cfg->ot_ss_k;
                        rc = ot_run(c0, a2, m2, nullptr);
                        if (rc) return rc;
                        ca.ot_val[0] = B.gc_val[0].p;
                        ca.ot_val[1] = B.gc_val[1].p;
                    }
                    // the chunk's children's sums (FE: atomics into the partials k_prune zeroed;
                    // FE255: one store per child)
                    if (pmode == 1) {
                        if (!(ltm && FHH_GT_FUSED_SUMS)) HIP_TRY(c0, launch_child_sums_fe(ca, part, c0->stream, false));
                    } else {
                        HIP_TRY(c0, launch_child_sums_fe255(ca, part, c0->stream));
                    }
                }
                if (timed) HIP_TRY(c0, timing_end(c0, gc_slot, kGcotTag));
            } else if (pmode == 0) {
                HIP_TRY(c0, launch_eq_count(a, part, c0->stream));
            } else if (pmode == 1) {
                HIP_TRY(c0, launch_child_sums_fe(a, part, c0->stream, false));
            } else {
                HIP_TRY(c0, launch_child_sums_fe255(a, part, c0->stream));
            }
            // -- cross-rank sum (client-sharded multi-GPU)
            // (the count is the capacity bound: entries past C are never read)
            if (cfg->comm) {
                std::string err;
                size_t ar_slot = 0;
                if (timed) HIP_TRY(c0, timing_begin(c0, &ar_slot));
                if (comm_allreduce(cfg->comm, part, B.red(), C_cap * per, c0->stream, &err))
                    return c0->fail(FHH_E_COMM, err);
                if (timed) HIP_TRY(c0, timing_end(c0, ar_slot, kAllreduceTag));
            } else if (cfg->allreduce) {
                const uint64_t count = C_cap * per;
                if (!cfg->xchg_dev || cfg->xchg_capacity < count)
                    return c0->fail(FHH_E_ARG, "sim: all-reduce exchange buffer too small");
                HIP_TRY(c0, hipMemcpyAsync(cfg->xchg_dev, part, count * 8, hipMemcpyDeviceToDevice, c0->stream));
                rc = sync(c0);
                if (rc) return rc;
                if (cfg->allreduce(cfg->xchg_dev, count, cfg->allreduce_user) != 0)
                    return c0->fail(FHH_E_CALLBACK, "all-reduce callback failed");
                HIP_TRY(c0, hipMemcpyAsync(B.red(), cfg->xchg_dev, count * 8, hipMemcpyDeviceToDevice, c0->stream));
            }
            if (record) {
                const size_t off = B.rec_off.empty() ? 0 : B.rec_off.back() + (size_t)B.rec_stride.back();
                const size_t need = (off + C_cap * per) * 8;
                if (B.rec.bytes < need) {
                    PinnedBuf nb;
                    HIP_TRY(c0, hipStreamSynchronize(c0->stream));
                    HIP_TRY(c0, nb.ensure(std::max(need * 2, (size_t)1 << 20)));
                    if (B.rec.p) std::memcpy(nb.p, B.rec.p, B.rec.bytes);
                    std::swap(B.rec.p, nb.p);
                    std::swap(B.rec.bytes, nb.bytes);
                }
                B.rec_off.resize(lv + 1);
                B.rec_stride.resize(lv + 1);
                B.rec_off[lv] = off;
                B.rec_stride[lv] = (uint32_t)(C_cap * per);   // u64 words recorded for this level
                // mode 0: counts; FE: the 4 limbs; FE255: the 16 limbs (v0 - v1 derived at the end)
                const size_t cpy = (size_t)C_cap * per * 8;
                HIP_TRY(c0, hipMemcpyAsync(B.rec.as<uint64_t>() + off, B.red(), cpy, hipMemcpyDeviceToHost, c0->stream));
            }
        }
        prune_only = false;
        // -- leader keep decision + prune (or final list at the last level)
        if (last) HIP_TRY(c0, B.final_vals.ensure((size_t)B.F_cap * 20 * 4));
        PruneArgs pa{};
        pa.ctl = B.ctl.as<LoopCtl>();
        pa.partials = B.red();
        pa.mode = pmode;
        pa.d = d;
        pa.thr = thr;
        pa.thr_last = thr_last;
        pa.last = last ? 1 : 0;
        pa.pos_in = B.pos[par].as<uint32_t>();
        pa.pos_out = B.pos[1 - par].as<uint32_t>();
        for (uint32_t j = 0; j < kMaxDims; j++)
            pa.live_out[j] = B.live[1 - par].as<uint32_t>() + (size_t)std::min(j, d - 1) * B.E_cap;
        pa.mark = B.mark.as<uint32_t>();
        pa.hist_out = B.hist_ptr[lv];
        pa.sizes_out = B.sizes.as<uint32_t>() + (size_t)lv * (4 + kMaxDims);
        pa.final_vals = last ? B.final_vals.as<uint32_t>() : nullptr;
        pa.E_cap = B.E_cap;
        pa.F_cap = B.F_cap;
        pa.level = lv;
        pa.nw = (uint32_t)c0->nw;
        pa.njobs_per_ctx = d;
        pa.nctx = 2;
        pa.grid_waves = grid_waves;
        pa.unit = (uint32_t)c0->nw;
        pa.max_group = expand_max_group(variant);
        pa.tail_split = expand_tail_split(variant) ? 1u : 0u;
        pa.max_wpi = expand_max_wpi(variant);
        pa.zero_partials = (cfg->mode != 0 && !last) ? B.partials.as<uint64_t>() : nullptr;
        pa.ring32 = ring32 && !last ? 1u : 0u;
        pa.zero_count = (uint64_t)C_cap * 4;
        HIP_TRY(c0, launch_prune(pa, c0->stream));
        lv++;
        if (lv % kBatch == 0 || lv == levels) {
            HIP_TRY(c0, hipMemcpyAsync(B.ctl_host.p, B.ctl.p, sizeof(LoopCtl), hipMemcpyDeviceToHost, c0->stream));
            rc = sync(c0);
            if (rc) return rc;
            const LoopCtl* h = B.ctl_host.as<LoopCtl>();
            if (h->abort) {
                // grow, keep what the prune of abort_level reads, resume there
                const uint32_t la = h->abort_level;
                const bool la_last = la + 1 == levels;
                uint32_t nE = 0;
                rc = loop_entry_cap(cs, cfg, B, d, B.E_cap, std::max<uint32_t>(h->need_entries, 1), la, nE);
                if (rc) return rc;
                const uint32_t nF = std::max(B.F_cap, next_pow2(std::max<uint32_t>(h->need_nodes, 1)) * 2);
                const uint32_t la_per = cfg->mode == 0 ? 1 : (la_last ? 16 : 4);
                if (std::getenv("FHH_DEBUG_LOOP"))
                    std::fprintf(stderr, "[fhh loop] abort at level %u (batch end %u): need_entries %u need_nodes %u "
                                 "F %u C %u -> E_cap %u F_cap %u\n", la, lv, h->need_entries, h->need_nodes, h->F,
                                 h->C, nE, nF);
                // the tables of parity la & 1 are rewritten by level la + 1: released first, so the
                // peak while the preserved ones are copied is one old table, not all of them
                for (fhh_ctx* c : cs)
                    for (uint32_t j = 0; j < d; j++) table_release(c->tab[j], la & 1);
                for (fhh_ctx* c : cs)
                    for (uint32_t j = 0; j < d; j++) {
                        // child tables of level la (parity 1 - la&1) hold 2 * n_live(la) entries
                        rc = table_grow(c, c->tab[j], 1 - (la & 1), nE, 2 * (size_t)h->n_live[j]);
                        if (rc) return rc;
                    }
                for (fhh_ctx* c : cs)
                    for (uint32_t j = 0; j < d; j++) {
                        rc = table_grow(c, c->tab[j], la & 1, nE, 0);
                        if (rc) return rc;
                    }
                rc = loop_resize(c0, B, nE, nF, levels, la, true, h->F, h->C, la_per);
                if (rc) return rc;
                const uint32_t zero = 0;
                HIP_TRY(c0, hipMemcpy(B.ctl.p, &zero, 4, hipMemcpyHostToDevice));   // abort = 0
                lv = la;
                prune_only = true;
                (void)per_level_per;
            }
        }
    }
    if (B.bot) {
        // every instance the crawl used was waited for at its upload; lookahead ones still running
        // are abandoned (the destructor stops the workers after their current instance)
        std::lock_guard<std::mutex> lk(B.bot->mu);
        c0->stats.base_ot_ms += B.bot->compute_ms;
        c0->stats.base_ot_stall_ms += B.bot->stall_ms;
        c0->stats.base_ot_instances += B.bot->computed;
    }
    c0->loop_cap_hint = std::max(B.E_cap, B.F_cap);   // the next crawl starts at this size
    pc.mark("loop");
    // ---- readback: sizes, hist, final values -> host-side state of both servers ----
    // every level's hist row is packed on the device (k_gather_hist) and copied in one transfer
    const uint64_t hist_cap = (uint64_t)levels * B.F_cap;
    HIP_TRY(c0, B.hist_rows.ensure((size_t)levels * sizeof(uint32_t*)));
    HIP_TRY(c0, B.hist_packed.ensure(hist_cap * 4));
    HIP_TRY(c0, hipMemcpyAsync(B.hist_rows.p, B.hist_ptr.data(), (size_t)levels * sizeof(uint32_t*),
                               hipMemcpyHostToDevice, c0->stream));
    HIP_TRY(c0, launch_gather_hist(B.sizes.as<uint32_t>(), 4 + kMaxDims, B.hist_rows.as<const uint32_t*>(), levels,
                                   B.hist_packed.as<uint32_t>(), hist_cap, c0->stream));
    // (the engine stream is non-blocking: plain hipMemcpy would not wait for k_gather_hist)
    std::vector<uint32_t> sz((size_t)levels * (4 + kMaxDims));
    HIP_TRY(c0, hipMemcpyAsync(sz.data(), B.sizes.p, sz.size() * 4, hipMemcpyDeviceToHost, c0->stream));
    HIP_TRY(c0, hipStreamSynchronize(c0->stream));
    uint64_t hist_total = 0;
    for (uint32_t lv = 0; lv < levels; lv++) hist_total += sz[(size_t)lv * (4 + kMaxDims) + 1];
    if (hist_total > hist_cap) return c0->fail(FHH_E_STATE, "loop: kept-children lists exceed their capacity");
    std::vector<uint32_t> packed(hist_total);
    if (hist_total) {
        HIP_TRY(c0, hipMemcpyAsync(packed.data(), B.hist_packed.p, hist_total * 4, hipMemcpyDeviceToHost, c0->stream));
        HIP_TRY(c0, hipStreamSynchronize(c0->stream));
    }
    std::vector<std::vector<std::pair<uint32_t, uint32_t>>> hist(levels);
    const uint32_t mask = (1u << d) - 1;
    for (uint32_t lv = 0, off = 0; lv < levels; lv++) {
        const uint32_t nf = sz[(size_t)lv * (4 + kMaxDims) + 1];
        hist[lv].reserve(nf);
        for (uint32_t k = 0; k < nf; k++) hist[lv].emplace_back(packed[off + k] >> d, packed[off + k] & mask);
        off += nf;
    }
    const uint32_t nfin = sz[(size_t)(levels - 1) * (4 + kMaxDims) + 1];
    std::vector<uint32_t> fv((size_t)nfin * 20);
    if (nfin) HIP_TRY(c0, hipMemcpy(fv.data(), B.final_vals.p, fv.size() * 4, hipMemcpyDeviceToHost));
    // frontier before the last crawl: depth levels-1, states in table buffer (levels-1)&1
    const int fpar = (levels - 1) & 1;
    const uint32_t Ffront = levels >= 2 ? sz[(size_t)(levels - 2) * (4 + kMaxDims) + 1] : 1;
    std::vector<uint32_t> fpos((size_t)Ffront * d);
    if (Ffront) HIP_TRY(c0, hipMemcpy(fpos.data(), B.pos[fpar].p, fpos.size() * 4, hipMemcpyDeviceToHost));
    std::vector<std::vector<uint32_t>> flive(d);
    for (uint32_t j = 0; j < d; j++) {
        const uint32_t nl = levels >= 2 ? sz[(size_t)(levels - 2) * (4 + kMaxDims) + 4 + j] : 1;
        flive[j].resize(nl);
        if (nl)
            HIP_TRY(c0, hipMemcpy(flive[j].data(), B.live[fpar].as<uint32_t>() + (size_t)j * B.E_cap, (size_t)nl * 4,
                                  hipMemcpyDeviceToHost));
    }
    for (int s = 0; s < 2; s++) {
        fhh_ctx* c = cs[s];
        c->hist.assign(hist.begin(), hist.begin() + (levels - 1));
        c->last_hist = c->hist;
        c->last_depth = levels;
        c->last_nodes = hist[levels - 1];
        c->last_values.assign(nfin, Limbs10{});
        for (uint32_t k = 0; k < nfin; k++) {
            if (cfg->mode == 0 && s == 1) continue;   // count mode: values on server 0 (host loop convention)
            std::memcpy(c->last_values[k].data(), &fv[(size_t)k * 20 + (cfg->mode == 0 ? 0 : 10 * s)], 40);
        }
        c->frontier.assign(Ffront, Node{});
        for (uint32_t k = 0; k < Ffront; k++)
            for (uint32_t j = 0; j < d; j++) c->frontier[k].pos[j] = fpos[(size_t)k * d + j];
        for (uint32_t j = 0; j < d; j++) {
            c->tab[j].live = flive[j];
            c->tab[j].cur = fpar;
            c->child_buf[j] = 1 - fpar;
        }
        c->level = levels - 1;
        c->pending_C = 0;
        c->phase = Phase::kFrontier;   // after tree_prune_last (collect.rs:931-942)
        for (uint32_t lv = 0; lv < levels; lv++) {
            const uint32_t* row = &sz[(size_t)lv * (4 + kMaxDims)];
            uint64_t live_sum = 0;
            for (uint32_t j = 0; j < d; j++) live_sum += lv == 0 ? 1 : sz[(size_t)(lv - 1) * (4 + kMaxDims) + 4 + j];
            c->stats.aes_blocks += live_sum * 4 * c->n;
            c->stats.ref_evals += (uint64_t)row[0] * c->n * 2 * d;
            c->stats.levels += 1;
        }
    }
    // expand_blocks_timed for c0's timed launches: both servers
    {
        uint64_t blocks = 0;
        for (uint32_t lv = 0; lv < levels; lv++) {
            uint64_t live_sum = 0;
            for (uint32_t j = 0; j < d; j++) live_sum += lv == 0 ? 1 : sz[(size_t)(lv - 1) * (4 + kMaxDims) + 4 + j];
            if (lv % c0->timing_every == 0) blocks += live_sum * 4 * c0->n * 2;
        }
        if (c0->timing) c0->stats.expand_blocks_timed += blocks;
    }
    // optional per-level records
    uint64_t off = 0;
    for (uint32_t lv = 0; lv < levels; lv++) {
        const uint32_t C = sz[(size_t)lv * (4 + kMaxDims)];
        if (cfg->level_children) cfg->level_children[lv] = C;
        if (cfg->level_kept) cfg->level_kept[lv] = sz[(size_t)lv * (4 + kMaxDims) + 1];
        if (record && lv < B.rec_off.size()) {
            const uint64_t* r = B.rec.as<uint64_t>() + B.rec_off[lv];
            const bool lvl_last = lv + 1 == levels;
            for (uint32_t c = 0; c < C && off + c < cfg->counts_capacity; c++) {
                uint64_t v;
                if (cfg->mode == 0) {
                    v = r[c];
                } else if (!lvl_last && ring32) {   // r06: Z_2^32 shares
                    v = (uint32_t)(r[c * 4] - r[c * 4 + 2]);
                } else if (!lvl_last) {
                    v = fe_sub_canon(fe_canon_from_limbs(r[c * 4], r[c * 4 + 1]), fe_canon_from_limbs(r[c * 4 + 2], r[c * 4 + 3]));
                } else {
                    const auto dv = fe255_sub(fe255_reduce(limbs_from_partials(r + (size_t)c * 16)),
                                              fe255_reduce(limbs_from_partials(r + (size_t)c * 16 + 8)));
                    v = (uint64_t)dv[0] | ((uint64_t)dv[1] << 32);
                }
                cfg->counts[off + c] = v;
            }
        }
        off += C;
    }
    if (cfg->probe_n_levels) {
        std::vector<uint32_t> pC(cfg->probe_n_levels);
        HIP_TRY(c0, hipMemcpy(pC.data(), B.probe_C.p, pC.size() * 4, hipMemcpyDeviceToHost));
        const size_t row = (size_t)cfg->probe_n_clients * d * 2;   // states per (server, child)
        const size_t cap = cfg->probe_capacity;
        for (uint32_t k = 0; k < cfg->probe_n_levels; k++) {
            cfg->probe_children[k] = pC[k];
            const size_t nc = std::min<size_t>(std::min<size_t>(pC[k], cap), B.probe_stride[k]);
            if (!nc || !B.probe_seed[k].p) continue;
            for (int s = 0; s < 2; s++) {
                uint8_t* hs = cfg->probe_seeds + (((size_t)k * 2 + s) * cap) * row * 16;
                uint8_t* ht = cfg->probe_ty + (((size_t)k * 2 + s) * cap) * row;
                HIP_TRY(c0, hipMemcpy(hs, B.probe_seed[k].as<uint8_t>() + (size_t)s * B.probe_stride[k] * row * 16,
                                      nc * row * 16, hipMemcpyDeviceToHost));
                HIP_TRY(c0, hipMemcpy(ht, B.probe_ty[k].as<uint8_t>() + (size_t)s * B.probe_stride[k] * row, nc * row,
                                      hipMemcpyDeviceToHost));
            }
        }
    }
    pc.mark("readback");
    return FHH_OK;
}

// ================================================================================================
// C ABI
// ================================================================================================
extern "C" {

const char* fhh_last_error(const fhh_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

int fhh_create(fhh_ctx** out, uint32_t data_len, uint32_t n_dims, int device) {
    if (!out) {
        g_err = "fhh_create: out is NULL";
        return FHH_E_ARG;
    }
    *out = nullptr;
    if (n_dims < 1 || n_dims > FHH_MAX_DIMS) {
        g_err = "fhh_create: n_dims must be in [1, " + std::to_string(FHH_MAX_DIMS) + "]";
        return FHH_E_ARG;
    }
    if (data_len < 1) {
        g_err = "fhh_create: data_len must be >= 1";
        return FHH_E_ARG;
    }
    hipError_t e = hipSetDevice(device);
    if (e != hipSuccess) {
        g_err = std::string("hipSetDevice: ") + hipGetErrorString(e);
        return FHH_E_HIP;
    }
    fhh_ctx* ctx = new fhh_ctx();
    ctx->device = device;
    ctx->L = data_len;
    ctx->d = n_dims;
    ctx->K = 2 * n_dims;
    e = hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking);
    ctx->stream = ctx->own_stream;
    if (e != hipSuccess) {
        g_err = std::string("hipStreamCreate: ") + hipGetErrorString(e);
        delete ctx;
        return FHH_E_HIP;
    }
    ctx->variant = kDefaultVariant;
    ctx->grid = expand_grid(device, ctx->variant);
    if (ctx->work_counter.ensure(kWorkCounterBytes) != hipSuccess ||
        hipMemset(ctx->work_counter.p, 0, kWorkCounterBytes) != hipSuccess) {
        g_err = "work counter allocation failed";
        (void)hipStreamDestroy(ctx->own_stream);
        delete ctx;
        return FHH_E_NOMEM;
    }
    *out = ctx;
    return FHH_OK;
}

void fhh_destroy(fhh_ctx* ctx) {
    if (!ctx) return;
    if (ctx->group) return group_destroy(ctx);
    if (ctx->party) party_destroy(ctx);
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->stream);
    for (auto& pr : ctx->ev_pool) {
        (void)hipEventDestroy(pr.first);
        (void)hipEventDestroy(pr.second);
    }
    if (ctx->side_stream) {
        (void)hipStreamSynchronize(ctx->side_stream);
        (void)hipStreamDestroy(ctx->side_stream);
    }
    for (hipEvent_t e : ctx->side_ev)
        if (e) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(ctx->own_stream);
    for (auto* b : ctx->stage) delete b;
    delete ctx;
}

int fhh_reset(fhh_ctx* ctx) {
    CTX_CHECK(ctx);
    if (ctx->group) return group_reset(ctx);
    int rc = set_device(ctx);
    if (rc) return rc;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ctx->h_key_idx.clear();
    ctx->h_root.clear();
    ctx->h_cws.clear();
    ctx->h_cwb.clear();
    ctx->h_n = 0;
    ctx->dev_keys = false;
    ctx->n = ctx->npad = ctx->nw = 0;
    ctx->phase = Phase::kNoInit;
    ctx->frontier.clear();
    ctx->hist.clear();
    ctx->last_nodes.clear();
    ctx->last_values.clear();
    ctx->last_hist.clear();
    ctx->pending_C = 0;
    ctx->level = 0;
    for (auto& T : ctx->tab) T.live.clear();
    return FHH_OK;
}

int fhh_set_client_base(fhh_ctx* ctx, uint64_t client_base) {
    CTX_CHECK(ctx);
    if (ctx->group) return group_set_client_base(ctx, client_base);
    ctx->client_base = client_base;
    return FHH_OK;
}

int fhh_add_keys(fhh_ctx* ctx, uint64_t n, const uint8_t* key_idx, const uint8_t* root_seed, const uint8_t* cw_seed,
                 const uint8_t* cw_bits) {
    CTX_CHECK(ctx);
    if (n == 0) return FHH_OK;
    if (!key_idx || !root_seed || !cw_seed || !cw_bits) return ctx->fail(FHH_E_ARG, "add_keys: NULL buffer");
    if (ctx->dev_keys) return ctx->fail(FHH_E_STATE, "add_keys after keys were placed on the device");
    const size_t K = ctx->K, L = ctx->L;
    ctx->h_key_idx.insert(ctx->h_key_idx.end(), key_idx, key_idx + n * K);
    ctx->h_root.insert(ctx->h_root.end(), root_seed, root_seed + n * K * 16);
    ctx->h_cws.insert(ctx->h_cws.end(), cw_seed, cw_seed + n * K * L * 16);
    ctx->h_cwb.insert(ctx->h_cwb.end(), cw_bits, cw_bits + n * K * L);
    ctx->h_n += n;
    return FHH_OK;
}

int fhh_gen_keys_pair(fhh_ctx* c0, fhh_ctx* c1, uint64_t n, const uint8_t* left_bits, const uint8_t* right_bits,
                      const uint8_t* root_seeds) {
    if (!c0 || !c1) {
        g_err = "null fhh_ctx";
        return FHH_E_ARG;
    }
    if (c0->group || c1->group) return group_gen_keys_pair(c0, c1, n, left_bits, right_bits, root_seeds);
    if (c0->device != c1->device || c0->d != c1->d || c0->L != c1->L)
        return c0->fail(FHH_E_ARG, "gen_keys_pair: ctxs differ in device/d/L");
    if (c0->dev_keys || c1->dev_keys || c0->h_n || c1->h_n)
        return c0->fail(FHH_E_STATE, "gen_keys_pair: ctxs must be empty");
    if (!left_bits || !right_bits || !root_seeds) return c0->fail(FHH_E_ARG, "gen_keys_pair: NULL buffer");
    int rc = set_device(c0);
    if (rc) return rc;
    rc = alloc_keys(c0, n);
    if (rc) return rc;
    rc = alloc_keys(c1, n);
    if (rc) return rc;
    const size_t d = c0->d, L = c0->L;
    DevBuf lb, rb, rs;
    HIP_TRY(c0, lb.ensure(n * d * L));
    HIP_TRY(c0, rb.ensure(n * d * L));
    HIP_TRY(c0, rs.ensure(n * d * 64));
    HIP_TRY(c0, hipMemcpyAsync(lb.p, left_bits, n * d * L, hipMemcpyHostToDevice, c0->stream));
    HIP_TRY(c0, hipMemcpyAsync(rb.p, right_bits, n * d * L, hipMemcpyHostToDevice, c0->stream));
    HIP_TRY(c0, hipMemcpyAsync(rs.p, root_seeds, n * d * 64, hipMemcpyHostToDevice, c0->stream));
    KeygenArgs a{};
    a.left_bits = lb.as<uint8_t>();
    a.right_bits = rb.as<uint8_t>();
    a.root_seeds = rs.as<uint8_t>();
    fhh_ctx* cs[2] = {c0, c1};
    for (int b = 0; b < 2; b++) {
        a.cw_seed[b] = cs[b]->cw_seed.as<uint4>();
        a.cw_bits[b] = cs[b]->cw_bits.as<uint64_t>();
        a.root[b] = cs[b]->root_seed.as<uint4>();
        a.key_idx[b] = cs[b]->key_idx.as<uint64_t>();
    }
    a.n = n;
    a.d = (uint32_t)d;
    a.L = (uint32_t)L;
    a.K = c0->K;
    a.npad = (uint32_t)c0->npad;
    a.nw = (uint32_t)c0->nw;
    hipEvent_t e0, e1;
    HIP_TRY(c0, hipEventCreate(&e0));
    HIP_TRY(c0, hipEventCreate(&e1));
    HIP_TRY(c0, hipEventRecord(e0, c0->stream));
    HIP_TRY(c0, launch_keygen(a, c0->stream));
    HIP_TRY(c0, hipEventRecord(e1, c0->stream));
    rc = sync(c0);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc) return rc;
    c0->stats.keygen_ms += ms;
    c0->dev_keys = c1->dev_keys = true;
    return FHH_OK;
}

int fhh_num_clients(const fhh_ctx* ctx, uint64_t* n) {
    CTX_CHECK(ctx);
    if (ctx->group) return group_num_clients(ctx, n);
    if (n) *n = ctx->dev_keys ? ctx->n : ctx->h_n;
    return FHH_OK;
}

int fhh_export_keys(fhh_ctx* ctx, uint8_t* key_idx, uint8_t* root_seed, uint8_t* cw_seed, uint8_t* cw_bits) {
    CTX_CHECK(ctx);
    if (ctx->group) return group_export_keys(ctx, key_idx, root_seed, cw_seed, cw_bits);
    int rc = set_device(ctx);
    if (rc) return rc;
    if (!ctx->dev_keys) {
        const size_t n = ctx->h_n;
        if (key_idx) std::memcpy(key_idx, ctx->h_key_idx.data(), ctx->h_key_idx.size());
        if (root_seed) std::memcpy(root_seed, ctx->h_root.data(), ctx->h_root.size());
        if (cw_seed) std::memcpy(cw_seed, ctx->h_cws.data(), ctx->h_cws.size());
        if (cw_bits) std::memcpy(cw_bits, ctx->h_cwb.data(), ctx->h_cwb.size());
        (void)n;
        return FHH_OK;
    }
    const size_t n = ctx->n, K = ctx->K, L = ctx->L, npad = ctx->npad, nw = ctx->nw;
    std::vector<uint8_t> cws(L * K * npad * 16), roots(K * npad * 16);
    std::vector<uint64_t> cwb(L * K * 4 * nw), kidx(K * nw);
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));   // uploads / keygen are async
    HIP_TRY(ctx, hipMemcpy(cws.data(), ctx->cw_seed.p, cws.size(), hipMemcpyDeviceToHost));
    HIP_TRY(ctx, hipMemcpy(roots.data(), ctx->root_seed.p, roots.size(), hipMemcpyDeviceToHost));
    HIP_TRY(ctx, hipMemcpy(cwb.data(), ctx->cw_bits.p, cwb.size() * 8, hipMemcpyDeviceToHost));
    HIP_TRY(ctx, hipMemcpy(kidx.data(), ctx->key_idx.p, kidx.size() * 8, hipMemcpyDeviceToHost));
    for (size_t c = 0; c < n; c++)
        for (size_t kk = 0; kk < K; kk++) {
            const size_t w = c / 64, bit = c % 64;
            if (key_idx) key_idx[c * K + kk] = (uint8_t)((kidx[kk * nw + w] >> bit) & 1);
            if (root_seed) std::memcpy(root_seed + (c * K + kk) * 16, &roots[(kk * npad + c) * 16], 16);
            for (size_t l = 0; l < L; l++) {
                const size_t row = l * K + kk;
                if (cw_seed) std::memcpy(cw_seed + ((c * K + kk) * L + l) * 16, &cws[(row * npad + c) * 16], 16);
                if (cw_bits) {
                    uint8_t nib = 0;
                    for (int b = 0; b < 4; b++) nib |= (uint8_t)(((cwb[(row * 4 + b) * nw + w] >> bit) & 1) << b);
                    cw_bits[(c * K + kk) * L + l] = nib;
                }
            }
        }
    return FHH_OK;
}

int fhh_add_keys_bincode(fhh_ctx* ctx, const uint8_t* req, uint64_t len) {
    CTX_CHECK(ctx);
    if (ctx->group) return group_add_keys_bincode(ctx, req, len);
    int rc = set_device(ctx);
    if (rc) return rc;
    if (!req || len < 8) return ctx->fail(FHH_E_ARG, "add_keys_bincode: buffer shorter than the u64 length");
    if (ctx->dev_keys || ctx->h_n) return ctx->fail(FHH_E_STATE, "add_keys_bincode: ctx already holds keys");
    uint64_t n = 0;
    for (int i = 0; i < 8; i++) n |= (uint64_t)req[i] << (8 * i);
    const uint64_t KB = 25 + 20ull * ctx->L, R = 8 + (uint64_t)ctx->K * KB;
    if (n == 0) return ctx->fail(FHH_E_ARG, "add_keys_bincode: no clients");
    if (n > (len - 8) / R || 8 + n * R != len)
        return ctx->fail(FHH_E_ARG, "add_keys_bincode: length does not match n clients x n_dims x data_len");
    return add_keys_bincode_records(ctx, n, req + 8);
}

int fhh_tree_init(fhh_ctx* ctx) {
    CTX_CHECK(ctx);
    if (ctx->group) return group_tree_init(ctx);
    int rc = set_device(ctx);
    if (rc) return rc;
    rc = upload_staged_keys(ctx);
    if (rc) return rc;
    if (!ctx->dev_keys || ctx->n == 0) return ctx->fail(FHH_E_STATE, "tree_init with no keys (collect.rs:83)");
    for (uint32_t j = 0; j < ctx->d; j++) {
        DimTable& T = ctx->tab[j];
        T.cur = 0;
        rc = table_ensure(ctx, T, 0, 1);
        if (rc) return rc;
        HIP_TRY(ctx, launch_init_tables(ctx->root_seed.as<uint4>(), ctx->key_idx.as<uint64_t>(), j, ctx->K,
                                        (uint32_t)ctx->npad, (uint32_t)ctx->nw, T.seed[0].as<uint4>(),
                                        T.t[0].as<uint64_t>(), T.y[0].as<uint64_t>(), ctx->stream));
        T.live.assign(1, 0);
    }
    ctx->frontier.assign(1, Node{});
    ctx->hist.clear();
    ctx->last_nodes.clear();
    ctx->last_values.clear();
    ctx->last_hist.clear();
    ctx->level = 0;
    ctx->pending_C = 0;
    ctx->phase = Phase::kFrontier;
    return sync(ctx);
}

int fhh_tree_crawl(fhh_ctx* ctx, uint64_t* n_children, uint64_t* share_planes) {
    CTX_CHECK(ctx);
    if (ctx->group) return group_tree_crawl(ctx, false, n_children, share_planes);
    int rc = set_device(ctx);
    if (rc) return rc;
    return crawl_level(ctx, false, n_children, share_planes, ctx->nw, 0);
}

int fhh_tree_crawl_last(fhh_ctx* ctx, uint64_t* n_children, uint64_t* share_planes) {
    CTX_CHECK(ctx);
    if (ctx->group) return group_tree_crawl(ctx, true, n_children, share_planes);
    int rc = set_device(ctx);
    if (rc) return rc;
    return crawl_level(ctx, true, n_children, share_planes, ctx->nw, 0);
}

// node sums of one ctx (single GPU): partials on the device, one copy back, host finish
static int node_sums_single(fhh_ctx* ctx, const void* vals, bool host, uint64_t ld, uint32_t fmt, void* out_a,
                            void* out_b) {
    int rc = set_device(ctx);
    if (rc) return rc;
    uint64_t* part = nullptr;
    rc = node_partials(ctx, vals, fmt, ld, 0, host, &part);
    if (rc) return rc;
    const uint64_t per = fmt_is_fe255(fmt) ? 8 : 2;
    std::vector<uint64_t> h(ctx->pending_C * per);
    if (!h.empty()) HIP_TRY(ctx, hipMemcpyAsync(h.data(), part, h.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    rc = sync(ctx);
    if (rc) return rc;
    return node_sums_finish(ctx, h.data(), fmt, out_a, out_b);
}

int fhh_node_sums_fe(fhh_ctx* ctx, const uint64_t* vals, uint64_t* sums) {
    CTX_CHECK(ctx);
    if (!sums) return ctx->fail(FHH_E_ARG, "node_sums_fe: NULL sums");
    if (ctx->group) {
        const void* v[1] = {vals};
        return group_node_sums(ctx, v, true, 0, FHH_VALS_FE_U64, sums, nullptr);
    }
    return node_sums_single(ctx, vals, true, ctx->n, FHH_VALS_FE_U64, sums, nullptr);
}

int fhh_node_sums_fe255(fhh_ctx* ctx, const uint32_t* vals, uint32_t* sums_unreduced, uint32_t* sums_canonical) {
    CTX_CHECK(ctx);
    if (ctx->group) {
        const void* v[1] = {vals};
        return group_node_sums(ctx, v, true, 0, FHH_VALS_FE255_LIMBS, sums_unreduced, sums_canonical);
    }
    return node_sums_single(ctx, vals, true, ctx->n, FHH_VALS_FE255_LIMBS, sums_unreduced, sums_canonical);
}

int fhh_node_sums_fe_device(fhh_ctx* ctx, const void* const* vals_dev, uint64_t ld, uint32_t format, uint64_t* sums) {
    CTX_CHECK(ctx);
    if (format != FHH_VALS_FE_U64 && format != FHH_VALS_FE_BLOCK)
        return ctx->fail(FHH_E_ARG, "node_sums_fe_device: format must be FHH_VALS_FE_U64 or FHH_VALS_FE_BLOCK");
    if (!vals_dev || !sums) return ctx->fail(FHH_E_ARG, "node_sums_fe_device: NULL vals_dev / sums");
    if (ctx->group) return group_node_sums(ctx, vals_dev, false, ld, format, sums, nullptr);
    return node_sums_single(ctx, vals_dev[0], false, ld ? ld : ctx->n, format, sums, nullptr);
}

int fhh_node_sums_fe255_device(fhh_ctx* ctx, const void* const* vals_dev, uint64_t ld, uint32_t format,
                               uint32_t* sums_unreduced, uint32_t* sums_canonical) {
    CTX_CHECK(ctx);
    if (format != FHH_VALS_FE255_LIMBS && format != FHH_VALS_FE255_BLOCKPAIR)
        return ctx->fail(FHH_E_ARG, "node_sums_fe255_device: format must be FHH_VALS_FE255_LIMBS or _BLOCKPAIR");
    if (!vals_dev) return ctx->fail(FHH_E_ARG, "node_sums_fe255_device: NULL vals_dev");
    if (ctx->group) return group_node_sums(ctx, vals_dev, false, ld, format, sums_unreduced, sums_canonical);
    return node_sums_single(ctx, vals_dev[0], false, ld ? ld : ctx->n, format, sums_unreduced, sums_canonical);
}

int fhh_tree_prune(fhh_ctx* ctx, const uint8_t* keep, uint64_t n) {
    CTX_CHECK(ctx);
    if (n && !keep) return ctx->fail(FHH_E_ARG, "tree_prune: NULL keep");
    if (ctx->group) return group_tree_prune(ctx, keep, n, false);
    return prune_impl(ctx, keep, n);
}

int fhh_tree_prune_last(fhh_ctx* ctx, const uint8_t* keep, uint64_t n) {
    CTX_CHECK(ctx);
    if (n && !keep) return ctx->fail(FHH_E_ARG, "tree_prune_last: NULL keep");
    if (ctx->group) return group_tree_prune(ctx, keep, n, true);
    if (ctx->phase != Phase::kPendingLast && ctx->last_nodes.empty() && n != 0)
        return ctx->fail(FHH_E_STATE, "tree_prune_last without tree_crawl_last");
    if (n != ctx->last_nodes.size())
        return ctx->fail(FHH_E_ARG, "tree_prune_last: keep.len() != frontier_last.len() (collect.rs:932)");
    std::vector<std::pair<uint32_t, uint32_t>> nodes;
    std::vector<Limbs10> vals;
    for (uint64_t k = 0; k < n; k++)
        if (keep[k]) {
            nodes.push_back(ctx->last_nodes[k]);
            vals.push_back(ctx->last_values[k]);
        }
    ctx->last_nodes = std::move(nodes);
    ctx->last_values = std::move(vals);
    if (ctx->phase == Phase::kPendingLast) ctx->phase = Phase::kFrontier;   // frontier unchanged (collect.rs:909-914)
    ctx->pending_C = 0;
    return FHH_OK;
}

int fhh_frontier_size(const fhh_ctx* ctx, uint64_t* n_frontier, uint64_t* n_frontier_last) {
    CTX_CHECK(ctx);
    if (ctx->group) {
        if (!group_lead(ctx)) {
            if (n_frontier) *n_frontier = 0;
            if (n_frontier_last) *n_frontier_last = 0;
            return FHH_OK;
        }
        return fhh_frontier_size(group_lead(ctx), n_frontier, n_frontier_last);
    }
    if (n_frontier) *n_frontier = ctx->phase == Phase::kPending ? ctx->pending_C : ctx->frontier.size();
    if (n_frontier_last) *n_frontier_last = ctx->last_nodes.size();
    return FHH_OK;
}

int fhh_final_shares(fhh_ctx* ctx, uint64_t* n_final, uint32_t* levels, uint8_t* paths, uint32_t* values) {
    CTX_CHECK(ctx);
    if (ctx->group) {
        fhh_ctx* lead = group_lead(ctx);
        if (!lead) return ctx->fail(FHH_E_STATE, "final_shares: no keys placed on the shards");
        const int rc = fhh_final_shares(lead, n_final, levels, paths, values);
        if (rc) ctx->fail(rc, lead->err);
        return rc;
    }
    const uint64_t F = ctx->last_nodes.size();
    if (n_final) *n_final = F;
    if (levels) *levels = ctx->last_depth;
    if (F == 0) return FHH_OK;
    const uint32_t len = ctx->last_depth;
    for (uint64_t k = 0; k < F; k++) {
        if (paths) node_path(ctx->last_hist, len - 1, ctx->last_nodes[k].first, ctx->last_nodes[k].second, ctx->d,
                             paths + k * ctx->d * len);
        if (values) std::memcpy(values + k * 10, ctx->last_values[k].data(), 40);
    }
    return FHH_OK;
}

int fhh_export_states(fhh_ctx* ctx, uint64_t* n_nodes, uint8_t* seeds, uint8_t* t, uint8_t* y) {
    CTX_CHECK(ctx);
    if (ctx->group) return group_export_states(ctx, n_nodes, seeds, t, y);
    int rc = set_device(ctx);
    if (rc) return rc;
    if (ctx->phase == Phase::kNoInit) return ctx->fail(FHH_E_STATE, "export_states before tree_init");
    const bool pending = ctx->phase == Phase::kPending || ctx->phase == Phase::kPendingLast;
    const uint64_t F = pending ? ctx->pending_C : ctx->frontier.size();
    if (n_nodes) *n_nodes = F;
    if (!seeds && !t && !y) return FHH_OK;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const size_t n = ctx->n, npad = ctx->npad, nw = ctx->nw, d = ctx->d;
    for (uint32_t j = 0; j < d; j++) {
        DimTable& T = ctx->tab[j];
        const int buf = pending ? ctx->child_buf[j] : T.cur;
        const size_t E = pending ? 2 * ctx->frontier.size() : T.live.size();
        (void)E;
        // copy the whole buffer (tests only)
        std::vector<uint8_t> hs(T.cap[buf] * 2 * npad * 16);
        std::vector<uint64_t> ht(T.cap[buf] * 2 * nw), hy(T.cap[buf] * 2 * nw);
        HIP_TRY(ctx, hipMemcpy(hs.data(), T.seed[buf].p, hs.size(), hipMemcpyDeviceToHost));
        HIP_TRY(ctx, hipMemcpy(ht.data(), T.t[buf].p, ht.size() * 8, hipMemcpyDeviceToHost));
        HIP_TRY(ctx, hipMemcpy(hy.data(), T.y[buf].p, hy.size() * 8, hipMemcpyDeviceToHost));
        for (uint64_t node = 0; node < F; node++) {
            uint32_t e;
            if (pending) {
                const uint64_t p = node >> d;
                const uint32_t i = (uint32_t)(node & ((1u << d) - 1));
                e = 2 * ctx->frontier[p].pos[j] + ((i >> j) & 1);
            } else {
                e = T.live[ctx->frontier[node].pos[j]];
            }
            for (size_t c = 0; c < n; c++)
                for (int s = 0; s < 2; s++) {
                    const size_t o = ((node * n + c) * d + j) * 2 + s;
                    if (seeds) std::memcpy(seeds + o * 16, &hs[(((size_t)e * 2 + s) * npad + c) * 16], 16);
                    if (t) t[o] = (uint8_t)((ht[((size_t)e * 2 + s) * nw + c / 64] >> (c % 64)) & 1);
                    if (y) y[o] = (uint8_t)((hy[((size_t)e * 2 + s) * nw + c / 64] >> (c % 64)) & 1);
                }
        }
    }
    return FHH_OK;
}

int fhh_keep_values(uint64_t threshold, const uint64_t* vals0, const uint64_t* vals1, uint64_t n, uint8_t* keep) {
    if (n && (!vals0 || !vals1 || !keep)) {
        g_err = "keep_values: NULL buffer";
        return FHH_E_ARG;
    }
    const uint64_t t = fe_canon(threshold);
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t a = fe_canon(vals0[i]), b = fe_canon(vals1[i]);
        const uint64_t v = a >= b ? a - b : a + (kFeP - b);
        keep[i] = v >= t;
    }
    return FHH_OK;
}

int fhh_keep_values_last(uint32_t threshold, const uint32_t* vals0, const uint32_t* vals1, uint64_t n, uint8_t* keep) {
    if (n && (!vals0 || !vals1 || !keep)) {
        g_err = "keep_values_last: NULL buffer";
        return FHH_E_ARG;
    }
    for (uint64_t i = 0; i < n; i++) {
        Limbs10 a{}, b{};
        std::memcpy(a.data(), vals0 + i * 10, 40);
        std::memcpy(b.data(), vals1 + i * 10, 40);
        auto v = fe255_sub(fe255_reduce(a), fe255_reduce(b));   // v0.reduce(); v1.reduce(); v0 - v1
        keep[i] = fe255_ge_u32(v, threshold);
    }
    return FHH_OK;
}

int fhh_final_values(const uint32_t* vals0, const uint32_t* vals1, uint64_t n, uint32_t* out) {
    if (n && (!vals0 || !vals1 || !out)) {
        g_err = "final_values: NULL buffer";
        return FHH_E_ARG;
    }
    for (uint64_t i = 0; i < n; i++) {
        Limbs10 a{}, b{};
        std::memcpy(a.data(), vals0 + i * 10, 40);
        std::memcpy(b.data(), vals1 + i * 10, 40);
        auto v = fe255_sub(fe255_reduce(a), fe255_reduce(b));
        std::memcpy(out + i * 8, v.data(), 32);
    }
    return FHH_OK;
}

int fhh_sim_eq_count(fhh_ctx* c0, fhh_ctx* c1, uint64_t* counts) {
    if (!c0 || !c1) {
        g_err = "null fhh_ctx";
        return FHH_E_ARG;
    }
    if (c0->group || c1->group) return c0->fail(FHH_E_ARG, "sim_eq_count: per-shard harness entry (use fhh_sim_crawl on a multi-device ctx)");
    int rc = set_device(c0);
    if (rc) return rc;
    if (!counts) return c0->fail(FHH_E_ARG, "sim_eq_count: NULL counts");
    return sim_eq_count_impl(c0, c1, nullptr, counts);
}

int fhh_sim_ot_sums(fhh_ctx* c0, fhh_ctx* c1, uint64_t prf_seed, void* sums0, void* sums1) {
    if (!c0 || !c1) {
        g_err = "null fhh_ctx";
        return FHH_E_ARG;
    }
    if (c0->group || c1->group) return c0->fail(FHH_E_ARG, "sim_ot_sums: per-shard harness entry (use fhh_sim_crawl on a multi-device ctx)");
    int rc = set_device(c0);
    if (rc) return rc;
    if (!sums0 || !sums1) return c0->fail(FHH_E_ARG, "sim_ot_sums: NULL buffer");
    return sim_ot_sums_impl(c0, c1, nullptr, prf_seed, sums0, sums1);
}

int fhh_sim_crawl(fhh_ctx* c0, fhh_ctx* c1, const fhh_sim_config* cfg) {
    if (!c0 || !c1 || !cfg) {
        g_err = "sim_crawl: NULL argument";
        return FHH_E_ARG;
    }
    if (c0->group || c1->group) return group_sim_crawl(c0, c1, cfg);
    int rc = set_device(c0);
    if (rc) return rc;
    const uint32_t levels = cfg->levels ? cfg->levels : c0->L;
    if (levels > c0->L) return c0->fail(FHH_E_ARG, "sim_crawl: levels > data_len");
    if (cfg->mode > 1) return c0->fail(FHH_E_ARG, "sim_crawl: bad mode");
    if (cfg->gc > 3)
        return c0->fail(FHH_E_ARG, "sim_crawl: gc must be 0, 1 (ideal OT), 2 (OT extension) or 3 (2 with the circuit at every level)");
    if (cfg->gc && (cfg->mode != 1 || cfg->host_loop))
        return c0->fail(FHH_E_ARG, "sim_crawl: gc needs mode 1 (OT share values) and the device loop");
    if (cfg->gc && 2 * c0->d > (uint32_t)kGcMaxBits) return c0->fail(FHH_E_ARG, "sim_crawl: gc supports d <= 4");
    if (cfg->ot_ss_k > 1 && cfg->ot_ss_k != 2 && cfg->ot_ss_k != 4)
        return c0->fail(FHH_E_ARG, "sim_crawl: ot_ss_k must be 0 / 1 (IKNP), 2 or 4 (SoftSpoken)");
    if (cfg->probe_n_levels && cfg->host_loop)
        return c0->fail(FHH_E_ARG, "sim_crawl: the probe instruments the device loop (host_loop = 0)");
    if (c0->device != c1->device) return c0->fail(FHH_E_ARG, "sim_crawl: ctxs on different devices");
    if (c0->d != c1->d || c0->L != c1->L) return c0->fail(FHH_E_ARG, "sim_crawl: ctx shapes differ");
    // leader.rs:193-194 and 245-246
    const uint64_t thr = std::max<uint64_t>(1, (uint64_t)(cfg->threshold * (double)cfg->nclients_total));
    // `as u32` in Rust saturates (leader.rs:245): clamp before narrowing
    const double thr_last_f = cfg->threshold * (double)cfg->nclients_total;
    const uint32_t thr_last =
        std::max<uint32_t>(1, thr_last_f >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)(uint64_t)thr_last_f);
    if (!cfg->host_loop) {
        PhaseClock total;
        rc = sim_crawl_device_loop(c0, c1, cfg, levels, thr, thr_last);   // incl. buffer teardown
        total.mark("total");
        return rc;
    }
    rc = fhh_tree_init(c0);
    if (rc) return rc;
    rc = fhh_tree_init(c1);
    if (rc) return rc;
    PairScope pair(c0, c1);
    uint64_t counts_off = 0;
    std::vector<uint64_t> vals, s0, s1;
    std::vector<uint32_t> l0, l1;
    std::vector<uint8_t> keep;
    for (uint32_t lv = 0; lv < levels; lv++) {
        const bool last = lv + 1 == levels;
        rc = crawl_pair(c0, c1, last);
        if (rc) return rc;
        const uint64_t C = c0->pending_C;
        keep.assign(C, 0);
        if (cfg->mode == 0) {
            vals.resize(C);
            rc = sim_eq_count_impl(c0, c1, cfg, vals.data());
            if (rc) return rc;
            for (uint64_t c = 0; c < C; c++) keep[c] = vals[c] >= (last ? (uint64_t)thr_last : thr);
            if (cfg->counts && counts_off + C <= cfg->counts_capacity)
                std::memcpy(cfg->counts + counts_off, vals.data(), C * 8);
            counts_off += C;
            if (last) {
                for (uint64_t c = 0; c < C; c++) {
                    Limbs10 v{};
                    v[0] = (uint32_t)vals[c];
                    v[1] = (uint32_t)(vals[c] >> 32);
                    c0->last_values[c] = v;
                    c1->last_values[c] = Limbs10{};
                }
            }
        } else if (!last) {
            s0.resize(C);
            s1.resize(C);
            rc = sim_ot_sums_impl(c0, c1, cfg, cfg->prf_seed, s0.data(), s1.data());
            if (rc) return rc;
            rc = fhh_keep_values(thr, s0.data(), s1.data(), C, keep.data());
            if (rc) return rc;
            if (cfg->counts && counts_off + C <= cfg->counts_capacity)
                for (uint64_t c = 0; c < C; c++)
                    cfg->counts[counts_off + c] = s0[c] >= s1[c] ? s0[c] - s1[c] : s0[c] + (kFeP - s1[c]);
            counts_off += C;
        } else {
            l0.resize(C * 10);
            l1.resize(C * 10);
            rc = sim_ot_sums_impl(c0, c1, cfg, cfg->prf_seed, l0.data(), l1.data());
            if (rc) return rc;
            rc = fhh_keep_values_last(thr_last, l0.data(), l1.data(), C, keep.data());
            if (rc) return rc;
            if (cfg->counts && counts_off + C <= cfg->counts_capacity) {
                std::vector<uint32_t> fv(C * 8);
                fhh_final_values(l0.data(), l1.data(), C, fv.data());
                for (uint64_t c = 0; c < C; c++)
                    cfg->counts[counts_off + c] = (uint64_t)fv[c * 8] | ((uint64_t)fv[c * 8 + 1] << 32);
            }
            counts_off += C;
        }
        uint64_t kept = 0;
        for (uint64_t c = 0; c < C; c++) kept += keep[c];
        if (cfg->level_children) cfg->level_children[lv] = C;
        if (cfg->level_kept) cfg->level_kept[lv] = kept;
        if (last) {
            rc = fhh_tree_prune_last(c0, keep.data(), C);
            if (rc) return rc;
            rc = fhh_tree_prune_last(c1, keep.data(), C);
            if (rc) return rc;
        } else {
            rc = prune_impl(c0, keep.data(), C);
            if (rc) return rc;
            rc = prune_impl(c1, keep.data(), C);
            if (rc) return rc;
        }
    }
    return FHH_OK;
}

int fhh_set_variant(fhh_ctx* ctx, int variant) {
    CTX_CHECK(ctx);
    if (ctx->group) return group_each(ctx, fhh_set_variant, variant);
    if (variant < 0 || variant >= expand_variant_count()) return ctx->fail(FHH_E_ARG, "set_variant: no such variant");
    if (!expand_threads(variant))
        return ctx->fail(FHH_E_ARG, "set_variant: variant " + std::to_string(variant) +
                                        " is not in this build (it holds 52 and 33; the r01-r03 A/B forms were removed)");
    ctx->variant = variant;
    ctx->grid = expand_grid(ctx->device, variant);
    return FHH_OK;
}

int fhh_variant_info(int variant, char* name, size_t cap, int* threads, int* grid_per_device) {
    if (variant < 0 || variant >= expand_variant_count() || !expand_threads(variant)) {
        g_err = "variant_info: no such variant in this build";
        return FHH_E_ARG;
    }
    if (name && cap) std::snprintf(name, cap, "%s", expand_variant_name(variant));
    if (threads) *threads = expand_threads(variant);
    if (grid_per_device) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        *grid_per_device = expand_grid(dev, variant);
    }
    return FHH_OK;
}

int fhh_get_stats(const fhh_ctx* ctx, fhh_stats* out) {
    CTX_CHECK(ctx);
    if (ctx->group) return group_get_stats(ctx, out);
    if (out) *out = ctx->stats;
    return FHH_OK;
}

int fhh_reset_stats(fhh_ctx* ctx) {
    CTX_CHECK(ctx);
    if (ctx->group) return group_each(ctx, [](fhh_ctx* c, int) { return fhh_reset_stats(c); }, 0);
    ctx->stats = fhh_stats{};
    return FHH_OK;
}

int fhh_set_timing(fhh_ctx* ctx, int enabled) {
    CTX_CHECK(ctx);
    if (ctx->group) return group_each(ctx, fhh_set_timing, enabled);
    if (enabled < 0) return ctx->fail(FHH_E_ARG, "set_timing: enabled must be >= 0");
    ctx->timing = enabled != 0;
    ctx->timing_every = enabled > 1 ? (uint32_t)enabled : 1;
    return FHH_OK;
}

int fhh_memcpy_device(int device, void* dst_dev, const void* src_dev, uint64_t bytes) {
    hipError_t e = hipSetDevice(device);
    // a device-to-device hipMemcpy may return before the copy lands; the engine's non-blocking
    // streams do not wait for the null stream, so finish it here
    if (e == hipSuccess && bytes) e = hipMemcpyAsync(dst_dev, src_dev, bytes, hipMemcpyDeviceToDevice, nullptr);
    if (e == hipSuccess && bytes) e = hipStreamSynchronize(nullptr);
    if (e != hipSuccess) {
        g_err = std::string("memcpy_device: ") + hipGetErrorString(e);
        return FHH_E_HIP;
    }
    return FHH_OK;
}

int fhh_device_info(int device, char* arch_name, size_t cap, int* num_cus) {
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, device);
    if (e != hipSuccess) {
        g_err = std::string("hipGetDeviceProperties: ") + hipGetErrorString(e);
        return FHH_E_HIP;
    }
    if (arch_name && cap) {
        std::snprintf(arch_name, cap, "%s", prop.gcnArchName);
    }
    if (num_cus) *num_cus = prop.multiProcessorCount;
    return FHH_OK;
}

}  // extern "C"

// ---- sketch + Beaver verification (row a9) ------------------------------------------------
namespace {
uint64_t fe_canon_u64(uint64_t v) {   // any FE val -> value() (fastfield.rs:86-107,147-152)
    const uint64_t mask = (1ull << 62) - 1;
    uint64_t r = (v & mask) + (v >> 62) + ((v >> 62) << 30);
    while (r >= kFeP) r -= kFeP;
    return r;
}
}  // namespace

int fhh_sketch_at_fe(fhh_ctx* ctx, uint64_t n_keys, uint32_t n_nodes, const uint8_t* seeds, const uint64_t* x,
                     const uint64_t* kx, uint64_t* sketch6) {
    CTX_CHECK(ctx);
    int rc = set_device(ctx);
    if (rc) return rc;
    if (n_keys == 0) return FHH_OK;
    if (!seeds || !sketch6 || (n_nodes && (!x || !kx))) return ctx->fail(FHH_E_ARG, "sketch_at_fe: NULL buffer");
    const size_t vb = (size_t)n_keys * n_nodes * 8;
    DevBuf ds, dx, dkx, dout;
    HIP_TRY(ctx, ds.ensure(n_keys * 16));
    HIP_TRY(ctx, dx.ensure(vb));
    HIP_TRY(ctx, dkx.ensure(vb));
    HIP_TRY(ctx, dout.ensure(n_keys * 48));
    HIP_TRY(ctx, hipMemcpyAsync(ds.p, seeds, n_keys * 16, hipMemcpyHostToDevice, ctx->stream));
    if (vb) {
        HIP_TRY(ctx, hipMemcpyAsync(dx.p, x, vb, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(dkx.p, kx, vb, hipMemcpyHostToDevice, ctx->stream));
    }
    SketchArgs a{};
    a.seeds = ds.as<uint8_t>();
    a.x = dx.as<uint64_t>();
    a.kx = dkx.as<uint64_t>();
    a.out = dout.as<uint64_t>();
    a.n_keys = n_keys;
    a.n_nodes = n_nodes;
    HIP_TRY(ctx, launch_sketch_fe(a, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(sketch6, dout.p, n_keys * 48, hipMemcpyDeviceToHost, ctx->stream));
    return sync(ctx);
}

static int mul_fe_host(fhh_ctx* ctx, uint32_t mode, int server_idx, uint64_t n, const uint64_t* sketch6,
                       const uint64_t* mac, const uint64_t* mac2, const uint64_t* triples9, const uint64_t* cor6,
                       uint64_t* out) {
    CTX_CHECK(ctx);
    int rc = set_device(ctx);
    if (rc) return rc;
    if (n == 0) return FHH_OK;
    if (!sketch6 || !mac || !mac2 || !triples9 || !out || (mode == 1 && !cor6))
        return ctx->fail(FHH_E_ARG, "mul_fe: NULL buffer");
    DevBuf dsk, dm, dm2, dt, dc, dout;
    const size_t out_words = mode == 0 ? 6 : 1;
    HIP_TRY(ctx, dsk.ensure(n * 48));
    HIP_TRY(ctx, dm.ensure(n * 8));
    HIP_TRY(ctx, dm2.ensure(n * 8));
    HIP_TRY(ctx, dt.ensure(n * 72));
    HIP_TRY(ctx, dc.ensure(n * 48));
    HIP_TRY(ctx, dout.ensure(n * 8 * out_words));
    HIP_TRY(ctx, hipMemcpyAsync(dsk.p, sketch6, n * 48, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(dm.p, mac, n * 8, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(dm2.p, mac2, n * 8, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(dt.p, triples9, n * 72, hipMemcpyHostToDevice, ctx->stream));
    if (mode == 1) HIP_TRY(ctx, hipMemcpyAsync(dc.p, cor6, n * 48, hipMemcpyHostToDevice, ctx->stream));
    MulArgs a{};
    a.sketch = dsk.as<uint64_t>();
    a.mac = dm.as<uint64_t>();
    a.mac2 = dm2.as<uint64_t>();
    a.triples = dt.as<uint64_t>();
    a.cor = dc.as<uint64_t>();
    a.out = dout.as<uint64_t>();
    a.n = n;
    a.mode = mode;
    a.server_idx = server_idx ? 1 : 0;
    a.triples_levels = 1;
    HIP_TRY(ctx, launch_mul_fe(a, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(out, dout.p, n * 8 * out_words, hipMemcpyDeviceToHost, ctx->stream));
    return sync(ctx);
}

int fhh_mul_cor_share_fe(fhh_ctx* ctx, uint64_t n, const uint64_t* sketch6, const uint64_t* mac_key,
                         const uint64_t* mac_key2, const uint64_t* triples9, uint64_t* cor_share6) {
    return mul_fe_host(ctx, 0, 0, n, sketch6, mac_key, mac_key2, triples9, nullptr, cor_share6);
}

int fhh_mul_out_share_fe(fhh_ctx* ctx, int server_idx, uint64_t n, const uint64_t* sketch6, const uint64_t* mac_key,
                         const uint64_t* mac_key2, const uint64_t* triples9, const uint64_t* cor6, uint64_t* out) {
    return mul_fe_host(ctx, 1, server_idx, n, sketch6, mac_key, mac_key2, triples9, cor6, out);
}

int fhh_mul_cor_fe(uint64_t n, const uint64_t* share0, const uint64_t* share1, uint64_t* cor6) {
    if (n && (!share0 || !share1 || !cor6)) {
        g_err = "mul_cor_fe: NULL buffer";
        return FHH_E_ARG;
    }
    for (uint64_t i = 0; i < 6 * n; i++) {
        const uint64_t s = fe_canon_u64(share0[i]) + fe_canon_u64(share1[i]);
        cor6[i] = s >= kFeP ? s - kFeP : s;
    }
    return FHH_OK;
}

int fhh_mul_verify_fe(uint64_t n, const uint64_t* out0, const uint64_t* out1, uint8_t* ok) {
    if (n && (!out0 || !out1 || !ok)) {
        g_err = "mul_verify_fe: NULL buffer";
        return FHH_E_ARG;
    }
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t s = fe_canon_u64(out0[i]) + fe_canon_u64(out1[i]);
        ok[i] = (s >= kFeP ? s - kFeP : s) == 0;
    }
    return FHH_OK;
}

int fhh_sim_sketch_verify_fe(fhh_ctx* ctx, const fhh_sketch_batch* b) {
    CTX_CHECK(ctx);
    int rc = set_device(ctx);
    if (rc) return rc;
    if (!b) return ctx->fail(FHH_E_ARG, "sim_sketch_verify_fe: NULL batch");
    if (b->n_keys == 0) return FHH_OK;
    if (!b->seeds_dev || !b->ok_dev) return ctx->fail(FHH_E_ARG, "sim_sketch_verify_fe: NULL buffer");
    for (int s = 0; s < 2; s++)
        if (!b->mac_dev[s] || !b->mac2_dev[s] || !b->triples_dev[s] || !b->sketch_dev[s] ||
            (b->n_nodes && (!b->x_dev[s] || !b->kx_dev[s])))
            return ctx->fail(FHH_E_ARG, "sim_sketch_verify_fe: NULL buffer");
    const uint32_t nl = b->n_levels ? b->n_levels : 1;
    const uint32_t tl = b->triples_levels ? b->triples_levels : 1;
    // every level takes fresh triples (MulState::new, mpc.rs:94-98): a batch without per-level
    // triples verifies one level only (reusing a Beaver triple across openings leaks x - x')
    if (!b->triples_levels && nl > 1)
        return ctx->fail(FHH_E_ARG, "sim_sketch_verify_fe: n_levels > 1 needs triples_levels (fresh triples per level)");
    if (b->triples_levels && b->level + nl > tl)
        return ctx->fail(FHH_E_ARG, "sim_sketch_verify_fe: levels past the triples held");
    // Several levels: a two-stage pipeline over two streams. The main stream runs every level's two
    // main sketch launches back to back; the side stream runs the level's sketch tails (disjoint
    // outputs) and, once both main launches are done, its verify. Level k's sketches go to slot
    // (nl - 1 - k) & 1 (slot 0 = the caller's sketch_dev, so the last level ends there; slot 1 =
    // sketch_alt), so level k + 1's main launches overlap level k's verify, and a slot is reused by
    // level k + 2 only after level k's verify has read it. FHH_SKETCH_OVERLAP=0: one stream.
    static const bool kOverlapEnv = [] {
        const char* e = std::getenv("FHH_SKETCH_OVERLAP");
        return !(e && e[0] == '0');
    }();
    const bool overlap = nl > 1 && kOverlapEnv;
    uint64_t* alt[2] = {nullptr, nullptr};
    // r05: when the batch's sketches fit (12 GiB), every level but the last writes a slot of its own, so
    // the main stream never waits for a verify: the two-slot scheme's wait put a barrier between every
    // two levels' main launches (11.5 us median gap, 1023 per configs[4] step)
    const size_t level_words = (size_t)2 * b->n_keys * 6;
    const bool own_slots = overlap && (size_t)(nl - 1) * level_words * 8 <= ((size_t)12 << 30);
    if (overlap) {
        if (!ctx->side_stream) HIP_TRY(ctx, hipStreamCreateWithFlags(&ctx->side_stream, hipStreamNonBlocking));
        for (hipEvent_t& e : ctx->side_ev)
            if (!e) HIP_TRY(ctx, hipEventCreateWithFlags(&e, hipEventDisableTiming));
        HIP_TRY(ctx, ctx->sketch_alt.ensure((own_slots ? (size_t)(nl - 1) : 1) * level_words * 8));
        for (int s = 0; s < 2; s++) alt[s] = ctx->sketch_alt.as<uint64_t>() + (size_t)s * b->n_keys * 6;
        // the side stream starts after everything already on the main stream (triples, uploads)
        HIP_TRY(ctx, hipEventRecord(ctx->side_ev[0], ctx->stream));
        HIP_TRY(ctx, hipStreamWaitEvent(ctx->side_stream, ctx->side_ev[0], 0));
    }
    hipStream_t side = overlap ? ctx->side_stream : ctx->stream;
    hipEvent_t* ev_main = ctx->side_ev;       // [slot]: the slot's main launches are done
    hipEvent_t* ev_ver = ctx->side_ev + 2;    // [slot]: the slot's verify is done
    // a failure part way leaves no side-stream work running on the caller's buffers
    struct SideDrain {
        hipStream_t st;
        bool armed;
        ~SideDrain() {
            if (armed && st) (void)hipStreamSynchronize(st);
        }
    } drain{overlap ? ctx->side_stream : nullptr, overlap};
    for (uint32_t k = 0; k < nl; k++) {
        const uint32_t lv = b->level + k;
        const int slot = own_slots ? 0 : overlap ? (int)((nl - 1 - k) & 1) : 0;
        uint64_t* out[2] = {slot ? alt[0] : b->sketch_dev[0], slot ? alt[1] : b->sketch_dev[1]};
        if (own_slots && k + 1 < nl)
            for (int s = 0; s < 2; s++) out[s] = alt[s] + (size_t)k * level_words;
        if (overlap && !own_slots && k >= 2) HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ev_ver[slot], 0));
        {   // both servers' sketches in one main launch (r05: one launch transition per level, not two)
            SketchArgs a{};
            a.seeds = b->seeds_dev;
            a.x = b->x_dev[0] + (size_t)k * b->x_level_stride;
            a.kx = b->kx_dev[0] + (size_t)k * b->x_level_stride;
            a.out = out[0];
            a.x1 = b->x_dev[1] + (size_t)k * b->x_level_stride;
            a.kx1 = b->kx_dev[1] + (size_t)k * b->x_level_stride;
            a.out1 = out[1];
            a.n_srv = b->n_keys;
            a.n_keys = 2 * b->n_keys;
            a.n_nodes = b->n_nodes;
            a.force_sequential = b->force_sequential;
            a.level = lv;
            HIP_TRY(ctx, launch_sketch_fe2(a, ctx->stream, side));
        }
        if (overlap) {
            HIP_TRY(ctx, hipEventRecord(ev_main[slot], ctx->stream));
            HIP_TRY(ctx, hipStreamWaitEvent(side, ev_main[slot], 0));
        }
        VerifyArgs v{};
        for (int s = 0; s < 2; s++) {
            v.sketch[s] = out[s];
            v.mac[s] = b->mac_dev[s];
            v.mac2[s] = b->mac2_dev[s];
            v.triples[s] = b->triples_dev[s];
        }
        v.ok = b->ok_dev + (size_t)k * b->n_keys;
        v.out_shares = b->out_shares_dev ? b->out_shares_dev + (size_t)k * 2 * b->n_keys : nullptr;
        v.n = b->n_keys;
        v.level = b->triples_levels ? lv : 0;
        v.triples_levels = tl;
        HIP_TRY(ctx, launch_verify_fe(v, side));
        if (overlap) HIP_TRY(ctx, hipEventRecord(ev_ver[slot], side));
    }
    if (overlap) HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ev_ver[0], 0));   // the last level's slot
    drain.armed = false;   // the main stream now waits for the side stream's last verify
    return sync(ctx);
}

int fhh_deal_triples_fe(fhh_ctx* ctx, uint64_t n, uint32_t levels, uint64_t seed, uint64_t* triples0_dev,
                        uint64_t* triples1_dev) {
    CTX_CHECK(ctx);
    int rc = set_device(ctx);
    if (rc) return rc;
    if (!triples0_dev || !triples1_dev) return ctx->fail(FHH_E_ARG, "deal_triples_fe: NULL buffer");
    HIP_TRY(ctx, launch_deal_triples_fe(n, levels, seed, triples0_dev, triples1_dev, ctx->stream));
    return sync(ctx);
}

// ---- U = FieldElm (the last level) -----------------------------------------------------------
int fhh_sketch_at_fe255(fhh_ctx* ctx, uint64_t n_keys, uint32_t n_nodes, const uint8_t* seeds, const uint32_t* x,
                        const uint32_t* kx, uint32_t* sketch6) {
    CTX_CHECK(ctx);
    int rc = set_device(ctx);
    if (rc) return rc;
    if (n_keys == 0) return FHH_OK;
    if (!seeds || !sketch6 || (n_nodes && (!x || !kx))) return ctx->fail(FHH_E_ARG, "sketch_at_fe255: NULL buffer");
    const size_t vb = (size_t)n_keys * n_nodes * 32;
    DevBuf ds, dx, dkx, dout;
    HIP_TRY(ctx, ds.ensure(n_keys * 16));
    HIP_TRY(ctx, dx.ensure(vb));
    HIP_TRY(ctx, dkx.ensure(vb));
    HIP_TRY(ctx, dout.ensure(n_keys * 192));
    HIP_TRY(ctx, hipMemcpyAsync(ds.p, seeds, n_keys * 16, hipMemcpyHostToDevice, ctx->stream));
    if (vb) {
        HIP_TRY(ctx, hipMemcpyAsync(dx.p, x, vb, hipMemcpyHostToDevice, ctx->stream));
        HIP_TRY(ctx, hipMemcpyAsync(dkx.p, kx, vb, hipMemcpyHostToDevice, ctx->stream));
    }
    Sketch255Args a{};
    a.seeds = ds.as<uint8_t>();
    a.x = dx.as<uint32_t>();
    a.kx = dkx.as<uint32_t>();
    a.out = dout.as<uint32_t>();
    a.n_keys = n_keys;
    a.n_nodes = n_nodes;
    HIP_TRY(ctx, launch_sketch_fe255(a, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(sketch6, dout.p, n_keys * 192, hipMemcpyDeviceToHost, ctx->stream));
    return sync(ctx);
}

static int mul_fe255_host(fhh_ctx* ctx, uint32_t mode, int server_idx, uint64_t n, const uint32_t* sketch6,
                          const uint32_t* mac, const uint32_t* mac2, const uint32_t* triples9, const uint32_t* cor6,
                          uint32_t* out) {
    CTX_CHECK(ctx);
    int rc = set_device(ctx);
    if (rc) return rc;
    if (n == 0) return FHH_OK;
    if (!sketch6 || !mac || !mac2 || !triples9 || !out || (mode == 1 && !cor6))
        return ctx->fail(FHH_E_ARG, "mul_fe255: NULL buffer");
    DevBuf dsk, dm, dm2, dt, dc, dout;
    const size_t out_bytes = mode == 0 ? 192 : 32;
    HIP_TRY(ctx, dsk.ensure(n * 192));
    HIP_TRY(ctx, dm.ensure(n * 32));
    HIP_TRY(ctx, dm2.ensure(n * 32));
    HIP_TRY(ctx, dt.ensure(n * 288));
    HIP_TRY(ctx, dc.ensure(n * 192));
    HIP_TRY(ctx, dout.ensure(n * out_bytes));
    HIP_TRY(ctx, hipMemcpyAsync(dsk.p, sketch6, n * 192, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(dm.p, mac, n * 32, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(dm2.p, mac2, n * 32, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(dt.p, triples9, n * 288, hipMemcpyHostToDevice, ctx->stream));
    if (mode == 1) HIP_TRY(ctx, hipMemcpyAsync(dc.p, cor6, n * 192, hipMemcpyHostToDevice, ctx->stream));
    Mul255Args a{};
    a.sketch = dsk.as<uint32_t>();
    a.mac = dm.as<uint32_t>();
    a.mac2 = dm2.as<uint32_t>();
    a.triples = dt.as<uint32_t>();
    a.cor = dc.as<uint32_t>();
    a.out = dout.as<uint32_t>();
    a.n = n;
    a.mode = mode;
    a.server_idx = server_idx ? 1 : 0;
    HIP_TRY(ctx, launch_mul_fe255(a, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(out, dout.p, n * out_bytes, hipMemcpyDeviceToHost, ctx->stream));
    return sync(ctx);
}

int fhh_mul_cor_share_fe255(fhh_ctx* ctx, uint64_t n, const uint32_t* sketch6, const uint32_t* mac_key,
                            const uint32_t* mac_key2, const uint32_t* triples9, uint32_t* cor_share6) {
    return mul_fe255_host(ctx, 0, 0, n, sketch6, mac_key, mac_key2, triples9, nullptr, cor_share6);
}

int fhh_mul_out_share_fe255(fhh_ctx* ctx, int server_idx, uint64_t n, const uint32_t* sketch6,
                            const uint32_t* mac_key, const uint32_t* mac_key2, const uint32_t* triples9,
                            const uint32_t* cor6, uint32_t* out) {
    return mul_fe255_host(ctx, 1, server_idx, n, sketch6, mac_key, mac_key2, triples9, cor6, out);
}

int fhh_mul_cor_fe255(uint64_t n, const uint32_t* share0, const uint32_t* share1, uint32_t* cor6) {
    if (n && (!share0 || !share1 || !cor6)) {
        g_err = "mul_cor_fe255: NULL buffer";
        return FHH_E_ARG;
    }
    for (uint64_t i = 0; i < 6 * n; i++) {   // MulState::cor (mpc.rs:160-180)
        uint32_t a[8], b[8], o[8];
        std::memcpy(a, share0 + 8 * i, 32);
        std::memcpy(b, share1 + 8 * i, 32);
        fe255_canonm(a);
        fe255_canonm(b);
        fe255_addm(a, b, o);
        std::memcpy(cor6 + 8 * i, o, 32);
    }
    return FHH_OK;
}

int fhh_mul_verify_fe255(uint64_t n, const uint32_t* out0, const uint32_t* out1, uint8_t* ok) {
    if (n && (!out0 || !out1 || !ok)) {
        g_err = "mul_verify_fe255: NULL buffer";
        return FHH_E_ARG;
    }
    for (uint64_t i = 0; i < n; i++) {   // MulState::verify (mpc.rs:214-220)
        uint32_t a[8], b[8], o[8];
        std::memcpy(a, out0 + 8 * i, 32);
        std::memcpy(b, out1 + 8 * i, 32);
        fe255_canonm(a);
        fe255_canonm(b);
        fe255_addm(a, b, o);
        uint32_t nz = 0;
        for (int k = 0; k < 8; k++) nz |= o[k];
        ok[i] = nz == 0;
    }
    return FHH_OK;
}

int fhh_sim_sketch_verify_fe255(fhh_ctx* ctx, const fhh_sketch_batch255* b) {
    CTX_CHECK(ctx);
    int rc = set_device(ctx);
    if (rc) return rc;
    if (!b) return ctx->fail(FHH_E_ARG, "sim_sketch_verify_fe255: NULL batch");
    if (b->n_keys == 0) return FHH_OK;
    if (!b->seeds_dev || !b->ok_dev) return ctx->fail(FHH_E_ARG, "sim_sketch_verify_fe255: NULL buffer");
    for (int s = 0; s < 2; s++)
        if (!b->mac_dev[s] || !b->mac2_dev[s] || !b->triples_dev[s] || !b->sketch_dev[s] ||
            (b->n_nodes && (!b->x_dev[s] || !b->kx_dev[s])))
            return ctx->fail(FHH_E_ARG, "sim_sketch_verify_fe255: NULL buffer");
    for (int s = 0; s < 2; s++) {
        Sketch255Args a{};
        a.seeds = b->seeds_dev;
        a.x = b->x_dev[s];
        a.kx = b->kx_dev[s];
        a.out = b->sketch_dev[s];
        a.n_keys = b->n_keys;
        a.n_nodes = b->n_nodes;
        a.force_sequential = b->force_sequential;
        a.level = b->level;
        HIP_TRY(ctx, launch_sketch_fe255(a, ctx->stream));
    }
    Verify255Args v{};
    for (int s = 0; s < 2; s++) {
        v.sketch[s] = b->sketch_dev[s];
        v.mac[s] = b->mac_dev[s];
        v.mac2[s] = b->mac2_dev[s];
        v.triples[s] = b->triples_dev[s];
    }
    v.ok = b->ok_dev;
    v.out_shares = b->out_shares_dev;
    v.n = b->n_keys;
    HIP_TRY(ctx, launch_verify_fe255(v, ctx->stream));
    return sync(ctx);
}
