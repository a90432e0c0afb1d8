// One KeyCollection over several GPUs (north_star: "clients shard across the 8 GPUs, and per-GPU
// partial prefix counts are combined with an RCCL all-reduce"; SURVEY §8(b) fhh_create(...,
// devices, n_devices), §8(e)).
//
// The reference server owns ONE `KeyCollection` behind a Mutex (src/bin/server.rs:44-52, 332-335)
// and its tarpc handlers call it per level (server.rs:64-171). A multi-device fhh_ctx keeps that
// shape: the caller still sees one collection, while its clients live on S shard ctxs, one per
// entry of `devices` (a device may repeat — two shards on one GPU exercise the same code on a
// one-GPU box). Shard k holds the contiguous client range [base_k, base_k + count_k), cut at
// whole 64-client words (the share-plane word of a client is then the same in the shard and in
// the collection, so gathering planes is one strided copy per shard). Every call fans out over
// the shards on one host thread each (each shard its own device and stream), and:
//   tree_crawl(_last)      each shard expands its clients; share planes land in the caller's
//                          [C][2d][nw] rows at the shard's word offset
//   node_sums_fe(255)      each shard sums its columns of the OT outputs into 32-bit-limb u64
//                          partials; the partials are summed over the shards — RCCL
//                          ncclAllReduce (ncclCommInitAll, one grouped call, one stream per
//                          device) when the devices are distinct, on the host otherwise — then
//                          reduced mod p once (the u64 limbs hold 2^32 clients of headroom)
//   tree_prune(_last)      the same keep mask on every shard (frontiers stay identical)
//   sim_crawl              one thread per shard pair runs the device-resident level loop; the
//                          loop's per-level all-reduce goes over the group's communicators
#include "fhh_engine.h"

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace fhh {
namespace eng {

// Sum of host buffers across the shard threads of one process (the hosted communicators of a
// group whose shards share a GPU, where RCCL refuses two ranks on one device). Barrier semantics:
// the last arrival publishes the sum; nobody can start the next round before every thread has
// copied this one's result, because the next round needs every thread to arrive.
struct ThreadReducer {
    int n = 0;
    std::mutex mu;
    std::condition_variable cv;
    std::vector<uint64_t> acc, result;
    int arrived = 0;
    uint64_t gen = 0;
    bool aborted = false;

    int reduce(uint64_t* buf, uint64_t count) {
        std::unique_lock<std::mutex> lk(mu);
        if (aborted) return 1;
        if (arrived == 0) acc.assign(count, 0);
        if (acc.size() != count) {   // ranks disagree on the shape: give up on every rank
            aborted = true;
            cv.notify_all();
            return 1;
        }
        for (uint64_t i = 0; i < count; i++) acc[i] += buf[i];
        const uint64_t my_gen = gen;
        if (++arrived == n) {
            result.swap(acc);
            arrived = 0;
            gen++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != my_gen || aborted; });
            if (gen == my_gen) return 1;   // aborted
        }
        std::memcpy(buf, result.data(), count * 8);
        return 0;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(mu);
        aborted = true;
        cv.notify_all();
    }
};

struct ReducerSlot {
    ThreadReducer* r;
};

static int reducer_cb(uint64_t* buf, uint64_t count, void* user) {
    return static_cast<ReducerSlot*>(user)->r->reduce(buf, count);
}

struct Group {
    std::vector<fhh_ctx*> shards;            // one per entry of devices[]
    std::vector<int> devices;
    std::vector<uint64_t> base, count;       // client range per shard (after placement)
    bool placed = false;                     // keys live on the shards
    uint64_t client_base = 0;                // fhh_set_client_base of the collection
    bool distinct = false;                   // every shard on its own GPU
    bool force_host = false;                 // FHH_GROUP_REDUCE=host
    bool force_rccl = false;                 // FHH_GROUP_REDUCE=rccl: the RCCL branch on a repeated device
                                             // (tests, with tests/stubs/librccl_stub.so loaded)
    std::vector<::fhh_comm*> comms;          // in-process RCCL communicators (distinct devices)
    std::string comm_err;

    std::vector<size_t> active() const {     // shards that hold clients
        std::vector<size_t> a;
        for (size_t k = 0; k < shards.size(); k++)
            if (!placed || count[k]) a.push_back(k);
        return a;
    }
    // FHH_REDUCE_*: RCCL only when every shard holds clients (all ranks join each collective)
    int reduction() const {
        if (shards.size() == 1) return FHH_REDUCE_NONE;
        if ((!distinct && !force_rccl) || force_host) return FHH_REDUCE_HOST;
        for (size_t k = 0; k < shards.size(); k++)
            if (placed && !count[k]) return FHH_REDUCE_HOST;
        return FHH_REDUCE_RCCL;
    }
};

namespace {

// contiguous ranges of whole 64-client words: shard k gets words [nw k / S, nw (k + 1) / S)
void plan(Group& G, uint64_t n) {
    const uint64_t S = G.shards.size(), nw = (n + 63) / 64;
    G.base.assign(S, 0);
    G.count.assign(S, 0);
    for (uint64_t k = 0; k < S; k++) {
        const uint64_t b = std::min<uint64_t>(n, 64 * (nw * k / S)), e = std::min<uint64_t>(n, 64 * (nw * (k + 1) / S));
        G.base[k] = b;
        G.count[k] = e - b;
    }
}

int shard_fail(fhh_ctx* g, size_t k, int rc) {
    const Group& G = *g->group;
    return g->fail(rc, "shard " + std::to_string(k) + " (device " + std::to_string(G.devices[k]) + "): " +
                           G.shards[k]->err);
}

// f(k, shard) on one host thread per active shard; the first failure is reported
template <class F>
int fan_out(fhh_ctx* g, F f) {
    Group& G = *g->group;
    const std::vector<size_t> act = G.active();
    std::vector<int> rc(act.size(), 0);
    if (act.size() == 1) {
        rc[0] = f(act[0], G.shards[act[0]]);
    } else {
        std::vector<std::thread> th;
        th.reserve(act.size());
        for (size_t i = 0; i < act.size(); i++) th.emplace_back([&, i] { rc[i] = f(act[i], G.shards[act[i]]); });
        for (auto& t : th) t.join();
    }
    for (size_t i = 0; i < act.size(); i++)
        if (rc[i]) return shard_fail(g, act[i], rc[i]);
    return FHH_OK;
}

int ensure_comms(fhh_ctx* g) {
    Group& G = *g->group;
    if (G.reduction() != FHH_REDUCE_RCCL) return FHH_OK;
    if (!G.comms.empty()) return FHH_OK;
    std::string err;
    if (comm_init_all((int)G.devices.size(), G.devices.data(), G.comms, &err))
        return g->fail(FHH_E_COMM, "multi-device ctx: " + err);
    return FHH_OK;
}

void drop_comms(Group& G) {
    for (auto* c : G.comms) fhh_comm_destroy(c);
    G.comms.clear();
}

void set_bases(Group& G) {
    for (size_t k = 0; k < G.shards.size(); k++) (void)fhh_set_client_base(G.shards[k], G.client_base + G.base[k]);
}

}  // namespace

void group_destroy(fhh_ctx* g) {
    Group* G = g->group;
    drop_comms(*G);
    for (auto* s : G->shards) fhh_destroy(s);
    delete G;
    g->group = nullptr;
    delete g;
}

int group_reset(fhh_ctx* g) {
    Group& G = *g->group;
    for (auto* s : G.shards) {
        const int rc = fhh_reset(s);
        if (rc) return g->fail(rc, s->err);
    }
    G.placed = false;
    g->h_key_idx.clear();
    g->h_root.clear();
    g->h_cws.clear();
    g->h_cwb.clear();
    g->h_n = 0;
    return FHH_OK;
}

int group_set_client_base(fhh_ctx* g, uint64_t base) {
    Group& G = *g->group;
    G.client_base = base;
    if (G.placed) set_bases(G);
    return FHH_OK;
}

int group_add_keys_bincode(fhh_ctx* g, const uint8_t* req, uint64_t len) {
    Group& G = *g->group;
    if (!req || len < 8) return g->fail(FHH_E_ARG, "add_keys_bincode: buffer shorter than the u64 length");
    if (G.placed || g->h_n) return g->fail(FHH_E_STATE, "add_keys_bincode: ctx already holds keys");
    uint64_t n = 0;
    for (int i = 0; i < 8; i++) n |= (uint64_t)req[i] << (8 * i);
    const uint64_t KB = 25 + 20ull * g->L, R = 8 + (uint64_t)g->K * KB;
    if (n == 0) return g->fail(FHH_E_ARG, "add_keys_bincode: no clients");
    if (n > (len - 8) / R || 8 + n * R != len)
        return g->fail(FHH_E_ARG, "add_keys_bincode: length does not match n clients x n_dims x data_len");
    plan(G, n);
    G.placed = true;
    // each shard uploads and decodes its own slice of the records (clients are fixed-size records)
    const int rc = fan_out(g, [&](size_t k, fhh_ctx* s) {
        return add_keys_bincode_records(s, G.count[k], req + 8 + G.base[k] * R);
    });
    if (rc) {
        (void)group_reset(g);
        return rc;
    }
    set_bases(G);
    return FHH_OK;
}

int group_gen_keys_pair(fhh_ctx* g0, fhh_ctx* g1, uint64_t n, const uint8_t* left, const uint8_t* right,
                        const uint8_t* roots) {
    if (!g0->group || !g1->group) return g0->fail(FHH_E_ARG, "gen_keys_pair: both ctxs must be multi-device ctxs");
    Group &G0 = *g0->group, &G1 = *g1->group;
    if (G0.devices != G1.devices || g0->d != g1->d || g0->L != g1->L)
        return g0->fail(FHH_E_ARG, "gen_keys_pair: the two collections differ in devices / d / L");
    if (G0.placed || G1.placed || g0->h_n || g1->h_n) return g0->fail(FHH_E_STATE, "gen_keys_pair: ctxs must be empty");
    if (!left || !right || !roots) return g0->fail(FHH_E_ARG, "gen_keys_pair: NULL buffer");
    plan(G0, n);
    plan(G1, n);
    G0.placed = G1.placed = true;
    const size_t dL = (size_t)g0->d * g0->L, dR = (size_t)g0->d * 64;
    const int rc = fan_out(g0, [&](size_t k, fhh_ctx* s) {
        return fhh_gen_keys_pair(s, G1.shards[k], G0.count[k], left + G0.base[k] * dL, right + G0.base[k] * dL,
                                 roots + G0.base[k] * dR);
    });
    if (rc) {
        (void)group_reset(g0);
        (void)group_reset(g1);
        return rc;
    }
    set_bases(G0);
    set_bases(G1);
    return FHH_OK;
}

int group_num_clients(const fhh_ctx* g, uint64_t* n) {
    const Group& G = *g->group;
    uint64_t v = g->h_n;
    if (G.placed)
        for (uint64_t c : G.count) v += c;
    if (n) *n = v;
    return FHH_OK;
}

int group_export_keys(fhh_ctx* g, uint8_t* key_idx, uint8_t* root_seed, uint8_t* cw_seed, uint8_t* cw_bits) {
    Group& G = *g->group;
    const size_t K = g->K, L = g->L;
    if (!G.placed) {   // still staged on the collection (add_keys before tree_init)
        if (key_idx) std::memcpy(key_idx, g->h_key_idx.data(), g->h_key_idx.size());
        if (root_seed) std::memcpy(root_seed, g->h_root.data(), g->h_root.size());
        if (cw_seed) std::memcpy(cw_seed, g->h_cws.data(), g->h_cws.size());
        if (cw_bits) std::memcpy(cw_bits, g->h_cwb.data(), g->h_cwb.size());
        return FHH_OK;
    }
    // every layout is client-major: shard k writes its clients' rows in place
    return fan_out(g, [&](size_t k, fhh_ctx* s) {
        const size_t b = G.base[k];
        return fhh_export_keys(s, key_idx ? key_idx + b * K : nullptr, root_seed ? root_seed + b * K * 16 : nullptr,
                               cw_seed ? cw_seed + b * K * L * 16 : nullptr, cw_bits ? cw_bits + b * K * L : nullptr);
    });
}

int group_tree_init(fhh_ctx* g) {
    Group& G = *g->group;
    if (g->h_n) {
        // keys staged by add_keys: cut them into the shards' client ranges now that n is known
        if (G.placed) return g->fail(FHH_E_STATE, "add_keys after the keys were placed on the shards");
        const uint64_t n = g->h_n;
        const size_t K = g->K, L = g->L;
        plan(G, n);
        G.placed = true;
        int rc = fan_out(g, [&](size_t k, fhh_ctx* s) {
            const size_t b = G.base[k];
            int r = fhh_reset(s);
            if (r) return r;
            return fhh_add_keys(s, G.count[k], g->h_key_idx.data() + b * K, g->h_root.data() + b * K * 16,
                                g->h_cws.data() + b * K * L * 16, g->h_cwb.data() + b * K * L);
        });
        if (rc) {
            G.placed = false;
            return rc;
        }
        g->h_key_idx.clear();
        g->h_root.clear();
        g->h_cws.clear();
        g->h_cwb.clear();
        g->h_key_idx.shrink_to_fit();
        g->h_root.shrink_to_fit();
        g->h_cws.shrink_to_fit();
        g->h_cwb.shrink_to_fit();
        g->h_n = 0;
        set_bases(G);
    }
    if (!G.placed) return g->fail(FHH_E_STATE, "tree_init with no keys (collect.rs:83)");
    int rc = fan_out(g, [&](size_t, fhh_ctx* s) { return fhh_tree_init(s); });
    if (rc) return rc;
    return ensure_comms(g);
}

int group_tree_crawl(fhh_ctx* g, bool last, uint64_t* n_children, uint64_t* planes) {
    Group& G = *g->group;
    if (!G.placed) return g->fail(FHH_E_STATE, "tree_crawl before tree_init");
    uint64_t n = 0;
    group_num_clients(g, &n);
    const uint64_t nw = (n + 63) / 64;
    std::vector<uint64_t> C(G.shards.size(), 0);
    int rc = fan_out(g, [&](size_t k, fhh_ctx* s) {
        int r = ctx_set_device(s);
        if (r) return r;
        return crawl_level(s, last, &C[k], planes, nw, G.base[k] / 64);
    });
    if (rc) return rc;
    const auto act = G.active();
    for (size_t k : act)
        if (C[k] != C[act[0]]) return g->fail(FHH_E_STATE, "tree_crawl: shards disagree on the frontier");
    if (n_children) *n_children = act.empty() ? 0 : C[act[0]];
    return FHH_OK;
}

int group_node_sums(fhh_ctx* g, const void* const* vals, bool host, uint64_t ld, uint32_t fmt, void* out_a,
                    void* out_b) {
    Group& G = *g->group;
    if (!G.placed) return g->fail(FHH_E_STATE, "node_sums without a pending crawl");
    uint64_t n = 0;
    group_num_clients(g, &n);
    const auto act = G.active();
    fhh_ctx* lead = G.shards[act[0]];
    const uint64_t C = lead->pending_C, per = fmt_is_fe255(fmt) ? 8 : 2;
    std::vector<uint64_t*> part(G.shards.size(), nullptr);
    // 1. every shard's partials of its own clients (host values: its column block of [C][n])
    int rc = fan_out(g, [&](size_t k, fhh_ctx* s) {
        int r = ctx_set_device(s);
        if (r) return r;
        if (s->pending_C != C) return s->fail(FHH_E_STATE, "node_sums: shards disagree on the frontier");
        if (host) return node_partials(s, vals[0], fmt, n, G.base[k], true, &part[k]);
        if (!vals[k]) return s->fail(FHH_E_ARG, "node_sums: NULL device values for this shard");
        return node_partials(s, vals[k], fmt, ld ? ld : s->n, 0, false, &part[k]);   // ld 0: the shard's n
    });
    if (rc) return rc;
    // 2. the sum over the shards
    std::vector<uint64_t> h(C * per, 0);
    if (C) {
        if (G.reduction() == FHH_REDUCE_RCCL) {
            rc = ensure_comms(g);
            if (rc) return rc;
            std::vector<hipStream_t> streams;
            for (auto* s : G.shards) streams.push_back(s->stream);
            std::string err;
            rc = comm_group_allreduce(G.comms, part, C * per, streams, &err);
            if (rc) return g->fail(rc, "node_sums: " + err);
            fhh_ctx* s0 = G.shards[0];
            HIP_TRY(g, hipSetDevice(s0->device));
            HIP_TRY(g, hipMemcpyAsync(h.data(), part[0], h.size() * 8, hipMemcpyDeviceToHost, s0->stream));
            rc = fan_out(g, [&](size_t, fhh_ctx* s) { return ctx_sync(s); });
            if (rc) return rc;
        } else {
            std::vector<std::vector<uint64_t>> hk(G.shards.size());
            rc = fan_out(g, [&](size_t k, fhh_ctx* s) {
                hk[k].resize(C * per);
                HIP_TRY(s, hipMemcpyAsync(hk[k].data(), part[k], C * per * 8, hipMemcpyDeviceToHost, s->stream));
                return ctx_sync(s);
            });
            if (rc) return rc;
            for (size_t k : act)
                for (uint64_t i = 0; i < C * per; i++) h[i] += hk[k][i];
        }
    }
    // 3. one modular reduction; a FieldElm level's sums become every shard's frontier_last values
    for (size_t k : act) {
        rc = node_sums_finish(G.shards[k], h.data(), fmt, k == act[0] ? out_a : nullptr, k == act[0] ? out_b : nullptr);
        if (rc) return shard_fail(g, k, rc);
    }
    return FHH_OK;
}

int group_tree_prune(fhh_ctx* g, const uint8_t* keep, uint64_t n, bool last) {
    Group& G = *g->group;
    if (!G.placed) return g->fail(FHH_E_STATE, "tree_prune without a pending tree_crawl");
    for (size_t k : G.active()) {   // host-only bookkeeping: sequential
        const int rc = last ? fhh_tree_prune_last(G.shards[k], keep, n) : fhh_tree_prune(G.shards[k], keep, n);
        if (rc) return shard_fail(g, k, rc);
    }
    return FHH_OK;
}

fhh_ctx* group_lead(const fhh_ctx* g) {
    const Group& G = *g->group;
    const auto act = G.active();
    return (G.placed && !act.empty()) ? G.shards[act[0]] : nullptr;
}

int group_export_states(fhh_ctx* g, uint64_t* n_nodes, uint8_t* seeds, uint8_t* t, uint8_t* y) {
    Group& G = *g->group;
    fhh_ctx* lead = group_lead(g);
    if (!lead) return g->fail(FHH_E_STATE, "export_states before tree_init");
    uint64_t F = 0;
    int rc = fhh_export_states(lead, &F, nullptr, nullptr, nullptr);
    if (rc) return g->fail(rc, lead->err);
    if (n_nodes) *n_nodes = F;
    if (!seeds && !t && !y) return FHH_OK;
    uint64_t n = 0;
    group_num_clients(g, &n);
    const size_t row = (size_t)g->d * 2;   // states per (node, client)
    // [node][client][d][2]: shard k's clients are a contiguous run inside every node's row
    return fan_out(g, [&](size_t k, fhh_ctx* s) {
        const uint64_t nk = G.count[k];
        std::vector<uint8_t> hs(seeds ? F * nk * row * 16 : 0), ht(t ? F * nk * row : 0), hy(y ? F * nk * row : 0);
        uint64_t Fk = 0;
        int r = fhh_export_states(s, &Fk, seeds ? hs.data() : nullptr, t ? ht.data() : nullptr, y ? hy.data() : nullptr);
        if (r) return r;
        if (Fk != F) return s->fail(FHH_E_STATE, "export_states: shards disagree on the frontier");
        for (uint64_t f = 0; f < F; f++) {
            const size_t dst = (f * n + G.base[k]) * row, src = f * nk * row;
            if (seeds) std::memcpy(seeds + dst * 16, hs.data() + src * 16, nk * row * 16);
            if (t) std::memcpy(t + dst, ht.data() + src, nk * row);
            if (y) std::memcpy(y + dst, hy.data() + src, nk * row);
        }
        return FHH_OK;
    });
}

int group_sim_crawl(fhh_ctx* g0, fhh_ctx* g1, const fhh_sim_config* cfg) {
    if (!g0->group || !g1->group) return g0->fail(FHH_E_ARG, "sim_crawl: both ctxs must be multi-device ctxs");
    Group &G0 = *g0->group, &G1 = *g1->group;
    if (G0.devices != G1.devices) return g0->fail(FHH_E_ARG, "sim_crawl: the two collections differ in devices");
    if (cfg->comm || cfg->allreduce)
        return g0->fail(FHH_E_ARG, "sim_crawl: a multi-device ctx brings its own reduction (no cfg->comm / allreduce)");
    if (!G0.placed || !G1.placed || G0.base != G1.base || G0.count != G1.count)
        return g0->fail(FHH_E_STATE, "sim_crawl: both collections need the same clients placed (gen_keys_pair)");
    const auto act = G0.active();
    if (cfg->probe_n_levels && act.size() > 1)
        return g0->fail(FHH_E_ARG, "sim_crawl: the state probe reads one shard (use a one-shard ctx)");
    if (act.size() == 1) {
        const int rc = fhh_sim_crawl(G0.shards[act[0]], G1.shards[act[0]], cfg);
        return rc ? shard_fail(g0, act[0], rc) : FHH_OK;
    }
    uint64_t n_total = 0;
    group_num_clients(g0, &n_total);
    // per-shard communicators for the device loop's per-level all-reduce
    const int red = G0.reduction();
    std::vector<::fhh_comm*> comms(G0.shards.size(), nullptr);
    ThreadReducer tr;
    tr.n = (int)act.size();
    ReducerSlot slot{&tr};
    std::vector<::fhh_comm*> hosted;
    if (red == FHH_REDUCE_RCCL) {
        int rc = ensure_comms(g0);
        if (rc) return rc;
        comms = G0.comms;
    } else {
        for (size_t i = 0; i < act.size(); i++) {
            const size_t k = act[i];
            ::fhh_comm* c = nullptr;
            if (fhh_comm_create_hosted(&c, (int)act.size(), (int)i, G0.devices[k], reducer_cb, &slot))
                return g0->fail(FHH_E_COMM, "sim_crawl: hosted communicator");
            comms[k] = c;
            hosted.push_back(c);
        }
    }
    std::vector<int> rcs(G0.shards.size(), 0);
    std::vector<std::thread> th;
    // the first failing shard releases its peers waiting in a collective, once for the whole call
    // (two shards failing together must not both abort the same communicators)
    std::once_flag abort_once;
    int root = -1;   // the shard whose failure started the abort (its peers then fail with "aborted")
    for (size_t k : act)
        th.emplace_back([&, k] {
            fhh_sim_config c = *cfg;
            c.nclients_total = cfg->nclients_total ? cfg->nclients_total : n_total;
            c.comm = comms[k];
            if (k != act[0]) {   // the per-level records come from the first shard (all hold the sums)
                c.level_children = c.level_kept = c.counts = nullptr;
                c.counts_capacity = 0;
            }
            rcs[k] = fhh_sim_crawl(G0.shards[k], G1.shards[k], &c);
            if (rcs[k])
                std::call_once(abort_once, [&] {
                    root = (int)k;
                    tr.abort();
                    if (red == FHH_REDUCE_RCCL)
                        for (auto* cm : comms) comm_abort(cm);
                });
        });
    for (auto& t : th) t.join();
    for (auto* c : hosted) fhh_comm_destroy(c);
    int first = root;
    for (size_t k : act)
        if (rcs[k] && first < 0) first = (int)k;
    if (first >= 0) {
        if (red == FHH_REDUCE_RCCL) drop_comms(G0);   // aborted communicators are rebuilt on the next use
        return shard_fail(g0, (size_t)first, rcs[(size_t)first]);
    }
    return FHH_OK;
}

int group_get_stats(const fhh_ctx* g, fhh_stats* out) {
    fhh_stats t{};
    for (auto* s : g->group->shards) {
        fhh_stats v{};
        (void)fhh_get_stats(s, &v);
        t.aes_blocks += v.aes_blocks;
        t.ref_evals += v.ref_evals;
        t.expand_launches += v.expand_launches;
        t.expand_ms += v.expand_ms;
        t.expand_blocks_timed += v.expand_blocks_timed;
        t.levels = std::max(t.levels, v.levels);
        t.keygen_ms += v.keygen_ms;
        t.expand_launches_timed += v.expand_launches_timed;
        t.base_ot_ms += v.base_ot_ms;
        t.base_ot_stall_ms += v.base_ot_stall_ms;
        t.base_ot_instances += v.base_ot_instances;
        t.allreduce_ms += v.allreduce_ms;
        t.allreduce_timed += v.allreduce_timed;
        t.gcot_ms += v.gcot_ms;
        t.gcot_timed += v.gcot_timed;
    }
    if (out) *out = t;
    return FHH_OK;
}

int group_each(fhh_ctx* g, int (*fn)(fhh_ctx*, int), int arg) {
    Group& G = *g->group;
    for (size_t k = 0; k < G.shards.size(); k++) {
        const int rc = fn(G.shards[k], arg);
        if (rc) return shard_fail(g, k, rc);
    }
    return FHH_OK;
}

}  // namespace eng
}  // namespace fhh

extern "C" {

int fhh_create_multi(fhh_ctx** out, uint32_t data_len, uint32_t n_dims, const int* devices, int n_devices) {
    if (!out || !devices || n_devices < 1) {
        g_err = "fhh_create_multi: need an output pointer and at least one device";
        return FHH_E_ARG;
    }
    *out = nullptr;
    if (n_dims < 1 || n_dims > FHH_MAX_DIMS || data_len < 1) {
        g_err = "fhh_create_multi: bad data_len / n_dims";
        return FHH_E_ARG;
    }
    auto* G = new Group();
    for (int k = 0; k < n_devices; k++) {
        fhh_ctx* s = nullptr;
        const int rc = fhh_create(&s, data_len, n_dims, devices[k]);
        if (rc) {
            const std::string e = "shard " + std::to_string(k) + ": " + g_err;
            for (auto* p : G->shards) fhh_destroy(p);
            delete G;
            g_err = e;
            return rc;
        }
        G->shards.push_back(s);
        G->devices.push_back(devices[k]);
    }
    std::vector<int> sorted(G->devices);
    std::sort(sorted.begin(), sorted.end());
    G->distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    const char* e = std::getenv("FHH_GROUP_REDUCE");
    G->force_host = e && std::string(e) == "host";
    G->force_rccl = e && std::string(e) == "rccl";
    auto* g = new fhh_ctx();
    g->device = devices[0];
    g->L = data_len;
    g->d = n_dims;
    g->K = 2 * n_dims;
    g->group = G;
    *out = g;
    return FHH_OK;
}

int fhh_shard_plan(uint64_t n_clients, int n_shards, uint64_t* client_base, uint64_t* n_clients_out) {
    if (n_shards < 1 || !client_base || !n_clients_out) {
        g_err = "shard_plan: bad arguments";
        return FHH_E_ARG;
    }
    Group G;
    G.shards.assign((size_t)n_shards, nullptr);
    plan(G, n_clients);
    for (int k = 0; k < n_shards; k++) {
        client_base[k] = G.base[(size_t)k];
        n_clients_out[k] = G.count[(size_t)k];
    }
    return FHH_OK;
}

int fhh_shard_info(const fhh_ctx* ctx, int shard, int* n_shards, int* device, uint64_t* client_base,
                   uint64_t* n_clients, int* reduction) {
    if (!ctx) {
        g_err = "null fhh_ctx";
        return FHH_E_ARG;
    }
    if (!ctx->group) {   // a one-GPU ctx is its own single shard
        if (shard != 0) return const_cast<fhh_ctx*>(ctx)->fail(FHH_E_ARG, "shard_info: no such shard");
        if (n_shards) *n_shards = 1;
        if (device) *device = ctx->device;
        if (client_base) *client_base = ctx->client_base;
        if (n_clients) *n_clients = ctx->dev_keys ? ctx->n : ctx->h_n;
        if (reduction) *reduction = FHH_REDUCE_NONE;
        return FHH_OK;
    }
    const Group& G = *ctx->group;
    if (shard < 0 || shard >= (int)G.shards.size())
        return const_cast<fhh_ctx*>(ctx)->fail(FHH_E_ARG, "shard_info: no such shard");
    if (n_shards) *n_shards = (int)G.shards.size();
    if (device) *device = G.devices[(size_t)shard];
    if (client_base) *client_base = G.client_base + (G.placed ? G.base[(size_t)shard] : 0);
    if (n_clients) *n_clients = G.placed ? G.count[(size_t)shard] : 0;
    if (reduction) *reduction = G.reduction();
    return FHH_OK;
}

int fhh_shard_ctx(fhh_ctx* ctx, int shard, fhh_ctx** out) {
    if (!ctx || !out) {
        g_err = "shard_ctx: NULL argument";
        return FHH_E_ARG;
    }
    if (!ctx->group) {
        if (shard != 0) return ctx->fail(FHH_E_ARG, "shard_ctx: no such shard");
        *out = ctx;
        return FHH_OK;
    }
    if (shard < 0 || shard >= (int)ctx->group->shards.size()) return ctx->fail(FHH_E_ARG, "shard_ctx: no such shard");
    *out = ctx->group->shards[(size_t)shard];
    return FHH_OK;
}

}  // extern "C"
