/*
 * fhh.h — C ABI of the MI355X-native evaluator for the per-level client-key evaluation
 * of sks-codes/fuzzyheavyhitters (the ibDCF tree crawl).
 *
 * Drop-in boundary: `impl KeyCollection<T = FE, U = FieldElm>` (src/collect.rs:45-1030),
 * called by the tarpc `Collector` handlers (src/bin/server.rs:64-171). One fhh_ctx is one
 * server's KeyCollection bound to one GPU (fhh_create) or sharded over several
 * (fhh_create_multi). Every entry point below names the reference
 * item it replaces. A reference-side binding (Rust `extern "C"` + build.rs) is shown in
 * INTEGRATION.md.
 *
 * Conventions
 *  - Return 0 on success, a negative FHH_E* code on error; fhh_last_error(ctx) explains.
 *    The reference panics (unwrap/assert, collect.rs:83,919,932,946,967,1008,1012); a
 *    caller that wants that behaviour aborts on nonzero.
 *  - All buffers are caller-owned HOST memory unless the name ends in `_dev` (device
 *    pointer on the ctx's GPU). The ctx owns its device memory and its HIP stream, a
 *    non-blocking stream: `_dev` inputs must be complete when a call is made (synchronise the
 *    stream that produced them), and a call returns after its `_dev` outputs are complete.
 *  - A ctx may be used from any thread, but not concurrently (the reference wraps the
 *    collection in a Mutex, server.rs:49). Calls are synchronous w.r.t. the host.
 *  - Key order: client-major, then dim j in [0,d), then (left, right) — the order of
 *    `add_key(Vec<(ibDCFKey, ibDCFKey)>)` (collect.rs:62) and `gen_l_inf_ball`
 *    (ibDCF.rs:175-188). K = 2*d keys per client.
 *  - cw_bits nibble per (key, level): bit0 = bits.0, bit1 = bits.1, bit2 = y_bits.0,
 *    bit3 = y_bits.1 of `CorWord` (ibDCF.rs:9-14).
 *  - Child order: parent order, then i in `all_bit_vectors(d)` (lib.rs:125-129): child i
 *    takes direction (i >> j) & 1 in dim j (collect.rs:379-391).
 *  - Share bits per (child, client): [left.y^left.t for each dim] ++ [right.y^right.t for
 *    each dim] (collect.rs:393-418). Exported as bit-planes [child][2d][nw] u64, bit
 *    (client % 64) of word (client / 64); nw = ceil(n_clients / 64).
 *  - FE = GF(2^62 - 2^30 - 1) (fastfield.rs:24-28); FE255 = GF(2^255 - 19) (field.rs:19).
 *    FE values may be passed in any u64 representation (FE::new semantics,
 *    fastfield.rs:112-118); sums are returned canonical (`value()`, fastfield.rs:147-152).
 */
#ifndef FHH_H
#define FHH_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FHH_OK 0
#define FHH_E_ARG (-1)      /* bad argument / shape mismatch (reference: assert_eq! panic) */
#define FHH_E_STATE (-2)    /* call out of protocol order (e.g. prune without crawl)       */
#define FHH_E_HIP (-3)      /* HIP runtime error                                           */
#define FHH_E_NOMEM (-4)    /* device allocation failed                                    */
#define FHH_E_CALLBACK (-5) /* all-reduce callback failed                                  */
#define FHH_E_COMM (-6)     /* RCCL not loadable / collective failed                        */

#define FHH_MAX_DIMS 4

typedef struct fhh_ctx fhh_ctx;

/* ---- lifecycle ------------------------------------------------------------------------ */

/* KeyCollection::new(seed, depth) (collect.rs:51-60). data_len = tree depth L (number of
 * crawl levels); n_dims = d. The PRG seed of `new` only feeds the unused rand_stream. */
int fhh_create(fhh_ctx** out, uint32_t data_len, uint32_t n_dims, int device);
void fhh_destroy(fhh_ctx* ctx);
/* Thread-local message of the last failure (ctx may be NULL for fhh_create failures). */
const char* fhh_last_error(const fhh_ctx* ctx);
/* `reset` RPC (server.rs:64-69): drop keys and frontier. */
int fhh_reset(fhh_ctx* ctx);
/* Global index of this ctx's first client (used by the simulated-OT PRF when clients are
 * sharded across GPUs); default 0. */
int fhh_set_client_base(fhh_ctx* ctx, uint64_t client_base);

/* ---- keys ----------------------------------------------------------------------------- */

/* KeyCollection::add_key (collect.rs:62-65), batched: append n clients.
 *   key_idx   [n][d][2]         (ibDCFKey.key_idx, ibDCF.rs:17)
 *   root_seed [n][d][2][16]     (ibDCFKey.root_seed)
 *   cw_seed   [n][d][2][L][16]  (CorWord.seed for levels 0..L-1)
 *   cw_bits   [n][d][2][L]      (nibble, see above)
 * Keys are staged on the host and transposed to the device layout at tree_init. */
int fhh_add_keys(fhh_ctx* ctx, uint64_t n, const uint8_t* key_idx, const uint8_t* root_seed,
                 const uint8_t* cw_seed, const uint8_t* cw_bits);

/* The `add_keys` RPC payload as it arrives at the server (rpc.rs:12-15, server.rs:71-77):
 * `AddKeysRequest.keys: Vec<Vec<(ibDCFKey, ibDCFKey)>>` in bincode 1.x legacy encoding
 * (`bincode::serialize`, as leader.rs:101 sizes a key: 1 + 16 + 8 + 20 L bytes), decoded on
 * the GPU straight into the device layout (no host AoS->SoA pass). Every
 * client must carry n_dims (left, right) pairs of data_len-level keys; bools must be 0/1.
 * The ctx must hold no keys yet. FHH_E_ARG on any malformed field (the reference's RPC
 * decode fails the request). */
int fhh_add_keys_bincode(fhh_ctx* ctx, const uint8_t* req, uint64_t len);

/* Leader-side batched `gen_l_inf_ball` keygen on the GPU (ibDCF.rs:84-119,138-188),
 * writing server 0's keys into ctx0 and server 1's into ctx1 (both must be empty and on the
 * same device). Replaces the leader's per-client `add_fuzzy_keys` loop (leader.rs:130-163).
 *   left_bits/right_bits [n][d][L] (0/1, MSB first: interval bounds l = a-δ, r = a+δ)
 *   root_seeds [n][d][2 side][2 server][16] (caller randomness; the reference uses
 *   thread_rng, prg.rs:153-158). */
int fhh_gen_keys_pair(fhh_ctx* ctx0, fhh_ctx* ctx1, uint64_t n, const uint8_t* left_bits,
                      const uint8_t* right_bits, const uint8_t* root_seeds);

/* ---- one KeyCollection over several GPUs (north_star) -----------------------
 * KeyCollection::new on n_devices GPUs: one collection whose clients are sharded over the devices
 * (devices[k] may repeat — two shards on one GPU run the same code on a one-GPU box). At
 * tree_init (or add_keys_bincode / gen_keys_pair) the clients are cut into contiguous ranges of
 * whole 64-client words, one per shard, and every KeyCollection entry point of this header fans
 * out over the shards (one host thread per shard, each on its own device and stream) with the
 * results of a one-GPU collection: share planes are gathered in client order, node sums are summed
 * over the shards as u64 32-bit-limb partials — an in-process RCCL all-reduce (ncclCommInitAll,
 * one grouped ncclAllReduce over the shards' streams) when the devices are distinct, on the host
 * otherwise (or with FHH_GROUP_REDUCE=host; FHH_GROUP_REDUCE=rccl takes the RCCL branch even on a
 * repeated device — for tests with a stand-in RCCL loaded by fhh_rccl_load) — and reduced mod p once; prune applies the keep mask
 * to every shard; fhh_sim_crawl runs the device level loop per shard pair with the per-level
 * all-reduce over the same communicators. The reference server holds one such collection behind
 * its Mutex (src/bin/server.rs:44-52, 332-335). */
int fhh_create_multi(fhh_ctx** out, uint32_t data_len, uint32_t n_dims, const int* devices, int n_devices);
#define FHH_REDUCE_NONE 0   /* one shard                        */
#define FHH_REDUCE_HOST 1   /* partials summed on the host      */
#define FHH_REDUCE_RCCL 2   /* in-process RCCL all-reduce       */
/* Shard k of a collection (a one-GPU ctx is one shard): shard count, device, first client and
 * client count (0 before the keys are placed), and the reduction the collection uses. */
int fhh_shard_info(const fhh_ctx* ctx, int shard, int* n_shards, int* device, uint64_t* client_base,
                   uint64_t* n_clients, int* reduction);
/* The placement fhh_create_multi uses (host arithmetic, no device call): shard k of n_shards gets
 * clients [client_base[k], client_base[k] + n_clients[k]) = the 64-client words
 * [nw k / n_shards, nw (k + 1) / n_shards), nw = ceil(n / 64). */
int fhh_shard_plan(uint64_t n_clients, int n_shards, uint64_t* client_base, uint64_t* n_clients_out);
/* The one-GPU ctx of shard k (the ctx itself for a one-GPU ctx): per-shard calls such as the
 * two-party GC + OT below run on it — one channel per shard, as the reference splits a level's
 * tests over its channels (collect.rs:423-430). Owned by the collection. */
int fhh_shard_ctx(fhh_ctx* ctx, int shard, fhh_ctx** out);

/* Number of clients (len of `keys`). */
int fhh_num_clients(const fhh_ctx* ctx, uint64_t* n);

/* Copy this ctx's keys back in add_keys layout (for parity checks). Any pointer may be NULL. */
int fhh_export_keys(fhh_ctx* ctx, uint8_t* key_idx, uint8_t* root_seed, uint8_t* cw_seed, uint8_t* cw_bits);

/* ---- crawl ---------------------------------------------------------------------------- */

/* tree_init (collect.rs:67-92) with eval_init per key (ibDCF.rs:229-236). */
int fhh_tree_init(fhh_ctx* ctx);

/* Frontier expansion of tree_crawl (collect.rs:379-418): evaluates every client's 2d keys
 * one level for every child of every frontier node. *n_children = C. share_planes (may be
 * NULL) receives [C][2d][nw] u64 — the GC input of collect.rs:415-418.
 * If the previous crawl was not pruned, its children become the frontier (as
 * `self.frontier = next_frontier`, collect.rs:505). */
int fhh_tree_crawl(fhh_ctx* ctx, uint64_t* n_children, uint64_t* share_planes);
/* tree_crawl_last (collect.rs:775-823): same expansion; children become frontier_last. */
int fhh_tree_crawl_last(fhh_ctx* ctx, uint64_t* n_children, uint64_t* share_planes);

/* Per-node sums of the OT outputs (collect.rs:487-501): vals [C][n] (client order),
 * sums [C] canonical FE. */
int fhh_node_sums_fe(fhh_ctx* ctx, const uint64_t* vals, uint64_t* sums);
/* Last level (collect.rs:891-905) in FieldElm: vals [C][n][8] u32 little-endian limbs
 * (< 2^256). sums_unreduced [C][10] u32 LE = the exact BigUint `add_lazy` sum
 * (field.rs:337-339); sums_canonical [C][8] = mod 2^255-19. Either may be NULL. The sums
 * become the frontier_last values (collect.rs:909-914). */
int fhh_node_sums_fe255(fhh_ctx* ctx, const uint32_t* vals, uint32_t* sums_unreduced, uint32_t* sums_canonical);

/* Node sums of OT outputs that are already in device memory (no host round trip), e.g. the
 * outputs of the GPU OT extension. vals_dev[k] = shard k's values [C][ld] (ld >= the shard's
 * client count; 0 = each shard's client count) on shard k's GPU; a one-GPU ctx passes one
 * pointer. Formats: */
#define FHH_VALS_FE_U64 0           /* u64, any FE representation (FE::new)                       */
#define FHH_VALS_FE_BLOCK 1         /* 16-B OT blocks, the FE little-endian in bytes 0..7
                                       (FE <-> Block, fastfield.rs:414-431)                       */
#define FHH_VALS_FE255_LIMBS 2      /* 8 x u32 little-endian limbs (< 2^256)                      */
#define FHH_VALS_FE255_BLOCKPAIR 3  /* 2 x 16-B OT blocks: the value's 32 big-endian bytes
                                       (FieldElm <-> BlockPair, field.rs:465-492)                 */
int fhh_node_sums_fe_device(fhh_ctx* ctx, const void* const* vals_dev, uint64_t ld, uint32_t format, uint64_t* sums);
int fhh_node_sums_fe255_device(fhh_ctx* ctx, const void* const* vals_dev, uint64_t ld, uint32_t format,
                               uint32_t* sums_unreduced, uint32_t* sums_canonical);

/* tree_prune (collect.rs:918-929) / tree_prune_last (collect.rs:931-942). */
int fhh_tree_prune(fhh_ctx* ctx, const uint8_t* keep, uint64_t n);
int fhh_tree_prune_last(fhh_ctx* ctx, const uint8_t* keep, uint64_t n);

/* Current frontier size / frontier_last size. */
int fhh_frontier_size(const fhh_ctx* ctx, uint64_t* n_frontier, uint64_t* n_frontier_last);

/* final_shares (collect.rs:993-1005): paths [F][d][levels] (0/1) and values [F][10] u32
 * (the unreduced FieldElm sum recorded by fhh_node_sums_fe255 / fhh_sim_ot_sums, zeros if
 * none). *levels receives the path length. Pass NULL buffers to query F and levels. */
int fhh_final_shares(fhh_ctx* ctx, uint64_t* n_final, uint32_t* levels, uint8_t* paths, uint32_t* values);

/* Export the seeds/t/y of the current frontier's (or pending children's, if unpruned)
 * evaluation states in reference layout [node][client][d][2] (seed 16 B, t, y): parity aid
 * (EvalState, ibDCF.rs:24-30). Returns the node count in *n_nodes; NULL buffers = query. */
int fhh_export_states(fhh_ctx* ctx, uint64_t* n_nodes, uint8_t* seeds, uint8_t* t, uint8_t* y);

/* ---- leader-side helpers (pure host arithmetic) ----------------------------------------- */

/* keep_values (collect.rs:945-964): v = v0 - v1 mod p_FE; keep iff v >= threshold. */
int fhh_keep_values(uint64_t threshold, const uint64_t* vals0, const uint64_t* vals1, uint64_t n, uint8_t* keep);
/* keep_values_last (collect.rs:966-989) on FE255 values given as [n][10] u32 LE limbs. */
int fhh_keep_values_last(uint32_t threshold, const uint32_t* vals0, const uint32_t* vals1, uint64_t n, uint8_t* keep);
/* final_values (collect.rs:1007-1029): out [n][8] canonical (v0 - v1 mod p255). */
int fhh_final_values(const uint32_t* vals0, const uint32_t* vals1, uint64_t n, uint32_t* out);

/* ---- in-process two-server harness ----------------------------------------------------- */
/* The reference computes the "client inside node" bit with a garbled-circuit equality test
 * + OT between the servers (equalitytest.rs:25-106, collect.rs:419-482) — out of scope.
 * These entry points stand in for it when both servers' ctxs live in one process on the
 * same GPU: plaintext equality of the two share strings (eq = mask ^ out), or simulated OT
 * share values (r0 from a fixed PRF, r1 = r0 + 1; v0 = r1, v1 = eq ? r0 : r1). */

/* counts [C]: clients whose two share strings are equal, per pending child. */
int fhh_sim_eq_count(fhh_ctx* ctx0, fhh_ctx* ctx1, uint64_t* counts);
/* Simulated OT share sums. Non-last level: sums0/sums1 [C] canonical FE. After
 * tree_crawl_last: [C][10] u32 unreduced FE255 (also recorded as frontier_last values). */
int fhh_sim_ot_sums(fhh_ctx* ctx0, fhh_ctx* ctx1, uint64_t prf_seed, void* sums0, void* sums1);

/* All-reduce hook for client-sharded multi-GPU runs: called with a device buffer of
 * `count` u64 partial sums (on the ctx's GPU, already complete); must sum it in place
 * across ranks and return 0 once the result is visible to the device. */
typedef int (*fhh_allreduce_fn)(uint64_t* buf_dev, uint64_t count, void* user);

/* ---- native RCCL communicator (client-sharded multi-GPU) ----------------------
 * The per-level exchange of the reference is an RPC of Vec<FE> per server to the leader
 * (collect.rs:487-501 -> leader.rs:182-197); with clients sharded over GPUs it becomes one
 * ncclAllReduce(sum, u64) of the per-child partial sums, enqueued on the engine's stream so a
 * crawl needs no host round trip per level. RCCL is dlopen'ed (the copy the process already
 * loaded — e.g. torch's — is preferred so one RCCL instance serves the process). */
typedef struct fhh_comm fhh_comm;
/* Load RCCL: `path` NULL -> an already loaded librccl, else the default search path. */
int fhh_rccl_load(const char* path);
/* Rank 0 creates the id (128 bytes) and distributes it out of band (e.g. torch.distributed). */
int fhh_comm_unique_id(uint8_t id[128]);
int fhh_comm_create(fhh_comm** out, int nranks, int rank, const uint8_t id[128], int device);
void fhh_comm_destroy(fhh_comm* comm);
/* Sum count u64 from send_dev into recv_dev (may alias) across ranks, on `stream`
 * (hipStream_t; NULL = the null stream). Asynchronous. */
int fhh_comm_allreduce_u64(fhh_comm* comm, const uint64_t* send_dev, uint64_t* recv_dev, uint64_t count,
                           void* stream);
/* A communicator without RCCL: fhh_comm_allreduce_u64 and the level loop's cfg->comm path
 * drain the stream, copy the partials to a host buffer, call fn(host_buf, count, user) to sum
 * them in place across ranks (e.g. over gloo), and copy the result back. For tests of the
 * comm path where RCCL ranks are not available (one GPU shared by several ranks). */
int fhh_comm_create_hosted(fhh_comm** out, int nranks, int rank, int device, fhh_allreduce_fn fn, void* user);
/* The rank count and rank RCCL itself reports for the communicator (ncclCommCount /
 * ncclCommUserRank) — what the bench records as the ranks the collective saw. */
int fhh_comm_info(fhh_comm* comm, int* nranks, int* rank);
/* Last error of the calling thread's fhh_rccl_* / fhh_comm_* call. */
const char* fhh_comm_last_error(void);

typedef struct fhh_sim_config {
    double threshold;          /* fraction, leader.rs:193-194 / 245-246             */
    uint64_t nclients_total;   /* nreqs (all ranks)                                   */
    uint32_t mode;             /* 0 = eq count, 1 = simulated OT shares (FE / FE255) */
    uint32_t levels;           /* 0 = data_len                                        */
    uint64_t prf_seed;         /* mode 1                                              */
    fhh_allreduce_fn allreduce;/* NULL on a single GPU                               */
    void* allreduce_user;
    uint64_t* xchg_dev;        /* device buffer handed to allreduce (>= capacity u64) */
    uint64_t xchg_capacity;
    /* optional per-level records (NULL to skip) */
    uint64_t* level_children;  /* [levels] */
    uint64_t* level_kept;      /* [levels] */
    uint64_t* counts;          /* concatenated per-level child counts/values (mode 0) */
    uint64_t counts_capacity;
    /* 0 (default): device-resident level loop — keep decision and prune run on the GPU and
     * the whole crawl is enqueued without per-level host round trips; 1: host-driven loop
     * (the same sequence the drop-in entry points perform). Identical results. */
    uint32_t host_loop;
    /* device loop: initial frontier / per-dim entry capacity (0 = 256); buffers grow on
     * demand (the loop pauses, grows, and resumes at the level that overflowed). */
    uint32_t init_capacity;
    /* native RCCL communicator (takes precedence over `allreduce`): the per-level sum is
     * ncclAllReduce on ctx0's stream, no host synchronisation per level. NULL on one GPU. */
    fhh_comm* comm;
    /* mode 1, device loop: the per-(child, client) equality bit comes from the garbled-circuit
     * equality test on the GPU (fhh_gc_*: server 0 garbles its share planes, server 1
     * evaluates), as tree_crawl does with gc_sender (collect.rs:419-482). 1 = the OTs (the
     * evaluator's input labels, the FE share conversion) are ideal; 2 = both run as GPU correlated
     * OT extension (fhh_cot_extend_host's modes: the labels as FHH_COT_RAW with the labels session's
     * s as Delta, the share as FHH_COT_FE / FHH_COT_FE255, a FieldElm share as a BlockPair = 2 OTs).
     * 2 takes the FE levels' test (2d <= 4) as one garbled table (fhh_gt_cot_host, r05d); 3 = 2 with
     * the half-gates circuit + output-label share (fhh_gc_cot_host's share outputs, r05c) at every FE
     * level instead. Same sums as 0. Material from prf_seed (a harness, not private): the mask fresh per chunk of
     * children; one base-OT session per level and OT kind, each chunk on its own row-PRG counter
     * range; gate tweaks carry the level (bits 40+). */
    uint32_t gc;
    /* parity probe of the device loop (tests; probe_n_levels = 0 disables it): right after level
     * probe_levels[k]'s k_expand, the pending children's EvalStates (ibDCF.rs:24-30) of the
     * local clients probe_clients[0..probe_n_clients) are gathered from both servers' tables.
     *   probe_seeds    [probe_n_levels][2 server][probe_capacity][probe_n_clients][d][2 side][16]
     *   probe_ty       [probe_n_levels][2][probe_capacity][probe_n_clients][d][2]: bit0 t, bit1 y
     *   probe_children [probe_n_levels]: C of that level (children past probe_capacity are not
     *                  copied; the caller checks C <= capacity)
     * Child order is the crawl's (parent order x all_bit_vectors), as fhh_export_states. The
     * gather is a separate kernel between k_expand and the count: the timed path is unchanged. */
    uint32_t probe_n_levels;   /* <= 16 */
    uint32_t probe_n_clients;
    const uint32_t* probe_levels;
    const uint64_t* probe_clients;
    uint64_t probe_capacity;
    uint8_t* probe_seeds;
    uint8_t* probe_ty;
    uint64_t* probe_children;
    /* gc = 2: 0 = ideal base OTs (seed pairs derived on the device per level); 1 = real base OTs:
     * Chou–Orlandi (fhh_base_ot_co15), a fresh instance for each of the 2 OT kinds of every level
     * (the evaluator's labels, then the FE / FieldElm share conversion), produced by a pool of host
     * threads (OMP_NUM_THREADS) a few levels ahead of the GPU (fhh_stats.base_ot_ms: their compute
     * time; base_ot_stall_ms: the time the loop waited for them) and uploaded as key schedules
     * before the level's OTs. */
    uint32_t base_ot;
    /* gc >= 2 (r06): the OT extension of both OT kinds — 0 or 1 = IKNP (128 rows of U: 16 B per OT on the
     * wire), 2 or 4 = SoftSpoken with k = ot_ss_k (fhh_cot_extend_ss_host: 128 / k rows, 16 / k B per OT,
     * 2^k - 1 ChaCha12 blocks per chunk and tile at the sender). Same sums. */
    uint32_t ot_ss_k;
    /* gc = 2, d = 1 (r06): 1 = the FE levels' garbled table carries its shares in Z_2^32 instead of FE (4-B
     * rows instead of 8: the per-child v0 - v1 is the count either way, < 2^32; the FieldElm level is
     * unchanged). Same sums, keep decisions and heavy hitters. */
    uint32_t table_ring32;
} fhh_sim_config;

/* Full leader level loop (leader.rs:417-440) over both servers: tree_init, L-1 x
 * (crawl, count/sums, [allreduce], keep_values, prune), crawl_last, keep_values_last,
 * prune_last. Heavy hitters are then read with fhh_final_shares(ctx0, ...). */
int fhh_sim_crawl(fhh_ctx* ctx0, fhh_ctx* ctx1, const fhh_sim_config* cfg);

/* ---- sketch + Beaver-triple verification ------------------------------
 * SketchDPFKey::sketch_at (src/sketch.rs:157-200) and MulState (src/mpc.rs:83-220), for
 * T = FE. Both files are fully commented out in the reference (parity unpinned beyond the
 * protocol's identities). FE values may be passed in any u64 representation; every output is
 * canonical. One key = one client's vector over the frontier: x[key][node], kx[key][node]
 * (the (x, k.x) pairs `vector_in` of sketch_at), with the key's rand_stream given as the
 * PrgStream seed (AES-128-CTR, key = seed, IV 0: PrgSeed::to_rng, prg.rs:82-90).
 * sketch6 per key = {r_x, r2_x, r_kx, rand1, rand2, rand3} (SketchOutput, sketch.rs:27-42).
 * triples9 per key = the level's 3 TripleShares {a, b, c} (mpc.rs:18-45). */

/* sketch_at for n_keys keys (host buffers: seeds [n][16], x / kx [n][n_nodes], out [n][6]). */
int fhh_sketch_at_fe(fhh_ctx* ctx, uint64_t n_keys, uint32_t n_nodes, const uint8_t* seeds, const uint64_t* x,
                     const uint64_t* kx, uint64_t* sketch6);
/* MulState::new + cor_share (mpc.rs:83-158): cor_share6 [n][6] = {d0, d1, d2, e0, e1, e2}. */
int fhh_mul_cor_share_fe(fhh_ctx* ctx, uint64_t n, const uint64_t* sketch6, const uint64_t* mac_key,
                         const uint64_t* mac_key2, const uint64_t* triples9, uint64_t* cor_share6);
/* MulState::cor (mpc.rs:160-180): cor6 = share0 + share1 (host arithmetic). */
int fhh_mul_cor_fe(uint64_t n, const uint64_t* share0, const uint64_t* share1, uint64_t* cor6);
/* MulState::out_share (mpc.rs:182-212); server_idx 1 adds d*e. out [n]. */
int fhh_mul_out_share_fe(fhh_ctx* ctx, int server_idx, uint64_t n, const uint64_t* sketch6, const uint64_t* mac_key,
                         const uint64_t* mac_key2, const uint64_t* triples9, const uint64_t* cor6, uint64_t* out);
/* MulState::verify (mpc.rs:214-220): ok[i] = out0[i] + out1[i] == 0 (host arithmetic). */
int fhh_mul_verify_fe(uint64_t n, const uint64_t* out0, const uint64_t* out1, uint8_t* ok);

/* In-process leader + both servers, device-resident batch (main.rs:14-70 verify_sketches):
 * both servers' sketch_at, cor shares, cor, out shares, verify. All pointers are device
 * pointers on ctx's GPU; synchronous. */
typedef struct fhh_sketch_batch {
    uint64_t n_keys;
    uint32_t n_nodes;
    uint32_t force_sequential;        /* 1: sequential-stream path for every key (tests)   */
    const uint8_t* seeds_dev;         /* [n][16], the same stream seeds on both servers    */
    const uint64_t* x_dev[2];         /* per server [n][n_nodes]                           */
    const uint64_t* kx_dev[2];
    const uint64_t* mac_dev[2];       /* [n] shares of the MAC key k                       */
    const uint64_t* mac2_dev[2];      /* [n] shares of k^2                                 */
    const uint64_t* triples_dev[2];   /* [n][9]                                            */
    uint64_t* sketch_dev[2];          /* out [n][6] (the last level verified)              */
    uint8_t* ok_dev;                  /* out [n_levels][n]                                 */
    uint64_t* out_shares_dev;         /* out [n_levels][2][n] or NULL                      */
    /* level batching (main.rs:14-70 runs verify_sketches once per level; SketchDPFKey::triples
     * holds TRIPLES_PER_LEVEL = 3 per level, sketch.rs:120-126, and MulState::new takes
     * triples[3 level .. 3 level + 3], mpc.rs:94-98): levels [level, level + n_levels) in one call. */
    uint32_t level;                   /* first level                                       */
    uint32_t n_levels;                /* 0 = 1                                             */
    uint32_t triples_levels;          /* triples_dev is [n][triples_levels][9] (0 = 1)     */
    uint32_t pad_;
    uint64_t x_level_stride;          /* elements between levels' x / kx (0: same vectors) */
} fhh_sketch_batch;
/* Level l's PrgStream seed is the key's seed with bytes 12..15 XORed with l (little-endian; level 0
 * = the seed itself): a harness convention — the reference's rand_stream is a collection-wide
 * stream (collect.rs:35,57) whose per-level use is in the absent dpf/sketch glue. */
int fhh_sim_sketch_verify_fe(fhh_ctx* ctx, const fhh_sketch_batch* batch);

/* Leader-side dealer for benches / tests: TripleShare::new (mpc.rs:18-45) for n keys x levels x
 * TRIPLES_PER_LEVEL, both servers' shares written to device buffers [n][levels][9] (a, b, c per
 * triple; a = a0 + a1, b = b0 + b1, c0 + c1 = a b). Randomness: a mix64 PRF of seed (the
 * reference draws thread_rng). */
int fhh_deal_triples_fe(fhh_ctx* ctx, uint64_t n, uint32_t levels, uint64_t seed, uint64_t* triples0_dev,
                        uint64_t* triples1_dev);
/* k_sketch_fe implementation for A/B (process-wide): 0 = default (four-table LDS layout, 1024
 * threads, each key's round keys computed once into LDS, lanes per key chosen per launch by
 * fhh_sketch_plan; the plan's tail launch in the producer / consumer form), 1 = the r01 kernel
 * (schedule in registers, 256 threads), 2 = 8 lanes per key with the round keys expanded on the fly
 * per pass, 3 = 0 at 8 lanes per key for every key, 4 = the producer / consumer form for every key
 * (AES waves and product waves paired through LDS). All are bit-identical; FHH_E_ARG for any other
 * value. */
int fhh_sketch_set_impl(int impl);
/* The default form's launch plan for n_keys keys of n_nodes nodes on `resident_waves` waves (CUs x
 * 16 on MI355X): keys [0, *n_main) run at *lpk_main lanes per key, the rest in a second launch at
 * *lpk_tail (host-only arithmetic, no device call). */
int fhh_sketch_plan(uint64_t n_keys, uint32_t n_nodes, uint64_t resident_waves, uint64_t* n_main, int* lpk_main,
                    int* lpk_tail);

/* ---- the last level, U = FieldElm (sketch_at_last, sketch.rs:202-245; MulState<FieldElm>) ----
 * FieldElm values are 8 x u32 little-endian limbs (any value < 2^256 is accepted as input, reduced
 * mod p = 2^255 - 19; outputs canonical). FieldElm::from_rng = num-bigint 0.3.3
 * gen_biguint_below(p) (field.rs:367-372): 32 stream bytes per attempt as 8 LE u32 digits, the top
 * digit >> 1, redrawn while >= p — num-bigint is not vendored: this digit order is an ASSUMPTION
 * (parity unpinned). sketch6 [n][6][8], mac / mac2 [n][8], triples9 [n][9][8]
 * (triples_last: 3 TripleShares {a, b, c}), cor_share6 / cor6 [n][6][8], out [n][8]. */
int fhh_sketch_at_fe255(fhh_ctx* ctx, uint64_t n_keys, uint32_t n_nodes, const uint8_t* seeds, const uint32_t* x,
                        const uint32_t* kx, uint32_t* sketch6);
int fhh_mul_cor_share_fe255(fhh_ctx* ctx, uint64_t n, const uint32_t* sketch6, const uint32_t* mac_key,
                            const uint32_t* mac_key2, const uint32_t* triples9, uint32_t* cor_share6);
int fhh_mul_cor_fe255(uint64_t n, const uint32_t* share0, const uint32_t* share1, uint32_t* cor6);
int fhh_mul_out_share_fe255(fhh_ctx* ctx, int server_idx, uint64_t n, const uint32_t* sketch6,
                            const uint32_t* mac_key, const uint32_t* mac_key2, const uint32_t* triples9,
                            const uint32_t* cor6, uint32_t* out);
int fhh_mul_verify_fe255(uint64_t n, const uint32_t* out0, const uint32_t* out1, uint8_t* ok);
typedef struct fhh_sketch_batch255 {
    uint64_t n_keys;
    uint32_t n_nodes;
    uint32_t force_sequential;
    const uint8_t* seeds_dev;         /* [n][16]                                           */
    const uint32_t* x_dev[2];         /* per server [n][n_nodes][8]                        */
    const uint32_t* kx_dev[2];
    const uint32_t* mac_dev[2];       /* [n][8] shares of mac_key_last                     */
    const uint32_t* mac2_dev[2];      /* [n][8] shares of mac_key2_last                    */
    const uint32_t* triples_dev[2];   /* [n][9][8] triples_last                            */
    uint32_t* sketch_dev[2];          /* out [n][6][8]                                     */
    uint8_t* ok_dev;                  /* out [n]                                           */
    uint32_t* out_shares_dev;         /* out [2][n][8] or NULL                             */
    uint32_t level;                   /* stream seed = seed with bytes 12..15 ^= level     */
    uint32_t pad_;
} fhh_sketch_batch255;
int fhh_sim_sketch_verify_fe255(fhh_ctx* ctx, const fhh_sketch_batch255* batch);

/* ---- garbled-circuit equality test -------------------------------------
 * multiple_gb_equality_test / multiple_ev_equality_test (equalitytest.rs:25-219): per test,
 * eq = AND_j NOT(x_j XOR y_j) over `bits` share bits, revealed to the evaluator as eq XOR mask.
 * Free-XOR + half-gates, hash TCCR(x, i) = pi(pi(x) ^ i) ^ pi(x) with pi = AES-128 under the
 * all-zero key (swanky's fixed key and wire format are not restatable: DESIGN.md §5.3). Labels
 * are 16-B blocks, colour = bit 0 of byte 0; the garbler's zero label of wire w of test t is
 * AES_label_key(LE128(label_nonce + t S + w)) with S the power of two >= 2 bits + 1 (w < bits: its
 * string, w = bits: the mask, w > bits: the evaluator's string; a label_nonce that is a multiple of
 * S lets the kernel share AES rounds 1-2 between a test's label blocks); AND gate k of test t has tweaks 2 g, 2 g + 1 with
 * g = gate_base + t (bits - 1) + k. Tests t = g N + i (g < groups, i < clients); inputs are bit
 * planes [groups][bits][words] (bit i % 64 of word i / 64, as fhh_tree_crawl's share planes);
 * outputs are SoA over t: tables [(bits-1) * 2][t] (T_G, T_E), gb_labels [bits + 1][t] (the
 * garbler's active labels, mask last), ev_labels [bits][t] (the evaluator's active labels — the
 * output of an ideal OT; a deployment runs OT extension instead), decode [t], out [t]. The
 * reference draws one mask per call (`rng.clone().gen_bool()`, equalitytest.rs:38-43, the clone
 * never advances), so `mask` is one bit for the whole batch. */
typedef struct fhh_gc_batch {
    uint64_t groups;
    uint32_t clients;              /* tests per group                                      */
    uint32_t words;                /* plane words per (group, bit), >= ceil(clients / 64)  */
    uint32_t bits;                 /* string length (2d), 1..8                             */
    uint32_t mask;                 /* garbler's mask bit                                   */
    uint8_t label_key[16];         /* garbler's label PRG key                              */
    uint8_t delta[16];             /* free-XOR offset (bit 0 is forced to 1)               */
    uint64_t label_nonce;
    uint64_t gate_base;
    const uint64_t* gb_planes_dev; /* garbler's bits   [groups][bits][words]               */
    const uint64_t* ev_planes_dev; /* evaluator's bits [groups][bits][words]               */
    uint8_t* tables_dev;           /* [(bits - 1) * 2][groups * clients][16]               */
    uint8_t* gb_labels_dev;        /* [bits + 1][groups * clients][16]                     */
    uint8_t* ev_labels_dev;        /* [bits][groups * clients][16]                         */
    uint8_t* decode_dev;           /* [groups * clients]                                   */
    uint8_t* out_dev;              /* [groups * clients] evaluator's eq XOR mask           */
} fhh_gc_batch;
/* Garbler then evaluator on ctx's stream (device buffers); returns after both finish. */
int fhh_gc_equality_device(fhh_ctx* ctx, const fhh_gc_batch* batch);
/* The same on host buffers, one group: gb_bits / ev_bits [n][bits] (0/1 bytes); outputs AoS
 * (tables [n][bits-1][2][16], gb_labels [n][bits+1][16], ev_labels [n][bits][16], decode [n],
 * out [n]); any output but `out` may be NULL. */
int fhh_gc_equality_host(fhh_ctx* ctx, uint64_t n, uint32_t bits, const uint8_t* gb_bits, const uint8_t* ev_bits,
                         uint32_t mask, const uint8_t label_key[16], const uint8_t delta[16], uint64_t label_nonce,
                         uint64_t gate_base, uint8_t* tables, uint8_t* gb_labels, uint8_t* ev_labels,
                         uint8_t* decode, uint8_t* out);

/* ---- OT extension (the OT of row f1) -------------------------------------------------------
 * IKNP OT extension in the ALSZ form, the protocol of ocelot's AlszSender / AlszReceiver that
 * the reference runs for the evaluator's input labels (equalitytest.rs:67-82) and the FE share
 * conversion (collect.rs:437-471): m 1-out-of-2 OTs of 16-B messages; the receiver gets
 * x_j^{choice_j}. kappa = 128 base OTs are ideal (the receiver's seed pairs base_seeds[i][0..1],
 * the sender's choice bits base_choice; the sender is handed base_seeds[i][s_i]). G = AES-128-CTR
 * under each seed (block c = LE128(c) gives OTs 128 c .. 128 c + 127, bit b of byte b / 8),
 * H(j, x) = scuttlebutt's cr_hash(j, x) = pi(x) ^ x, pi = AES-128 under the zero key (the hash
 * ocelot's ALSZ applies; j is not an input, so tweak_base is accepted and ignored).
 * x1 == NULL: correlated OT, x1 = x0 ^ delta.
 * The base material (base_seeds, base_choice) MUST be fresh for every batch — the reference
 * re-runs OtSender/OtReceiver::init per batch (collect.rs:454-471) — because the row PRG restarts
 * at counter 0: two batches on the same material repeat the pads, and U ^ U' reveals r ^ r'.
 * Device buffers: the call runs on the ctx's own (non-blocking) stream, so choices_dev / x0_dev /
 * x1_dev must be complete when it is made (synchronise the stream that produced them); it returns
 * after out_dev is complete. */
typedef struct fhh_ot_batch {
    uint64_t m;
    const uint32_t* choices_dev;    /* receiver's choice bits, bit j % 32 of word j / 32       */
    const uint8_t* x0_dev;          /* sender's messages [m][16] for choice 0                  */
    const uint8_t* x1_dev;          /* [m][16] for choice 1, or NULL (x0 ^ delta)              */
    uint8_t delta[16];
    uint8_t* out_dev;               /* receiver's messages [m][16]                             */
    uint8_t base_seeds[128][2][16];
    uint8_t base_choice[16];
    uint64_t tweak_base;            /* ignored by cr_hash (kept for ABI stability)             */
} fhh_ot_batch;
int fhh_ot_extend_device(fhh_ctx* ctx, const fhh_ot_batch* batch);
/* Host buffers: choices [m] 0/1 bytes; optional transcript u_out [128][ceil(m/128)][16] (the
 * receiver's message to the sender), y0_out / y1_out [m][16] (the sender's reply). */
int fhh_ot_extend_host(fhh_ctx* ctx, uint64_t m, const uint8_t* choices, const uint8_t* x0, const uint8_t* x1,
                       const uint8_t delta[16], const uint8_t base_seeds[128 * 2 * 16], const uint8_t base_choice[16],
                       uint64_t tweak_base, uint8_t* out, uint8_t* u_out, uint8_t* y0_out, uint8_t* y1_out);

/* ---- correlated OT extension (r05: the protocol's two OTs) ----------------------------------
 * The reference moves the evaluator's input labels (equalitytest.rs:67-82) and the FE shares
 * (collect.rs:437-471) with plain OTs of two chosen messages. Both pairs are correlated — labels
 * (x, x ^ Delta), shares (r, r +- 1) — so the build runs them as ALSZ correlated OT (ocelot's
 * AlszSender::send_correlated): the sender's first message is the hash itself, x0_j = H(q_j), and
 * only y_j = f(x0_j) ^ H(q_j ^ s) crosses. That removes the garbler's evaluator-label blocks, the
 * share PRF and half of each reply. Modes (oracle/fhh_oracle.c orc_cot_extend is the restatement):
 *   FHH_COT_LABELS  x1 = x0 ^ delta; y 16 B; out = r ? y ^ H(t) : H(t); sender_out = x0 [m][16]
 *   FHH_COT_FE      v = H(q_j) as a little-endian u128 mod p_FE; the garbler's pair is ordered by
 *                   its mask as collect.rs:447-451 orders (r0, r1): pair[0] = v, pair[1] = mask ?
 *                   v + 1 : v - 1, its node value r1 = v + mask (sender_out [m] u64); y = lo64(H(q_j
 *                   ^ s)) ^ pair[1] (8 B); out [m] u64 = r ? lo64(y ^ H(t)) : H(t) mod p
 *   FHH_COT_FE255   a test is the OT pair (2t, 2t + 1) with one choice (m even): V = the 32 big-endian
 *                   bytes H(q_2t) || H(q_2t+1) mod p255, pair[1] = mask ? V + 1 : V - 1 as a BlockPair
 *                   (field.rs:478-492); sender_out [m/2][32] = V + mask; y 16 B per OT; out [m/2][32]
 *                   = r ? y ^ H(t) : H(t), the raw BlockPair FieldElm::try_from reads unreduced
 *                   (field.rs:466-476)
 *   FHH_COT_RAW     (r05b, the labels OT since) the IKNP correlation itself: sender_out [m][16] = q_j,
 *                   out [m][16] = t_j = q_j ^ r_j s, no hash and no y (y_out unused). With the
 *                   sender's s as the free-XOR Delta (bit 0 of byte 0 set), q_j is the zero label of
 *                   the evaluator's input wire j and t_j its active label: the random correlated OT
 *                   that free-XOR garbling consumes (delta, mask unused).
 * ctr_off: the row PRG's first block (a multiple of 256): batches that extend one set of base OTs
 * must use disjoint counter ranges (the party ABI below keeps a running counter per session).
 * Host buffers: choices [m] 0/1 bytes; u_out [128][ceil(m/128)][16]; y_out [m][8 or 16]. */
#define FHH_COT_LABELS 1
#define FHH_COT_FE 2
#define FHH_COT_FE255 3
#define FHH_COT_RAW 4
int fhh_cot_extend_host(fhh_ctx* ctx, uint64_t m, uint32_t mode, const uint8_t* choices, const uint8_t delta[16],
                        uint32_t mask, const uint8_t base_seeds[128 * 2 * 16], const uint8_t base_choice[16],
                        uint64_t ctr_off, uint8_t* sender_out, uint8_t* out, uint8_t* u_out, uint8_t* y_out);
/* r06: the same on SoftSpoken OT extension (Roy, CRYPTO 2022; semi-honest small-field VOLE, repetition code)
 * with k = ss_k base OTs per chunk (1 = IKNP, exactly fhh_cot_extend_host; 2, 4): chunk c's k base OTs
 * become a (2^k - 1)-out-of-2^k OT of GGM leaf seeds, and the receiver's message U has 128 / k rows
 * (u_out [128 / ss_k][ceil(m / 128)][16]: 16 / k bytes per OT instead of 16) plus the GGM corrections
 * corr_out [128 / ss_k][ss_k][2][16] (4 KiB per base-OT session). The correlation q_j = t_j ^ r_j s with
 * s = base_choice is IKNP's, so the modes are unchanged. Restated in oracle/fhh_oracle.c cot_rows / ss_ggm
 * (tree PRG, masks and root derivation there). */
int fhh_cot_extend_ss_host(fhh_ctx* ctx, uint32_t ss_k, uint64_t m, uint32_t mode, const uint8_t* choices,
                           const uint8_t delta[16], uint32_t mask, const uint8_t base_seeds[128 * 2 * 16],
                           const uint8_t base_choice[16], uint64_t ctr_off, uint8_t* sender_out, uint8_t* out,
                           uint8_t* u_out, uint8_t* y_out, uint8_t* corr_out);
/* The labels step of one batch on host buffers: the labels OT (FHH_COT_RAW since r05b: choice bits =
 * the evaluator's bits at OT index j npad + i, npad = n rounded up to 64; the evaluator's zero labels
 * E_j = q_j, its active labels t_j, Delta = the sender's s, whose bit 0 must be 1), garbling with the
 * garbler's string and mask FOLDED into the circuit — the garbler knows x_j, so input z_j = NOT(x_j ^
 * y_j) takes the zero label E_j ^ (x_j ? 0 : Delta) and the evaluator's OT'd label is z_j's active
 * label; decode = colour(eq's zero label) ^ mask — and evaluation on the OT'd labels (out = colour ^
 * decode = eq ^ mask). No label PRG, no garbler labels and no labels-OT reply on the wire; gate tweaks
 * 2 g, 2 g + 1 with g = gate_base + t (bits - 1) + k as in fhh_gc_batch. Outputs AoS: tables
 * [n][bits-1][2][16], ev_zero / ev_active [n][bits][16], decode [n], out [n]; any but `out` may be
 * NULL. r05c, the FE share from the output labels (the party ABI's FE levels): with gb_share, ev_share
 * and share_y (uint64_t[n] each, all three or none) the garbler also forms the share pair from the
 * labels of o = eq ^ mask — W_0 (o = 0) and W_1 = W_0 ^ Delta in the roles of the share C-OT's q_j and
 * q_j ^ s: v = H(W_0) as a LE u128 mod p, node value r1 = v + mask (gb_share), y = lo64(H(W_1)) ^
 * (mask ? v + 1 : v - 1) (share_y, 8 B per test) — and the evaluator its node value from W_o: o ?
 * lo64(H(W_o)) ^ y : H(W_o) mod p (ev_share). H = cr_hash; gb_share - ev_share = eq ^ ... = the
 * test's equality bit mod p, as FHH_COT_FE gives it. */
int fhh_gc_cot_host(fhh_ctx* ctx, uint64_t n, uint32_t bits, const uint8_t* gb_bits, const uint8_t* ev_bits,
                    uint32_t mask, uint64_t gate_base, const uint8_t base_seeds[128 * 2 * 16],
                    const uint8_t base_choice[16], uint64_t ctr_off, uint8_t* tables, uint8_t* ev_zero,
                    uint8_t* ev_active, uint8_t* decode, uint8_t* out, uint64_t* gb_share, uint64_t* ev_share,
                    uint64_t* share_y);

/* r05d: the FE levels' garbled TABLE on host buffers (bits <= 4): the labels OT as in fhh_gc_cot_host,
 * then one garbled b-input gate instead of the half-gates chain + output-label share — Yao's garbled
 * gate with point-and-permute for "the share of eq ^ mask": the inputs are the folded garbler's zero
 * labels Z_k = q_k ^ (x_k ? 0 : Delta); the evaluator's OT'd t_k is z_k's active label and the colours
 * lsb(t_k) name its row r; row r's key is cr_hash(K_r), K_r = XOR_k sigma^k(z_k's label in row r) ^
 * (gate_base + t) (sigma = doubling in GF(2^128), x^128 + x^7 + x^2 + x + 1, block as LE u128); the
 * values are the share C-OT's pair (pair[0] = v, pair[1] = mask ? v + 1 : v - 1; the garbler's node
 * value r1 = v + mask) with pair[o_r], o_r = eq_r ^ mask; row 0's value is its hash mod p (no
 * message), rows 1 .. 2^b - 1 send lo64(hash) ^ pair[o_r]. Outputs: msgs [n][2^bits - 1] u64 (may be
 * NULL), gb_share / ev_share [n] (r1 and the evaluator's value: gb - ev = eq mod p), ev_zero /
 * ev_active [n][bits][16] (may be NULL). Garbler 2^b AES per test, evaluator 1. The labels OT's index
 * is k npad + i with npad = n rounded up to 64 (b = 3, 4) or, since r06, to 512 (b <= 2: the table kernels
 * read the OT's tile-major matrices, whose 512-OT tiles must hold one client range per bit). */
int fhh_gt_cot_host(fhh_ctx* ctx, uint64_t n, uint32_t bits, const uint8_t* gb_bits, const uint8_t* ev_bits,
                    uint32_t mask, uint64_t gate_base, const uint8_t base_seeds[128 * 2 * 16],
                    const uint8_t base_choice[16], uint64_t ctr_off, uint8_t* ev_zero, uint8_t* ev_active,
                    uint64_t* msgs, uint64_t* gb_share, uint64_t* ev_share);
/* r06: the same table with its shares in Z_2^32 (bits <= 2; fhh_sim_config.table_ring32's form): row 0's value
 * is lo32 of its hash, pair = (v, v +- 1 mod 2^32), rows 1 .. 2^b - 1 send lo32(hash) ^ pair[o_r] (4 B);
 * msgs / gb_share / ev_share as above, each value zero-extended to u64 (gb - ev = eq mod 2^32). Oracle:
 * orc_gt_garble_ring32 / orc_gt_eval_ring32. */
int fhh_gt_cot_ring32_host(fhh_ctx* ctx, uint64_t n, uint32_t bits, const uint8_t* gb_bits, const uint8_t* ev_bits,
                           uint32_t mask, uint64_t gate_base, const uint8_t base_seeds[128 * 2 * 16],
                           const uint8_t base_choice[16], uint64_t ctr_off, uint8_t* ev_zero, uint8_t* ev_active,
                           uint64_t* msgs, uint64_t* gb_share, uint64_t* ev_share);

/* ---- the two servers' halves of a level's GC + OT (row f1 split by party) ---------------------
 * tree_crawl with gc_sender = true on server 0 and false on server 1 (collect.rs:419-482;
 * equalitytest.rs:25-106): each server runs only its own half on its own ctx, right after its
 * fhh_tree_crawl / fhh_tree_crawl_last, with only its OWN secrets — the garbler's fhh_gb_cfg and the
 * evaluator's fhh_ev_cfg share nothing (each server draws its material itself: AesRng::new() per
 * channel, collect.rs:431; base OTs by fhh_co15_* over the channel, OtSender / OtReceiver::init,
 * collect.rs:454,460). Four byte buffers cross per chunk, in this order (y1 has 0 bytes since r05b; at
 * the FE levels u2 and y2 have 0 bytes too since r05c — the share rides in gc — so two carry data):
 *   server 0 (garbler, OT sender)                          server 1 (evaluator, OT receiver)
 *                                      <--------------  fhh_ev_ot_labels(ev_cfg) -> u1
 *   fhh_gb_ot_labels(gb_cfg, u1) -> y1 (empty)
 *   fhh_gb_garble -> gc               -------------->   fhh_ev_evaluate(gc, y1) -> u2
 *   fhh_gb_ot_shares(u2) -> y2        -------------->   fhh_ev_ot_shares(y2)
 *   fhh_party_node_sums                                  fhh_party_node_sums
 * Outputs are device buffers owned by the producing ctx, valid until its next party call; inputs are
 * device pointers on the receiving ctx's GPU (the caller moves the bytes: a network in a deployment, a
 * device copy in the in-process tests). OT 1 (FHH_COT_RAW) delivers the evaluator's input labels
 * (m = C x 2d x npad: its share planes are the choice bits; the garbler's labels-kind s is the
 * circuit's Delta, so no reply crosses). The share: at the FE levels (r05c) from the circuit's output
 * labels (fhh_gc_cot_host's share outputs: the garbler's r1 and y from W_0, W_0 ^ Delta, the evaluator's
 * value from its W_o) — and since r05d, for 2d <= 4, from one garbled table per test (fhh_gt_cot_host)
 * — so no second OT runs and the OT kind 1 base material is not read; at tree_crawl_last by OT 2
 * (FHH_COT_FE255: 2 OTs per test). The circuit is fhh_gc_cot_host's (the garbler's string and mask
 * folded in). gc at the FE levels, 2d <= 4: the table's rows 1 .. 2^(2d) - 1, 8 B each, SoA
 * [row][tests]; otherwise [tables (bits-1) x 2 | y 8 B (FE levels) | decode 1 B] per test; tests =
 * C x n child-major; u = the OT receiver's [128][m padded to 8192 / 128] blocks;
 * y1 0 B; u2 / y2: 0 B at the FE levels, FieldElm level: U and 16 B per OT. Each server's node values
 * (the garbler's r1 = v + mask, the evaluator's share output) stay on its device; fhh_party_node_sums sums them: non-last
 * level sums [C] canonical FE, last level [C][10] unreduced + [C][8] canonical FieldElm (the
 * frontier_last values). For a multi-device ctx run each shard (fhh_shard_ctx) with its own channel,
 * as the reference runs a level's tests over several channels (collect.rs:423-430).
 * Chunks of children: child_count > 0 runs the protocol for children [child_begin, child_begin +
 * child_count) only (C above = the chunk's children) — one protocol instance per chunk, as the
 * reference's channels each run a slice of the level's tests (collect.rs:423-430); this bounds the
 * level's buffers at 1M clients. Chunks run in order and together cover [0, C); fhh_party_node_sums
 * follows the last one. Both parties must use the same windows. child_count = 0: the whole level.
 * Freshness: Delta is the labels session's s (fresh with each base-OT run: run the base OTs per level,
 * as the reference's init per channel does); the mask should be fresh per chunk (gate tweaks are indexed
 * by the test's index in the whole level). Base OTs may be reused across chunks: each
 * ctx keeps, per OT kind, the running row-PRG counter of the base material it last saw and continues
 * it while the material is unchanged (a new set starts at 0), so pads never repeat. */
typedef struct fhh_gb_cfg {
    uint32_t mask;                       /* the chunk's mask bit (equalitytest.rs:38-43)           */
    uint32_t form;                       /* FE levels: 0 = the garbled table where 2d <= 4 (r05d),
                                            1 = the half-gates circuit (r05c); both parties alike  */
    uint8_t base_chosen[2][128][16];     /* per OT kind (0 labels, 1 shares — read at tree_crawl_last
                                            only since r05c): k_i^{s_i} from the                    */
    uint8_t base_choice[2][16];          /* base OTs, and s (bit i % 8 of byte i / 8); the labels
                                            kind's s is the free-XOR Delta: its bit 0 must be 1   */
    uint64_t child_begin;
    uint64_t child_count;
    uint32_t ot_ss_k;                    /* r06: the OT extension of both kinds, as the evaluator's:
                                            0 / 1 IKNP, 2 / 4 SoftSpoken (fhh_cot_extend_ss_host) */
    uint32_t pad_;
} fhh_gb_cfg;
typedef struct fhh_ev_cfg {
    uint8_t base_pairs[2][128][2][16];   /* per OT kind: both base-OT keys of every base OT (kind 1
                                            read at tree_crawl_last only, r05c)                    */
    uint32_t form;                       /* as fhh_gb_cfg.form (the public protocol choice)       */
    uint32_t ot_ss_k;                    /* r06: 0 / 1 IKNP, 2 / 4 SoftSpoken with k = ot_ss_k: the
                                            U messages carry 128 / k rows + 4 KiB of GGM
                                            corrections (u_bytes = 16 mp / k + 4096)              */
    uint64_t child_begin;
    uint64_t child_count;
} fhh_ev_cfg;
int fhh_ev_ot_labels(fhh_ctx* ctx, const fhh_ev_cfg* cfg, const uint8_t** u_dev, uint64_t* u_bytes);
int fhh_gb_ot_labels(fhh_ctx* ctx, const fhh_gb_cfg* cfg, const uint8_t* u_dev, uint64_t u_bytes, const uint8_t** y_dev,
                     uint64_t* y_bytes);
int fhh_gb_garble(fhh_ctx* ctx, const uint8_t** gc_msg_dev, uint64_t* gc_msg_bytes);
int fhh_ev_evaluate(fhh_ctx* ctx, const uint8_t* gc_msg_dev, uint64_t gc_msg_bytes, const uint8_t* y_dev,
                    uint64_t y_bytes, const uint8_t** u_dev, uint64_t* u_bytes);
int fhh_gb_ot_shares(fhh_ctx* ctx, const uint8_t* u_dev, uint64_t u_bytes, const uint8_t** y_dev, uint64_t* y_bytes);
int fhh_ev_ot_shares(fhh_ctx* ctx, const uint8_t* y_dev, uint64_t y_bytes);
/* sums_a = uint64_t[C] (non-last level) or uint32_t[C][10] unreduced (last); sums_b = NULL or
 * uint32_t[C][8] canonical (last level) */
int fhh_party_node_sums(fhh_ctx* ctx, void* sums_a, void* sums_b);
/* bytes this ctx sent in the level so far (its outgoing messages) */
int fhh_party_bytes_sent(const fhh_ctx* ctx, uint64_t* bytes);
/* TEST MODE ONLY: both parties' configs derived from one seed — the in-process level loop's material
 * (fhh_sim_config.gc = 2, ideal base OTs) for prf_seed and level, so a two-ctx run can mirror
 * fhh_sim_crawl. Not private (one seed knows both sides); a deployment draws each party's
 * material on its own side. */
int fhh_gc_party_test_cfgs(uint64_t prf_seed, uint32_t level, fhh_gb_cfg* gb, fhh_ev_cfg* ev);

/* ---- base OTs (the OT extension's init, collect.rs:454-471) -------------------------------
 * Chou–Orlandi "simplest OT" over NIST P-256 (ocelot runs it over Ristretto; not vendored, so the
 * group and the wire format differ: functionality only). Points are 65-byte uncompressed SEC1;
 * scalars are derived from the 32-byte seeds (pass fresh randomness per batch). The base-OT
 * sender ends with key pairs keys[count][2][16], the receiver with keys[count][16] =
 * pair[c_i] (choices: bit i % 8 of byte i / 8). */
int fhh_co15_sender_start(const uint8_t seed[32], uint8_t A_out[65]);
int fhh_co15_receiver(uint32_t count, const uint8_t A[65], const uint8_t* choices, const uint8_t seed[32],
                      uint8_t* B_out, uint8_t* keys);
int fhh_co15_sender_finish(uint32_t count, const uint8_t seed[32], const uint8_t* B, uint8_t* keys);
/* Both parties in one process (derives the two parties' seeds from `seed`). */
int fhh_base_ot_co15(uint32_t count, const uint8_t* choices, const uint8_t seed[32], uint8_t* sender_keys,
                     uint8_t* receiver_keys);
const char* fhh_base_ot_last_error(void);

/* ---- statistics ------------------------------------------------------------------------ */

typedef struct fhh_stats {
    uint64_t aes_blocks;        /* executed AES-128 blocks (eval_bit PRG calls)          */
    uint64_t ref_evals;         /* reference-equivalent eval_bit calls (C * n * 2d)      */
    uint64_t expand_launches;   /* k_expand launches                                     */
    double expand_ms;           /* summed k_expand duration (HIP events on ctx stream)   */
    uint64_t expand_blocks_timed; /* AES blocks covered by expand_ms                     */
    uint64_t levels;            /* crawled levels                                        */
    double keygen_ms;
    uint64_t expand_launches_timed; /* k_expand launches covered by expand_ms             */
    double base_ot_ms;          /* real base OTs (fhh_sim_config.base_ot): summed per-instance host
                                 * compute time (CO15 + key schedules) over the producer's threads */
    double allreduce_ms;        /* device loop, cfg->comm / allreduce: summed per-level cross-rank
                                 * all-reduce time (HIP events around it on the engine stream,
                                 * on the levels fhh_set_timing times)                      */
    uint64_t allreduce_timed;   /* all-reduces covered by allreduce_ms                        */
    double gcot_ms;             /* device loop, cfg->gc: summed per-level GC + OT step time (share
                                 * planes, garble, OTs, evaluate, share sums; HIP events on the
                                 * engine stream, on the levels fhh_set_timing times)        */
    uint64_t gcot_timed;        /* levels covered by gcot_ms                                  */
    double base_ot_stall_ms;    /* time the level loop's enqueueing thread waited for a base-OT
                                 * instance it needed (the base OTs on the crawl's critical path) */
    uint64_t base_ot_instances; /* base-OT instances (128 CO15 OTs each) computed              */
} fhh_stats;

int fhh_get_stats(const fhh_ctx* ctx, fhh_stats* out);
/* Select the k_expand variant: the product variant 52 (sibling-pair AES, multi-word
 * items) or the generic-AES variant 33; both are bit-identical. The measured-negative A/B forms of
 * r01-r03 were removed in r06: FHH_E_ARG for any other id. */
int fhh_set_variant(fhh_ctx* ctx, int variant);
/* Describe variant: layout name, workgroup size, persistent grid on the current device.
 * Returns FHH_E_ARG for an id not in this build. */
int fhh_variant_info(int variant, char* name, size_t cap, int* threads, int* grid_per_device);
int fhh_reset_stats(fhh_ctx* ctx);
/* 1 to time every k_expand launch with HIP events (default 1); K > 1 times every K-th launch
 * of the device level loop (a pair of event records costs the stream a few microseconds). */
int fhh_set_timing(fhh_ctx* ctx, int enabled);

/* Peak-rate microbenchmarks pinning the roofline denominators on the running device:
 * which = 0 -> v_xor_b32 lane-ops/s; which = 1 -> ds_read_b32 bytes/s (k_expand pattern);
 * 2 -> v_bitop3_b32 lane-ops/s; 3 -> v_bitop3_b32 at 2 waves/SIMD; 4 -> v_xor_b32 at 2 waves/SIMD. */
int fhh_microbench(int device, int which, double* rate);
// Lookup throughput (lookups/s, chip-wide) of k_gather_mix<NL, NG>: NL chains through the
// per-lane LDS table beside NG chains through a global table of gbytes (power of two,
// 256..65536); combo 0..8 = (8,0) (0,8) (0,16) (8,1) (8,2) (8,4) (6,2) (4,4) (12,2).
int fhh_microbench_gather(int device, int combo, uint32_t gbytes, double* rate);
// k_hybrid_mix: nb (0, 2, 4, 6, 8) of a 16-wave workgroup's waves run v_bitop3 chains while
// the others run LDS lookup chains; rates[0] = lookups/s, rates[1] = bitop3 lane-ops/s.
int fhh_microbench_hybrid(int device, int nb, double* rates);
/* Device time per kernel of `reps` back-to-back launches of an empty kernel on one stream
 * (launch-overhead probe for the level loop): which = 0 -> 256 x 1024 threads, 4 KiB LDS;
 * 1 -> 256 x 1024, 128 KiB LDS (k_expand's footprint); 2 -> alternating 256 x 1024 / 128 KiB and
 * 1 x 1024 (expand -> prune); 3 -> 1 x 1024; 4 / 5 -> alternating a 64 MiB writer (normal /
 * nontemporal stores) with 1 x 1024; 6 / 7 -> as 2 / 4 captured in a hipGraph and replayed. */
int fhh_debug_launch_gaps(int device, int which, int reps, double* us_per_kernel);
/* Wave timeline of the profiling k_expand variant 36 (tools/tail_profile.py): arm with a device
 * buffer of cap launches x grid waves x 3 u64 ({start after the LDS table fill, exit, items},
 * 100 MHz s_memrealtime ticks; buf NULL disarms); launches = launches recorded so far. */
int fhh_wave_profile_arm(int device, uint64_t* buf, uint32_t cap);
int fhh_wave_profile_launches(int device, uint32_t* launches);

/* Device-to-device copy (synchronous): the channel stand-in of the in-process two-party runs,
 * which move each party's messages into buffers the other party owns. */
int fhh_memcpy_device(int device, void* dst_dev, const void* src_dev, uint64_t bytes);

/* Device properties the library targets (gfx950). */
int fhh_device_info(int device, char* arch_name, size_t cap, int* num_cus);

#ifdef __cplusplus
}
#endif
#endif /* FHH_H */
