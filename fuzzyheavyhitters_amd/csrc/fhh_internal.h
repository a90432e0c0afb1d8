// Internal interface between the host engine (fhh_host.cpp) and the HIP kernels
// (fhh_kernels.hip). Not part of the public C ABI (include/fhh.h).
//
// Device layout of one server's keys and evaluation states (SoA, lane = client):
//   npad = 64 * nw clients (padded), K = 2*d keys per client, kk = 2*j + side
//   cw_seed   [L][K][npad]   uint4      CorWord.seed            (ibDCF.rs:9-14)
//   cw_bits   [L][K][4][nw]  u64 planes bits.0, bits.1, y.0, y.1
//   root_seed [K][npad]      uint4      ibDCFKey.root_seed      (ibDCF.rs:16-21)
//   key_idx   [K][nw]        u64 plane  ibDCFKey.key_idx
//   per dim j, prefix table (double buffered), entry e = one dim-j prefix:
//     seed [E][2][npad] uint4, t [E][2][nw] u64, y [E][2][nw] u64   (EvalState, ibDCF.rs:24-30)
// A frontier node is a tuple of d entries (one per dim); a dim-j prefix shared by several
// nodes is evaluated once (the reference re-evaluates it per node, collect.rs:94-119).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

struct fhh_comm;   // include/fhh.h (fhh_comm.cpp)

namespace fhh {

constexpr int kMaxDims = 4;
constexpr int kMaxJobs = 2 * kMaxDims;      // two servers' ctxs x dims in one launch
constexpr int kExpandThreads = 512;
constexpr int kReduceThreads = 256;

struct ExpandJob {
    const uint4* cw_seed;
    const uint64_t* cw_bits;
    const uint4* src_seed;
    const uint64_t* src_t;
    const uint64_t* src_y;
    uint4* dst_seed;
    uint64_t* dst_t;
    uint64_t* dst_y;
    const uint32_t* live;   // [n_live] src entries, in frontier order
    uint32_t n_live;
    uint32_t level;
    uint32_t dim;
    uint32_t K;
    uint32_t npad;
    uint32_t nw;
    uint32_t group;         // entries per work item (CW reuse factor)
    uint32_t wpi;           // words (64-client units) per work item (item_layout; 1 = one word)
    uint64_t item_begin;
    // end-of-launch phase (item_layout): entries [split, n_live) as items of group_b entries,
    // numbered from item_begin_b after every job's bulk items; e_base = first entry of the
    // segment an item belongs to (set by the kernel)
    uint32_t split;
    uint32_t group_b;
    uint32_t e_base;
    uint32_t pad2_;
    uint64_t item_begin_b;
};

// Device-resident level loop (fhh_sim_crawl with the GPU loop): the frontier sizes live in
// device memory, written by k_prune and read by the next level's kernels, so a whole crawl is
// enqueued without host round trips. `abort` is sticky: once a capacity check fails every
// later kernel is a no-op and the host grows the buffers and resumes from abort_level.
struct LoopCtl {
    uint32_t abort;
    uint32_t abort_level;
    uint32_t need_entries;      // entries a dim table must hold to continue
    uint32_t need_nodes;        // frontier nodes to continue
    uint32_t F;                 // frontier nodes
    uint32_t C;                 // pending children (F << d)
    uint32_t n_live[kMaxDims];  // live entries per dim (same for both servers)
    uint32_t group;             // entries per work item for the next k_expand
    uint32_t group_b;           // entries per end-phase item
    uint32_t wpi;               // words per bulk item (item_layout)
    uint32_t pad_;
    uint64_t item_begin[kMaxJobs];
    uint64_t total_items;
    uint64_t items_a;           // bulk items of all jobs precede the end-phase items
    uint64_t item_begin_b[kMaxJobs];
    uint32_t split[kMaxJobs];
};

// k_expand work decomposition, shared by the host (finalize_launch) and the device loop
// (k_prune, k_loop_init). Bulk: items of g entries x one word unit (64 clients), g sized so
// each wave gets >= 2 items, capped at max_group. A launch ends when its slowest wave finishes
// its last item, and with 16-entry items that tail averaged 8.7 % of k_expand's time
// (tools/tail_profile.py). So about one item per wave of work at the end is re-cut as items
// of g_b = min(g, kTailGroup) entries, dealt after every job's bulk items. The end phase must
// not outrun the single work counter (≈ 88 dequeues/µs): 4-entry items at 2 per wave did
// (8 % slower), hence 8 entries and one item per wave.
// Words per item (max_wpi > 1, no end phase): when the frontier is narrow (d = 2 at data_len 16,
// or the first levels of any crawl) a group holds only a few entries, so one-word items are too
// small for the single counter — configs[3] at 1M clients made 62 500 items of ~2.5 entries per
// level and k_expand ran at the counter's 88 items/µs (25 G blocks/s). A bulk item then spans
// wpi = max_group / (entries per group) consecutive words (64-client units), lowered until the
// launch still has kMwItemsPerWave items per wave; wide levels (groups of ≥ max_group / 2 entries)
// keep wpi = 1.
constexpr uint32_t kTailGroup = 8;
// r05: 4 (was 2) since k_expand draws from 8 per-XCD heads on narrow levels: configs[3] k_expand
// 0.44 -> 0.47 of the VALU roofline, the d = 1 headline unchanged (profiles/r05/expand_heads/)
// (r06 A/B, profiles/r06/ab_mw_ipw/: 2 -> 0.459, 8 or 16 -> 0.166 — wpi falls to 1 — against 0.478)
#ifndef FHH_MW_IPW
#define FHH_MW_IPW 4
#endif
constexpr uint64_t kMwItemsPerWave = FHH_MW_IPW;
struct ItemLayout {
    uint32_t g, g_b, wpi;
    uint64_t items_a, total;
    uint64_t begin_a[kMaxJobs], begin_b[kMaxJobs];
    uint32_t split[kMaxJobs];
};
__host__ __device__ inline void item_layout(const uint32_t* n_live, uint32_t njobs, uint32_t unit, uint32_t max_group,
                                            uint64_t grid_waves, bool tail_split, ItemLayout& L,
                                            uint32_t max_wpi = 1) {
    uint64_t entries = 0;
    for (uint32_t k = 0; k < njobs; k++) entries += n_live[k];
    const uint64_t entry_words = entries * unit;
    uint64_t g = entry_words / (2 * grid_waves);
    g = g < 1 ? 1 : (g > max_group ? max_group : g);
    const uint64_t gb = g < kTailGroup ? g : kTailGroup;
    L.g = (uint32_t)g;
    L.g_b = (uint32_t)gb;
    uint64_t wpi = 1;
    if (max_wpi > 1 && !tail_split) {
        uint64_t groups = 0;
        for (uint32_t k = 0; k < njobs; k++) groups += (n_live[k] + g - 1) / g;
        if (groups) {
            const uint64_t e_eff = entries / groups;   // >= 1: every group holds an entry
            wpi = e_eff >= max_group ? 1 : max_group / e_eff;
            if (wpi > max_wpi) wpi = max_wpi;
            while (wpi > 1 && groups * ((unit + wpi - 1) / wpi) < kMwItemsPerWave * grid_waves) wpi--;
        }
    }
    L.wpi = (uint32_t)wpi;
    const uint64_t units = (unit + wpi - 1) / wpi;   // bulk items per entry group
    // end-phase entries wanted in all: one item of g_b entries per wave
    const uint64_t want = (tail_split && gb < g) ? (grid_waves * gb + unit - 1) / unit : 0;
    for (uint32_t k = 0; k < njobs; k++) {
        uint32_t split = n_live[k];
        if (want && entries) {
            const uint64_t bk = (n_live[k] * want + entries - 1) / entries;   // job's share, rounded up
            split = bk >= n_live[k] ? 0u : (uint32_t)(n_live[k] - bk);
        }
        L.split[k] = split;
    }
    uint64_t begin = 0;
    for (uint32_t k = 0; k < njobs; k++) {
        L.begin_a[k] = begin;
        begin += units * ((L.split[k] + g - 1) / g);
    }
    L.items_a = begin;
    for (uint32_t k = 0; k < njobs; k++) {
        L.begin_b[k] = begin;
        begin += (uint64_t)unit * ((n_live[k] - L.split[k] + gb - 1) / gb);
    }
    L.total = begin;
}

// k_expand's dynamic work heads inside fhh_ctx::work_counter (kWorkCounterBytes): two sets of
// kExpandHeads per-XCD heads (one 64-B line each) by launch parity (the kernel zeroes the next
// launch's set), then the wave-timeline exit count of the profiling variant; words 0-1 belong to the
// r01 A/B kernels' re-armed counter (unused since r06)
constexpr uint32_t kExpandHeads = 8, kExpandSlot0 = 16, kExpandSlotStride = 16;
constexpr uint32_t kExpandProfSlot = kExpandSlot0 + 2 * kExpandHeads * kExpandSlotStride;
constexpr size_t kWorkCounterBytes = 2048;
static_assert((kExpandProfSlot + 1) * 4 <= kWorkCounterBytes, "work counter layout");

struct ExpandLaunch {
    ExpandJob job[kMaxJobs];
    uint32_t njobs;
    uint32_t jobs_per_ctx;      // = d (LoopCtl::n_live index = job % jobs_per_ctx)
    uint64_t total_items;
    uint64_t items_a;           // host-driven launches: bulk items (== total_items without a tail phase)
    uint32_t wpi;               // host-driven launches: words per bulk item (item_layout)
    uint32_t seq;               // the counter's launch number (fhh_ctx::expand_seq): k_expand counter slot
    const LoopCtl* ctl;         // non-null: n_live / group / item_begin / total_items from here
};

// Pending children: child c -> parent p = c >> d, i = c & (2^d - 1); its dim-j entry in
// the child table is 2 * parent_pos[p*d + j] + ((i >> j) & 1).
struct PlaneSet {
    const uint64_t* t[kMaxDims];
    const uint64_t* y[kMaxDims];
};

struct ChildArgs {
    PlaneSet s0, s1;            // server 0 / server 1 child tables (s1 unused for share export)
    const uint32_t* parent_pos; // [F][d]
    const uint64_t* valid;      // [nw]
    uint64_t C;
    uint32_t d;
    uint32_t nw;
    uint64_t client_base;       // global index of client 0 (simulated-OT PRF)
    uint64_t prf_seed;
    uint32_t level;
    uint32_t n;                 // real clients on this ctx
    const LoopCtl* ctl;         // non-null: C from here (0 once aborted)
    // GC mode (row f1): the equality bit of (child c, client i) is the evaluator's garbled-
    // circuit output gc_out[c * gc_N + i] XOR the garbler's mask (ideal OT, collect.rs:437-471)
    const uint8_t* gc_out;
    uint32_t gc_N;
    uint32_t gc_mask;
    // OT mode (r05: correlated OT, OtArgs modes 2 / 3): the two servers' node values of (c, i) are
    // the C-OT's outputs — FE levels u64 ot_val[s][(c - c_off) * gc_N + i] (s = 0 the garbler's
    // v + mask, s = 1 the receiver's); the last level BlockPairs (2 blocks per value: the garbler's
    // canonical V + mask, the receiver's raw FieldElm::try_from(BlockPair))
    const void* ot_val[2];
    // child window of the GC + OT kernels (a chunk of the level's children, as the reference splits
    // a level's tests over its channels, collect.rs:423-430): children [c_off, c_off + c_cnt) only,
    // gc_out / ot_recv / OT messages indexed (c - c_off) * gc_N + i; c_cnt = 0: every child
    uint64_t c_off;
    uint64_t c_cnt;
    // k_share_planes' row stride in words (0: nw); words nw .. plane_nw - 1 are written as zero (r06: the
    // tile-major garbled table wants rows of whole 512-client tiles, plane_nw a multiple of 8)
    uint32_t plane_nw;
};

// Garbled-circuit equality tests (row f1, equalitytest.rs:25-219): tests t = g * N + i for
// groups g < G (children) and i < N (clients); a test compares the garbler's `bits`-bit string
// with the evaluator's. Inputs are bit planes [G][bits][nw] (as k_share_planes writes them);
// outputs are SoA over t (16-B blocks; one lane per test, coalesced).
constexpr int kGcMaxBits = 8;
struct GcArgs {
    const uint64_t* gb_planes;   // garbler's share bits
    const uint64_t* ev_planes;   // evaluator's share bits (ideal OT: only their labels leave)
    uint64_t G;
    uint32_t N, nw, bits, mask;
    uint32_t rk_label[11][4];    // garbler's label PRG key schedule (AES-128-CTR)
    uint32_t delta[4];           // free-XOR offset, lsb 1
    uint64_t label_nonce;        // label of (t, w) = AES_k(label_nonce + t S + w), S = pow2 >= W (W = 2 bits + 1, ev_ot: bits + 1)
    uint64_t gate_base;          // half-gate tweaks 2 (gate_base + t (bits - 1) + k) (+1)
    uint4* tables;               // [(bits-1)][2][n]  (T_G, T_E)
    uint4* gb_labels;            // [bits + 1][n]     garbler's active input labels (+ mask)
    uint4* ev_labels;            // [bits][n]         evaluator's active labels (ideal OT out)
    uint8_t* decode;             // [n]               output decoding bit
    uint8_t* out;                // [n]               evaluator's output bit = eq ^ mask
    const LoopCtl* ctl;          // non-null (level loop): groups = min(G, ctl->C), 0 once aborted;
                                 // G * N stays the SoA stride
    uint32_t ev_ot;              // 1 (r05, the labels OT is a correlated OT): ev_labels holds the
                                 // evaluator's labels at OT index (g bits + j) Npad + i (Npad = 64 nw:
                                 // its share planes are the OT's choice bits) — k_gc_garble reads the
                                 // ZERO labels there (the C-OT's sender messages) and draws only its
                                 // own wires and the mask (label stride pow2 >= bits + 1), k_gc_eval
                                 // reads its OT'd active labels there. 0: ideal OT (every label drawn
                                 // by the garbler, the evaluator's active ones written to ev_labels)
    uint32_t out_dup;            // out_packed: each output bit repeated out_dup (1 or 2) times
    uint32_t* out_packed;        // non-null: k_gc_eval also writes the outputs as bit words
                                 // (tests t0.. of a 64-aligned wave slice; the FE-share OT choices)
    uint64_t g_off;              // chunk: groups [g_off, g_off + G) of the planes; tests, labels and
                                 // gate tweaks keep their whole-level index (g_off N + t)
    // r05c (ev_ot, FE levels): the FE share from the output labels instead of a second OT, [G N] each
    // (oracle gc_share_garbler / gc_share_evaluator): k_gc_garble_cot writes the garbler's node value
    // r1 = v + mask to sh_gb and the 8-B message y to sh_y; k_gc_eval reads sh_y and writes the
    // evaluator's node value to sh_ev. Null: no share.
    uint64_t* sh_gb;
    uint64_t* sh_y;
    uint64_t* sh_ev;
    // r05d (FE levels, bits <= kGtMaxBits): the garbled table (oracle orc_gt_garble / orc_gt_eval):
    // k_gt_garble writes rows 1 .. 2^bits - 1's messages SoA [2^bits - 1][G N] and the garbler's node
    // values to sh_gb, k_gt_eval reads them and writes the evaluator's to sh_ev
    uint64_t* gt_msgs;
    // r06: 1 = ev_labels is the labels OT's tile-major matrix itself (Q for k_gt_garble, T for k_gt_eval;
    // fhh_ot.hip ot_tmaj) instead of one row-major label per OT (k_ot_rows_out); needs nw % 8 == 0 (the OT
    // index (g bits + k) 64 nw + i puts a test's labels at one position of 512-OT tiles)
    uint32_t lab_tm;
    // r06 (lab_tm): non-null = the table kernels add their node values' 32-bit limbs per child into
    // node_partials [C][4] u64 (k_child_sums_fe's layout: garbler lo, hi; evaluator lo, hi) by one wave sum
    // and atomic per 512-test tile, instead of storing them for k_child_sums_fe (sh_gb / sh_ev may be null)
    uint64_t* node_partials;
    uint64_t node_off;   // node_partials row of the launch's group 0 beyond g_off (the party ABI: its chunk's c_off)
    // r06 (lab_tm): 1 = the table's shares live in Z_2^32 instead of FE (row value lo32 of the
    // hash, pair (v, v +- 1 mod 2^32), 4-B messages [2^b - 1][n] u32; the partials' low sums taken mod 2^32)
    uint32_t ring32;
};
constexpr int kGtMaxBits = 4;   // 16 rows (d = 2); wider tests keep the half-gates chain
constexpr int kGtTmMaxBits = 2;   // r06: the table kernels read the tile-major labels (lab_tm) for b <= 2 (d = 1)

struct PruneArgs {
    LoopCtl* ctl;
    const uint64_t* partials;   // [C][per] u64 (after the cross-rank sum)
    uint32_t mode;              // 0 counts, 1 FE limbs [C][4], 2 FE255 limbs [C][16] (last level)
    uint32_t d;
    uint64_t thr;               // leader.rs:193-194
    uint32_t thr_last;          // leader.rs:245-246
    uint32_t last;              // tree_crawl_last: record final values
    const uint32_t* pos_in;     // [F][d]
    uint32_t* pos_out;          // [F'][d]
    uint32_t* live_out[kMaxDims];
    uint32_t* mark;             // scratch [kMaxDims][E_cap]
    uint32_t* hist_out;         // [F_cap] kept children of this level (child index c)
    uint32_t* sizes_out;        // [4 + kMaxDims]: C, F', abort, -, n_live'...
    uint32_t* final_vals;       // last level: [F_cap][20] u32 (server 0 / server 1 unreduced)
    uint32_t E_cap, F_cap;
    uint32_t level;
    uint32_t nw;
    uint32_t njobs_per_ctx;     // = d
    uint32_t nctx;              // 2 (pair)
    uint64_t grid_waves;        // persistent k_expand waves (for the group size)
    uint32_t unit;              // k_expand items per entry group (nw)
    uint32_t max_group;         // entries per item cap
    uint32_t tail_split;        // item_layout end phase (expand_tail_split)
    uint32_t max_wpi;           // item_layout words-per-item cap (expand_max_wpi)
    // FE levels: k_child_sums_fe adds its client chunks into the partials by atomics, so a prune that
    // completes zeroes them for the next level (a memset node would also run after a sticky
    // abort and wipe the sums the resumed prune re-reads)
    uint64_t* zero_partials;
    uint64_t zero_count;
    uint32_t ring32;            // r06, mode 1: the level's shares are in Z_2^32 (GcArgs::ring32): v0 - v1 mod 2^32
};

struct KeygenArgs {
    const uint8_t* left_bits;   // [n][d][L]
    const uint8_t* right_bits;
    const uint8_t* root_seeds;  // [n][d][2 side][2 server][16]
    uint4* cw_seed[2];
    uint64_t* cw_bits[2];
    uint4* root[2];
    uint64_t* key_idx[2];
    uint64_t n;
    uint32_t d, L, K, npad, nw;
};

// ---- launch wrappers (fhh_kernels.hip); all asynchronous on `stream` ----
// seq: the counter's launch count (fhh_ctx::expand_seq), advanced per k_expand launch
hipError_t launch_expand(const ExpandLaunch& a, int variant, int grid, uint32_t* work_counter, uint32_t* seq,
                         hipStream_t stream);
int expand_variant_count();
const char* expand_variant_name(int variant);
int expand_threads(int variant);
hipError_t launch_eq_count(const ChildArgs& a, uint64_t* counts, hipStream_t stream);
hipError_t launch_share_planes(const ChildArgs& a, uint64_t* out, hipStream_t stream);
// zero: clear partials first (host-driven launches); the device loop's k_prune clears them instead
hipError_t launch_child_sums_fe(const ChildArgs& a, uint64_t* partials /*[C][4]*/, hipStream_t stream, bool zero);
hipError_t launch_child_sums_fe255(const ChildArgs& a, uint64_t* partials /*[C][16]*/, hipStream_t stream);
// per-child limb partials of values [C][ld] (n per row) in format fmt (FHH_VALS_*): FE -> [C][2],
// FE255 -> [C][8]
hipError_t launch_sum_vals(const void* vals, uint32_t fmt, uint64_t C, uint64_t n, uint64_t ld, uint64_t* partials,
                           hipStream_t stream);
hipError_t launch_keygen(const KeygenArgs& a, hipStream_t stream);
hipError_t launch_init_tables(const uint4* root, const uint64_t* key_idx, uint32_t dim, uint32_t K, uint32_t npad,
                              uint32_t nw, uint4* seed, uint64_t* t, uint64_t* y, hipStream_t stream);
hipError_t launch_keys_from_aos(const uint8_t* key_idx, const uint8_t* root_seed, const uint8_t* cw_seed,
                                const uint8_t* cw_bits, uint64_t n, uint32_t K, uint32_t L, uint32_t npad, uint32_t nw,
                                uint4* d_cw_seed, uint64_t* d_cw_bits, uint4* d_root, uint64_t* d_key_idx,
                                hipStream_t stream);
hipError_t launch_keys_from_bincode(const uint8_t* buf, uint64_t n, uint32_t d, uint32_t L, uint32_t npad, uint32_t nw,
                                    uint4* d_cw_seed, uint64_t* d_cw_bits, uint4* d_root, uint64_t* d_key_idx,
                                    uint32_t* err, hipStream_t stream);
// occupancy-derived persistent grid for k_expand variant on `device`
int expand_grid(int device, int variant);
// RCCL all-reduce (sum, u64) on `stream` (fhh_comm.cpp); asynchronous
int comm_allreduce(::fhh_comm* c, const uint64_t* send, uint64_t* recv, uint64_t count, hipStream_t stream,
                   std::string* err);
// in-process communicators over distinct devices (ncclCommInitAll), a grouped in-place all-reduce
// (ncclGroupStart/End, one stream per communicator) and abort (fhh_comm.cpp)
int comm_init_all(int n, const int* devices, std::vector<::fhh_comm*>& out, std::string* err);
int comm_group_allreduce(const std::vector<::fhh_comm*>& comms, const std::vector<uint64_t*>& bufs, uint64_t count,
                         const std::vector<hipStream_t>& streams, std::string* err);
// abort once (a second call, or one racing it from another shard thread, is a no-op); the handle
// stays valid until fhh_comm_destroy, which then skips ncclCommDestroy
void comm_abort(::fhh_comm* c);
int comm_rank(const ::fhh_comm* c);   // the rank given at creation
// device-resident level loop (fhh_loop.hip); `unit` = items per entry group, `max_group` =
// entries per item cap (see expand_unit)
hipError_t launch_prune(const PruneArgs& a, hipStream_t stream);
// IKNP / ALSZ OT extension (row f1's OT): m OTs of 16-B messages; base OTs given as key schedules
// (the sender's are those of k_i^{s_i}). Bit matrices are [128 rows][mp / 128] uint4 blocks, read per
// OT by the hashes (transposed on the fly). With ctl set (level loop) only the first
// per_group * min(groups, ctl->C) OTs run.
// Modes (r05; oracle/fhh_oracle.c orc_ot_extend / orc_cot_extend):
//   0  plain OT: y_j^b = x_j^b ^ H(q_j ^ b s) (x1 == nullptr: x1 = x0 ^ delta); out = y_j^{r_j} ^ H(t_j)
//   1  correlated OT, XOR delta (the labels OT): sender writes sx[j] = H(q_j) (the evaluator's zero
//      label) and Y0[j] = H(q_j) ^ delta ^ H(q_j ^ s); out = r_j ? Y0[j] ^ H(t_j) : H(t_j)
//   2  correlated OT, FE share: v = H(q_j) as LE u128 mod p; sender value v + mask -> sx (u64 [m]),
//      Y0 (8 B [m]) = lo64(H(q_j ^ s)) ^ (mask ? v + 1 : v - 1); out (u64 [m]) = r_j ? lo64(Y0[j] ^
//      H(t_j)) : H(t_j) mod p
//   3  correlated OT, FieldElm share, raw pass: sx[j] = H(q_j), Y0[j] = H(q_j ^ s); k_cot_fe255_finish
//      turns OT pairs (2t, 2t + 1) into the sender's node values and y; out = r_j ? Y0[j] ^ H(t_j) : H(t_j)
//   4  (r05b) the IKNP correlation itself, the labels OT: no hash, no y — sx[j] = q_j, out[j] = t_j =
//      q_j ^ r_j s (k_ot_rows_out transposes Q / T); with s as the free-XOR Delta, q_j is the zero label
//      of the evaluator's input wire j and t_j its active label
struct OtArgs {
    uint64_t m;                  // OTs (capacity)
    uint64_t mp;                 // m padded to a multiple of 8192 (whole waves per row)
    const uint32_t* rk;          // [3][128][44]: receiver k_i^0, k_i^1, sender k_i^{s_i}
    uint32_t s[4];               // sender's base choice bits
    const uint32_t* choices;     // [mp / 32] receiver's choice bits (0 past m)
    uint4 *T, *U, *Q;            // tile-major (fhh_ot.hip ot_tmaj): T, Q, and since r06 U (the wire) too
    const uint4 *x0, *x1;        // mode 0: [m]; x1 == nullptr: x1 = x0 ^ delta (correlated messages)
    uint32_t delta[4];           // modes 0 (x1 == nullptr) and 1
    uint4 *Y0, *Y1, *out;        // mode 0: Y0, Y1 [m]; modes 1-3: y in Y0 (mode 2: 8 B per OT); out [m]
    uint64_t tweak_base;
    const LoopCtl* ctl;
    uint64_t per_group;
    uint64_t g_off;              // level loop chunk: OTs of groups [g_off, ctl->C) only
    uint32_t mode;               // 0..4 above; 5 = 4 left tile-major (expands only: the r06 garbled table
                                 // reads Q / T itself, GcArgs::lab_tm)
    uint32_t mask;               // modes 2, 3: the garbler's mask bit
    uint64_t ctr_off;            // the row PRG's first block (a multiple of 256): a base-OT session's
                                 // running counter, so batches extending one session never repeat pads
    void* sx;                    // modes 1, 3, 4: uint4 [m]; mode 2: u64 [m] (the sender's node values)
    // r06: 0 / 1 = IKNP; 2, 4 = SoftSpoken with k = ss_k (fhh_ot.hip k_ss_*): U is then 128 / k rows
    // (tile-major, tile stride 128 / k rows), ss_leaf [2][128 / k][2^k] the GGM leaves (receiver, sender),
    // ss_corr [128 / k][k][2] the receiver's GGM corrections (the wire)
    uint32_t ss_k;
    uint32_t ss_role;            // k_ss_ggm: 0 both parties (the level loop), 1 the receiver (leaves + corrections),
                                 // 2 the sender (its leaves from ss_corr, the received corrections) — the party ABI
    uint4* ss_leaf;
    uint4* ss_corr;
};
// SoftSpoken GGM trees of both parties from rk / s (one workgroup; before the expands)
hipError_t launch_ss_ggm(const OtArgs& a, hipStream_t stream);
hipError_t launch_ot_recv_expand(const OtArgs& a, hipStream_t stream);
hipError_t launch_ot_send_expand(const OtArgs& a, hipStream_t stream);
// the hashes reading T / Q in row form with the transpose fused in (no Tt / Qt pass)
hipError_t launch_ot_send_hash_rows(const OtArgs& a, hipStream_t stream);
hipError_t launch_ot_recv_hash_rows(const OtArgs& a, hipStream_t stream);
// *word &= mask (one lane; the tail of a choice-bit buffer)
hipError_t launch_mask_word(uint32_t* word, uint32_t mask, hipStream_t stream);
// the 128 Chou–Orlandi base OTs of OT extension k (fhh_base_ot.cpp)
int base_ot_instance(uint64_t k, const uint8_t seed[32], const uint8_t choices[16], uint8_t* pairs, uint8_t* chosen,
                     std::string* err);
hipError_t launch_ot_level_keys(uint64_t prf, uint32_t level, uint32_t salt, const uint32_t s[4], uint32_t* rk,
                                hipStream_t stream);
// mode 3's second pass (the garbler, FieldElm share): per test t, V = H(q_2t) || H(q_2t+1) (32
// big-endian bytes, sx) mod p255 -> sx pair = V + mask (its node value, a canonical BlockPair), Y0 pair
// ^= (mask ? V + 1 : V - 1); tests = the active OT pairs (ctl-aware as the hashes)
hipError_t launch_cot_fe255_finish(const OtArgs& a, hipStream_t stream);
// mode 4: the tile-major Q (sender: -> sx) or T (receiver: -> out) as one 16-B row per OT
hipError_t launch_ot_rows_out(const OtArgs& a, bool sender, hipStream_t stream);
hipError_t launch_gc_garble(const GcArgs& a, hipStream_t stream);
hipError_t launch_gc_eval(const GcArgs& a, hipStream_t stream);
hipError_t launch_gt_garble(const GcArgs& a, hipStream_t stream);   // r05d garbled table
hipError_t launch_gt_eval(const GcArgs& a, hipStream_t stream);
hipError_t launch_gather_hist(const uint32_t* sizes, uint32_t stride, const uint32_t* const* rows, uint32_t levels,
                              uint32_t* out, uint64_t cap, hipStream_t stream);
// parity probe of the device loop (fhh_sim_config.probe_*): the pending children's states of a
// client sample, both servers, gathered between k_expand and the count (fhh_loop.hip)
struct ProbeArgs {
    const uint4* seed[2][kMaxDims];     // child tables [E][2][npad] of server s, dim j
    const uint64_t* t[2][kMaxDims];     // [E][2][nw]
    const uint64_t* y[2][kMaxDims];
    const uint32_t* parent_pos;         // [F][d]
    const uint64_t* clients;            // [n_probe] local client indices (< n)
    const LoopCtl* ctl;                 // C (0 once aborted)
    uint4* out_seed;                    // [2][C_cap][n_probe][d][2]
    uint8_t* out_ty;                    // [2][C_cap][n_probe][d][2]: bit0 t, bit1 y
    uint32_t* out_C;                    // C of the level (written unless aborted)
    uint64_t C_cap;
    uint64_t npad, nw;
    uint32_t n_probe, d;
};
hipError_t launch_probe_states(const ProbeArgs& a, hipStream_t stream);
hipError_t launch_loop_init(LoopCtl* ctl, uint32_t d, uint32_t unit, uint32_t max_group, uint32_t max_wpi,
                            uint32_t njobs_per_ctx, uint32_t nctx, uint64_t grid_waves, uint32_t* pos0,
                            uint32_t* live0[kMaxDims], hipStream_t stream);

// ---- sketch + Beaver verification (fhh_sketch.hip), FE values as u64 (any representation) ----
struct SketchArgs {
    const uint8_t* seeds;   // [n_keys][16] PrgStream seeds (sketch_at's rand_stream)
    const uint64_t* x;      // [n_keys][n_nodes]
    const uint64_t* kx;     // [n_keys][n_nodes]
    uint64_t* out;          // [n_keys][6] canonical {r_x, r2_x, r_kx, rand1, rand2, rand3}
    uint64_t n_keys;
    uint32_t n_nodes;
    uint32_t force_sequential;   // 1: every key takes the sequential-stream path (tests)
    uint32_t level;              // the level's stream seed = seed with bytes 12..15 ^= level
    // r05: both servers in one k_sketch_fe launch (the level batch): keys [n_srv, n_keys) are server
    // 1's keys k - n_srv (same seeds, its own x1 / kx1 / out1); n_srv = 0: one server
    uint64_t n_srv;
    const uint64_t* x1;
    const uint64_t* kx1;
    uint64_t* out1;
};
// k_sketch_fe launch plan: keys [0, n_main) at lpk_main lanes per key, the rest at lpk_tail
struct SketchPlan {
    uint64_t n_main;
    int lpk_main, lpk_tail;
};
SketchPlan plan_sketch(uint64_t n_keys, uint32_t n_nodes, uint64_t resident_waves);
// U = FieldElm: values as 8 x u32 little-endian limbs
struct Sketch255Args {
    const uint8_t* seeds;
    const uint32_t* x;      // [n_keys][n_nodes][8]
    const uint32_t* kx;
    uint32_t* out;          // [n_keys][6][8]
    uint64_t n_keys;
    uint32_t n_nodes;
    uint32_t force_sequential;
    uint32_t level;
};
struct Mul255Args {
    const uint32_t* sketch;   // [n][6][8]
    const uint32_t* mac;      // [n][8]
    const uint32_t* mac2;     // [n][8]
    const uint32_t* triples;  // [n][9][8]
    const uint32_t* cor;      // [n][6][8] (mode 1)
    uint32_t* out;            // mode 0: [n][6][8]; mode 1: [n][8]
    uint64_t n;
    uint32_t mode;
    uint32_t server_idx;
};
struct Verify255Args {
    const uint32_t* sketch[2];
    const uint32_t* mac[2];
    const uint32_t* mac2[2];
    const uint32_t* triples[2];
    uint8_t* ok;
    uint32_t* out_shares;     // [2][n][8] or null
    uint64_t n;
};
struct MulArgs {
    const uint64_t* sketch;   // [n][6]
    const uint64_t* mac;      // [n]
    const uint64_t* mac2;     // [n]
    const uint64_t* triples;  // [n][triples_levels][3][a, b, c]
    const uint64_t* cor;      // [n][6] (mode 1)
    uint64_t* out;            // mode 0: [n][6] cor share; mode 1: [n] out share
    uint64_t n;
    uint32_t mode;
    uint32_t server_idx;
    uint32_t level;           // the level's triples (MulState::new's triples[3 level ..], mpc.rs:94-98)
    uint32_t triples_levels;  // levels the triple arrays hold (>= 1)
};
struct VerifyArgs {
    const uint64_t* sketch[2];
    const uint64_t* mac[2];
    const uint64_t* mac2[2];
    const uint64_t* triples[2];
    uint8_t* ok;              // [n]
    uint64_t* out_shares;     // [2][n] or null
    uint64_t n;
    uint32_t level;
    uint32_t triples_levels;
};
hipError_t launch_sketch_fe(const SketchArgs& a, hipStream_t stream);
hipError_t launch_sketch_fe2(const SketchArgs& a, hipStream_t stream, hipStream_t tail_stream);
hipError_t launch_mul_fe(const MulArgs& a, hipStream_t stream);
hipError_t launch_verify_fe(const VerifyArgs& a, hipStream_t stream);
hipError_t launch_deal_triples_fe(uint64_t n, uint32_t levels, uint64_t seed, uint64_t* t0, uint64_t* t1,
                                  hipStream_t stream);
hipError_t launch_sketch_fe255(const Sketch255Args& a, hipStream_t stream);
hipError_t launch_mul_fe255(const Mul255Args& a, hipStream_t stream);
hipError_t launch_verify_fe255(const Verify255Args& a, hipStream_t stream);

// entries per work item (CW reuse and counter traffic vs. end-of-level tail): variant 29 is
// variant 3 drawing the next item one entry ahead; 30 / 31 are variant 3 with up to 16 / 32
// entries per item; 32 / 33 store child seeds nontemporally with up to 8 / 16 entries per item;
// 34 / 35 are 33 / 32 with the sibling-pair AES (aes0_mmo_pair); 36 is 34 + wave timeline;
// 37 / 38 are 34 / 36 with the end-of-launch phase of small items (item_layout); 39 / 40 are
// 34 at 768 / 512 threads (3 / 2 waves per SIMD: a VGPR budget of 168 / 256 lets the
// scheduler keep more T-table lookups in flight per wave); 41 is 39 drawing the next item ahead;
// 42 is 34 with the next entry's seeds prefetched under the current entry's AES; 43 / 44 are
// DIAGNOSTIC builds of 34 that store no / only the dir-0 child seeds (HBM-write A/B; their states
// are incomplete by design and no product path selects them); 45 / 46 / 47 / 48 are the hybrid:
// 34 with the last 2 / 4 / 6 / 8 of each workgroup's 16 waves running the pair-sliced VALU AES
// (expand_ps.h) on the same items; 49 runs every wave as a VALU wave (the test variant that
// pins expand_item_ps: in 45-48 which items the VALU waves take depends on timing); 50 is 34 with
// ordinary (write-back) child-seed stores instead of nontemporal ones (the power-bound A/B)
inline uint32_t expand_max_group(int variant) {
    return (variant == 30 || variant == 33 || variant == 34 || (variant >= 36 && variant <= 52))
               ? 16u : variant == 31 ? 32u : 8u;
}
// 51 is 34 with multi-word items on narrow levels and each wave's first item taken statically
// (k_expand FLAGS bit 12), the only variants whose item_layout may set wpi > 1 are 51 and 52 (51 with
// nontemporal parent-seed loads, FLAGS bit 13)
inline uint32_t expand_max_wpi(int variant) { return variant == 51 || variant == 52 ? 16u : 1u; }
inline bool expand_tail_split(int variant) { return variant == 37 || variant == 38; }

}  // namespace fhh
