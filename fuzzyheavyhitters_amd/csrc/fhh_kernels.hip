// HIP kernels for gfx950 (MI355X): the per-level ibDCF key evaluation of
// sks-codes/fuzzyheavyhitters and the kernels around it.
//
//   k_expand        ibDCFKey::eval_bit for every (dim-prefix, client, side, dir)
//                   (ibDCF.rs:208-227, prg.rs:92-122, collect.rs:379-391). Integer/LDS bound.
//   k_eq_count      plaintext stand-in for the GC equality test: clients whose two share
//                   strings agree, per child (collect.rs:393-482 replaced)
//   k_share_planes  share-bit planes for the GC (collect.rs:393-418)
//   k_child_sums_fe* per-child sums of the share values: the in-process harness's simulated OT
//                   shares, or (ot_val set) the real protocol's garbled-table / C-OT outputs
//                   (collect.rs:439-501, 846-905; named k_sim_ot_fe before r06)
//   k_sum_fe*       per-child sums of host-provided FE / FE255 values (collect.rs:487-501)
//   k_keygen        batched gen_interval keygen (ibDCF.rs:84-173)
//   k_init_table    eval_init for every key (ibDCF.rs:229-236, collect.rs:67-92)
//   k_keys_from_aos add_key wire layout -> SoA device layout
#include "fhh_internal.h"
#include "expand_kernel.h"
#include "../../include/fhh.h"
// The measured-negative k_expand forms of r01-r03 (bitsliced VALU AES, the T-table + pair-sliced
// hybrid, the earlier T-table variants) and their generated AES programs were removed in r06; they are
// in git history at commit 78c7ebe (fhh_expand_bs.hip, expand_ps.h, aes_bs_gen.h, aes_ps_gen.h,
// tools/gen_aes_bs.py, tools/gen_aes_ps.py). The build holds the product
// variant 52 and the generic-AES variant 33 the parity suite compares it with.

namespace fhh {

__constant__ WordTable c_T0 = T0;

__device__ __forceinline__ uint32_t wave_id_uniform() {
    return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

__device__ __forceinline__ void fill_table(uint32_t* tbl) {
    for (int i = threadIdx.x; i < kTableWords; i += blockDim.x) tbl[i] = c_T0.v[i / kTableReplicas];
    __syncthreads();
}

// --------------------------------------------------------------------------------------
// k_expand: one wave = 64 consecutive clients of one dim-j prefix group. Per entry and
// lane: 2 sides x 2 directions = 4 AES blocks (NB = 4 in lockstep, or NB = 2 per side).
// CorWords of (level, dim, side, client) are loaded once per work item and reused for
// `group` entries. Work items are dealt grid-stride (static) or from an atomic counter.
// --------------------------------------------------------------------------------------
// ahead != nullptr: draw the next work item from the counter right after the first entry's
// seeds have been consumed, so the (contended) atomic completes under that entry's AES instead
// of stalling the next item's start (vmcnt retires in issue order, so it must not precede the
// loads this item waits on)
typedef uint32_t v4u32_t __attribute__((ext_vector_type(4)));

// NT: child seeds are written with the nontemporal hint — they are read again only at the next
// level, and 1.3 GB per launch left dirty in L2 costs a writeback at every kernel boundary
// STORE (diagnostic A/B only, never a product variant): 0 = every child seed, 1 = none (a store
// guarded by an output value that never occurs, so the AES stays live), 2 = dir-0 children only
// (about the half that survives a prune) — the HBM-write share of k_expand's time and power
// (entry group g, word w): clients 64 w .. 64 w + 63 of entries [e_base + g group, + group).
// NTL: parent seeds read with the nontemporal hint (each is read once per level; the CWs are
// re-read by every entry group of the level and should keep the L2)
template <class Tab, int NB, bool NT = false, bool PAIR = false, int STORE = 0, bool NTL = false>
__device__ __forceinline__ void expand_item_wg(const ExpandJob& J, uint32_t w, uint32_t g, const uint32_t* tbl,
                                               uint32_t lane, uint32_t b0, uint32_t b1, uint32_t* ahead = nullptr,
                                               uint32_t* next = nullptr) {
    const uint32_t c = w * 64 + lane;
    const size_t npad = J.npad, nw = J.nw;

    // CorWord for (level, dim, side) — ibDCF.rs:215-217 `cor_words[state.level]`
    const size_t krow = (size_t)J.level * J.K + 2 * J.dim;
    uint4 cw[2];
    uint64_t cwp[2][4];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        cw[s] = J.cw_seed[(krow + s) * npad + c];
#pragma unroll
        for (int b = 0; b < 4; b++) cwp[s][b] = J.cw_bits[((krow + s) * 4 + b) * nw + w];
    }

    const uint32_t e_begin = J.e_base + g * J.group;
    const uint32_t e_end = min(e_begin + J.group, J.n_live);
    for (uint32_t e = e_begin; e < e_end; e++) {
        const uint32_t src = J.live[e];
#pragma unroll
        for (int s0 = 0; s0 < 2; s0 += NB / 2) {
            uint32_t blk[NB][4];      // index (s - s0)*2 + dir
            uint64_t tw[NB / 2], yw[NB / 2];
            uint64_t pb[NB], py[NB];  // PRG control bits (tau.bits / tau.y_bits) as ballot planes
#pragma unroll
            for (int q = 0; q < NB / 2; q++) {
                const int s = s0 + q;
                uint4 sd;
                if constexpr (NTL) {
                    const v4u32_t v = __builtin_nontemporal_load(
                        reinterpret_cast<const v4u32_t*>(J.src_seed + ((size_t)src * 2 + s) * npad + c));
                    sd = make_uint4(v[0], v[1], v[2], v[3]);
                } else {
                    sd = J.src_seed[((size_t)src * 2 + s) * npad + c];
                }
                tw[q] = J.src_t[((size_t)src * 2 + s) * nw + w];
                yw[q] = J.src_y[((size_t)src * 2 + s) * nw + w];
                const uint32_t sw[4] = {sd.x, sd.y, sd.z, sd.w};
#pragma unroll
                for (int dir = 0; dir < 2; dir++) {
                    prg_ctr(sw, dir, blk[q * 2 + dir]);
                    uint32_t bit, ybit;
                    prg_ctrl_bits(blk[q * 2 + dir][0], dir, bit, ybit);
                    pb[q * 2 + dir] = __ballot(bit);
                    py[q * 2 + dir] = __ballot(ybit);
                }
            }
            if (ahead && e == e_begin && s0 == 0 && lane == 0) *next = atomicAdd(ahead, 1u);

            if constexpr (PAIR) aes0_mmo_pair<DevOpsX, Tab, NB>(blk, tbl, b0, b1);
            else aes0_mmo_tab<DevOpsX, Tab, NB>(blk, tbl, b0, b1);

#pragma unroll
            for (int q = 0; q < NB / 2; q++) {
                const int s = s0 + q;
                const uint32_t tmask = 0u - (uint32_t)((tw[q] >> lane) & 1);   // if state.bit
#pragma unroll
                for (int dir = 0; dir < 2; dir++) {
                    const uint32_t* o = blk[q * 2 + dir];
                    uint4 out;
                    out.x = o[0] ^ (cw[s].x & tmask);
                    out.y = o[1] ^ (cw[s].y & tmask);
                    out.z = o[2] ^ (cw[s].z & tmask);
                    out.w = o[3] ^ (cw[s].w & tmask);
                    const size_t de = (size_t)(2 * e + dir) * 2 + s;
                    const bool st = STORE == 0 || (STORE == 2 && dir == 0) ||
                                    (STORE == 1 && (out.x ^ out.y ^ out.z ^ out.w) == 0x5EED5EEDu && out.x == 0);
                    if (!st) {
                    } else if constexpr (NT) {
                        v4u32_t o4 = {out.x, out.y, out.z, out.w};
                        __builtin_nontemporal_store(o4, reinterpret_cast<v4u32_t*>(J.dst_seed + de * npad + c));
                    } else {
                        J.dst_seed[de * npad + c] = out;
                    }
                    if (lane == 0) {
                        // new_bit = tau.bits[dir] ^ (t & cw.bits[dir]);
                        // new_y = tau.y_bits[dir] ^ (t & cw.y_bits[dir]) ^ y   (ibDCF.rs:211-219)
                        J.dst_t[de * nw + w] = pb[q * 2 + dir] ^ (tw[q] & cwp[s][dir]);
                        J.dst_y[de * nw + w] = py[q * 2 + dir] ^ (tw[q] & cwp[s][2 + dir]) ^ yw[q];
                    }
                }
            }
        }
    }
}

template <class Tab, int NB, bool NT = false, bool PAIR = false, int STORE = 0>
__device__ __forceinline__ void expand_item(const ExpandJob& J, uint64_t local, const uint32_t* tbl, uint32_t lane,
                                            uint32_t b0, uint32_t b1, uint32_t* ahead = nullptr,
                                            uint32_t* next = nullptr) {
    expand_item_wg<Tab, NB, NT, PAIR, STORE>(J, (uint32_t)(local % J.nw), (uint32_t)(local / J.nw), tbl, lane, b0, b1,
                                             ahead, next);
}

// NB = 4 with the next entry's seeds / t / y prefetched while the current entry's AES runs.
template <class Tab, bool NT = false, bool PAIR = false>
__device__ __forceinline__ void expand_item_pf(const ExpandJob& J, uint64_t local, const uint32_t* tbl, uint32_t lane,
                                               uint32_t b0, uint32_t b1) {
    const uint32_t w = (uint32_t)(local % J.nw);
    const uint32_t g = (uint32_t)(local / J.nw);
    const uint32_t c = w * 64 + lane;
    const size_t npad = J.npad, nw = J.nw;
    const size_t krow = (size_t)J.level * J.K + 2 * J.dim;
    uint4 cw[2];
    uint64_t cwp[2][4];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        cw[s] = J.cw_seed[(krow + s) * npad + c];
#pragma unroll
        for (int b = 0; b < 4; b++) cwp[s][b] = J.cw_bits[((krow + s) * 4 + b) * nw + w];
    }
    const uint32_t e_begin = J.e_base + g * J.group;
    const uint32_t e_end = min(e_begin + J.group, J.n_live);
    if (e_begin >= e_end) return;
    uint4 sd[2];
    uint64_t tw[2], yw[2];
    {
        const uint32_t src = J.live[e_begin];
#pragma unroll
        for (int s = 0; s < 2; s++) {
            sd[s] = J.src_seed[((size_t)src * 2 + s) * npad + c];
            tw[s] = J.src_t[((size_t)src * 2 + s) * nw + w];
            yw[s] = J.src_y[((size_t)src * 2 + s) * nw + w];
        }
    }
    for (uint32_t e = e_begin; e < e_end; e++) {
        uint32_t blk[4][4];
        uint64_t pb[4], py[4];
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const uint32_t sw[4] = {sd[s].x, sd[s].y, sd[s].z, sd[s].w};
#pragma unroll
            for (int dir = 0; dir < 2; dir++) {
                prg_ctr(sw, dir, blk[s * 2 + dir]);
                uint32_t bit, ybit;
                prg_ctrl_bits(blk[s * 2 + dir][0], dir, bit, ybit);
                pb[s * 2 + dir] = __ballot(bit);
                py[s * 2 + dir] = __ballot(ybit);
            }
        }
        const uint64_t ctw[2] = {tw[0], tw[1]}, cyw[2] = {yw[0], yw[1]};
        if (e + 1 < e_end) {   // prefetch (wave-uniform branch)
            const uint32_t src = J.live[e + 1];
#pragma unroll
            for (int s = 0; s < 2; s++) {
                sd[s] = J.src_seed[((size_t)src * 2 + s) * npad + c];
                tw[s] = J.src_t[((size_t)src * 2 + s) * nw + w];
                yw[s] = J.src_y[((size_t)src * 2 + s) * nw + w];
            }
        }
        if constexpr (PAIR) aes0_mmo_pair<DevOpsX, Tab, 4>(blk, tbl, b0, b1);
        else aes0_mmo_tab<DevOpsX, Tab, 4>(blk, tbl, b0, b1);
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const uint32_t tmask = 0u - (uint32_t)((ctw[s] >> lane) & 1);
#pragma unroll
            for (int dir = 0; dir < 2; dir++) {
                const uint32_t* o = blk[s * 2 + dir];
                uint4 out;
                out.x = o[0] ^ (cw[s].x & tmask);
                out.y = o[1] ^ (cw[s].y & tmask);
                out.z = o[2] ^ (cw[s].z & tmask);
                out.w = o[3] ^ (cw[s].w & tmask);
                const size_t de = (size_t)(2 * e + dir) * 2 + s;
                if constexpr (NT) {
                    v4u32_t o4 = {out.x, out.y, out.z, out.w};
                    __builtin_nontemporal_store(o4, reinterpret_cast<v4u32_t*>(J.dst_seed + de * npad + c));
                } else {
                    J.dst_seed[de * npad + c] = out;
                }
                if (lane == 0) {
                    J.dst_t[de * nw + w] = pb[s * 2 + dir] ^ (ctw[s] & cwp[s][dir]);
                    J.dst_y[de * nw + w] = py[s * 2 + dir] ^ (ctw[s] & cwp[s][2 + dir]) ^ cyw[s];
                }
            }
        }
    }
}

// Wave timeline of the profiling variant (FLAGS bit 3, tools/tail_profile.py): per launch and
// wave {start after the LDS fill, exit, items} in 100 MHz s_memrealtime ticks, written by lane 0
// with vector stores into a caller buffer of g_wprof_cap launches; the last wave out bumps the
// launch index (the same exit detection that re-arms the work counter).
__device__ uint64_t* g_wprof_buf = nullptr;
__device__ uint32_t g_wprof_cap = 0;
__device__ uint32_t g_wprof_launch = 0;

// FLAGS: bit 0 = draw the next item one entry ahead, bit 1 = nontemporal child-seed stores,
// bit 2 = sibling-pair AES (dir 0 / dir 1 share rounds 1-2, aes0_mmo_pair), bit 3 = wave timeline,
// bit 4 = decode the end-phase items of item_layout (only the variants that lay them out:
// the extra decode state made the 1024-thread kernel spill), bits 7-11 were the r02 hybrid's VALU
// waves (removed in r06),
// bit 12 = MW: a bulk item may span wpi consecutive words (item_layout, narrow levels), and each
// wave's first item is its wave index instead of a counter draw (the counter then hands out items
// from nwaves on: 4 096 simultaneous first draws cost ≈ 46 µs at the counter's 88 per µs)
template <class Tab, int NB, int THR, int MINW, bool PF = false, int FLAGS = 0>
__global__ __launch_bounds__(THR, MINW) void k_expand(ExpandLaunch a, uint32_t* work_counter) {
    constexpr bool AHEAD = (FLAGS & 1) != 0;
    constexpr bool NT = (FLAGS & 2) != 0;
    constexpr bool PAIR = (FLAGS & 4) != 0;
    constexpr bool PROF = (FLAGS & 8) != 0;
    constexpr bool TAIL = (FLAGS & 16) != 0;
    constexpr int STORE = (FLAGS >> 5) & 3;   // diagnostic variants 43 / 44 only
    constexpr bool MW = (FLAGS & 4096) != 0;
    constexpr bool NTL = (FLAGS & 8192) != 0;   // bit 13: nontemporal parent-seed loads (MW path)
    static_assert(!(MW && (AHEAD || TAIL || PF)), "MW: plain dynamic items only");
    static_assert(((FLAGS >> 7) & 31) == 0, "the hybrid VALU waves were removed in r06");
    __shared__ uint32_t tbl[Tab::kWords];
    __shared__ uint32_t s_drained;   // bit h: a wave of this workgroup found head h dry
    for (int i = threadIdx.x; i < Tab::kWords; i += THR) tbl[i] = Tab::word(c_T0.v, i);
    if (threadIdx.x == 0) s_drained = 0;
    __syncthreads();
    uint64_t prof_t0 = 0, prof_items = 0;
    if constexpr (PROF) prof_t0 = wall_clock64();

    const uint32_t lane = threadIdx.x & 63;
    uint32_t b0, b1;
    Tab::bases(lane, b0, b1);
    const uint64_t wpb = THR / 64;
    const uint64_t nwaves = (uint64_t)gridDim.x * wpb;
    // sizes: kernel arguments (host-driven crawl) or LoopCtl (device-resident loop)
    const LoopCtl* ctl = a.ctl;
    const uint64_t total = ctl ? (ctl->abort ? 0 : ctl->total_items) : a.total_items;
    // Dynamic items come from H heads, one per XCD (blocks b and b + 8 share an XCD: one word
    // saturates at ≈88 dequeues/µs, 8 per-XCD heads do not), head h handing out items
    // draw_base + h + H·v. A block draws from its own head first, then from the others once they
    // run dry. The heads of a launch alternate between two sets by launch number: the first block
    // zeroes the other set for the next launch on the stream (the previous launch, done, used it),
    // so there is no exit count (4 096 same-address exit atomics alone cost ≈46 µs per launch).
    constexpr uint32_t H = AHEAD ? 1u : kExpandHeads;
    uint32_t* heads = work_counter ? work_counter + kExpandSlot0 + (a.seq & 1) * kExpandHeads * kExpandSlotStride : nullptr;
    if (work_counter && blockIdx.x == 0 && threadIdx.x < kExpandHeads)
        atomicExch(work_counter + kExpandSlot0 + ((a.seq + 1) & 1) * kExpandHeads * kExpandSlotStride +
                       threadIdx.x * kExpandSlotStride, 0u);
    // (MW: wide levels, one-word items, keep one head — the per-XCD split measured ≈1 % slower there)
    const uint32_t nh = MW ? (__builtin_amdgcn_readfirstlane(ctl ? ctl->wpi : a.wpi) > 1 ? H : 1u) : H;
    const uint32_t home = blockIdx.x & (nh - 1);
    const uint64_t draw_base = MW ? nwaves : 0;   // the first nwaves items are dealt statically (MW)
    // lane 0 draws; bit h of s_drained: a wave of this block found head h dry (its siblings skip it)
    auto draw = [&]() -> uint64_t {
        uint64_t it = total;
        if (lane == 0) {
            for (uint32_t k = 0; k < nh; k++) {
                const uint32_t h = (home + k) & (nh - 1);
                if ((*(volatile uint32_t*)&s_drained >> h) & 1u) continue;
                const uint32_t v = atomicAdd(heads + h * kExpandSlotStride, 1u);
                const uint64_t cand = draw_base + h + (uint64_t)nh * v;
                if (cand < total) {
                    it = cand;
                    break;
                }
                atomicOr(&s_drained, 1u << h);
            }
        }
        return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(it >> 32)) << 32) |
               __builtin_amdgcn_readfirstlane((uint32_t)it);
    };
    uint64_t item = (uint64_t)blockIdx.x * wpb + wave_id_uniform();   // static, MW
    if (heads && !MW) item = draw();
    const uint64_t items_a = TAIL ? (ctl ? ctl->items_a : a.items_a) : total;
    while (item < total) {
        // bulk items [0, items_a), then the end phase (item_layout): same job order in each
        const bool tail = TAIL && item >= items_a;
        uint32_t ji = 0;
        if (ctl) {
            const uint64_t* beg = tail ? ctl->item_begin_b : ctl->item_begin;
            while (ji + 1 < a.njobs && item >= beg[ji + 1]) ji++;
        } else if (tail) {
            while (ji + 1 < a.njobs && item >= a.job[ji + 1].item_begin_b) ji++;
        } else {
            while (ji + 1 < a.njobs && item >= a.job[ji + 1].item_begin) ji++;
        }
        ExpandJob J = a.job[ji];
        if (ctl) {
            J.n_live = ctl->n_live[ji % a.jobs_per_ctx];
            J.group = ctl->group;
            J.item_begin = ctl->item_begin[ji];
            if constexpr (TAIL) {
                J.group_b = ctl->group_b;
                J.split = ctl->split[ji];
                J.item_begin_b = ctl->item_begin_b[ji];
            }
        }
        J.e_base = 0;
        if constexpr (TAIL) {
            if (tail) {
                J.e_base = J.split;
                J.group = J.group_b;
                J.item_begin = J.item_begin_b;
            } else {
                J.n_live = J.split;
            }
        }
        uint32_t nxt = 0;
        if constexpr (PROF) prof_items++;
        if constexpr (MW) {
            // bulk item = (entry group, chunk of wpi words): local = group * ceil(nw / wpi) + chunk
            // (wpi = 1 is the one-word item of the other variants: grp = local / nw, w = local % nw)
            const uint32_t wpi = __builtin_amdgcn_readfirstlane(ctl ? ctl->wpi : a.wpi);
            const uint64_t local = item - J.item_begin;
            const uint32_t nwi = (J.nw + wpi - 1) / wpi;
            const uint32_t grp = (uint32_t)(local / nwi), w0 = (uint32_t)(local % nwi) * wpi, w1 = min(J.nw, w0 + wpi);
            for (uint32_t w = w0; w < w1; w++)
                expand_item_wg<Tab, NB, NT, PAIR, STORE, NTL>(J, w, grp, tbl, lane, b0, b1);
        } else if constexpr (PF) expand_item_pf<Tab, NT, PAIR>(J, item - J.item_begin, tbl, lane, b0, b1);
        else if constexpr (AHEAD) expand_item<Tab, NB, NT, PAIR, STORE>(J, item - J.item_begin, tbl, lane, b0, b1, heads, &nxt);
        else expand_item<Tab, NB, NT, PAIR, STORE>(J, item - J.item_begin, tbl, lane, b0, b1);
        if (heads) {
            if constexpr (AHEAD) item = (uint64_t)__builtin_amdgcn_readfirstlane(nxt) + draw_base;   // H = 1
            else item = draw();
        } else {
            item += nwaves;
        }
    }
    if constexpr (PROF) {
        const uint64_t t1 = wall_clock64();
        const uint32_t L = g_wprof_launch;
        if (lane == 0 && g_wprof_buf && L < g_wprof_cap) {
            uint64_t* r = g_wprof_buf + ((uint64_t)L * nwaves + (uint64_t)blockIdx.x * wpb + wave_id_uniform()) * 3;
            r[0] = prof_t0;
            r[1] = t1;
            r[2] = prof_items;
        }
    }
    if constexpr (PROF) {   // the wave timeline's launch index: the last wave out bumps it
        if (work_counter && lane == 0) {
            const uint32_t done = atomicAdd(work_counter + kExpandProfSlot, 1u);
            if (done + 1 == (uint32_t)nwaves) {
                atomicAdd(&g_wprof_launch, 1u);
                atomicExch(work_counter + kExpandProfSlot, 0u);
            }
        }
    }
}

// arm the wave timeline: buf = device buffer of cap launches x grid waves x 3 u64 (NULL disarms)
extern "C" int fhh_wave_profile_arm(int device, uint64_t* buf, uint32_t cap) {
    if (hipSetDevice(device) != hipSuccess) return FHH_E_HIP;
    const uint32_t zero = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_wprof_buf), &buf, sizeof buf) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_wprof_cap), &cap, sizeof cap) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_wprof_launch), &zero, sizeof zero) != hipSuccess)
        return FHH_E_HIP;
    return FHH_OK;
}

extern "C" int fhh_wave_profile_launches(int device, uint32_t* launches) {
    if (hipSetDevice(device) != hipSuccess || !launches) return FHH_E_HIP;
    return hipMemcpyFromSymbol(launches, HIP_SYMBOL(g_wprof_launch), sizeof *launches) == hipSuccess ? FHH_OK : FHH_E_HIP;
}

// Variant table (fhh_set_variant): id, table layout, blocks per lane, threads, min waves, dynamic
// items, [prefetch, FLAGS]: 52 is the product default, 33 the generic-AES form the parity suite
// compares it with (the other ids of r01-r03 were removed in r06).
#define FHH_EXPAND_VARIANTS(X)                                   \
    X(33, Tab4T32<DevOpsX>, 4, 1024, 1, true, false, 2)            \
    X(52, Tab4T32<DevOpsX>, 4, 1024, 1, true, false, 6 | 4096 | 8192)

struct VariantInfo {
    const void* fn;
    int threads;
    bool dynamic;
    const char* name;
};

static VariantInfo variant_info(int v) {
    switch (v) {
#define FHH_CASE(id, TAB, NB, THR, MINW, DYN, ...) \
    case id: return VariantInfo{reinterpret_cast<const void*>(&k_expand<TAB, NB, THR, MINW, ##__VA_ARGS__>), THR, DYN, TAB::kName};
        FHH_EXPAND_VARIANTS(FHH_CASE)
#undef FHH_CASE
        default: return VariantInfo{nullptr, 0, false, ""};
    }
}

int expand_variant_count() { return 53; }   // ids 0..52; this build holds 33 and 52

const char* expand_variant_name(int v) { return variant_info(v).name; }

hipError_t launch_expand(const ExpandLaunch& a0, int variant, int grid, uint32_t* work_counter, uint32_t* seq,
                         hipStream_t stream) {
    if (a0.total_items == 0) return hipSuccess;
    ExpandLaunch a = a0;
    // the head set of this launch is chosen by the sequence's parity, and the launch zeroes the other
    // set for the next one: the sequence advances only once a dynamic launch has been enqueued, so a
    // refused or failed launch cannot make the next one draw from a set the launch before used up
    a.seq = *seq;
    const VariantInfo vi = variant_info(variant);
    if (!vi.fn) return hipErrorInvalidValue;
    const uint64_t wpb = vi.threads / 64;
    const uint64_t blocks_needed = (a.total_items + wpb - 1) / wpb;
    // device-resident loop: the item count is only known on the device -> full persistent grid
    const int g = a.ctl ? grid : (int)(blocks_needed < (uint64_t)grid ? blocks_needed : (uint64_t)grid);
    // dynamic mode: the counter slot of launch a.seq must be zero at launch (the previous
    // k_expand on this counter zeroed it; fhh_create zeroes both)
    uint32_t* ctr = vi.dynamic ? work_counter : nullptr;
    switch (variant) {
#define FHH_CASE(id, TAB, NB, THR, MINW, DYN, ...) \
    case id: hipLaunchKernelGGL((k_expand<TAB, NB, THR, MINW, ##__VA_ARGS__>), dim3(g), dim3(THR), 0, stream, a, ctr); break;
        FHH_EXPAND_VARIANTS(FHH_CASE)
#undef FHH_CASE
        default: return hipErrorInvalidValue;
    }
    const hipError_t e = hipGetLastError();
    if (e == hipSuccess && ctr) ++*seq;
    return e;
}

int expand_grid(int device, int variant) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
    const VariantInfo vi = variant_info(variant);
    int per_cu = 0;
    const size_t dyn = 0;
    if (!vi.fn || hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, vi.fn, vi.threads, dyn) != hipSuccess ||
        per_cu <= 0)
        per_cu = 1;
    return cus * per_cu;
}

int expand_threads(int variant) { return variant_info(variant).threads; }

// --------------------------------------------------------------------------------------
// Child-level kernels (one block per child, grid-stride).
// --------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

template <int NV>
__device__ __forceinline__ void block_sum_u64(uint64_t (&v)[NV], uint64_t* red /*[NV][kReduceThreads/64]*/) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nwv = blockDim.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; k++) v[k] = wave_sum_u64(v[k]);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < NV; k++) red[k * (kReduceThreads / 64) + wid] = v[k];
    __syncthreads();
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < NV; k++) {
            uint64_t s = 0;
            for (int i = 0; i < nwv; i++) s += red[k * (kReduceThreads / 64) + i];
            v[k] = s;
        }
    }
    __syncthreads();
}

__device__ __forceinline__ uint64_t child_count(const ChildArgs& a) {
    return a.ctl ? (a.ctl->abort ? 0 : a.ctl->C) : a.C;
}

// the children a windowed kernel (GC + OT glue) visits: [c_off, min(C, c_off + c_cnt))
__device__ __forceinline__ uint64_t child_end(const ChildArgs& a) {
    const uint64_t C = child_count(a);
    if (!a.c_cnt) return C;
    const uint64_t e = a.c_off + a.c_cnt;
    return e < C ? e : C;
}

__device__ __forceinline__ void child_entries(const ChildArgs& a, uint64_t c, uint32_t (&e)[kMaxDims]) {
    const uint64_t p = c >> a.d;
    const uint32_t i = (uint32_t)(c & ((1u << a.d) - 1));
#pragma unroll
    for (int j = 0; j < kMaxDims; j++)
        if (j < (int)a.d) e[j] = 2 * a.parent_pos[p * a.d + j] + ((i >> j) & 1);
}

// eq word: bit = 1 iff the client's share string is identical on both servers
__device__ __forceinline__ uint64_t eq_word(const ChildArgs& a, const uint32_t (&e)[kMaxDims], uint32_t w) {
    uint64_t m = a.valid[w];
#pragma unroll
    for (int j = 0; j < kMaxDims; j++) {
        if (j < (int)a.d) {
#pragma unroll
            for (int s = 0; s < 2; s++) {
                const size_t idx = ((size_t)e[j] * 2 + s) * a.nw + w;
                const uint64_t e0 = a.s0.t[j][idx] ^ a.s0.y[j][idx];
                const uint64_t e1 = a.s1.t[j][idx] ^ a.s1.y[j][idx];
                m &= ~(e0 ^ e1);
            }
        }
    }
    return m;
}

// 1024 threads per child and two words per thread per pass, both words' loads issued before
// either popcount: at configs[1] (nw = 1563) one pass covers a child, so the kernel is one
// round of load latency instead of six dependent ones (r01: 10 us per level at 256 threads)
constexpr int kEqThreads = 1024;
__global__ __launch_bounds__(kEqThreads) void k_eq_count(ChildArgs a, uint64_t* counts) {
    __shared__ uint64_t red[kEqThreads / 64];
    const uint64_t C_ = child_count(a);
    for (uint64_t c = blockIdx.x; c < C_; c += gridDim.x) {
        uint32_t e[kMaxDims];
        child_entries(a, c, e);
        uint64_t v[1] = {0};
        for (uint32_t w = threadIdx.x; w < a.nw; w += 2 * kEqThreads) {
            const uint32_t w1 = w + kEqThreads;
            const uint64_t m0 = eq_word(a, e, w);
            const uint64_t m1 = w1 < a.nw ? eq_word(a, e, w1) : 0;
            v[0] += __popcll(m0) + __popcll(m1);
        }
        block_sum_u64<1>(v, red);
        if (threadIdx.x == 0) counts[c] = v[0];
    }
}

static int child_grid(uint64_t C) { return (int)(C < 65535 ? (C ? C : 1) : 65535); }
static uint64_t window_cap(const ChildArgs& a) { return a.c_cnt && a.c_cnt < a.C ? a.c_cnt : a.C; }

hipError_t launch_eq_count(const ChildArgs& a, uint64_t* counts, hipStream_t stream) {
    if (a.C == 0) return hipSuccess;
    hipLaunchKernelGGL(k_eq_count, dim3(child_grid(a.C)), dim3(kEqThreads), 0, stream, a, counts);
    return hipGetLastError();
}

// out [C][2d][nw]: left dims then right dims, E = y ^ t (collect.rs:399-405); with a child window
// (c_cnt > 0) only children [c_off, c_off + c_cnt), at rows c - c_off
__global__ __launch_bounds__(kReduceThreads) void k_share_planes(ChildArgs a, uint64_t* out) {
    const uint64_t C_ = child_end(a);
    for (uint64_t c = a.c_off + blockIdx.x; c < C_; c += gridDim.x) {
        uint32_t e[kMaxDims];
        child_entries(a, c, e);
        const uint32_t pnw = a.plane_nw ? a.plane_nw : a.nw;
        for (uint32_t w = threadIdx.x; w < pnw; w += blockDim.x) {
#pragma unroll
            for (int s = 0; s < 2; s++)
#pragma unroll
                for (int j = 0; j < kMaxDims; j++)
                    if (j < (int)a.d) {
                        const size_t idx = ((size_t)e[j] * 2 + s) * a.nw + w;
                        out[((size_t)(c - a.c_off) * 2 * a.d + (size_t)s * a.d + j) * pnw + w] =
                            w < a.nw ? (a.s0.t[j][idx] ^ a.s0.y[j][idx]) & a.valid[w] : 0ull;
                    }
        }
    }
}

hipError_t launch_share_planes(const ChildArgs& a, uint64_t* out, hipStream_t stream) {
    if (a.C == 0) return hipSuccess;
    hipLaunchKernelGGL(k_share_planes, dim3(child_grid(window_cap(a))), dim3(kReduceThreads), 0, stream, a, out);
    return hipGetLastError();
}

// ---- simulated OT share values --------------------------------------------------------
// PRF: mix64 chain (SplitMix64 finaliser) over (seed, level, child, client, word).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

constexpr uint64_t kFeP = (1ull << 62) - (1ull << 30) - 1;

// the equality bit the OT conversion consumes: plaintext (t, y) comparison, or in GC mode the
// evaluator's garbled-circuit output XOR the garbler's mask (the OT receiver's choice bit and
// the sender's message order, collect.rs:437-471: the received value is r0 iff eq)
__device__ __forceinline__ bool sim_eq_bit(const ChildArgs& a, const uint32_t (&e)[kMaxDims], uint64_t c, uint32_t i) {
    if (a.gc_out) return ((a.gc_out[(c - a.c_off) * a.gc_N + i] ^ a.gc_mask) & 1u) != 0;
    return (eq_word(a, e, i >> 6) >> (i & 63)) & 1;
}

// grid (children, client chunks of kSimOtChunk): one child per block row would leave the chip
// at ~3 waves per CU for the usual few hundred children (255 µs per level at configs[1]); the
// chunks' limb sums meet in partials by 64-bit atomics (zeroed by the launcher)
constexpr uint32_t kSimOtChunk = 16 * kReduceThreads;
__global__ __launch_bounds__(kReduceThreads) void k_child_sums_fe(ChildArgs a, uint64_t* partials) {
    __shared__ uint64_t red[4 * (kReduceThreads / 64)];
    const uint64_t base = mix64(a.prf_seed ^ a.level);
    const uint64_t C_ = child_end(a);
    const uint32_t i_begin = blockIdx.y * kSimOtChunk;
    const uint32_t i_end = min(i_begin + kSimOtChunk, a.n);
    for (uint64_t c = a.c_off + blockIdx.x; c < C_; c += gridDim.x) {
        uint32_t e[kMaxDims];
        child_entries(a, c, e);
        const uint64_t bc = mix64(base ^ c);
        uint64_t v[4] = {0, 0, 0, 0};
        for (uint32_t i = i_begin + threadIdx.x; i < i_end; i += blockDim.x) {
            uint64_t r1, v1;
            if (a.ot_val[0]) {   // the correlated OT's node values (OtArgs mode 2): garbler v + mask, receiver
                const size_t t = (c - a.c_off) * a.gc_N + i;
                r1 = static_cast<const uint64_t*>(a.ot_val[0])[t];
                v1 = static_cast<const uint64_t*>(a.ot_val[1])[t];
            } else {             // simulated OT shares (ideal OT harness)
                uint64_t r0 = mix64(mix64(bc ^ (a.client_base + i)) ^ 0ull) & ((1ull << 62) - 1);
                if (r0 >= kFeP) r0 -= kFeP;
                r1 = (r0 + 1 == kFeP) ? 0 : r0 + 1;              // r1 = r0 + one (collect.rs:443-444)
                v1 = sim_eq_bit(a, e, c, i) ? r0 : r1;           // receiver gets pair[o] (A.5)
            }
            v[0] += r1 & 0xFFFFFFFFull;
            v[1] += r1 >> 32;
            v[2] += v1 & 0xFFFFFFFFull;
            v[3] += v1 >> 32;
        }
        block_sum_u64<4>(v, red);
        if (threadIdx.x == 0)
            for (int k = 0; k < 4; k++) atomicAdd(reinterpret_cast<unsigned long long*>(partials + c * 4 + k), v[k]);
    }
}

hipError_t launch_child_sums_fe(const ChildArgs& a, uint64_t* partials, hipStream_t stream, bool zero) {
    if (a.C == 0) return hipSuccess;
    if (zero) {
        const hipError_t e = hipMemsetAsync(partials, 0, (size_t)a.C * 4 * sizeof(uint64_t), stream);
        if (e != hipSuccess) return e;
    }
    const uint32_t chunks = a.n ? (a.n + kSimOtChunk - 1) / kSimOtChunk : 1;
    hipLaunchKernelGGL(k_child_sums_fe, dim3(child_grid(window_cap(a)), chunks), dim3(kReduceThreads), 0, stream, a,
                       partials);
    return hipGetLastError();
}

// 255-bit helpers on 4 x u64 little-endian
__device__ __forceinline__ void fe255_canon(uint64_t (&x)[4]) {
    // x < 2^255; subtract p = 2^255 - 19 when x >= p (i.e. x + 19 carries into bit 255)
    uint64_t t[4];
    unsigned __int128 acc = (unsigned __int128)x[0] + 19;
    t[0] = (uint64_t)acc;
    acc = (unsigned __int128)x[1] + (uint64_t)(acc >> 64);
    t[1] = (uint64_t)acc;
    acc = (unsigned __int128)x[2] + (uint64_t)(acc >> 64);
    t[2] = (uint64_t)acc;
    acc = (unsigned __int128)x[3] + (uint64_t)(acc >> 64);
    t[3] = (uint64_t)acc;
    if (t[3] >> 63) {
        x[0] = t[0];
        x[1] = t[1];
        x[2] = t[2];
        x[3] = t[3] & 0x7FFFFFFFFFFFFFFFull;
    }
}

// BlockPair <-> 4 x u64 little-endian limbs: the value's 32 big-endian bytes, block 0 = bytes
// 0..15 (limbs 3, 2), block 1 = bytes 16..31 (limbs 1, 0) (field.rs:465-492); a block's 16
// bytes as four little-endian u32 words
__device__ __forceinline__ uint4 limbs_to_block(uint64_t hi, uint64_t lo) {
    return make_uint4(__builtin_bswap32((uint32_t)(hi >> 32)), __builtin_bswap32((uint32_t)hi),
                      __builtin_bswap32((uint32_t)(lo >> 32)), __builtin_bswap32((uint32_t)lo));
}
__device__ __forceinline__ void blockpair_to_limbs(uint4 b0, uint4 b1, uint64_t (&r)[4]) {
    r[3] = ((uint64_t)__builtin_bswap32(b0.x) << 32) | __builtin_bswap32(b0.y);
    r[2] = ((uint64_t)__builtin_bswap32(b0.z) << 32) | __builtin_bswap32(b0.w);
    r[1] = ((uint64_t)__builtin_bswap32(b1.x) << 32) | __builtin_bswap32(b1.y);
    r[0] = ((uint64_t)__builtin_bswap32(b1.z) << 32) | __builtin_bswap32(b1.w);
}

__global__ __launch_bounds__(kReduceThreads) void k_child_sums_fe255(ChildArgs a, uint64_t* partials) {
    __shared__ uint64_t red[16 * (kReduceThreads / 64)];
    const uint64_t base = mix64(a.prf_seed ^ a.level);
    const uint64_t C_ = child_end(a);
    for (uint64_t c = a.c_off + blockIdx.x; c < C_; c += gridDim.x) {
        uint32_t e[kMaxDims];
        child_entries(a, c, e);
        const uint64_t bc = mix64(base ^ c);
        uint64_t v[16];
#pragma unroll
        for (int k = 0; k < 16; k++) v[k] = 0;
        for (uint32_t i = threadIdx.x; i < a.n; i += blockDim.x) {
            uint64_t r1[4], got[4];
            if (a.ot_val[0]) {   // the correlated OT's node values (OtArgs mode 3), BlockPairs; the receiver's
                                 // unreduced, as FieldElm::try_from(BlockPair) reads them (field.rs:466-476)
                const size_t t = (c - a.c_off) * a.gc_N + i;
                const uint4* g = static_cast<const uint4*>(a.ot_val[0]);
                const uint4* r = static_cast<const uint4*>(a.ot_val[1]);
                blockpair_to_limbs(g[2 * t], g[2 * t + 1], r1);
                blockpair_to_limbs(r[2 * t], r[2 * t + 1], got);
            } else {             // simulated OT shares (ideal OT harness)
                const bool eq = sim_eq_bit(a, e, c, i);
                const uint64_t bi = mix64(bc ^ (a.client_base + i));
                uint64_t r0[4];
#pragma unroll
                for (int k = 0; k < 4; k++) r0[k] = mix64(bi ^ (uint64_t)k);
                r0[3] &= 0x7FFFFFFFFFFFFFFFull;
                fe255_canon(r0);
                // r1 = r0 + 1 mod p
                unsigned __int128 acc = (unsigned __int128)r0[0] + 1;
                r1[0] = (uint64_t)acc;
#pragma unroll
                for (int k = 1; k < 4; k++) {
                    acc = (unsigned __int128)r0[k] + (uint64_t)(acc >> 64);
                    r1[k] = (uint64_t)acc;
                }
                fe255_canon(r1);
#pragma unroll
                for (int k = 0; k < 4; k++) got[k] = eq ? r0[k] : r1[k];
            }
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint64_t x1 = got[k];
                v[2 * k] += r1[k] & 0xFFFFFFFFull;
                v[2 * k + 1] += r1[k] >> 32;
                v[8 + 2 * k] += x1 & 0xFFFFFFFFull;
                v[8 + 2 * k + 1] += x1 >> 32;
            }
        }
        block_sum_u64<16>(v, red);
        if (threadIdx.x == 0)
            for (int k = 0; k < 16; k++) partials[c * 16 + k] = v[k];
    }
}

hipError_t launch_child_sums_fe255(const ChildArgs& a, uint64_t* partials, hipStream_t stream) {
    if (a.C == 0) return hipSuccess;
    hipLaunchKernelGGL(k_child_sums_fe255, dim3(child_grid(window_cap(a))), dim3(kReduceThreads), 0, stream, a, partials);
    return hipGetLastError();
}

// ---- per-child sums of the OT outputs (collect.rs:487-501, 891-905) ----------------------------
// Values [C][ld] in one of the FHH_VALS_* formats (include/fhh.h): host-provided u64 / u32 limbs
// (staged by the engine) or OT outputs left on the device (16-B blocks: an FE little-endian in
// bytes 0..7, fastfield.rs:414-431; a FieldElm as a BlockPair of 32 big-endian bytes,
// field.rs:465-492). Sums are 32-bit-limb partials in u64 (2^32 clients of headroom), reduced once
// on the host: [C][2] for FE, [C][8] for FE255 (the exact unreduced BigUint add_lazy sum).
__global__ __launch_bounds__(kReduceThreads) void k_sum_fe(const uint64_t* vals, uint64_t C, uint64_t n, uint64_t ld,
                                                          uint32_t stride, uint64_t* partials) {
    __shared__ uint64_t red[2 * (kReduceThreads / 64)];
    for (uint64_t c = blockIdx.x; c < C; c += gridDim.x) {
        uint64_t v[2] = {0, 0};
        for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
            const uint64_t x = vals[(c * ld + i) * stride];
            v[0] += x & 0xFFFFFFFFull;
            v[1] += x >> 32;
        }
        block_sum_u64<2>(v, red);
        if (threadIdx.x == 0) {
            partials[c * 2] = v[0];
            partials[c * 2 + 1] = v[1];
        }
    }
}

template <bool BLOCKPAIR>
__global__ __launch_bounds__(kReduceThreads) void k_sum_fe255(const uint32_t* vals, uint64_t C, uint64_t n,
                                                             uint64_t ld, uint64_t* partials) {
    __shared__ uint64_t red[8 * (kReduceThreads / 64)];
    for (uint64_t c = blockIdx.x; c < C; c += gridDim.x) {
        uint64_t v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
            const uint4* p = reinterpret_cast<const uint4*>(vals + (c * ld + i) * 8);
            const uint4 lo = p[0], hi = p[1];
            if (BLOCKPAIR) {
                uint64_t r[4];
                blockpair_to_limbs(lo, hi, r);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    v[2 * k] += r[k] & 0xFFFFFFFFull;
                    v[2 * k + 1] += r[k] >> 32;
                }
            } else {
                v[0] += lo.x; v[1] += lo.y; v[2] += lo.z; v[3] += lo.w;
                v[4] += hi.x; v[5] += hi.y; v[6] += hi.z; v[7] += hi.w;
            }
        }
        block_sum_u64<8>(v, red);
        if (threadIdx.x == 0)
            for (int k = 0; k < 8; k++) partials[c * 8 + k] = v[k];
    }
}

hipError_t launch_sum_vals(const void* vals, uint32_t fmt, uint64_t C, uint64_t n, uint64_t ld, uint64_t* partials,
                           hipStream_t stream) {
    if (C == 0) return hipSuccess;
    switch (fmt) {
        case FHH_VALS_FE_U64:
        case FHH_VALS_FE_BLOCK:
            hipLaunchKernelGGL(k_sum_fe, dim3(child_grid(C)), dim3(kReduceThreads), 0, stream,
                               static_cast<const uint64_t*>(vals), C, n, ld, fmt == FHH_VALS_FE_BLOCK ? 2u : 1u,
                               partials);
            break;
        case FHH_VALS_FE255_LIMBS:
            hipLaunchKernelGGL(k_sum_fe255<false>, dim3(child_grid(C)), dim3(kReduceThreads), 0, stream,
                               static_cast<const uint32_t*>(vals), C, n, ld, partials);
            break;
        case FHH_VALS_FE255_BLOCKPAIR:
            hipLaunchKernelGGL(k_sum_fe255<true>, dim3(child_grid(C)), dim3(kReduceThreads), 0, stream,
                               static_cast<const uint32_t*>(vals), C, n, ld, partials);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// --------------------------------------------------------------------------------------
// k_keygen: one wave = 64 clients of one key (dim j, side). Restates gen_cor_word
// (ibDCF.rs:84-119) level by level; 4 AES blocks per level per lane (both seeds, both
// directions). Writes server 0's and server 1's key arrays (shared cor_words).
// --------------------------------------------------------------------------------------
__global__ __launch_bounds__(kExpandThreads) void k_keygen(KeygenArgs a) {
    __shared__ uint32_t tbl[kTableWords];
    fill_table(tbl);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t lanebase = lane * 4;
    const uint64_t wpb = blockDim.x >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * wpb;
    const uint64_t items = (uint64_t)a.K * a.nw;
    for (uint64_t item = (uint64_t)blockIdx.x * wpb + wave_id_uniform(); item < items; item += nwaves) {
        const uint32_t kk = (uint32_t)(item / a.nw);
        const uint32_t w = (uint32_t)(item % a.nw);
        const uint32_t j = kk >> 1, side_idx = kk & 1;
        const uint32_t side = side_idx == 0 ? 1u : 0u;   // left key: side=true, right: false (ibDCF.rs:170-171)
        const uint64_t c = (uint64_t)w * 64 + lane;
        const bool valid = c < a.n;
        const uint8_t* alpha = (side_idx == 0 ? a.left_bits : a.right_bits) + (valid ? (c * a.d + j) * a.L : 0);

        uint32_t seed[2][4];
        if (valid) {
            const uint4* rs = reinterpret_cast<const uint4*>(a.root_seeds + ((c * a.d + j) * 2 + side_idx) * 32);
            const uint4 r0 = rs[0], r1 = rs[1];
            seed[0][0] = r0.x; seed[0][1] = r0.y; seed[0][2] = r0.z; seed[0][3] = r0.w;
            seed[1][0] = r1.x; seed[1][1] = r1.y; seed[1][2] = r1.z; seed[1][3] = r1.w;
        } else {
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int k = 0; k < 4; k++) seed[b][k] = 0;
        }
#pragma unroll
        for (int b = 0; b < 2; b++)
            a.root[b][(size_t)kk * a.npad + c] = make_uint4(seed[b][0], seed[b][1], seed[b][2], seed[b][3]);
        if (lane == 0) {
            a.key_idx[0][(size_t)kk * a.nw + w] = 0;         // key_idx = false
            a.key_idx[1][(size_t)kk * a.nw + w] = ~0ull;     // key_idx = true (ibDCF.rs:153-161)
        }
        uint32_t t[2] = {0u, 1u};                           // root_bits = (false, true), ibDCF.rs:140

        for (uint32_t l = 0; l < a.L; l++) {
            const uint32_t bit = valid ? (alpha[l] ? 1u : 0u) : 0u;
            uint32_t blk[4][4];                             // index b*2 + dir
            uint32_t pbit[4], pyb[4];
#pragma unroll
            for (int b = 0; b < 2; b++)
#pragma unroll
                for (int dir = 0; dir < 2; dir++) {
                    prg_ctr(seed[b], dir, blk[b * 2 + dir]);
                    prg_ctrl_bits(blk[b * 2 + dir][0], dir, pbit[b * 2 + dir], pyb[b * 2 + dir]);
                }
            aes0_mmo<DevOps, 4>(blk, tbl, lanebase);

            const uint32_t keep = bit, lose = bit ^ 1u;
            uint32_t cws[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t l0 = lose ? blk[1][k] : blk[0][k];
                const uint32_t l1 = lose ? blk[3][k] : blk[2][k];
                cws[k] = l0 ^ l1;                                   // ibDCF.rs:91
            }
            // data.b.bits.k = pbit[b*2+k], data.b.y_bits.k = pyb[b*2+k]
            const uint32_t cb0 = pbit[0] ^ pbit[2] ^ bit ^ 1u;       // :93
            const uint32_t cb1 = pbit[1] ^ pbit[3] ^ bit;            // :94
            const uint32_t cy0 = pyb[0] ^ pyb[2] ^ (bit & (side ^ 1u) & 1u);   // :97 bit & !side
            const uint32_t cy1 = pyb[1] ^ pyb[3] ^ ((bit ^ 1u) & side);        // :98 !bit & side
            const uint32_t cwb_keep = keep ? cb1 : cb0;
#pragma unroll
            for (int b = 0; b < 2; b++) {                            // :103-116
                const uint32_t tm = 0u - t[b];
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint32_t kept = keep ? blk[b * 2 + 1][k] : blk[b * 2][k];
                    seed[b][k] = kept ^ (cws[k] & tm);
                }
                const uint32_t nb = (keep ? pbit[b * 2 + 1] : pbit[b * 2]) ^ (t[b] & cwb_keep);
                t[b] = nb;
            }
            const size_t row = (size_t)l * a.K + kk;
            const uint4 cwv = make_uint4(cws[0], cws[1], cws[2], cws[3]);
            a.cw_seed[0][row * a.npad + c] = cwv;
            a.cw_seed[1][row * a.npad + c] = cwv;
            const uint64_t q0 = __ballot(cb0), q1 = __ballot(cb1), q2 = __ballot(cy0), q3 = __ballot(cy1);
            if (lane == 0) {
                const uint64_t q[4] = {q0, q1, q2, q3};
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    a.cw_bits[0][(row * 4 + b) * a.nw + w] = q[b];
                    a.cw_bits[1][(row * 4 + b) * a.nw + w] = q[b];
                }
            }
        }
    }
}

hipError_t launch_keygen(const KeygenArgs& a, hipStream_t stream) {
    const uint64_t items = (uint64_t)a.K * a.nw;
    if (items == 0) return hipSuccess;
    const uint64_t wpb = kExpandThreads / 64;
    uint64_t blocks = (items + wpb - 1) / wpb;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_keygen, dim3((unsigned)blocks), dim3(kExpandThreads), 0, stream, a);
    return hipGetLastError();
}

// --------------------------------------------------------------------------------------
// eval_init for dim `dim` -> entry 0 of that dim's table: seed = root_seed, t = y = key_idx
// --------------------------------------------------------------------------------------
__global__ void k_init_table(const uint4* root, const uint64_t* key_idx, uint32_t dim, uint32_t npad, uint32_t nw,
                             uint4* seed, uint64_t* t, uint64_t* y) {
    const uint64_t total = (uint64_t)2 * npad;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = (uint32_t)(i / npad), c = (uint32_t)(i % npad);
        seed[(size_t)s * npad + c] = root[((size_t)2 * dim + s) * npad + c];
        if (c < nw) {
            const uint64_t k = key_idx[((size_t)2 * dim + s) * nw + c];
            t[(size_t)s * nw + c] = k;
            y[(size_t)s * nw + c] = k;
        }
    }
}

hipError_t launch_init_tables(const uint4* root, const uint64_t* key_idx, uint32_t dim, uint32_t K, uint32_t npad,
                              uint32_t nw, uint4* seed, uint64_t* t, uint64_t* y, hipStream_t stream) {
    (void)K;
    const uint64_t total = (uint64_t)2 * npad;
    unsigned blocks = (unsigned)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_init_table, dim3(blocks), dim3(256), 0, stream, root, key_idx, dim, npad, nw, seed, t, y);
    return hipGetLastError();
}

// --------------------------------------------------------------------------------------
// add_key wire layout (AoS, client-major) -> SoA. One wave = 64 clients of one (level, key).
// --------------------------------------------------------------------------------------
// fhh_add_keys (collect.rs:62 add_key, host AoS -> device SoA): an item is 8 consecutive levels of
// one key for 64 clients, so a lane reads its client's 128 contiguous bytes of CorWord seeds (one
// cache line, 16-B aligned: the AoS stride is L x 16 B) and 8 bits bytes, and the wave writes 8
// coalesced 1 KiB rows (one level per item read a 16-B sliver of 64 lines and came back to the same
// lines for the next 7 levels); the item past the last level block holds the roots / key_idx
__global__ void k_keys_from_aos(const uint8_t* key_idx, const uint8_t* root_seed, const uint8_t* cw_seed,
                                const uint8_t* cw_bits, uint64_t n, uint32_t K, uint32_t L, uint32_t npad, uint32_t nw,
                                uint4* d_cw_seed, uint64_t* d_cw_bits, uint4* d_root, uint64_t* d_key_idx) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wpb = blockDim.x >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * wpb;
    const uint32_t nlb = (L + 7) / 8;
    const uint64_t items = (uint64_t)(nlb + 1) * K * nw;
    for (uint64_t item = (uint64_t)blockIdx.x * wpb + wave_id_uniform(); item < items; item += nwaves) {
        const uint32_t w = (uint32_t)(item % nw);
        const uint32_t kk = (uint32_t)((item / nw) % K);
        const uint32_t lb = (uint32_t)(item / ((uint64_t)nw * K));
        const uint64_t c = (uint64_t)w * 64 + lane;
        const bool valid = c < n;
        if (lb < nlb) {
            const uint32_t l0 = lb * 8, nl = min(8u, L - l0);
            const uint4* p = reinterpret_cast<const uint4*>(cw_seed) + (c * K + kk) * L + l0;
            const uint8_t* pb = cw_bits + (c * K + kk) * L + l0;
            uint4 v[8];
            uint32_t nib[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                v[k] = (valid && (uint32_t)k < nl) ? p[k] : make_uint4(0, 0, 0, 0);
                nib[k] = (valid && (uint32_t)k < nl) ? pb[k] : 0u;
            }
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if ((uint32_t)k >= nl) break;   // wave-uniform
                const size_t row = (size_t)(l0 + k) * K + kk;
                d_cw_seed[row * npad + c] = v[k];
                uint64_t q[4];
#pragma unroll
                for (int b = 0; b < 4; b++) q[b] = __ballot((nib[k] >> b) & 1);
                if (lane == 0)
#pragma unroll
                    for (int b = 0; b < 4; b++) d_cw_bits[(row * 4 + b) * nw + w] = q[b];
            }
        } else {
            uint4 v = make_uint4(0, 0, 0, 0);
            uint32_t ki = 0;
            if (valid) {
                const uint8_t* p = root_seed + (c * K + kk) * 16;
                uint32_t x[4];
                for (int k = 0; k < 4; k++)
                    x[k] = (uint32_t)p[4 * k] | ((uint32_t)p[4 * k + 1] << 8) | ((uint32_t)p[4 * k + 2] << 16) |
                           ((uint32_t)p[4 * k + 3] << 24);
                v = make_uint4(x[0], x[1], x[2], x[3]);
                ki = key_idx[c * K + kk] ? 1u : 0u;
            }
            d_root[(size_t)kk * npad + c] = v;
            const uint64_t q = __ballot(ki);
            if (lane == 0) d_key_idx[(size_t)kk * nw + w] = q;
        }
    }
}

// AddKeysRequest.keys (rpc.rs:12-15) in bincode 1.x legacy encoding (as `bincode::serialize`,
// leader.rs:101): u64 n, then per client u64 d and d x (ibDCFKey left, ibDCFKey right); an
// ibDCFKey (ibDCF.rs:16-21) = key_idx bool (1 B), root_seed (16 B), u64 L, L x CorWord
// (ibDCF.rs:9-14: seed 16 B, bits.0, bits.1, y_bits.0, y_bits.1 as 1-byte bools). Records
// are fixed-size, so every (level, key, 64-client word) item is decoded in place into the
// SoA device layout; malformed bools / lengths set bits of *err (bool > 1: 1, L: 2, d: 4).
__device__ __forceinline__ uint64_t load_u64_le(const uint8_t* p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v |= (uint64_t)p[i] << (8 * i);
    return v;
}

__device__ __forceinline__ uint4 load_seed(const uint8_t* p) {
    uint32_t x[4];
    for (int k = 0; k < 4; k++)
        x[k] = (uint32_t)p[4 * k] | ((uint32_t)p[4 * k + 1] << 8) | ((uint32_t)p[4 * k + 2] << 16) |
               ((uint32_t)p[4 * k + 3] << 24);
    return make_uint4(x[0], x[1], x[2], x[3]);
}

// (one lane per client: the CW levels [l_first, L) byte by byte, then level L = roots / key_idx;
// the CW levels go through k_bincode_cw_tiles below, so the launch starts at l_first = L)
__global__ void k_keys_from_bincode(const uint8_t* buf, uint64_t n, uint32_t d, uint32_t L, uint32_t npad,
                                    uint32_t nw, uint4* d_cw_seed, uint64_t* d_cw_bits, uint4* d_root,
                                    uint64_t* d_key_idx, uint32_t* err, uint32_t l_first) {
    const uint32_t K = 2 * d;
    const uint64_t KB = 25 + 20ull * L;      // one serialized ibDCFKey
    const uint64_t R = 8 + (uint64_t)K * KB;  // one client: u64 d + d (left, right) pairs
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wpb = blockDim.x >> 6;
    const uint64_t nwaves = (uint64_t)gridDim.x * wpb;
    const uint64_t items = (uint64_t)(L + 1) * K * nw;   // level L = roots / key_idx
    for (uint64_t item = (uint64_t)l_first * K * nw + (uint64_t)blockIdx.x * wpb + wave_id_uniform(); item < items;
         item += nwaves) {
        const uint32_t w = (uint32_t)(item % nw);
        const uint32_t kk = (uint32_t)((item / nw) % K);
        const uint32_t l = (uint32_t)(item / ((uint64_t)nw * K));
        const uint64_t c = (uint64_t)w * 64 + lane;
        const bool valid = c < n;
        const uint8_t* rec = buf + 8 + c * R;
        const uint8_t* key = rec + 8 + (uint64_t)kk * KB;
        uint32_t bad = 0;
        if (l < L) {
            uint4 v = make_uint4(0, 0, 0, 0);
            uint32_t nib = 0;
            if (valid) {
                const uint8_t* cw = key + 25 + 20ull * l;
                v = load_seed(cw);
                for (int b = 0; b < 4; b++) {
                    const uint32_t x = cw[16 + b];
                    bad |= x > 1 ? 1u : 0u;
                    nib |= (x & 1u) << b;
                }
            }
            const size_t row = (size_t)l * K + kk;
            d_cw_seed[row * npad + c] = v;
            uint64_t q[4];
            for (int b = 0; b < 4; b++) q[b] = __ballot((nib >> b) & 1);
            if (lane == 0)
                for (int b = 0; b < 4; b++) d_cw_bits[(row * 4 + b) * nw + w] = q[b];
        } else {
            uint4 v = make_uint4(0, 0, 0, 0);
            uint32_t ki = 0;
            if (valid) {
                ki = key[0];
                bad |= ki > 1 ? 1u : 0u;
                v = load_seed(key + 1);
                bad |= load_u64_le(key + 17) != L ? 2u : 0u;
                if (kk == 0) bad |= load_u64_le(rec) != d ? 4u : 0u;
            }
            d_root[(size_t)kk * npad + c] = v;
            const uint64_t q = __ballot(ki & 1u);
            if (lane == 0) d_key_idx[(size_t)kk * nw + w] = q;
        }
        if (bad) atomicOr(err, bad);
    }
}

// The correction words as tiles of 64 clients x kBcLevels levels of one key: a client's window of
// the payload (20 B per level, at an arbitrary byte offset) is staged into LDS by contiguous aligned
// dword loads (644 B per client, one wave per client at a time), then each lane (= client) extracts
// its levels with v_alignbit and the tile leaves as 1 KiB rows of [level][key][client] seeds plus
// the bit-plane ballots. The byte-per-load form (one lane per client and level, 20 global_load_ubyte
// 20 KiB apart) reached 0.58 TB/s on 2 GB; row f4, rpc.rs:12-15.
constexpr int kBcLevels = 32;
constexpr int kBcRow = 5 * kBcLevels + 1;   // dwords staged per client (odd: conflict-free rows)
__global__ __launch_bounds__(256) void k_bincode_cw_tiles(const uint8_t* buf, uint64_t n, uint32_t d, uint32_t L,
                                                          uint32_t npad, uint32_t nw, uint4* d_cw_seed,
                                                          uint64_t* d_cw_bits, uint32_t* err) {
    __shared__ uint32_t st[64 * kBcRow];
    const uint32_t K = 2 * d;
    const uint64_t KB = 25 + 20ull * L, R = 8 + (uint64_t)K * KB;
    const uint32_t nlb = (L + kBcLevels - 1) / kBcLevels;
    const uint64_t tiles = (uint64_t)nw * K * nlb;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint64_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        const uint32_t w = (uint32_t)(tile % nw);
        const uint32_t kk = (uint32_t)((tile / nw) % K);
        const uint32_t l0 = (uint32_t)(tile / ((uint64_t)nw * K)) * kBcLevels;
        const uint32_t nl = min((uint32_t)kBcLevels, L - l0);
        // stage: wave wv takes clients wv + 4 i (i < 16); all 48 loads of a lane are issued before
        // the first LDS write (a load -> write pair per client serialised 16 HBM latencies per tile)
        uint32_t v[16][3];
#pragma unroll
        for (int i = 0; i < 16; i++) {
            const uint64_t c = (uint64_t)w * 64 + wv + 4 * i;
            const uint64_t s0 = 8 + c * R + 8 + kk * KB + 25 + 20ull * l0;   // level l0's CorWord
            const uint64_t a0 = s0 & ~3ull;
            const uint32_t ndw = c < n ? (uint32_t)((s0 + 20ull * nl + 3 - a0) / 4) : 0u;   // <= kBcRow
            const uint32_t* src = reinterpret_cast<const uint32_t*>(buf + a0);
#pragma unroll
            for (int r = 0; r < 3; r++) {
                const uint32_t j = lane + 64 * r;
                v[i][r] = j < ndw ? src[j] : 0u;
            }
        }
#pragma unroll
        for (int i = 0; i < 16; i++)
#pragma unroll
            for (int r = 0; r < 3; r++) {
                const uint32_t j = lane + 64 * r;
                if (j < (uint32_t)kBcRow) st[(wv + 4 * i) * kBcRow + j] = v[i][r];
            }
        __syncthreads();
        const uint64_t c = (uint64_t)w * 64 + lane;
        const bool valid = c < n;
        const uint32_t sh = (uint32_t)((8 + c * R + 8 + kk * KB + 25 + 20ull * l0) & 3) * 8;
        uint32_t bad = 0;
        for (uint32_t li = wv; li < nl; li += 4) {
            uint4 v = make_uint4(0, 0, 0, 0);
            uint32_t nib = 0;
            if (valid) {
                const uint32_t* row = st + lane * kBcRow + 5 * li;   // 5 li + 5 < kBcRow
                uint32_t u[5];
#pragma unroll
                for (int k = 0; k < 5; k++) u[k] = __builtin_amdgcn_alignbit(row[k + 1], row[k], sh);
                v = make_uint4(u[0], u[1], u[2], u[3]);
#pragma unroll
                for (int b = 0; b < 4; b++) {   // bits.0, bits.1, y_bits.0, y_bits.1 as bincode bools
                    const uint32_t x = (u[4] >> (8 * b)) & 0xFFu;
                    bad |= x > 1 ? 1u : 0u;
                    nib |= (x & 1u) << b;
                }
            }
            const size_t rowi = (size_t)(l0 + li) * K + kk;
            d_cw_seed[rowi * npad + c] = v;
            uint64_t q[4];
#pragma unroll
            for (int b = 0; b < 4; b++) q[b] = __ballot((nib >> b) & 1);
            if (lane == 0)
#pragma unroll
                for (int b = 0; b < 4; b++) d_cw_bits[(rowi * 4 + b) * nw + w] = q[b];
        }
        if (bad) atomicOr(err, bad);
        __syncthreads();
    }
}

hipError_t launch_keys_from_bincode(const uint8_t* buf, uint64_t n, uint32_t d, uint32_t L, uint32_t npad, uint32_t nw,
                                    uint4* d_cw_seed, uint64_t* d_cw_bits, uint4* d_root, uint64_t* d_key_idx,
                                    uint32_t* err, hipStream_t stream) {
    int dev = 0, cus = 256;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    const uint64_t tiles = (uint64_t)nw * 2 * d * ((L + kBcLevels - 1) / kBcLevels);
    if (tiles) {
        const uint64_t cap = (uint64_t)cus * 8;
        hipLaunchKernelGGL(k_bincode_cw_tiles, dim3((unsigned)(tiles < cap ? tiles : cap)), dim3(256), 0, stream, buf,
                           n, d, L, npad, nw, d_cw_seed, d_cw_bits, err);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    const uint64_t items = (uint64_t)2 * d * nw;   // level L: roots / key_idx / headers
    uint64_t blocks = (items + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_keys_from_bincode, dim3((unsigned)blocks), dim3(256), 0, stream, buf, n, d, L, npad, nw,
                       d_cw_seed, d_cw_bits, d_root, d_key_idx, err, L);
    return hipGetLastError();
}

hipError_t launch_keys_from_aos(const uint8_t* key_idx, const uint8_t* root_seed, const uint8_t* cw_seed,
                                const uint8_t* cw_bits, uint64_t n, uint32_t K, uint32_t L, uint32_t npad, uint32_t nw,
                                uint4* d_cw_seed, uint64_t* d_cw_bits, uint4* d_root, uint64_t* d_key_idx,
                                hipStream_t stream) {
    const uint64_t items = (uint64_t)((L + 7) / 8 + 1) * K * nw;
    uint64_t blocks = (items + 3) / 4;
    if (blocks > 8192) blocks = 8192;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_keys_from_aos, dim3((unsigned)blocks), dim3(256), 0, stream, key_idx, root_seed, cw_seed,
                       cw_bits, n, K, L, npad, nw, d_cw_seed, d_cw_bits, d_root, d_key_idx);
    return hipGetLastError();
}

}  // namespace fhh
