// Bitsliced k_expand for gfx950: ibDCFKey::eval_bit (ibDCF.rs:208-227) with the PRG
// expand_dir (prg.rs:92-122) as a bitsliced AES-128 on the VALU (v_bitop3_b32), no LDS.
//
// Layout ("bs"): every 16-byte seed array (correction-word seeds, root seeds, prefix-table
// seeds) is stored per key row as [32 quads][ng] uint4, ng = npad / 32 client groups: quad q of
// group g holds the bitsliced words 4q..4q+3 of clients 32g..32g+31 — word i bit j = bit i of
// client (32g + j)'s seed (bit i = bit (i & 7) of byte (i >> 3)). A row has the same size as
// the client-major [npad] uint4 row, so every row-level copy (init, growth) is layout-blind.
// t / y / control-bit planes keep their u64 [..][nw] layout; as u32 words they are indexed by
// the client group directly (little-endian halves).
//
// One lane = 32 clients of one (prefix entry, side, direction); one work item = one
// (entry, side, dir) for 64 lanes = 2048 clients. Per item: load the parent seeds (32 dwordx4
// per lane, 1 KiB per wave instruction), mask the low nibble of byte 0 (prg.rs:96), +1 on the
// upper u64 lane for dir 1 (prg.rs:273-276, a bitsliced ripple carry), AES-128 with the zero
// key (aes_bs_gen.h, generated), feed-forward + correction word (reloaded from L2), store.
#include "fhh_internal.h"
#include "aes_bs_gen.h"
#include "bitslice.h"

namespace fhh {

#ifndef FHH_BS_FENCE_EVERY
#define FHH_BS_FENCE_EVERY 2
#endif

struct BsDevOps {
    // bound the scheduler's reordering to FHH_BS_FENCE_EVERY S-box / MixColumns units
    template <int unit>
    static __device__ __forceinline__ void fence() {
        if constexpr (FHH_BS_FENCE_EVERY > 0 && unit % FHH_BS_FENCE_EVERY == FHH_BS_FENCE_EVERY - 1)
            __builtin_amdgcn_sched_barrier(0);
    }
    template <int imm>
    static __device__ __forceinline__ uint32_t b3(uint32_t a, uint32_t b, uint32_t c) {
        return __builtin_amdgcn_bitop3_b32(a, b, c, imm);
    }
};

// to_bs = 1: client-major [rows][npad] uint4 -> bs [rows][32][ng]; 0: the inverse.
__global__ __launch_bounds__(256) void k_bitslice(const uint4* __restrict__ in, uint4* __restrict__ out,
                                                  uint64_t rows, uint32_t npad, int to_bs) {
    const uint32_t ng = npad / 32;
    const uint64_t total = rows * ng;
    for (uint64_t id = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; id < total;
         id += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t row = id / ng;
        const uint32_t g = (uint32_t)(id % ng);
        uint32_t w[4][32];
        if (to_bs) {
#pragma unroll
            for (int j = 0; j < 32; j++) {
                const uint4 v = in[row * npad + 32 * g + j];
                w[0][j] = v.x; w[1][j] = v.y; w[2][j] = v.z; w[3][j] = v.w;
            }
#pragma unroll
            for (int k = 0; k < 4; k++) transpose32(w[k]);
#pragma unroll
            for (int q = 0; q < 32; q++) {
                const int k = q >> 3, b = (q & 7) * 4;
                out[(row * 32 + q) * ng + g] = make_uint4(w[k][b], w[k][b + 1], w[k][b + 2], w[k][b + 3]);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 32; q++) {
                const uint4 v = in[(row * 32 + q) * ng + g];
                const int k = q >> 3, b = (q & 7) * 4;
                w[k][b] = v.x; w[k][b + 1] = v.y; w[k][b + 2] = v.z; w[k][b + 3] = v.w;
            }
#pragma unroll
            for (int k = 0; k < 4; k++) transpose32(w[k]);
#pragma unroll
            for (int j = 0; j < 32; j++) out[row * npad + 32 * g + j] = make_uint4(w[0][j], w[1][j], w[2][j], w[3][j]);
        }
    }
}

hipError_t launch_bitslice(const uint4* in, uint4* out, uint64_t rows, uint32_t npad, int to_bs, hipStream_t stream) {
    const uint64_t total = rows * (npad / 32);
    if (total == 0) return hipSuccess;
    const uint64_t blocks = (total + 255) / 256;
    hipLaunchKernelGGL(k_bitslice, dim3((unsigned)(blocks < 65536 ? blocks : 65536)), dim3(256), 0, stream, in, out,
                       rows, npad, to_bs);
    return hipGetLastError();
}

typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

// buffer resource over one key row ([32][ng] uint4): wave-uniform base in SGPRs, so the 32
// quads of a row are addressed with one lane offset + a scalar offset per quad (no per-quad
// 64-bit VGPR addresses, which would not fit beside the 128-word state)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void* base, uint32_t ng) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)(32u * ng * 16u), 0x00020000);
}

__device__ __forceinline__ void bs_item(const ExpandJob& J, uint64_t local, uint32_t lane) {
    const uint32_t ng = 2 * J.nw;
    const uint32_t nch = (ng + 63) / 64;
    const uint32_t ch = (uint32_t)(local % nch);
    const uint64_t rest = local / nch;
    const int dir = (int)(rest & 1);
    const int s = (int)((rest >> 1) & 1);
    const uint32_t e = (uint32_t)(rest >> 2);
    const uint32_t g = ch * 64 + lane;
    const bool act = g < ng;
    const uint32_t gg = act ? g : 0;   // clamp: inactive lanes read group 0, never store

    const uint32_t src = J.live[e];
    const size_t row = (size_t)src * 2 + s;
    const size_t krow = (size_t)J.level * J.K + 2 * J.dim + s;
    const uint32_t* t32 = reinterpret_cast<const uint32_t*>(J.src_t);
    const uint32_t* y32 = reinterpret_cast<const uint32_t*>(J.src_y);
    const uint32_t* cwb32 = reinterpret_cast<const uint32_t*>(J.cw_bits);
    const uint32_t tw = t32[row * ng + gg];
    const uint32_t yw = y32[row * ng + gg];
    const uint32_t cb = cwb32[(krow * 4 + dir) * ng + gg];       // CorWord.bits[dir]
    const uint32_t cy = cwb32[(krow * 4 + 2 + dir) * ng + gg];   // CorWord.y_bits[dir]
    const __amdgpu_buffer_rsrc_t xs = row_rsrc(J.src_seed + row * 32 * ng, ng);
    const __amdgpu_buffer_rsrc_t cws = row_rsrc(J.cw_seed + krow * 32 * ng, ng);
    const int voff = (int)(gg * 16u);
    const int qstride = (int)(ng * 16u);

    uint32_t st[128];
#pragma unroll
    for (int q = 0; q < 32; q++) {
        const v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(xs, voff, q * qstride, 0);
        st[4 * q] = v.x; st[4 * q + 1] = v.y; st[4 * q + 2] = v.z; st[4 * q + 3] = v.w;
    }
    // key_short[0] &= 0xF0 (prg.rs:96); then the control bits read from the masked byte
    // (prg.rs:101-104): bits[dir] = (k[0] & (1 << dir)) == 0, y_bits[dir] = (k[0] & (4 << dir)) == 0
#pragma unroll
    for (int i = 0; i < 4; i++) st[i] = 0;
    const uint32_t pb = ~(dir ? st[1] : st[0]);   // static indices: st stays in registers
    const uint32_t py = ~(dir ? st[3] : st[2]);
    if (dir) {   // ctr + 1 in the upper u64 lane, little-endian, no carry into bytes 0..7
        uint32_t carry = ~0u;
#pragma unroll
        for (int i = 64; i < 128; i++) {
            const uint32_t v = st[i];
            st[i] = v ^ carry;
            carry &= v;
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    aes0_bs<BsDevOps>(st);
    __builtin_amdgcn_sched_barrier(0);

    // MMO feed-forward (prg.rs:227-230) with the counter reloaded, then
    // seed ^= t ? cw.seed : 0 (ibDCF.rs:215-217)
    const size_t de = ((size_t)(2 * e + dir)) * 2 + s;
    const __amdgpu_buffer_rsrc_t out = row_rsrc(J.dst_seed + de * 32 * ng, ng);
    uint32_t carry = dir ? ~0u : 0u;
#pragma unroll
    for (int q = 0; q < 32; q++) {
        const v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(xs, voff, q * qstride, 0);
        const v4u32 c = __builtin_amdgcn_raw_buffer_load_b128(cws, voff, q * qstride, 0);
        uint32_t x[4] = {v.x, v.y, v.z, v.w};
        const uint32_t cw[4] = {c.x, c.y, c.z, c.w};
        if (q == 0)
#pragma unroll
            for (int i = 0; i < 4; i++) x[i] = 0;
        if (q >= 16)
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint32_t xv = x[i];
                x[i] = xv ^ carry;
                carry &= xv;
            }
        v4u32 o;
        o.x = __builtin_amdgcn_bitop3_b32(st[4 * q + 0], x[0], tw & cw[0], 0x96);
        o.y = __builtin_amdgcn_bitop3_b32(st[4 * q + 1], x[1], tw & cw[1], 0x96);
        o.z = __builtin_amdgcn_bitop3_b32(st[4 * q + 2], x[2], tw & cw[2], 0x96);
        o.w = __builtin_amdgcn_bitop3_b32(st[4 * q + 3], x[3], tw & cw[3], 0x96);
        if (act) __builtin_amdgcn_raw_buffer_store_b128(o, out, voff, q * qstride, 0);
    }
    if (act) {
        // new_bit = tau.bits[dir] ^ (t & cw.bits[dir]); new_y = tau.y_bits[dir] ^ (t & cw.y_bits[dir]) ^ y
        reinterpret_cast<uint32_t*>(J.dst_t)[de * ng + g] = pb ^ (tw & cb);
        reinterpret_cast<uint32_t*>(J.dst_y)[de * ng + g] = py ^ (tw & cy) ^ yw;
    }
}

template <int THR>
__global__ __launch_bounds__(THR, 2) void k_expand_bs(ExpandLaunch a, uint32_t* work_counter) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t nwaves = (uint64_t)gridDim.x * (THR / 64);
    const LoopCtl* ctl = a.ctl;
    const uint64_t total = ctl ? (ctl->abort ? 0 : ctl->total_items) : a.total_items;
    uint32_t v = 0;
    if (lane == 0) v = atomicAdd(work_counter, 1u);
    uint64_t item = __builtin_amdgcn_readfirstlane(v);
    while (item < total) {
        uint32_t ji = 0;
        if (ctl) {
            while (ji + 1 < a.njobs && item >= ctl->item_begin[ji + 1]) ji++;
        } else {
            while (ji + 1 < a.njobs && item >= a.job[ji + 1].item_begin) ji++;
        }
        ExpandJob J = a.job[ji];
        if (ctl) {
            J.n_live = ctl->n_live[ji % a.jobs_per_ctx];
            J.item_begin = ctl->item_begin[ji];
        }
        bs_item(J, item - J.item_begin, lane);
        v = 0;
        if (lane == 0) v = atomicAdd(work_counter, 1u);
        item = __builtin_amdgcn_readfirstlane(v);
    }
    // every wave drew exactly one item past the end; the last wave re-arms the counter
    if (lane == 0) {
        const uint32_t done = atomicAdd(work_counter + 1, 1u);
        if (done + 1 == (uint32_t)nwaves) {
            atomicExch(work_counter, 0u);
            atomicExch(work_counter + 1, 0u);
        }
    }
}

constexpr int kBsThreads = 256;

hipError_t launch_expand_bs(const ExpandLaunch& a, int grid, uint32_t* work_counter, hipStream_t stream) {
    if (a.total_items == 0) return hipSuccess;
    const uint64_t wpb = kBsThreads / 64;
    const uint64_t blocks_needed = (a.total_items + wpb - 1) / wpb;
    const int g = a.ctl ? grid : (int)(blocks_needed < (uint64_t)grid ? blocks_needed : (uint64_t)grid);
    hipLaunchKernelGGL(k_expand_bs<kBsThreads>, dim3(g), dim3(kBsThreads), 0, stream, a, work_counter);
    return hipGetLastError();
}

const void* expand_bs_fn() { return reinterpret_cast<const void*>(&k_expand_bs<kBsThreads>); }
int expand_bs_threads() { return kBsThreads; }

}  // namespace fhh
