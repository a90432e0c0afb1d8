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
#ifdef FHH_AB_VARIANTS   // A/B builds only (fhh_kernels.hip's variant table); the default build has stubs below
#include "aes_bs_gen.h"
#include "aes_tables.h"
#include "bitslice.h"

namespace fhh {

// FENCE: a scheduling barrier after every FENCE S-box / MixColumns units bounds how far the
// compiler may interleave units (and so the registers it needs); 0 = none.
template <int FENCE>
struct BsDevOps {
    template <int unit>
    static __device__ __forceinline__ void fence() {
        if constexpr (FENCE > 0 && unit % FENCE == FENCE - 1) __builtin_amdgcn_sched_barrier(0);
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

// Work-item coordinates are wave-uniform by construction; say so, so the compiler keeps them
// (and the buffer resources built from them) in SGPRs — a VGPR resource turns every buffer
// access into a readfirstlane waterfall loop.
__device__ __forceinline__ uint64_t uniform_u64(uint64_t x) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint32_t uniform_u32(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

__constant__ RoundKeys c_zero_rk = ZERO_RK;

// AES_0 on 32 bitsliced blocks. ROLLED: rounds 1..9 as one loop body (~12 KiB of code instead of
// ~120 KiB) with AddRoundKey applied at run time (one v_xor with an s_bfe_i32 mask per bit).
template <int FENCE, bool ROLLED>
__device__ __forceinline__ void aes_bs(uint32_t (&st)[128]) {
    if constexpr (ROLLED) {
#pragma unroll 1
        for (int r = 1; r < 10; r++) {
            aes0_bs_round<BsDevOps<FENCE>>(st);
            uint32_t rk[4];
#pragma unroll
            for (int c = 0; c < 4; c++) rk[c] = __builtin_amdgcn_readfirstlane(c_zero_rk.w[r][c]);
#pragma unroll
            for (int i = 0; i < 128; i++) st[i] ^= (uint32_t)(-(int32_t)((rk[i >> 5] >> (i & 31)) & 1u));
        }
        aes0_bs_last<BsDevOps<FENCE>>(st);
    } else {
        aes0_bs<BsDevOps<FENCE>>(st);
    }
}

// buffer resource over one key row ([32][ng] uint4): wave-uniform base in SGPRs, so the 32
// quads of a row are addressed with one lane offset + a scalar offset per quad (no per-quad
// 64-bit VGPR addresses, which would not fit beside the 128-word state)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void* base, uint32_t ng) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)(32u * ng * 16u), 0x00020000);
}

template <int FENCE, bool ROLLED>
__device__ __forceinline__ void bs_item(const ExpandJob& J, uint64_t local, uint32_t lane) {
    local = uniform_u64(local);
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

    const uint32_t src = uniform_u32(J.live[e]);
    const size_t row = (size_t)src * 2 + s;
    const size_t krow = (size_t)J.level * J.K + 2 * J.dim + s;
    const __amdgpu_buffer_rsrc_t xs = row_rsrc(J.src_seed + row * 32 * ng, ng);
    const __amdgpu_buffer_rsrc_t cws = row_rsrc(J.cw_seed + krow * 32 * ng, ng);
    // inactive lanes: an offset past num_records -> buffer loads return 0, stores are dropped
    // (no exec-mask branches around the 32 quad stores)
    const int voff = act ? (int)(g * 16u) : (int)0x80000000u;
    const int qstride = (int)(ng * 16u);

    uint32_t st[128];
#pragma unroll
    for (int q = 0; q < 32; q++) {
        const v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(xs, voff, q * qstride, 0);
        st[4 * q] = v.x; st[4 * q + 1] = v.y; st[4 * q + 2] = v.z; st[4 * q + 3] = v.w;
    }
    // key_short[0] &= 0xF0 (prg.rs:96): bits 0..3 of byte 0 = bitsliced words 0..3
#pragma unroll
    for (int i = 0; i < 4; i++) st[i] = 0;
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
    aes_bs<FENCE, ROLLED>(st);
    __builtin_amdgcn_sched_barrier(0);

    // loaded only now: nothing but the 128 state words is live across the AES
    const uint32_t* t32 = reinterpret_cast<const uint32_t*>(J.src_t);
    const uint32_t* y32 = reinterpret_cast<const uint32_t*>(J.src_y);
    const uint32_t* cwb32 = reinterpret_cast<const uint32_t*>(J.cw_bits);
    const uint32_t tw = t32[row * ng + gg];
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
        __builtin_amdgcn_raw_buffer_store_b128(o, out, voff, q * qstride, 0);
        // bound the reload look-ahead: the state still occupies 4 * (32 - q) registers, so the
        // batches grow as it drains (1, 1, 2, 4, 8, 8, 8 quads)
        if (q == 0 || q == 1 || q == 3 || q == 7 || q == 15 || q == 23) __builtin_amdgcn_sched_barrier(0);
    }
    if (act) {
        // control bits of expand_dir read from the MASKED byte 0 (prg.rs:101-104):
        // bits[dir] = (k[0] & (1 << dir)) == 0, y_bits[dir] = (k[0] & (4 << dir)) == 0
        const uint32_t masked_lo[4] = {0u, 0u, 0u, 0u};   // words 0..3 after key_short[0] &= 0xF0
        const uint32_t pb = ~masked_lo[dir];
        const uint32_t py = ~masked_lo[2 + dir];
        const uint32_t yw = y32[row * ng + gg];
        const uint32_t cb = cwb32[(krow * 4 + dir) * ng + gg];       // CorWord.bits[dir]
        const uint32_t cy = cwb32[(krow * 4 + 2 + dir) * ng + gg];   // CorWord.y_bits[dir]
        // new_bit = tau.bits[dir] ^ (t & cw.bits[dir]); new_y = tau.y_bits[dir] ^ (t & cw.y_bits[dir]) ^ y
        reinterpret_cast<uint32_t*>(J.dst_t)[de * ng + g] = pb ^ (tw & cb);
        reinterpret_cast<uint32_t*>(J.dst_y)[de * ng + g] = py ^ (tw & cy) ^ yw;
    }
}

// ---- pair mode: one 2-wave workgroup per (entry, side, 2048-client chunk) -------------------
// Wave 0 computes dir 0, wave 1 dir 1. The parent seeds are fetched from HBM once per pair
// (each wave loads half) into LDS (32 KiB per workgroup) and serve both waves' counter load and
// their MMO feed-forward: no global re-fetch of the seeds (the single-wave kernel fetches them
// up to 4 times, ~46 B/block of HBM reads, r01 PMC).
typedef v4u32 SeedQuads[32][64];

// phase-time profile (PROF variants only): cycles summed over waves, read by fhh_debug_bs_profile
__device__ unsigned long long g_bs_prof[8];

template <bool PROF>
__device__ __forceinline__ void prof_mark(uint64_t& last, uint64_t (&acc)[8], int phase) {
    if constexpr (PROF) {
        const uint64_t now = __builtin_amdgcn_s_memtime();
        acc[phase] += now - last;
        last = now;
    }
}

template <int FENCE, bool ROLLED, bool PROF = false>
__device__ __forceinline__ void bs_pair_item(const ExpandJob& J, uint64_t local, uint32_t lane, int dir,
                                             SeedQuads& xl, uint64_t& tl, uint64_t (&acc)[8]) {
    local = uniform_u64(local);
    const uint32_t ng = 2 * J.nw;
    const uint32_t nch = (ng + 63) / 64;
    const uint32_t ch = (uint32_t)(local % nch);
    const uint64_t rest = local / nch;
    const int s = (int)(rest & 1);
    const uint32_t e = (uint32_t)(rest >> 1);
    const uint32_t g = ch * 64 + lane;
    const bool act = g < ng;
    const uint32_t gg = act ? g : 0;

    const uint32_t src = uniform_u32(J.live[e]);
    const size_t row = (size_t)src * 2 + s;
    const size_t krow = (size_t)J.level * J.K + 2 * J.dim + s;
    const __amdgpu_buffer_rsrc_t xs = row_rsrc(J.src_seed + row * 32 * ng, ng);
    const __amdgpu_buffer_rsrc_t cws = row_rsrc(J.cw_seed + krow * 32 * ng, ng);
    const int voff = act ? (int)(g * 16u) : (int)0x80000000u;   // OOB: loads 0, stores dropped
    const int qstride = (int)(ng * 16u);

    // cooperative fetch: wave d brings quads [16d, 16d + 16) into LDS
#pragma unroll
    for (int qq = 0; qq < 16; qq++) {
        const int q = 16 * dir + qq;
        xl[q][lane] = __builtin_amdgcn_raw_buffer_load_b128(xs, voff, q * qstride, 0);
    }
    __syncthreads();
    prof_mark<PROF>(tl, acc, 1);   // 1: seed fetch + barrier

    uint32_t st[128];
#pragma unroll
    for (int q = 0; q < 32; q++) {
        const v4u32 v = xl[q][lane];
        st[4 * q] = v.x; st[4 * q + 1] = v.y; st[4 * q + 2] = v.z; st[4 * q + 3] = v.w;
    }
    // key_short[0] &= 0xF0 (prg.rs:96): bits 0..3 of byte 0 = bitsliced words 0..3
#pragma unroll
    for (int i = 0; i < 4; i++) st[i] = 0;
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
    __builtin_amdgcn_s_waitcnt(0);
    prof_mark<PROF>(tl, acc, 2);   // 2: LDS -> registers, mask, increment
    aes_bs<FENCE, ROLLED>(st);
    __builtin_amdgcn_sched_barrier(0);
    prof_mark<PROF>(tl, acc, 3);   // 3: AES

    const uint32_t* t32 = reinterpret_cast<const uint32_t*>(J.src_t);
    const uint32_t* y32 = reinterpret_cast<const uint32_t*>(J.src_y);
    const uint32_t* cwb32 = reinterpret_cast<const uint32_t*>(J.cw_bits);
    const uint32_t tw = t32[row * ng + gg];
    // MMO feed-forward (prg.rs:227-230) with the counter from LDS, then
    // seed ^= t ? cw.seed : 0 (ibDCF.rs:215-217)
    const size_t de = ((size_t)(2 * e + dir)) * 2 + s;
    const __amdgpu_buffer_rsrc_t out = row_rsrc(J.dst_seed + de * 32 * ng, ng);
    uint32_t carry = dir ? ~0u : 0u;
#pragma unroll
    for (int q = 0; q < 32; q++) {
        const v4u32 v = xl[q][lane];
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
        __builtin_amdgcn_raw_buffer_store_b128(o, out, voff, q * qstride, 0);
        if (q == 0 || q == 1 || q == 3 || q == 7 || q == 15 || q == 23) __builtin_amdgcn_sched_barrier(0);
    }
    if (act) {
        // control bits of expand_dir read from the MASKED byte 0 (prg.rs:101-104)
        const uint32_t masked_lo[4] = {0u, 0u, 0u, 0u};
        const uint32_t pb = ~masked_lo[dir];
        const uint32_t py = ~masked_lo[2 + dir];
        const uint32_t yw = y32[row * ng + gg];
        const uint32_t cb = cwb32[(krow * 4 + dir) * ng + gg];
        const uint32_t cy = cwb32[(krow * 4 + 2 + dir) * ng + gg];
        reinterpret_cast<uint32_t*>(J.dst_t)[de * ng + g] = pb ^ (tw & cb);
        reinterpret_cast<uint32_t*>(J.dst_y)[de * ng + g] = py ^ (tw & cy) ^ yw;
    }
    prof_mark<PROF>(tl, acc, 4);   // 4: MMO + stores
}

template <int WAVES, int FENCE, bool ROLLED, bool PROF = false>
__global__ __launch_bounds__(128, WAVES) void k_expand_bs_pair(ExpandLaunch a, uint32_t* work_counter) {
    __shared__ SeedQuads xl;
    __shared__ uint32_t item_slot;
    const uint32_t lane = threadIdx.x & 63;
    const int dir = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const LoopCtl* ctl = a.ctl;
    const uint64_t total = ctl ? (ctl->abort ? 0 : ctl->total_items) : a.total_items;
    uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tl = PROF ? __builtin_amdgcn_s_memtime() : 0;
    for (;;) {
        if (threadIdx.x == 0) item_slot = atomicAdd(work_counter, 1u);
        __syncthreads();
        prof_mark<PROF>(tl, acc, 0);   // 0: item fetch
        const uint64_t item = __builtin_amdgcn_readfirstlane(item_slot);
        if (item >= total) break;
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
        bs_pair_item<FENCE, ROLLED, PROF>(J, item - J.item_begin, lane, dir, xl, tl, acc);
        __syncthreads();   // both waves are done with xl / item_slot
        prof_mark<PROF>(tl, acc, 5);   // 5: end barrier
    }
    if constexpr (PROF) {
        if (lane == 0)
            for (int k = 0; k < 6; k++) atomicAdd(&g_bs_prof[k], (unsigned long long)acc[k]);
    }
    // every workgroup drew exactly one item past the end; the last one re-arms the counter
    if (threadIdx.x == 0) {
        const uint32_t done = atomicAdd(work_counter + 1, 1u);
        if (done + 1 == gridDim.x) {
            atomicExch(work_counter, 0u);
            atomicExch(work_counter + 1, 0u);
        }
    }
}

// ---- pair mode v2: no global loads after the AES ---------------------------------------------
// Item start: both waves load the 32 seed quads into registers (HBM once, the partner's copy
// hits L2/L1) and wave d loads correction-word quads [16d, 16d+16); wave d writes
// y = mask(x) ^ (t & cw) for its half to LDS. After the AES the feed-forward + correction word
// is out = AES(ctr) ^ y (^ the dir-1 increment's flipped bits, kept in registers for the first
// kCarryWords (24) bits of the upper lane; a longer carry — P ~ 2^-24 per block, ~1e-4 per item
// — takes a slow path that reloads the seed quads). The next item's index is fetched one item ahead.
template <int FENCE, bool ROLLED, bool PROF, int kCarryWords>
__device__ __forceinline__ void bs_pair2_item(const ExpandJob& J, uint64_t local, uint32_t lane, int dir,
                                              SeedQuads& yl, uint64_t& tl, uint64_t (&acc)[8]) {
    local = uniform_u64(local);
    const uint32_t ng = 2 * J.nw;
    const uint32_t nch = (ng + 63) / 64;
    const uint32_t ch = (uint32_t)(local % nch);
    const uint64_t rest = local / nch;
    const int s = (int)(rest & 1);
    const uint32_t e = (uint32_t)(rest >> 1);
    const uint32_t g = ch * 64 + lane;
    const bool act = g < ng;
    const uint32_t gg = act ? g : 0;

    const uint32_t src = uniform_u32(J.live[e]);
    const size_t row = (size_t)src * 2 + s;
    const size_t krow = (size_t)J.level * J.K + 2 * J.dim + s;
    const __amdgpu_buffer_rsrc_t xs = row_rsrc(J.src_seed + row * 32 * ng, ng);
    const __amdgpu_buffer_rsrc_t cws = row_rsrc(J.cw_seed + krow * 32 * ng, ng);
    const int voff = act ? (int)(g * 16u) : (int)0x80000000u;   // OOB: loads 0, stores dropped
    const int qstride = (int)(ng * 16u);
    const uint32_t* t32 = reinterpret_cast<const uint32_t*>(J.src_t);
    const uint32_t tw = t32[row * ng + gg];

    uint32_t st[128];
#pragma unroll
    for (int q = 0; q < 32; q++) {
        const v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(xs, voff, q * qstride, 0);
        st[4 * q] = v.x; st[4 * q + 1] = v.y; st[4 * q + 2] = v.z; st[4 * q + 3] = v.w;
    }
    // key_short[0] &= 0xF0 (prg.rs:96): bits 0..3 of byte 0 = bitsliced words 0..3
#pragma unroll
    for (int i = 0; i < 4; i++) st[i] = 0;
    // y = ctr0 ^ (t & cw.seed) for this wave's half (prg.rs:227-230 feed-forward of the dir-0
    // counter, ibDCF.rs:215-217 correction word)
#pragma unroll
    for (int qq = 0; qq < 16; qq++) {
        const int q = 16 * dir + qq;   // wave-uniform
        const v4u32 c = __builtin_amdgcn_raw_buffer_load_b128(cws, voff, q * qstride, 0);
        uint32_t xq[4];
#pragma unroll
        for (int i = 0; i < 4; i++) xq[i] = dir ? st[64 + 4 * qq + i] : st[4 * qq + i];
        v4u32 y;
        y.x = xq[0] ^ (tw & c.x);
        y.y = xq[1] ^ (tw & c.y);
        y.z = xq[2] ^ (tw & c.z);
        y.w = xq[3] ^ (tw & c.w);
        yl[q][lane] = y;
    }
    // dir 1: ctr + 1 in the upper u64 lane (prg.rs:273-276); d[k] = bits flipped at 64 + k
    uint32_t d[kCarryWords];
    bool tail = false;    // carry alive past bit 64 + kCarryWords in some lane (wave-uniform)
    uint32_t c_tail = 0;  // carry entering bit 64 + kCarryWords
    if (dir) {
        uint32_t carry = ~0u;
#pragma unroll
        for (int k = 0; k < kCarryWords; k++) {
            const uint32_t v = st[64 + k];
            d[k] = carry;
            st[64 + k] = v ^ carry;
            carry &= v;
        }
        c_tail = carry;
        tail = __ballot(carry != 0) != 0;
        if (tail) {
#pragma unroll
            for (int i = 64 + kCarryWords; i < 128; i++) {
                const uint32_t v = st[i];
                st[i] = v ^ carry;
                carry &= v;
            }
        }
    }
    __builtin_amdgcn_sched_barrier(0);
    prof_mark<PROF>(tl, acc, 1);   // 1: seed / cw fetch, y, increment
    aes_bs<FENCE, ROLLED>(st);
    __builtin_amdgcn_sched_barrier(0);
    prof_mark<PROF>(tl, acc, 3);   // 3: AES
    __syncthreads();               // the partner's half of y is in LDS
    prof_mark<PROF>(tl, acc, 2);   // 2: mid barrier

    // out = AES(ctr) ^ ctr ^ (t & cw) = AES(ctr) ^ y (^ flipped bits for dir 1)
    const size_t de = ((size_t)(2 * e + dir)) * 2 + s;
    const __amdgpu_buffer_rsrc_t out = row_rsrc(J.dst_seed + de * 32 * ng, ng);
    uint32_t cur = c_tail;
#pragma unroll
    for (int q = 0; q < 32; q++) {
        const v4u32 y = yl[q][lane];
        uint32_t o[4] = {y.x, y.y, y.z, y.w};
        if (q >= 16 && (q - 16) * 4 < kCarryWords) {
            if (dir)
#pragma unroll
                for (int i = 0; i < 4; i++) o[i] ^= d[(q - 16) * 4 + i];
        } else if (q >= 16 && tail) {
            // slow path: continue the carry chain over the parent seed's upper-lane bits
            const v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(xs, voff, q * qstride, 0);
            const uint32_t xv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int i = 0; i < 4; i++) {
                o[i] ^= cur;
                cur &= xv[i];
            }
        }
        v4u32 ov;
        ov.x = st[4 * q + 0] ^ o[0];
        ov.y = st[4 * q + 1] ^ o[1];
        ov.z = st[4 * q + 2] ^ o[2];
        ov.w = st[4 * q + 3] ^ o[3];
        __builtin_amdgcn_raw_buffer_store_b128(ov, out, voff, q * qstride, 0);
    }
    if (act) {
        const uint32_t* y32 = reinterpret_cast<const uint32_t*>(J.src_y);
        const uint32_t* cwb32 = reinterpret_cast<const uint32_t*>(J.cw_bits);
        // control bits of expand_dir read from the MASKED byte 0 (prg.rs:101-104)
        const uint32_t masked_lo[4] = {0u, 0u, 0u, 0u};
        const uint32_t pb = ~masked_lo[dir];
        const uint32_t py = ~masked_lo[2 + dir];
        const uint32_t yw = y32[row * ng + gg];
        const uint32_t cb = cwb32[(krow * 4 + dir) * ng + gg];
        const uint32_t cy = cwb32[(krow * 4 + 2 + dir) * ng + gg];
        reinterpret_cast<uint32_t*>(J.dst_t)[de * ng + g] = pb ^ (tw & cb);
        reinterpret_cast<uint32_t*>(J.dst_y)[de * ng + g] = py ^ (tw & cy) ^ yw;
    }
    prof_mark<PROF>(tl, acc, 4);   // 4: feed-forward + stores
}

// WAVES >= 3: the LDS (32 KiB per pair) admits 5 pairs = 2.5 waves/SIMD, which the compiler's
// occupancy model floors to 2 — cap the VGPRs explicitly so 3 waves fit on a SIMD
template <int FENCE, bool ROLLED, bool PROF, int CWORDS>
__device__ __forceinline__ void bs_pair2_body(const ExpandLaunch& a, uint32_t* work_counter, SeedQuads& yl,
                                              uint32_t& item_slot) {
    const uint32_t lane = threadIdx.x & 63;
    const int dir = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const LoopCtl* ctl = a.ctl;
    const uint64_t total = ctl ? (ctl->abort ? 0 : ctl->total_items) : a.total_items;
    uint64_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tl = PROF ? __builtin_amdgcn_s_memtime() : 0;
    if (threadIdx.x == 0) item_slot = atomicAdd(work_counter, 1u);
    __syncthreads();
    uint64_t item = __builtin_amdgcn_readfirstlane(item_slot);
    __syncthreads();
    prof_mark<PROF>(tl, acc, 0);
    while (item < total) {
        uint32_t nxt = 0;
        if (threadIdx.x == 0) nxt = atomicAdd(work_counter, 1u);   // one item ahead
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
        prof_mark<PROF>(tl, acc, 0);   // 0: item / job lookup
        bs_pair2_item<FENCE, ROLLED, PROF, CWORDS>(J, item - J.item_begin, lane, dir, yl, tl, acc);
        if (threadIdx.x == 0) item_slot = nxt;
        __syncthreads();   // both waves are done with yl; the next item is published
        item = __builtin_amdgcn_readfirstlane(item_slot);
        __syncthreads();   // the slot may alias y storage: both waves read it before y is rewritten
        prof_mark<PROF>(tl, acc, 5);   // 5: end barrier
    }
    if constexpr (PROF) {
        if (lane == 0)
            for (int k = 0; k < 6; k++) atomicAdd(&g_bs_prof[k], (unsigned long long)acc[k]);
    }
    // every workgroup drew exactly one item past the end; the last one re-arms the counter
    if (threadIdx.x == 0) {
        const uint32_t done = atomicAdd(work_counter + 1, 1u);
        if (done + 1 == gridDim.x) {
            atomicExch(work_counter, 0u);
            atomicExch(work_counter + 1, 0u);
        }
    }
}

template <int WAVES, int FENCE, bool ROLLED, bool PROF = false, int CWORDS = 24>
__global__ __launch_bounds__(128, 2) void k_expand_bs_pair2(ExpandLaunch a, uint32_t* work_counter) {
    // exactly 32 KiB of LDS (the item slot lives in the last y word, see bs_pair2_body), so a
    // pair fits beside a 128 KiB T-table workgroup on one CU (hybrid runs)
    __shared__ SeedQuads yl;
    bs_pair2_body<FENCE, ROLLED, PROF, CWORDS>(a, work_counter, yl, reinterpret_cast<uint32_t*>(&yl[31][63])[3]);
}

// 3 waves/SIMD: the LDS (32 KiB per pair) admits 5 pairs = 2.5 waves/SIMD, which the
// compiler's occupancy model floors to 2 — the LDS is dynamic so the 168-VGPR budget holds
constexpr size_t kPair2DynLds = sizeof(SeedQuads);
template <int FENCE, bool ROLLED, int CWORDS>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_expand_bs_pair2_w3(
    ExpandLaunch a, uint32_t* work_counter) {
    // dynamic LDS (kPair2DynLds bytes at launch): invisible to the compiler's occupancy model
    extern __shared__ uint8_t dyn_lds[];
    SeedQuads& yl = *reinterpret_cast<SeedQuads*>(dyn_lds);
    uint32_t& item_slot = reinterpret_cast<uint32_t*>(&yl[31][63])[3];
    bs_pair2_body<FENCE, ROLLED, false, CWORDS>(a, work_counter, yl, item_slot);
}

// WAVES: waves per SIMD the register budget must admit (2: 256 VGPRs, 3: 168)
template <int THR, int WAVES, int FENCE, bool ROLLED>
__global__ __launch_bounds__(THR, WAVES) void k_expand_bs(ExpandLaunch a, uint32_t* work_counter) {
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
        bs_item<FENCE, ROLLED>(J, item - J.item_begin, lane);
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

// bitsliced variants: (waves per SIMD, fence granularity, pair mode, rolled rounds);
// index = variant - kBsVariant
#define FHH_BS_VARIANTS(X) \
    X(0, 2, 2, 0, 0)       \
    X(1, 3, 1, 0, 0)       \
    X(2, 2, 2, 1, 0)       \
    X(3, 3, 1, 1, 0)       \
    X(4, 2, 2, 1, 1)       \
    X(5, 2, 2, 0, 1)       \
    X(6, 2, 2, 3, 1)       \
    X(7, 2, 2, 4, 1)       \
    X(8, 2, 2, 5, 1)       \
    X(9, 2, 2, 4, 0)       \
    X(10, 2, 2, 6, 1)      \
    X(11, 3, 1, 7, 1)      \
    X(12, 3, 1, 7, 0)

// P (mode): 0 single-wave items, 1 pair, 3 pair + phase profile, 4 pair v2, 5 pair v2 + profile,
// 6 pair v2 with a 4-bit register carry window (exercises the long-carry slow path; tests),
// 7 pair v2 with a 16-bit carry window (register budget of 3 waves/SIMD)
template <int W, int F, int P, int R>
static const void* bs_fn() {
    if constexpr (P == 6) return reinterpret_cast<const void*>(&k_expand_bs_pair2<W, F, R != 0, false, 4>);
    else if constexpr (P == 7) return reinterpret_cast<const void*>(&k_expand_bs_pair2_w3<F, R != 0, 16>);
    else if constexpr (P == 4 || P == 5) return reinterpret_cast<const void*>(&k_expand_bs_pair2<W, F, R != 0, P == 5>);
    else if constexpr (P) return reinterpret_cast<const void*>(&k_expand_bs_pair<W, F, R != 0, P == 3>);
    else return reinterpret_cast<const void*>(&k_expand_bs<kBsThreads, W, F, R != 0>);
}

template <int W, int F, int P, int R>
static void bs_launch(const ExpandLaunch& a, int g, uint32_t* work_counter, hipStream_t stream) {
    if constexpr (P == 6)
        hipLaunchKernelGGL((k_expand_bs_pair2<W, F, R != 0, false, 4>), dim3(g), dim3(128), 0, stream, a,
                           work_counter);
    else if constexpr (P == 7)
        hipLaunchKernelGGL((k_expand_bs_pair2_w3<F, R != 0, 16>), dim3(g), dim3(128), kPair2DynLds, stream, a,
                           work_counter);
    else if constexpr (P == 4 || P == 5)
        hipLaunchKernelGGL((k_expand_bs_pair2<W, F, R != 0, P == 5>), dim3(g), dim3(128), 0, stream, a,
                           work_counter);
    else if constexpr (P)
        hipLaunchKernelGGL((k_expand_bs_pair<W, F, R != 0, P == 3>), dim3(g), dim3(128), 0, stream, a,
                           work_counter);
    else
        hipLaunchKernelGGL((k_expand_bs<kBsThreads, W, F, R != 0>), dim3(g), dim3(kBsThreads), 0, stream, a,
                           work_counter);
}

hipError_t launch_expand_bs(const ExpandLaunch& a, int which, int grid, uint32_t* work_counter, hipStream_t stream) {
    if (a.total_items == 0) return hipSuccess;
    const int thr = expand_bs_threads(which);
    const uint64_t per_block = bs_pair_mode(which) ? 1 : (uint64_t)thr / 64;   // items in flight per block
    const uint64_t blocks_needed = (a.total_items + per_block - 1) / per_block;
    const int g = a.ctl ? grid : (int)(blocks_needed < (uint64_t)grid ? blocks_needed : (uint64_t)grid);
    switch (which) {
#define FHH_BS_CASE(id, W, F, P, R) \
    case id: bs_launch<W, F, P, R>(a, g, work_counter, stream); break;
        FHH_BS_VARIANTS(FHH_BS_CASE)
#undef FHH_BS_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

const void* expand_bs_fn(int which) {
    switch (which) {
#define FHH_BS_CASE(id, W, F, P, R) \
    case id: return bs_fn<W, F, P, R>();
        FHH_BS_VARIANTS(FHH_BS_CASE)
#undef FHH_BS_CASE
        default: return nullptr;
    }
}

int expand_bs_count() { return kBsCount; }
size_t expand_bs_dyn_lds(int which) { return (which == 11 || which == 12) ? kPair2DynLds : 0; }

}  // namespace fhh

// debug: phase-cycle profile of the profiling pair variant (kBsVariant + 6); reset after read
extern "C" int fhh_debug_bs_profile(double* out6) {
    unsigned long long h[8] = {0};
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(fhh::g_bs_prof), sizeof h) != hipSuccess) return -3;
    for (int k = 0; k < 6; k++) out6[k] = (double)h[k];
    unsigned long long z[8] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(fhh::g_bs_prof), z, sizeof z) != hipSuccess) return -3;
    return 0;
}

namespace fhh {
int expand_bs_threads(int which) { return bs_pair_mode(which) ? 128 : kBsThreads; }

}  // namespace fhh

#else   // !FHH_AB_VARIANTS: no bitsliced variant in this build (set_variant refuses 14..26)
namespace fhh {
hipError_t launch_expand_bs(const ExpandLaunch&, int, int, uint32_t*, hipStream_t) { return hipErrorInvalidValue; }
const void* expand_bs_fn(int) { return nullptr; }
int expand_bs_count() { return 0; }
int expand_bs_threads(int) { return 0; }
size_t expand_bs_dyn_lds(int) { return 0; }
hipError_t launch_bitslice(const uint4*, uint4*, uint64_t, uint32_t, int, hipStream_t) { return hipErrorInvalidValue; }
}  // namespace fhh
#endif
