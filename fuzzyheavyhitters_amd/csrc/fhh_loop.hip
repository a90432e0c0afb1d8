// Device-resident level loop: the leader's keep decision and the servers' prune
// (keep_values / keep_values_last, collect.rs:945-989; tree_prune, collect.rs:918-929) run on
// the GPU so that k_expand -> count/sums -> [all-reduce] -> k_prune repeat without host round
// trips. Sizes of the next level live in LoopCtl (device memory).
//
// k_prune is one 1024-thread workgroup: C (children) and n_live (entries) are at most a few
// thousand, so the scans fit one workgroup.
#include "fhh_internal.h"
#include "field_arith.h"

namespace fhh {

constexpr int kPruneThreads = 1024;

// exclusive scan of one u32 per thread over the workgroup; *total = sum (uniform)
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds /*[16]*/, uint32_t* total) {
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off, 64);
        if (lane >= (uint32_t)off) x += y;
    }
    if (lane == 63) lds[wid] = x;
    __syncthreads();
    uint32_t wbase = 0, tot = 0;
    for (uint32_t i = 0; i < nw; i++) {
        const uint32_t t = lds[i];
        if (i < wid) wbase += t;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return wbase + x - v;
}

__device__ __forceinline__ bool keep_of(const PruneArgs& a, uint32_t c) {
    if (a.mode == 0) return a.partials[c] >= (a.last ? (uint64_t)a.thr_last : a.thr);
    if (a.mode == 1 && a.ring32) {   // r06: Z_2^32 shares (the count is < 2^32)
        const uint64_t* p = a.partials + (size_t)c * 4;
        return (uint64_t)(uint32_t)(p[0] - p[2]) >= a.thr;
    }
    if (a.mode == 1) {
        const uint64_t* p = a.partials + (size_t)c * 4;
        const uint64_t s0 = fe_canon_from_limbs(p[0], p[1]), s1 = fe_canon_from_limbs(p[2], p[3]);
        return fe_sub_canon(s0, s1) >= a.thr % kFieldFeP;
    }
    const uint64_t* p = a.partials + (size_t)c * 16;
    uint32_t v0[10], v1[10], r0[8], r1[8], d[8];
    limbs10_from_partials(p, v0);
    limbs10_from_partials(p + 8, v1);
    fe255_reduce(v0, r0);
    fe255_reduce(v1, r1);
    fe255_sub(r0, r1, d);
    return fe255_ge_u32(d, a.thr_last);
}

__global__ __launch_bounds__(kPruneThreads) void k_prune(PruneArgs a) {
    __shared__ uint32_t lds[16];
    LoopCtl* ctl = a.ctl;
    if (ctl->abort) return;
    const uint32_t C = ctl->C, d = a.d, mask = (1u << d) - 1;

    // 1. keep flags -> ordered list of kept children (tree_prune keeps order, collect.rs:918-929)
    uint32_t nf = 0;
    for (uint32_t base = 0; base < C; base += blockDim.x) {
        const uint32_t c = base + threadIdx.x;
        const uint32_t flag = (c < C && keep_of(a, c)) ? 1u : 0u;
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan(flag, lds, &tot);
        if (flag && nf + ex < a.F_cap) a.hist_out[nf + ex] = c;
        nf += tot;
    }
    if (threadIdx.x == 0) {
        a.sizes_out[0] = C;
        a.sizes_out[1] = nf;
    }
    __syncthreads();

    if (a.last) {
        // tree_crawl_last: the kept children are frontier_last; record their values
        if (nf > a.F_cap) {
            if (threadIdx.x == 0) {
                ctl->need_nodes = nf;
                ctl->abort_level = a.level;
                ctl->abort = 1;
                a.sizes_out[2] = 1;
            }
            return;
        }
        for (uint32_t k = threadIdx.x; k < nf; k += blockDim.x) {
            const uint32_t c = a.hist_out[k];
            uint32_t* out = a.final_vals + (size_t)k * 20;
            if (a.mode == 2) {
                limbs10_from_partials(a.partials + (size_t)c * 16, out);
                limbs10_from_partials(a.partials + (size_t)c * 16 + 8, out + 10);
            } else {
                const uint64_t v = a.mode == 0 ? a.partials[c]
                                               : fe_sub_canon(fe_canon_from_limbs(a.partials[c * 4], a.partials[c * 4 + 1]),
                                                              fe_canon_from_limbs(a.partials[c * 4 + 2],
                                                                                  a.partials[c * 4 + 3]));
                for (int q = 0; q < 20; q++) out[q] = 0;
                out[0] = (uint32_t)v;
                out[1] = (uint32_t)(v >> 32);
            }
        }
        return;   // frontier unchanged by tree_crawl_last (collect.rs:909-914)
    }

    // 2. per dim: referenced child entries -> new live list (sorted) and node positions
    uint32_t n_live_new[kMaxDims] = {0, 0, 0, 0};
    bool fits = nf <= a.F_cap;
    if (!fits)   // entries are not counted then; n_live' <= nf bounds them (one abort, not two)
        for (uint32_t j = 0; j < d; j++) n_live_new[j] = nf;
    for (uint32_t j = 0; j < d && fits; j++) {
        const uint32_t E = 2 * ctl->n_live[j];
        uint32_t* mk = a.mark + (size_t)j * a.E_cap;
        for (uint32_t e = threadIdx.x; e < E; e += blockDim.x) mk[e] = 0;
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < nf; k += blockDim.x) {
            const uint32_t c = a.hist_out[k], p = c >> d, i = c & mask;
            mk[2 * a.pos_in[(size_t)p * d + j] + ((i >> j) & 1)] = 1;
        }
        __syncthreads();
        uint32_t nl = 0;
        for (uint32_t base = 0; base < E; base += blockDim.x) {
            const uint32_t e = base + threadIdx.x;
            const uint32_t flag = e < E ? mk[e] : 0u;
            uint32_t tot;
            const uint32_t ex = block_exclusive_scan(flag, lds, &tot);
            if (flag) {
                mk[e] = nl + ex + 1;                     // index + 1
                if (nl + ex < a.E_cap) a.live_out[j][nl + ex] = e;
            }
            nl += tot;
        }
        n_live_new[j] = nl;
        if (2 * nl > a.E_cap) fits = false;             // next k_expand writes 2 * nl entries
        __syncthreads();
        if (fits)
            for (uint32_t k = threadIdx.x; k < nf; k += blockDim.x) {
                const uint32_t c = a.hist_out[k], p = c >> d, i = c & mask;
                a.pos_out[(size_t)k * d + j] = mk[2 * a.pos_in[(size_t)p * d + j] + ((i >> j) & 1)] - 1;
            }
        __syncthreads();
    }
    // the next FE level's atomically-added partials start from zero (every read of this level's
    // partials is behind the barriers above; an aborted prune leaves them for its resumption)
    if (fits && a.zero_partials)
        for (uint64_t k = threadIdx.x; k < a.zero_count; k += blockDim.x) a.zero_partials[k] = 0;
    if (threadIdx.x != 0) return;
    if (!fits) {
        uint32_t need = 0;
        for (uint32_t j = 0; j < d; j++) need = max(need, 2 * n_live_new[j]);
        ctl->need_entries = need;
        ctl->need_nodes = nf;
        ctl->abort_level = a.level;
        ctl->abort = 1;
        a.sizes_out[2] = 1;
        return;
    }
    // 3. next level's sizes and k_expand work decomposition (item_layout, as finalize_launch)
    uint32_t job_live[kMaxJobs] = {};
    for (uint32_t j = 0; j < d; j++) {
        ctl->n_live[j] = n_live_new[j];
        a.sizes_out[4 + j] = n_live_new[j];
    }
    const uint32_t njobs = a.nctx * a.njobs_per_ctx;
    for (uint32_t k = 0; k < njobs; k++) job_live[k] = n_live_new[k % a.njobs_per_ctx];
    ItemLayout lay;
    item_layout(job_live, njobs, a.unit, a.max_group, a.grid_waves, a.tail_split != 0, lay, a.max_wpi);
    for (uint32_t k = 0; k < njobs; k++) {
        ctl->item_begin[k] = lay.begin_a[k];
        ctl->item_begin_b[k] = lay.begin_b[k];
        ctl->split[k] = lay.split[k];
    }
    ctl->group = lay.g;
    ctl->group_b = lay.g_b;
    ctl->wpi = lay.wpi;
    ctl->items_a = lay.items_a;
    ctl->total_items = lay.total;
    ctl->F = nf;
    ctl->C = nf << d;
}

hipError_t launch_prune(const PruneArgs& a, hipStream_t stream) {
    hipLaunchKernelGGL(k_prune, dim3(1), dim3(kPruneThreads), 0, stream, a);
    return hipGetLastError();
}

// End-of-crawl readback: pack every level's kept-children list (hist rows live at per-level
// pointers, possibly in several capacity epochs) into one array, so the host copies it with
// one D2H transfer instead of one synchronous copy per level. Block lv computes its offset as
// the sum of the kept counts of the levels before it (sizes[k * stride + 1]).
__global__ __launch_bounds__(256) void k_gather_hist(const uint32_t* sizes, uint32_t stride,
                                                     const uint32_t* const* rows, uint32_t* out, uint64_t cap) {
    __shared__ uint64_t red[4];
    const uint32_t lv = blockIdx.x;
    uint64_t v = 0;
    for (uint32_t k = threadIdx.x; k < lv; k += blockDim.x) v += sizes[(size_t)k * stride + 1];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    const uint64_t base = red[0] + red[1] + red[2] + red[3];
    const uint32_t nf = sizes[(size_t)lv * stride + 1];
    const uint32_t* src = rows[lv];
    for (uint32_t i = threadIdx.x; i < nf && base + i < cap; i += blockDim.x) out[base + i] = src[i];
}

hipError_t launch_gather_hist(const uint32_t* sizes, uint32_t stride, const uint32_t* const* rows, uint32_t levels,
                              uint32_t* out, uint64_t cap, hipStream_t stream) {
    if (levels == 0) return hipSuccess;
    hipLaunchKernelGGL(k_gather_hist, dim3(levels), dim3(256), 0, stream, sizes, stride, rows, out, cap);
    return hipGetLastError();
}

// One lane per (server, child, probed client, dim, side): child c's dim-j entry in the child
// table is 2 * parent_pos[(c >> d) * d + j] + ((c >> j) & 1), as k_eq_count reads it.
__global__ __launch_bounds__(256) void k_probe_states(ProbeArgs a) {
    const LoopCtl* ctl = a.ctl;
    if (ctl->abort) return;   // re-run after the resumption
    const uint64_t C = ctl->C < a.C_cap ? ctl->C : a.C_cap;
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.out_C = ctl->C;
    const uint32_t d = a.d, mask = (1u << d) - 1;
    const uint64_t per_c = (uint64_t)a.n_probe * d * 2;
    const uint64_t total = 2 * C * per_c;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < total;
         k += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t s = (uint32_t)(k & 1);
        uint64_t r = k >> 1;
        const uint32_t j = (uint32_t)(r % d);
        r /= d;
        const uint32_t i = (uint32_t)(r % a.n_probe);
        r /= a.n_probe;
        const uint64_t c = r % C;
        const uint32_t srv = (uint32_t)(r / C);
        const uint32_t e = 2 * a.parent_pos[(c >> d) * d + j] + (((uint32_t)(c & mask) >> j) & 1);
        const uint64_t x = a.clients[i];
        const size_t row = (size_t)e * 2 + s;
        const uint4 sd = a.seed[srv][j][row * a.npad + x];
        const uint64_t tb = (a.t[srv][j][row * a.nw + (x >> 6)] >> (x & 63)) & 1;
        const uint64_t yb = (a.y[srv][j][row * a.nw + (x >> 6)] >> (x & 63)) & 1;
        const size_t o = (((size_t)srv * a.C_cap + c) * a.n_probe + i) * d * 2 + (size_t)j * 2 + s;
        a.out_seed[o] = sd;
        a.out_ty[o] = (uint8_t)(tb | (yb << 1));
    }
}

hipError_t launch_probe_states(const ProbeArgs& a, hipStream_t stream) {
    const uint64_t most = 2 * a.C_cap * a.n_probe * a.d * 2;
    const uint64_t blocks = (most + 255) / 256;
    hipLaunchKernelGGL(k_probe_states, dim3((uint32_t)(blocks < 4096 ? (blocks ? blocks : 1) : 4096)), dim3(256), 0,
                       stream, a);
    return hipGetLastError();
}

__global__ void k_loop_init(LoopCtl* ctl, uint32_t d, uint32_t unit, uint32_t max_group, uint32_t max_wpi,
                            uint32_t njobs_per_ctx,
                            uint32_t nctx,
                            uint64_t grid_waves, uint32_t* pos0, uint32_t* l0, uint32_t* l1, uint32_t* l2,
                            uint32_t* l3) {
    if (threadIdx.x != 0) return;
    uint32_t* lv[kMaxDims] = {l0, l1, l2, l3};
    ctl->abort = 0;
    ctl->abort_level = 0;
    ctl->need_entries = 0;
    ctl->need_nodes = 0;
    ctl->F = 1;
    ctl->C = 1u << d;
    for (uint32_t j = 0; j < kMaxDims; j++) ctl->n_live[j] = j < d ? 1 : 0;
    for (uint32_t j = 0; j < d; j++) {
        pos0[j] = 0;
        lv[j][0] = 0;
    }
    // level 0: one root entry per job (no end phase: far fewer items than waves)
    const uint32_t njobs = nctx * njobs_per_ctx;
    uint32_t job_live[kMaxJobs];
    for (uint32_t k = 0; k < kMaxJobs; k++) job_live[k] = 1;
    ItemLayout lay;
    item_layout(job_live, njobs, unit, max_group, grid_waves, false, lay, max_wpi);
    for (uint32_t k = 0; k < njobs; k++) {
        ctl->item_begin[k] = lay.begin_a[k];
        ctl->item_begin_b[k] = lay.begin_b[k];
        ctl->split[k] = lay.split[k];
    }
    ctl->group = lay.g;
    ctl->group_b = lay.g_b;
    ctl->wpi = lay.wpi;
    ctl->items_a = lay.items_a;
    ctl->total_items = lay.total;
}

hipError_t launch_loop_init(LoopCtl* ctl, uint32_t d, uint32_t unit, uint32_t max_group, uint32_t max_wpi,
                            uint32_t njobs_per_ctx, uint32_t nctx, uint64_t grid_waves, uint32_t* pos0,
                            uint32_t* live0[kMaxDims], hipStream_t stream) {
    hipLaunchKernelGGL(k_loop_init, dim3(1), dim3(64), 0, stream, ctl, d, unit, max_group, max_wpi, njobs_per_ctx, nctx,
                       grid_waves, pos0,
                       live0[0], live0[1], live0[2], live0[3]);
    return hipGetLastError();
}

}  // namespace fhh
