// Peak-rate microbenchmarks that pin the roofline denominators on the box itself
// ("confirm P_int with a v_xor_b32 throughput microbenchmark"):
//   which = 0: v_xor_b32 lane-ops/s, every CU, 8 waves/SIMD, independent chains
//   which = 1: ds_read_b32 bytes/s with the k_expand access pattern (per-lane replica,
//              bank-conflict free, data-dependent byte index)
//   which = 5: v_mad_u64_u32 lane-ops/s (the 32 x 32 + 64 -> 64 multiply-add of the FE products of
//              k_sketch_fe), 8 waves/SIMD, independent chains; 6: the same at 4 waves/SIMD
//   which = 7 / 8: v_alignbit_b32 / v_add_u32 lane-ops/s (r06: the ChaCha12 row PRG's rotate and add),
//              8 waves/SIMD; 9: ChaCha double rounds over 2 independent states per lane (12 ops per
//              quarter round counted), 8 waves/SIMD; 10: the same at 2 waves/SIMD; 11 / 12: v_perm_b32 /
//              v_lshl_or_b32
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/fhh.h"

namespace fhh {

__global__ __launch_bounds__(256) void k_valu_peak(uint32_t* out, uint32_t iters, uint32_t seed) {
    uint32_t x[16];
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = seed * (threadIdx.x + 1) + k * 0x9e3779b9u + blockIdx.x;
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < 8; r++) {
#pragma unroll
            for (int k = 0; k < 16; k++) x[k] ^= x[(k + 1 + r) & 15];
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) acc ^= x[k];
    if (acc == 0x12345678u) out[0] = acc;   // keep live
}

// v_bitop3_b32 with three distinct VGPR sources (the bitsliced AES's only op)
__global__ __launch_bounds__(256) void k_bitop3_peak(uint32_t* out, uint32_t iters, uint32_t seed) {
    uint32_t x[16];
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = seed * (threadIdx.x + 1) + k * 0x9e3779b9u + blockIdx.x;
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < 8; r++) {
#pragma unroll
            for (int k = 0; k < 16; k++)
                x[k] = __builtin_amdgcn_bitop3_b32(x[k], x[(k + 1 + r) & 15], x[(k + 6 + r) & 15], 0x6A);
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) acc ^= x[k];
    if (acc == 0x12345678u) out[0] = acc;   // keep live
}

// v_mad_u64_u32: 16 independent 64-bit accumulators, each step one 32 x 32 + 64 multiply-add
__global__ __launch_bounds__(256) void k_mad64_peak(uint32_t* out, uint32_t iters, uint32_t seed) {
    uint64_t x[16];
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = (uint64_t)(seed * (threadIdx.x + 1) + k * 0x9e3779b9u + blockIdx.x) << 7;
    const uint32_t m = seed | 0x10001u;
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < 8; r++) {
#pragma unroll
            for (int k = 0; k < 16; k++) x[k] = (uint64_t)(uint32_t)x[(k + 1 + r) & 15] * (m + r) + x[k];
        }
    }
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) acc ^= x[k];
    if (acc == 0x12345678u) out[0] = (uint32_t)acc;   // keep live
}

// v_alignbit_b32 (OP 0) / v_add_u32 (OP 1) over 16 independent words, as k_valu_peak
template <int OP>
__global__ __launch_bounds__(256) void k_valu_op_peak(uint32_t* out, uint32_t iters, uint32_t seed) {
    uint32_t x[16];
#pragma unroll
    for (int k = 0; k < 16; k++) x[k] = seed * (threadIdx.x + 1) + k * 0x9e3779b9u + blockIdx.x;
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int r = 0; r < 8; r++) {
#pragma unroll
            for (int k = 0; k < 16; k++) {
                if constexpr (OP == 0) x[k] = __builtin_amdgcn_alignbit(x[(k + 1 + r) & 15], x[k], 7 + r);
                else if constexpr (OP == 2) x[k] = __builtin_amdgcn_perm(x[(k + 1 + r) & 15], x[k], 0x05040302u + r);
                else if constexpr (OP == 3) x[k] = (x[k] << (7 + r)) | x[(k + 1 + r) & 15];
                else x[k] += x[(k + 1 + r) & 15];
            }
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) acc ^= x[k];
    if (acc == 0x12345678u) out[0] = acc;   // keep live
}

__device__ __forceinline__ uint32_t mb_rotl(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, 32 - n); }
__device__ __forceinline__ void mb_qr(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
    a += b; d ^= a; d = mb_rotl(d, 16);
    c += d; b ^= c; b = mb_rotl(b, 12);
    a += b; d ^= a; d = mb_rotl(d, 8);
    c += d; b ^= c; b = mb_rotl(b, 7);
}

// ChaCha double rounds over 2 independent 16-word states per lane (the expands' ILP)
__global__ __launch_bounds__(256) void k_chacha_peak(uint32_t* out, uint32_t iters, uint32_t seed) {
    uint32_t x[2][16];
#pragma unroll
    for (int q = 0; q < 2; q++)
#pragma unroll
        for (int k = 0; k < 16; k++) x[q][k] = seed * (threadIdx.x + 1) + (16 * q + k) * 0x9e3779b9u + blockIdx.x;
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int q = 0; q < 2; q++) {
            mb_qr(x[q][0], x[q][4], x[q][8], x[q][12]);
            mb_qr(x[q][1], x[q][5], x[q][9], x[q][13]);
            mb_qr(x[q][2], x[q][6], x[q][10], x[q][14]);
            mb_qr(x[q][3], x[q][7], x[q][11], x[q][15]);
            mb_qr(x[q][0], x[q][5], x[q][10], x[q][15]);
            mb_qr(x[q][1], x[q][6], x[q][11], x[q][12]);
            mb_qr(x[q][2], x[q][7], x[q][8], x[q][13]);
            mb_qr(x[q][3], x[q][4], x[q][9], x[q][14]);
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int q = 0; q < 2; q++)
#pragma unroll
        for (int k = 0; k < 16; k++) acc ^= x[q][k];
    if (acc == 0x12345678u) out[0] = acc;   // keep live
}

__global__ __launch_bounds__(512) void k_lds_peak(uint32_t* out, uint32_t iters) {
    __shared__ uint32_t tbl[256 * 64];
    for (int i = threadIdx.x; i < 256 * 64; i += blockDim.x) tbl[i] = (uint32_t)i * 2654435761u;
    __syncthreads();
    const uint32_t lb = (threadIdx.x & 63) * 4;
    uint32_t x[8];
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = threadIdx.x * 31 + k * 77;
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint32_t a = __builtin_amdgcn_perm(lb, x[k], 0x0C0C0104u);
            x[k] = *(const uint32_t*)((const char*)tbl + a);
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) acc ^= x[k];
    if (acc == 0x12345678u) out[0] = acc;
}

// Mixed lookup paths: NL dependent chains through the per-lane-replica LDS table (as
// k_lds_peak / k_expand) and NG dependent chains through a read-only global table of
// `gbytes` bytes (4-byte entries, L1/L2 resident), issued as buffer_load_dword with a
// data-dependent offset. Measures whether the vector-memory path adds lookup throughput
// beside a saturated LDS (fhh_microbench_gather).
template <int NL, int NG>
__global__ __launch_bounds__(512) void k_gather_mix(const uint32_t* __restrict__ gtab, uint32_t gmask,
                                                    uint32_t* out, uint32_t iters) {
    __shared__ uint32_t tbl[256 * 64];
    for (int i = threadIdx.x; i < 256 * 64; i += blockDim.x) tbl[i] = (uint32_t)i * 2654435761u;
    __syncthreads();
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(gtab), 0, (int)((gmask + 1) * 4), 0x00020000);
    const uint32_t lb = (threadIdx.x & 63) * 4;
    uint32_t x[NL > 0 ? NL : 1], y[NG > 0 ? NG : 1];
#pragma unroll
    for (int k = 0; k < (NL > 0 ? NL : 1); k++) x[k] = threadIdx.x * 31 + k * 77;
#pragma unroll
    for (int k = 0; k < (NG > 0 ? NG : 1); k++) y[k] = threadIdx.x * 131 + k * 7919 + blockIdx.x;
    for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < NL; k++) {
            const uint32_t a = __builtin_amdgcn_perm(lb, x[k], 0x0C0C0104u);
            x[k] = *(const uint32_t*)((const char*)tbl + a);
        }
#pragma unroll
        for (int k = 0; k < NG; k++)
            y[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)((y[k] & gmask) << 2), 0, 0);
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < NL; k++) acc ^= x[k];
#pragma unroll
    for (int k = 0; k < NG; k++) acc ^= y[k];
    if (acc == 0x12345678u) out[0] = acc;
}

// Can VALU-only waves add work beside LDS-bound waves in the same workgroup? 1024-thread
// workgroups (4 waves/SIMD, <= 128 VGPRs); waves 0 .. 15-NB run k_expand-shaped lookup chains
// (one ds_read_b32 + one v_perm + one v_bitop3 per lookup, ~ the T-table's 1.7 VALU per
// lookup), waves 16-NB .. 15 run independent v_bitop3 chains over 48 live words (a bitsliced
// AES's shape) until the lookup waves are done (LDS flag). counts[0] += lookups,
// counts[1] += bitop3 lane-ops (fhh_microbench_hybrid).
template <int NB>
__global__ __launch_bounds__(1024) void k_hybrid_mix(unsigned long long* counts, uint32_t iters) {
    __shared__ uint32_t tbl[256 * 64];
    __shared__ uint32_t done;
    for (int i = threadIdx.x; i < 256 * 64; i += blockDim.x) tbl[i] = (uint32_t)i * 2654435761u;
    if (threadIdx.x == 0) done = 0;
    __syncthreads();
    const int w = threadIdx.x >> 6;
    if (w < 16 - NB) {
        const uint32_t lb = (threadIdx.x & 63) * 4;
        uint32_t x[8];
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = threadIdx.x * 31 + k * 77;
        for (uint32_t i = 0; i < iters; i++) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                const uint32_t a = __builtin_amdgcn_perm(lb, x[k], 0x0C0C0104u);
                const uint32_t v = *(const uint32_t*)((const char*)tbl + a);
                x[k] = __builtin_amdgcn_bitop3_b32(v, x[k], x[(k + 1) & 7], 0x96);
            }
        }
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) acc ^= x[k];
        if (acc == 0x12345678u) counts[2] = acc;
        __atomic_fetch_add(&done, 1u, __ATOMIC_RELAXED);
        if ((threadIdx.x & 63) == 0) atomicAdd(&counts[0], (unsigned long long)iters * 8 * 64);
    } else {
        uint32_t x[48];
#pragma unroll
        for (int k = 0; k < 48; k++) x[k] = threadIdx.x * (k + 3) + k * 0x9e3779b9u + blockIdx.x;
        uint32_t n = 0;
        while (__atomic_load_n(&done, __ATOMIC_RELAXED) < (uint32_t)(64 * (16 - NB))) {
#pragma unroll
            for (int r = 0; r < 4; r++) {
#pragma unroll
                for (int k = 0; k < 48; k++)
                    x[k] = __builtin_amdgcn_bitop3_b32(x[k], x[(k + 1 + r) % 48], x[(k + 17 + r) % 48], 0x6A);
            }
            n++;
        }
        uint32_t acc = 0;
#pragma unroll
        for (int k = 0; k < 48; k++) acc ^= x[k];
        if (acc == 0x12345678u) counts[2] = acc;
        if ((threadIdx.x & 63) == 0) atomicAdd(&counts[1], (unsigned long long)n * 4 * 48 * 64);
    }
}

// launch-gap probe: a kernel that only touches its dynamic LDS (so the LDS allocation is
// real) and, from one lane, one word of global memory
__global__ void k_gap_probe(uint32_t* out, uint32_t tag) {
    extern __shared__ uint32_t lds_dyn[];
    lds_dyn[threadIdx.x] = tag;
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0) out[1] = lds_dyn[(threadIdx.x + 1) % blockDim.x];
}

// writes `words_per_thread` u32 per thread (coalesced), normal or nontemporal stores
template <bool NT>
__global__ void k_gap_writer(uint32_t* dst, uint32_t words_per_thread) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint32_t k = 0; k < words_per_thread; k++, i += stride) {
        if (NT) __builtin_nontemporal_store((uint32_t)k, dst + i);
        else dst[i] = (uint32_t)k;
    }
}

}  // namespace fhh

// Device time per kernel of a back-to-back chain on one stream (HIP events around `reps`
// launches). which: 0 = 256 x 1024 threads, no LDS; 1 = 256 x 1024, 128 KiB LDS (k_expand's
// footprint); 2 = alternate 256 x 1024 / 128 KiB with 1 x 1024 / 4 KiB (expand -> prune);
// 3 = 1 x 1024 threads, 4 KiB (prune alone); 4 / 5 = alternate a 256 x 1024 kernel writing
// 64 MiB (normal / nontemporal stores) with 1 x 1024 (does dirty L2 cost the next launch?).
extern "C" int fhh_debug_launch_gaps(int device, int which, int reps, double* us_per_kernel) {
    if (!us_per_kernel || reps < 1 || which < 0 || which > 7) return FHH_E_ARG;
    const bool graph = which >= 6;   // 6 / 7: as 2 / 4, captured once into a hipGraph and replayed
    if (graph) which = which == 6 ? 2 : 4;
    if (hipSetDevice(device) != hipSuccess) return FHH_E_HIP;
    uint32_t* out = nullptr;
    if (hipMalloc(&out, 64u << 20) != hipSuccess) return FHH_E_NOMEM;
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
        (void)hipFree(out);
        return FHH_E_HIP;
    }
    (void)hipFuncSetAttribute((const void*)fhh::k_gap_probe, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    float ms = 0.f;
    hipGraphExec_t gexec = nullptr;
    for (int pass = 0; pass < 2; pass++) {
        if (graph && gexec) {
            (void)hipEventRecord(a, st);
            (void)hipGraphLaunch(gexec, st);
            (void)hipEventRecord(b, st);
            if (hipEventSynchronize(b) != hipSuccess) break;
            (void)hipEventElapsedTime(&ms, a, b);
            continue;
        }
        hipGraph_t g = nullptr;
        if (graph) {
            if (hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) != hipSuccess) break;
        } else {
            (void)hipEventRecord(a, st);
        }
        for (int r = 0; r < reps; r++) {
            if (which >= 4 && (r & 1) == 0) {
                if (which == 4) hipLaunchKernelGGL(fhh::k_gap_writer<false>, dim3(256), dim3(1024), 0, st, out, 64u);
                else hipLaunchKernelGGL(fhh::k_gap_writer<true>, dim3(256), dim3(1024), 0, st, out, 64u);
                continue;
            }
            const bool big = which == 1 || (which == 2 && (r & 1) == 0);
            const bool one = which >= 3 || (which == 2 && (r & 1) == 1);
            hipLaunchKernelGGL(fhh::k_gap_probe, dim3(one ? 1 : 256), dim3(1024), big ? 131072 : 4096, st, out,
                               (uint32_t)r);
        }
        if (graph) {
            if (hipStreamEndCapture(st, &g) != hipSuccess) break;
            const hipError_t ge = hipGraphInstantiate(&gexec, g, nullptr, nullptr, 0);
            (void)hipGraphDestroy(g);
            if (ge != hipSuccess) break;
            (void)hipGraphLaunch(gexec, st);   // warm-up replay; pass 1 times the next one
            (void)hipStreamSynchronize(st);
            continue;
        }
        (void)hipEventRecord(b, st);
        if (hipEventSynchronize(b) != hipSuccess) break;
        (void)hipEventElapsedTime(&ms, a, b);
    }
    if (gexec) (void)hipGraphExecDestroy(gexec);
    const hipError_t e = hipGetLastError();
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipStreamDestroy(st);
    (void)hipFree(out);
    if (e != hipSuccess) return FHH_E_HIP;
    *us_per_kernel = ms * 1e3 / reps;
    return FHH_OK;
}

extern "C" int fhh_microbench(int device, int which, double* rate) {
    if (!rate) return FHH_E_ARG;
    if (hipSetDevice(device) != hipSuccess) return FHH_E_HIP;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return FHH_E_HIP;
    uint32_t* out = nullptr;
    if (hipMalloc(&out, 4) != hipSuccess) return FHH_E_NOMEM;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int threads = 256;
    double ops = 0;
    float ms = 0.f;
    for (int rep = 0; rep < 2; rep++) {   // first pass warms clocks
        if (which == 0 || which >= 2) {
            // 0: v_xor_b32, 8 waves/SIMD; 2: v_bitop3_b32, 8 waves/SIMD;
            // 3: v_bitop3_b32, 2 waves/SIMD; 4: v_xor_b32, 2 waves/SIMD
            const int wps = (which == 3 || which == 4 || which == 10) ? 2 : (which == 6 ? 4 : 8);
            const int blocks = cus * wps;   // 256-thread blocks = 4 waves = one per SIMD
            const uint32_t iters = 4096;
            (void)hipEventRecord(a, 0);
            if (which == 7)
                hipLaunchKernelGGL(fhh::k_valu_op_peak<0>, dim3(blocks), dim3(threads), 0, 0, out, iters, 7u);
            else if (which == 8)
                hipLaunchKernelGGL(fhh::k_valu_op_peak<1>, dim3(blocks), dim3(threads), 0, 0, out, iters, 7u);
            else if (which == 11)
                hipLaunchKernelGGL(fhh::k_valu_op_peak<2>, dim3(blocks), dim3(threads), 0, 0, out, iters, 7u);
            else if (which == 12)
                hipLaunchKernelGGL(fhh::k_valu_op_peak<3>, dim3(blocks), dim3(threads), 0, 0, out, iters, 7u);
            else if (which == 9 || which == 10)
                hipLaunchKernelGGL(fhh::k_chacha_peak, dim3(blocks), dim3(threads), 0, 0, out, iters / 8, 7u);
            else if (which == 0 || which == 4)
                hipLaunchKernelGGL(fhh::k_valu_peak, dim3(blocks), dim3(threads), 0, 0, out, iters, 7u);
            else if (which == 5 || which == 6)
                hipLaunchKernelGGL(fhh::k_mad64_peak, dim3(blocks), dim3(threads), 0, 0, out, iters, 7u);
            else
                hipLaunchKernelGGL(fhh::k_bitop3_peak, dim3(blocks), dim3(threads), 0, 0, out, iters, 7u);
            (void)hipEventRecord(b, 0);
            ops = (double)blocks * threads * iters * 8 * 16;
            if (which == 9 || which == 10) ops = (double)blocks * threads * (iters / 8) * 2 * 8 * 12;
        } else {
            const int blocks = cus * 2;   // 64 KiB LDS -> 2 blocks/CU of 512 threads (as k_expand)
            const uint32_t iters = 8192;
            (void)hipEventRecord(a, 0);
            hipLaunchKernelGGL(fhh::k_lds_peak, dim3(blocks), dim3(512), 0, 0, out, iters);
            (void)hipEventRecord(b, 0);
            ops = (double)blocks * 512 * iters * 8 * 4;   // bytes
        }
        if (hipEventSynchronize(b) != hipSuccess) {
            (void)hipFree(out);
            return FHH_E_HIP;
        }
        (void)hipEventElapsedTime(&ms, a, b);
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipFree(out);
    *rate = ops / (ms * 1e-3);
    return FHH_OK;
}

// Lookup throughput of the LDS and vector-memory gather paths, alone and mixed
// (k_gather_mix<NL, NG>): combo 0..8 = (NL, NG) in the table below; gbytes = global table
// span (256 .. 65536). rate = lookups per second over the chip (both paths).
extern "C" int fhh_microbench_gather(int device, int combo, uint32_t gbytes, double* rate) {
    static const int kCombos[][2] = {{8, 0}, {0, 8}, {0, 16}, {8, 1}, {8, 2}, {8, 4}, {6, 2}, {4, 4}, {12, 2}};
    if (!rate || combo < 0 || combo >= (int)(sizeof kCombos / sizeof kCombos[0]) || gbytes < 256 ||
        gbytes > 65536 || (gbytes & (gbytes - 1)))
        return FHH_E_ARG;
    if (hipSetDevice(device) != hipSuccess) return FHH_E_HIP;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return FHH_E_HIP;
    uint32_t* out = nullptr;
    uint32_t* g = nullptr;
    if (hipMalloc(&out, 4) != hipSuccess) return FHH_E_NOMEM;
    if (hipMalloc(&g, 65536) != hipSuccess) {
        (void)hipFree(out);
        return FHH_E_NOMEM;
    }
    {
        uint32_t h[16384];
        for (uint32_t i = 0; i < 16384; i++) h[i] = i * 2654435761u + 12345u;
        (void)hipMemcpy(g, h, sizeof h, hipMemcpyHostToDevice);
    }
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const int nl = kCombos[combo][0], ng = kCombos[combo][1];
    const uint32_t gmask = gbytes / 4 - 1;
    const int blocks = cus * 2;
    const uint32_t iters = 4096;
    float ms = 0.f;
    hipError_t e = hipSuccess;
    for (int rep = 0; rep < 3 && e == hipSuccess; rep++) {
        (void)hipEventRecord(a, 0);
#define FHH_GM(L, G) \
    if (nl == L && ng == G) hipLaunchKernelGGL((fhh::k_gather_mix<L, G>), dim3(blocks), dim3(512), 0, 0, g, gmask, out, iters);
        FHH_GM(8, 0) FHH_GM(0, 8) FHH_GM(0, 16) FHH_GM(8, 1) FHH_GM(8, 2) FHH_GM(8, 4) FHH_GM(6, 2) FHH_GM(4, 4)
        FHH_GM(12, 2)
#undef FHH_GM
        (void)hipEventRecord(b, 0);
        e = hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
    }
    if (e == hipSuccess) e = hipGetLastError();
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipFree(out);
    (void)hipFree(g);
    if (e != hipSuccess) return FHH_E_HIP;
    *rate = (double)blocks * 512 * iters * (nl + ng) / (ms * 1e-3);
    return FHH_OK;
}

// k_hybrid_mix with nb VALU-only waves (0, 2, 4, 6, 8) per 16-wave workgroup; rates[0] =
// LDS lookups/s, rates[1] = v_bitop3 lane-ops/s, chip-wide, over the kernel time.
extern "C" int fhh_microbench_hybrid(int device, int nb, double* rates) {
    if (!rates || (nb != 0 && nb != 2 && nb != 4 && nb != 6 && nb != 8)) return FHH_E_ARG;
    if (hipSetDevice(device) != hipSuccess) return FHH_E_HIP;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) return FHH_E_HIP;
    unsigned long long* c = nullptr;
    if (hipMalloc(&c, 32) != hipSuccess) return FHH_E_NOMEM;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const uint32_t iters = 8192;
    float ms = 0.f;
    unsigned long long h[4] = {0, 0, 0, 0};
    hipError_t e = hipSuccess;
    for (int rep = 0; rep < 3 && e == hipSuccess; rep++) {
        (void)hipMemset(c, 0, 32);
        (void)hipEventRecord(a, 0);
#define FHH_HM(N) \
    if (nb == N) hipLaunchKernelGGL((fhh::k_hybrid_mix<N>), dim3(cus), dim3(1024), 0, 0, c, iters);
        FHH_HM(0) FHH_HM(2) FHH_HM(4) FHH_HM(6) FHH_HM(8)
#undef FHH_HM
        (void)hipEventRecord(b, 0);
        e = hipEventSynchronize(b);
        (void)hipEventElapsedTime(&ms, a, b);
        if (e == hipSuccess) e = hipMemcpy(h, c, 32, hipMemcpyDeviceToHost);
    }
    if (e == hipSuccess) e = hipGetLastError();
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipFree(c);
    if (e != hipSuccess) return FHH_E_HIP;
    rates[0] = (double)h[0] / (ms * 1e-3);
    rates[1] = (double)h[1] / (ms * 1e-3);
    return FHH_OK;
}
