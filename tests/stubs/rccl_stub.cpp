// TEST-ONLY stand-in for librccl (never part of the product; built by __graft_entry__.build() into
// tests/stubs/librccl_stub.so and loaded through fhh_rccl_load(path) by tests/test_rccl_stub.py).
//
// The in-process RCCL branch of a multi-device collection (fhh_comm.cpp comm_init_all /
// comm_group_allreduce / comm_abort, fhh_group.cpp) needs distinct GPUs with real RCCL, which a
// one-GPU box cannot give. This library implements the 11 entry points fhh_comm.cpp resolves, with
// RCCL's own signatures (rccl/rccl.h), so that branch runs unchanged on a repeated device: a clique of
// ncclCommInitAll communicators sums u64 buffers on the host —
//   * grouped calls (ncclGroupStart, one ncclAllReduce per communicator, ncclGroupEnd, issued by one
//     thread — fhh_group.cpp's node sums): at ncclGroupEnd every op's stream is drained, the buffers
//     summed, the sum copied back to every op's recv buffer;
//   * ungrouped calls (one thread per rank — the device level loop's per-level cfg->comm all-reduce):
//     a host rendezvous; each rank drains its stream, contributes, waits for the clique, copies back.
// ncclCommAbort marks the clique aborted and wakes every waiter, which returns ncclRemoteError (the
// abort path of a failing shard). FHH_RCCL_STUB_FAIL="rank:call" makes that rank's call-th ungrouped
// all-reduce fail (fault injection for the abort path). fhh_rccl_stub_stats reports what ran.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <set>
#include <string>
#include <vector>

namespace {

struct Clique {
    int n = 0;
    std::mutex mu;
    std::condition_variable cv;
    bool aborted = false;
    int arrived = 0;
    uint64_t gen = 0, count = 0;
    std::vector<uint64_t> acc, result;
};

struct Stats {
    std::atomic<uint64_t> init_all{0}, init_rank{0}, calls{0}, grouped{0}, group_ends{0}, aborts{0}, destroys{0},
        max_count{0}, failed{0};
    std::mutex mu;
    std::set<void*> streams;
} g_stats;

thread_local int t_group_depth = 0;
struct Op {
    const void* send;
    void* recv;
    size_t count;
    ncclComm_t comm;
    hipStream_t stream;
};
thread_local std::vector<Op> t_ops;

void note(size_t count, hipStream_t s) {
    uint64_t m = g_stats.max_count.load();
    while (count > m && !g_stats.max_count.compare_exchange_weak(m, count)) {
    }
    std::lock_guard<std::mutex> lk(g_stats.mu);
    g_stats.streams.insert((void*)s);
}

bool fail_now(int rank, uint64_t call) {
    const char* e = std::getenv("FHH_RCCL_STUB_FAIL");
    if (!e) return false;
    int r = -1;
    unsigned long long c = 0;
    if (std::sscanf(e, "%d:%llu", &r, &c) != 2) return false;
    return r == rank && c == call;
}

}  // namespace

struct ncclComm {
    Clique* cl = nullptr;
    int rank = 0, device = 0;
    uint64_t calls = 0;
};

extern "C" {

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "stub: success";
        case ncclInvalidArgument: return "stub: invalid argument";
        case ncclInvalidUsage: return "stub: invalid usage";
        case ncclRemoteError: return "stub: a peer aborted the communicator";
        case ncclSystemError: return "stub: injected failure (FHH_RCCL_STUB_FAIL)";
        default: return "stub: error";
    }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    std::memset(id, 0x5A, sizeof(*id));
    return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist) {
    if (!comms || ndev < 1) return ncclInvalidArgument;
    auto* cl = new Clique();
    cl->n = ndev;
    for (int k = 0; k < ndev; k++) {
        auto* c = new ncclComm();
        c->cl = cl;
        c->rank = k;
        c->device = devlist ? devlist[k] : k;
        comms[k] = c;
    }
    g_stats.init_all++;
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId, int rank) {
    // multi-process ranks need a transport this stand-in does not have
    if (!comm || nranks != 1 || rank != 0) return ncclInvalidUsage;
    int dev = 0;
    (void)hipGetDevice(&dev);
    g_stats.init_rank++;
    return ncclCommInitAll(comm, 1, &dev);
}

ncclResult_t ncclCommCount(const ncclComm_t comm, int* count) {
    if (!comm || !count) return ncclInvalidArgument;
    *count = comm->cl->n;
    return ncclSuccess;
}

ncclResult_t ncclCommUserRank(const ncclComm_t comm, int* rank) {
    if (!comm || !rank) return ncclInvalidArgument;
    *rank = comm->rank;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    if (!comm) return ncclInvalidArgument;
    g_stats.destroys++;
    delete comm;   // the clique is left to the process (every rank's comm points at it)
    return ncclSuccess;
}

ncclResult_t ncclCommAbort(ncclComm_t comm) {
    if (!comm) return ncclInvalidArgument;
    g_stats.aborts++;
    {
        std::lock_guard<std::mutex> lk(comm->cl->mu);
        comm->cl->aborted = true;
    }
    comm->cl->cv.notify_all();
    return ncclSuccess;   // the comm object stays valid (fhh_comm_destroy skips an aborted comm)
}

ncclResult_t ncclGroupStart() {
    t_group_depth++;
    return ncclSuccess;
}

ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype, ncclRedOp_t op,
                           ncclComm_t comm, hipStream_t stream) {
    if (!comm || datatype != ncclUint64 || op != ncclSum) return ncclInvalidArgument;
    g_stats.calls++;
    note(count, stream);
    if (t_group_depth > 0) {   // collected; summed at ncclGroupEnd
        g_stats.grouped++;
        t_ops.push_back(Op{sendbuff, recvbuff, count, comm, stream});
        return ncclSuccess;
    }
    Clique* cl = comm->cl;
    if (fail_now(comm->rank, comm->calls++)) {
        g_stats.failed++;
        return ncclSystemError;
    }
    std::vector<uint64_t> h(count);
    if (hipSetDevice(comm->device) != hipSuccess || hipStreamSynchronize(stream) != hipSuccess ||
        (count && hipMemcpy(h.data(), sendbuff, count * 8, hipMemcpyDeviceToHost) != hipSuccess))
        return ncclUnhandledCudaError;
    std::unique_lock<std::mutex> lk(cl->mu);
    if (cl->aborted) return ncclRemoteError;
    if (cl->arrived == 0) {
        cl->acc = h;
        cl->count = count;
    } else {
        if (count != cl->count) return ncclInvalidUsage;
        for (size_t i = 0; i < count; i++) cl->acc[i] += h[i];
    }
    const uint64_t my = cl->gen;
    if (++cl->arrived == cl->n) {
        cl->result = cl->acc;
        cl->arrived = 0;
        cl->gen++;
        cl->cv.notify_all();
    } else {
        cl->cv.wait(lk, [&] { return cl->gen != my || cl->aborted; });
        if (cl->gen == my) return ncclRemoteError;   // aborted while waiting
    }
    h = cl->result;
    lk.unlock();
    if (count && hipMemcpy(recvbuff, h.data(), count * 8, hipMemcpyHostToDevice) != hipSuccess)
        return ncclUnhandledCudaError;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (t_group_depth <= 0) return ncclInvalidUsage;
    if (--t_group_depth > 0) return ncclSuccess;
    g_stats.group_ends++;
    std::vector<Op> ops;
    ops.swap(t_ops);
    if (ops.empty()) return ncclSuccess;
    Clique* cl = ops[0].comm->cl;
    if ((int)ops.size() != cl->n) return ncclInvalidUsage;   // one op per rank of one clique
    {
        std::lock_guard<std::mutex> lk(cl->mu);
        if (cl->aborted) return ncclRemoteError;
    }
    const size_t count = ops[0].count;
    std::vector<uint64_t> acc(count, 0), h(count);
    for (const Op& o : ops) {
        if (o.comm->cl != cl || o.count != count) return ncclInvalidUsage;
        if (hipSetDevice(o.comm->device) != hipSuccess || hipStreamSynchronize(o.stream) != hipSuccess ||
            (count && hipMemcpy(h.data(), o.send, count * 8, hipMemcpyDeviceToHost) != hipSuccess))
            return ncclUnhandledCudaError;
        for (size_t i = 0; i < count; i++) acc[i] += h[i];
    }
    for (const Op& o : ops)
        if (hipSetDevice(o.comm->device) != hipSuccess ||
            (count && hipMemcpy(o.recv, acc.data(), count * 8, hipMemcpyHostToDevice) != hipSuccess))
            return ncclUnhandledCudaError;
    return ncclSuccess;
}

// what ran: [ncclCommInitAll, ncclCommInitRank, ncclAllReduce calls, grouped ones, ncclGroupEnd,
// ncclCommAbort, ncclCommDestroy, largest count, distinct streams, injected failures]
int fhh_rccl_stub_stats(uint64_t out[10]) {
    out[0] = g_stats.init_all;
    out[1] = g_stats.init_rank;
    out[2] = g_stats.calls;
    out[3] = g_stats.grouped;
    out[4] = g_stats.group_ends;
    out[5] = g_stats.aborts;
    out[6] = g_stats.destroys;
    out[7] = g_stats.max_count;
    {
        std::lock_guard<std::mutex> lk(g_stats.mu);
        out[8] = g_stats.streams.size();
    }
    out[9] = g_stats.failed;
    return 0;
}

}  // extern "C"
