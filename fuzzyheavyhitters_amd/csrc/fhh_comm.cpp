// Native RCCL communicator for client-sharded multi-GPU crawls (include/fhh.h).
//
// The reference moves per-child sums as an RPC of Vec<FE> from each server to the leader
// once per level (collect.rs:487-501, leader.rs:182-197). Sharding clients over G GPUs turns
// the per-server sum into a sum over ranks as well: one ncclAllReduce(sum, u64) of the
// per-child 32-bit-limb partials (≤ C x 16 u64, a few tens of KB — latency bound over xGMI),
// enqueued on the engine's stream between the child kernel and k_prune.
//
// RCCL is dlopen'ed instead of linked: a PyTorch process already carries its own librccl,
// and reusing that instance (RTLD_NOLOAD first) avoids two RCCL runtimes in one process.
#include "fhh_internal.h"
#include "../../include/fhh.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

struct fhh_comm {
    ncclComm_t comm = nullptr;
    int nranks = 0, rank = 0, device = 0;
    // set once by comm_abort (ncclCommAbort freed the communicator; `comm` itself is left in place
    // so a peer thread inside comm_allreduce never sees it change)
    std::atomic<bool> aborted{false};
    // threads between their `aborted` check and the return of their ncclAllReduce: comm_abort waits
    // for them (briefly) so no thread can pass the check and then enqueue on a freed communicator
    std::atomic<int> inflight{0};
    // hosted communicator (fhh_comm_create_hosted): the same cfg->comm code path of the level
    // loop, with the sum done by a host callback instead of RCCL (tests without RCCL ranks)
    fhh_allreduce_fn hosted = nullptr;
    void* hosted_user = nullptr;
    std::vector<uint64_t> host_buf;
};

namespace {

thread_local std::string g_comm_err;

struct Rccl {
    void* handle = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclCommCount) comm_count = nullptr;
    decltype(&ncclCommUserRank) comm_user_rank = nullptr;
    // in-process communicators (one KeyCollection over several GPUs, fhh_group.cpp)
    decltype(&ncclCommInitAll) comm_init_all = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclCommAbort) comm_abort = nullptr;
};

Rccl g_rccl;
std::mutex g_rccl_mu;

int fail(int code, const std::string& msg) {
    g_comm_err = msg;
    return code;
}

int nccl_fail(ncclResult_t r, const char* what) {
    std::string m = std::string(what) + ": ";
    m += g_rccl.error_string ? g_rccl.error_string(r) : "rccl error";
    return fail(FHH_E_COMM, m);
}

int load_locked(const char* path) {
    if (g_rccl.handle) return FHH_OK;
    void* h = nullptr;
    if (path && *path) {
        // an explicit library (a chosen RCCL build, or tests/stubs/librccl_stub.so): resolved through
        // its own handle only, so it never interposes on the process's other nccl* users
        h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    } else {
        for (const char* name : {"librccl.so", "librccl.so.1"}) {
            h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);   // already in the process (e.g. torch's)
            if (h) break;
        }
        if (!h)
            for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
                h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
                if (h) break;
            }
    }
    if (!h) return fail(FHH_E_COMM, std::string("dlopen librccl failed: ") + (dlerror() ? dlerror() : "?"));
    Rccl r;
    r.handle = h;
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
    r.comm_count = reinterpret_cast<decltype(r.comm_count)>(dlsym(h, "ncclCommCount"));
    r.comm_user_rank = reinterpret_cast<decltype(r.comm_user_rank)>(dlsym(h, "ncclCommUserRank"));
    r.comm_init_all = reinterpret_cast<decltype(r.comm_init_all)>(dlsym(h, "ncclCommInitAll"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
    r.comm_abort = reinterpret_cast<decltype(r.comm_abort)>(dlsym(h, "ncclCommAbort"));
    if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_reduce || !r.error_string ||
        !r.comm_count || !r.comm_user_rank || !r.comm_init_all || !r.group_start || !r.group_end || !r.comm_abort)
        return fail(FHH_E_COMM, "librccl lacks an expected symbol");
    g_rccl = r;
    return FHH_OK;
}

int ensure_loaded() {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    return load_locked(nullptr);
}

}  // namespace

namespace fhh {

int comm_allreduce(fhh_comm* c, const uint64_t* send, uint64_t* recv, uint64_t count, hipStream_t stream,
                   std::string* err) {
    if (c->hosted) {
        // stream order: wait for the partials, sum on the host, put the result back before the
        // host returns to enqueue the consumers (blocking copies after the stream drained)
        c->host_buf.resize(count);
        if (hipStreamSynchronize(stream) != hipSuccess ||
            hipMemcpy(c->host_buf.data(), send, count * 8, hipMemcpyDeviceToHost) != hipSuccess) {
            if (err) *err = "hosted comm: device to host copy failed";
            return FHH_E_HIP;
        }
        if (c->hosted(c->host_buf.data(), count, c->hosted_user) != 0) {
            if (err) *err = "hosted comm: all-reduce callback failed";
            return FHH_E_CALLBACK;
        }
        if (hipMemcpy(recv, c->host_buf.data(), count * 8, hipMemcpyHostToDevice) != hipSuccess) {
            if (err) *err = "hosted comm: host to device copy failed";
            return FHH_E_HIP;
        }
        return FHH_OK;
    }
    // increment before the check, so an abort that set `aborted` after this thread's check sees it
    // in flight and waits for the enqueue to return (check-then-use race)
    c->inflight.fetch_add(1);
    if (c->aborted.load()) {
        c->inflight.fetch_sub(1);
        if (err) *err = "ncclAllReduce: communicator aborted by a failing peer";
        return FHH_E_COMM;
    }
    const ncclResult_t r = g_rccl.all_reduce(send, recv, count, ncclUint64, ncclSum, c->comm, stream);
    c->inflight.fetch_sub(1);
    if (r != ncclSuccess) {
        if (err) *err = std::string("ncclAllReduce: ") + g_rccl.error_string(r);
        return FHH_E_COMM;
    }
    return FHH_OK;
}

// One process driving several GPUs (fhh_create_multi): ncclCommInitAll over the shards' devices,
// which must be distinct (RCCL refuses two ranks on one GPU: "Duplicate GPU detected").
int comm_init_all(int n, const int* devices, std::vector<::fhh_comm*>& out, std::string* err) {
    out.clear();
    if (ensure_loaded()) {
        if (err) *err = g_comm_err;
        return FHH_E_COMM;
    }
    std::vector<ncclComm_t> comms((size_t)n, nullptr);
    const ncclResult_t r = g_rccl.comm_init_all(comms.data(), n, devices);
    if (r != ncclSuccess) {
        if (err) *err = std::string("ncclCommInitAll: ") + g_rccl.error_string(r);
        return FHH_E_COMM;
    }
    for (int k = 0; k < n; k++) {
        auto* c = new ::fhh_comm();
        c->comm = comms[(size_t)k];
        c->nranks = n;
        c->rank = k;
        c->device = devices[k];
        out.push_back(c);
    }
    return FHH_OK;
}

// The same all-reduce on every in-process communicator (each on its shard's stream), fused in
// one ncclGroupStart / ncclGroupEnd: one host thread issues all ranks' halves.
int comm_group_allreduce(const std::vector<::fhh_comm*>& comms, const std::vector<uint64_t*>& bufs, uint64_t count,
                         const std::vector<hipStream_t>& streams, std::string* err) {
    ncclResult_t r = g_rccl.group_start();
    if (r != ncclSuccess) {
        if (err) *err = std::string("ncclGroupStart: ") + g_rccl.error_string(r);
        return FHH_E_COMM;
    }
    for (size_t k = 0; k < comms.size(); k++) {
        if (hipSetDevice(comms[k]->device) != hipSuccess) {
            (void)g_rccl.group_end();
            if (err) *err = "hipSetDevice failed";
            return FHH_E_HIP;
        }
        r = g_rccl.all_reduce(bufs[k], bufs[k], count, ncclUint64, ncclSum, comms[k]->comm, streams[k]);
        if (r != ncclSuccess) {
            (void)g_rccl.group_end();
            if (err) *err = std::string("ncclAllReduce: ") + g_rccl.error_string(r);
            return FHH_E_COMM;
        }
    }
    r = g_rccl.group_end();
    if (r != ncclSuccess) {
        if (err) *err = std::string("ncclGroupEnd: ") + g_rccl.error_string(r);
        return FHH_E_COMM;
    }
    return FHH_OK;
}

// Unblock peers stuck in a collective after one shard failed (RCCL comms: ncclCommAbort; hosted
// comms: the thread reducer's abort flag, see ThreadReducer).
void comm_abort(::fhh_comm* c) {
    if (!c || !c->comm || !g_rccl.comm_abort) return;
    if (c->aborted.exchange(true)) return;   // another thread got here first
    // an enqueue that passed its check returns promptly; one still inside after 100 ms is blocked in
    // the collective itself (a peer never arrived), which is what ncclCommAbort exists to release
    const auto t0 = std::chrono::steady_clock::now();
    while (c->inflight.load() > 0 && std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(100))
        std::this_thread::yield();
    (void)hipSetDevice(c->device);
    (void)g_rccl.comm_abort(c->comm);
}

int comm_rank(const ::fhh_comm* c) { return c ? c->rank : 0; }

}  // namespace fhh

extern "C" {

int fhh_rccl_load(const char* path) {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    return load_locked(path);
}

int fhh_comm_unique_id(uint8_t id[128]) {
    if (!id) return fail(FHH_E_ARG, "null id");
    int rc = ensure_loaded();
    if (rc) return rc;
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId u;
    const ncclResult_t r = g_rccl.get_unique_id(&u);
    if (r != ncclSuccess) return nccl_fail(r, "ncclGetUniqueId");
    std::memcpy(id, &u, 128);
    return FHH_OK;
}

int fhh_comm_create(fhh_comm** out, int nranks, int rank, const uint8_t id[128], int device) {
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(FHH_E_ARG, "bad comm arguments");
    *out = nullptr;
    int rc = ensure_loaded();
    if (rc) return rc;
    if (hipSetDevice(device) != hipSuccess) return fail(FHH_E_HIP, "hipSetDevice failed");
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    auto* c = new fhh_comm();
    const ncclResult_t r = g_rccl.comm_init_rank(&c->comm, nranks, u, rank);
    if (r != ncclSuccess) {
        delete c;
        return nccl_fail(r, "ncclCommInitRank");
    }
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    *out = c;
    return FHH_OK;
}

int fhh_comm_create_hosted(fhh_comm** out, int nranks, int rank, int device, fhh_allreduce_fn fn, void* user) {
    if (!out || !fn || nranks < 1 || rank < 0 || rank >= nranks) return fail(FHH_E_ARG, "bad hosted comm arguments");
    auto* c = new fhh_comm();
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    c->hosted = fn;
    c->hosted_user = user;
    *out = c;
    return FHH_OK;
}

void fhh_comm_destroy(fhh_comm* comm) {
    if (!comm) return;
    if (comm->comm && !comm->aborted.load() && g_rccl.comm_destroy) {
        (void)hipSetDevice(comm->device);
        (void)g_rccl.comm_destroy(comm->comm);
    }
    delete comm;
}

int fhh_comm_allreduce_u64(fhh_comm* comm, const uint64_t* send_dev, uint64_t* recv_dev, uint64_t count,
                           void* stream) {
    if (!comm || !send_dev || !recv_dev) return fail(FHH_E_ARG, "null comm or buffer");
    if (hipSetDevice(comm->device) != hipSuccess) return fail(FHH_E_HIP, "hipSetDevice failed");
    std::string err;
    const int rc = fhh::comm_allreduce(comm, send_dev, recv_dev, count, static_cast<hipStream_t>(stream), &err);
    if (rc) return fail(rc, err);
    return FHH_OK;
}

int fhh_comm_info(fhh_comm* comm, int* nranks, int* rank) {
    if (!comm || !nranks || !rank) return fail(FHH_E_ARG, "null comm or output");
    if (comm->hosted) {
        *nranks = comm->nranks;
        *rank = comm->rank;
        return FHH_OK;
    }
    ncclResult_t r = g_rccl.comm_count(comm->comm, nranks);
    if (r != ncclSuccess) return nccl_fail(r, "ncclCommCount");
    r = g_rccl.comm_user_rank(comm->comm, rank);
    if (r != ncclSuccess) return nccl_fail(r, "ncclCommUserRank");
    return FHH_OK;
}

const char* fhh_comm_last_error(void) { return g_comm_err.c_str(); }

}  // extern "C"
