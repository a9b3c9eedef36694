// comm.hip -- the one per-control-step collective of a candidate-sharded get_action, owned by the
// library (include/bcmpc.h, bcmpc_comm_*).
//
// The K candidates of a control step are independent rollouts of one state (controllers.py:63-71);
// the only cross-candidate operation is np.argmin (controllers.py:82).  Each rank (one process per
// GPU) runs its contiguous shard; its argmin launch leaves a 144-byte bcmpc_result (global index,
// f64 cost, f64 first action).  With a communicator attached to the engine, the same stream then
// runs ONE RCCL all-gather of those records over xGMI and a one-wave kernel that applies
// np.argmin's rule to them (NaN first, smaller cost, lowest global index on ties; np.argmax for the
// learned reward), so every rank's d_result holds the global answer before anything returns to the
// host.  An exact min-loc needs the f64 cost and the index (128 bits), more than a 64-bit
// all-reduce(MIN) key holds without rounding the cost -- hence an all-gather of tiny records
// (latency-bound: 144 B x N), not an all-reduce.  The reference's only collective
// (train_mpc_ppo.py:388, an mpi4py allgather of episode statistics) is not on this path.
//
// RCCL is loaded with dlopen on first use (librccl.so.1: the copy PyTorch-ROCm already mapped when
// present, else /opt/rocm's), so libbcmpc itself has no link-time dependency on it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdint.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <string>
#include <thread>

#include "../../include/bcmpc.h"
#include "kernels.h"

namespace bcmpc {

namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclCommAbort) abort = nullptr;
    decltype(&ncclCommGetAsyncError) async_error = nullptr;
    std::string error;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            r.error = std::string("cannot load librccl.so.1: ") + dlerror();
            return;
        }
        r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
        r.init_rank = reinterpret_cast<decltype(r.init_rank)>(dlsym(h, "ncclCommInitRank"));
        r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(h, "ncclCommDestroy"));
        r.all_gather = reinterpret_cast<decltype(r.all_gather)>(dlsym(h, "ncclAllGather"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
        r.abort = reinterpret_cast<decltype(r.abort)>(dlsym(h, "ncclCommAbort"));
        r.async_error = reinterpret_cast<decltype(r.async_error)>(dlsym(h, "ncclCommGetAsyncError"));
        if (!r.get_unique_id || !r.init_rank || !r.destroy || !r.all_gather || !r.error_string || !r.abort ||
            !r.async_error)
            r.error = "librccl.so.1 lacks an expected symbol";
    });
    return r;
}

// np.argmin order on result records (cost already sign-flipped for argmax)
__host__ __device__ inline bool record_better(double ca, int64_t ia, double cb, int64_t ib) {
    const bool an = ca != ca, bn = cb != cb;
    if (an != bn) return an;
    if (!an && ca != cb) return ca < cb;
    return ia < ib;
}

__host__ __device__ inline int select_index(const bcmpc_result* r, int n, int maximize) {
    const double sg = maximize ? -1.0 : 1.0;
    int best = 0;
    for (int k = 1; k < n; ++k)
        if (record_better(sg * r[k].best_cost, r[k].best_index, sg * r[best].best_cost, r[best].best_index)) best = k;
    return best;
}

// one wave: d_out = the best of n gathered records (n is the communicator size: a handful)
__global__ __launch_bounds__(64) void select_records_kernel(const bcmpc_result* __restrict__ recs, int n,
                                                           int maximize, bcmpc_result* __restrict__ out) {
    const int best = select_index(recs, n, maximize);
    const uint64_t* src = reinterpret_cast<const uint64_t*>(recs + best);
    uint64_t* dst = reinterpret_cast<uint64_t*>(out);
    constexpr int kWords = sizeof(bcmpc_result) / sizeof(uint64_t);
    for (int w = threadIdx.x; w < kWords; w += 64) dst[w] = src[w];
}

// What travels in the exchange: the rank's result record plus its status flags (bit 0: this rank's
// team kernel gave up, so its record is not a result).  Every rank sees every flag, so every rank
// takes the same decision: select, or rerun the step together on the fallback engines.
struct WireRecord {
    bcmpc_result r;
    uint32_t flags;
    uint32_t pad[3];
};
static_assert(sizeof(WireRecord) % 16 == 0, "wire record");

// one wave: the rank's record and its team error word (mapped host memory, written by the team
// kernel earlier on this stream) into the send slot
__global__ __launch_bounds__(64) void pack_wire_kernel(const bcmpc_result* __restrict__ res,
                                                       const unsigned* team_err, unsigned force,
                                                       WireRecord* __restrict__ wire) {
    const uint64_t* src = reinterpret_cast<const uint64_t*>(res);
    uint64_t* dst = reinterpret_cast<uint64_t*>(&wire->r);
    constexpr int kWords = sizeof(bcmpc_result) / sizeof(uint64_t);
    for (int w = threadIdx.x; w < kWords; w += 64) dst[w] = src[w];
    if (threadIdx.x == 0) {
        const unsigned f = team_err ? __hip_atomic_load(team_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
        wire->flags = (f || force) ? 1u : 0u;
        wire->pad[0] = wire->pad[1] = wire->pad[2] = 0u;
    }
}

// one wave: np.argmin's rule over the n gathered records (valid ones; all are valid unless a flag is
// set), and the OR of every rank's flags into the mapped word the host reads after the stream
__global__ __launch_bounds__(64) void select_wire_kernel(const WireRecord* __restrict__ recs, int n, int maximize,
                                                         bcmpc_result* __restrict__ out, unsigned* any_flags) {
    const double sg = maximize ? -1.0 : 1.0;
    int best = 0;
    unsigned f = recs[0].flags;
    for (int k = 1; k < n; ++k) {
        f |= recs[k].flags;
        if (record_better(sg * recs[k].r.best_cost, recs[k].r.best_index, sg * recs[best].r.best_cost,
                          recs[best].r.best_index))
            best = k;
    }
    const uint64_t* src = reinterpret_cast<const uint64_t*>(&recs[best].r);
    uint64_t* dst = reinterpret_cast<uint64_t*>(out);
    constexpr int kWords = sizeof(bcmpc_result) / sizeof(uint64_t);
    for (int w = threadIdx.x; w < kWords; w += 64) dst[w] = src[w];
    if (threadIdx.x == 0) __hip_atomic_store(any_flags, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int comm_fail(int code, const std::string& msg) { return set_error(code, msg); }   // -> bcmpc_last_error()

// the exchange's select (also bcmpc_select_results_async): "" or the launch error
std::string launch_select_records(const bcmpc_result* recs, int n, int maximize, bcmpc_result* out, hipStream_t st) {
    hipLaunchKernelGGL(select_records_kernel, dim3(1), dim3(64), 0, st, recs, n, maximize, out);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? std::string() : std::string("select_records_kernel: ") + hipGetErrorString(e);
}

}  // namespace

}  // namespace bcmpc

struct bcmpc_comm {
    ncclComm_t nccl = nullptr;
    int nranks = 0, rank = 0, device = 0;
    bcmpc::WireRecord* d_send = nullptr;     // this rank's record + flags
    bcmpc::WireRecord* d_gather = nullptr;   // [nranks]
    unsigned* h_flags = nullptr;             // mapped: OR of every rank's flags of the last exchange
    unsigned* d_flags = nullptr;
    bool aborted = false;                    // ncclCommAbort'ed after a timed-out exchange
    int force_flags = 0;                     // (test hook, BCMPC_COMM_FORCE_FLAGS=n: the first n exchanges carry
                                             //  a set flag, as if another rank's team had given up)
};

namespace bcmpc {

// enqueue the exchange after the argmin launch: pack (record + this rank's team status), all-gather
// every rank's, select in place (+ the OR of the flags into the mapped word comm_any_flags reads)
int comm_exchange(bcmpc_comm* c, bcmpc_result* d_result, int maximize, hipStream_t st, std::string* err,
                  const unsigned* d_team_err) {
    if (c->aborted) {
        *err = "the communicator was aborted after an exchange timed out; create a new one";
        return BCMPC_ERR_STATE;
    }
    const Rccl& r = rccl();
    const unsigned force = c->force_flags > 0 ? 1u : 0u;
    if (c->force_flags > 0) --c->force_flags;
    hipLaunchKernelGGL(pack_wire_kernel, dim3(1), dim3(64), 0, st, d_result, d_team_err, force, c->d_send);
    if (hipGetLastError() != hipSuccess) {
        *err = "pack_wire_kernel launch failed";
        return BCMPC_ERR_HIP;
    }
    const ncclResult_t rc = r.all_gather(c->d_send, c->d_gather, sizeof(WireRecord), ncclUint8, c->nccl, st);
    if (rc != ncclSuccess) {
        *err = std::string("ncclAllGather: ") + r.error_string(rc);
        return BCMPC_ERR_HIP;
    }
    hipLaunchKernelGGL(select_wire_kernel, dim3(1), dim3(64), 0, st, c->d_gather, c->nranks, maximize, d_result,
                       c->d_flags);
    if (hipGetLastError() != hipSuccess) {
        *err = "select_wire_kernel launch failed";
        return BCMPC_ERR_HIP;
    }
    return BCMPC_OK;
}

// after the stream has completed: did any rank flag its record (a team that gave up)?  Cleared here.
bool comm_any_flags(bcmpc_comm* c) {
    const unsigned f = __atomic_load_n(c->h_flags, __ATOMIC_ACQUIRE);
    __atomic_store_n(c->h_flags, 0u, __ATOMIC_RELEASE);
    return f != 0;
}

// Bounded wait for a stream whose work includes this communicator's exchange.  A rank that never joins
// (crashed, or stuck in a collective of its own) would otherwise hold every other rank in
// hipStreamSynchronize forever: poll the stream and RCCL's asynchronous error, and after timeout_ms
// abort the communicator (ncclCommAbort ends its pending collectives) and report.  The communicator is
// unusable afterwards (every later exchange fails with BCMPC_ERR_STATE).
// Polls back to back (yielding the core) for the first 2 ms, which covers every control step, then sleeps
// 50 us between polls: a sleep request of a few microseconds already costs ~50-60 us of timer slack, so a
// poll that slept would add up to that to the completion of any step longer than the tight-poll window.
int comm_wait(bcmpc_comm* c, hipStream_t st, int64_t timeout_ms, std::string* err) {
    const Rccl& r = rccl();
    const auto t0 = std::chrono::steady_clock::now();
    bool tight = true;
    for (uint32_t i = 0;; ++i) {
        const hipError_t q = hipStreamQuery(st);
        if (q == hipSuccess) return BCMPC_OK;
        if (q != hipErrorNotReady) {
            *err = std::string("exchange stream: ") + hipGetErrorString(q);
            return BCMPC_ERR_HIP;
        }
        if ((i & 63) == 0) {
            ncclResult_t ae = ncclSuccess;
            if (r.async_error(c->nccl, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
                *err = std::string("RCCL asynchronous error during the exchange: ") + r.error_string(ae);
                (void)r.abort(c->nccl);
                c->nccl = nullptr;
                c->aborted = true;
                return BCMPC_ERR_HIP;
            }
            const auto el = std::chrono::steady_clock::now() - t0;
            tight = el < std::chrono::milliseconds(2);
            if (el > std::chrono::milliseconds(timeout_ms)) {
                (void)r.abort(c->nccl);
                c->nccl = nullptr;
                c->aborted = true;
                (void)hipStreamSynchronize(st);           // (the aborted collective has returned)
                *err = "exchange timed out after " + std::to_string(timeout_ms) +
                       " ms (a rank did not join the all-gather); the communicator was aborted";
                return BCMPC_ERR_HIP;
            }
        }
        if (tight)
            std::this_thread::yield();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
}

int comm_rank(const bcmpc_comm* c) { return c->rank; }
int comm_size(const bcmpc_comm* c) { return c->nranks; }
int comm_device(const bcmpc_comm* c) { return c->device; }

}  // namespace bcmpc

extern "C" {

int bcmpc_comm_unique_id(uint8_t* id) {
    using namespace bcmpc;
    if (!id) return comm_fail(BCMPC_ERR_ARG, "null argument");
    const Rccl& r = rccl();
    if (!r.error.empty()) return comm_fail(BCMPC_ERR_UNSUPPORTED, r.error);
    ncclUniqueId u;
    const ncclResult_t rc = r.get_unique_id(&u);
    if (rc != ncclSuccess) return comm_fail(BCMPC_ERR_HIP, std::string("ncclGetUniqueId: ") + r.error_string(rc));
    static_assert(sizeof(u.internal) == BCMPC_COMM_ID_BYTES, "RCCL unique id size");
    std::memcpy(id, u.internal, BCMPC_COMM_ID_BYTES);
    return BCMPC_OK;
}

int bcmpc_comm_init(const uint8_t* id, int32_t nranks, int32_t rank, int32_t device, bcmpc_comm** out) {
    using namespace bcmpc;
    if (!id || !out) return comm_fail(BCMPC_ERR_ARG, "null argument");
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks) return comm_fail(BCMPC_ERR_ARG, "rank must be in [0, nranks)");
    const Rccl& r = rccl();
    if (!r.error.empty()) return comm_fail(BCMPC_ERR_UNSUPPORTED, r.error);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return comm_fail(BCMPC_ERR_ARG, "device ordinal out of range");
    if (hipSetDevice(device) != hipSuccess) return comm_fail(BCMPC_ERR_HIP, "hipSetDevice failed");
    bcmpc_comm* c = new bcmpc_comm();
    c->nranks = nranks; c->rank = rank; c->device = device;
    if (const char* v = std::getenv("BCMPC_COMM_FORCE_FLAGS")) {     // (test hook: announced on stderr)
        c->force_flags = std::max(0, std::atoi(v));
        announce_test_hook("BCMPC_COMM_FORCE_FLAGS", v);
    }
    auto release = [&]() {
        if (c->d_send) (void)hipFree(c->d_send);
        if (c->d_gather) (void)hipFree(c->d_gather);
        if (c->h_flags) (void)hipHostFree(c->h_flags);
        delete c;
    };
    if (hipMalloc(&c->d_send, sizeof(WireRecord)) != hipSuccess ||
        hipMalloc(&c->d_gather, (size_t)nranks * sizeof(WireRecord)) != hipSuccess ||
        hipHostMalloc(&c->h_flags, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&c->d_flags, c->h_flags, 0) != hipSuccess) {
        release();
        return comm_fail(BCMPC_ERR_HIP, "device allocation failed");
    }
    *c->h_flags = 0u;
    ncclUniqueId u;
    std::memcpy(u.internal, id, BCMPC_COMM_ID_BYTES);
    const ncclResult_t rc = r.init_rank(&c->nccl, nranks, u, rank);   // collective over the nranks
    if (rc != ncclSuccess) {
        release();
        return comm_fail(BCMPC_ERR_HIP, std::string("ncclCommInitRank: ") + r.error_string(rc));
    }
    *out = c;
    return BCMPC_OK;
}

int bcmpc_comm_destroy(bcmpc_comm* c) {
    using namespace bcmpc;
    if (!c) return BCMPC_OK;
    (void)hipSetDevice(c->device);
    if (c->nccl) (void)rccl().destroy(c->nccl);
    if (c->d_send) (void)hipFree(c->d_send);
    if (c->d_gather) (void)hipFree(c->d_gather);
    if (c->h_flags) (void)hipHostFree(c->h_flags);
    delete c;
    return BCMPC_OK;
}

int bcmpc_select_results(const bcmpc_result* recs, int32_t n, int32_t maximize, bcmpc_result* out) {
    using namespace bcmpc;
    if (!recs || !out || n < 1) return comm_fail(BCMPC_ERR_ARG, "need n >= 1 records");
    *out = recs[select_index(recs, n, maximize)];
    return BCMPC_OK;
}

int bcmpc_select_results_async(const bcmpc_result* d_recs, int32_t n, int32_t maximize, bcmpc_result* d_out,
                               void* stream) {
    using namespace bcmpc;
    if (!d_recs || !d_out || n < 1 || n > 4096) return comm_fail(BCMPC_ERR_ARG, "need 1 <= n <= 4096 records");
    if (d_out + 1 > d_recs && d_out < d_recs + n) return comm_fail(BCMPC_ERR_ARG, "d_out overlaps d_recs");
    const std::string err = launch_select_records(d_recs, n, maximize, d_out, (hipStream_t)stream);
    if (!err.empty()) return comm_fail(BCMPC_ERR_HIP, err);
    return BCMPC_OK;
}

}  // extern "C"
