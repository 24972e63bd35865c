// The data-parallel gradient exchange issued from native code: one RCCL communicator per process over
// the ranks of the job (xGMI within the node), its own stream and two events, and SUM all-reduces of
// the flat gradient bucket / loss partials ordered against the caller's stream by events.  Replaces
// the per-minibatch torch.distributed calls (ProcessGroupNCCL: tens of us of host per collective, which
// made the dp-forced per-rank minibatch host-bound); the reference is single-process (SURVEY.md §2,
// the sharded step is ppo.py:241-244).
//
// RCCL is resolved at run time from the library the process already has loaded (torch's librccl.so:
// the caller passes its path), so one RCCL instance serves both torch's communicators and this one.
#include <dlfcn.h>

#include <cstring>

#include <rccl/rccl.h>

#include "common.h"

namespace {

struct Rccl {
    void* h = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
};

Rccl g_rccl;

struct DpComm {
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    // ready: the caller's point an asynchronous reduction starts after; done: the end of the last
    // asynchronous reduction; mark: the end of the last blocking one, recorded lazily on its stream when the
    // next reduction comes from another stream
    hipEvent_t ready = nullptr, done = nullptr, mark = nullptr;
    int world = 0, rank = 0, device = 0;
    // the stream the communicator's last reduction was ordered on (the caller's for a blocking one, the
    // communicator's own for an asynchronous one; null before the first): every reduction is ordered after
    // it, so the reductions run one at a time in issue order whichever streams issue them — the order every
    // rank issues them in (two RCCL kernels of one communicator running out of order could pair
    // different buffers across ranks, or deadlock)
    hipStream_t last = nullptr;
    bool inflight = false;  // an asynchronous reduction not yet waited for by a caller's stream
};

int rccl_fail(const char* what, ncclResult_t r) {
    ppox::set_error("%s: %s", what, g_rccl.error_string ? g_rccl.error_string(r) : "rccl error");
    return PPOX_EINVAL;
}

}  // namespace

extern "C" int ppox_dp_load(const char* rccl_path) {
    if (g_rccl.h) return PPOX_OK;
    PPOX_REQUIRE(rccl_path && rccl_path[0], "ppox_dp_load: no library path");
    void* h = dlopen(rccl_path, RTLD_NOW | RTLD_LOCAL);
    PPOX_REQUIRE(h, "ppox_dp_load: %s", dlerror());
    Rccl r;
    r.h = h;
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(dlsym(h, "ncclAllReduce"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
    PPOX_REQUIRE(r.get_unique_id && r.comm_init_rank && r.comm_destroy && r.all_reduce && r.error_string,
                 "ppox_dp_load: %s lacks the RCCL entry points", rccl_path);
    g_rccl = r;
    return PPOX_OK;
}

extern "C" int ppox_dp_unique_id_bytes(void) { return NCCL_UNIQUE_ID_BYTES; }

extern "C" int ppox_dp_unique_id(uint8_t* id_host) {
    PPOX_REQUIRE(g_rccl.h, "ppox_dp_unique_id: ppox_dp_load first");
    PPOX_REQUIRE(id_host, "ppox_dp_unique_id: null id");
    ncclUniqueId id;
    ncclResult_t r = g_rccl.get_unique_id(&id);
    if (r != ncclSuccess) return rccl_fail("ncclGetUniqueId", r);
    std::memcpy(id_host, id.internal, NCCL_UNIQUE_ID_BYTES);
    return PPOX_OK;
}

extern "C" int ppox_dp_comm_init(const uint8_t* id_host, int32_t world, int32_t rank, int32_t device, void** comm_out) {
    PPOX_REQUIRE(g_rccl.h, "ppox_dp_comm_init: ppox_dp_load first");
    PPOX_REQUIRE(id_host && comm_out, "ppox_dp_comm_init: null argument");
    PPOX_REQUIRE(world >= 1 && rank >= 0 && rank < world && device >= 0,
                 "ppox_dp_comm_init: rank %d of world %d on device %d", rank, world, device);
    *comm_out = nullptr;
    PPOX_HIP(hipSetDevice(device), "ppox_dp_comm_init");
    ncclUniqueId id;
    std::memcpy(id.internal, id_host, NCCL_UNIQUE_ID_BYTES);
    auto* c = new DpComm;
    c->world = world, c->rank = rank, c->device = device;
    ncclResult_t r = g_rccl.comm_init_rank(&c->comm, world, id, rank);
    if (r != ncclSuccess) {
        delete c;
        return rccl_fail("ncclCommInitRank", r);
    }
    // the exchange overlaps the conv backward (the fc + head bucket starts while the conv dgrads run).
    // HIP multiplexes the streams of one priority class over GPU_MAX_HW_QUEUES hardware queues, and two
    // streams on one queue run in order: a stream sharing the main stream's queue would hold the main
    // stream's later kernels behind its wait for the side stream (per-rank 196 -> 242 ms measured).  So
    // the stream is high-priority, the class of the backward's side stream (convs.side_stream), and the
    // main stream (the default stream) is not
    int lo = 0, hi = 0;
    hipDeviceGetStreamPriorityRange(&lo, &hi);
    hipError_t e = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ready, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->mark, hipEventDisableTiming);
    if (e != hipSuccess) {
        g_rccl.comm_destroy(c->comm);
        if (c->ready) hipEventDestroy(c->ready);
        if (c->done) hipEventDestroy(c->done);
        if (c->stream) hipStreamDestroy(c->stream);
        delete c;
        ppox::set_error("ppox_dp_comm_init: %s", hipGetErrorString(e));
        return -static_cast<int>(e);
    }
    *comm_out = c;
    return PPOX_OK;
}

// Waits for the communicator's work (its own stream and the last blocking reduction's stream), then
// destroys it.  Call before the process group and the HIP runtime go away: a communicator left alive to
// the exit-time destructors took a profiled run down with SIGSEGV in __cxa_finalize.
extern "C" int ppox_dp_comm_destroy(void* comm) {
    if (!comm) return PPOX_OK;
    auto* c = static_cast<DpComm*>(comm);
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e == hipSuccess && c->last && c->last != c->stream) e = hipStreamSynchronize(c->last);
    ncclResult_t r = g_rccl.comm_destroy(c->comm);
    hipEventDestroy(c->ready);
    hipEventDestroy(c->done);
    hipEventDestroy(c->mark);
    hipStreamDestroy(c->stream);
    delete c;
    if (e != hipSuccess) {
        ppox::set_error("ppox_dp_comm_destroy: %s", hipGetErrorString(e));
        return -static_cast<int>(e);
    }
    return r == ncclSuccess ? PPOX_OK : rccl_fail("ncclCommDestroy", r);
}

namespace {
// `s` waits for the communicator's last reduction (nothing when that was ordered on `s` itself)
hipError_t order_after_last(DpComm* c, hipStream_t s) {
    if (!c->last || c->last == s) return hipSuccess;
    if (c->last == c->stream) return hipStreamWaitEvent(s, c->done, 0);
    // the last was a blocking reduction on another caller stream: mark that stream now (the mark also covers
    // what was enqueued there after the reduction — more order than needed, never less)
    hipError_t e = hipEventRecord(c->mark, c->last);
    return e == hipSuccess ? hipStreamWaitEvent(s, c->mark, 0) : e;
}
}  // namespace

// SUM all-reduce of buf (in place) after the work already on `stream` and after the communicator's previous
// reduction (whichever stream issued it).  wait == 0: on the communicator's stream (the caller joins later with
// ppox_dp_wait; a second asynchronous reduction before that join is refused); wait != 0, the blocking form: on
// `stream` itself (each cross-stream event hop idles the GPU several us: per-rank 213 -> 198 ms).
extern "C" int ppox_dp_all_reduce(void* comm, void* buf, int64_t count, int32_t dtype, int32_t wait, void* stream) {
    PPOX_REQUIRE(comm, "ppox_dp_all_reduce: null communicator");
    PPOX_REQUIRE(count >= 0 && (count == 0 || buf), "ppox_dp_all_reduce: %lld elements at %p", (long long)count, buf);
    PPOX_REQUIRE(dtype == 0 || dtype == 1, "ppox_dp_all_reduce: dtype %d (0 = float32, 1 = float64)", dtype);
    auto* c = static_cast<DpComm*>(comm);
    PPOX_REQUIRE(wait || !c->inflight,
                 "ppox_dp_all_reduce: an asynchronous reduction is in flight (join it with ppox_dp_wait first)");
    hipStream_t s = ppox::as_stream(stream);
    if (count == 0) return PPOX_OK;
    const ncclDataType_t type = dtype ? ncclFloat64 : ncclFloat32;
    if (wait) {
        PPOX_HIP(order_after_last(c, s), "ppox_dp_all_reduce");
        c->inflight = false;
        ncclResult_t r = g_rccl.all_reduce(buf, buf, static_cast<size_t>(count), type, ncclSum, c->comm, s);
        if (r != ncclSuccess) return rccl_fail("ncclAllReduce", r);
        c->last = s;
        return PPOX_OK;
    }
    PPOX_HIP(hipEventRecord(c->ready, s), "ppox_dp_all_reduce");
    PPOX_HIP(hipStreamWaitEvent(c->stream, c->ready, 0), "ppox_dp_all_reduce");
    if (c->last != s) PPOX_HIP(order_after_last(c, c->stream), "ppox_dp_all_reduce");
    ncclResult_t r = g_rccl.all_reduce(buf, buf, static_cast<size_t>(count), type, ncclSum, c->comm, c->stream);
    if (r != ncclSuccess) return rccl_fail("ncclAllReduce", r);
    PPOX_HIP(hipEventRecord(c->done, c->stream), "ppox_dp_all_reduce");
    c->last = c->stream;
    c->inflight = true;
    return PPOX_OK;
}

// `stream` waits for every reduction issued on the communicator so far.
extern "C" int ppox_dp_wait(void* comm, void* stream) {
    PPOX_REQUIRE(comm, "ppox_dp_wait: null communicator");
    auto* c = static_cast<DpComm*>(comm);
    hipStream_t s = ppox::as_stream(stream);
    PPOX_HIP(order_after_last(c, s), "ppox_dp_wait");
    if (c->last) c->last = s;
    c->inflight = false;
    return PPOX_OK;
}

// Events for the fork / join of the backward's two streams (convs.fork / join).  torch's events record with a
// system-scope release (a cache writeback + invalidate for host visibility) — the trace showed each fork idling
// the main stream ~6-7 us at the per-rank shape; the streams here only need device-scope visibility.
extern "C" void ppox_ktime_arm(void* event) { ppox::ktime() = ppox::KTime{event, 0}; }

extern "C" int ppox_ktime_take(void) {
    const int used = ppox::ktime().used;
    ppox::ktime() = ppox::KTime{};
    return used;
}

// flags: hipEventCreateWithFlags flags (hipEventDisableTiming is added).
extern "C" int ppox_event_create(uint32_t flags, void** event_out) {
    PPOX_REQUIRE(event_out, "ppox_event_create: null output");
    hipEvent_t e = nullptr;
    PPOX_HIP(hipEventCreateWithFlags(&e, flags | hipEventDisableTiming), "ppox_event_create");
    *event_out = e;
    return PPOX_OK;
}

extern "C" int ppox_event_destroy(void* event) {
    if (event) PPOX_HIP(hipEventDestroy(static_cast<hipEvent_t>(event)), "ppox_event_destroy");
    return PPOX_OK;
}

// `wait_stream` waits for everything enqueued so far on `record_stream` (one event record + one wait)
extern "C" int ppox_stream_order(void* event, void* record_stream, void* wait_stream) {
    PPOX_REQUIRE(event, "ppox_stream_order: null event");
    PPOX_HIP(hipEventRecord(static_cast<hipEvent_t>(event), ppox::as_stream(record_stream)), "ppox_stream_order");
    PPOX_HIP(hipStreamWaitEvent(ppox::as_stream(wait_stream), static_cast<hipEvent_t>(event), 0), "ppox_stream_order");
    return PPOX_OK;
}
