// tests/cpp/fake_rccl.cpp -- TEST-ONLY stand-in for the part of librccl's ABI
// that librt_mi355x.so uses for its framebuffer gather (rt_render.cpp):
// ncclGetUniqueId, ncclCommInitRank, ncclCommInitAll, ncclCommDestroy,
// ncclSend, ncclRecv, ncclGroupStart / ncclGroupEnd, ncclGetErrorString.
//
// Selected with RT_RCCL_LIB=<this .so> (rt_render.cpp rccl()); built by
// tests/test_gather_standin_gpu.py; never linked into the product.  Real RCCL
// allows one rank per device, so a one-GPU box cannot run a gather of more
// than one rank with it.  This stand-in accepts any number of ranks on any
// devices -- several ncclCommInitRank ranks in one process (one host thread
// each), or a device list with repeats in ncclCommInitAll -- and moves each
// send to its matching receive with hipMemcpyPeerAsync, ordered as RCCL
// orders it: the copy waits for the sender's stream up to the send, the
// receiver's stream up to the receive, and the sender's stream continues only
// after the copy (the send buffer is free again).
//
// Matching follows RCCL's rule for point-to-point operations: the k-th send
// from rank a to rank b pairs with the k-th receive on b from a.  A pair whose
// byte counts differ is ncclInvalidUsage (the gather's counts are what the
// tests check); a receive whose send never comes times out (ncclSystemError)
// instead of hanging the test.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>
#include <unistd.h>

namespace {

struct Post {
    const void* buf = nullptr;
    size_t bytes = 0;
    int device = -1;
    hipEvent_t ready = nullptr;  // on the sender's stream after the send was enqueued
    hipEvent_t done = nullptr;   // on the receiver's stream after the copy
    bool has_done = false;
    bool failed = false;
};

// The ranks of one communicator (one unique id, or one ncclCommInitAll call).
struct Clique {
    std::mutex m;
    std::condition_variable cv;
    int nranks = 0, arrived = 0;
    std::map<std::tuple<int, int, uint64_t>, Post> mail;  // (src, dst, seq)
    std::map<std::pair<int, int>, uint64_t> send_seq, recv_seq;
    std::vector<hipEvent_t> events;  // destroyed with the last communicator
    int alive = 0;
};

struct Comm {
    std::shared_ptr<Clique> clique;
    int rank = 0, device = -1;
};

struct Op {
    bool send;
    void* buf;
    size_t bytes;
    int peer;
    Comm* comm;
    hipStream_t stream;
};

std::mutex g_ids_m;
std::map<std::string, std::shared_ptr<Clique>> g_ids;  // unique id -> clique (InitRank)
thread_local int t_depth = 0;
thread_local std::vector<Op> t_ops;
std::atomic<uint64_t> g_id_counter{1};
std::atomic<uint64_t> g_copies{0}, g_bytes{0};  // for the tests: what went through the stand-in

constexpr auto TIMEOUT = std::chrono::seconds(60);

size_t type_bytes(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        case ncclInt64: case ncclUint64: case ncclFloat64: return 8;
        default: return 0;
    }
}

ncclResult_t new_event(Clique& c, int device, hipStream_t stream, hipEvent_t& ev) {
    if (hipSetDevice(device) != hipSuccess) return ncclUnhandledCudaError;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return ncclUnhandledCudaError;
    if (hipEventRecord(ev, stream) != hipSuccess) return ncclUnhandledCudaError;
    c.events.push_back(ev);
    return ncclSuccess;
}

// One group's operations: every send is posted before any receive waits, so
// ranks whose groups run on different threads (or all of one ncclCommInitAll
// set in one thread's group) cannot wait on each other in a cycle.
ncclResult_t run_ops(std::vector<Op>& ops) {
    int saved = -1;
    (void)hipGetDevice(&saved);
    ncclResult_t res = ncclSuccess;
    std::vector<std::tuple<Clique*, int, int, uint64_t, Op*>> sends;
    for (Op& o : ops) {
        if (!o.send) continue;
        Clique& c = *o.comm->clique;
        std::unique_lock<std::mutex> lk(c.m);
        const uint64_t seq = c.send_seq[{o.comm->rank, o.peer}]++;
        Post p;
        p.buf = o.buf;
        p.bytes = o.bytes;
        p.device = o.comm->device;
        if ((res = new_event(c, o.comm->device, o.stream, p.ready)) != ncclSuccess) break;
        c.mail[{o.comm->rank, o.peer, seq}] = p;
        sends.emplace_back(&c, o.comm->rank, o.peer, seq, &o);
        c.cv.notify_all();
    }
    for (Op& o : ops) {
        if (o.send || res != ncclSuccess) continue;
        Clique& c = *o.comm->clique;
        std::unique_lock<std::mutex> lk(c.m);
        const uint64_t seq = c.recv_seq[{o.peer, o.comm->rank}]++;
        const auto key = std::make_tuple(o.peer, o.comm->rank, seq);
        if (!c.cv.wait_for(lk, TIMEOUT, [&] { return c.mail.count(key) != 0; })) {
            res = ncclSystemError;
            break;
        }
        Post& p = c.mail[key];
        if (p.bytes != o.bytes) {
            p.failed = true;
            p.has_done = true;
            c.cv.notify_all();
            res = ncclInvalidUsage;
            break;
        }
        if (hipSetDevice(o.comm->device) != hipSuccess || hipStreamWaitEvent(o.stream, p.ready, 0) != hipSuccess ||
            (p.bytes && hipMemcpyPeerAsync(o.buf, o.comm->device, p.buf, p.device, p.bytes, o.stream) != hipSuccess)) {
            res = ncclUnhandledCudaError;
            break;
        }
        if ((res = new_event(c, o.comm->device, o.stream, p.done)) != ncclSuccess) break;
        ++g_copies;
        g_bytes += p.bytes;
        p.has_done = true;
        c.cv.notify_all();
    }
    for (auto& [cp, src, dst, seq, op] : sends) {
        if (res != ncclSuccess) break;
        Clique& c = *cp;
        std::unique_lock<std::mutex> lk(c.m);
        const auto key = std::make_tuple(src, dst, seq);
        if (!c.cv.wait_for(lk, TIMEOUT, [&] { return c.mail[key].has_done; })) {
            res = ncclSystemError;
            break;
        }
        Post p = c.mail[key];
        c.mail.erase(key);
        if (p.failed) {
            res = ncclInvalidUsage;
            break;
        }
        if (hipSetDevice(op->comm->device) != hipSuccess || hipStreamWaitEvent(op->stream, p.done, 0) != hipSuccess) {
            res = ncclUnhandledCudaError;
            break;
        }
    }
    if (saved >= 0) (void)hipSetDevice(saved);
    return res;
}

ncclResult_t enqueue(Op o) {
    if (!o.comm || o.peer < 0 || o.peer >= o.comm->clique->nranks) return ncclInvalidArgument;
    t_ops.push_back(o);
    if (t_depth > 0) return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(t_ops);
    return run_ops(ops);
}

}  // namespace

extern "C" {

// test hook: copies and bytes moved so far (tests/test_gather_standin_gpu.py)
void fake_rccl_counts(uint64_t out[2]) {
    out[0] = g_copies.load();
    out[1] = g_bytes.load();
}

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (stand-in)";
        case ncclUnhandledCudaError: return "HIP call failed (stand-in)";
        case ncclSystemError: return "timed out waiting for the peer (stand-in)";
        case ncclInvalidArgument: return "invalid argument (stand-in)";
        case ncclInvalidUsage: return "send / receive byte counts differ (stand-in)";
        default: return "error (stand-in)";
    }
}

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    std::memset(id, 0, sizeof *id);
    const uint64_t v[2] = {(uint64_t)getpid(), g_id_counter++};
    std::memcpy(id, v, sizeof v);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* out, int nranks, ncclUniqueId id, int rank) {
    if (!out || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    const std::string key(reinterpret_cast<const char*>(&id), sizeof id);
    std::shared_ptr<Clique> c;
    {
        std::lock_guard<std::mutex> lk(g_ids_m);
        auto& slot = g_ids[key];
        if (!slot) {
            slot = std::make_shared<Clique>();
            slot->nranks = nranks;
        }
        c = slot;
    }
    if (c->nranks != nranks) return ncclInvalidArgument;
    auto* comm = new Comm();
    comm->clique = c;
    comm->rank = rank;
    (void)hipGetDevice(&comm->device);
    // like RCCL: returns once every rank of the id has arrived
    std::unique_lock<std::mutex> lk(c->m);
    ++c->arrived;
    ++c->alive;
    c->cv.notify_all();
    if (!c->cv.wait_for(lk, TIMEOUT, [&] { return c->arrived >= c->nranks; })) {
        --c->alive;
        delete comm;
        return ncclSystemError;
    }
    *out = reinterpret_cast<ncclComm_t>(comm);
    return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist) {
    if (!comms || ndev < 1) return ncclInvalidArgument;
    auto c = std::make_shared<Clique>();
    c->nranks = ndev;
    c->arrived = ndev;
    c->alive = ndev;
    for (int k = 0; k < ndev; ++k) {
        auto* comm = new Comm();
        comm->clique = c;
        comm->rank = k;
        comm->device = devlist ? devlist[k] : k;
        comms[k] = reinterpret_cast<ncclComm_t>(comm);
    }
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    auto* c = reinterpret_cast<Comm*>(comm);
    if (!c) return ncclInvalidArgument;
    std::shared_ptr<Clique> q = c->clique;
    delete c;
    std::lock_guard<std::mutex> lk(q->m);
    if (--q->alive == 0) {
        (void)hipDeviceSynchronize();
        for (hipEvent_t e : q->events) (void)hipEventDestroy(e);
        q->events.clear();
    }
    return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
    ++t_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (t_depth <= 0) return ncclInvalidUsage;
    if (--t_depth > 0) return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(t_ops);
    return run_ops(ops);
}

ncclResult_t ncclSend(const void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm,
                      hipStream_t stream) {
    const size_t b = type_bytes(type);
    if (!b) return ncclInvalidArgument;
    return enqueue(Op{true, const_cast<void*>(buf), count * b, peer, reinterpret_cast<Comm*>(comm), stream});
}

ncclResult_t ncclRecv(void* buf, size_t count, ncclDataType_t type, int peer, ncclComm_t comm, hipStream_t stream) {
    const size_t b = type_bytes(type);
    if (!b) return ncclInvalidArgument;
    return enqueue(Op{false, buf, count * b, peer, reinterpret_cast<Comm*>(comm), stream});
}

}  // extern "C"
