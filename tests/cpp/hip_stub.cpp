// tests/cpp/hip_stub.cpp -- TEST HARNESS: a CPU stand-in for the device layer
// under librt_mi355x.so's launcher (rt_render.cpp), so that the launcher's
// concurrent host code -- one host thread per device part, the shared
// FlatWorld, the cached ncclCommInitAll sets and their group locks, the
// communicator ranks, the RcclApi initialisation -- runs under ThreadSanitizer
// on a machine without a GPU (tests/test_launcher_tsan_cpu.py).
//
// It implements the HIP runtime calls rt_render.cpp makes (nm -u of its
// object) with HIP's ordering rules, asynchronously: every stream is a worker
// thread running its queue in order; an event record is a queue entry that
// marks the event; hipStreamWaitEvent queues a wait for the event's last
// record; hipStreamSynchronize / hipDeviceSynchronize drain queues; hipFree
// waits for the device's streams, as HIP's does.  Devices are host memory,
// HIP_STUB_DEVICES of them (default 8), each reporting gfx950.
//
// The device-side entry points of rt_kernel.h (rtk_launch_frame, the gather's
// deinterleave, to_rgb) are queue entries too.  The stub "path kernel" does
// not trace rays: it writes pixel (y, x, c) = stub_value(y, x, c) for the
// image rows of its shard (row_offset + k * row_stride), and its sRGB byte, so
// that the driver can check that every row of a gathered frame arrived where
// it belongs.  The frame plan (rtk_row_parts, rtk_tail_split, ...) is the
// product's own code (csrc/rt_plan.h).
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../raytracer-2025_amd/csrc/rt_kernel.h"
#include "../../raytracer-2025_amd/csrc/rt_plan.h"

extern "C" float stub_value(uint32_t y, uint32_t x, uint32_t c) { return (float)(y * 4096u + x * 4u + c + 1u) * 0.25f; }
extern "C" uint8_t stub_byte(uint32_t y, uint32_t x, uint32_t c) { return (uint8_t)((y * 7u + x * 3u + c) & 0xffu); }

namespace {

using Clock = std::chrono::steady_clock;

struct Stream {
    int device = 0;
    std::mutex m;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    uint64_t enq = 0, done = 0;
    bool stop = false;
    std::thread th;
    Stream(int dev) : device(dev) {
        th = std::thread([this] {
            std::unique_lock<std::mutex> lk(m);
            for (;;) {
                cv.wait(lk, [this] { return stop || !q.empty(); });
                if (q.empty()) return;
                std::function<void()> f = std::move(q.front());
                q.pop_front();
                lk.unlock();
                f();
                lk.lock();
                ++done;
                cv.notify_all();
            }
        });
    }
    void push(std::function<void()> f) {
        std::lock_guard<std::mutex> lk(m);
        q.push_back(std::move(f));
        ++enq;
        cv.notify_all();
    }
    void drain() {
        std::unique_lock<std::mutex> lk(m);
        const uint64_t target = enq;
        cv.wait(lk, [&] { return done >= target; });
    }
    ~Stream() {
        {
            std::lock_guard<std::mutex> lk(m);
            stop = true;
            cv.notify_all();
        }
        th.join();
    }
};

struct Event {
    std::mutex m;
    std::condition_variable cv;
    uint64_t enq = 0, done = 0;
    Clock::time_point t{};
};

struct Runtime {
    int n_devices = 8;
    std::mutex m;  // streams, null_streams
    std::vector<Stream*> null_streams;
    std::vector<std::shared_ptr<Stream>> streams;  // created ones (a drain holds its own reference)
    Runtime() {
        if (const char* e = std::getenv("HIP_STUB_DEVICES")) n_devices = std::max(1, std::atoi(e));
        for (int d = 0; d < n_devices; ++d) null_streams.push_back(new Stream(d));
    }
    // never destroyed: worker threads may still be parked at exit
};
Runtime& rt() {
    static Runtime* r = new Runtime();
    return *r;
}
thread_local int t_device = 0;

// HIP_STUB_DELAY_US: every stub kernel first sleeps this long, so that the
// host runs ahead of the "device" as it does on a GPU (a host access the
// launcher has not ordered after the kernel then precedes the kernel's, with
// no lock of the stream queue between them: TSan sees it)
void kernel_delay() {
    static const long us = std::getenv("HIP_STUB_DELAY_US") ? std::atol(std::getenv("HIP_STUB_DELAY_US")) : 0;
    if (us > 0) std::this_thread::sleep_for(std::chrono::microseconds(us));
}

Stream* resolve(hipStream_t s) {
    if (s) return reinterpret_cast<Stream*>(s);
    return rt().null_streams[t_device];
}
void drain_device(int dev) {
    Runtime& R = rt();
    std::vector<std::shared_ptr<Stream>> v;
    Stream* null_stream = R.null_streams[dev];
    {
        std::lock_guard<std::mutex> lk(R.m);
        for (const auto& s : R.streams)
            if (s->device == dev) v.push_back(s);
    }
    null_stream->drain();
    for (const auto& s : v) s->drain();
}

}  // namespace

extern "C" {

hipError_t hipGetDevice(int* d) {
    *d = t_device;
    return hipSuccess;
}
hipError_t hipSetDevice(int d) {
    if (d < 0 || d >= rt().n_devices) return hipErrorInvalidDevice;
    t_device = d;
    return hipSuccess;
}
hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_tR0600* p, int d) {
    if (d < 0 || d >= rt().n_devices) return hipErrorInvalidDevice;
    std::memset(p, 0, sizeof *p);
    std::strcpy(p->name, "stub");
    std::strcpy(p->gcnArchName, "gfx950:sramecc+:xnack-");
    p->multiProcessorCount = 4;
    p->totalGlobalMem = (size_t)64 << 30;
    return hipSuccess;
}
hipError_t hipMemGetInfo(size_t* free_b, size_t* total) {
    *free_b = *total = (size_t)64 << 30;
    return hipSuccess;
}
const char* hipGetErrorString(hipError_t) { return "hip stub error"; }
hipError_t hipGetLastError(void) { return hipSuccess; }

hipError_t hipMalloc(void** p, size_t n) {
    *p = std::calloc(1, n ? n : 1);  // zeroed: a stub kernel's unwritten bytes read as 0, not as garbage
    return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void* p) {
    // HIP's hipFree synchronises the device: no queued work may still use it
    for (int d = 0; d < rt().n_devices; ++d) drain_device(d);
    std::free(p);
    return hipSuccess;
}
hipError_t hipMemcpy(void* dst, const void* src, size_t n, hipMemcpyKind) {
    resolve(nullptr)->drain();  // ordered after the current device's null stream
    std::memcpy(dst, src, n);
    return hipSuccess;
}
hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t s) {
    resolve(s)->push([=] { std::memset(p, v, n); });
    return hipSuccess;
}
hipError_t hipMemcpyPeerAsync(void* dst, int, const void* src, int, size_t n, hipStream_t s) {
    resolve(s)->push([=] { std::memcpy(dst, src, n); });
    return hipSuccess;
}
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t n, hipMemcpyKind, hipStream_t s) {
    resolve(s)->push([=] { std::memcpy(dst, src, n); });
    return hipSuccess;
}

hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned int) {
    auto st = std::make_shared<Stream>(t_device);
    {
        std::lock_guard<std::mutex> lk(rt().m);
        rt().streams.push_back(st);
    }
    *s = reinterpret_cast<hipStream_t>(st.get());
    return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
    std::shared_ptr<Stream> st;
    {
        std::lock_guard<std::mutex> lk(rt().m);
        auto& v = rt().streams;
        for (auto it = v.begin(); it != v.end(); ++it)
            if (it->get() == reinterpret_cast<Stream*>(s)) {
                st = *it;
                v.erase(it);
                break;
            }
    }
    if (!st) return hipErrorInvalidHandle;
    st->drain();  // the worker is joined when the last reference goes
    return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t s) {
    resolve(s)->drain();
    return hipSuccess;
}
hipError_t hipDeviceSynchronize(void) {
    drain_device(t_device);
    return hipSuccess;
}

hipError_t hipEventCreate(hipEvent_t* e) {
    *e = reinterpret_cast<hipEvent_t>(new Event());
    return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned int) { return hipEventCreate(e); }
hipError_t hipEventDestroy(hipEvent_t e) {
    Event* ev = reinterpret_cast<Event*>(e);
    {  // (HIP defers the release of a recorded event until it completes)
        std::unique_lock<std::mutex> lk(ev->m);
        ev->cv.wait(lk, [ev] { return ev->done >= ev->enq; });
    }
    delete ev;
    return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) {
    Event* ev = reinterpret_cast<Event*>(e);
    uint64_t seq;
    {
        std::lock_guard<std::mutex> lk(ev->m);
        seq = ++ev->enq;
    }
    resolve(s)->push([ev, seq] {
        std::lock_guard<std::mutex> lk(ev->m);
        if (seq > ev->done) {
            ev->done = seq;
            ev->t = Clock::now();
        }
        ev->cv.notify_all();
    });
    return hipSuccess;
}
hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned int) {
    Event* ev = reinterpret_cast<Event*>(e);
    uint64_t target;
    {
        std::lock_guard<std::mutex> lk(ev->m);
        target = ev->enq;
    }
    resolve(s)->push([ev, target] {
        std::unique_lock<std::mutex> lk(ev->m);
        ev->cv.wait(lk, [&] { return ev->done >= target; });
    });
    return hipSuccess;
}
hipError_t hipEventElapsedTime(float* ms, hipEvent_t a, hipEvent_t b) {
    Event *ea = reinterpret_cast<Event*>(a), *eb = reinterpret_cast<Event*>(b);
    Clock::time_point ta, tb;
    {
        std::lock_guard<std::mutex> lk(ea->m);
        if (ea->done < ea->enq || ea->enq == 0) return hipErrorNotReady;
        ta = ea->t;
    }
    {
        std::lock_guard<std::mutex> lk(eb->m);
        if (eb->done < eb->enq || eb->enq == 0) return hipErrorNotReady;
        tb = eb->t;
    }
    *ms = std::chrono::duration<float, std::milli>(tb - ta).count() + 1e-3f;  // > 0: a timed gather ran
    return hipSuccess;
}

// ---------------------------------------------------------------- rt_kernel.h
int rtk_tier_for(uint32_t features, uint32_t stack_need) {
    return rtk::plan::tier_for(features, stack_need, true, RT_STACK_BASIC);
}
uint32_t rtk_stack_entries(int tier) { return tier == rtk::TIER_BASIC ? RT_STACK_BASIC : RT_STACK_MAX; }
int rtk_basic_bvh4(void) { return 1; }
int rtk_mesh_bvh4(void) { return 1; }
int rtk_full_bvh4(void) { return 1; }
int rtk_planar_filter(void) { return 0; }
int rtk_block_threads(int tier) { return tier == rtk::TIER_BASIC ? RT_BLOCK_BASIC : RT_BLOCK; }
uint32_t rtk_row_parts(uint32_t S, uint32_t part_samples) { return rtk::plan::row_parts(S, part_samples); }
uint32_t rtk_tail_rows(uint32_t W, uint32_t H, uint32_t S, uint32_t parts, uint64_t budget, uint32_t permille) {
    return rtk::plan::tail_rows(W, H, S, parts, budget, permille);
}
void rtk_tail_split(uint32_t W, uint32_t H, uint32_t S, uint32_t parts, uint32_t parts2, uint64_t budget,
                    uint32_t permille, uint32_t fine_permille, uint32_t* tail, uint32_t* fine) {
    rtk::plan::tail_split(W, H, S, parts, parts2, budget, permille, fine_permille, tail, fine);
}
uint32_t rtk_shard_whole_rows(uint32_t H, uint32_t tail, uint32_t off, uint32_t stride, uint32_t rows) {
    return rtk::plan::shard_whole_rows(H, tail, off, stride, rows);
}
size_t rtk_params_bytes(void) { return 4096; }
int rtk_path_kernel_occupancy(int, int* blocks_per_cu) {
    *blocks_per_cu = 2;
    return 0;
}
int rtk_check_read(unsigned long long* out, int) {
    out[0] = out[1] = 0;
    return 0;
}

// The stub path kernel + reduce: the shard's rows of stub_value / stub_byte.
hipError_t rtk_launch_frame(const rtk::SceneView* view, const rtk_frame_desc* fd, uint32_t* queue, double* partial,
                            unsigned long long* stats, float* out, uint8_t* srgb, int, hipStream_t stream, int, int,
                            void* params_dev, void*) {
    const rtk_frame_desc f = *fd;          // the launch's parameters are copied at enqueue,
    const rtk::SceneView v = *view;        // as the real launcher's hipMemcpyAsync of KParams
    Stream* st = resolve(stream);
    if (f.ev_start) (void)hipEventRecord((hipEvent_t)f.ev_start, stream);
    st->push([=] {
        kernel_delay();
        // read the uploaded world and the launch's device buffers, as the kernel does
        volatile uint32_t sink = v.world_root + (v.n_nodes4 ? ((const uint32_t*)v.nodes4)[0] : 0u);
        (void)sink;
        std::memset(params_dev, 0, 64);
        queue[0] = 0;
        for (uint32_t k = 0; k < f.rows; ++k) {
            const uint32_t y = f.row_offset + k * f.row_stride;
            for (uint32_t x = 0; x < f.W; ++x)
                for (uint32_t c = 0; c < 3; ++c) {
                    const size_t i = ((size_t)k * f.W + x) * 3 + c;
                    out[i] = stub_value(y, x, c);
                    if (srgb) srgb[i] = stub_byte(y, x, c);
                }
        }
        partial[0] = 1.0;
        stats[0] = (unsigned long long)f.W * f.rows * f.S;
        stats[1] = 0;
    });
    if (f.ev_stop) (void)hipEventRecord((hipEvent_t)f.ev_stop, stream);
    return hipSuccess;
}
hipError_t rtk_launch_deinterleave(const float* staging, size_t slice, float* out, uint32_t rows, uint32_t W,
                                   uint32_t parts, hipStream_t stream) {
    resolve(stream)->push([=] {
        kernel_delay();
        const uint64_t row_floats = (uint64_t)W * 3;
        for (uint32_t j = 0; j < rows; ++j)
            std::memcpy(out + (uint64_t)j * row_floats, staging + (uint64_t)(j % parts) * slice + (uint64_t)(j / parts) * row_floats,
                        row_floats * sizeof(float));
    });
    return hipSuccess;
}
hipError_t rtk_launch_deinterleave_u8(const uint8_t* staging, size_t slice, uint8_t* out, uint32_t rows, uint32_t W,
                                      uint32_t parts, hipStream_t stream) {
    resolve(stream)->push([=] {
        kernel_delay();
        const uint64_t row_bytes = (uint64_t)W * 3;
        for (uint32_t j = 0; j < rows; ++j)
            std::memcpy(out + (uint64_t)j * row_bytes, staging + (uint64_t)(j % parts) * slice + (uint64_t)(j / parts) * row_bytes,
                        row_bytes);
    });
    return hipSuccess;
}
hipError_t rtk_launch_to_rgb(const float* lin, uint8_t* srgb, uint64_t n, int, hipStream_t stream) {
    resolve(stream)->push([=] {
        for (uint64_t i = 0; i < n; ++i) srgb[i] = (uint8_t)lin[i];
    });
    return hipSuccess;
}
hipError_t rtk_launch_math(int, int, const double*, const double*, double*, uint64_t, hipStream_t) {
    return hipErrorNotSupported;
}

}  // extern "C"
