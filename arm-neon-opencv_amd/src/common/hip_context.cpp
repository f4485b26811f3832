// Stream / scratch leasing for the C++ layer (see hip_context.h).
#include "hip_context.h"

#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace vision {
namespace detail {

void fail(const char* fn, const char* why) {
    throw std::runtime_error(std::string(fn) + ": " + why);
}

void check(const char* fn, int status) {
    if (status != VACV_OK) fail(fn, vacv_status_string(status));
}

void check_hip(const char* fn, hipError_t e) {
    if (e != hipSuccess) fail(fn, hipGetErrorString(e));
}

int compute_device(const Tensor& t) {
    if (t.on_device()) return t.device();
    int d = 0;
    check_hip("vacv", hipGetDevice(&d));
    return d;
}

struct Lease::Ctx {
    hipStream_t stream = nullptr;
    void* slot[kSlots] = {};
    size_t cap[kSlots] = {};
};

namespace {
std::mutex g_mu;
// idle contexts per device; never destroyed (streams outlive static teardown)
std::map<int, std::vector<Lease::Ctx*>>& idle() {
    static auto* m = new std::map<int, std::vector<Lease::Ctx*>>;
    return *m;
}
}  // namespace

Lease::Lease(int device) : _ctx(nullptr), _device(device), _prev(-1) {
    check_hip("vacv", hipGetDevice(&_prev));
    if (_prev != device) check_hip("vacv: hipSetDevice", hipSetDevice(device));
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto& v = idle()[device];
        if (!v.empty()) {
            _ctx = v.back();
            v.pop_back();
        }
    }
    if (!_ctx) {
        _ctx = new Ctx;
        hipError_t e = hipStreamCreateWithFlags(&_ctx->stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            delete _ctx;
            _ctx = nullptr;
            if (_prev != device) (void)hipSetDevice(_prev);
            check_hip("vacv: hipStreamCreate", e);
        }
    }
}

Lease::~Lease() {
    if (_ctx) {
        std::lock_guard<std::mutex> lk(g_mu);
        idle()[_device].push_back(_ctx);
    }
    if (_prev >= 0 && _prev != _device) (void)hipSetDevice(_prev);
}

hipStream_t Lease::stream() const { return _ctx->stream; }

void* Lease::scratch(int slot, size_t bytes) {
    if (slot < 0 || slot >= kSlots) fail("vacv", "scratch slot out of range");
    if (_ctx->cap[slot] < bytes) {
        if (_ctx->slot[slot]) {
            // queued work may still read the old block
            check_hip("vacv: hipStreamSynchronize", hipStreamSynchronize(_ctx->stream));
            (void)hipFree(_ctx->slot[slot]);
            _ctx->slot[slot] = nullptr;
            _ctx->cap[slot] = 0;
        }
        const size_t cap = bytes < (size_t(1) << 20) ? (size_t(1) << 20) : (bytes + 4095) & ~size_t(4095);
        check_hip("vacv: hipMalloc(scratch)", hipMalloc(&_ctx->slot[slot], cap));
        _ctx->cap[slot] = cap;
    }
    return _ctx->slot[slot];
}

void Lease::sync(const char* fn) { check_hip(fn, hipStreamSynchronize(_ctx->stream)); }

vacv_image describe(const Tensor& t, void* data) {
    vacv_image d{};
    d.data = data;
    d.n = 1;
    d.w = t.w;
    d.h = t.h;
    d.c = t.c;
    d.dtype = t.dtype;
    d.layout = t.layout;
    return d;  // pitches 0 = dense
}

Staging::Staging(const char* fn, const Tensor& anchor)
    : _fn(fn), _placement(anchor.device()), _lease(compute_device(anchor)) {}

Staging::~Staging() {
    if (!_keep.empty()) (void)hipStreamSynchronize(_lease.stream());
}

vacv_image Staging::in(const Tensor& t, int slot) {
    if (t.empty()) fail(_fn, "empty input tensor");
    _keep.push_back(t);
    if (t.on_device()) {
        if (t.device() != _lease.device()) fail(_fn, "operands live on different devices");
        return describe(t);
    }
    void* d = _lease.scratch(slot, t.len());
    check_hip(_fn, hipMemcpyAsync(d, t.data, t.len(), hipMemcpyHostToDevice, _lease.stream()));
    return describe(t, d);
}

vacv_image Staging::out(Tensor& dst, int w, int h, int c, DType dtype, DLayout layout, int slot, bool keep) {
    dst.create_on(_placement, w, h, c, dtype, layout);
    if (dst.len() > 0 && !dst.data) fail(_fn, "out of memory creating the output tensor");
    if (dst.on_device()) return describe(dst);
    void* d = _lease.scratch(slot, dst.len());
    if (keep && dst.len() > 0)  // the scratch slot holds an earlier call's bytes: seed it with dst's
        check_hip(_fn, hipMemcpyAsync(d, dst.data, dst.len(), hipMemcpyHostToDevice, _lease.stream()));
    _d2h.push_back({dst.data, d, dst.len()});
    _keep.push_back(dst);
    return describe(dst, d);
}

void Staging::finish() {
    for (const Copy& c : _d2h)
        check_hip(_fn, hipMemcpyAsync(c.host, c.dev, c.bytes, hipMemcpyDeviceToHost, _lease.stream()));
    _d2h.clear();
    _lease.sync(_fn);
    _keep.clear();
}

// ---- FramePipeline --------------------------------------------------------
// Two streams: `load` runs H2D(i) then kernel(i) in order, `store` runs
// D2H(i) behind kernel(i)'s event, so H2D(i+1) overlaps D2H(i).  Slot reuse is
// throttled on the HOST (hipEventSynchronize on the slot's last event before
// its buffers are overwritten).  Measured on MI355X (tools/pcie_bench.cpp,
// profiles/r02_pcie_bench.jsonl): device-side waits for slot reuse
// (hipStreamWaitEvent on an event of the other stream, recorded but not yet
// complete at enqueue) stalled the copy engines -- 0.26-0.28 ms per 1080p
// frame against 0.13 ms for the same chain without backward waits.
struct FramePipeline::Ctx {
    hipStream_t load = nullptr, store = nullptr;
    void* din[kRing] = {};
    size_t din_cap[kRing] = {};
    void* dout[kRing] = {};
    size_t dout_cap[kRing] = {};
    hipEvent_t ev_kern[kRing] = {};  // kernel done: input slot free, output ready
    hipEvent_t ev_out[kRing] = {};   // D2H done: output slot free
    hipEvent_t* last[kRing] = {};    // the slot's last event (host-side throttle)
};

namespace {
std::mutex g_pipe_mu;
std::map<int, std::vector<FramePipeline::Ctx*>>& idle_pipes() {
    static auto* m = new std::map<int, std::vector<FramePipeline::Ctx*>>;
    return *m;
}

void grow(void*& p, size_t& cap, size_t bytes) {
    if (cap >= bytes) return;
    if (p) (void)hipFree(p);  // the slot is idle (its last event was waited for)
    p = nullptr;
    cap = 0;
    const size_t c = (bytes + 4095) & ~size_t(4095);
    check_hip("vacv: hipMalloc(pipeline slot)", hipMalloc(&p, c));
    cap = c;
}
}  // namespace

FramePipeline::FramePipeline(const char* fn, int device)
    : _fn(fn), _device(device), _prev(-1), _ctx(nullptr), _count(0) {
    check_hip(fn, hipGetDevice(&_prev));
    if (_prev != device) check_hip("vacv: hipSetDevice", hipSetDevice(device));
    {
        std::lock_guard<std::mutex> lk(g_pipe_mu);
        auto& v = idle_pipes()[device];
        if (!v.empty()) {
            _ctx = v.back();
            v.pop_back();
        }
    }
    if (!_ctx) {
        Ctx* c = new Ctx;
        bool ok = hipStreamCreateWithFlags(&c->load, hipStreamNonBlocking) == hipSuccess &&
                  hipStreamCreateWithFlags(&c->store, hipStreamNonBlocking) == hipSuccess;
        for (int k = 0; k < kRing && ok; ++k)
            ok = hipEventCreateWithFlags(&c->ev_kern[k], hipEventDisableTiming) == hipSuccess &&
                 hipEventCreateWithFlags(&c->ev_out[k], hipEventDisableTiming) == hipSuccess;
        if (!ok) {
            if (_prev != device) (void)hipSetDevice(_prev);
            fail(fn, "could not create the pipeline's streams");
        }
        _ctx = c;
    }
    for (int k = 0; k < kRing; ++k) _ctx->last[k] = nullptr;
}

FramePipeline::~FramePipeline() {
    if (_ctx) {
        // an early exit (exception): let queued work finish before the kept
        // operands and the slots are released
        (void)hipStreamSynchronize(_ctx->load);
        (void)hipStreamSynchronize(_ctx->store);
        std::lock_guard<std::mutex> lk(g_pipe_mu);
        idle_pipes()[_device].push_back(_ctx);
    }
    if (_prev >= 0 && _prev != _device) (void)hipSetDevice(_prev);
}

void FramePipeline::frame(const Tensor& src, Tensor& dst, int w, int h, int c, DType dtype, DLayout layout,
                          const Launch& launch) {
    if (src.empty()) fail(_fn, "empty input tensor");
    const int k = (int)(_count++ % kRing);
    Ctx& x = *_ctx;
    if (x.last[k]) check_hip(_fn, hipEventSynchronize(*x.last[k]));  // the slot's previous frame is done
    _keep.push_back(src);
    vacv_image s;
    if (src.on_device()) {
        if (src.device() != _device) fail(_fn, "operands live on different devices");
        s = describe(src);
    } else {
        grow(x.din[k], x.din_cap[k], src.len());
        check_hip(_fn, hipMemcpyAsync(x.din[k], src.data, src.len(), hipMemcpyHostToDevice, x.load));
        s = describe(src, x.din[k]);
    }
    dst.create_on(src.device(), w, h, c, dtype, layout);
    if (dst.len() > 0 && !dst.data) fail(_fn, "out of memory creating the output tensor");
    _keep.push_back(dst);
    vacv_image d;
    if (dst.on_device()) {
        d = describe(dst);
    } else {
        grow(x.dout[k], x.dout_cap[k], dst.len());
        d = describe(dst, x.dout[k]);
    }
    check(_fn, launch(s, d, x.load));
    check_hip(_fn, hipEventRecord(x.ev_kern[k], x.load));
    x.last[k] = &x.ev_kern[k];
    if (!dst.on_device()) {
        check_hip(_fn, hipStreamWaitEvent(x.store, x.ev_kern[k], 0));
        check_hip(_fn, hipMemcpyAsync(dst.data, x.dout[k], dst.len(), hipMemcpyDeviceToHost, x.store));
        check_hip(_fn, hipEventRecord(x.ev_out[k], x.store));
        x.last[k] = &x.ev_out[k];
    }
}

void FramePipeline::finish() {
    check_hip(_fn, hipStreamSynchronize(_ctx->load));
    check_hip(_fn, hipStreamSynchronize(_ctx->store));
    _keep.clear();
}

}  // namespace detail
}  // namespace vision
