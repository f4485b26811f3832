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

vacv_image Staging::out(Tensor& dst, int w, int h, int c, DType dtype, DLayout layout, int slot) {
    dst.create_on(_placement, w, h, c, dtype, layout);
    if (dst.len() > 0 && !dst.data) fail(_fn, "out of memory creating the output tensor");
    if (dst.on_device()) return describe(dst);
    void* d = _lease.scratch(slot, dst.len());
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

}  // namespace detail
}  // namespace vision
