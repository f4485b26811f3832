// vision::Tensor -- refcounted image buffer, host or HBM (see tensor.h).
//
// Semantics follow the reference's src/common/tensor.cpp:
//   copy/assign share the buffer and bump a refcount (:103-144); release()
//   drops it and zeroes the shape (:554-569); create() is a no-op when the
//   shape already matches (:512-514); size() = stride*c elements, len() its
//   bytes (:571-590).
// The pixel work of change_layout / change_dtype (:393-502) runs on the GPU
// through the C ABI, never on the host CPU.
#include "tensor.h"

#include <atomic>
#include <cstring>

#include "hip_context.h"
#include "va_allocator.h"

namespace vision {

struct Tensor::Block {
    std::atomic<int> refs{1};
    void* ptr = nullptr;
    int device = kHost;
};

size_t dtype_size(DType dtype) {
    switch (dtype) {
        case FP64: return 8;
        case FP32: return 4;
        case FP16: return 2;
        case INT8: return 1;
        default: return 0;
    }
}

static int dims_of(int h, int c) { return (h == 1 && c == 1) ? 1 : (c == 1 ? 2 : 3); }

Tensor::Tensor()
    : w(0), h(0), c(0), stride(0), dims(0), data(nullptr), dtype(FP32), layout(NCHW),
      _block(nullptr), _device(kHost) {}

Tensor::Tensor(int w_, DType dt, DLayout ly) : Tensor() { create(w_, 1, 1, dt, ly); }
Tensor::Tensor(int w_, int h_, DType dt, DLayout ly) : Tensor() { create(w_, h_, 1, dt, ly); }
Tensor::Tensor(int w_, int h_, int c_, DType dt, DLayout ly) : Tensor() { create(w_, h_, c_, dt, ly); }
Tensor::Tensor(int w_, DLayout ly, DType dt) : Tensor(w_, dt, ly) {}
Tensor::Tensor(int w_, int h_, DLayout ly, DType dt) : Tensor(w_, h_, dt, ly) {}
Tensor::Tensor(int w_, int h_, int c_, DLayout ly, DType dt) : Tensor(w_, h_, c_, dt, ly) {}

Tensor::Tensor(int w_, int h_, int c_, void* p, DType dt, DLayout ly) : Tensor() {
    w = w_;
    h = h_;
    c = c_;
    stride = w_ * h_;
    // the reference records the constructor's arity, not the shape (tensor.cpp:72-85)
    dims = 3;
    data = p;
    dtype = dt;
    layout = ly;
}
Tensor::Tensor(int w_, void* p, DType dt, DLayout ly) : Tensor(w_, 1, 1, p, dt, ly) { dims = 1; }
Tensor::Tensor(int w_, int h_, void* p, DType dt, DLayout ly) : Tensor(w_, h_, 1, p, dt, ly) { dims = 2; }
Tensor::Tensor(int w_, void* p, DLayout ly, DType dt) : Tensor(w_, p, dt, ly) {}
Tensor::Tensor(int w_, int h_, void* p, DLayout ly, DType dt) : Tensor(w_, h_, p, dt, ly) {}
Tensor::Tensor(int w_, int h_, int c_, void* p, DLayout ly, DType dt) : Tensor(w_, h_, c_, p, dt, ly) {}

Tensor Tensor::device_view(int device, int w_, int h_, int c_, void* p, DType dt, DLayout ly) {
    Tensor t(w_, h_, c_, p, dt, ly);
    t._device = device;
    return t;
}

void Tensor::retain() const {
    if (_block) _block->refs.fetch_add(1, std::memory_order_relaxed);
}

void Tensor::adopt(const Tensor& t) {
    w = t.w;
    h = t.h;
    c = t.c;
    stride = t.stride;
    dims = t.dims;
    data = t.data;
    dtype = t.dtype;
    layout = t.layout;
    _name = t._name;
    _block = t._block;
    _device = t._device;
}

Tensor::Tensor(const Tensor& t) : _block(nullptr), _device(kHost) {
    t.retain();
    adopt(t);
}

Tensor& Tensor::operator=(const Tensor& t) {
    if (this == &t) return *this;
    t.retain();  // before release(): t may share our block
    release();
    adopt(t);
    return *this;
}

Tensor::~Tensor() { release(); }

void Tensor::release() {
    if (_block && _block->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        if (_block->device == kHost) {
            VaAllocator::deallocate(_block->ptr);
        } else {
            VaAllocator::deallocate_device(_block->ptr, _block->device);
        }
        delete _block;
    }
    _block = nullptr;
    data = nullptr;
    dtype = FP32;
    layout = NCHW;
    stride = 0;
    dims = 0;
    w = h = c = 0;
    _device = kHost;
    _name.clear();
}

void Tensor::create_on(int device, int w_, int h_, int c_, DType dt, DLayout ly) {
    if (w == w_ && h == h_ && c == c_ && dtype == dt && layout == ly && _device == device &&
        (data || (size_t)w_ * h_ * c_ == 0))
        return;
    release();
    w = w_;
    h = h_;
    c = c_;
    dtype = dt;
    layout = ly;
    stride = w_ * h_;
    dims = dims_of(h_, c_);
    _device = device;
    const size_t bytes = len();
    if (bytes == 0) return;
    void* p = device == kHost ? VaAllocator::allocate(bytes) : VaAllocator::allocate_device(bytes, device);
    if (!p) {
        release();
        detail::fail("vision::Tensor::create", device == kHost ? "host allocation failed" : "device allocation failed");
    }
    _block = new Block;
    _block->ptr = p;
    _block->device = device;
    data = p;
}

void Tensor::create(int w_, int h_, int c_, DType dt, DLayout ly) {
    // keeps this tensor's placement (a default-constructed Tensor is host)
    create_on(_device, w_, h_, c_, dt, ly);
}
void Tensor::create(int w_, DType dt, DLayout ly) { create(w_, 1, 1, dt, ly); }
void Tensor::create(int w_, int h_, DType dt, DLayout ly) { create(w_, h_, 1, dt, ly); }
void Tensor::create(int w_, DLayout ly, DType dt) { create(w_, 1, 1, dt, ly); }
void Tensor::create(int w_, int h_, DLayout ly, DType dt) { create(w_, h_, 1, dt, ly); }
void Tensor::create(int w_, int h_, int c_, DLayout ly, DType dt) { create(w_, h_, c_, dt, ly); }

bool Tensor::empty() const { return data == nullptr || size() == 0; }
size_t Tensor::size() const { return (size_t)stride * c; }
size_t Tensor::len() const { return size() * dtype_size(dtype); }
void Tensor::set_name(const std::string& name) { _name = name; }
std::string Tensor::get_name() const { return _name; }
int Tensor::get_ref_count() const { return _block ? _block->refs.load() : 0; }

Tensor Tensor::clone() const {
    if (empty()) return Tensor();
    Tensor t;
    t.create_on(_device, w, h, c, dtype, layout);
    t.dims = dims;
    if (_device == kHost) {
        std::memcpy(t.data, data, len());
    } else {
        detail::Lease lease(_device);
        detail::check_hip("vision::Tensor::clone",
                          hipMemcpyAsync(t.data, data, len(), hipMemcpyDeviceToDevice, lease.stream()));
        lease.sync("vision::Tensor::clone");
    }
    return t;
}

Tensor Tensor::to_device(int device) const {
    if (empty()) return Tensor();
    if (_device == device) return *this;
    Tensor t;
    t.create_on(device, w, h, c, dtype, layout);
    t.dims = dims;
    detail::Lease lease(device);
    const hipMemcpyKind kind = _device == kHost ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice;
    detail::check_hip("vision::Tensor::to_device", hipMemcpyAsync(t.data, data, len(), kind, lease.stream()));
    lease.sync("vision::Tensor::to_device");
    return t;
}

Tensor Tensor::to_host() const {
    if (empty()) return Tensor();
    if (_device == kHost) return *this;
    Tensor t;
    t.create_on(kHost, w, h, c, dtype, layout);
    t.dims = dims;
    detail::Lease lease(_device);
    detail::check_hip("vision::Tensor::to_host",
                      hipMemcpyAsync(t.data, data, len(), hipMemcpyDeviceToHost, lease.stream()));
    lease.sync("vision::Tensor::to_host");
    return t;
}

Tensor Tensor::change_layout(DLayout to) {
    if (empty()) return Tensor();
    if (c == 1 || to == layout) return clone();  // tensor.cpp:398-400
    static const char* fn = "vision::Tensor::change_layout";
    Tensor t;
    detail::Staging st(fn, *this);
    const vacv_image s = st.in(*this, 0);
    const vacv_image d = st.out(t, w, h, c, dtype, to, 1);
    st.run(vacv_change_layout(&s, &d, st.stream()));
    st.finish();
    return t;
}

Tensor Tensor::change_dtype(DType to) {
    if (empty()) return Tensor();
    if (to == dtype) return clone();  // tensor.cpp:464-466
    static const char* fn = "vision::Tensor::change_dtype";
    if (!((dtype == INT8 && to == FP32) || (dtype == FP32 && to == INT8)))
        detail::fail(fn, "only INT8 <-> FP32 is supported (the reference returns an uninitialised tensor)");
    Tensor t;
    detail::Staging st(fn, *this);
    const vacv_image s = st.in(*this, 0);
    const vacv_image d = st.out(t, w, h, c, to, layout, 1);
    st.run(vacv_change_dtype(&s, &d, st.stream()));
    st.finish();
    return t;
}

}  // namespace vision
