// vision::Tensor for the MI355X build of vacv.
//
// Source-compatible with the reference's Tensor (src/common/tensor.h:9-89 of
// b1xian/arm-neon-opencv): same enums and values, same public fields, same
// constructor/create() overload set, same refcounted-copy semantics
// (tensor.cpp:103-144) and the same "create() keeps the buffer when the shape
// already matches" rule (tensor.cpp:512-514).
//
// What is new is placement.  A reference Tensor is always host memory.  Here a
// Tensor is either
//   - HOST   (the default, as in the reference): `data` is a host pointer the
//            caller may read directly.  Buffers come from VaAllocator's pinned
//            pool, so the va_cv:: ops stage them to HBM at DMA speed; or
//   - DEVICE (opt-in: to_device(), create_on()): `data` is an HBM pointer on
//            one GPU.  Chains of va_cv:: ops on device tensors never cross PCIe.
// va_cv:: outputs take the placement of their input.
#ifndef VISION_TENSOR_H
#define VISION_TENSOR_H

#include <cstddef>
#include <memory>
#include <string>
#include <vector>

namespace vision {

/// element type (reference tensor.h:12-18; values are ABI)
enum DType {
    FP32 = 0,
    FP16 = 1,
    INT8 = 2,  // unsigned bytes
    FP64 = 3,
    DTYPE_UNKNOWN
};

/// memory layout (reference tensor.h:21-24)
enum DLayout {
    NCHW = 0,  // planar
    NHWC = 1   // interleaved
};

/// where `data` lives; kHost or a HIP device ordinal (>= 0)
constexpr int kHost = -1;

class Tensor {
public:
    Tensor();
    explicit Tensor(int w, DLayout layout = NCHW, DType dtype = FP32);
    Tensor(int w, int h, DLayout layout = NCHW, DType dtype = FP32);
    Tensor(int w, int h, int c, DLayout layout = NCHW, DType type = FP32);

    explicit Tensor(int w, DType dtype = FP32, DLayout layout = NCHW);
    Tensor(int w, int h, DType dtype = FP32, DLayout layout = NCHW);
    Tensor(int w, int h, int c, DType type = FP32, DLayout layout = NCHW);

    // non-owning views of caller memory (host pointers)
    Tensor(int w, void* data, DType dtype = FP32, DLayout layout = NCHW);
    Tensor(int w, int h, void* data, DType dtype = FP32, DLayout layout = NCHW);
    Tensor(int w, int h, int c, void* data, DType type = FP32, DLayout layout = NCHW);

    Tensor(int w, void* data, DLayout layout = NCHW, DType dtype = FP32);
    Tensor(int w, int h, void* data, DLayout layout = NCHW, DType dtype = FP32);
    Tensor(int w, int h, int c, void* data, DLayout layout = NCHW, DType type = FP32);

    Tensor(const Tensor& t);
    ~Tensor();

    Tensor& operator=(const Tensor& t);
    /// deep copy, same placement
    Tensor clone() const;

    /// HWC <-> CHW / u8 <-> fp32 on the GPU; result has this tensor's placement
    Tensor change_layout(DLayout layout);
    Tensor change_dtype(DType dtype);

    void create(int w, DType dtype = FP32, DLayout layout = NCHW);
    void create(int w, int h, DType dtype = FP32, DLayout layout = NCHW);
    void create(int w, int h, int c, DType dtype = FP32, DLayout layout = NCHW);
    void create(int w, DLayout layout = NCHW, DType dtype = FP32);
    void create(int w, int h, DLayout layout = NCHW, DType dtype = FP32);
    void create(int w, int h, int c, DLayout layout = NCHW, DType dtype = FP32);
    void release();

    bool empty() const;
    size_t size() const;  // elements
    size_t len() const;   // bytes
    void set_name(const std::string& name);
    std::string get_name() const;
    int get_ref_count() const;

    // ---- placement (additions; the reference has host tensors only) -------
    /// kHost, or the device ordinal holding `data`
    int device() const { return _device; }
    bool on_device() const { return _device != kHost; }
    /// create() with an explicit placement (device = kHost or an ordinal);
    /// keeps the buffer when shape, dtype, layout and placement all match
    void create_on(int device, int w, int h, int c, DType dtype, DLayout layout);
    /// copy to HBM of `device` (a no-op share when already there)
    Tensor to_device(int device = 0) const;
    /// copy back to (pinned) host memory (a no-op share when already host)
    Tensor to_host() const;
    /// non-owning view of device memory
    static Tensor device_view(int device, int w, int h, int c, void* data, DType dtype, DLayout layout);

    int w;
    int h;
    int c;
    int stride;  // w * h
    int dims;
    void* data;
    DType dtype;
    DLayout layout;

private:
    struct Block;  // owned storage + refcount (tensor.cpp)
    void retain() const;
    void adopt(const Tensor& t);
    std::string _name;
    Block* _block;
    int _device;
};

using TensorArray = std::vector<Tensor>;
using TensorPtr = std::shared_ptr<Tensor>;

size_t dtype_size(DType dtype);

}  // namespace vision

#endif  // VISION_TENSOR_H
