// Internal: per-device HIP streams and staging scratch for the C++ layer.
// Not installed with the public headers.
#ifndef VACV_HIP_CONTEXT_H
#define VACV_HIP_CONTEXT_H

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <functional>
#include <vector>

#include "../../../include/vacv_hip.h"
#include "tensor.h"

namespace vision {
namespace detail {

/// Throws std::runtime_error("<fn>: <reason>") when status != VACV_OK.
void check(const char* fn, int status);
void check_hip(const char* fn, hipError_t e);
[[noreturn]] void fail(const char* fn, const char* why);

/// The device an op on `t` runs on: its own for device tensors, else the
/// calling thread's current HIP device.
int compute_device(const Tensor& t);

/// A stream plus grow-only HBM scratch slots on one device, leased from a
/// process-wide pool for the duration of one operator call (so concurrent
/// callers never share a stream or scratch).  Makes `device` current for the
/// lease and restores the previous device afterwards.
class Lease {
public:
    explicit Lease(int device);
    ~Lease();
    Lease(const Lease&) = delete;
    Lease& operator=(const Lease&) = delete;

    int device() const { return _device; }
    hipStream_t stream() const;
    /// HBM scratch of >= bytes in slot 0..kSlots-1 (contents undefined)
    void* scratch(int slot, size_t bytes);
    /// wait for everything queued on the stream; throws on a HIP error
    void sync(const char* fn);

    static constexpr int kSlots = 4;
    struct Ctx;  // stream + scratch, defined in hip_context.cpp

private:
    Ctx* _ctx;
    int _device;
    int _prev;
};

/// Descriptor of a dense single image (n = 1) at `data`.
vacv_image describe(const Tensor& t, void* data);
inline vacv_image describe(const Tensor& t) { return describe(t, t.data); }

/// One operator call: leases the compute device's stream, gives the kernels
/// HBM views of every operand, and moves host operands across PCIe.
///   in():  a device tensor is used in place; a host tensor is copied
///          (hipMemcpyAsync, DMA from the pinned pool) into scratch.
///   out(): creates `dst` with the anchor's placement (the reference's
///          dst.create, tensor.cpp:512-540); a host dst gets a scratch HBM
///          buffer whose bytes finish() copies back.
///   finish(): queues the copies back and waits for the stream -- the
///          reference's ops are synchronous and so are these.
/// Inputs are kept alive (refcount) until finish(), so `dst` may alias `src`.
class Staging {
public:
    Staging(const char* fn, const Tensor& anchor);
    /// on an early exit (exception) waits for queued work before the kept
    /// operands are released
    ~Staging();
    Staging(const Staging&) = delete;
    Staging& operator=(const Staging&) = delete;
    vacv_image in(const Tensor& t, int slot);
    /// keep = the kernel reads dst's current bytes (BORDER_TRANSPARENT): a
    /// host dst is first copied into its device scratch
    vacv_image out(Tensor& dst, int w, int h, int c, DType dtype, DLayout layout, int slot, bool keep = false);
    /// fail loudly on a non-OK status from the C ABI
    void run(int status) { check(_fn, status); }
    void finish();
    hipStream_t stream() const { return _lease.stream(); }
    int placement() const { return _placement; }

private:
    struct Copy {
        void* host;
        const void* dev;
        size_t bytes;
    };
    const char* _fn;
    int _placement;
    Lease _lease;
    std::vector<Tensor> _keep;
    std::vector<Copy> _d2h;
};

/// A sequence of frames through the same operator with the PCIe copies
/// overlapped (the batched va_cv:: entry points).  Host
/// frames go through a ring of kRing HBM slot pairs on two streams: H2D(i)
/// and kernel(i) in order on one, D2H(i) on the other behind the kernel's
/// event, so the H2D of frame i+1 runs while frame i's result comes back;
/// the host waits for a slot's previous frame before reusing it.  Device
/// frames skip their copies.  Every operand is kept alive until finish(),
/// which waits for both streams.
class FramePipeline {
public:
    using Launch = std::function<int(const vacv_image& src, const vacv_image& dst, hipStream_t stream)>;
    FramePipeline(const char* fn, int device);
    ~FramePipeline();
    FramePipeline(const FramePipeline&) = delete;
    FramePipeline& operator=(const FramePipeline&) = delete;
    /// queue one frame: dst is created (placement of src) as (w, h, c, dtype,
    /// layout) and written by launch() on the compute stream
    void frame(const Tensor& src, Tensor& dst, int w, int h, int c, DType dtype, DLayout layout,
               const Launch& launch);
    void finish();

    static constexpr int kRing = 6;
    struct Ctx;  // streams, events and the slot ring (hip_context.cpp)

private:
    const char* _fn;
    int _device;
    int _prev;
    Ctx* _ctx;
    long _count;
    std::vector<Tensor> _keep;
};

}  // namespace detail
}  // namespace vision

#endif  // VACV_HIP_CONTEXT_H
