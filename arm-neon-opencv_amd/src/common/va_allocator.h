// Host and device buffer pools behind vision::Tensor.
//
// The reference allocates every Tensor with malloc, or -- its unfinished
// USE_CUDA direction -- with mapped pinned memory (va_allocator.cpp:12-31,
// cuda.md).  Here:
//   - host buffers are page-locked (hipHostMalloc) so staging them to HBM runs
//     at DMA speed, and recycled through a size-class pool because pinning is
//     expensive (milliseconds per call); without a HIP device (build/CPU test
//     hosts) they fall back to aligned malloc;
//   - device buffers are hipMalloc'd HBM, recycled the same way (hipMalloc and
//     hipFree synchronise).
// Pools are process-wide and thread-safe.  trim() returns cached blocks.
#ifndef VISION_VA_ALLOCATOR_H
#define VISION_VA_ALLOCATOR_H

#include <cstddef>

namespace vision {

class VaAllocator {
public:
    /// host buffer of >= len bytes, 64-byte aligned; nullptr on failure
    static void* allocate(size_t len);
    static void deallocate(void* ptr);

    /// HBM buffer of >= len bytes on `device`; nullptr on failure
    static void* allocate_device(size_t len, int device);
    static void deallocate_device(void* ptr, int device);

    /// round up to a multiple of n (n a power of two), as va_allocator.cpp:37-39
    static size_t align_size(size_t sz, size_t n);

    /// true when host buffers are page-locked (a HIP device is present and
    /// VACV_PINNED_HOST is not "0")
    static bool host_pinned();

    /// free every cached (unused) block, host and device
    static void trim();

    /// bytes currently cached (unused) in the pools
    static size_t cached_host_bytes();
    static size_t cached_device_bytes();
};

}  // namespace vision

#endif  // VISION_VA_ALLOCATOR_H
