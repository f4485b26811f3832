// fetchcal.hip -- calibrates rocprofv3's FETCH_SIZE for the access shapes the
// vacv gather kernels use (MI355X_MICROARCH.md: FETCH_SIZE is calibrated only
// for 16-byte-per-lane streaming reads, where it reads 1/2 of the bytes).
// Each kernel reads a KNOWN set of bytes, once, from buffers far larger than
// the 256 MiB Infinity Cache, and writes one dword per workgroup:
//   stream16   16 B per lane, lane-consecutive: N bytes
//   gather8    unaligned 8-byte loads at a 9-byte stride (the headline's tap
//              loads), every third 5,760-byte row of 1080p frames, never past a
//              row's last byte: exactly the rows' bytes
//   gather8al  8-byte loads at an 8-byte stride (dense, aligned): N bytes
// Run under `rocprofv3 --pmc FETCH_SIZE --kernel-trace`; the per-dispatch
// FETCH_SIZE (KB) divided by the bytes printed here is the correction.
//   hipcc -O3 --offload-arch=gfx950 tools/fetchcal.hip -o tools/fetchcal
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                            \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void stream16(const u32x4* __restrict__ a, unsigned* sink, int64_t n16) {
    unsigned acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (int64_t)gridDim.x * 256) {
        const u32x4 v = __builtin_nontemporal_load(a + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

// one workgroup per (image, output row): 640 pixels, tap bytes 9x+3 .. 9x+10 of
// source row 3y+1 (5,760 bytes), the last pixel pulled back to end at byte 5759
__global__ __launch_bounds__(256) void gather8(const unsigned char* __restrict__ src, unsigned* sink) {
    const int row = blockIdx.x;             // image * 360 + y
    const int img = row / 360, y = row - img * 360;
    const unsigned char* r = src + (int64_t)img * 6220800 + (int64_t)(3 * y + 1) * 5760;
    unsigned acc = 0;
    for (int x = threadIdx.x; x < 640; x += 256) {
        int off = 9 * x + 3;
        if (off + 8 > 5760) off = 5760 - 8;
        uint64_t v;
        __builtin_memcpy(&v, r + off, 8);
        acc ^= (unsigned)v ^ (unsigned)(v >> 32);
    }
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void gather8al(const uint2* __restrict__ a, unsigned* sink, int64_t n8) {
    unsigned acc = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
        const uint2 v = a[i];
        acc ^= v.x ^ v.y;
    }
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

int main() {
    const int64_t frames = 256, frame = 6220800;  // 1080p u8 x3
    const int64_t bytes = frames * frame;          // 1.59 GB
    unsigned char* buf;
    unsigned* sink;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&sink, 1 << 22));
    CHECK(hipMemset(buf, 1, bytes));
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(stream16, dim3(4096), dim3(256), 0, 0, (const u32x4*)buf, sink, bytes / 16);
        hipLaunchKernelGGL(gather8, dim3((unsigned)(frames * 360)), dim3(256), 0, 0, buf, sink);
        hipLaunchKernelGGL(gather8al, dim3(4096), dim3(256), 0, 0, (const uint2*)buf, sink, bytes / 8);
    }
    CHECK(hipDeviceSynchronize());
    std::printf("{\"stream16_bytes\": %lld, \"gather8_bytes\": %lld, \"gather8al_bytes\": %lld}\n", (long long)bytes,
                (long long)(frames * 360 * 5760), (long long)bytes);
    return 0;
}
