// membench.hip -- HBM ceilings for the access mixes of the resize kernels.
//
//   hipcc -O3 --offload-arch=gfx950 tools/membench.hip -o tools/membench && tools/membench
//
// Prints one JSON line per pattern: GB/s of (bytes read + bytes written).
//   copy        dense 16-B read + 16-B write (the guide's float4 copy)
//   rows3_read  every third row of 256 1080p u8 frames (the 3x downscale's
//               source traffic, 531 MB), 16-B loads, no writes
//   write_f32   dense 16-B stores of 256 x 640x360x3 fp32 (708 MB)
//   mix         rows3_read and write_f32 in one kernel, each workgroup reading
//               its rows and writing its share of the output (the
//               resize_normalize traffic: 531 MB in + 708 MB out)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <type_traits>
#include <vector>

#define CHECK(x)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                \
        }                                                                                \
    } while (0)

constexpr int kImgs = 256, kW = 1920, kH = 1080, kRowB = kW * 3;
constexpr int64_t kImgB = (int64_t)kRowB * kH;
constexpr int kOutRows = 360, kOutRowB = 640 * 3 * 4;
constexpr int64_t kOutImgB = (int64_t)kOutRowB * kOutRows;

__global__ void copy_kernel(const uint4* __restrict__ a, uint4* __restrict__ b, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// one workgroup per (image, strip of output rows); reads source rows 3r+1,
// G rows' loads in flight per thread group (G * 360 16-B chunks).  Loads and
// stores through buffer resources with cache-policy aux bits LA / SA
// (gfx950: 1 = sc0, 2 = nt, 16 = sc1).
template <int G, int LA, int SA>
__global__ void rows3_kernel(const unsigned char* __restrict__ src, float* __restrict__ dst, uint32_t* sink,
                             int strips, int write) {
    constexpr int kChunks = kRowB / 16;                  // 360
    constexpr int kL = (G * kChunks + 255) / 256;        // loads per thread per group
    const int img = blockIdx.x / strips, strip = blockIdx.x % strips;
    const int rows_per = kOutRows / strips;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(src + img * kImgB), (short)0, (int)kImgB, 0x00020000);
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)((unsigned char*)dst + img * kOutImgB), (short)0, (int)kOutImgB, 0x00020000);
    uint32_t acc = 0;
    const int r1 = (strip + 1) * rows_per;
    for (int r0 = strip * rows_per; r0 < r1; r0 += G) {
        u32x4 v[kL];
#pragma unroll
        for (int q = 0; q < kL; ++q) {
            const int k = threadIdx.x + q * 256;
            const int r = r0 + k / kChunks;
            v[q] = u32x4{0, 0, 0, 0};
            if (k < G * kChunks && r < r1)
                v[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, (3 * r + 1) * kRowB + (k % kChunks) * 16, 0, LA);
        }
#pragma unroll
        for (int q = 0; q < kL; ++q) acc ^= v[q].x ^ v[q].y ^ v[q].z ^ v[q].w;
        if (write) {
            constexpr int kOC = kOutRowB / 16;           // 480
            for (int k = threadIdx.x; k < G * kOC; k += 256) {
                const int r = r0 + k / kOC;
                if (r < r1) {
                    u32x4 d = {acc, (uint32_t)k, (uint32_t)r, (uint32_t)img};
                    __builtin_amdgcn_raw_buffer_store_b128(d, rd, r * kOutRowB + (k % kOC) * 16, 0, SA);
                }
            }
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void write_kernel(uint4* __restrict__ b, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        b[i] = make_uint4((uint32_t)i, 1, 2, 3);
}

__global__ void write_nt_kernel(uint4* __restrict__ b, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(u32x4{(uint32_t)i, 1, 2, 3}, reinterpret_cast<u32x4*>(b) + i);
}

__global__ void copy_nt_kernel(const uint4* __restrict__ a, uint4* __restrict__ b, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a) + i), reinterpret_cast<u32x4*>(b) + i);
}

template <typename F>
float time_ms(F f, int iters) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    f();
    CHECK(hipDeviceSynchronize());
    std::vector<float> t;
    for (int i = 0; i < iters; ++i) {
        CHECK(hipEventRecord(e0));
        f();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main() {
    unsigned char* src;
    float* dst;
    uint32_t* sink;
    CHECK(hipMalloc(&src, kImgs * kImgB));
    CHECK(hipMalloc(&dst, kImgs * kOutImgB));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(src, 1, kImgs * kImgB));
    auto report = [](const char* name, double bytes, float ms) {
        std::printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, bytes / ms / 1e6);
    };
    const int64_t ncopy = (int64_t)kImgs * kOutImgB / 16;  // 708 MB each way
    report("copy", 2.0 * ncopy * 16, time_ms([&] { copy_kernel<<<8192, 256>>>((const uint4*)src, (uint4*)dst, ncopy); }, 20));
    const double rd = (double)kImgs * kOutRows * kRowB, wr = (double)kImgs * kOutImgB;
    auto run = [&](auto gtag, auto ltag, auto stag, int strips, bool wr_on) {
        constexpr int G = decltype(gtag)::value, LA = decltype(ltag)::value, SA = decltype(stag)::value;
        char nm[96];
        std::snprintf(nm, sizeof nm, "%s_g%d_s%d_la%d_sa%d", wr_on ? "mix" : "rows3_read", G, strips, LA, SA);
        report(nm, wr_on ? rd + wr : rd,
               time_ms([&] { rows3_kernel<G, LA, SA><<<kImgs * strips, 256>>>(src, dst, sink, strips, wr_on); }, 20));
    };
    using I1 = std::integral_constant<int, 1>;
    using I5 = std::integral_constant<int, 5>;
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    using P2 = std::integral_constant<int, 2>;
    using P3 = std::integral_constant<int, 3>;
    using P16 = std::integral_constant<int, 16>;
    using P18 = std::integral_constant<int, 18>;
    for (int strips : {4, 8}) {
        run(I5{}, P0{}, P0{}, strips, false);
        run(I5{}, P2{}, P0{}, strips, false);
        run(I5{}, P0{}, P0{}, strips, true);
        run(I5{}, P2{}, P0{}, strips, true);
        run(I5{}, P0{}, P2{}, strips, true);
        run(I5{}, P2{}, P2{}, strips, true);
        run(I5{}, P0{}, P1{}, strips, true);
        run(I5{}, P0{}, P3{}, strips, true);
        run(I5{}, P0{}, P16{}, strips, true);
        run(I5{}, P0{}, P18{}, strips, true);
        run(I1{}, P0{}, P2{}, strips, true);
    }
    report("write_f32", wr, time_ms([&] { write_kernel<<<8192, 256>>>((uint4*)dst, ncopy); }, 20));
    report("write_f32_nt", wr, time_ms([&] { write_nt_kernel<<<8192, 256>>>((uint4*)dst, ncopy); }, 20));
    report("write_f32_2048", wr, time_ms([&] { write_kernel<<<2048, 256>>>((uint4*)dst, ncopy); }, 20));
    report("copy_nt", 2.0 * ncopy * 16, time_ms([&] { copy_nt_kernel<<<8192, 256>>>((const uint4*)src, (uint4*)dst, ncopy); }, 20));
    CHECK(hipFree(src));
    CHECK(hipFree(dst));
    CHECK(hipFree(sink));
    return 0;
}
