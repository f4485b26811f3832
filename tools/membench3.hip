// membench3.hip -- the streaming ceiling for cfg3's traffic (NV21 1080p ->
// BGR fp32: 3,110,400 B read + 24,883,200 B written per frame, 256 frames):
// write-only and 1:8 read:write streams of that size, 16-B nt accesses.
//   hipcc -O3 --offload-arch=gfx950 tools/membench3.hip -o tools/membench3 && tools/membench3
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                \
        }                                                                                \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, int POL>
__global__ __launch_bounds__(256) void write_k(u32x4* __restrict__ b, int64_t n) {
    const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const int64_t i = base + (int64_t)k * 256;
        const u32x4 v = {(unsigned)i, 1u, 2u, 3u};
        if (i < n) {
            if (POL) __builtin_nontemporal_store(v, b + i);
            else b[i] = v;
        }
    }
}

// each thread: one 16-B chunk read, W chunks written (cfg3: W = 8)
template <int W, int POL>
__global__ __launch_bounds__(256) void mix_k(const u32x4* __restrict__ a, u32x4* __restrict__ b, int64_t n_in) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n_in) return;
    const u32x4 v = __builtin_nontemporal_load(a + i);
    const int64_t o = (int64_t)blockIdx.x * 256 * W + threadIdx.x;
#pragma unroll
    for (int k = 0; k < W; ++k) {
        const u32x4 w = {v.x + k, v.y, v.z, v.w};
        if (POL) __builtin_nontemporal_store(w, b + o + 256 * k);
        else b[o + 256 * k] = w;
    }
}

// 1:4 (dtype u8 -> fp32): A = 4 B read / 16 B written per thread (the dtype
// kernel's shape); B = 16 B read / 4 x 16 B written per thread, every store
// instruction 1 KiB contiguous per wave.  RP / WP: non-temporal loads / stores.
template <int RP, int WP>
__global__ __launch_bounds__(256) void mixA_k(const uint32_t* __restrict__ a, u32x4* __restrict__ b, int64_t n4) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const uint32_t w = RP ? __builtin_nontemporal_load(a + i) : a[i];
    const u32x4 f = {w & 0xFF, (w >> 8) & 0xFF, (w >> 16) & 0xFF, w >> 24};
    if (WP) __builtin_nontemporal_store(f, b + i);
    else b[i] = f;
}
template <int RP, int WP>
__global__ __launch_bounds__(256) void mixB_k(const u32x4* __restrict__ a, u32x4* __restrict__ b, int64_t n16) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n16) return;
    const u32x4 w = RP ? __builtin_nontemporal_load(a + i) : a[i];
    const int64_t o = (int64_t)blockIdx.x * 1024 + threadIdx.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const u32x4 f = {w[k] & 0xFF, (w[k] >> 8) & 0xFF, (w[k] >> 16) & 0xFF, w[k] >> 24};
        if (WP) __builtin_nontemporal_store(f, b + o + 256 * k);
        else b[o + 256 * k] = f;
    }
}

template <typename F>
float time_ms(F f, int iters) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    f();
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
    const int64_t wbytes = (int64_t)256 * 24883200, rbytes = (int64_t)256 * 3110400;
    const int64_t nw = wbytes / 16, nr = rbytes / 16;
    u32x4 *a, *b;
    CHECK(hipMalloc(&a, rbytes));
    CHECK(hipMalloc(&b, wbytes));
    CHECK(hipMemset(a, 1, rbytes));
    auto rep = [&](const char* what, int u, int pol, double by, float ms) {
        std::printf("{\"pattern\": \"%s\", \"U\": %d, \"policy\": %d, \"ms\": %.4f, \"GBps\": %.1f, \"frac_8TBps\": %.4f}\n",
                    what, u, pol, ms, by / ms / 1e6, by / ms / 1e6 / 8000.0);
        std::fflush(stdout);
    };
    rep("write", 1, 1, (double)wbytes, time_ms([&] { write_k<1, 1><<<(unsigned)((nw + 255) / 256), 256>>>(b, nw); }, 15));
    rep("write", 4, 1, (double)wbytes, time_ms([&] { write_k<4, 1><<<(unsigned)((nw + 1023) / 1024), 256>>>(b, nw); }, 15));
    rep("write", 1, 0, (double)wbytes, time_ms([&] { write_k<1, 0><<<(unsigned)((nw + 255) / 256), 256>>>(b, nw); }, 15));
    rep("mix1:8", 8, 1, (double)(wbytes + rbytes), time_ms([&] { mix_k<8, 1><<<(unsigned)((nr + 255) / 256), 256>>>(a, b, nr); }, 15));
    rep("mix1:8", 8, 0, (double)(wbytes + rbytes), time_ms([&] { mix_k<8, 0><<<(unsigned)((nr + 255) / 256), 256>>>(a, b, nr); }, 15));
    {
        const int64_t rb = (int64_t)64 * 1920 * 1080 * 3, n4 = rb / 4, n16 = rb / 16;
        const double by = (double)rb * 5;
        rep("dtypeA", 1, 11, by, time_ms([&] { mixA_k<1, 1><<<(unsigned)((n4 + 255) / 256), 256>>>((const uint32_t*)a, b, n4); }, 15));
        rep("dtypeA", 1, 1, by, time_ms([&] { mixA_k<0, 1><<<(unsigned)((n4 + 255) / 256), 256>>>((const uint32_t*)a, b, n4); }, 15));
        rep("dtypeA", 1, 10, by, time_ms([&] { mixA_k<1, 0><<<(unsigned)((n4 + 255) / 256), 256>>>((const uint32_t*)a, b, n4); }, 15));
        rep("dtypeB", 4, 11, by, time_ms([&] { mixB_k<1, 1><<<(unsigned)((n16 + 255) / 256), 256>>>(a, b, n16); }, 15));
        rep("dtypeB", 4, 10, by, time_ms([&] { mixB_k<1, 0><<<(unsigned)((n16 + 255) / 256), 256>>>(a, b, n16); }, 15));
    }
    return 0;
}
