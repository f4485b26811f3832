// pcie_bench.cpp -- the PCIe-inclusive rate of the source-compatible C++
// layer on HOST tensors: 1080p u8 frames ->
// va_cv::resize_normalize(640x360, mean/std) -> host fp32, measured
//   percall  one va_cv:: call per frame (H2D, kernel, D2H serialised on one
//            leased stream: the reference's calling convention)
//   batched  the batched overload (FramePipeline: H2D / kernel / D2H of
//            consecutive frames overlapped on three streams)
// next to the link itself: pinned hipMemcpyAsync H2D alone, D2H alone, and
// both directions at once.  One JSON line; wall clock (steady_clock).
//   make -C tools pcie_bench && tools/pcie_bench [frames]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../arm-neon-opencv_amd/src/cv/cv.h"

using namespace vision;
using clk = std::chrono::steady_clock;

static double ms_since(clk::time_point t0) {
    return std::chrono::duration<double, std::milli>(clk::now() - t0).count();
}

#define CHECK(x)                                                                            \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
            std::exit(1);                                                                   \
        }                                                                                   \
    } while (0)

int main(int argc, char** argv) {
    const int n = argc > 1 ? std::atoi(argv[1]) : 64;
    const size_t in_b = 1920 * 1080 * 3, out_b = 640 * 360 * 3 * 4;
    std::vector<Tensor> src(n);
    for (int i = 0; i < n; ++i) {
        src[i] = Tensor(1920, 1080, 3, INT8, NHWC);
        unsigned char* p = static_cast<unsigned char*>(src[i].data);
        uint64_t s = 0x9E3779B97F4A7C15ull * (i + 1);
        for (size_t b = 0; b < in_b; ++b) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            p[b] = (unsigned char)s;
        }
    }
    Tensor mean(3, 1, 1, FP32, NHWC), stdv(3, 1, 1, FP32, NHWC);
    const float mv[3] = {103.94f, 116.78f, 123.68f}, sv[3] = {57.375f, 57.12f, 58.395f};
    std::memcpy(mean.data, mv, sizeof(mv));
    std::memcpy(stdv.data, sv, sizeof(sv));

    // the link: pinned copies of the same byte counts
    void *d_in, *d_out, *h_out;
    CHECK(hipMalloc(&d_in, in_b * 4));
    CHECK(hipMalloc(&d_out, out_b * 4));
    CHECK(hipHostMalloc(&h_out, out_b * n, hipHostMallocDefault));
    hipStream_t s1, s2;
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    auto h2d = [&](hipStream_t s) {
        for (int i = 0; i < n; ++i) CHECK(hipMemcpyAsync((char*)d_in + (i % 4) * in_b, src[i].data, in_b, hipMemcpyHostToDevice, s));
    };
    auto d2h = [&](hipStream_t s) {
        for (int i = 0; i < n; ++i) CHECK(hipMemcpyAsync((char*)h_out + i * out_b, (char*)d_out + (i % 4) * out_b, out_b, hipMemcpyDeviceToHost, s));
    };
    h2d(s1); d2h(s2);
    CHECK(hipDeviceSynchronize());
    auto t0 = clk::now();
    h2d(s1);
    CHECK(hipStreamSynchronize(s1));
    const double ms_h2d = ms_since(t0);
    t0 = clk::now();
    d2h(s2);
    CHECK(hipStreamSynchronize(s2));
    const double ms_d2h = ms_since(t0);
    t0 = clk::now();
    h2d(s1);
    d2h(s2);
    CHECK(hipStreamSynchronize(s1));
    CHECK(hipStreamSynchronize(s2));
    const double ms_both = ms_since(t0);

    // the copy structure alone, hipMemsetAsync standing in for the kernel:
    //  chain3  three streams (H2D | kernel | D2H), a 3-slot ring, events both ways
    //  chain2  two streams: H2D(i) then the kernel(i) in order on one, D2H on
    //          the other after the kernel's event; a 3-slot ring
    //  chain2n chain2 without slot reuse (n buffers): no backward waits
    double ms_chain[3] = {0, 0, 0};
    {
        hipStream_t a, b, c;
        CHECK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
        CHECK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
        CHECK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
        std::vector<hipEvent_t> e1(n), e2(n), e3(n);
        for (int k = 0; k < n; ++k) {
            CHECK(hipEventCreateWithFlags(&e1[k], hipEventDisableTiming));
            CHECK(hipEventCreateWithFlags(&e2[k], hipEventDisableTiming));
            CHECK(hipEventCreateWithFlags(&e3[k], hipEventDisableTiming));
        }
        void* big_in;
        void* big_out;
        CHECK(hipMalloc(&big_in, in_b * n));
        CHECK(hipMalloc(&big_out, out_b * n));
        for (int mode = 0; mode < 3; ++mode) {
            for (int rep = 0; rep < 2; ++rep) {
                CHECK(hipDeviceSynchronize());
                t0 = clk::now();
                for (int i = 0; i < n; ++i) {
                    const int k = mode == 2 ? i : i % 3;
                    char* din = mode == 2 ? (char*)big_in + (size_t)i * in_b : (char*)d_in + k * in_b;
                    char* dout = mode == 2 ? (char*)big_out + (size_t)i * out_b : (char*)d_out + k * out_b;
                    if (mode == 0) {
                        if (i >= 3) CHECK(hipStreamWaitEvent(a, e2[k], 0));
                        CHECK(hipMemcpyAsync(din, src[i].data, in_b, hipMemcpyHostToDevice, a));
                        CHECK(hipEventRecord(e1[k], a));
                        CHECK(hipStreamWaitEvent(b, e1[k], 0));
                        if (i >= 3) CHECK(hipStreamWaitEvent(b, e3[k], 0));
                        CHECK(hipMemsetAsync(dout, i, 4096, b));
                        CHECK(hipEventRecord(e2[k], b));
                        CHECK(hipStreamWaitEvent(c, e2[k], 0));
                        CHECK(hipMemcpyAsync((char*)h_out + i * out_b, dout, out_b, hipMemcpyDeviceToHost, c));
                        CHECK(hipEventRecord(e3[k], c));
                    } else {
                        if (mode == 1 && i >= 3) CHECK(hipStreamWaitEvent(a, e3[k], 0));
                        CHECK(hipMemcpyAsync(din, src[i].data, in_b, hipMemcpyHostToDevice, a));
                        CHECK(hipMemsetAsync(dout, i, 4096, a));
                        CHECK(hipEventRecord(e2[k], a));
                        CHECK(hipStreamWaitEvent(c, e2[k], 0));
                        CHECK(hipMemcpyAsync((char*)h_out + i * out_b, dout, out_b, hipMemcpyDeviceToHost, c));
                        CHECK(hipEventRecord(e3[k], c));
                    }
                }
                CHECK(hipDeviceSynchronize());
                ms_chain[mode] = ms_since(t0);
            }
        }
        CHECK(hipFree(big_in));
        CHECK(hipFree(big_out));
    }

    // the operator, warmed up first
    std::vector<Tensor> out_a(n), out_b2;
    for (int w = 0; w < n; ++w)  // allocates every output (pinned host) before the timed loops
        va_cv::resize_normalize(src[w], out_a[w], va_cv::VSize(640, 360), 0, 0, va_cv::INTER_LINEAR, mean, stdv);
    va_cv::resize_normalize(src, out_b2, va_cv::VSize(640, 360), 0, 0, va_cv::INTER_LINEAR, mean, stdv);
    t0 = clk::now();
    for (int i = 0; i < n; ++i)
        va_cv::resize_normalize(src[i], out_a[i], va_cv::VSize(640, 360), 0, 0, va_cv::INTER_LINEAR, mean, stdv);
    const double ms_percall = ms_since(t0);
    t0 = clk::now();
    va_cv::resize_normalize(src, out_b2, va_cv::VSize(640, 360), 0, 0, va_cv::INTER_LINEAR, mean, stdv);
    const double ms_batched = ms_since(t0);
    int same = 1;
    for (int i = 0; i < n; ++i) same &= std::memcmp(out_a[i].data, out_b2[i].data, out_b) == 0;

    const double gb = (double)n * (in_b + out_b) / 1e9;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    std::printf("{\"what\": \"va_cv::resize_normalize 1920x1080x3 u8 -> 640x360x3 fp32, HOST tensors (PCIe-inclusive)\", "
                "\"device\": \"%s\", \"frames\": %d, \"bytes_per_frame\": %zu, "
                "\"link_h2d_GBps\": %.1f, \"link_d2h_GBps\": %.1f, \"link_both_GBps\": %.1f, \"chain3_ms_per_frame\": %.4f, \"chain2_ms_per_frame\": %.4f, \"chain2n_ms_per_frame\": %.4f, "
                "\"percall_ms_per_frame\": %.4f, \"percall_GBps\": %.1f, \"percall_Mpx_s\": %.1f, "
                "\"batched_ms_per_frame\": %.4f, \"batched_GBps\": %.1f, \"batched_Mpx_s\": %.1f, "
                "\"batched_equals_percall\": %s}\n",
                prop.name, n, in_b + out_b, n * in_b / 1e6 / ms_h2d, n * out_b / 1e6 / ms_d2h,
                gb * 1e3 / ms_both, ms_chain[0] / n, ms_chain[1] / n, ms_chain[2] / n, ms_percall / n, gb * 1e3 / ms_percall, n * 1920.0 * 1080 / 1e3 / ms_percall,
                ms_batched / n, gb * 1e3 / ms_batched, n * 1920.0 * 1080 / 1e3 / ms_batched, same ? "true" : "false");
    return same ? 0 : 1;
}
