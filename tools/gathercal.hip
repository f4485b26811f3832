// gathercal.hip -- the vector-memory cost of the warp sampler's tap gathers as
// a function of their shape: per wave instruction, 64 lanes load W dwords
// (buffer_load_dword{,x2,x3,x4}, dword-aligned) from R source rows, 64/R lanes
// per row at a byte step S (6 = two 3-channel pixels), the rows PITCH bytes
// apart.  The working set (WS bytes) is L1- or L2-resident, so the time is the
// TA/TD/TCP cost of the instruction stream, not HBM.  Prints one JSON line per
// shape: cycles per wave instruction per CU at 2.4 GHz.
//   hipcc -O3 --offload-arch=gfx950 tools/gathercal.hip -o tools/gathercal
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

constexpr int kIters = 256;
constexpr int kUnroll = 8;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <int W>
__global__ __launch_bounds__(256) void gpat(const unsigned char* buf, uint32_t ws, int R, int step, int pitch, unsigned* sink) {
    const auto r = rsrc(buf, ws + 64);
    const int lane = threadIdx.x & 63;
    const int wave = (int)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int per = 64 / R;
    // per-lane offset fixed; the wave's base moves in the scalar soffset, so
    // the loop costs no vector ALU per load
    const uint32_t lo = (uint32_t)((lane / per) * pitch + (lane % per) * step) & ~3u;
    const uint32_t span = (ws - (uint32_t)(R * pitch + per * step + 16) - 8u * 1556u) & ~1023u;  // multiple of 1 KiB
    uint32_t base = __builtin_amdgcn_readfirstlane(((uint32_t)wave * 40960u) % span);
    unsigned acc = 0;
    for (int it = 0; it < kIters; it += kUnroll) {
#pragma unroll
        for (int u = 0; u < kUnroll; ++u) {
            const uint32_t so = base + (uint32_t)u * 1556u;  // < span + 8 * 1556
            if constexpr (W == 1) {
                acc ^= (unsigned)__builtin_amdgcn_raw_buffer_load_b32(r, (int)lo, (int)so, 0);
            } else if constexpr (W == 2) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)lo, (int)so, 0);
                acc ^= v[0] ^ v[1];
            } else if constexpr (W == 3) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b96(r, (int)lo, (int)so, 0);
                acc ^= v[0] ^ v[1] ^ v[2];
            } else {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)lo, (int)so, 0);
                acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
            }
        }
        base += 8u * 1556u;
        base = base >= span ? base - span : base;
    }
    if (acc == 0x9E3779B9u) sink[wave] = acc;
}

template <int W>
double run(const unsigned char* buf, uint32_t ws, int R, int step, int pitch, unsigned* sink, int blocks) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL(gpat<W>, dim3(blocks), dim3(256), 0, 0, buf, ws, R, step, pitch, sink);
    CHECK(hipEventRecord(a));
    constexpr int kReps = 5;
    for (int i = 0; i < kReps; ++i) hipLaunchKernelGGL(gpat<W>, dim3(blocks), dim3(256), 0, 0, buf, ws, R, step, pitch, sink);
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    const double instr_per_cu = (double)blocks * 4 * kIters / 256.0;
    return ms / kReps * 1e-3 * 2.4e9 / instr_per_cu;
}

int main(int argc, char** argv) {
    const int blocks = 256 * 8 * 4;  // 8 waves per SIMD
    unsigned char* buf;
    unsigned* sink;
    const uint32_t big = 64u << 20;
    CHECK(hipMalloc(&buf, big + 4096));
    CHECK(hipMemset(buf, 7, big + 4096));
    CHECK(hipMalloc(&sink, blocks * 4 * sizeof(unsigned)));
    // (working set, row pitch): L1-resident rows 256 B apart; L2-resident 1280x3 rows
    const uint32_t wss[] = {32u << 10, 2u << 20};
    const int pitches[] = {256, 3840};
    const int Rs[] = {1, 2, 4, 8, 16, 32, 64};
    for (int wi = 0; wi < 2; ++wi) {
        const uint32_t ws = wss[wi];
        const int pitch = pitches[wi];
        for (int step : {3, 6, 12}) {
            for (int R : Rs) {
                const double c1 = run<1>(buf, ws, R, step, pitch, sink, blocks);
                const double c2 = run<2>(buf, ws, R, step, pitch, sink, blocks);
                const double c3 = run<3>(buf, ws, R, step, pitch, sink, blocks);
                const double c4 = run<4>(buf, ws, R, step, pitch, sink, blocks);
                std::printf("{\"ws_bytes\": %u, \"pitch\": %d, \"step\": %d, \"rows\": %d, \"cyc_b32\": %.2f, \"cyc_b64\": %.2f, "
                            "\"cyc_b96\": %.2f, \"cyc_b128\": %.2f}\n",
                            ws, pitch, step, R, c1, c2, c3, c4);
                std::fflush(stdout);
            }
        }
    }
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    return 0;
}
