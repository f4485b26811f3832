// segbench.hip -- what HBM delivers when a kernel moves a frame batch as 2D
// tiles whose rows are SHORT segments (the access pattern of the warp boxes
// and the two-tap resize strips: 200-320 B per row at a 3840-5760 B pitch),
// against whole-row streams.
//
//   hipcc -O3 --offload-arch=gfx950 tools/segbench.hip -o tools/segbench && tools/segbench
// Each workgroup (256 threads) copies one tile of TR rows x L bytes of one
// frame (16-byte lanes, each row's segment split over the lanes), tiles in
// row-major order within a frame, frames outer, blocks dealt XCD-contiguously
// (as the vacv kernels do).  One JSON line per (L, TR, mode): GB/s of bytes
// read + written.  mode 0 copy, 1 read only (a checksum written per tile),
// 2 read by LDS-DMA, 3 write only (16 bytes per lane), 4 write only (4 bytes
// per lane: the store width of the u8 strip / area kernels).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void seg_copy(const unsigned char* src, unsigned char* dst, int frames, int H,
                                                int pitch, int L, int TR, int tiles_x, int tiles_y, int mode,
                                                unsigned* sink) {
    const int total = frames * tiles_x * tiles_y;
    const int per_xcd = (total + 7) / 8;
    const int id = (int)(blockIdx.x % 8) * per_xcd + (int)(blockIdx.x / 8);
    if (id >= total) return;
    const int f = id / (tiles_x * tiles_y), t = id - f * tiles_x * tiles_y;
    const int ty = t / tiles_x, tx = t - ty * tiles_x;
    const int chunks = L / 16;  // per row
    const int64_t fbase = (int64_t)f * H * pitch;
    unsigned acc = 0;
    if (mode == 4) {  // dword e of the tile (row-major), lanes contiguous
        const int dw = L / 4;
        for (int e = threadIdx.x; e < TR * dw; e += 256) {
            const int r = e / dw, c = e - r * dw;
            const int row = ty * TR + r;
            if (row >= H) break;
            __builtin_nontemporal_store((unsigned)e, reinterpret_cast<unsigned*>(dst + fbase + (int64_t)row * pitch + (int64_t)tx * L + 4 * c));
        }
        return;
    }
    for (int e = threadIdx.x; e < TR * chunks; e += 256) {
        const int r = e / chunks, c = e - r * chunks;
        const int row = ty * TR + r;
        if (row >= H) break;
        const int64_t off = fbase + (int64_t)row * pitch + (int64_t)tx * L + 16 * c;
        if (mode == 3) {
            __builtin_nontemporal_store(u32x4{(unsigned)e, 1u, 2u, 3u}, reinterpret_cast<u32x4*>(dst + off));
            continue;
        }
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + off));
        if (mode == 0) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + off));
        else acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    if (mode == 1 && acc == 0x12345678u) sink[0] = acc;  // keeps the loads
}

// mode 2: the same tiles read by LDS-DMA (buffer_load_dwordx4 ... lds), 16
// bytes per lane straight into LDS (the warp kernel's staging path): each
// wave instruction lands 1 KiB contiguous in a 16 KiB per-workgroup area
__global__ __launch_bounds__(256) void seg_dma(const unsigned char* src, int frames, int H, int pitch, int L, int TR,
                                               int tiles_x, int tiles_y, unsigned* sink) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[16384];
    const int total = frames * tiles_x * tiles_y;
    const int per_xcd = (total + 7) / 8;
    const int id = (int)(blockIdx.x % 8) * per_xcd + (int)(blockIdx.x / 8);
    if (id >= total) return;
    const int f = id / (tiles_x * tiles_y), t = id - f * tiles_x * tiles_y;
    const int ty = t / tiles_x, tx = t - ty * tiles_x;
    const int chunks = L / 16;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned char*>(src) + (int64_t)f * H * pitch, (short)0, H * pitch, 0x00020000);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int i = 0;
    for (int e0 = wave * 64; e0 < TR * chunks; e0 += 256, ++i) {
        const int e = e0 + lane;
        const int rr = e / chunks, c = e - rr * chunks;
        const int row = ty * TR + rr;
        const int off = (e < TR * chunks && row < H) ? row * pitch + tx * L + 16 * c : (int)0x80000000;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, (__attribute__((address_space(3))) void*)(lds + ((wave * 4 + (i & 3)) * 1024) % 16384), 16, off, 0, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (lds[threadIdx.x * 7] == 0x5A && threadIdx.x == 1000) sink[0] = 1;
}

int main() {
    const int frames = 128, H = 720, pitch = 3840;  // cfg4's batch: 128 x 720p x 3 bytes
    const size_t bytes = (size_t)frames * H * pitch;
    unsigned char *a = nullptr, *b = nullptr;
    unsigned* sink = nullptr;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(a, 1, bytes));
    CHECK(hipMemset(b, 0, bytes));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int Ls[] = {192, 256, 320, 384, 640, 1280, 3840};
    const int TRs[] = {32, 8};
    for (int mode = 0; mode < 5; ++mode) {
        for (int TR : TRs) {
            for (int L : Ls) {
                const int tiles_x = pitch / L, tiles_y = (H + TR - 1) / TR;
                const int total = frames * tiles_x * tiles_y;
                const int blocks = (total + 7) / 8 * 8;
                auto launch = [&]() {
                    if (mode == 2)
                        hipLaunchKernelGGL(seg_dma, dim3(blocks), dim3(256), 0, 0, a, frames, H, pitch, L, TR, tiles_x,
                                           tiles_y, sink);
                    else
                        hipLaunchKernelGGL(seg_copy, dim3(blocks), dim3(256), 0, 0, a, b, frames, H, pitch, L, TR,
                                           tiles_x, tiles_y, mode, sink);
                };
                for (int w = 0; w < 3; ++w) launch();
                CHECK(hipDeviceSynchronize());
                std::vector<float> ms;
                for (int it = 0; it < 10; ++it) {
                    CHECK(hipEventRecord(e0, 0));
                    launch();
                    CHECK(hipEventRecord(e1, 0));
                    CHECK(hipEventSynchronize(e1));
                    float t = 0;
                    CHECK(hipEventElapsedTime(&t, e0, e1));
                    ms.push_back(t);
                }
                std::sort(ms.begin(), ms.end());
                const double moved = (double)bytes * (mode == 0 ? 2 : 1);
                const char* names[] = {"copy", "read", "read_dma", "write16", "write4"};
                std::printf("{\"L\": %d, \"TR\": %d, \"mode\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", L, TR,
                            names[mode], ms[5], moved / ms[5] / 1e6);
                std::fflush(stdout);
            }
        }
    }
    return 0;
}
