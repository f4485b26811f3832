// ldsprobe.hip -- semantics checks, on the GPU, of the two primitives the
// LDS-ring warp kernel builds on (k_warp_frames.hip):
//  1. buffer LDS-DMA, 16 bytes per lane (__builtin_amdgcn_raw_ptr_buffer_load_lds):
//     lane l lands at M0 + 16 l; an out-of-range lane writes zeros to its
//     slot; an exec-masked lane writes nothing; a source offset that is not
//     16-byte aligned (only 4-byte aligned) reads the right bytes;
//  2. ds_read_b64 at byte addresses that are not 8- (or 4-) byte aligned
//     returns the 8 bytes at that address.
// Prints one JSON line; exit status 0 iff every check passes.
//   hipcc -O3 --offload-arch=gfx950 tools/ldsprobe.hip -o tools/ldsprobe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                           \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// out[0 .. 4096): the LDS image after the DMA (1024 dwords of a 4 KiB area
// first filled with 0xAB bytes); out[4096 ..): unaligned ds_read_b64 results
__global__ __launch_bounds__(64) void probe(const unsigned char* src, int src_bytes, unsigned* out) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[4096 + 64];
    const int lane = threadIdx.x;
    for (int i = lane; i < (4096 + 64) / 4; i += 64) reinterpret_cast<unsigned*>(lds)[i] = 0xABABABABu;
    __syncthreads();
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(src), (short)0, src_bytes, 0x00020000);
    // instruction 0: every lane in range, aligned: src[16 l .. 16 l + 16) -> lds[0 ..)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(lds + 0), 16, 16 * lane, 0, 0, 0);
    // instruction 1: lanes >= 32 out of range (offset 0x80000000): zeros expected there
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(lds + 1024), 16,
                                             lane < 32 ? 16 * lane : (int)0x80000000, 0, 0, 0);
    // instruction 2: 4-byte aligned offsets 4 + 12 l (unaligned for 16 bytes)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(lds + 2048), 16, 4 + 12 * lane, 0, 0, 0);
    // instruction 3: exec-masked lanes (odd lanes off): their slots keep 0xAB
    if (lane & 1)
        ;
    else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(lds + 3072), 16, 16 * lane, 0, 0, 0);
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0) expcnt(0)
    __syncthreads();
    for (int i = lane; i < 1024; i += 64) out[i] = reinterpret_cast<const unsigned*>(lds)[i];
    // unaligned 8-byte LDS reads over the first kilobyte (the source bytes)
    for (int k = 0; k < 4; ++k) {
        const int a = 13 * lane + k;  // every residue mod 8
        u32x2 v;
        asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"((unsigned)(uintptr_t)(lds + a)) : "memory");
        out[1024 + 2 * (4 * lane + k)] = v[0];
        out[1024 + 2 * (4 * lane + k) + 1] = v[1];
    }
}

int main() {
    const int n = 2048;
    std::vector<unsigned char> h(n);
    for (int i = 0; i < n; ++i) h[i] = (unsigned char)(i * 7 + (i >> 8) * 13 + 1);
    unsigned char* d = nullptr;
    unsigned* o = nullptr;
    CHECK(hipMalloc(&d, n));
    CHECK(hipMalloc(&o, (1024 + 512) * 4));
    CHECK(hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, n, o);
    CHECK(hipGetLastError());
    std::vector<unsigned> out(1024 + 512);
    CHECK(hipMemcpy(out.data(), o, out.size() * 4, hipMemcpyDeviceToHost));
    const unsigned char* lb = reinterpret_cast<const unsigned char*>(out.data());
    int bad[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < 1024; ++i) bad[0] += lb[i] != h[i];
    for (int i = 0; i < 1024; ++i) bad[1] += lb[1024 + i] != (i < 512 ? h[i] : 0);
    for (int l = 0; l < 64; ++l)
        for (int b = 0; b < 16; ++b) bad[2] += lb[2048 + 16 * l + b] != h[4 + 12 * l + b];
    for (int l = 0; l < 64; ++l)
        for (int b = 0; b < 16; ++b) bad[3] += lb[3072 + 16 * l + b] != ((l & 1) ? 0xAB : h[16 * l + b]);
    for (int l = 0; l < 64; ++l)
        for (int k = 0; k < 4; ++k) {
            const int a = 13 * l + k;
            const unsigned char* v = lb + 4096 + 8 * (4 * l + k);
            for (int b = 0; b < 8; ++b) bad[4] += v[b] != h[a + b];
        }
    const bool ok = !(bad[0] | bad[1] | bad[2] | bad[3] | bad[4]);
    std::printf("{\"dma_aligned_bad\": %d, \"dma_oob_zero_bad\": %d, \"dma_unaligned_src_bad\": %d, "
                "\"dma_exec_masked_bad\": %d, \"ds_read_b64_unaligned_bad\": %d, \"ok\": %s}\n",
                bad[0], bad[1], bad[2], bad[3], bad[4], ok ? "true" : "false");
    return ok ? 0 : 1;
}
