// k_pixel.hip -- streaming per-pixel operators: crop (row copy), HWC<->CHW,
// u8<->fp32, NV21/NV12 -> BGR (+normalize), normalize, per-channel sums.
// All HBM-bound; every kernel moves 16 bytes per lane per access where the
// alignment allows and falls back to narrower accesses only at row tails.
#pragma clang fp contract(off)

#include <cstdlib>
#include <cstring>

#include "vacv_device.hpp"

namespace vacv {
namespace {

__device__ __forceinline__ int64_t gtid() { return (int64_t)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ int64_t gstride() { return (int64_t)gridDim.x * blockDim.x; }

constexpr int kColorPairs = 1;  // row pairs per wave in color_kernel (4 measured 15 % slower)

int grid_for(int64_t work_items, int cap = 256 * 16) {
    int64_t g = (work_items + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (int)g;
}

// --------------------------------------------------------------------------
// crop / clone: copy `row_bytes` from every (image, plane, row) of src to dst.
// crop.cpp:44-125 restated as one strided 2-D copy per plane.
__global__ void __launch_bounds__(kBlock) row_copy_kernel(CopyLaunch L) {
    const int64_t rows_per_img = (int64_t)L.src.planes * L.src.h;
    const int64_t rows = rows_per_img * L.n;
    const int row_in_block = threadIdx.x / 64;  // 4 waves, one row each per step
    const int lane = threadIdx.x & 63;
    for (int64_t r = (int64_t)blockIdx.x * 4 + row_in_block; r < rows; r += (int64_t)gridDim.x * 4) {
        const int64_t img = r / rows_per_img;
        const int64_t rr = r - img * rows_per_img;
        const int64_t plane = rr / L.src.h, y = rr - plane * L.src.h;
        const unsigned char* s = L.src.base + img * L.src.img_pitch + plane * L.src.plane_pitch + y * L.src.row_pitch;
        unsigned char* d = const_cast<unsigned char*>(L.dst.base) + img * L.dst.img_pitch +
                           plane * L.dst.plane_pitch + y * L.dst.row_pitch;
        const uintptr_t mis = (reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d));
        if ((mis & 15) == 0) {
            const int64_t n16 = L.row_bytes >> 4;
            for (int64_t i = lane; i < n16; i += 64)
                reinterpret_cast<uint4*>(d)[i] = reinterpret_cast<const uint4*>(s)[i];
            for (int64_t i = (n16 << 4) + lane; i < L.row_bytes; i += 64) d[i] = s[i];
        } else if ((mis & 3) == 0) {
            const int64_t n4 = L.row_bytes >> 2;
            for (int64_t i = lane; i < n4; i += 64)
                reinterpret_cast<uint32_t*>(d)[i] = reinterpret_cast<const uint32_t*>(s)[i];
            for (int64_t i = (n4 << 2) + lane; i < L.row_bytes; i += 64) d[i] = s[i];
        } else {
            for (int64_t i = lane; i < L.row_bytes; i += 64) d[i] = s[i];
        }
    }
}

// --------------------------------------------------------------------------
// HWC <-> CHW (tensor.cpp:160-182).  Generic: one element per step.
template <typename T>
__global__ void __launch_bounds__(kBlock) layout_kernel(LayoutLaunch L) {
    const int64_t hw = (int64_t)L.w * L.h;
    const int64_t per_img = hw * L.c;
    const int64_t total = per_img * L.n;
    for (int64_t e = gtid(); e < total; e += gstride()) {
        const int64_t img = e / per_img;
        const int64_t r = e - img * per_img;
        // e indexes the DESTINATION densely -> writes are coalesced
        int64_t si;
        if (L.to_chw) {
            const int64_t k = r / hw, i = r - k * hw;
            si = i * L.c + k;
        } else {
            const int64_t i = r / L.c, k = r - i * L.c;
            si = k * hw + i;
        }
        reinterpret_cast<T*>(L.dst + img * L.dst_img)[r] = reinterpret_cast<const T*>(L.src + img * L.src_img)[si];
    }
}

// u8, c == 3, HWC -> CHW: 4 pixels per step, dword loads and stores.
__global__ void __launch_bounds__(kBlock) hwc3_to_chw_u8_kernel(LayoutLaunch L) {
    const int64_t hw = (int64_t)L.w * L.h;
    const int64_t groups = hw / 4;
    const int64_t total = groups * L.n;
    for (int64_t gi = gtid(); gi < total; gi += gstride()) {
        const int64_t img = gi / groups, g = gi - img * groups;
        const uint32_t* s = reinterpret_cast<const uint32_t*>(L.src + img * L.src_img) + g * 3;
        const uint32_t a = s[0], b = s[1], c = s[2];  // b0 g0 r0 b1 | g1 r1 b2 g2 | r2 b3 g3 r3
        uint32_t ch0 = (a & 0xFFu) | (((a >> 24) & 0xFFu) << 8) | (((b >> 16) & 0xFFu) << 16) | (((c >> 8) & 0xFFu) << 24);
        uint32_t ch1 = ((a >> 8) & 0xFFu) | ((b & 0xFFu) << 8) | (((b >> 24) & 0xFFu) << 16) | (((c >> 16) & 0xFFu) << 24);
        uint32_t ch2 = ((a >> 16) & 0xFFu) | (((b >> 8) & 0xFFu) << 8) | ((c & 0xFFu) << 16) | (((c >> 24) & 0xFFu) << 24);
        uint32_t* d = reinterpret_cast<uint32_t*>(L.dst + img * L.dst_img);
        d[g] = ch0;
        d[groups + g] = ch1;
        d[2 * groups + g] = ch2;
    }
}

// u8, c == 3, CHW -> HWC: 4 pixels per step.
__global__ void __launch_bounds__(kBlock) chw_to_hwc3_u8_kernel(LayoutLaunch L) {
    const int64_t hw = (int64_t)L.w * L.h;
    const int64_t groups = hw / 4;
    const int64_t total = groups * L.n;
    for (int64_t gi = gtid(); gi < total; gi += gstride()) {
        const int64_t img = gi / groups, g = gi - img * groups;
        const uint32_t* s = reinterpret_cast<const uint32_t*>(L.src + img * L.src_img);
        const uint32_t x = s[g], y = s[groups + g], z = s[2 * groups + g];
        const uint32_t a = (x & 0xFFu) | ((y & 0xFFu) << 8) | ((z & 0xFFu) << 16) | (((x >> 8) & 0xFFu) << 24);
        const uint32_t b = ((y >> 8) & 0xFFu) | (((z >> 8) & 0xFFu) << 8) | (((x >> 16) & 0xFFu) << 16) | (((y >> 16) & 0xFFu) << 24);
        const uint32_t c = ((z >> 16) & 0xFFu) | (((x >> 24) & 0xFFu) << 8) | (((y >> 24) & 0xFFu) << 16) | (((z >> 24) & 0xFFu) << 24);
        uint32_t* d = reinterpret_cast<uint32_t*>(L.dst + img * L.dst_img) + g * 3;
        d[0] = a;
        d[1] = b;
        d[2] = c;
    }
}

// --------------------------------------------------------------------------
// u8 <-> f32 over a dense buffer (tensor.cpp:459-502).
__global__ void __launch_bounds__(kBlock) u8_to_f32_kernel(DtypeLaunch L) {
    const int64_t n16 = L.count >> 4;
    for (int64_t i = gtid(); i < n16; i += gstride()) {
        const uint4 v = reinterpret_cast<const uint4*>(L.src)[i];
        float4* d = reinterpret_cast<float4*>(L.dst) + i * 4;
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j)
            d[j] = make_float4((float)(w[j] & 0xFF), (float)((w[j] >> 8) & 0xFF), (float)((w[j] >> 16) & 0xFF),
                               (float)(w[j] >> 24));
    }
    for (int64_t i = (n16 << 4) + gtid(); i < L.count; i += gstride())
        reinterpret_cast<float*>(L.dst)[i] = (float)L.src[i];
}

// One dword of u8 in, one 16-byte float4 out per thread over a grid that
// covers the buffer once, in order (the shape that streams fastest on MI355X,
// tools/membench2.hip); non-temporal stores.  Needs 4-byte aligned u8 and
// 16-byte aligned fp32; the last count % 4 elements go through the tail.
__global__ void __launch_bounds__(kBlock) u8_to_f32_flat_kernel(DtypeLaunch L) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t n4 = L.count >> 2;
    if (i < n4) {
        const uint32_t w = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(L.src) + i);
        const u32x4 f = {__float_as_uint((float)(w & 0xFF)), __float_as_uint((float)((w >> 8) & 0xFF)),
                         __float_as_uint((float)((w >> 16) & 0xFF)), __float_as_uint((float)(w >> 24))};
        __builtin_nontemporal_store(f, reinterpret_cast<u32x4*>(L.dst) + i);
    } else if (i - n4 < (L.count & 3)) {
        const int64_t e = (n4 << 2) + (i - n4);
        reinterpret_cast<float*>(L.dst)[e] = (float)L.src[e];
    }
}

__global__ void __launch_bounds__(kBlock) f32_to_u8_flat_kernel(DtypeLaunch L) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    const int64_t n4 = L.count >> 2;
    if (i < n4) {
        const u32x4 f = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(L.src) + i);
        const uint32_t w = (uint32_t)f32_to_u8_neon(__uint_as_float(f.x)) |
                           ((uint32_t)f32_to_u8_neon(__uint_as_float(f.y)) << 8) |
                           ((uint32_t)f32_to_u8_neon(__uint_as_float(f.z)) << 16) |
                           ((uint32_t)f32_to_u8_neon(__uint_as_float(f.w)) << 24);
        __builtin_nontemporal_store(w, reinterpret_cast<uint32_t*>(L.dst) + i);
    } else if (i - n4 < (L.count & 3)) {
        const int64_t e = (n4 << 2) + (i - n4);
        L.dst[e] = f32_to_u8_neon(reinterpret_cast<const float*>(L.src)[e]);
    }
}

__global__ void __launch_bounds__(kBlock) f32_to_u8_kernel(DtypeLaunch L) {
    const int64_t n16 = L.count >> 4;
    for (int64_t i = gtid(); i < n16; i += gstride()) {
        const float4* s = reinterpret_cast<const float4*>(L.src) + i * 4;
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 f = s[j];
            w[j] = (uint32_t)f32_to_u8_neon(f.x) | ((uint32_t)f32_to_u8_neon(f.y) << 8) |
                   ((uint32_t)f32_to_u8_neon(f.z) << 16) | ((uint32_t)f32_to_u8_neon(f.w) << 24);
        }
        reinterpret_cast<uint4*>(L.dst)[i] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    for (int64_t i = (n16 << 4) + gtid(); i < L.count; i += gstride())
        L.dst[i] = f32_to_u8_neon(reinterpret_cast<const float*>(L.src)[i]);
}

// --------------------------------------------------------------------------
// YUV420sp -> BGR (cvt_color.cpp:39-135).  One thread = a 4x2 pixel block:
// two 4-byte Y loads and one 4-byte chroma load (two VU pairs), 2 rows x
// 4 pixels x 3 channels out.
template <int OUT>
__global__ void __launch_bounds__(kBlock) color_kernel(ColorLaunch L) {
    using TOut = typename std::conditional<(OUT == kOutSame), uint8_t, float>::type;
    // normalisation in registers (normalize_u8v: the host-verified fp64
    // multiply, else the reference's divide); a per-workgroup 768-entry LDS
    // table cost 3 fp64 divides per thread and a barrier for 8 pixels
    const int img = blockIdx.z;
    ChanNorm cn[3] = {};
    if (OUT == kOutNorm) {
#pragma unroll
        for (int k = 0; k < 3; ++k) cn[k] = chan_norm(L.norm, img, k);
    }
    // fp32 output: a wave's 64 lanes x 48 B of one row go out through LDS as
    // three 1 KiB contiguous non-temporal stores (lane-strided 48-B stores
    // measured 0.37 of the HBM roofline)
    constexpr bool kXch = OUT != kOutSame;
    __shared__ u32x4 xch[kXch ? 4 : 1][kXch ? 192 : 1];
    const int x0 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
    if (x0 >= L.w) return;
    const bool wave_full = (int)(blockIdx.x + 1) * 256 <= L.w;  // uniform: every lane has 4 pixels
    // each wave takes kColorPairs row pairs (the block's table is built once)
    for (int it = 0; it < kColorPairs; ++it) {
    const int yy = (blockIdx.y * kColorPairs + it) * blockDim.y + threadIdx.y;  // row pair (wave-uniform)
    if (2 * yy >= L.h) break;

    const unsigned char* yb = L.src + (int64_t)img * L.src_img;
    const unsigned char* y0p = yb + (int64_t)(2 * yy) * L.src_row + x0;
    const unsigned char* y1p = y0p + L.src_row;
    const unsigned char* uvp = yb + (int64_t)L.h * L.src_row + (int64_t)yy * L.src_row + x0;
    const int valid = min(4, L.w - x0);

    uint8_t ys[2][4], uv[4];
    if (valid == 4 && ((reinterpret_cast<uintptr_t>(y0p) | reinterpret_cast<uintptr_t>(y1p) |
                        reinterpret_cast<uintptr_t>(uvp)) & 3) == 0) {
        const uint32_t a = *reinterpret_cast<const uint32_t*>(y0p);
        const uint32_t b = *reinterpret_cast<const uint32_t*>(y1p);
        const uint32_t c = *reinterpret_cast<const uint32_t*>(uvp);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            ys[0][j] = (a >> (8 * j)) & 0xFF;
            ys[1][j] = (b >> (8 * j)) & 0xFF;
            uv[j] = (c >> (8 * j)) & 0xFF;
        }
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int jj = j < valid ? j : 0;
            ys[0][j] = y0p[jj];
            ys[1][j] = y1p[jj];
            uv[j] = uvp[jj];
        }
    }

#pragma unroll
    for (int r = 0; r < 2; ++r) {
        TOut out[12];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int pair = (j >> 1) * 2;
            const int v = L.v_first ? uv[pair] : uv[pair + 1];
            const int u = L.v_first ? uv[pair + 1] : uv[pair];
            const Chroma ch = chroma_terms(u, v);
            const int Y = ys[r][j];
            const int R = clamp_u8(Y + ch.ra), G = clamp_u8(Y - ch.ga), B = clamp_u8(Y + ch.ba);
            const int c0 = L.rgb ? R : B, c2 = L.rgb ? B : R;
            if (OUT == kOutSame) {
                out[3 * j + 0] = (TOut)c0; out[3 * j + 1] = (TOut)G; out[3 * j + 2] = (TOut)c2;
            } else if (OUT == kOutF32) {
                out[3 * j + 0] = (TOut)(float)c0; out[3 * j + 1] = (TOut)(float)G; out[3 * j + 2] = (TOut)(float)c2;
            } else {
                out[3 * j + 0] = normalize_u8v(cn[0], c0);
                out[3 * j + 1] = normalize_u8v(cn[1], G);
                out[3 * j + 2] = normalize_u8v(cn[2], c2);
            }
        }
        unsigned char* dp = L.dst + (int64_t)img * L.dst_img + (int64_t)(2 * yy + r) * L.dst_row +
                            (int64_t)x0 * 3 * sizeof(TOut);
        constexpr int kBytes = 12 * (int)sizeof(TOut);
        if constexpr (kXch) {
            unsigned char* wbase = L.dst + (int64_t)img * L.dst_img + (int64_t)(2 * yy + r) * L.dst_row +
                                   (int64_t)blockIdx.x * 256 * 12;
            if (wave_full && (reinterpret_cast<uintptr_t>(wbase) & 15) == 0) {  // uniform
                const int lane = threadIdx.x;
                u32x4* w = xch[threadIdx.y];
#pragma unroll
                for (int b = 0; b < 3; ++b)
                    w[lane * 3 + b] = u32x4{__float_as_uint(out[4 * b]), __float_as_uint(out[4 * b + 1]),
                                            __float_as_uint(out[4 * b + 2]), __float_as_uint(out[4 * b + 3])};
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
                for (int b = 0; b < 3; ++b) {
                    __builtin_nontemporal_store(w[b * 64 + lane], reinterpret_cast<u32x4*>(wbase) + b * 64 + lane);
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();  // the next row reuses the exchange buffer
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                continue;
            }
        }
        if (valid == 4 && (kBytes % 16 == 0) && ((reinterpret_cast<uintptr_t>(dp) & 15) == 0)) {
#pragma unroll
            for (int b = 0; b < kBytes / 16; ++b) reinterpret_cast<uint4*>(dp)[b] = reinterpret_cast<const uint4*>(out)[b];
        } else if (valid == 4 && ((reinterpret_cast<uintptr_t>(dp) & 3) == 0)) {
#pragma unroll
            for (int b = 0; b < kBytes / 4; ++b) reinterpret_cast<uint32_t*>(dp)[b] = reinterpret_cast<const uint32_t*>(out)[b];
        } else {
            TOut* o = reinterpret_cast<TOut*>(dp);
#pragma unroll
            for (int e = 0; e < 12; ++e)
                if (e < 3 * valid) o[e] = out[e];
        }
    }
    }  // row pairs
}


// --------------------------------------------------------------------------
// normalize (normalize_naive.cpp:74-90) over rows of (w * cc) elements.
// One thread = 4 consecutive elements of a row.
template <typename TIn>
__global__ void __launch_bounds__(kBlock) normalize_kernel(NormLaunch L) {
    const int64_t row_elems = (int64_t)L.src.w * L.src.cc;
    const int64_t chunks = (row_elems + 3) / 4;
    const int64_t rows_per_plane = L.src.h;
    const int64_t total = chunks * rows_per_plane * L.src.planes * L.n;
    for (int64_t i = gtid(); i < total; i += gstride()) {
        int64_t r = i / chunks;
        const int64_t cidx = i - r * chunks;
        const int64_t y = r % rows_per_plane;
        r /= rows_per_plane;
        const int64_t plane = r % L.src.planes;
        const int64_t img = r / L.src.planes;
        const TIn* s = reinterpret_cast<const TIn*>(L.src.base + img * L.src.img_pitch + plane * L.src.plane_pitch +
                                                    y * L.src.row_pitch);
        float* d = reinterpret_cast<float*>(const_cast<unsigned char*>(L.dst.base) + img * L.dst.img_pitch +
                                            plane * L.dst.plane_pitch + y * L.dst.row_pitch);
        const int64_t e0 = cidx * 4;
        float o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t e = e0 + j < row_elems ? e0 + j : row_elems - 1;
            const int ch = (L.src.cc == 1) ? (int)plane : (int)(e % L.src.cc);
            float m, sd;
            norm_params(L.norm, (int)img, ch, m, sd);
            o[j] = normalize_value((float)s[e], m, sd);
        }
        if (e0 + 4 <= row_elems && ((reinterpret_cast<uintptr_t>(d + e0) & 15) == 0)) {
            *reinterpret_cast<float4*>(d + e0) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (e0 + j < row_elems) d[e0 + j] = o[j];
        }
    }
}

// --------------------------------------------------------------------------
// Per-channel (Sum x, Sum x^2).  Each workgroup reduces a contiguous range of
// one plane (dense) in chunks of 16*CC elements, so element j of a chunk is
// always channel j % CC; partials are written per block and summed in a
// fixed order by stats_reduce_kernel (deterministic).
template <int CC, typename TIn>
__global__ void __launch_bounds__(kBlock) channel_sums_kernel(SumsLaunch L) {
    constexpr int kChunk = 16 * CC;
    const int pidx = blockIdx.y;  // image * planes + plane
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;
    const TIn* base = reinterpret_cast<const TIn*>(L.src.base + (int64_t)img * L.src.img_pitch +
                                                   (int64_t)plane * L.src.plane_pitch);
    const int64_t elems = (int64_t)L.src.w * L.src.h * CC;
    const int64_t nchunks = L.scalar_only ? 0 : elems / kChunk;
    const int64_t per_block = (nchunks + gridDim.x - 1) / gridDim.x;
    const int64_t c_begin = blockIdx.x * per_block;
    const int64_t c_end = min(nchunks, c_begin + per_block);

    double s1[CC], s2[CC];
#pragma unroll
    for (int k = 0; k < CC; ++k) { s1[k] = 0.0; s2[k] = 0.0; }

    if (sizeof(TIn) == 1) {
        uint32_t a1[CC], a2[CC];
#pragma unroll
        for (int k = 0; k < CC; ++k) { a1[k] = 0; a2[k] = 0; }
        int steps = 0;
        for (int64_t c = c_begin + threadIdx.x; c < c_end; c += kBlock) {
            const uint4* p = reinterpret_cast<const uint4*>(base + c * kChunk);
#pragma unroll
            for (int q = 0; q < CC; ++q) {
                const uint4 v = p[q];
                const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const uint32_t b = (w[j >> 2] >> (8 * (j & 3))) & 0xFFu;
                    const int k = (q * 16 + j) % CC;
                    a1[k] += b;
                    a2[k] += b * b;
                }
            }
            // a2 grows by <= 16*65025 per step: flush well before 2^32
            if (++steps == 2048) {
#pragma unroll
                for (int k = 0; k < CC; ++k) { s1[k] += a1[k]; s2[k] += a2[k]; a1[k] = 0; a2[k] = 0; }
                steps = 0;
            }
        }
#pragma unroll
        for (int k = 0; k < CC; ++k) { s1[k] += a1[k]; s2[k] += a2[k]; }
    } else {
        // fp32: lane-consecutive float4 loads (1 KiB per wave instruction).
        // Block ranges and wave steps are multiples of 192 float4s, so the
        // channel of element j of load m (float4 192k + 64m + lane) is
        // (lane + m + j) % 3 for CC = 3 (4 = 1 mod 3) and j % CC otherwise:
        // accumulate by the lane-relative slot, un-rotate once at the end.
        const int64_t n4 = L.scalar_only ? 0 : elems / 4;
        const int64_t groups = (n4 + 191) / 192;
        const int64_t g_per_block = (groups + gridDim.x - 1) / gridDim.x;
        const int64_t g_begin = blockIdx.x * g_per_block;
        const int64_t g_end = min(groups, g_begin + g_per_block);
        const int wave = threadIdx.x >> 6, ln = threadIdx.x & 63;
        typedef float f32x4_t __attribute__((ext_vector_type(4)));
        const f32x4_t* b4 = reinterpret_cast<const f32x4_t*>(base);
        double r1[CC], r2[CC];
#pragma unroll
        for (int k = 0; k < CC; ++k) { r1[k] = 0.0; r2[k] = 0.0; }
        for (int64_t g = g_begin + wave; g < g_end; g += kBlock / 64) {
            f32x4_t v[3];
#pragma unroll
            for (int m = 0; m < 3; ++m) {
                const int64_t i = g * 192 + 64 * m + ln;
                v[m] = i < n4 ? __builtin_nontemporal_load(b4 + i) : f32x4_t{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll
            for (int m = 0; m < 3; ++m) {
                const float f[4] = {v[m][0], v[m][1], v[m][2], v[m][3]};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int slot = CC == 3 ? (m + j) % 3 : j % CC;
                    const double d = f[j];
                    r1[slot] += d;
                    r2[slot] += d * d;
                }
            }
        }
        // slot -> channel: (slot + lane) % 3 for CC = 3, the identity otherwise
        const int rot = CC == 3 ? ln % 3 : 0;
#pragma unroll
        for (int k = 0; k < CC; ++k) {
#pragma unroll
            for (int sl = 0; sl < CC; ++sl) {
                if (CC == 3 ? ((sl + rot) % 3 == k) : (sl == k)) {
                    s1[k] += r1[sl];
                    s2[k] += r2[sl];
                }
            }
        }
    }
    // tail elements (all of them on a misaligned plane), split over blocks
    {
        const int64_t t0 = sizeof(TIn) == 1 ? nchunks * kChunk : (L.scalar_only ? 0 : elems / 4 * 4);
        const int64_t tn = elems - t0;
        const int64_t tper = (tn + gridDim.x - 1) / gridDim.x;
        const int64_t tb = t0 + blockIdx.x * tper, te = min(elems, tb + tper);
        for (int64_t e = tb + threadIdx.x; e < te; e += kBlock) {
            const double d = (double)base[e];
            const int k = (int)(e % CC);
#pragma unroll
            for (int kk = 0; kk < CC; ++kk)
                if (kk == k) { s1[kk] += d; s2[kk] += d * d; }
        }
    }

    __shared__ double red[kBlock / 64][2 * CC];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < CC; ++k) {
        const double t1 = wave_sum(s1[k]);
        const double t2 = wave_sum(s2[k]);
        if (lane == 0) { red[wave][2 * k] = t1; red[wave][2 * k + 1] = t2; }
    }
    __syncthreads();
    if (threadIdx.x < 2 * CC) {
        double acc = 0.0;
#pragma unroll
        for (int wv = 0; wv < kBlock / 64; ++wv) acc += red[wv][threadIdx.x];
        // partials[img][plane][block][CC][2]
        const int64_t o = (((int64_t)pidx * gridDim.x) + blockIdx.x) * (2 * CC) + threadIdx.x;
        L.partials[o] = acc;
    }
}

// sums[g][c][2] from partials, fixed order: image-major, then plane, block.
// One workgroup per (group, channel, moment): thread t sums partials t,
// t + 256, ... in order, then a fixed LDS tree -- the same order on every run
// (deterministic), and parallel: a whole-batch sum over n * blocks partials
// took 262 us as one sequential loop per output (cfg5, n = 128).
__global__ void __launch_bounds__(kBlock) stats_reduce_kernel(SumsLaunch L, int cc) {
    __shared__ double red[kBlock];
    const int c = L.c;
    const int idx = blockIdx.x;  // < groups * c * 2
    const int g = idx / (2 * c);
    const int r = idx - g * 2 * c;
    const int ch = r >> 1, mom = r & 1;
    const int plane = (cc == 1) ? ch : 0;  // NCHW: channel = plane
    const int k = (cc == 1) ? 0 : ch;
    const int img_lo = L.per_image ? g : 0, img_hi = L.per_image ? g + 1 : L.n;
    const int64_t terms = (int64_t)(img_hi - img_lo) * L.blocks_per_image;
    auto term = [&](int64_t t) {
        const int img = img_lo + (int)(t / L.blocks_per_image);
        const int b = (int)(t - (int64_t)(img - img_lo) * L.blocks_per_image);
        const int64_t pidx = (int64_t)img * L.src.planes + plane;
        return L.partials[((pidx * L.blocks_per_image) + b) * (2 * cc) + 2 * k + mom];
    };
    // thread t adds terms t, t + 256, ... in that order; 16 loads are issued
    // before their adds (a load-add chain per term took 78 us for cfg5's
    // 50K per-wave partials), the order of the adds is unchanged
    constexpr int kDepth = 16;
    double acc = 0.0;
    int64_t t = threadIdx.x;
    for (; t + (kDepth - 1) * kBlock < terms; t += kDepth * kBlock) {
        double v[kDepth];
#pragma unroll
        for (int q = 0; q < kDepth; ++q) v[q] = term(t + q * kBlock);
#pragma unroll
        for (int q = 0; q < kDepth; ++q) acc += v[q];
    }
    for (; t < terms; t += kBlock) acc += term(t);
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int h = kBlock / 2; h > 0; h >>= 1) {
        if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
        __syncthreads();
    }
    if (threadIdx.x == 0) L.sums[idx] = red[0];
}

__global__ void stats_kernel(const double* sums, int groups, int c, double count, float* mean, float* stddev) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= groups * c) return;
    const double m = sums[2 * idx] / count;
    double var = sums[2 * idx + 1] / count - m * m;
    if (var < 0) var = 0;
    mean[idx] = (float)m;
    stddev[idx] = (float)sqrt(var);
}

template <int CC, typename TIn>
hipError_t launch_sums_cc(const SumsLaunch& L, hipStream_t s) {
    dim3 grid(L.blocks_per_image, L.n * L.src.planes);
    hipLaunchKernelGGL((channel_sums_kernel<CC, TIn>), grid, dim3(kBlock), 0, s, L);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int groups = L.per_image ? L.n : 1;
    const int work = groups * L.c * 2;
    hipLaunchKernelGGL(stats_reduce_kernel, dim3(work), dim3(kBlock), 0, s, L, CC);
    return hipGetLastError();
}

template <typename TIn>
hipError_t launch_sums_t(const SumsLaunch& L, hipStream_t s) {
    switch (L.src.cc) {
        case 1: return launch_sums_cc<1, TIn>(L, s);
        case 2: return launch_sums_cc<2, TIn>(L, s);
        case 3: return launch_sums_cc<3, TIn>(L, s);
        case 4: return launch_sums_cc<4, TIn>(L, s);
        default: return hipErrorInvalidValue;
    }
}

// --------------------------------------------------------------------------
// INTER_NEAREST resize (cv::resize -> resizeNN of the pinned OpenCV 2.4,
// which the reference hands every mode but LINEAR/CUBIC to, resize.cpp:44-49):
// sx = min(floor(x * ifx), w - 1), ifx = 1 / ((double)w_out / w_in), the same
// for y.  One thread per output pixel (all cc channels); a workgroup row is
// one output row, so sy is uniform.  Optional widen / normalize epilogue.
template <typename TIn, int OUT>
__global__ void __launch_bounds__(kBlock) nearest_kernel(ResizeLaunch L) {
    using TOut = typename std::conditional<(OUT == kOutSame), TIn, float>::type;
    const int x = blockIdx.x * kBlock + threadIdx.x;
    const int y = blockIdx.y;
    const int pidx = blockIdx.z;  // image * planes + plane
    if (x >= L.dst.w) return;
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;
    int sx = (int)floor((double)x * L.scale_xd);
    int sy = (int)floor((double)y * L.scale_yd);
    sx = min(sx, L.src.w - 1);
    sy = min(sy, L.src.h - 1);
    const int cc = L.src.cc;
    const TIn* sp = reinterpret_cast<const TIn*>(L.src.base + (int64_t)img * L.src.img_pitch +
                                                 (int64_t)plane * L.src.plane_pitch + (int64_t)sy * L.src.row_pitch) +
                    (int64_t)sx * cc;
    TOut* dp = reinterpret_cast<TOut*>(const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                                       (int64_t)plane * L.dst.plane_pitch + (int64_t)y * L.dst.row_pitch) +
               (int64_t)x * cc;
    for (int k = 0; k < cc; ++k) {
        const TIn v = sp[k];
        if (OUT == kOutSame) {
            dp[k] = (TOut)v;
        } else if (OUT == kOutF32) {
            dp[k] = (TOut)(float)v;
        } else {
            const ChanNorm cn = chan_norm(L.norm, img, cc == 1 ? plane % L.norm.c_total : k);
            dp[k] = (TOut)(std::is_same<TIn, uint8_t>::value ? normalize_u8v(cn, (int)v) : normalize_f(cn, (float)v));
        }
    }
}

// INTER_NEAREST with the source row staged in LDS: a workgroup takes one
// output row, reads its source row sy once as coalesced 16-byte loads (a
// gather per pixel moves the same 128 B lines whenever the sample stride is
// under a line, but with one load instruction per pixel per lane), then one
// thread per output element picks from LDS and stores (adjacent elements per
// lane).  Same index arithmetic as nearest_kernel, so bit-identical.
constexpr int kNearestRowBytes = 64 * 1024;
template <typename TIn, int OUT>
__global__ void __launch_bounds__(kBlock) nearest_row_kernel(ResizeLaunch L) {
    using TOut = typename std::conditional<(OUT == kOutSame), TIn, float>::type;
    extern __shared__ uint4 row_lds[];
    const int y = blockIdx.x;
    const int pidx = blockIdx.y;
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;
    const int cc = L.src.cc;
    const int sy = min((int)floor((double)y * L.scale_yd), L.src.h - 1);
    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch +
                              (int64_t)sy * L.src.row_pitch;
    const int row_bytes = L.src.w * cc * (int)sizeof(TIn);
    const int n16 = row_bytes >> 4;
    for (int i = threadIdx.x; i < n16; i += kBlock) row_lds[i] = reinterpret_cast<const uint4*>(sp)[i];
    unsigned char* lb = reinterpret_cast<unsigned char*>(row_lds);
    for (int i = (n16 << 4) + threadIdx.x; i < row_bytes; i += kBlock) lb[i] = sp[i];
    __syncthreads();
    const TIn* row = reinterpret_cast<const TIn*>(lb);
    TOut* dp = reinterpret_cast<TOut*>(const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                                       (int64_t)plane * L.dst.plane_pitch + (int64_t)y * L.dst.row_pitch);
    const int n_el = L.dst.w * cc;
    for (int e = threadIdx.x; e < n_el; e += kBlock) {
        const int x = e / cc, k = e - x * cc;
        const int sx = min((int)floor((double)x * L.scale_xd), L.src.w - 1);
        const TIn v = row[sx * cc + k];
        if (OUT == kOutSame) {
            dp[e] = (TOut)v;
        } else if (OUT == kOutF32) {
            dp[e] = (TOut)(float)v;
        } else {
            const ChanNorm cn = chan_norm(L.norm, img, cc == 1 ? plane % L.norm.c_total : k);
            dp[e] = (TOut)(std::is_same<TIn, uint8_t>::value ? normalize_u8v(cn, (int)v) : normalize_f(cn, (float)v));
        }
    }
}

// INTER_NEAREST, one output row per WAVE (four per workgroup, no barrier):
// the wave stages its source row sy in its own LDS slice with 16-byte loads,
// then each lane takes 4 consecutive output pixels -- the index arithmetic of
// nearest_row_kernel, CC a compile-time constant -- and writes them with one
// 4*CC-element store (u8: dwords; fp32: 16-byte stores).  nearest_row_kernel
// stored one element per lane per instruction (byte stores for u8).
template <typename TIn, int OUT, int CC>
__global__ void __launch_bounds__(kBlock) nearest_wave_kernel(ResizeLaunch L, int row_slice) {
    using TOut = typename std::conditional<(OUT == kOutSame), TIn, float>::type;
    extern __shared__ uint4 row_lds[];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int y = blockIdx.x * 4 + wave;
    if (y >= L.dst.h) return;  // whole wave; no workgroup barrier below
    const int pidx = blockIdx.y;
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;
    const int sy = min((int)floor((double)y * L.scale_yd), L.src.h - 1);
    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch +
                              (int64_t)sy * L.src.row_pitch;
    const int row_bytes = L.src.w * CC * (int)sizeof(TIn);
    uint4* slice = row_lds + wave * (row_slice >> 4);
    const int n16 = row_bytes >> 4;
    for (int i = lane; i < n16; i += 64) {
        const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sp) + i);
        slice[i] = make_uint4(t[0], t[1], t[2], t[3]);
    }
    unsigned char* lb = reinterpret_cast<unsigned char*>(slice);
    for (int i = (n16 << 4) + lane; i < row_bytes; i += 64) lb[i] = sp[i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const TIn* row = reinterpret_cast<const TIn*>(lb);

    ChanNorm cn[CC] = {};
    if (OUT == kOutNorm) {
#pragma unroll
        for (int k = 0; k < CC; ++k) cn[k] = chan_norm(L.norm, img, CC == 1 ? plane % L.norm.c_total : k);
    }
    unsigned char* dp = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                        (int64_t)plane * L.dst.plane_pitch + (int64_t)y * L.dst.row_pitch;
    // vector stores need the output row aligned to the store width
    constexpr int kStore = OUT == kOutSame ? (int)sizeof(TIn) * 4 * CC : 16;
    const bool vec = (reinterpret_cast<uintptr_t>(dp) & ((OUT == kOutSame && sizeof(TIn) == 1) ? 3 : 15)) == 0;
    for (int x0 = 4 * lane; x0 < L.dst.w; x0 += 256) {
        TOut v[4 * CC];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            const int x = min(x0 + p, L.dst.w - 1);
            const int sx = min((int)floor((double)x * L.scale_xd), L.src.w - 1);
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                const TIn t = row[sx * CC + k];
                if (OUT == kOutSame) v[p * CC + k] = (TOut)t;
                else if (OUT == kOutF32) v[p * CC + k] = (TOut)(float)t;
                else v[p * CC + k] = (TOut)(std::is_same<TIn, uint8_t>::value ? normalize_u8v(cn[k], (int)t)
                                                                              : normalize_f(cn[k], (float)t));
            }
        }
        TOut* o = reinterpret_cast<TOut*>(dp) + (int64_t)x0 * CC;
        if (vec && x0 + 4 <= L.dst.w) {
            if constexpr (OUT == kOutSame && sizeof(TIn) == 1) {
#pragma unroll
                for (int d = 0; d < CC; ++d) {
                    const uint32_t w = (uint32_t)v[4 * d] | ((uint32_t)v[4 * d + 1] << 8) | ((uint32_t)v[4 * d + 2] << 16) |
                                       ((uint32_t)v[4 * d + 3] << 24);
                    __builtin_nontemporal_store(w, reinterpret_cast<uint32_t*>(o) + d);
                }
            } else {
#pragma unroll
                for (int q = 0; q < CC; ++q) {
                    u32x4 w;
#pragma unroll
                    for (int e = 0; e < 4; ++e) w[e] = __builtin_bit_cast(uint32_t, v[4 * q + e]);
                    __builtin_nontemporal_store(w, reinterpret_cast<u32x4*>(o) + q);
                }
            }
        } else {
            for (int p = 0; p < 4 && x0 + p < L.dst.w; ++p)
#pragma unroll
                for (int k = 0; k < CC; ++k) o[p * CC + k] = v[p * CC + k];
        }
    }
    (void)kStore;
}

template <typename TIn, int OUT>
hipError_t launch_nearest_wave_cc(const ResizeLaunch& L, hipStream_t s) {
    const int row_slice = (int)(((size_t)L.src.w * L.src.cc * sizeof(TIn) + 15) & ~(size_t)15);
    const dim3 grid((L.dst.h + 3) / 4, L.n * L.src.planes);
    const size_t lds = 4 * (size_t)row_slice;
    switch (L.src.cc) {
        case 1: hipLaunchKernelGGL((nearest_wave_kernel<TIn, OUT, 1>), grid, dim3(kBlock), lds, s, L, row_slice); break;
        case 2: hipLaunchKernelGGL((nearest_wave_kernel<TIn, OUT, 2>), grid, dim3(kBlock), lds, s, L, row_slice); break;
        case 3: hipLaunchKernelGGL((nearest_wave_kernel<TIn, OUT, 3>), grid, dim3(kBlock), lds, s, L, row_slice); break;
        case 4: hipLaunchKernelGGL((nearest_wave_kernel<TIn, OUT, 4>), grid, dim3(kBlock), lds, s, L, row_slice); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <typename TIn>
hipError_t launch_nearest_wave_t(const ResizeLaunch& L, hipStream_t s) {
    if (L.out == kOutSame) return launch_nearest_wave_cc<TIn, kOutSame>(L, s);
    if (L.out == kOutF32) return launch_nearest_wave_cc<TIn, kOutF32>(L, s);
    return launch_nearest_wave_cc<TIn, kOutNorm>(L, s);
}

template <typename TIn>
hipError_t launch_nearest_row_t(const ResizeLaunch& L, hipStream_t s) {
    const dim3 grid(L.dst.h, L.n * L.src.planes);
    const size_t lds = ((size_t)L.src.w * L.src.cc * sizeof(TIn) + 15) & ~(size_t)15;
    if (L.out == kOutSame) hipLaunchKernelGGL((nearest_row_kernel<TIn, kOutSame>), grid, dim3(kBlock), lds, s, L);
    else if (L.out == kOutF32) hipLaunchKernelGGL((nearest_row_kernel<TIn, kOutF32>), grid, dim3(kBlock), lds, s, L);
    else hipLaunchKernelGGL((nearest_row_kernel<TIn, kOutNorm>), grid, dim3(kBlock), lds, s, L);
    return hipGetLastError();
}

template <typename TIn>
hipError_t launch_nearest_t(const ResizeLaunch& L, hipStream_t s) {
    const dim3 grid((L.dst.w + kBlock - 1) / kBlock, L.dst.h, L.n * L.src.planes);
    if (L.out == kOutSame) hipLaunchKernelGGL((nearest_kernel<TIn, kOutSame>), grid, dim3(kBlock), 0, s, L);
    else if (L.out == kOutF32) hipLaunchKernelGGL((nearest_kernel<TIn, kOutF32>), grid, dim3(kBlock), 0, s, L);
    else hipLaunchKernelGGL((nearest_kernel<TIn, kOutNorm>), grid, dim3(kBlock), 0, s, L);
    return hipGetLastError();
}

// --------------------------------------------------------------------------
// INTER_AREA at an integer scale (cv::resize -> resizeAreaFast_ of the pinned
// OpenCV 2.4, the other mode the reference hands to OpenCV, resize.cpp:44-49;
// the reference's own area attempt, src_deprecated/img_resize_inter_area.cpp,
// stops after building the same ofs/xofs tables).  Output pixel (x, y) is the
// mean of the area_x * area_y block at (x * area_x, y * area_y), summed in
// OpenCV's order (block rows, then columns; four taps grouped per add as its
// CV_ENABLE_UNROLLED loop does, which only matters for fp32) and scaled by
// the fp32 1/area; u8 rounds half to even (saturate_cast = cvRound), except
// 2x2 blocks of 1, 3 or 4 channels, which OpenCV routes through
// ResizeAreaFastVec's fast_mode: (a + b + c + d + 2) >> 2, half up
// (L.area_half_up).  One thread per output pixel; a wave reads 64 * area_x *
// cc contiguous elements per block row.
template <typename TIn, int OUT>
__global__ void __launch_bounds__(kBlock) area_fast_kernel(ResizeLaunch L) {
    using TOut = typename std::conditional<(OUT == kOutSame), TIn, float>::type;
    using TSum = typename std::conditional<std::is_same<TIn, uint8_t>::value, int, float>::type;
    const int x = blockIdx.x * kBlock + threadIdx.x;
    const int y = blockIdx.y;
    const int pidx = blockIdx.z;
    if (x >= L.dst.w) return;
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;
    const int cc = L.src.cc, ax = L.area_x, ay = L.area_y, area = ax * ay;
    const unsigned char* row0 = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch +
                                (int64_t)y * ay * L.src.row_pitch;
    TOut* dp = reinterpret_cast<TOut*>(const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                                       (int64_t)plane * L.dst.plane_pitch + (int64_t)y * L.dst.row_pitch) +
               (int64_t)x * cc;
    for (int k = 0; k < cc; ++k) {
        // tap t of the block: row t / ax, column t % ax (OpenCV's ofs table)
        auto tap = [&](int t) -> TSum {
            const int r = t / ax, col = t - r * ax;
            const TIn* sp = reinterpret_cast<const TIn*>(row0 + (int64_t)r * L.src.row_pitch);
            return (TSum)sp[((int64_t)x * ax + col) * cc + k];
        };
        TSum sum = 0;
        int t = 0;
        for (; t <= area - 4; t += 4) sum = sum + (((tap(t) + tap(t + 1)) + tap(t + 2)) + tap(t + 3));
        for (; t < area; ++t) sum = sum + tap(t);
        const float m = __fmul_rn((float)sum, L.area_scale);
        TIn v;
        if (std::is_same<TIn, uint8_t>::value) v = (TIn)(L.area_half_up ? ((int)sum + 2) >> 2 : (int)rintf(m));
        else v = (TIn)m;
        if (OUT == kOutSame) {
            dp[k] = (TOut)v;
        } else if (OUT == kOutF32) {
            dp[k] = (TOut)(float)v;
        } else {
            const ChanNorm cn = chan_norm(L.norm, img, cc == 1 ? plane % L.norm.c_total : k);
            dp[k] = (TOut)(std::is_same<TIn, uint8_t>::value ? normalize_u8v(cn, (int)v) : normalize_f(cn, (float)v));
        }
    }
}

// u8 INTER_AREA by column sums.  An integer sum does not depend on its order,
// so a workgroup takes one output row segment of TW pixels: its threads read
// the ay source rows of the segment as coalesced dwords (a wave reads 256 B per
// instruction), sum each byte column over the ay rows in registers, and park
// the column sums in LDS; then one thread per output element adds its ax
// column sums, rounds and stores (adjacent bytes per lane).  Needs a dword
// aligned source (checked on the host); bit-identical to area_fast_kernel.
constexpr int kAreaSeg = 4096;  // source bytes per segment row (16 KiB of LDS sums)
// u8 INTER_AREA at integer scales: column sums.  A workgroup takes R = 2
// output rows of one segment (tw output pixels): every thread issues the
// loads of its 16-byte (VB) column chunk for all R * ay source rows first --
// twice the bytes in flight of one row at a time, which is what bounded the
// one-row version (measured 0.42 / 0.55 ms at 3x3 / 2x2) -- sums them per
// output row into u16 column sums in LDS (<= 255 * ay), then one thread per
// output element adds its ax column sums.  Integer sums do not depend on
// their order, so the result is resizeAreaFast_'s.
template <int OUT, int VB, int CC>  // VB: source bytes per thread per row (4 or 16); CC: channels (1..4)
__global__ void __launch_bounds__(kBlock) area_u8_colsum_kernel(ResizeLaunch L, int tw, int rows) {
    using TOut = typename std::conditional<(OUT == kOutSame), uint8_t, float>::type;
    using TV = typename std::conditional<(VB == 16), uint4, uint32_t>::type;
    constexpr int R = 2;  // output rows per pass
    __shared__ __attribute__((aligned(16))) unsigned short colsum[R][kAreaSeg];
    const int pidx = blockIdx.z;
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;
    constexpr int cc = CC;
    const int ax = L.area_x, ay = L.area_y;
    const int x0 = blockIdx.x * tw;
    const int pw = min(tw, L.dst.w - x0);          // output pixels in this segment
    const int seg = pw * ax * cc;                  // source bytes per row in this segment
    const int row_bytes = L.src.w * cc;
    const int b0 = x0 * ax * cc;                   // multiple of VB (host picks tw)
    const unsigned char* pbase = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch + b0;
    const int y_end = min(L.dst.h, (int)(blockIdx.y + 1) * rows);
    for (int yp = blockIdx.y * rows; yp < y_end; yp += R) {
        if (yp != (int)blockIdx.y * rows) __syncthreads();  // the previous pass's sums are consumed
        const int nr = min(R, y_end - yp);
        for (int j = threadIdx.x; j * VB < seg; j += kBlock) {
            // packed u16 column sums: even / odd bytes of each dword in two
            // 16-bit lanes (<= 255 * ay < 2^16: no carry crosses a lane)
            constexpr int ND = VB / 4;
            uint32_t ev[R][ND], od[R][ND];
#pragma unroll
            for (int q = 0; q < R; ++q)
#pragma unroll
                for (int d = 0; d < ND; ++d) ev[q][d] = od[q][d] = 0u;
            if (b0 + (j + 1) * VB <= row_bytes) {
                for (int r = 0; r < ay; ++r) {
                    TV t[R];
#pragma unroll
                    for (int q = 0; q < R; ++q)  // both output rows' loads in flight
                        if (q < nr)
                            t[q] = *reinterpret_cast<const TV*>(pbase + (int64_t)((yp + q) * ay + r) * L.src.row_pitch + j * VB);
#pragma unroll
                    for (int q = 0; q < R; ++q) {
                        if (q >= nr) continue;
                        const uint32_t* w = reinterpret_cast<const uint32_t*>(&t[q]);
#pragma unroll
                        for (int d = 0; d < ND; ++d) {
                            ev[q][d] += w[d] & 0x00FF00FFu;
                            od[q][d] += (w[d] >> 8) & 0x00FF00FFu;
                        }
                    }
                }
            } else {  // the row's last partial chunk
                const int lim = row_bytes - (b0 + j * VB);
                for (int q = 0; q < nr; ++q)
                    for (int r = 0; r < ay; ++r) {
                        const unsigned char* p = pbase + (int64_t)((yp + q) * ay + r) * L.src.row_pitch + j * VB;
#pragma unroll
                        for (int i = 0; i < VB; ++i)
                            if (i < lim) {
                                const uint32_t v = (uint32_t)p[i] << (16 * ((i >> 1) & 1));
                                if (i & 1) od[q][i >> 2] += v;
                                else ev[q][i >> 2] += v;
                            }
                    }
            }
#pragma unroll
            for (int q = 0; q < R; ++q)
#pragma unroll
                for (int d = 0; d < ND; ++d) {
                    // bytes 4d .. 4d+3 -> u16 sums {ev.lo, od.lo, ev.hi, od.hi}
                    uint32_t* cw = reinterpret_cast<uint32_t*>(&colsum[q][j * VB + 4 * d]);
                    cw[0] = __builtin_amdgcn_perm(od[q][d], ev[q][d], 0x05040100u);
                    cw[1] = __builtin_amdgcn_perm(od[q][d], ev[q][d], 0x07060302u);
                }
        }
        __syncthreads();
        for (int q = 0; q < nr; ++q) {
            const int y = yp + q;
            TOut* dp = reinterpret_cast<TOut*>(const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                                               (int64_t)plane * L.dst.plane_pitch + (int64_t)y * L.dst.row_pitch) +
                       (int64_t)x0 * cc;
            for (int e = threadIdx.x; e < pw * cc; e += kBlock) {
                const int xl = e / cc, k = e - xl * cc;
                const unsigned short* cs = colsum[q] + xl * ax * cc + k;
                int sum = 0;
                for (int a = 0; a < ax; ++a) sum += cs[a * cc];
                const uint8_t v = L.area_half_up ? (uint8_t)((sum + 2) >> 2)
                                                 : (uint8_t)(int)rintf(__fmul_rn((float)sum, L.area_scale));
                if (OUT == kOutSame) {
                    dp[e] = v;
                } else if (OUT == kOutF32) {
                    dp[e] = (float)v;
                } else {
                    const ChanNorm cn = chan_norm(L.norm, img, cc == 1 ? plane % L.norm.c_total : k);
                    dp[e] = normalize_u8v(cn, (int)v);
                }
            }
        }
    }
}

// u8 INTER_AREA at integer scales, streaming (round 3): a lane owns a UNIT of
// PX output pixels of one row -- U = lcm(16, AX*CC) source bytes of each of
// its ay source rows (16-byte loads, the rows' loads in flight together),
// summed down the rows into packed u16 column sums in registers, then across
// each pixel's AX columns with compile-time byte positions.  No LDS, no
// barrier: the memory shape of a copy (a wave reads 64 consecutive units of
// a row and writes their outputs contiguously).  The LDS column-sum kernel
// above alternated a load phase and an LDS/output phase per workgroup that
// never overlapped (diagnosis builds at 2x2: loads alone 0.263 ms, the rest
// alone 0.250, both 0.519).  Integer sums: bit-identical to it.
// cache policy of the unit kernel's stores (A/B builds: EXTRA=-D0=n)
template <int AX, int CC>
struct AreaUnit {
    static constexpr int gcd(int a, int b) { return b == 0 ? a : gcd(b, a % b); }
    static constexpr int U = 16 / gcd(16, AX * CC) * AX * CC;  // lcm(16, AX * CC)
    static constexpr int NCH = U / 16;                         // 16-byte chunks per row
    static constexpr int PX = U / (AX * CC);                   // output pixels per unit
    static constexpr int OB = PX * CC;                         // output elements per unit
};

template <int OUT, int AX, int CC>
__global__ void __launch_bounds__(kBlock) area_u8_unit_kernel(ResizeLaunch L, int units_per_row, int total, int dst_al,
                                                               int packed) {
    using A = AreaUnit<AX, CC>;
    constexpr int NCH = A::NCH, ND = 4 * NCH, PX = A::PX, OB = A::OB;
    // the wave's 64 units' column sums, chunk-major: 32 bytes (ev, od) per chunk
    __shared__ __attribute__((aligned(16))) uint32_t xch[kBlock / 64][64 * NCH * 8];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int wu0 = (int)blockIdx.x * kBlock + wave * 64;  // the wave's first unit (uniform)
    if (wu0 >= total) return;  // uniform
    const int per_plane = L.dst.h * units_per_row;
    const int ay = L.area_y;
    const uint32_t rp = (uint32_t)L.src.row_pitch;
    // ---- loads: instruction c moves chunk q = 64c + lane of the wave's units
    // (unit q / NCH, its chunk q % NCH), so each is a contiguous run of source
    // bytes, not 64 strided pieces (a unit-per-lane load: 0.60 ms at 2x2 vs
    // 0.52 for the LDS column sums); the column sums are summed per chunk
    // down the rows, then exchanged through the wave's LDS slice
    uint32_t ev[ND], od[ND];
    const unsigned char* cbase[NCH];
    uint32_t coff[NCH];
    bool cok[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const int q = 64 * c + lane;
        const int uq = wu0 + q / NCH, cq = q % NCH;
        cok[c] = uq < total;
        const int g = min(uq, total - 1);
        const int pidx = g / per_plane;
        const int rem = g - pidx * per_plane;
        const int y = rem / units_per_row, u = rem - y * units_per_row;
        const int img = pidx / L.src.planes, plane = pidx - img * L.src.planes;
        cbase[c] = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
        coff[c] = (uint32_t)(y * ay) * rp + (uint32_t)(u * A::U + 16 * cq);
    }
#pragma unroll
    for (int d = 0; d < ND; ++d) ev[d] = od[d] = 0u;
    auto add = [&](int c, const uint4& t) {
        const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            ev[4 * c + d] += w[d] & 0x00FF00FFu;
            od[4 * c + d] += (w[d] >> 8) & 0x00FF00FFu;
        }
    };
    auto load = [&](int c, uint32_t roff) -> uint4 {
        const Rsrc srs = make_rsrc(cbase[c], L.src.plane_bytes);
        const uint32_t lim = (uint32_t)L.src.plane_bytes + srs.delta;
        const uint32_t oc = coff[c] + roff + srs.delta;
        if (!cok[c]) return make_uint4(0u, 0u, 0u, 0u);
        if (oc + 16u <= lim) return load16(srs, oc);
        uint32_t d[4] = {0u, 0u, 0u, 0u};  // the plane's last bytes: a straddling 16-byte load reads as zeros
#pragma unroll 1
        for (uint32_t e = 0; e < 16u; ++e)
            if (oc + e < lim) d[e >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(srs.r, (int)(oc + e), 0, 0) << (8 * (e & 3));
        return make_uint4(d[0], d[1], d[2], d[3]);
    };
    int r = 0;
    for (; r + 2 <= ay; r += 2) {  // two rows of every chunk in flight
        uint4 t0[NCH], t1[NCH];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            t0[c] = load(c, (uint32_t)r * rp);
            t1[c] = load(c, (uint32_t)(r + 1) * rp);
        }
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            add(c, t0[c]);
            add(c, t1[c]);
        }
    }
    if (r < ay) {
#pragma unroll
        for (int c = 0; c < NCH; ++c) add(c, load(c, (uint32_t)r * rp));
    }
    // ---- exchange: chunk q's sums -> slot q; lane l takes its unit's chunks
    uint32_t* xw = xch[wave];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const int q = 64 * c + lane;
        *reinterpret_cast<uint4*>(xw + 8 * q) = make_uint4(ev[4 * c], ev[4 * c + 1], ev[4 * c + 2], ev[4 * c + 3]);
        *reinterpret_cast<uint4*>(xw + 8 * q + 4) = make_uint4(od[4 * c], od[4 * c + 1], od[4 * c + 2], od[4 * c + 3]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
        const int q = NCH * lane + c;
        const uint4 e4 = *reinterpret_cast<const uint4*>(xw + 8 * q);
        const uint4 o4 = *reinterpret_cast<const uint4*>(xw + 8 * q + 4);
        ev[4 * c] = e4.x; ev[4 * c + 1] = e4.y; ev[4 * c + 2] = e4.z; ev[4 * c + 3] = e4.w;
        od[4 * c] = o4.x; od[4 * c + 1] = o4.y; od[4 * c + 2] = o4.z; od[4 * c + 3] = o4.w;
    }
    const int gid = wu0 + lane;
    if (gid >= total) return;
    const int pidx = gid / per_plane;
    const int rem = gid - pidx * per_plane;
    const int y = rem / units_per_row, u = rem - y * units_per_row;
    const int img = pidx / L.src.planes, plane = pidx - img * L.src.planes;
    // output element e: pixel p = e / CC, channel k; its source bytes
    // j = (p * AX + a) * CC + k, a < AX -- all positions compile-time
    auto colsum = [&](int j) -> int {
        const uint32_t w = (j & 1) ? od[j >> 2] : ev[j >> 2];
        return (int)((w >> (16 * ((j >> 1) & 1))) & 0xFFFFu);
    };
    const int vx = min(PX, L.dst.w - u * PX);  // valid pixels (the row's last unit may be partial)
    unsigned char* dp = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                        (int64_t)plane * L.dst.plane_pitch;
    const Rsrc drs = make_rsrc(dp, L.dst.plane_bytes);
    constexpr int ES = OUT == kOutSame ? 1 : 4;
    const uint32_t ro = (uint32_t)y * (uint32_t)L.dst.row_pitch + (uint32_t)(u * OB * ES) + drs.delta;
    uint32_t outw[OUT == kOutSame ? OB / 4 : OB];
#pragma unroll
    for (int e = 0; e < OB; ++e) {
        const int p = e / CC, k = e - p * CC;
        int sum = 0;
#pragma unroll
        for (int a = 0; a < AX; ++a) sum += colsum((p * AX + a) * CC + k);
        const int v = L.area_half_up ? (sum + 2) >> 2 : (int)rintf(__fmul_rn((float)sum, L.area_scale));
        if constexpr (OUT == kOutSame) {
            if (e % 4 == 0) outw[e / 4] = 0u;
            outw[e / 4] |= (uint32_t)(v & 0xFF) << (8 * (e % 4));
        } else if constexpr (OUT == kOutF32) {
            outw[e] = __builtin_bit_cast(uint32_t, (float)v);
        } else {
            const ChanNorm cn = chan_norm(L.norm, img, CC == 1 ? plane % L.norm.c_total : k);
            outw[e] = __builtin_bit_cast(uint32_t, normalize_u8v(cn, v));
        }
    }
    // a packed destination (rows and images back to back, whole units, 16-byte
    // aligned; host-checked) and a whole wave: the 64 units' outputs are one
    // contiguous run -- through the wave's LDS slice as 16-byte non-temporal
    // stores, 1 KiB per instruction (round 5; the lanes' own stores sit a
    // unit's bytes apart)
    if (packed && wu0 + 64 <= total) {  // uniform
        constexpr int NW = OUT == kOutSame ? OB / 4 : OB;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // every lane has read its column sums back
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (int i = 0; i < NW; ++i) xw[NW * lane + i] = outw[i];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        u32x4* o = reinterpret_cast<u32x4*>(const_cast<unsigned char*>(L.dst.base) + (int64_t)wu0 * OB * ES);
#pragma unroll
        for (int j = 0; j < (NW + 3) / 4; ++j) {
            const int q = 64 * j + lane;
            if (q < 16 * NW) __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(xw + 4 * q), o + q);
        }
        return;
    }
    if (vx == PX && dst_al) {  // dword stores (OB * ES is a multiple of 4)
        constexpr int NW = OUT == kOutSame ? OB / 4 : OB;
        if constexpr (NW % 4 == 0) {
#pragma unroll
            for (int i = 0; i < NW; i += 4)
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{outw[i], outw[i + 1], outw[i + 2], outw[i + 3]}, drs.r,
                                                       (int)(ro + 4u * (uint32_t)i), 0, 0);
        } else if constexpr (NW % 2 == 0) {
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int i = 0; i < NW; i += 2)
                __builtin_amdgcn_raw_buffer_store_b64(u32x2{outw[i], outw[i + 1]}, drs.r, (int)(ro + 4u * (uint32_t)i), 0,
                                                      0);
        } else {
#pragma unroll
            for (int i = 0; i < NW; ++i)
                __builtin_amdgcn_raw_buffer_store_b32(outw[i], drs.r, (int)(ro + 4u * (uint32_t)i), 0, 0);
        }
    } else {  // the row's partial last unit or an unaligned destination: element by element
#pragma unroll
        for (int e = 0; e < OB; ++e) {
            if (e >= vx * CC) break;
            if constexpr (OUT == kOutSame)
                __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(outw[e / 4] >> (8 * (e % 4))), drs.r, (int)(ro + (uint32_t)e), 0,
                                                     0);
            else
                __builtin_amdgcn_raw_buffer_store_b32(outw[e], drs.r, (int)(ro + 4u * (uint32_t)e), 0, 0);
        }
    }
}

template <int AX, int CC>
hipError_t launch_area_u8_unit_c(const ResizeLaunch& L, hipStream_t s) {
    using A = AreaUnit<AX, CC>;
    const int upr = (L.dst.w + A::PX - 1) / A::PX;
    const int64_t total = (int64_t)upr * L.dst.h * L.n * L.src.planes;
    if (total >= 0x7FFFFF00LL) return hipErrorInvalidValue;
    const int es = L.out == kOutSame ? 1 : 4;
    const uintptr_t dbits = reinterpret_cast<uintptr_t>(L.dst.base) | (uintptr_t)L.dst.img_pitch |
                            (uintptr_t)L.dst.plane_pitch | (uintptr_t)L.dst.row_pitch;
    // the vector stores need their own width's alignment: a unit's bytes
    // start at u * OB * es within the row
    const int ob = A::OB * es;
    const int wst = ob % 16 == 0 ? 16 : ob % 8 == 0 ? 8 : 4;
    const int dst_al = (dbits % (uintptr_t)wst) == 0;
    // packed: unit g's output starts at g * ob bytes from the base
    const int packed = L.dst.w % A::PX == 0 && L.src.planes == 1 &&
                       L.dst.row_pitch == (int64_t)upr * ob && L.dst.img_pitch == (int64_t)L.dst.h * L.dst.row_pitch &&
                       (reinterpret_cast<uintptr_t>(L.dst.base) & 15) == 0;
    const dim3 grid((unsigned)((total + kBlock - 1) / kBlock));
    if (L.out == kOutSame) hipLaunchKernelGGL((area_u8_unit_kernel<kOutSame, AX, CC>), grid, dim3(kBlock), 0, s, L, upr, (int)total, dst_al, packed);
    else if (L.out == kOutF32) hipLaunchKernelGGL((area_u8_unit_kernel<kOutF32, AX, CC>), grid, dim3(kBlock), 0, s, L, upr, (int)total, dst_al, packed);
    else hipLaunchKernelGGL((area_u8_unit_kernel<kOutNorm, AX, CC>), grid, dim3(kBlock), 0, s, L, upr, (int)total, dst_al, packed);
    return hipGetLastError();
}

// the unit kernel's (AX, CC) instances: U = lcm(16, AX*CC) <= 48 bytes per
// row, so a unit's column sums fit in 24 registers; plane bytes < 2^31
bool area_unit_applies(const ResizeLaunch& L) {
    const int ax = L.area_x, cc = L.src.cc;
    const bool inst = (ax == 2 && cc >= 1 && cc <= 4) || (ax == 3 && cc == 1) || (ax == 4 && cc >= 1 && cc <= 4);
    return inst && L.area_y >= 1 && L.area_y <= 257 && L.src.plane_bytes < (1LL << 31) - 64 &&
           L.dst.plane_bytes < (1LL << 31) - 64;
}

hipError_t launch_area_u8_unit(const ResizeLaunch& L, hipStream_t s) {
    switch (L.area_x * 8 + L.src.cc) {
        case 17: return launch_area_u8_unit_c<2, 1>(L, s);
        case 18: return launch_area_u8_unit_c<2, 2>(L, s);
        case 19: return launch_area_u8_unit_c<2, 3>(L, s);
        case 20: return launch_area_u8_unit_c<2, 4>(L, s);
        case 25: return launch_area_u8_unit_c<3, 1>(L, s);
        case 33: return launch_area_u8_unit_c<4, 1>(L, s);
        case 34: return launch_area_u8_unit_c<4, 2>(L, s);
        case 35: return launch_area_u8_unit_c<4, 3>(L, s);
        case 36: return launch_area_u8_unit_c<4, 4>(L, s);
        default: return hipErrorInvalidValue;
    }
}

template <int VB, int CC>
hipError_t launch_area_u8_colsum_c(const ResizeLaunch& L, hipStream_t s, int tw, int rows, dim3 grid) {
    if (L.out == kOutSame) hipLaunchKernelGGL((area_u8_colsum_kernel<kOutSame, VB, CC>), grid, dim3(kBlock), 0, s, L, tw, rows);
    else if (L.out == kOutF32) hipLaunchKernelGGL((area_u8_colsum_kernel<kOutF32, VB, CC>), grid, dim3(kBlock), 0, s, L, tw, rows);
    else hipLaunchKernelGGL((area_u8_colsum_kernel<kOutNorm, VB, CC>), grid, dim3(kBlock), 0, s, L, tw, rows);
    return hipGetLastError();
}

template <int VB>
hipError_t launch_area_u8_colsum_t(const ResizeLaunch& L, hipStream_t s, int tw, int rows, dim3 grid) {
    switch (L.src.cc) {  // NHWC c <= 4 (vacv_abi.cpp), NCHW planes have cc = 1
        case 1: return launch_area_u8_colsum_c<VB, 1>(L, s, tw, rows, grid);
        case 2: return launch_area_u8_colsum_c<VB, 2>(L, s, tw, rows, grid);
        case 3: return launch_area_u8_colsum_c<VB, 3>(L, s, tw, rows, grid);
        case 4: return launch_area_u8_colsum_c<VB, 4>(L, s, tw, rows, grid);
        default: return hipErrorInvalidValue;
    }
}

// vb: the source's alignment (4 or 16); segments of tw pixels start vb-aligned
hipError_t launch_area_u8_colsum(const ResizeLaunch& L, hipStream_t s, int vb) {
    const int per_px = L.area_x * L.src.cc;
    const int tw_max = (kAreaSeg / per_px) & ~(vb - 1);
    const int nblk = (L.dst.w + tw_max - 1) / tw_max;
    const int tw = ((L.dst.w + nblk - 1) / nblk + vb - 1) & ~(vb - 1);
    const int rows = std::max(1, tune_or(VACV_TUNE_AREA_ROWS, 4));  // output rows per workgroup (2 per pass; 4: 0.51 vs 0.53 ms at 2x2)
    const dim3 grid(nblk, (L.dst.h + rows - 1) / rows, L.n * L.src.planes);
    return vb == 16 ? launch_area_u8_colsum_t<16>(L, s, tw, rows, grid)
                    : launch_area_u8_colsum_t<4>(L, s, tw, rows, grid);
}

// u8 INTER_AREA at integer scales, lane-stationary (round 5), for the shapes
// whose unit (lcm(16, AX*CC) bytes) is too wide for area_u8_unit_kernel's
// registers -- 3x3 over BGR / BGRA, 1080p -> 640x360 among them.  A lane
// owns PXL = 4 / gcd(4, AX*CC) consecutive output pixels of one row, i.e. NW
// = PXL*AX*CC/4 whole, dword-aligned source dwords of each of its AY source
// rows (no byte shifts, no LDS): all AY rows' loads are issued together,
// summed down the rows as packed u16 pairs (even / odd bytes, 255 * AY <
// 2^16), then across each pixel's AX columns at compile-time byte positions.
// A wave is 64 * PXL output pixels of a row; its loads of a source row cover
// one contiguous run of 256 * NW bytes (3x3 BGR: 2,304 B = 18 whole lines
// where the row starts on a line), its output one contiguous run too.
// Integer sums, then OpenCV's rounding: bit-identical to the other kernels.
template <int AX, int CC>
struct AreaLane {
    static constexpr int gcd(int a, int b) { return b == 0 ? a : gcd(b, a % b); }
    static constexpr int PXL = 4 / gcd(4, AX * CC);  // output pixels per lane
    static constexpr int NW = PXL * AX * CC / 4;      // source dwords per lane and row
    static constexpr int OB = PXL * CC;               // output elements per lane
};

// area_lane_kernel: output rows per wave, the next row's loads in flight while
// one is summed (1 / 2 / 4 / 8: 0.369 / 0.382 / 0.385 / 0.418 ms)
constexpr int kAreaRG = 1;
template <int OUT, int AX, int CC>
__global__ void __launch_bounds__(kBlock) area_lane_kernel(ResizeLaunch L, int blocks_per_row, int tasks, int dst_al) {
    using A = AreaLane<AX, CC>;
    constexpr int PXL = A::PXL, NW = A::NW, OB = A::OB;
    constexpr int RG = kAreaRG;
    static_assert(OB % 4 == 0 || OUT != kOutSame, "u8 output as whole dwords");
    const int lane = threadIdx.x & 63;
    const int task = (int)blockIdx.x * (kBlock / 64) + __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    if (task >= tasks) return;  // whole wave
    const int groups = (L.dst.h + RG - 1) / RG;
    const int blk = task % blocks_per_row;
    const int rest = task / blocks_per_row;
    const int y0 = (rest % groups) * RG;
    const int pidx = rest / groups;
    const int img = pidx / L.src.planes, plane = pidx - img * L.src.planes;
    const int x0 = (blk * 64 + lane) * PXL;  // the lane's first output pixel
    const int vx = min(PXL, L.dst.w - x0);    // its valid pixels (<= 0: none)
    const bool full = (blk + 1) * 64 * PXL <= L.dst.w;  // uniform: every lane has PXL pixels
    const Rsrc srs = make_rsrc(L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch,
                               L.src.plane_bytes);
    const uint32_t rp = (uint32_t)L.src.row_pitch;
    const uint32_t lo = (uint32_t)(x0 * AX * CC) + srs.delta;

    // one source row's NW dwords: 16-byte loads where the wave is whole; else
    // dword loads, and bytewise the one dword that straddles the plane's
    // last byte (a straddling load reads as zeros)
    const uint32_t slim = (uint32_t)L.src.plane_bytes + srs.delta;
    auto load_row = [&](uint32_t off, uint32_t (&d)[NW]) {
        if (full) {
            int q = 0;
#pragma unroll
            for (; q + 4 <= NW; q += 4) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(srs.r, (int)(off + 4 * q), 0, 0);
                d[q] = v[0]; d[q + 1] = v[1]; d[q + 2] = v[2]; d[q + 3] = v[3];
            }
            if constexpr (NW % 4 == 3) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b96(srs.r, (int)(off + 4 * q), 0, 0);
                d[q] = v[0]; d[q + 1] = v[1]; d[q + 2] = v[2];
            } else if constexpr (NW % 4 == 2) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b64(srs.r, (int)(off + 4 * q), 0, 0);
                d[q] = v[0]; d[q + 1] = v[1];
            } else if constexpr (NW % 4 == 1) {
                d[q] = __builtin_amdgcn_raw_buffer_load_b32(srs.r, (int)(off + 4 * q), 0, 0);
            }
        } else {
#pragma unroll
            for (int q = 0; q < NW; ++q) {
                const uint32_t o = off + 4u * (uint32_t)q;
                if (o + 4u <= slim) {
                    d[q] = __builtin_amdgcn_raw_buffer_load_b32(srs.r, (int)o, 0, 0);
                } else {
                    uint32_t v = 0;
#pragma unroll
                    for (uint32_t e = 0; e < 4u; ++e)
                        if (o + e < slim) v |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(srs.r, (int)(o + e), 0, 0) << (8 * e);
                    d[q] = v;
                }
            }
        }
    };
    uint32_t ev[NW], od[NW];
    auto clear = [&]() {
#pragma unroll
        for (int q = 0; q < NW; ++q) ev[q] = od[q] = 0u;
    };
    auto add = [&](const uint32_t (&d)[NW]) {
#pragma unroll
        for (int q = 0; q < NW; ++q) {
            ev[q] += __builtin_amdgcn_perm(0u, d[q], 0x0C020C00u);  // bytes 0, 2 as u16 pairs
            od[q] += __builtin_amdgcn_perm(0u, d[q], 0x0C030C01u);  // bytes 1, 3
        }
    };
    // output element e: pixel p = e / CC, channel k; its source bytes
    // j = (p * AX + a) * CC + k, a < AX -- all positions compile-time
    auto colsum = [&](int j) -> int {
        const uint32_t w = (j & 1) ? od[j >> 2] : ev[j >> 2];
        return (int)((w >> (16 * ((j >> 1) & 1))) & 0xFFFFu);
    };
    unsigned char* dp = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                        (int64_t)plane * L.dst.plane_pitch;
    const Rsrc drs = make_rsrc(dp, L.dst.plane_bytes);
    constexpr int ES = OUT == kOutSame ? 1 : 4;
    auto emit = [&](int y) {
        if (vx <= 0) return;
        const uint32_t ro = (uint32_t)y * (uint32_t)L.dst.row_pitch + (uint32_t)(x0 * CC * ES) + drs.delta;
        uint32_t outw[OUT == kOutSame ? (OB + 3) / 4 : OB];
#pragma unroll
        for (int e = 0; e < OB; ++e) {
            const int p = e / CC, k = e - p * CC;
            int sum = 0;
#pragma unroll
            for (int a = 0; a < AX; ++a) sum += colsum((p * AX + a) * CC + k);
            const int v = L.area_half_up ? (sum + 2) >> 2 : (int)rintf(__fmul_rn((float)sum, L.area_scale));
            if constexpr (OUT == kOutSame) {
                if (e % 4 == 0) outw[e / 4] = 0u;
                outw[e / 4] |= (uint32_t)(v & 0xFF) << (8 * (e % 4));
            } else if constexpr (OUT == kOutF32) {
                outw[e] = __builtin_bit_cast(uint32_t, (float)v);
            } else {
                const ChanNorm cn = chan_norm(L.norm, img, CC == 1 ? plane % L.norm.c_total : k);
                outw[e] = __builtin_bit_cast(uint32_t, normalize_u8v(cn, v));
            }
        }
        constexpr int NO = OUT == kOutSame ? OB / 4 : OB;  // output dwords per lane
        if (vx == PXL && dst_al) {
            int i = 0;
#pragma unroll
            for (; i + 4 <= NO; i += 4)
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{outw[i], outw[i + 1], outw[i + 2], outw[i + 3]}, drs.r,
                                                       (int)(ro + 4u * (uint32_t)i), 0, 0);
            if constexpr (NO % 4 == 3) {
                typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
                __builtin_amdgcn_raw_buffer_store_b96(u32x3{outw[i], outw[i + 1], outw[i + 2]}, drs.r, (int)(ro + 4u * (uint32_t)i), 0, 0);
            } else if constexpr (NO % 4 == 2) {
                typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                __builtin_amdgcn_raw_buffer_store_b64(u32x2{outw[i], outw[i + 1]}, drs.r, (int)(ro + 4u * (uint32_t)i), 0, 0);
            } else if constexpr (NO % 4 == 1) {
                __builtin_amdgcn_raw_buffer_store_b32(outw[i], drs.r, (int)(ro + 4u * (uint32_t)i), 0, 0);
            }
        } else {  // the row's partial last lane or an unaligned destination: element by element
#pragma unroll
            for (int e = 0; e < OB; ++e) {
                if (e >= vx * CC) break;
                if constexpr (OUT == kOutSame)
                    __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(outw[e / 4] >> (8 * (e % 4))), drs.r, (int)(ro + (uint32_t)e), 0, 0);
                else
                    __builtin_amdgcn_raw_buffer_store_b32(outw[e], drs.r, (int)(ro + 4u * (uint32_t)e), 0, 0);
            }
        }
    };
    if (full && L.area_y <= 257) {
        // uniform (whole waves): the wave's run of 16 NW chunks of a source
        // row moves as lane-contiguous 16-byte loads (chunk 64 i + lane), is
        // summed down the rows per chunk, and goes to the lanes' windows
        // through the wave's own LDS slice -- the loads then cover whole lines
        // per instruction instead of 64 windows NW dwords apart
        constexpr int NCK = 16 * NW;           // 16-byte chunks of the run (64 lanes x NW dwords)
        constexpr int NI = (NCK + 63) / 64;    // load instructions per source row
        __shared__ __attribute__((aligned(16))) uint32_t xs[kBlock / 64][2][4 * NCK];
        const int wv = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
        const uint32_t run = (uint32_t)(blk * 64 * PXL * AX * CC) + srs.delta;  // the run's first byte
        for (int k = 0; k < RG; ++k) {
            const int y = y0 + k;
            if (y >= L.dst.h) break;  // uniform
            uint32_t cev[NI][4], cod[NI][4];
#pragma unroll
            for (int i = 0; i < NI; ++i) {
#pragma unroll
                for (int d = 0; d < 4; ++d) cev[i][d] = cod[i][d] = 0u;
            }
            const uint32_t ry = run + (uint32_t)(y * L.area_y) * rp;
            for (int r = 0; r < L.area_y; ++r) {
                u32x4 t[NI];
#pragma unroll
                for (int i = 0; i < NI; ++i) {
                    const int q = 64 * i + lane;
                    t[i] = q < NCK ? __builtin_amdgcn_raw_buffer_load_b128(srs.r, (int)(ry + (uint32_t)r * rp + 16u * (uint32_t)q), 0, 0)
                                   : u32x4{0u, 0u, 0u, 0u};
                }
#pragma unroll
                for (int i = 0; i < NI; ++i) {
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        cev[i][d] += __builtin_amdgcn_perm(0u, t[i][d], 0x0C020C00u);
                        cod[i][d] += __builtin_amdgcn_perm(0u, t[i][d], 0x0C030C01u);
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < NI; ++i) {
                const int q = 64 * i + lane;
                if (q < NCK) {
                    *reinterpret_cast<u32x4*>(&xs[wv][0][4 * q]) = u32x4{cev[i][0], cev[i][1], cev[i][2], cev[i][3]};
                    *reinterpret_cast<u32x4*>(&xs[wv][1][4 * q]) = u32x4{cod[i][0], cod[i][1], cod[i][2], cod[i][3]};
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int q = 0; q < NW; ++q) {
                ev[q] = xs[wv][0][NW * lane + q];
                od[q] = xs[wv][1][NW * lane + q];
            }
            emit(y);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();  // the next row reuses the slice
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
        return;
    }
    if (L.area_y == 3) {
        // uniform: the 3 source rows of output row y + 1 are in flight while
        // row y is summed and stored
        uint32_t b[2][3][NW];
        auto issue = [&](int y, uint32_t (&t)[3][NW]) {
#pragma unroll
            for (int i = 0; i < 3; ++i) load_row(lo + (uint32_t)(3 * y + i) * rp, t[i]);
        };
        issue(y0, b[0]);
#pragma unroll
        for (int k = 0; k < RG; ++k) {
            const int y = y0 + k;
            if (y >= L.dst.h) break;  // uniform
            if (k + 1 < RG && y + 1 < L.dst.h) issue(y + 1, b[(k + 1) & 1]);
            clear();
#pragma unroll
            for (int i = 0; i < 3; ++i) add(b[k & 1][i]);
            emit(y);
        }
        return;
    }
    for (int k = 0; k < RG; ++k) {
        const int y = y0 + k;
        if (y >= L.dst.h) break;  // uniform
        clear();
        const uint32_t ry = lo + (uint32_t)(y * L.area_y) * rp;
        int r = 0;
        for (; r + 2 <= L.area_y; r += 2) {  // two rows in flight
            uint32_t d0[NW], d1[NW];
            load_row(ry + (uint32_t)r * rp, d0);
            load_row(ry + (uint32_t)(r + 1) * rp, d1);
            add(d0);
            add(d1);
        }
        if (r < L.area_y) {
            uint32_t d0[NW];
            load_row(ry + (uint32_t)r * rp, d0);
            add(d0);
        }
        emit(y);
    }
}

template <int AX, int CC>
hipError_t launch_area_lane_c(const ResizeLaunch& L, hipStream_t s) {
    using A = AreaLane<AX, CC>;
    const int bpr = (L.dst.w + 64 * A::PXL - 1) / (64 * A::PXL);
    const int64_t tasks = (int64_t)bpr * ((L.dst.h + kAreaRG - 1) / kAreaRG) * L.n * L.src.planes;
    if (tasks >= 0x7FFFFF00LL) return hipErrorInvalidValue;
    const int es = L.out == kOutSame ? 1 : 4;
    const uintptr_t dbits = reinterpret_cast<uintptr_t>(L.dst.base) | (uintptr_t)L.dst.img_pitch |
                            (uintptr_t)L.dst.plane_pitch | (uintptr_t)L.dst.row_pitch;
    // a lane's output starts at x0 * CC * es bytes: aligned to the widest store it issues
    const int ob = A::OB * es;
    const int wst = ob % 16 == 0 ? 16 : ob % 8 == 0 ? 8 : 4;
    const int dst_al = (dbits % (uintptr_t)wst) == 0;
    const dim3 grid((unsigned)((tasks + kBlock / 64 - 1) / (kBlock / 64)));
    if (L.out == kOutSame) hipLaunchKernelGGL((area_lane_kernel<kOutSame, AX, CC>), grid, dim3(kBlock), 0, s, L, bpr, (int)tasks, dst_al);
    else if (L.out == kOutF32) hipLaunchKernelGGL((area_lane_kernel<kOutF32, AX, CC>), grid, dim3(kBlock), 0, s, L, bpr, (int)tasks, dst_al);
    else hipLaunchKernelGGL((area_lane_kernel<kOutNorm, AX, CC>), grid, dim3(kBlock), 0, s, L, bpr, (int)tasks, dst_al);
    return hipGetLastError();
}

// the lane kernel's (AX, CC) instances; plane bytes < 2^31
bool area_lane_applies(const ResizeLaunch& L) {
    const int ax = L.area_x, cc = L.src.cc;
    return ((ax == 3 && (cc == 3 || cc == 4))) && L.area_y >= 1 && L.area_y <= 257 &&
           L.src.plane_bytes < (1LL << 31) - 64 && L.dst.plane_bytes < (1LL << 31) - 64;
}

hipError_t launch_area_lane(const ResizeLaunch& L, hipStream_t s) {
    if (L.src.cc == 3) return launch_area_lane_c<3, 3>(L, s);
    return launch_area_lane_c<3, 4>(L, s);
}

template <typename TIn>
hipError_t launch_area_t(const ResizeLaunch& L, hipStream_t s) {
    const dim3 grid((L.dst.w + kBlock - 1) / kBlock, L.dst.h, L.n * L.src.planes);
    if (L.out == kOutSame) hipLaunchKernelGGL((area_fast_kernel<TIn, kOutSame>), grid, dim3(kBlock), 0, s, L);
    else if (L.out == kOutF32) hipLaunchKernelGGL((area_fast_kernel<TIn, kOutF32>), grid, dim3(kBlock), 0, s, L);
    else hipLaunchKernelGGL((area_fast_kernel<TIn, kOutNorm>), grid, dim3(kBlock), 0, s, L);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_resize_nearest(const ResizeLaunch& L, hipStream_t s) {
    if (L.dst.h > 65535 || (int64_t)L.n * L.src.planes > 65535) return hipErrorInvalidValue;
    const int64_t row_bytes = (int64_t)L.src.w * L.src.cc * L.src.esize;
    const uintptr_t bits = reinterpret_cast<uintptr_t>(L.src.base) | (uintptr_t)L.src.img_pitch |
                           (uintptr_t)L.src.plane_pitch | (uintptr_t)L.src.row_pitch;
    // the row kernel reads the whole source row: only where the samples are
    // at most a cache line apart, so it moves no more lines than the gathers
    // (a 4096-px fp32 row sampled 32 times would read 64 KiB for 32 pixels)
    const bool dense_samples = L.scale_xd * L.src.cc * L.src.esize <= 128.0;
    const int knob = tune(VACV_TUNE_NEAREST_KERNEL);  // 0 per-pixel, 1 row per workgroup, else row per wave
    if ((bits & 15) == 0 && row_bytes <= kNearestRowBytes / 4 && dense_samples && L.src.cc <= 4 && knob != 0 && knob != 1)
        return L.src.esize == 1 ? launch_nearest_wave_t<uint8_t>(L, s) : launch_nearest_wave_t<float>(L, s);
    if ((bits & 15) == 0 && row_bytes <= kNearestRowBytes && dense_samples && knob != 0)
        return L.src.esize == 1 ? launch_nearest_row_t<uint8_t>(L, s) : launch_nearest_row_t<float>(L, s);
    return L.src.esize == 1 ? launch_nearest_t<uint8_t>(L, s) : launch_nearest_t<float>(L, s);
}

hipError_t launch_resize_area(const ResizeLaunch& L, hipStream_t s) {
    if (L.dst.h > 65535 || (int64_t)L.n * L.src.planes > 65535) return hipErrorInvalidValue;
    if (L.area_x < 1 || L.area_y < 1 || (int64_t)L.dst.w * L.area_x != L.src.w ||
        (int64_t)L.dst.h * L.area_y != L.src.h)
        return hipErrorInvalidValue;  // the kernel reads exactly the source extent
    if (L.src.esize == 1) {
        const uintptr_t bits = reinterpret_cast<uintptr_t>(L.src.base) | (uintptr_t)L.src.img_pitch |
                               (uintptr_t)L.src.plane_pitch | (uintptr_t)L.src.row_pitch;
        // A/B: 1 per-pixel, 2 dword column sums, 3 16-byte column sums (LDS);
        // default: the unit kernel, else the lane kernel, where they apply
        const int knob = tune(VACV_TUNE_AREA_KERNEL);
        if ((bits & 15) == 0 && knob <= 0 && area_unit_applies(L)) return launch_area_u8_unit(L, s);
        if ((bits & 3) == 0 && knob <= 0 && area_lane_applies(L)) return launch_area_lane(L, s);
        const int vb = (bits & 15) == 0 && L.area_x * L.src.cc <= 256 ? 16 : (bits & 3) == 0 ? 4 : 0;
        if (vb && L.area_x * L.src.cc <= 1024 && L.area_y <= 257 && knob != 1)  // u16 column sums: 255 * ay < 2^16
            return launch_area_u8_colsum(L, s, knob == 2 ? 4 : vb);
        return launch_area_t<uint8_t>(L, s);
    }
    return launch_area_t<float>(L, s);
}

namespace {

}  // namespace

hipError_t launch_row_copy(const CopyLaunch& L, hipStream_t s) {
    const int64_t rows = (int64_t)L.src.planes * L.src.h * L.n;
    int g = (int)std::min<int64_t>((rows + 3) / 4, 256 * 32);
    hipLaunchKernelGGL(row_copy_kernel, dim3(g < 1 ? 1 : g), dim3(kBlock), 0, s, L);
    return hipGetLastError();
}

hipError_t launch_layout(const LayoutLaunch& L, hipStream_t s) {
    const int64_t hw = (int64_t)L.w * L.h;
    const bool aligned = ((reinterpret_cast<uintptr_t>(L.src) | reinterpret_cast<uintptr_t>(L.dst)) & 3) == 0 &&
                         (L.src_img & 3) == 0 && (L.dst_img & 3) == 0;
    if (L.esize == 1 && L.c == 3 && hw % 4 == 0 && aligned) {
        const int g = grid_for(hw / 4 * L.n);
        if (L.to_chw) hipLaunchKernelGGL(hwc3_to_chw_u8_kernel, dim3(g), dim3(kBlock), 0, s, L);
        else hipLaunchKernelGGL(chw_to_hwc3_u8_kernel, dim3(g), dim3(kBlock), 0, s, L);
        return hipGetLastError();
    }
    const int g = grid_for(hw * L.c * L.n);
    switch (L.esize) {
        case 1: hipLaunchKernelGGL(layout_kernel<uint8_t>, dim3(g), dim3(kBlock), 0, s, L); break;
        case 2: hipLaunchKernelGGL(layout_kernel<uint16_t>, dim3(g), dim3(kBlock), 0, s, L); break;
        case 4: hipLaunchKernelGGL(layout_kernel<uint32_t>, dim3(g), dim3(kBlock), 0, s, L); break;
        case 8: hipLaunchKernelGGL(layout_kernel<uint64_t>, dim3(g), dim3(kBlock), 0, s, L); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_dtype(const DtypeLaunch& L, hipStream_t s) {
    const uintptr_t a8 = reinterpret_cast<uintptr_t>(L.to_f32 ? L.src : L.dst);
    const uintptr_t a32 = reinterpret_cast<uintptr_t>(L.to_f32 ? L.dst : L.src);
    const int64_t threads = (L.count >> 2) + (L.count & 3);
    if ((a8 & 3) == 0 && (a32 & 15) == 0 && threads <= (int64_t)0x7FFFFFFF * kBlock) {
        const unsigned blocks = (unsigned)((threads + kBlock - 1) / kBlock);
        if (L.to_f32) hipLaunchKernelGGL(u8_to_f32_flat_kernel, dim3(blocks), dim3(kBlock), 0, s, L);
        else hipLaunchKernelGGL(f32_to_u8_flat_kernel, dim3(blocks), dim3(kBlock), 0, s, L);
        return hipGetLastError();
    }
    const int g = grid_for(L.count / 16 + 1);
    if (L.to_f32) hipLaunchKernelGGL(u8_to_f32_kernel, dim3(g), dim3(kBlock), 0, s, L);
    else hipLaunchKernelGGL(f32_to_u8_kernel, dim3(g), dim3(kBlock), 0, s, L);
    return hipGetLastError();
}

hipError_t launch_color(const ColorLaunch& L, hipStream_t s) {
    dim3 block(64, 4);
    dim3 grid((L.w / 4 + 64) / 64, (L.h / 2 + 4 * kColorPairs - 1) / (4 * kColorPairs), L.n);
    if (L.out == kOutSame) hipLaunchKernelGGL(color_kernel<kOutSame>, grid, block, 0, s, L);
    else if (L.out == kOutF32) hipLaunchKernelGGL(color_kernel<kOutF32>, grid, block, 0, s, L);
    else hipLaunchKernelGGL(color_kernel<kOutNorm>, grid, block, 0, s, L);
    return hipGetLastError();
}

hipError_t launch_normalize(const NormLaunch& L, hipStream_t s) {
    const int64_t row_elems = (int64_t)L.src.w * L.src.cc;
    const int64_t total = (row_elems + 3) / 4 * L.src.h * L.src.planes * L.n;
    const int g = grid_for(total);
    if (L.src_u8) hipLaunchKernelGGL(normalize_kernel<uint8_t>, dim3(g), dim3(kBlock), 0, s, L);
    else hipLaunchKernelGGL(normalize_kernel<float>, dim3(g), dim3(kBlock), 0, s, L);
    return hipGetLastError();
}

hipError_t launch_channel_sums(const SumsLaunch& L, hipStream_t s) {
    if (L.src_u8) return launch_sums_t<uint8_t>(L, s);
    return launch_sums_t<float>(L, s);
}

hipError_t launch_stats(const double* sums, int groups, int c, double count, float* mean, float* stddev,
                        hipStream_t s) {
    const int work = groups * c;
    hipLaunchKernelGGL(stats_kernel, dim3((work + 255) / 256), dim3(256), 0, s, sums, groups, c, count, mean, stddev);
    return hipGetLastError();
}

}  // namespace vacv
