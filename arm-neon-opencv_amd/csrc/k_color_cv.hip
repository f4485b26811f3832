// k_color_cv.hip -- the cvt_color codes the reference hands to cv::cvtColor
// (cvt_color.cpp:139-141; cv.h:62-74), restated from OpenCV 2.4.13:
//  * COLOR_YUV2RGBA/BGRA_NV12/NV21 (94-97) and COLOR_YUV2BGR_YV12 (99):
//    YUV420sp2RGB8 / YUV420p2RGB8 -- ITU-R BT.601 in 20-bit fixed point,
//      y' = max(0, Y - 16) * 1220542
//      R = sat((y' + 2^19 + 1673527 v) >> 20)
//      G = sat((y' + 2^19 - 852492 v - 409993 u) >> 20)
//      B = sat((y' + 2^19 + 2116026 u) >> 20),    u = U - 128, v = V - 128
//    (the constants as OpenCV 2.4.13.4's own YUV2RGBA_NV12 kernel states
//    them); alpha 255;
//  * COLOR_GRAY2BGR (8) / GRAY2BGRA: the value in every colour channel.
// The codes the reference decodes itself (YUV2BGR_NV21 / _NV12, its 7-bit
// naive arithmetic) stay in color_kernel (k_pixel.hip).  Parity unpinned: the
// oracle (oracle_yuv420_cv, oracle_gray_to_bgr) restates the same formulas
// and no OpenCV runs here.
//
// Memory-bound and off the benchmarked path: one thread decodes a 2x2 block
// (shared chroma) and writes its two row pairs with the widest store the
// destination alignment allows (host-checked).
#pragma clang fp contract(off)

#include "vacv_device.hpp"

namespace vacv {
namespace {

__device__ __forceinline__ uint32_t sat_u8(int v) { return (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// one pixel: BGR(A) or RGB(A) bytes packed little-endian (byte k = channel k)
__device__ __forceinline__ uint32_t bt601(int Y, int ruv, int guv, int buv, int bidx) {
    const int yy = max(0, Y - 16) * 1220542;
    const uint32_t r = sat_u8((yy + ruv) >> 20), g = sat_u8((yy + guv) >> 20), b = sat_u8((yy + buv) >> 20);
    return bidx == 0 ? (b | (g << 8) | (r << 16) | 0xFF000000u) : (r | (g << 8) | (b << 16) | 0xFF000000u);
}

// layout: 0 NV12, 1 NV21, 2 YV12 (Y, V, U planes), 3 IYUV (Y, U, V)
template <int DCN>
__global__ void __launch_bounds__(256) yuv420_cv_kernel(CvColorLaunch L) {
    const int bw = L.w >> 1, bh = L.h >> 1;
    const int64_t blocks = (int64_t)bw * bh;
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int img = blockIdx.y;
    if (t >= blocks) return;
    const int by = (int)(t / bw), bx = (int)(t - (int64_t)by * bw);
    const unsigned char* s = L.src + (int64_t)img * L.src_img;
    const unsigned char* y0 = s + (int64_t)(2 * by) * L.src_row + 2 * bx;
    int U, V;
    if (L.layout <= 1) {
        const unsigned char* uv = s + (int64_t)(L.h + by) * L.src_row + 2 * bx;
        U = uv[L.layout];
        V = uv[1 - L.layout];
    } else {
        // planar chroma: (w/2) x (h/2) planes right after the Y plane, rows
        // of w/2 bytes (OpenCV's contiguous YUV420p)
        const unsigned char* c0 = s + (int64_t)L.h * L.src_row;
        const int64_t q = (int64_t)bw * bh, k = (int64_t)by * bw + bx;
        const int p0 = c0[k], p1 = c0[q + k];
        U = L.layout == 2 ? p1 : p0;
        V = L.layout == 2 ? p0 : p1;
    }
    const int u = U - 128, v = V - 128;
    const int ruv = (1 << 19) + 1673527 * v;
    const int guv = (1 << 19) - 852492 * v - 409993 * u;
    const int buv = (1 << 19) + 2116026 * u;
    unsigned char* d = L.dst + (int64_t)img * L.dst_img + (int64_t)(2 * by) * L.dst_row + (int64_t)(2 * bx) * DCN;
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const unsigned char* yr = y0 + r * L.src_row;
        const uint32_t p0 = bt601(yr[0], ruv, guv, buv, L.bidx), p1 = bt601(yr[1], ruv, guv, buv, L.bidx);
        unsigned char* o = d + r * L.dst_row;
        if (DCN == 4 && L.aligned) {
            *reinterpret_cast<uint2*>(o) = make_uint2(p0, p1);
        } else if (DCN == 3 && L.aligned) {  // 6 bytes at a 2-byte aligned address
            unsigned short* o2 = reinterpret_cast<unsigned short*>(o);
            o2[0] = (unsigned short)p0;
            o2[1] = (unsigned short)(((p0 >> 16) & 0xFFu) | (p1 << 8));  // r0, b1 (not p0's alpha)
            o2[2] = (unsigned short)(p1 >> 8);
        } else {
#pragma unroll
            for (int k = 0; k < DCN; ++k) {
                o[k] = (unsigned char)(p0 >> (8 * k));
                o[DCN + k] = (unsigned char)(p1 >> (8 * k));
            }
        }
    }
}

// GRAY2BGR(A): a thread takes a unit of PX pixels of one row (u8: 16, one
// 16-byte load and 3 or 4 16-byte stores; fp32: 4, the same in floats) where
// the unit is whole and the host found every base and pitch 16-byte aligned;
// elementwise otherwise (a row's last partial unit, unaligned images).  Round
// 3's one-pixel-per-thread kernel (byte loads, 3 byte stores) ran at 0.21 of
// 8 TB/s; 4-pixel u8 units (a dword in, dwordx3 out) 0.56.
// The same decode with a thread per 8 x 2 pixels (4 chroma samples), for
// images whose width is a multiple of 8 with every base and pitch aligned
// (host-checked): Y as two 8-byte loads, the chroma as one 8-byte (NV12/21)
// or two 4-byte (planar) loads, each output row segment as 16-byte (BGRA: 32
// bytes) or 8-byte (BGR: 24 bytes) stores.  The 2 x 2 kernel above issued
// byte loads and 2-byte stores (nv21 -> BGRA 0.48, YV12 -> BGR 0.35 of 8 TB/s).
template <int DCN>
__global__ void __launch_bounds__(256) yuv420_cv8_kernel(CvColorLaunch L, int upr) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int img = blockIdx.y;
    const int bh = L.h >> 1;
    if (t >= (int64_t)upr * bh) return;
    const int by = (int)(t / upr), u = (int)(t - (int64_t)by * upr);
    const int x0 = 8 * u;
    const unsigned char* s = L.src + (int64_t)img * L.src_img;
    uint32_t cu, cv;  // 4 U and 4 V bytes
    if (L.layout <= 1) {
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 c = *reinterpret_cast<const u32x2*>(s + (int64_t)(L.h + by) * L.src_row + x0);
        // bytes u0 v0 u1 v1 | u2 v2 u3 v3 (NV12); V first for NV21
        const uint32_t ev = __builtin_amdgcn_perm(c[1], c[0], 0x06040200u);  // bytes 0 2 4 6
        const uint32_t od = __builtin_amdgcn_perm(c[1], c[0], 0x07050301u);  // bytes 1 3 5 7
        cu = L.layout == 0 ? ev : od;
        cv = L.layout == 0 ? od : ev;
    } else {
        const unsigned char* c0 = s + (int64_t)L.h * L.src_row;
        const int64_t q = (int64_t)(L.w >> 1) * bh, k = (int64_t)by * (L.w >> 1) + (x0 >> 1);
        const uint32_t p0 = *reinterpret_cast<const uint32_t*>(c0 + k);
        const uint32_t p1 = *reinterpret_cast<const uint32_t*>(c0 + q + k);
        cu = L.layout == 2 ? p1 : p0;
        cv = L.layout == 2 ? p0 : p1;
    }
    int ruv[4], guv[4], buv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int uu = (int)((cu >> (8 * i)) & 0xFFu) - 128, vv = (int)((cv >> (8 * i)) & 0xFFu) - 128;
        ruv[i] = (1 << 19) + 1673527 * vv;
        guv[i] = (1 << 19) - 852492 * vv - 409993 * uu;
        buv[i] = (1 << 19) + 2116026 * uu;
    }
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 yv = *reinterpret_cast<const u32x2*>(s + (int64_t)(2 * by + r) * L.src_row + x0);
        uint32_t px[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int Y = (int)((yv[j >> 2] >> (8 * (j & 3))) & 0xFFu);
            px[j] = bt601(Y, ruv[j >> 1], guv[j >> 1], buv[j >> 1], L.bidx);
        }
        unsigned char* o = L.dst + (int64_t)img * L.dst_img + (int64_t)(2 * by + r) * L.dst_row + (int64_t)x0 * DCN;
        if constexpr (DCN == 4) {
            reinterpret_cast<u32x4*>(o)[0] = u32x4{px[0], px[1], px[2], px[3]};
            reinterpret_cast<u32x4*>(o)[1] = u32x4{px[4], px[5], px[6], px[7]};
        } else {
            // 8 pixels' 24 bytes: drop each pixel's alpha byte
            uint32_t w[6];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint32_t a = px[4 * i], b = px[4 * i + 1], c = px[4 * i + 2], d = px[4 * i + 3];
                w[3 * i] = __builtin_amdgcn_perm(b, a, 0x04020100u);      // a0 a1 a2 b0
                w[3 * i + 1] = __builtin_amdgcn_perm(c, b, 0x05040201u);  // b1 b2 c0 c1
                w[3 * i + 2] = __builtin_amdgcn_perm(d, c, 0x06050402u);  // c2 d0 d1 d2
            }
            typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int k = 0; k < 3; ++k) reinterpret_cast<u32x2*>(o)[k] = u32x2{w[2 * k], w[2 * k + 1]};
        }
    }
}

// The same decode with each WAVE on 64 consecutive 8 x 2 units of ONE row
// pair (round 5): its output row segment (64 x 8 pixels x DCN bytes) is
// contiguous, so the lanes' pixels go through the wave's own LDS slice and
// leave as 16-byte stores, each instruction 1 KiB of one row.  The kernel
// above wrote each lane's 32 (BGRA) / 24 (BGR) bytes from the lane itself,
// its store instructions' lanes 32 / 24 bytes apart.  Needs 16-byte aligned
// destination rows (host-checked).
template <int DCN>
__global__ void __launch_bounds__(256) yuv420_cv8x_kernel(CvColorLaunch L, int upr, int wrow) {
    __shared__ __attribute__((aligned(16))) uint32_t xch[4][64 * 2 * DCN];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int img = blockIdx.y;
    const int bh = L.h >> 1;
    const int task = (int)blockIdx.x * 4 + wave;
    if (task >= wrow * bh) return;  // whole wave
    const int by = task / wrow, blk = task - by * wrow;
    const int nl = min(64, upr - blk * 64);  // live lanes (uniform)
    const int u = blk * 64 + min(lane, nl - 1);  // idle lanes decode the last live unit again
    const int x0 = 8 * u;
    const unsigned char* s = L.src + (int64_t)img * L.src_img;
    uint32_t cu, cv;
    if (L.layout <= 1) {
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 c = *reinterpret_cast<const u32x2*>(s + (int64_t)(L.h + by) * L.src_row + x0);
        const uint32_t ev = __builtin_amdgcn_perm(c[1], c[0], 0x06040200u);
        const uint32_t od = __builtin_amdgcn_perm(c[1], c[0], 0x07050301u);
        cu = L.layout == 0 ? ev : od;
        cv = L.layout == 0 ? od : ev;
    } else {
        const unsigned char* c0 = s + (int64_t)L.h * L.src_row;
        const int64_t q = (int64_t)(L.w >> 1) * bh, k = (int64_t)by * (L.w >> 1) + (x0 >> 1);
        const uint32_t p0 = *reinterpret_cast<const uint32_t*>(c0 + k);
        const uint32_t p1 = *reinterpret_cast<const uint32_t*>(c0 + q + k);
        cu = L.layout == 2 ? p1 : p0;
        cv = L.layout == 2 ? p0 : p1;
    }
    int ruv[4], guv[4], buv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int uu = (int)((cu >> (8 * i)) & 0xFFu) - 128, vv = (int)((cv >> (8 * i)) & 0xFFu) - 128;
        ruv[i] = (1 << 19) + 1673527 * vv;
        guv[i] = (1 << 19) - 852492 * vv - 409993 * uu;
        buv[i] = (1 << 19) + 2116026 * uu;
    }
    uint32_t* xw = xch[wave];
    const int nck = nl * 8 * DCN / 16;  // whole 16-byte chunks of the segment
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
        const u32x2 yv = *reinterpret_cast<const u32x2*>(s + (int64_t)(2 * by + r) * L.src_row + x0);
        uint32_t px[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int Y = (int)((yv[j >> 2] >> (8 * (j & 3))) & 0xFFu);
            px[j] = bt601(Y, ruv[j >> 1], guv[j >> 1], buv[j >> 1], L.bidx);
        }
        if constexpr (DCN == 4) {
            *reinterpret_cast<u32x4*>(xw + 8 * lane) = u32x4{px[0], px[1], px[2], px[3]};
            *reinterpret_cast<u32x4*>(xw + 8 * lane + 4) = u32x4{px[4], px[5], px[6], px[7]};
        } else {
            uint32_t w[6];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const uint32_t a = px[4 * i], b = px[4 * i + 1], c = px[4 * i + 2], d = px[4 * i + 3];
                w[3 * i] = __builtin_amdgcn_perm(b, a, 0x04020100u);
                w[3 * i + 1] = __builtin_amdgcn_perm(c, b, 0x05040201u);
                w[3 * i + 2] = __builtin_amdgcn_perm(d, c, 0x06050402u);
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) *reinterpret_cast<u32x2*>(xw + 6 * lane + 2 * k) = u32x2{w[2 * k], w[2 * k + 1]};
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        unsigned char* o = L.dst + (int64_t)img * L.dst_img + (int64_t)(2 * by + r) * L.dst_row + (int64_t)blk * 64 * 8 * DCN;
#pragma unroll
        for (int j = 0; j < (2 * DCN + 3) / 4; ++j) {  // 16-byte chunks per lane, rounded up: BGRA 2, BGR 2
            const int q = 64 * j + lane;
            if (q < nck) {
                const u32x4 v = *reinterpret_cast<const u32x4*>(xw + 4 * q);
                __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(o) + q);
            }
        }
        if (DCN == 3 && (nl & 1) && lane == 0)  // an odd lane count leaves 8 bytes
            *reinterpret_cast<u32x2*>(o + 16 * nck) = *reinterpret_cast<const u32x2*>(xw + 4 * nck);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();  // the next row reuses the slice
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

template <typename T>
constexpr int gray_px() { return sizeof(T) == 1 ? 16 : 4; }
template <int DCN, typename T>
__global__ void __launch_bounds__(256) gray_kernel(CvColorLaunch L, int upr) {
    constexpr int PX = gray_px<T>();
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int img = blockIdx.y;
    if (t >= (int64_t)upr * L.h) return;
    const int y = (int)(t / upr), u = (int)(t - (int64_t)y * upr);
    const int x0 = PX * u;
    const unsigned char* srow = L.src + (int64_t)img * L.src_img + (int64_t)y * L.src_row;
    unsigned char* drow = L.dst + (int64_t)img * L.dst_img + (int64_t)y * L.dst_row;
    constexpr T alpha = sizeof(T) == 1 ? (T)255 : (T)1;
    if (L.aligned && x0 + PX <= L.w) {
        if constexpr (sizeof(T) == 1) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(srow + x0);
            u32x4* o = reinterpret_cast<u32x4*>(drow + DCN * x0);
            if constexpr (DCN == 3) {
                // per source dword: bytes v0 v0 v0 v1 | v1 v1 v2 v2 | v2 v3 v3 v3
                uint32_t w[12];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    w[3 * i] = __builtin_amdgcn_perm(v[i], v[i], 0x01000000u);
                    w[3 * i + 1] = __builtin_amdgcn_perm(v[i], v[i], 0x02020101u);
                    w[3 * i + 2] = __builtin_amdgcn_perm(v[i], v[i], 0x03030302u);
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) o[k] = u32x4{w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]};
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t a = 0xFF000000u, d = v[i];
                    o[i] = u32x4{(d & 0xFFu) * 0x010101u | a, ((d >> 8) & 0xFFu) * 0x010101u | a,
                                 ((d >> 16) & 0xFFu) * 0x010101u | a, (d >> 24) * 0x010101u | a};
                }
            }
        } else {
            const float4 v = *reinterpret_cast<const float4*>(srow + 4 * x0);
            float4* o = reinterpret_cast<float4*>(drow + 4 * DCN * x0);
            if constexpr (DCN == 3) {
                o[0] = make_float4(v.x, v.x, v.x, v.y);
                o[1] = make_float4(v.y, v.y, v.z, v.z);
                o[2] = make_float4(v.z, v.w, v.w, v.w);
            } else {
                o[0] = make_float4(v.x, v.x, v.x, alpha);
                o[1] = make_float4(v.y, v.y, v.y, alpha);
                o[2] = make_float4(v.z, v.z, v.z, alpha);
                o[3] = make_float4(v.w, v.w, v.w, alpha);
            }
        }
        return;
    }
    for (int x = x0; x < min(x0 + PX, L.w); ++x) {
        const T v = *reinterpret_cast<const T*>(srow + (int64_t)x * sizeof(T));
        T* o = reinterpret_cast<T*>(drow) + (int64_t)x * DCN;
        o[0] = v;
        o[1] = v;
        o[2] = v;
        if (DCN == 4) o[3] = alpha;
    }
}

// GRAY2BGR(A) with each WAVE on 64 units of ONE row (round 5), for aligned
// images whose width is a whole number of units: the lanes' expanded pixels
// go through the wave's LDS slice and leave as 16-byte non-temporal stores,
// each instruction 1 KiB of the row (gray_kernel's lanes wrote their own
// 48 / 64 bytes, its store instructions' lanes that far apart).
template <int DCN, typename T>
__global__ void __launch_bounds__(256) gray_x_kernel(CvColorLaunch L, int upr, int wrow) {
    constexpr int PX = gray_px<T>();
    constexpr int OW = PX * DCN * (int)sizeof(T) / 4;  // output dwords per lane: 12 (BGR) or 16 (BGRA)
    __shared__ __attribute__((aligned(16))) uint32_t xch[4][64 * OW];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int img = blockIdx.y;
    const int task = (int)blockIdx.x * 4 + wave;
    if (task >= wrow * L.h) return;  // whole wave
    const int y = task / wrow, blk = task - y * wrow;
    const int nl = min(64, upr - blk * 64);  // live lanes (uniform)
    const int x0 = PX * (blk * 64 + min(lane, nl - 1));
    const unsigned char* srow = L.src + (int64_t)img * L.src_img + (int64_t)y * L.src_row;
    unsigned char* o = L.dst + (int64_t)img * L.dst_img + (int64_t)y * L.dst_row + (int64_t)blk * 64 * PX * DCN * sizeof(T);
    const u32x4 v = *reinterpret_cast<const u32x4*>(srow + (int64_t)x0 * sizeof(T));
    uint32_t w[OW];
    if constexpr (sizeof(T) == 1) {
        if constexpr (DCN == 3) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                w[3 * i] = __builtin_amdgcn_perm(v[i], v[i], 0x01000000u);
                w[3 * i + 1] = __builtin_amdgcn_perm(v[i], v[i], 0x02020101u);
                w[3 * i + 2] = __builtin_amdgcn_perm(v[i], v[i], 0x03030302u);
            }
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) w[i] = ((v[i >> 2] >> (8 * (i & 3))) & 0xFFu) * 0x010101u | 0xFF000000u;
        }
    } else {
        if constexpr (DCN == 3) {
            const uint32_t e[12] = {v[0], v[0], v[0], v[1], v[1], v[1], v[2], v[2], v[2], v[3], v[3], v[3]};
#pragma unroll
            for (int i = 0; i < 12; ++i) w[i] = e[i];
        } else {
            const uint32_t one = __float_as_uint(1.f);
#pragma unroll
            for (int i = 0; i < 4; ++i) { w[4 * i] = w[4 * i + 1] = w[4 * i + 2] = v[i]; w[4 * i + 3] = one; }
        }
    }
    uint32_t* xw = xch[wave];
#pragma unroll
    for (int k = 0; k < OW / 4; ++k)
        *reinterpret_cast<u32x4*>(xw + OW * lane + 4 * k) = u32x4{w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]};
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int nck = nl * OW / 4;  // 16-byte chunks of the wave's output run
#pragma unroll
    for (int j = 0; j < OW / 4; ++j) {
        const int q = 64 * j + lane;
        if (q < nck) __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(xw + 4 * q), reinterpret_cast<u32x4*>(o) + q);
    }
}

}  // namespace

hipError_t launch_color_cv(const CvColorLaunch& L, hipStream_t s) {
    const int upr = L.esize == 4 ? (L.w + 3) / 4 : (L.w + 15) / 16;  // gray: units per row (gray_px)
    const int64_t units = L.gray ? (int64_t)upr * L.h : (int64_t)(L.w / 2) * (L.h / 2);
    const int64_t grid = (units + 255) / 256;
    if (grid > 0x7FFFFFFF || L.n > 65535) return hipErrorInvalidValue;
    const dim3 g((unsigned)grid, (unsigned)L.n);
    if (L.gray) {
        CvColorLaunch G = L;
        // the vector path: every base and pitch 16-byte aligned
        const uintptr_t bits = reinterpret_cast<uintptr_t>(L.src) | reinterpret_cast<uintptr_t>(L.dst) |
                               (uintptr_t)L.src_img | (uintptr_t)L.src_row | (uintptr_t)L.dst_img | (uintptr_t)L.dst_row;
        G.aligned = (bits & 15) == 0;
        const int px = L.esize == 4 ? 4 : 16;
        if (G.aligned && L.w % px == 0 && tune(VACV_TUNE_RESIZE_DIRECT) != 2) {
            // a wave per 64 units of a row (VACV_TUNE_RESIZE_DIRECT = 2: gray_kernel, A/B)
            const int wrow = (upr + 63) / 64;
            const dim3 gg((unsigned)(((int64_t)wrow * L.h + 3) / 4), (unsigned)L.n);
            if (L.esize == 4) {
                if (L.dcn == 4) hipLaunchKernelGGL((gray_x_kernel<4, float>), gg, dim3(256), 0, s, G, upr, wrow);
                else hipLaunchKernelGGL((gray_x_kernel<3, float>), gg, dim3(256), 0, s, G, upr, wrow);
            } else {
                if (L.dcn == 4) hipLaunchKernelGGL((gray_x_kernel<4, unsigned char>), gg, dim3(256), 0, s, G, upr, wrow);
                else hipLaunchKernelGGL((gray_x_kernel<3, unsigned char>), gg, dim3(256), 0, s, G, upr, wrow);
            }
            return hipGetLastError();
        }
        if (L.esize == 4) {
            if (L.dcn == 4) hipLaunchKernelGGL((gray_kernel<4, float>), g, dim3(256), 0, s, G, upr);
            else hipLaunchKernelGGL((gray_kernel<3, float>), g, dim3(256), 0, s, G, upr);
        } else {
            if (L.dcn == 4) hipLaunchKernelGGL((gray_kernel<4, unsigned char>), g, dim3(256), 0, s, G, upr);
            else hipLaunchKernelGGL((gray_kernel<3, unsigned char>), g, dim3(256), 0, s, G, upr);
        }
    } else if ((L.w & 7) == 0 &&
               ((reinterpret_cast<uintptr_t>(L.src) | (uintptr_t)L.src_img | (uintptr_t)L.src_row) & 7) == 0 &&
               ((reinterpret_cast<uintptr_t>(L.dst) | (uintptr_t)L.dst_img | (uintptr_t)L.dst_row) & (L.dcn == 4 ? 15 : 7)) == 0) {
        // 8 x 2 pixels per thread (the planar chroma rows are w / 2 bytes: 4-byte aligned as w % 8 == 0)
        const int upr8 = L.w >> 3;
        const bool dst16 = ((reinterpret_cast<uintptr_t>(L.dst) | (uintptr_t)L.dst_img | (uintptr_t)L.dst_row) & 15) == 0;
        if (dst16 && tune(VACV_TUNE_RESIZE_DIRECT) != 2) {
            // a wave per 64 units of a row pair (VACV_TUNE_RESIZE_DIRECT = 2: the kernel below, A/B)
            const int wrow = (upr8 + 63) / 64;
            const int64_t gx = ((int64_t)wrow * (L.h >> 1) + 3) / 4;
            const dim3 gg((unsigned)gx, (unsigned)L.n);
            if (L.dcn == 4) hipLaunchKernelGGL(yuv420_cv8x_kernel<4>, gg, dim3(256), 0, s, L, upr8, wrow);
            else hipLaunchKernelGGL(yuv420_cv8x_kernel<3>, gg, dim3(256), 0, s, L, upr8, wrow);
            return hipGetLastError();
        }
        const int64_t g8 = ((int64_t)upr8 * (L.h >> 1) + 255) / 256;
        const dim3 gg((unsigned)g8, (unsigned)L.n);
        if (L.dcn == 4) hipLaunchKernelGGL(yuv420_cv8_kernel<4>, gg, dim3(256), 0, s, L, upr8);
        else hipLaunchKernelGGL(yuv420_cv8_kernel<3>, gg, dim3(256), 0, s, L, upr8);
    } else if (L.dcn == 4) {
        hipLaunchKernelGGL(yuv420_cv_kernel<4>, g, dim3(256), 0, s, L);
    } else {
        hipLaunchKernelGGL(yuv420_cv_kernel<3>, g, dim3(256), 0, s, L);
    }
    return hipGetLastError();
}

}  // namespace vacv
