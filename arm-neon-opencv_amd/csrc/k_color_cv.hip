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

template <int DCN, typename T>
__global__ void __launch_bounds__(256) gray_kernel(CvColorLaunch L) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int img = blockIdx.y;
    if (t >= (int64_t)L.w * L.h) return;
    const int y = (int)(t / L.w), x = (int)(t - (int64_t)y * L.w);
    const T v = *reinterpret_cast<const T*>(L.src + (int64_t)img * L.src_img + (int64_t)y * L.src_row +
                                            (int64_t)x * sizeof(T));
    T* o = reinterpret_cast<T*>(L.dst + (int64_t)img * L.dst_img + (int64_t)y * L.dst_row) + (int64_t)x * DCN;
    o[0] = v;
    o[1] = v;
    o[2] = v;
    if (DCN == 4) o[3] = sizeof(T) == 1 ? (T)255 : (T)1;
}

}  // namespace

hipError_t launch_color_cv(const CvColorLaunch& L, hipStream_t s) {
    const int64_t units = L.gray ? (int64_t)L.w * L.h : (int64_t)(L.w / 2) * (L.h / 2);
    const int64_t grid = (units + 255) / 256;
    if (grid > 0x7FFFFFFF || L.n > 65535) return hipErrorInvalidValue;
    const dim3 g((unsigned)grid, (unsigned)L.n);
    if (L.gray) {
        if (L.esize == 4) {
            if (L.dcn == 4) hipLaunchKernelGGL((gray_kernel<4, float>), g, dim3(256), 0, s, L);
            else hipLaunchKernelGGL((gray_kernel<3, float>), g, dim3(256), 0, s, L);
        } else {
            if (L.dcn == 4) hipLaunchKernelGGL((gray_kernel<4, unsigned char>), g, dim3(256), 0, s, L);
            else hipLaunchKernelGGL((gray_kernel<3, unsigned char>), g, dim3(256), 0, s, L);
        }
    } else if (L.dcn == 4) {
        hipLaunchKernelGGL(yuv420_cv_kernel<4>, g, dim3(256), 0, s, L);
    } else {
        hipLaunchKernelGGL(yuv420_cv_kernel<3>, g, dim3(256), 0, s, L);
    }
    return hipGetLastError();
}

}  // namespace vacv
