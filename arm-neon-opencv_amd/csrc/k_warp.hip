// k_warp.hip -- affine bilinear sampler with BORDER_CONSTANT, u8 / fp32,
// optional fused normalisation.
//
// Reference: WarpAffineNaive::warp_affine_naive_hwc_u8 / _fp32
// (warp_affine_naive.cpp:9-106) driven by WarpAffine::warp_affine_naive
// (warp_affine.cpp:111-169), which inverts M on the host side.  Per output
// pixel: f = float(m0*x + m1*y + m2) in float; floor; skip when the top-left
// tap is outside [0,w-2]x[0,h-2]; u8 weights SAT((1-f)*2048) and 2048-that;
// value (Sum S*wx*wy) >> 22.  Skipped pixels get the border value here.
//
// One thread = 4 consecutive output pixels of one row (vector stores); a
// 64x4-thread block covers a 256x4 output tile so the source footprint of a
// block is compact (L1/L2 reuse of the gathered taps).
#pragma clang fp contract(off)

#include "vacv_device.hpp"

namespace vacv {
namespace {

constexpr int kPx = 4;

template <int CC, typename TIn, int OUT>
__global__ void __launch_bounds__(kBlock)
warp_kernel(WarpLaunch L) {
    using TOut = typename std::conditional<(OUT == kOutSame), TIn, float>::type;
    constexpr bool kLut = std::is_same<TIn, uint8_t>::value && (OUT == kOutNorm);
    __shared__ float lut[kLut ? 256 * CC : 1];

    const int pidx = blockIdx.z;
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;
    const int y = blockIdx.y * 4 + threadIdx.y;
    const int x0 = (blockIdx.x * 64 + threadIdx.x) * kPx;

    float nmean[CC], nstd[CC];
    if (OUT == kOutNorm) {
#pragma unroll
        for (int k = 0; k < CC; ++k) norm_params(L.norm, img, CC == 1 ? plane : k, nmean[k], nstd[k]);
    }
    if (kLut) {
        const int tid = threadIdx.y * 64 + threadIdx.x;
        for (int i = tid; i < 256 * CC; i += kBlock) {
            const int k = i >> 8;
            lut[i] = normalize_value((float)(i & 255), nmean[k], nstd[k]);
        }
        __syncthreads();
    }
    if (y >= L.dst.h || x0 >= L.dst.w) return;

    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
    unsigned char* dp = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                        (int64_t)plane * L.dst.plane_pitch + (int64_t)y * L.dst.row_pitch +
                        (int64_t)x0 * CC * sizeof(TOut);
    const int64_t rp = L.src.row_pitch;
    const float fy_row = L.inv[1] * (float)y;
    const float gy_row = L.inv[4] * (float)y;

    TOut out[kPx * CC];
#pragma unroll
    for (int q = 0; q < kPx; ++q) {
        const int x = x0 + q;
        // warp_affine_naive.cpp:23-24: (m0*x + m1*y) + m2, all float
        const float fx = L.inv[0] * (float)x + fy_row + L.inv[2];
        const float fy = L.inv[3] * (float)x + gy_row + L.inv[5];
        int sx = 0, sy = 0;
        float ax = 0.f, ay = 0.f;
        const bool ok = affine_tap(fy, L.src.h, sy, ay) && affine_tap(fx, L.src.w, sx, ax);
        if (!ok) {
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                if (OUT == kOutNorm) {
                    out[q * CC + k] = kLut ? (TOut)lut[k * 256 + (int)L.border[k]]
                                           : (TOut)normalize_value(L.border[k], nmean[k], nstd[k]);
                } else {
                    out[q * CC + k] = (TOut)L.border[k];
                }
            }
            continue;
        }
        const unsigned char* r0 = sp + (int64_t)sy * rp + (int64_t)sx * CC * sizeof(TIn);
        const unsigned char* r1 = r0 + rp;
        if (std::is_same<TIn, uint8_t>::value) {
            const int wy0 = sat_short_away((1.f - ay) * 2048.f), wy1 = 2048 - wy0;
            const int wx0 = sat_short_away((1.f - ax) * 2048.f), wx1 = 2048 - wx0;
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                const int tl = r0[k], tr = r0[CC + k], bl = r1[k], br = r1[CC + k];
                // warp_affine_naive.cpp:50-54
                const int v = ((tl * wx0 * wy0 + bl * wx0 * wy1 + tr * wx1 * wy0 + br * wx1 * wy1) >> 22) & 0xFF;
                if (OUT == kOutSame) out[q * CC + k] = (TOut)v;
                else if (OUT == kOutF32) out[q * CC + k] = (TOut)(float)v;
                else out[q * CC + k] = (TOut)lut[k * 256 + v];
            }
        } else {
            const float y0 = 1.f - ay, y1 = ay, xa = 1.f - ax, xb = ax;
            const float* f0 = reinterpret_cast<const float*>(r0);
            const float* f1 = reinterpret_cast<const float*>(r1);
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                // warp_affine_naive.cpp:98-102, left to right
                float v = f0[k] * xa * y0;
                v += f1[k] * xa * y1;
                v += f0[CC + k] * xb * y0;
                v += f1[CC + k] * xb * y1;
                if (OUT == kOutNorm) v = normalize_value(v, nmean[k], nstd[k]);
                out[q * CC + k] = (TOut)v;
            }
        }
    }

    const int valid = min(kPx, L.dst.w - x0);
    constexpr int kBytes = kPx * CC * (int)sizeof(TOut);
    if (valid == kPx && (kBytes % 16 == 0) && ((reinterpret_cast<uintptr_t>(dp) & 15) == 0)) {
#pragma unroll
        for (int b = 0; b < kBytes / 16; ++b) reinterpret_cast<uint4*>(dp)[b] = reinterpret_cast<const uint4*>(out)[b];
    } else if (valid == kPx && (kBytes % 4 == 0) && ((reinterpret_cast<uintptr_t>(dp) & 3) == 0)) {
#pragma unroll
        for (int b = 0; b < kBytes / 4; ++b) reinterpret_cast<uint32_t*>(dp)[b] = reinterpret_cast<const uint32_t*>(out)[b];
    } else {
        TOut* o = reinterpret_cast<TOut*>(dp);
#pragma unroll
        for (int e = 0; e < kPx * CC; ++e)
            if (e < valid * CC) o[e] = out[e];
    }
}

template <int CC, typename TIn, int OUT>
hipError_t launch_one(const WarpLaunch& L, hipStream_t s) {
    dim3 block(64, 4);
    dim3 grid((L.dst.w + 64 * kPx - 1) / (64 * kPx), (L.dst.h + 3) / 4, L.n * L.src.planes);
    hipLaunchKernelGGL((warp_kernel<CC, TIn, OUT>), grid, block, 0, s, L);
    return hipGetLastError();
}

template <typename TIn, int OUT>
hipError_t launch_cc(const WarpLaunch& L, hipStream_t s) {
    switch (L.src.cc) {
        case 1: return launch_one<1, TIn, OUT>(L, s);
        case 2: return launch_one<2, TIn, OUT>(L, s);
        case 3: return launch_one<3, TIn, OUT>(L, s);
        case 4: return launch_one<4, TIn, OUT>(L, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

hipError_t launch_warp(const WarpLaunch& L, hipStream_t s) {
    if (L.src.esize == 1) {
        if (L.out == kOutSame) return launch_cc<uint8_t, kOutSame>(L, s);
        if (L.out == kOutF32) return launch_cc<uint8_t, kOutF32>(L, s);
        return launch_cc<uint8_t, kOutNorm>(L, s);
    }
    if (L.out == kOutNorm) return launch_cc<float, kOutNorm>(L, s);
    return launch_cc<float, kOutSame>(L, s);
}

}  // namespace vacv
