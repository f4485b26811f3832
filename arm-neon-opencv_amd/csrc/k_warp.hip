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
// A workgroup owns a 64*kPx x 4 output tile.  Each gather instruction
// samples one 64-pixel output row segment (16 x 4 lane blocks, a more compact
// rotated footprint, measured no faster in round 1).  kPx = 8 lane blocks per
// wave for byte output (10 when that pads the output width less, e.g. 1280;
// VACV_TUNE_WARP_PX overrides): more gathers in flight per wave, and the
// per-workgroup setup spread over twice the pixels (0.30 -> 0.28 -> 0.27 ms
// at 720p rot15); 4 for fp32 output.  The tile is re-assembled in LDS and each wave writes one of its
// rows with 16-byte stores.  Taps: one dword-aligned 8/12-byte buffer load per source row
// (load_taps, vacv_device.hpp), packed
// u16 dot products for the fixed-point sum.  Blocks are ordered so each XCD
// walks a contiguous range (its L2 keeps the shared source rows).
// These gather kernels serve fp32 sources, the non-CONSTANT border modes,
// and geometries whose source box is over the LDS plan of the u8 frames
// kernel (k_warp_frames.hip), which takes the rest: it stages the source in
// LDS and computes the taps once for 8 frames.
#pragma clang fp contract(off)

#include <cmath>
#include <map>
#include <mutex>

#include "vacv_device.hpp"

namespace vacv {
namespace {


// EXT: border modes other than CONSTANT (a separate instance: their slow path
// costs the CONSTANT kernel registers even when it never runs)
template <int CC, typename TIn, int OUT, int kPx, bool EXT>
__global__ void __launch_bounds__(kBlock)
warp_kernel(WarpLaunch L, int gx, int gy, int total) {
    constexpr int LW = 64, LH = 1;  // a lane block is one 64-pixel row segment; the tile is 4 rows
    using TOut = typename std::conditional<(OUT == kOutSame), TIn, float>::type;
    // u8 normalisation in registers (normalize_u8v); a per-workgroup LDS
    // table cost 3 fp64 divides per thread and a barrier (NV21 kernel: 0.58 ->
    // 0.71 of the roofline without it)
    constexpr bool kU8Norm = std::is_same<TIn, uint8_t>::value && (OUT == kOutNorm);
    constexpr int kRowBytes = 64 * kPx * CC * (int)sizeof(TOut);  // one wave's output row segment
    __shared__ __attribute__((aligned(16))) unsigned char xch[4][kRowBytes];

    // XCD-aware block order: workgroup b runs on XCD b % 8, and each XCD
    // walks one contiguous range of (plane, row band, column) blocks, so the
    // rotated source rows that neighbouring blocks share stay in one L2
    // (measured: scattered blocks fetched 3.7x the source bytes past L2)
    const int per_xcd = (total + 7) / 8;
    const int id = (int)(blockIdx.x % 8) * per_xcd + (int)(blockIdx.x / 8);
    if (id >= total) return;  // uniform
    const int pidx = id / (gx * gy);
    const int rem = id - pidx * gx * gy;
    const int by = rem / gx, bx = rem - by * gx;
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;
    const int lane = threadIdx.x;
    const int xw = bx * 64 * kPx;        // the tile's first column
    // wave (wx, wy) of the tile's LH x (4/LH) wave grid covers kPx lane blocks
    // side by side: columns [cx0, cx0 + kPx*LW), rows [ry0, ry0 + LH)
    const int cx0 = (int)(threadIdx.y % LH) * kPx * LW + lane % LW;
    const int ry = (int)(threadIdx.y / LH) * LH + lane / LW;  // tile row of this lane
    const int y = by * 4 + ry;

    float nmean[CC], nstd[CC];
    if (OUT == kOutNorm) {
#pragma unroll
        for (int k = 0; k < CC; ++k) norm_params(L.norm, img, CC == 1 ? plane : k, nmean[k], nstd[k]);
    }
    ChanNorm cn[CC] = {};
    if (kU8Norm) {
#pragma unroll
        for (int k = 0; k < CC; ++k) cn[k] = chan_norm(L.norm, img, CC == 1 ? plane : k);
    }

    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
    const int64_t rp = L.src.row_pitch;
    const float fy_row = L.inv[1] * (float)y;
    const float gy_row = L.inv[4] * (float)y;
    const Rsrc srs = make_rsrc(sp, L.src.plane_bytes);
    const uint32_t slimit = (uint32_t)L.src.plane_bytes + srs.delta;
    const uint32_t rp32 = (rp < (1 << 24) && L.src.h < (1 << 24)) ? (uint32_t)rp : 0u;  // 24-bit row offsets
    TOut* xrow = reinterpret_cast<TOut*>(xch[ry]);
    if (EXT && L.border_mode == kBorderTransparent && y < L.dst.h) {
        // pixels outside the source keep dst's bytes: start from them
        const int vb = min(64 * kPx, L.dst.w - xw) * CC * (int)sizeof(TOut);
        const unsigned char* drow = L.dst.base + (int64_t)img * L.dst.img_pitch + (int64_t)plane * L.dst.plane_pitch +
                                    (int64_t)y * L.dst.row_pitch + (int64_t)xw * CC * sizeof(TOut);
        for (int e = lane; e < vb; e += 64) xch[ry][e] = drow[e];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }

    // pass q samples the lane block at tile columns cx0 + q*LW (+ lane % LW).
    // With LW = 64 each gather instruction reads 64 CONSECUTIVE output
    // pixels, whose rotated source footprint spans ~20 cache lines instead of
    // 64 (adjacent pixels per lane would put every lane on its own row).
#pragma unroll
    for (int q = 0; q < kPx; ++q) {
        const int cx = cx0 + q * LW;
        const int x = xw + cx;
        if (x >= L.dst.w || y >= L.dst.h) continue;
        TOut* o = xrow + cx * CC;
        // warp_affine_naive.cpp:23-24: (m0*x + m1*y) + m2, all float
        const float fx = L.inv[0] * (float)x + fy_row + L.inv[2];
        const float fy = L.inv[3] * (float)x + gy_row + L.inv[5];
        int sx = 0, sy = 0;
        float ax = 0.f, ay = 0.f;
        const bool ok = affine_tap(fy, L.src.h, sy, ay) && affine_tap(fx, L.src.w, sx, ax);
        if (!ok) {
            if (EXT && L.border_mode == kBorderTransparent) continue;  // xrow holds dst's own bytes
            if (EXT && L.border_mode != kBorderConstant) {
                int vi[CC];
                float vf[CC];
                warp_border_sample<CC, TIn>(sp, rp, L.src.w, L.src.h, L.border_mode, fx, fy, vi, vf);
#pragma unroll
                for (int k = 0; k < CC; ++k) {
                    if (std::is_same<TIn, uint8_t>::value) {
                        if (OUT == kOutSame) o[k] = (TOut)vi[k];
                        else if (OUT == kOutF32) o[k] = (TOut)(float)vi[k];
                        else o[k] = (TOut)normalize_u8v(cn[k], vi[k]);
                    } else {
                        o[k] = (TOut)(OUT == kOutNorm ? normalize_value(vf[k], nmean[k], nstd[k]) : vf[k]);
                    }
                }
                continue;
            }
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                if (OUT == kOutNorm) {
                    o[k] = kU8Norm ? (TOut)normalize_u8v(cn[k], (int)L.border[k])
                                : (TOut)normalize_value(L.border[k], nmean[k], nstd[k]);
                } else {
                    o[k] = (TOut)L.border[k];
                }
            }
            continue;
        }
        const unsigned char* r0 = sp + (int64_t)sy * rp + (int64_t)sx * CC * sizeof(TIn);
        const unsigned char* r1 = r0 + rp;
        if (std::is_same<TIn, uint8_t>::value) {
            // SATURATE_CAST_SHORT of a value in (0, 2048]: the +0.5f branch, no clamp
            const int wy0 = (int)((1.f - ay) * 2048.f + 0.5f), wy1 = 2048 - wy0;
            const int wx0 = (int)((1.f - ax) * 2048.f + 0.5f), wx1 = 2048 - wx0;
            // the 2*CC tap bytes of each row in ONE dword-aligned buffer load;
            // a load past the plane's end (its last pixel) falls back to bytes
            uint32_t a0 = 0, a1 = 0, c0 = 0, c1 = 0;
            const uint32_t o0 = (rp32 ? __umul24((uint32_t)sy, rp32) : (uint32_t)((int64_t)sy * rp)) +
                                (uint32_t)(sx * CC) + srs.delta;
            const uint32_t o1 = o0 + (uint32_t)rp;
            if (CC <= 4 && (o1 & ~3u) + 4u * kTapDwords<CC, true> <= slimit) {
                load_taps<CC, true, 0>(srs, o0, a0, a1);
                load_taps<CC, true, 0>(srs, o1, c0, c1);
            } else {
#pragma unroll
                for (int e = 0; e < 2 * CC && e < 8; ++e) {
                    if (e < 4) { a0 |= (uint32_t)r0[e] << (8 * e); c0 |= (uint32_t)r1[e] << (8 * e); }
                    else { a1 |= (uint32_t)r0[e] << (8 * (e - 4)); c1 |= (uint32_t)r1[e] << (8 * (e - 4)); }
                }
            }
            // warp_affine_naive.cpp:50-54 as (tl*wx0 + tr*wx1)*wy0 + (bl*wx0 +
            // br*wx1)*wy1: the same int32 value (exact, no overflow: <= 255*2^22),
            // as one packed u16 dot product per row (v_dot2_u32_u16, tap pair
            // gathered by v_perm_b32) and two full-rate 24-bit multiplies
            typedef unsigned short us2 __attribute__((ext_vector_type(2)));
            const us2 wx = __builtin_bit_cast(us2, (uint32_t)wx0 | ((uint32_t)wx1 << 16));
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                uint32_t top, bot;
                if (CC <= 4) {
                    const uint32_t sel = (uint32_t)k | (0x0Cu << 8) | ((uint32_t)(CC + k) << 16) | (0x0Cu << 24);
                    top = __builtin_amdgcn_perm(a1, a0, sel);
                    bot = __builtin_amdgcn_perm(c1, c0, sel);
                } else {
                    top = (uint32_t)r0[k] | ((uint32_t)r0[CC + k] << 16);
                    bot = (uint32_t)r1[k] | ((uint32_t)r1[CC + k] << 16);
                }
                const uint32_t ht = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, top), wx, 0u, false);
                const uint32_t hb = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, bot), wx, 0u, false);
                const int v = (int)((__umul24(ht, (uint32_t)wy0) + __umul24(hb, (uint32_t)wy1)) >> 22);
                if (OUT == kOutSame) o[k] = (TOut)v;
                else if (OUT == kOutF32) o[k] = (TOut)(float)v;
                else o[k] = (TOut)normalize_u8v(cn[k], v);
            }
        } else {
            const float yy0 = 1.f - ay, yy1 = ay, xa = 1.f - ax, xb = ax;
            const float* f0 = reinterpret_cast<const float*>(r0);
            const float* f1 = reinterpret_cast<const float*>(r1);
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                // warp_affine_naive.cpp:98-102, left to right
                float v = f0[k] * xa * yy0;
                v += f1[k] * xa * yy1;
                v += f0[CC + k] * xb * yy0;
                v += f1[CC + k] * xb * yy1;
                if (OUT == kOutNorm) v = normalize_value(v, nmean[k], nstd[k]);
                o[k] = (TOut)v;
            }
        }
    }
    __syncthreads();

    // ---- wave r writes tile row r, LDS -> HBM in 16-byte chunks ----------------
    const int yo = by * 4 + (int)threadIdx.y;
    if (yo >= L.dst.h) return;
    const int vbytes = min(64 * kPx, L.dst.w - xw) * CC * (int)sizeof(TOut);
    unsigned char* drow = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                          (int64_t)plane * L.dst.plane_pitch + (int64_t)yo * L.dst.row_pitch +
                          (int64_t)xw * CC * sizeof(TOut);
    const unsigned char* xs = xch[threadIdx.y];
    if ((reinterpret_cast<uintptr_t>(drow) & 15) == 0) {  // uniform
        for (int c = lane; c * 16 < vbytes; c += 64) {
            if (c * 16 + 16 <= vbytes) {
                __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(xs + 16 * c),
                                            reinterpret_cast<u32x4*>(drow) + c);
            } else {
                for (int e = c * 16; e < vbytes; ++e) drow[e] = xs[e];
            }
        }
    } else {
        for (int e = lane; e < vbytes; e += 64) drow[e] = xs[e];
    }
}

// u8 input, BORDER_CONSTANT: the same sampler with its gathers batched.
// warp_kernel handles one pixel per step behind two branches (outside the
// source / past the plane end), so a wave has two 8/12-byte gathers in flight
// and waits on each pair before the next; here G pixels per lane compute
// their taps first (branch-free: a pixel outside the source loads the plane's
// first bytes and is replaced by the border value afterwards), issue all 2*G
// gathers, and only then blend -- 2*G gathers in flight per wave.
template <int CC, int OUT, int kPx, int G>
__global__ void __launch_bounds__(kBlock)
warp_u8_kernel(WarpLaunch L, int gx, int gy, int total) {
    static_assert(kPx % G == 0, "groups");
    using TOut = typename std::conditional<(OUT == kOutSame), uint8_t, float>::type;
    constexpr int kRowBytes = 64 * kPx * CC * (int)sizeof(TOut);  // one wave's output row segment
    constexpr uint32_t kTD = kTapDwords<CC, true>;                // dwords per tap row
    __shared__ __attribute__((aligned(16))) unsigned char xch[4][kRowBytes];

    const int per_xcd = (total + 7) / 8;  // XCD-aware block order (see warp_kernel)
    const int id = (int)(blockIdx.x % 8) * per_xcd + (int)(blockIdx.x / 8);
    if (id >= total) return;  // uniform
    const int pidx = id / (gx * gy);
    const int rem = id - pidx * gx * gy;
    const int by = rem / gx, bx = rem - by * gx;
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;
    const int lane = threadIdx.x;
    const int xw = bx * 64 * kPx;
    const int y = by * 4 + (int)threadIdx.y;
    const bool row_ok = y < L.dst.h;

    ChanNorm cn[CC] = {};
    if (OUT == kOutNorm) {
#pragma unroll
        for (int k = 0; k < CC; ++k) cn[k] = chan_norm(L.norm, img, CC == 1 ? plane : k);
    }
    TOut bval[CC];
#pragma unroll
    for (int k = 0; k < CC; ++k)
        bval[k] = OUT == kOutNorm ? (TOut)normalize_u8v(cn[k], (int)L.border[k]) : (TOut)L.border[k];

    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
    const int64_t rp = L.src.row_pitch;
    const float fy_row = L.inv[1] * (float)y;
    const float gy_row = L.inv[4] * (float)y;
    const Rsrc srs = make_rsrc(sp, L.src.plane_bytes);
    const uint32_t slimit = (uint32_t)L.src.plane_bytes + srs.delta;
    const uint32_t rp32 = (uint32_t)rp;  // plane_bytes < 2^31 (kMaxPlaneBytes)
    TOut* xrow = reinterpret_cast<TOut*>(xch[threadIdx.y]);
    typedef unsigned short us2v __attribute__((ext_vector_type(2)));

#pragma unroll
    for (int g = 0; g < kPx; g += G) {
        uint32_t tp[G][2][kTD];
        uint32_t wxp[G], wy0[G], sh[G], sh1[G];
        bool val[G], far[G];
        // ---- taps and gathers of G pixels (no branches) ----------------------
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int x = xw + (g + j) * 64 + lane;
            // warp_affine_naive.cpp:23-24: (m0*x + m1*y) + m2, all float
            const float fx = L.inv[0] * (float)x + fy_row + L.inv[2];
            const float fy = L.inv[3] * (float)x + gy_row + L.inv[5];
            int sx = 0, sy = 0;
            float ax = 0.f, ay = 0.f;
            const bool ok = row_ok && x < L.dst.w && affine_tap(fy, L.src.h, sy, ay) && affine_tap(fx, L.src.w, sx, ax);
            // SATURATE_CAST_SHORT of a value in (0, 2048]: the +0.5f branch, no clamp
            const uint32_t w0 = (uint32_t)(int)((1.f - ay) * 2048.f + 0.5f);
            const uint32_t x0 = (uint32_t)(int)((1.f - ax) * 2048.f + 0.5f);
            wy0[j] = w0;
            wxp[j] = x0 | ((2048u - x0) << 16);
            const uint32_t o0 = ok ? __umul24((uint32_t)sy, rp32) + (uint32_t)(sx * CC) + srs.delta : srs.delta;
            const uint32_t o1 = ok ? o0 + rp32 : srs.delta;
            const bool inr = (o1 & ~3u) + 4u * kTD <= slimit;
            val[j] = ok;
            far[j] = ok && !inr;  // the plane's last pixel: bytes, below
            sh[j] = o0 & 3u;
            sh1[j] = o1 & 3u;  // differs from sh when the row pitch is not a multiple of 4
            const int a0 = (int)((inr ? o0 : srs.delta) & ~3u), a1 = (int)((inr ? o1 : srs.delta) & ~3u);
            if constexpr (kTD == 2) {
                const auto v0 = __builtin_amdgcn_raw_buffer_load_b64(srs.r, a0, 0, 0);
                const auto v1 = __builtin_amdgcn_raw_buffer_load_b64(srs.r, a1, 0, 0);
                tp[j][0][0] = v0[0]; tp[j][0][1] = v0[1];
                tp[j][1][0] = v1[0]; tp[j][1][1] = v1[1];
            } else {
                const auto v0 = __builtin_amdgcn_raw_buffer_load_b96(srs.r, a0, 0, 0);
                const auto v1 = __builtin_amdgcn_raw_buffer_load_b96(srs.r, a1, 0, 0);
#pragma unroll
                for (uint32_t d = 0; d < kTD; ++d) { tp[j][0][d] = v0[d]; tp[j][1][d] = v1[d]; }
            }
            if (far[j]) {  // rare: re-read the tap bytes singly (the 12-byte load would overhang)
                const unsigned char* r0 = sp + (int64_t)sy * rp + (int64_t)sx * CC;
                uint32_t b[2][3] = {{0u, 0u, 0u}, {0u, 0u, 0u}};
#pragma unroll
                for (int e = 0; e < 2 * CC; ++e) {
                    b[0][e >> 2] |= (uint32_t)r0[e] << (8 * (e & 3));
                    b[1][e >> 2] |= (uint32_t)r0[rp + e] << (8 * (e & 3));
                }
#pragma unroll
                for (uint32_t d = 0; d < kTD; ++d) { tp[j][0][d] = b[0][d]; tp[j][1][d] = b[1][d]; }
                sh[j] = sh1[j] = 0u;
            }
        }
        // ---- blends --------------------------------------------------------
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int cxl = (g + j) * 64 + lane;
            TOut* o = xrow + cxl * CC;
            const uint32_t a0 = __builtin_amdgcn_alignbyte(tp[j][0][1], tp[j][0][0], sh[j]);
            const uint32_t c0 = __builtin_amdgcn_alignbyte(tp[j][1][1], tp[j][1][0], sh1[j]);
            uint32_t a1 = 0u, c1 = 0u;
            if constexpr (kTD == 3) {
                a1 = __builtin_amdgcn_alignbyte(tp[j][0][2], tp[j][0][1], sh[j]);
                c1 = __builtin_amdgcn_alignbyte(tp[j][1][2], tp[j][1][1], sh1[j]);
            }
            const us2v wx = __builtin_bit_cast(us2v, wxp[j]);
            const uint32_t wA = wy0[j], wB = 2048u - wy0[j];
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                // warp_affine_naive.cpp:50-54 as (tl*wx0 + tr*wx1)*wy0 +
                // (bl*wx0 + br*wx1)*wy1 (exact int32, <= 255*2^22)
                const uint32_t sel = (uint32_t)k | (0x0Cu << 8) | ((uint32_t)(CC + k) << 16) | (0x0Cu << 24);
                const uint32_t top = __builtin_amdgcn_perm(a1, a0, sel);
                const uint32_t bot = __builtin_amdgcn_perm(c1, c0, sel);
                const uint32_t ht = __builtin_amdgcn_udot2(__builtin_bit_cast(us2v, top), wx, 0u, false);
                const uint32_t hb = __builtin_amdgcn_udot2(__builtin_bit_cast(us2v, bot), wx, 0u, false);
                const int v = (int)((__umul24(ht, wA) + __umul24(hb, wB)) >> 22);
                TOut ov;
                if (OUT == kOutSame) ov = (TOut)v;
                else if (OUT == kOutF32) ov = (TOut)(float)v;
                else ov = (TOut)normalize_u8v(cn[k], v);
                o[k] = val[j] ? ov : bval[k];
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- the wave's row, LDS -> HBM in 16-byte chunks ---------------------
    if (!row_ok) return;
    const int vbytes = min(64 * kPx, L.dst.w - xw) * CC * (int)sizeof(TOut);
    unsigned char* drow = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                          (int64_t)plane * L.dst.plane_pitch + (int64_t)y * L.dst.row_pitch +
                          (int64_t)xw * CC * sizeof(TOut);
    const unsigned char* xs = xch[threadIdx.y];
    if ((reinterpret_cast<uintptr_t>(drow) & 15) == 0) {  // uniform
        for (int c = lane; c * 16 < vbytes; c += 64) {
            if (c * 16 + 16 <= vbytes) {
                __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(xs + 16 * c),
                                            reinterpret_cast<u32x4*>(drow) + c);
            } else {
                for (int e = c * 16; e < vbytes; ++e) drow[e] = xs[e];
            }
        }
    } else {
        for (int e = lane; e < vbytes; e += 64) drow[e] = xs[e];
    }
}

// default: 8 or 10 lane blocks per wave for byte output, whichever pads the
// output width less (1280: 10 -> 2 tiles of 640 exactly, 0.271 ms, vs 8 ->
// 2.5 tiles, 0.281 ms at 720p rot15; 8 vs 4: 0.283 vs 0.304), 4 for fp32
// output (0.538 vs 0.614 ms: 8 blocks double the LDS row buffers and halve
// the resident workgroups).  VACV_TUNE_WARP_PX = 4, 5, 8 or 10 overrides.
int warp_blocks_per_wave(bool byte_out, int w) {
    const int px = tune(VACV_TUNE_WARP_PX);
    if (px == 4 || px == 5 || px == 8 || px == 10) return px;
    if (!byte_out) return 4;
    const auto pad = [w](int k) { return (w + 64 * k - 1) / (64 * k) * (64 * k) - w; };
    return pad(10) < pad(8) ? 10 : 8;
}

// warp_u8_kernel (2*G gathers in flight per wave) or warp_kernel (2)?  Batching
// pays while a 64-pixel output row segment stays within a few source rows
// (720p, scale 0.9: rotation 0 deg 0.256 -> 0.227 ms, 5 deg 0.268 -> 0.231)
// and loses once its gathers spread over many (15 deg, 18 rows: 0.272 ->
// 0.289; 45 deg: 0.369 -> 0.413): more lines in flight than the CU's vector
// cache holds.  VACV_TUNE_WARP_KERNEL: 0 warp_kernel, 2 warp_u8_kernel.
int warp_batched(const WarpLaunch& L) {
    const int knob = tune(VACV_TUNE_WARP_KERNEL);
    if (knob == 0 || knob == 2) return knob;
    return 64.f * std::fabs(L.inv[3]) <= 10.f ? 2 : 0;
}

template <int CC, typename TIn, int OUT, int kPx>
hipError_t launch_px(const WarpLaunch& L, hipStream_t s) {
    const int gx = (L.dst.w + 64 * kPx - 1) / (64 * kPx), gy = (L.dst.h + 3) / 4;
    const int64_t total = (int64_t)gx * gy * L.n * L.src.planes;
    if (total >= 0x7FFFFFF0LL) return hipErrorInvalidValue;
    const int64_t blocks = (total + 7) / 8 * 8;
    constexpr int G = kPx % 5 == 0 ? 5 : 4;
    if (L.border_mode == kBorderConstant && std::is_same<TIn, uint8_t>::value && warp_batched(L) == 2)
        hipLaunchKernelGGL((warp_u8_kernel<CC, OUT, kPx, G>), dim3((unsigned)blocks), dim3(64, 4), 0, s, L, gx, gy,
                           (int)total);
    else if (L.border_mode == kBorderConstant)
        hipLaunchKernelGGL((warp_kernel<CC, TIn, OUT, kPx, false>), dim3((unsigned)blocks), dim3(64, 4), 0, s, L, gx,
                           gy, (int)total);
    else
        hipLaunchKernelGGL((warp_kernel<CC, TIn, OUT, kPx, true>), dim3((unsigned)blocks), dim3(64, 4), 0, s, L, gx,
                           gy, (int)total);
    return hipGetLastError();
}

template <int CC, typename TIn, int OUT>
hipError_t launch_one(const WarpLaunch& L, hipStream_t s) {
    if constexpr (std::is_same<TIn, uint8_t>::value) {
        // u8 CONSTANT: the LDS-staged frames kernel (k_warp_frames.hip),
        // unless its box plan does not fit
        WarpFramesPlan P;
        if (warp_frames_plan(L, P)) return launch_warp_frames(L, P, s);
    }
    switch (warp_blocks_per_wave(OUT == kOutSame && sizeof(TIn) == 1, L.dst.w)) {
        case 10: return launch_px<CC, TIn, OUT, 10>(L, s);
        case 5: return launch_px<CC, TIn, OUT, 5>(L, s);
        case 8: return launch_px<CC, TIn, OUT, 8>(L, s);
        default: return launch_px<CC, TIn, OUT, 4>(L, s);
    }
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

namespace {

// ---------------------------------------------------------------------------
// INTER_NEAREST: OpenCV 2.4.13's warpAffine (imgwarp.cpp) -- the map in fp64
// fixed point with AB_BITS = 10:
//   X0 = cvRound((M1 y + M2) 1024) + 512,  adelta = cvRound(M0 x 1024)
//   X  = (X0 + adelta) >> 10            (the same for Y with M3, M4, M5)
// then remap's nearest sampler: inside -> the source pixel; outside -> the
// border value (CONSTANT), dst untouched (TRANSPARENT), or the pixel at
// borderInterpolate(X), borderInterpolate(Y).  Parity unpinned (no OpenCV
// runs here; oracle_warp_affine_nn restates the same).  One thread per
// output pixel of one plane: a rarely used mode, gather-bound.
template <int CC, typename TIn, int OUT>
__global__ void __launch_bounds__(kBlock) warp_nearest_kernel(WarpLaunch L) {
    using TOut = typename std::conditional<(OUT == kOutSame), TIn, float>::type;
    const int x = blockIdx.x * kBlock + threadIdx.x, y = blockIdx.y, pidx = blockIdx.z;
    if (x >= L.dst.w) return;
    const int img = pidx / L.src.planes, pl = pidx - img * L.src.planes;
    const double* M = L.invd;
    const int X0 = (int)rint((M[1] * y + M[2]) * 1024.0) + 512;
    const int Y0 = (int)rint((M[4] * y + M[5]) * 1024.0) + 512;
    int X = (int)((uint32_t)X0 + (uint32_t)(int)rint(M[0] * x * 1024.0)) >> 10;
    int Y = (int)((uint32_t)Y0 + (uint32_t)(int)rint(M[3] * x * 1024.0)) >> 10;
    X = min(max(X, -32768), 32767);  // remap's short map (saturate_cast<short>)
    Y = min(max(Y, -32768), 32767);
    const bool inside = (unsigned)X < (unsigned)L.src.w && (unsigned)Y < (unsigned)L.src.h;
    if (!inside && L.border_mode == kBorderTransparent) return;
    TOut* d = reinterpret_cast<TOut*>(const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                                      (int64_t)pl * L.dst.plane_pitch + (int64_t)y * L.dst.row_pitch) + (int64_t)x * CC;
    const TIn* sp = nullptr;
    if (inside || L.border_mode != kBorderConstant) {
        const int sx = inside ? X : border_index(X, L.src.w, L.border_mode);
        const int sy = inside ? Y : border_index(Y, L.src.h, L.border_mode);
        sp = reinterpret_cast<const TIn*>(L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)pl * L.src.plane_pitch +
                                          (int64_t)sy * L.src.row_pitch) + (int64_t)sx * CC;
    }
#pragma unroll
    for (int k = 0; k < CC; ++k) {
        const int ch = L.src.planes > 1 ? pl : k;
        const TIn v = sp ? sp[k] : (TIn)L.border[ch];
        if constexpr (OUT == kOutSame) {
            d[k] = v;
        } else if constexpr (OUT == kOutF32) {
            d[k] = (float)v;
        } else {
            const ChanNorm cn = chan_norm(L.norm, img, ch);
            if constexpr (std::is_same<TIn, uint8_t>::value) d[k] = normalize_u8v(cn, (int)v);
            else d[k] = normalize_f(cn, (float)v);
        }
    }
}

// u8 -> u8 nearest (all border modes but TRANSPARENT, 4-byte aligned
// destination): one pixel per lane as above (consecutive lanes gather
// neighbouring source pixels, so a load instruction touches few lines), but
// the pixel's CC bytes by ONE unaligned dword gather (bytewise only where that
// dword would reach past the plane), and each lane quad's 4 CC output bytes
// packed across the quad (quad_pack, DPP) into CC dword stores instead of
// CC byte stores per lane.
template <int CC>
__global__ void __launch_bounds__(kBlock) warp_nearest4_kernel(WarpLaunch L) {
    const int x = blockIdx.x * kBlock + threadIdx.x, y = blockIdx.y, pidx = blockIdx.z;
    const int xq = x & ~3;
    if (xq >= L.dst.w) return;  // whole quads leave together (the DPP reads quad neighbours)
    const int lane = (int)threadIdx.x & 63;
    const int img = pidx / L.src.planes, pl = pidx - img * L.src.planes;
    const double* M = L.invd;
    const int xc = min(x, L.dst.w - 1);
    const int X0 = (int)rint((M[1] * y + M[2]) * 1024.0) + 512;
    const int Y0 = (int)rint((M[4] * y + M[5]) * 1024.0) + 512;
    int X = (int)((uint32_t)X0 + (uint32_t)(int)rint(M[0] * xc * 1024.0)) >> 10;
    int Y = (int)((uint32_t)Y0 + (uint32_t)(int)rint(M[3] * xc * 1024.0)) >> 10;
    X = min(max(X, -32768), 32767);  // remap's short map (saturate_cast<short>)
    Y = min(max(Y, -32768), 32767);
    const bool inside = (unsigned)X < (unsigned)L.src.w && (unsigned)Y < (unsigned)L.src.h;
    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)pl * L.src.plane_pitch;
    const Rsrc srs = make_rsrc(sp, L.src.plane_bytes);
    const uint32_t lim = (uint32_t)L.src.plane_bytes + srs.delta;
    uint32_t own = 0;
#pragma unroll
    for (int k = 0; k < CC; ++k) own |= (uint32_t)(int)L.border[L.src.planes > 1 ? pl : k] << (8 * k);
    if (inside || L.border_mode != kBorderConstant) {
        const int sx = inside ? X : border_index(X, L.src.w, L.border_mode);
        const int sy = inside ? Y : border_index(Y, L.src.h, L.border_mode);
        const uint32_t o = (uint32_t)sy * (uint32_t)L.src.row_pitch + (uint32_t)(sx * CC) + srs.delta;
        if (o + 4u <= lim) {
            own = __builtin_amdgcn_raw_buffer_load_b32(srs.r, (int)o, 0, 0);
        } else {  // the plane's last pixel: bytewise (an overhanging load reads zeros)
            uint32_t v = 0;
#pragma unroll
            for (int k = 0; k < CC; ++k)
                v |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(srs.r, (int)(o + k), 0, 0) << (8 * k);
            own = v;
        }
    }
    if constexpr (CC < 4) own &= (1u << (8 * CC)) - 1u;  // the gathered dword's other bytes (quad_pack ORs bytes)
    const uint32_t word = quad_pack<CC>(own, lane & 3);
    unsigned char* d = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                       (int64_t)pl * L.dst.plane_pitch + (int64_t)y * L.dst.row_pitch;
    if (xq + 4 <= L.dst.w) {
        if ((lane & 3) < CC) *reinterpret_cast<uint32_t*>(d + xq * CC + 4 * (lane & 3)) = word;
    } else if (x < L.dst.w) {  // the row's last partial quad: bytes
#pragma unroll
        for (int k = 0; k < CC; ++k) d[x * CC + k] = (unsigned char)(own >> (8 * k));
    }
}

template <typename TIn, int OUT>
hipError_t launch_nearest_t(const WarpLaunch& L, hipStream_t s) {
    const dim3 grid((unsigned)((L.dst.w + kBlock - 1) / kBlock), (unsigned)L.dst.h, (unsigned)(L.n * L.src.planes));
    if ((int64_t)L.n * L.src.planes > 65535 || L.dst.h > 65535) return hipErrorInvalidValue;
    switch (L.src.cc) {
        case 1: hipLaunchKernelGGL((warp_nearest_kernel<1, TIn, OUT>), grid, dim3(kBlock), 0, s, L); break;
        case 2: hipLaunchKernelGGL((warp_nearest_kernel<2, TIn, OUT>), grid, dim3(kBlock), 0, s, L); break;
        case 3: hipLaunchKernelGGL((warp_nearest_kernel<3, TIn, OUT>), grid, dim3(kBlock), 0, s, L); break;
        case 4: hipLaunchKernelGGL((warp_nearest_kernel<4, TIn, OUT>), grid, dim3(kBlock), 0, s, L); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace

hipError_t launch_warp_nearest(const WarpLaunch& L, hipStream_t s) {
    {
        // 3-channel u8 CONSTANT: the LDS-staged kernel (k_warp_frames.hip)
        WarpFramesPlan P;
        if (warp_exp_nn_plan(L, P)) return launch_warp_exp_nn(L, P, s);
    }
    const bool al4 = ((reinterpret_cast<uintptr_t>(L.dst.base) | (uintptr_t)L.dst.row_pitch | (uintptr_t)L.dst.img_pitch |
                       (uintptr_t)L.dst.plane_pitch) & 3) == 0;
    if (L.src.esize == 1 && L.out == kOutSame && L.border_mode != kBorderTransparent && al4 &&
        L.src.plane_bytes <= kMaxPlaneBytes && tune(VACV_TUNE_WARP_KERNEL) != 5) {
        const dim3 grid((unsigned)((L.dst.w + kBlock - 1) / kBlock), (unsigned)L.dst.h, (unsigned)(L.n * L.src.planes));
        if ((int64_t)L.n * L.src.planes > 65535 || L.dst.h > 65535) return hipErrorInvalidValue;
        switch (L.src.cc) {
            case 1: hipLaunchKernelGGL((warp_nearest4_kernel<1>), grid, dim3(kBlock), 0, s, L); break;
            case 2: hipLaunchKernelGGL((warp_nearest4_kernel<2>), grid, dim3(kBlock), 0, s, L); break;
            case 3: hipLaunchKernelGGL((warp_nearest4_kernel<3>), grid, dim3(kBlock), 0, s, L); break;
            case 4: hipLaunchKernelGGL((warp_nearest4_kernel<4>), grid, dim3(kBlock), 0, s, L); break;
            default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    if (L.src.esize == 1) {
        if (L.out == kOutSame) return launch_nearest_t<uint8_t, kOutSame>(L, s);
        if (L.out == kOutF32) return launch_nearest_t<uint8_t, kOutF32>(L, s);
        return launch_nearest_t<uint8_t, kOutNorm>(L, s);
    }
    if (L.out == kOutNorm) return launch_nearest_t<float, kOutNorm>(L, s);
    return launch_nearest_t<float, kOutSame>(L, s);
}

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
