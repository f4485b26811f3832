// k_warp_tile.hip -- affine bilinear warp of u8 images (BORDER_CONSTANT) with
// the source footprint of each output tile staged in LDS.
//
// Reference: WarpAffineNaive::warp_affine_naive_hwc_u8 (warp_affine_naive.cpp:
// 9-58) driven by WarpAffine::warp_affine_naive (warp_affine.cpp:111-169):
// per output pixel f = float(m0*x + m1*y + m2) in float, floor, skip when the
// top-left tap is outside [0,w-2]x[0,h-2], weights SAT((1-f)*2048) and
// 2048-that, value (Sum S*wx*wy) >> 22.  Skipped pixels get the border value
// here (the reference leaves them untouched).  The per-pixel
// arithmetic is warp_kernel's (k_warp.hip), bit for bit.
//
// Why staging: warp_kernel gathers each tap row with one 8-byte load per lane,
// and PMC shows the texture data path at ~1 lane per clock per CU (TD_TD_BUSY
// ~95 % of the kernel, TA ~85 %): the kernel is bound by per-lane gathers, not
// HBM.  Here a workgroup owns a 64 x 16 output tile, loads the tile's source
// bounding box (a parallelogram's box, a few KB) with coalesced 16-byte
// loads -- ~0.4 lane-loads per output pixel instead of 2 --
// and reads the taps from LDS (two aligned 8-byte LDS reads per tap row,
// v_alignbyte to the tap's byte offset).  Pixels whose taps fall outside the
// box (only possible through rounding at the box edge, or non-finite
// matrices) take warp_kernel's global gather, so correctness never depends on
// the box computation.  Outputs leave through a per-wave LDS exchange as
// 16-byte non-temporal stores.
#pragma clang fp contract(off)

#include <cmath>
#include <cstdlib>

#include "vacv_device.hpp"

namespace vacv {
namespace {

constexpr int kTW = 64;   // tile width (one pixel per lane)
constexpr int kTH = 16;   // tile height (4 rows per wave)
constexpr int kBoxBudget = 24 * 1024;  // LDS bytes for the staged box

// Box geometry every tile of this launch fits (host and device agree):
// width/height in pixels and the LDS row stride in bytes.
struct BoxCap {
    int w, h, stride;
};

__host__ __device__ inline BoxCap box_cap(const float inv[6], int cc) {
    // the tile's source footprint spans |m0|*(TW-1) + |m1|*(TH-1) in x (and
    // the same with m3, m4 in y); +6 covers the floor, the second tap, the
    // one-pixel margins and rounding
    const float ex = fabsf(inv[0]) * (kTW - 1) + fabsf(inv[1]) * (kTH - 1);
    const float ey = fabsf(inv[3]) * (kTW - 1) + fabsf(inv[4]) * (kTH - 1);
    BoxCap b{0, 0, 0};
    if (!(ex < 4096.f && ey < 4096.f)) return b;  // also NaN
    b.w = (int)ex + 6;
    b.h = (int)ey + 6;
    int stride = ((b.w * cc + 15 + 16) + 15) & ~15;  // head (<16) + chunk overhang
    if ((stride & 255) == 0) stride += 16;           // rows on different LDS banks
    b.stride = stride;
    return b;
}

// 8 bytes at LDS byte address a (two aligned 8-byte reads + byte align)
__device__ __forceinline__ void lds_tap8(const unsigned char* lds, uint32_t a, uint32_t& lo, uint32_t& hi) {
    const uint32_t a8 = a & ~7u;
    const uint2 p = *reinterpret_cast<const uint2*>(lds + a8);
    const uint2 q = *reinterpret_cast<const uint2*>(lds + a8 + 8);
    const uint32_t s = a & 7u;
    if (s < 4) {
        lo = __builtin_amdgcn_alignbyte(p.y, p.x, s);
        hi = __builtin_amdgcn_alignbyte(q.x, p.y, s);
    } else {
        lo = __builtin_amdgcn_alignbyte(q.x, p.y, s - 4);
        hi = __builtin_amdgcn_alignbyte(q.y, q.x, s - 4);
    }
}

template <int CC, int OUT>
__global__ void __launch_bounds__(kBlock)
warp_tile_kernel(WarpLaunch L, BoxCap cap, int tiles_x, int tiles_y, int total) {
    using TOut = typename std::conditional<(OUT == kOutSame), uint8_t, float>::type;
    constexpr bool kLut = OUT == kOutNorm;
    constexpr int kRowOut = kTW * CC * (int)sizeof(TOut);  // bytes of one tile row
    __shared__ float lut[kLut ? 256 * CC : 1];
    __shared__ __attribute__((aligned(16))) unsigned char xch[4][4 * kRowOut];
    extern __shared__ __attribute__((aligned(16))) unsigned char box[];

    // XCD-contiguous tile order (block b runs on XCD b % 8): neighbouring
    // tiles share box rows, so they should share an L2
    const int per_xcd = (total + 7) / 8;
    const int id = (int)(blockIdx.x % 8) * per_xcd + (int)(blockIdx.x / 8);
    if (id >= total) return;  // uniform, before any barrier
    const int pidx = id / (tiles_x * tiles_y);
    const int rem = id - pidx * tiles_x * tiles_y;
    const int ty = rem / tiles_x, tx = rem - ty * tiles_x;
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;
    const int tid = (int)(threadIdx.y * 64 + threadIdx.x);
    const int lane = threadIdx.x, wave = threadIdx.y;
    const int X0 = tx * kTW, Y0 = ty * kTH;

    if (kLut) {
        for (int i = tid; i < 256 * CC; i += kBlock) {
            const int k = i >> 8;
            float m, sd;
            norm_params(L.norm, img, CC == 1 ? plane % L.norm.c_total : k, m, sd);
            lut[i] = normalize_value((float)(i & 255), m, sd);
        }
    }

    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
    const Rsrc srs = make_rsrc(sp, L.src.plane_bytes);
    const uint32_t slimit = (uint32_t)L.src.plane_bytes + srs.delta;
    const uint32_t rp32 = (uint32_t)L.src.row_pitch;  // plane < 2^31 bytes
    const int Ws = L.src.w, Hs = L.src.h;

    // ---- the tile's source box (uniform) from its corner coordinates --------
    float fx_min = INFINITY, fx_max = -INFINITY, fy_min = INFINITY, fy_max = -INFINITY;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float x = (float)(X0 + ((c & 1) ? kTW - 1 : 0));
        const float y = (float)(Y0 + ((c & 2) ? kTH - 1 : 0));
        const float fx = L.inv[0] * x + L.inv[1] * y + L.inv[2];
        const float fy = L.inv[3] * x + L.inv[4] * y + L.inv[5];
        fx_min = fminf(fx_min, fx); fx_max = fmaxf(fx_max, fx);
        fy_min = fminf(fy_min, fy); fy_max = fmaxf(fy_max, fy);
    }
    int bx0 = 0, bx1 = -1, by0 = 0, by1 = -1;
    if (fx_min > -1e8f && fx_max < 1e8f && fy_min > -1e8f && fy_max < 1e8f) {
        bx0 = max(0, (int)floorf(fx_min) - 1);
        bx1 = min(Ws - 1, (int)floorf(fx_max) + 2);
        by0 = max(0, (int)floorf(fy_min) - 1);
        by1 = min(Hs - 1, (int)floorf(fy_max) + 2);
    }
    if (bx1 - bx0 + 1 > cap.w || by1 - by0 + 1 > cap.h) { bx1 = bx0 - 1; by1 = by0 - 1; }  // nothing staged
    const int nrows = max(0, by1 - by0 + 1);
    const int ncols = max(0, bx1 - bx0 + 1);

    // ---- stage it: 16-byte chunks, row heads aligned down --------------------
    const int cpr = ncols > 0 ? (ncols * CC + 15 + 15) / 16 : 0;  // chunks per row (head < 16)
    auto chunk = [&](int i) {
        const int r = i / cpr, c = i - r * cpr;
        const uint32_t a = (((uint32_t)(by0 + r) * rp32 + srs.delta + (uint32_t)(bx0 * CC)) & ~15u) + 16u * c;
        uint4 v;
        if (a + 16u <= slimit) {
            // default cache policy: neighbouring tiles re-read these lines from L2
            auto t = __builtin_amdgcn_raw_buffer_load_b128(srs.r, (int)a, 0, 0);
            v = *reinterpret_cast<uint4*>(&t);
        } else {
            uint32_t w[4] = {0, 0, 0, 0};  // the chunk crossing the plane's end
            for (int b = 0; b < 16; ++b)
                if (a + b < slimit)
                    w[b >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(srs.r, (int)(a + b), 0, 0) << (8 * (b & 3));
            v = make_uint4(w[0], w[1], w[2], w[3]);
        }
        return v;
    };
    const int nchunks = nrows * cpr;
    for (int i = tid; i < nchunks; i += 2 * kBlock) {  // two loads in flight per thread
        const int i2 = i + kBlock;
        const uint4 v0 = chunk(i);
        uint4 v1 = make_uint4(0, 0, 0, 0);
        if (i2 < nchunks) v1 = chunk(i2);
        *reinterpret_cast<uint4*>(box + (i / cpr) * cap.stride + 16 * (i % cpr)) = v0;
        if (i2 < nchunks) *reinterpret_cast<uint4*>(box + (i2 / cpr) * cap.stride + 16 * (i2 % cpr)) = v1;
    }
    __syncthreads();

    // ---- sample: wave w takes tile rows 4w..4w+3, lane = column -------------
    TOut* xo = reinterpret_cast<TOut*>(xch[wave]);
    const int x = X0 + lane;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int y = Y0 + wave * 4 + q;
        TOut* o = xo + (q * kTW + lane) * CC;
        if (x >= L.dst.w || y >= L.dst.h) continue;
        // warp_affine_naive.cpp:23-24: (m0*x + m1*y) + m2, all float
        const float fx = L.inv[0] * (float)x + L.inv[1] * (float)y + L.inv[2];
        const float fy = L.inv[3] * (float)x + L.inv[4] * (float)y + L.inv[5];
        int sx = 0, sy = 0;
        float ax = 0.f, ay = 0.f;
        if (!(affine_tap(fy, Hs, sy, ay) && affine_tap(fx, Ws, sx, ax))) {
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                if (OUT == kOutNorm) o[k] = lut[k * 256 + (int)L.border[k]];
                else o[k] = (TOut)L.border[k];
            }
            continue;
        }
        const int wy0 = (int)((1.f - ay) * 2048.f + 0.5f), wy1 = 2048 - wy0;
        const int wx0 = (int)((1.f - ax) * 2048.f + 0.5f), wx1 = 2048 - wx0;
        uint32_t a0, a1, c0, c1;
        if (sx >= bx0 && sx + 1 <= bx1 && sy >= by0 && sy + 1 <= by1) {
            const int r = sy - by0;
            const uint32_t head = ((uint32_t)sy * rp32 + srs.delta + (uint32_t)(bx0 * CC)) & 15u;
            const uint32_t la = (uint32_t)(r * cap.stride) + head + (uint32_t)((sx - bx0) * CC);
            const uint32_t headb = ((uint32_t)(sy + 1) * rp32 + srs.delta + (uint32_t)(bx0 * CC)) & 15u;
            const uint32_t lb = (uint32_t)((r + 1) * cap.stride) + headb + (uint32_t)((sx - bx0) * CC);
            lds_tap8(box, la, a0, a1);
            lds_tap8(box, lb, c0, c1);
        } else {
            // outside the staged box (rounding at its edge): gather as warp_kernel
            const uint32_t o0 = (uint32_t)sy * rp32 + (uint32_t)(sx * CC) + srs.delta;
            const uint32_t o1 = o0 + rp32;
            a0 = a1 = c0 = c1 = 0u;
            if (o1 + 8u <= slimit) {
                auto va = __builtin_amdgcn_raw_buffer_load_b64(srs.r, (int)o0, 0, 0);
                auto vc = __builtin_amdgcn_raw_buffer_load_b64(srs.r, (int)o1, 0, 0);
                a0 = va[0]; a1 = va[1]; c0 = vc[0]; c1 = vc[1];
            } else {
                const unsigned char* r0 = sp + (int64_t)sy * L.src.row_pitch + (int64_t)sx * CC;
                for (int e = 0; e < 2 * CC && e < 8; ++e) {
                    const uint32_t ta = r0[e], tb = r0[L.src.row_pitch + e];
                    if (e < 4) { a0 |= ta << (8 * e); c0 |= tb << (8 * e); }
                    else { a1 |= ta << (8 * (e - 4)); c1 |= tb << (8 * (e - 4)); }
                }
            }
        }
        // warp_affine_naive.cpp:50-54 as (tl*wx0 + tr*wx1)*wy0 + (bl*wx0 +
        // br*wx1)*wy1: the same int32 value (exact: <= 255*2^22)
        typedef unsigned short us2 __attribute__((ext_vector_type(2)));
        const us2 wx = __builtin_bit_cast(us2, (uint32_t)wx0 | ((uint32_t)wx1 << 16));
#pragma unroll
        for (int k = 0; k < CC; ++k) {
            const uint32_t sel = (uint32_t)k | (0x0Cu << 8) | ((uint32_t)(CC + k) << 16) | (0x0Cu << 24);
            const uint32_t top = __builtin_amdgcn_perm(a1, a0, sel);
            const uint32_t bot = __builtin_amdgcn_perm(c1, c0, sel);
            const uint32_t ht = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, top), wx, 0u, false);
            const uint32_t hb = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, bot), wx, 0u, false);
            const int v = (int)((__umul24(ht, (uint32_t)wy0) + __umul24(hb, (uint32_t)wy1)) >> 22);
            if (OUT == kOutSame) o[k] = (TOut)v;
            else if (OUT == kOutF32) o[k] = (TOut)(float)v;
            else o[k] = lut[k * 256 + v];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

    // ---- the wave's 4 row segments, LDS -> HBM ------------------------------------
    const int nx = min(kTW, L.dst.w - X0);
    const int vbytes = nx * CC * (int)sizeof(TOut);
    unsigned char* dbase = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                           (int64_t)plane * L.dst.plane_pitch + (int64_t)X0 * CC * sizeof(TOut);
    const unsigned char* xs = xch[wave];
    const bool aligned = ((reinterpret_cast<uintptr_t>(dbase) | (uintptr_t)L.dst.row_pitch) & 15) == 0;
    const int rows = max(0, min(4, L.dst.h - (Y0 + wave * 4)));
    if (aligned) {
        const int cpr_o = (vbytes + 15) / 16;
        for (int i = lane; i < rows * cpr_o; i += 64) {
            const int q = i / cpr_o, c = i - q * cpr_o;
            unsigned char* drow = dbase + (int64_t)(Y0 + wave * 4 + q) * L.dst.row_pitch;
            const unsigned char* s = xs + q * kRowOut;
            if (16 * c + 16 <= vbytes) {
                __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(s + 16 * c),
                                            reinterpret_cast<u32x4*>(drow) + c);
            } else {
                for (int e = 16 * c; e < vbytes; ++e) drow[e] = s[e];
            }
        }
    } else {
        for (int i = lane; i < rows * vbytes; i += 64) {
            const int q = i / vbytes, e = i - q * vbytes;
            dbase[(int64_t)(Y0 + wave * 4 + q) * L.dst.row_pitch + e] = xs[q * kRowOut + e];
        }
    }
}

template <int CC, int OUT>
hipError_t launch_one(const WarpLaunch& L, const BoxCap& cap, hipStream_t s) {
    const int tiles_x = (L.dst.w + kTW - 1) / kTW, tiles_y = (L.dst.h + kTH - 1) / kTH;
    const int64_t total = (int64_t)tiles_x * tiles_y * L.n * L.src.planes;
    if (total >= 0x7FFFFFF0LL) return hipErrorInvalidValue;
    const int64_t blocks = (total + 7) / 8 * 8;
    const size_t lds = (size_t)cap.h * cap.stride + 16;  // +16: the last tap read's window
    hipLaunchKernelGGL((warp_tile_kernel<CC, OUT>), dim3((unsigned)blocks), dim3(64, 4), lds, s, L, cap, tiles_x,
                       tiles_y, (int)total);
    return hipGetLastError();
}

template <int OUT>
hipError_t launch_cc(const WarpLaunch& L, const BoxCap& cap, hipStream_t s) {
    switch (L.src.cc) {
        case 1: return launch_one<1, OUT>(L, cap, s);
        case 2: return launch_one<2, OUT>(L, cap, s);
        case 3: return launch_one<3, OUT>(L, cap, s);
        case 4: return launch_one<4, OUT>(L, cap, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

// Opt-in (VACV_WARP_TILE=1), for A/B measurement: u8 warps whose tile
// footprint fits the LDS budget.  Measured slower than warp_kernel at 720p
// rot15 (0.395 vs 0.315 ms): the per-pixel LDS address / byte-align work and
// the staging barrier cost more than the gathers saved.
bool warp_tile_applies(const WarpLaunch& L) {
    const char* env = std::getenv("VACV_WARP_TILE");
    if (!(env && env[0] == '1')) return false;
    if (L.src.esize != 1 || L.src.cc > 4) return false;
    const BoxCap cap = box_cap(L.inv, L.src.cc);
    return cap.w > 0 && (int64_t)cap.h * cap.stride <= kBoxBudget;
}

hipError_t launch_warp_tile(const WarpLaunch& L, hipStream_t s) {
    const BoxCap cap = box_cap(L.inv, L.src.cc);
    if (L.out == kOutSame) return launch_cc<kOutSame>(L, cap, s);
    if (L.out == kOutF32) return launch_cc<kOutF32>(L, cap, s);
    return launch_cc<kOutNorm>(L, cap, s);
}

}  // namespace vacv
