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
// Why staging: warp_kernel gathers each tap row with one 8/12-byte load per
// lane; adjacent lanes' windows overlap but are not contiguous, so the
// texture path processes them about one lane per clock per CU (TA/TD busy
// ~90 % of the kernel): the gather kernel is bound by per-lane address
// processing, not HBM.  Here a workgroup owns a 64 x TH output tile and
// stages the tile's source bounding box into LDS with CONTIGUOUS lane loads
// (lane i loads pixels 4i..4i+3 of a box row: CC dwords, 4-byte aligned),
// widening every pixel to one LDS dword.  A tap pair is then two aligned
// LDS dwords (ds_read2), so the sampler spends ~2 LDS instructions per
// output pixel and no byte alignment.  Pixels whose taps fall outside the
// box (rounding at its edge, non-finite matrices) take warp_kernel's global
// gather, so correctness never depends on the box computation.  Outputs
// leave through a per-wave LDS exchange as 16-byte non-temporal stores.
#pragma clang fp contract(off)

#include <cmath>
#include <cstdlib>

#include "vacv_device.hpp"

namespace vacv {
namespace {

constexpr int kTW = 64;                  // tile width (one pixel per lane)
constexpr int kBoxBudget = 40 * 1024;    // LDS bytes for the staged box

// Tile height: a multiple of 16 (each wave samples TH/4 rows, 4 at a time).
// 48 by default: at 1280x720 rot15 a 64 x 48 tile's box is ~1.7x its
// footprint, and 720 rows split into whole tiles.
int tile_height() {
    const char* env = std::getenv("VACV_WARP_TH");
    const int v = env ? std::atoi(env) : 48;
    return (v >= 16 && v <= 128 && v % 16 == 0) ? v : 48;
}

// Box geometry every tile of this launch fits (host and device agree):
// width/height in pixels and the LDS row stride in dwords (one per pixel).
struct BoxCap {
    int w, h, stride;
};

__host__ __device__ inline BoxCap box_cap(const float inv[6], int th) {
    // the tile's source footprint spans |m0|*(TW-1) + |m1|*(TH-1) in x (and
    // the same with m3, m4 in y); +6 covers the floor, the second tap, the
    // one-pixel margins and rounding
    const float ex = fabsf(inv[0]) * (kTW - 1) + fabsf(inv[1]) * (th - 1);
    const float ey = fabsf(inv[3]) * (kTW - 1) + fabsf(inv[4]) * (th - 1);
    BoxCap b{0, 0, 0};
    if (!(ex < 4096.f && ey < 4096.f)) return b;  // also NaN
    b.w = (int)ex + 6;
    b.h = (int)ey + 6;
    int stride = (b.w + 3 + 4 + 3) & ~3;  // align-down head (<4) + the last chunk's overhang
    if (stride % 32 == 0) stride += 4;    // successive rows on different banks
    b.stride = stride;
    return b;
}

template <int CC>
__device__ __forceinline__ void widen4(const uint32_t* w, uint32_t* px) {
    if constexpr (CC == 1) {
        px[0] = w[0]; px[1] = w[0] >> 8; px[2] = w[0] >> 16; px[3] = w[0] >> 24;
    } else if constexpr (CC == 2) {
        px[0] = w[0]; px[1] = w[0] >> 16; px[2] = w[1]; px[3] = w[1] >> 16;
    } else if constexpr (CC == 3) {
        px[0] = w[0];
        px[1] = __builtin_amdgcn_alignbyte(w[1], w[0], 3);
        px[2] = __builtin_amdgcn_alignbyte(w[2], w[1], 2);
        px[3] = w[2] >> 8;
    } else {
        px[0] = w[0]; px[1] = w[1]; px[2] = w[2]; px[3] = w[3];
    }
}

template <int CC, int OUT>
__global__ void __launch_bounds__(kBlock)
warp_tile_kernel(WarpLaunch L, BoxCap cap, int th, int tiles_x, int tiles_y, int total) {
    using TOut = typename std::conditional<(OUT == kOutSame), uint8_t, float>::type;
    constexpr bool kLut = OUT == kOutNorm;
    constexpr int kRowOut = kTW * CC * (int)sizeof(TOut);  // bytes of one tile row
    __shared__ float lut[kLut ? 256 * CC : 1];
    __shared__ __attribute__((aligned(16))) unsigned char xch[4][4 * kRowOut];
    extern __shared__ __attribute__((aligned(16))) uint32_t box[];

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
    const int X0 = tx * kTW, Y0 = ty * th;

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
    const int Yend = min(Y0 + th, L.dst.h);

    // ---- the tile's source box (uniform) from its corner coordinates --------
    float fx_min = INFINITY, fx_max = -INFINITY, fy_min = INFINITY, fy_max = -INFINITY;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float x = (float)(X0 + ((c & 1) ? kTW - 1 : 0));
        const float y = (float)(Y0 + ((c & 2) ? th - 1 : 0));
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
    const int bxa = bx0 & ~3;  // chunks start on 4-pixel boundaries: 4-byte aligned loads
    const int nrows = max(0, by1 - by0 + 1);
    const int cpr = bx1 >= bx0 ? (bx1 - bxa) / 4 + 1 : 0;  // 4-pixel chunks per row

    // ---- stage it: lane-contiguous CC-dword loads, one LDS dword per pixel ---
    // Every load of a pass is issued before any is consumed (no branch between
    // them), so a tile costs one HBM/L2 round trip.  A chunk that crosses the
    // plane's end reads as zeros from the buffer resource and is re-read byte
    // by byte afterwards.
    auto addr = [&](int i) {
        const int r = i / cpr, c = i - r * cpr;
        return (uint32_t)(by0 + r) * rp32 + srs.delta + (uint32_t)((bxa + 4 * c) * CC);
    };
    auto load_chunk = [&](uint32_t a, uint32_t* w) {
        // default cache policy: neighbouring tiles re-read these lines from L2
        if constexpr (CC == 1) {
            w[0] = __builtin_amdgcn_raw_buffer_load_b32(srs.r, (int)a, 0, 0);
        } else if constexpr (CC == 2) {
            auto t = __builtin_amdgcn_raw_buffer_load_b64(srs.r, (int)a, 0, 0);
            w[0] = t[0]; w[1] = t[1];
        } else if constexpr (CC == 3) {
            auto t = __builtin_amdgcn_raw_buffer_load_b96(srs.r, (int)a, 0, 0);
            w[0] = t[0]; w[1] = t[1]; w[2] = t[2];
        } else {
            auto t = __builtin_amdgcn_raw_buffer_load_b128(srs.r, (int)a, 0, 0);
            w[0] = t[0]; w[1] = t[1]; w[2] = t[2]; w[3] = t[3];
        }
    };
    constexpr int kInFlight = 6;
    const int nchunks = nrows * cpr;
    for (int i0 = tid; i0 < nchunks; i0 += kInFlight * kBlock) {
        uint32_t w[kInFlight][CC], a[kInFlight];
#pragma unroll
        for (int j = 0; j < kInFlight; ++j) {
            a[j] = i0 + j * kBlock < nchunks ? addr(i0 + j * kBlock) : 0u;
            load_chunk(a[j], w[j]);
        }
#pragma unroll
        for (int j = 0; j < kInFlight; ++j) {
            const int i = i0 + j * kBlock;
            if (i < nchunks) {
                if (a[j] + 4u * CC > slimit) {  // the chunk crossing the plane's end
#pragma unroll
                    for (int d = 0; d < CC; ++d) w[j][d] = 0;
                    for (int e = 0; e < 4 * CC; ++e)
                        if (a[j] + e < slimit)
                            w[j][e >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(srs.r, (int)(a[j] + e), 0, 0)
                                            << (8 * (e & 3));
                }
                uint32_t px[4];
                widen4<CC>(w[j], px);
                *reinterpret_cast<uint4*>(box + (i / cpr) * cap.stride + 4 * (i % cpr)) =
                    make_uint4(px[0], px[1], px[2], px[3]);
            }
        }
    }
    __syncthreads();

    // ---- sample: wave w takes rows [Y0 + w*th/4, +th/4), 4 at a time --------
    TOut* xo = reinterpret_cast<TOut*>(xch[wave]);
    const int x = X0 + lane;
    const int nx = min(kTW, L.dst.w - X0);
    const int vbytes = nx * CC * (int)sizeof(TOut);
    unsigned char* dbase = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                           (int64_t)plane * L.dst.plane_pitch + (int64_t)X0 * CC * sizeof(TOut);
    const bool aligned = ((reinterpret_cast<uintptr_t>(dbase) | (uintptr_t)L.dst.row_pitch) & 15) == 0;
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    const float fxc = L.inv[0] * (float)x, fyc = L.inv[3] * (float)x;

    for (int yg = Y0 + wave * (th / 4); yg < min(Y0 + (wave + 1) * (th / 4), Yend); yg += 4) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int y = yg + q;
            TOut* o = xo + (q * kTW + lane) * CC;
            if (x >= L.dst.w || y >= Yend) continue;
            // warp_affine_naive.cpp:23-24: (m0*x + m1*y) + m2, all float
            const float fx = fxc + L.inv[1] * (float)y + L.inv[2];
            const float fy = fyc + L.inv[4] * (float)y + L.inv[5];
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
                const uint32_t* t = box + (sy - by0) * cap.stride + (sx - bxa);
                a0 = t[0]; a1 = t[1]; c0 = t[cap.stride]; c1 = t[cap.stride + 1];
            } else {
                // outside the staged box (rounding at its edge): gather the
                // 2*CC tap bytes of both rows, one pixel per dword
                const unsigned char* r0 = sp + (int64_t)sy * L.src.row_pitch + (int64_t)sx * CC;
                a0 = a1 = c0 = c1 = 0u;
                for (int e = 0; e < CC; ++e) {
                    a0 |= (uint32_t)r0[e] << (8 * e);
                    a1 |= (uint32_t)r0[CC + e] << (8 * e);
                    c0 |= (uint32_t)r0[L.src.row_pitch + e] << (8 * e);
                    c1 |= (uint32_t)r0[L.src.row_pitch + CC + e] << (8 * e);
                }
            }
            // warp_affine_naive.cpp:50-54 as (tl*wx0 + tr*wx1)*wy0 + (bl*wx0 +
            // br*wx1)*wy1: the same int32 value (exact: <= 255*2^22)
            const us2 wx = __builtin_bit_cast(us2, (uint32_t)wx0 | ((uint32_t)wx1 << 16));
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                const uint32_t sel = (uint32_t)k | (0x0Cu << 8) | ((uint32_t)(4 + k) << 16) | (0x0Cu << 24);
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

        // ---- the wave's 4 row segments, LDS -> HBM ------------------------------
        const int rows = max(0, min(4, Yend - yg));
        const unsigned char* xs = xch[wave];
        if (aligned) {
            const int cpr_o = (vbytes + 15) / 16;
            for (int i = lane; i < rows * cpr_o; i += 64) {
                const int q = i / cpr_o, c = i - q * cpr_o;
                unsigned char* drow = dbase + (int64_t)(yg + q) * L.dst.row_pitch;
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
                dbase[(int64_t)(yg + q) * L.dst.row_pitch + e] = xs[q * kRowOut + e];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

template <int CC, int OUT>
hipError_t launch_one(const WarpLaunch& L, const BoxCap& cap, int th, hipStream_t s) {
    const int tiles_x = (L.dst.w + kTW - 1) / kTW, tiles_y = (L.dst.h + th - 1) / th;
    const int64_t total = (int64_t)tiles_x * tiles_y * L.n * L.src.planes;
    if (total >= 0x7FFFFFF0LL) return hipErrorInvalidValue;
    const int64_t blocks = (total + 7) / 8 * 8;
    const size_t lds = (size_t)cap.h * cap.stride * 4 + 16;  // +16: the last tap pair past the last row
    hipLaunchKernelGGL((warp_tile_kernel<CC, OUT>), dim3((unsigned)blocks), dim3(64, 4), lds, s, L, cap, th,
                       tiles_x, tiles_y, (int)total);
    return hipGetLastError();
}

template <int OUT>
hipError_t launch_cc(const WarpLaunch& L, const BoxCap& cap, int th, hipStream_t s) {
    switch (L.src.cc) {
        case 1: return launch_one<1, OUT>(L, cap, th, s);
        case 2: return launch_one<2, OUT>(L, cap, th, s);
        case 3: return launch_one<3, OUT>(L, cap, th, s);
        case 4: return launch_one<4, OUT>(L, cap, th, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace

// Opt-in (VACV_WARP_TILE=1), for A/B measurement: u8 warps whose tile box
// fits the LDS budget and whose source rows are 4-byte aligned (the staging
// loads are dword loads).  Measured slower than warp_kernel at 720p rot15
// (0.357 vs 0.283 ms u8 out; 0.599 vs 0.538 ms normalized): PMC shows ~10x
// the gather kernel's LDS bank-conflict cycles (the rotated tap reads of 64
// lanes spread over ~18 box rows) and no drop in texture-path busy time,
// which counts outstanding requests rather than a throughput limit
// (DESIGN.md 3.3).
bool warp_tile_applies(const WarpLaunch& L) {
    const char* env = std::getenv("VACV_WARP_TILE");
    if (!(env && env[0] == '1')) return false;
    if (L.src.esize != 1 || L.src.cc > 4) return false;
    const uint64_t al = reinterpret_cast<uintptr_t>(L.src.base) | (uint64_t)L.src.row_pitch |
                        (uint64_t)L.src.img_pitch | (uint64_t)L.src.plane_pitch;
    if (al & 3) return false;
    const BoxCap cap = box_cap(L.inv, tile_height());
    return cap.w > 0 && (int64_t)cap.h * cap.stride * 4 + 16 <= kBoxBudget;
}

hipError_t launch_warp_tile(const WarpLaunch& L, hipStream_t s) {
    const int th = tile_height();
    const BoxCap cap = box_cap(L.inv, th);
    if (L.out == kOutSame) return launch_cc<kOutSame>(L, cap, th, s);
    if (L.out == kOutF32) return launch_cc<kOutF32>(L, cap, th, s);
    return launch_cc<kOutNorm>(L, cap, th, s);
}

}  // namespace vacv
