// k_warp_frames.hip -- u8 affine bilinear warp, BORDER_CONSTANT, 1 to 4
// interleaved channels or NCHW planes: the per-pixel geometry computed once
// for many frames, the source boxes copied HBM -> LDS by LDS-DMA.  A "frame"
// here is what one sampler pass sees: a whole NHWC image, or one plane of an
// NCHW image.
//
// Reference: WarpAffineNaive::warp_affine_naive_hwc_u8 (warp_affine_naive.cpp:
// 9-58) driven by WarpAffine::warp_affine_naive (warp_affine.cpp:111-169).
// Per output pixel: f = (m0*x + m1*y) + m2 in float; floor; skip when the
// top-left tap is outside [0,w-2]x[0,h-2]; weights SAT((1-f)*2048) and
// 2048-that; value (Sum S*wx*wy) >> 22.  Skipped pixels get the border value.
//
// Why this shape.  The gather kernels of k_warp.hip are
// bound by the vector cache's tag lookups (one per lane quad and cache line of
// every gather instruction).  But one launch warps a whole batch with ONE
// matrix, so everything but the source bytes -- coordinates, weights, LDS
// addresses -- is the same for every frame.  A workgroup owns a 64 x TH
// output tile of kf consecutive frames:
//  1. once: each lane computes its NP pixels' taps and the workgroup reduces
//     them to the source box the tile's taps reach, and per box row the span
//     its parallelogram needs;
//  2. per frame: the box rows' spans are copied into an LDS slot by
//     buffer_load_dwordx4 ... lds (no VGPR staging; the next frame's copy is
//     in flight while this one is sampled); each pixel reads the dwords under
//     its two tap pairs and blends in the reference's fixed point.
// Pixels outside the source read a border pattern kept at the head of each
// slot, with weights (2048, 0) x (2048, 0), so they need no select.  A tile
// no pixel of which taps the source writes the border value without any
// sampling; a tile whose box exceeds the plan (never for the planned
// geometry; the plan's bound is conservative) takes its taps from memory.
#pragma clang fp contract(off)

#include <climits>
#include <cstring>
#include <cmath>
#include <map>
#include <mutex>
#include <vector>

#include "vacv_device.hpp"

namespace vacv {
namespace {

constexpr int kFrTileW = 64;   // output columns per tile (one per lane)

template <int CC>
__device__ __forceinline__ uint32_t pack_bytes(const unsigned char* p) {
    uint32_t v = 0;
#pragma unroll
    for (int k = 0; k < CC; ++k) v |= (uint32_t)p[k] << (8 * k);
    return v;
}

// The taps of pixel (x, y) from memory, bytewise, or the border pattern
// outside the source: the rare path of a tile whose box exceeds the LDS plan.
template <int CC>
__device__ __forceinline__ void direct_taps(const WarpLaunch& L, const unsigned char* sp, int x, int y, uint32_t& tl,
                                         uint32_t& tr, uint32_t& bl, uint32_t& br) {
    const float* M = L.inv;
    const float fx = (M[0] * (float)x + M[1] * (float)y) + M[2];
    const float fy = (M[3] * (float)x + M[4] * (float)y) + M[5];
    if ((x < L.dst.w) & (fx >= 0.f) & (fx < (float)(L.src.w - 1)) & (fy >= 0.f) & (fy < (float)(L.src.h - 1))) {
        const unsigned char* r0 = sp + (int64_t)(int)fy * L.src.row_pitch + (int64_t)(int)fx * CC;
        tl = pack_bytes<CC>(r0);
        tr = pack_bytes<CC>(r0 + CC);
        bl = pack_bytes<CC>(r0 + L.src.row_pitch);
        br = pack_bytes<CC>(r0 + L.src.row_pitch + CC);
    } else {
        uint32_t bp = 0;
#pragma unroll
        for (int k = 0; k < CC; ++k) bp |= (uint32_t)(int)L.border[k] << (8 * k);
        tl = tr = bl = br = bp;
    }
}

// ---------------------------------------------------------------------------
// warp_ring_kernel: the frames kernel with its staging moved off the
// registers.  Boxes are copied HBM -> LDS by LDS-DMA (buffer_load_dwordx4 ...
// lds: 16 bytes per lane straight into LDS, no VGPR destination) as raw pixel
// bytes, into a ring of ns LDS slots, so ns - 1 frames' boxes are in flight
// while a frame is sampled (the register-staged kernel had one, and its blend
// and staging halves serialised on that one HBM round trip: DESIGN.md §3.3).
// A tap row's 2 CC bytes are read as the dwords covering them and shifted
// into place (v_alignbyte), so there is no re-spread pass either.
//
// Synchronisation (the compiler does not track LDS-DMA, so it is explicit):
// every wave issues, per frame, exactly n_w DMA instructions and, per sampled
// frame, exactly kStores stores (every store is issued, out-of-range lanes at
// an offset past the buffer), so before frame f's barrier the wave waits for
// vmcnt <= (ns - 2) n_w + (stores issued since frame f's DMA): its own DMA of
// frame f has landed, the later frames' stay in flight (gfx950 retires
// vector-memory operations in issue order).  The barrier then publishes every
// wave's part, and frame f + ns - 1's DMA reuses the slot that frame f - 1
// was sampled from -- every wave has consumed those reads before the barrier.
constexpr int kRingMaxIt = 6;  // DMA instructions per wave and frame, at most (a box of 24 KiB)

// L: launch block; gx, gy: tiles per frame; kf: frames per workgroup; S: LDS
// bytes per staged row (a multiple of 16); rows_max: staged rows per slot;
// ns, slot: LDS slots and their bytes; dst_al: the destination allows dword
// (u8 out) stores; ginv = ceil(2^20 / (S / 16)) (row of chunk c = c ginv >> 20,
// exact for c < 4096 and S / 16 <= 256).
// u8 output: pixels whose taps are read before their blends.  4: 103 VGPRs, 4
// waves per SIMD; 2: 95, 5 waves (round 4, one box, 720p rot15: 0.1761 /
// 0.1776 vs 0.1807 / 0.1812 ms; round 2's register-staged kernel preferred 2).
// Other outputs keep 2.
constexpr int kRingGrp = 4;
template <int CC, int OUT, int NP, bool PLANAR>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1)))
warp_ring_kernel(WarpLaunch L, int gx, int gy, int kf, int S, int rows_max, int ns, int slot, int dst_al,
                 uint32_t ginv) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int TH = 4 * NP;
    // staging loads: sc0 for byte output (neighbouring tiles' boxes share
    // rows through L2), non-temporal for fp32 output, whose 4x larger stores
    // want the L2
    constexpr int kAux = OUT == kOutSame ? 1 : VACV_LOAD_AUX;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int* red = reinterpret_cast<int*>(lds + ns * slot);  // 4 waves x 4 ints
    unsigned char* xch = lds + ns * slot + 64 + (tid >> 6) * (2 * 64 * CC);

    const int tiles = gx * gy;
    const int nfr = L.n * L.src.planes;
    const int total = tiles * ((nfr + kf - 1) / kf);
    const int per_xcd = (total + 7) / 8;
    const int id = (int)(blockIdx.x % 8) * per_xcd + (int)(blockIdx.x / 8);
    if (id >= total) return;  // uniform
    const int fg = id / tiles, tile = id - fg * tiles;
    const int by = tile / gx, bx = tile - by * gx;
    const int f0 = fg * kf, f1 = min(f0 + kf, nfr);
    auto frame_img = [&](int f) { return PLANAR ? f / L.src.planes : f; };
    auto frame_off = [&](int f, const PlaneGeom& g) {
        const int img = frame_img(f), pl = f - img * L.src.planes;
        return PLANAR ? (int64_t)img * g.img_pitch + (int64_t)pl * g.plane_pitch : (int64_t)f * g.img_pitch;
    };
    const float* M = L.inv;
    const float wlim = (float)(L.src.w - 1), hlim = (float)(L.src.h - 1);
    const int x = bx * kFrTileW + lane;
    const int yw = by * TH + wave * NP;
    const uint32_t rp = (uint32_t)L.src.row_pitch;

    // ---- 1. per-pixel taps, once for every frame ---------------------------
    const float axm = M[0] * (float)x, aym = M[3] * (float)x;
    // per pixel until the box is known: sx | sy << 16 and v0 | wa4 << 16
    // (16 registers instead of 32 at the kernel's register peak)
    uint32_t sxy[NP], vwa[NP], okm = 0;
    int xmin = INT_MAX, xmax = INT_MIN, ymin = INT_MAX, ymax = INT_MIN;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const int y = yw + j;
        // warp_affine_naive.cpp:23-24: (m0*x + m1*y) + m2, all float
        const float fx = (axm + M[1] * (float)y) + M[2];
        const float fy = (aym + M[4] * (float)y) + M[5];
        // warp_affine_naive.cpp:26-39: floor(f) in [0, n-2] <=> 0 <= f < n-1
        const bool ok = (x < L.dst.w) & (y < L.dst.h) & (fx >= 0.f) & (fx < wlim) & (fy >= 0.f) & (fy < hlim);
        const int sx = ok ? (int)fx : 0, sy = ok ? (int)fy : 0;
        const float ax = fx - (float)sx, ay = fy - (float)sy;
        const uint32_t w0 = (uint32_t)(int)((1.f - ay) * 2048.f + 0.5f);
        const uint32_t v0 = (uint32_t)(int)((1.f - ax) * 2048.f + 0.5f);
        sxy[j] = (uint32_t)sx | ((uint32_t)sy << 16);
        vwa[j] = ok ? (v0 | ((4u * w0) << 16)) : (2048u | (8192u << 16));
        okm |= (uint32_t)ok << j;
        if (ok) {
            xmin = min(xmin, sx);
            xmax = max(xmax, sx);
            ymin = min(ymin, sy);
            ymax = max(ymax, sy);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        xmin = min(xmin, __shfl_xor(xmin, o, 64));
        xmax = max(xmax, __shfl_xor(xmax, o, 64));
        ymin = min(ymin, __shfl_xor(ymin, o, 64));
        ymax = max(ymax, __shfl_xor(ymax, o, 64));
    }
    if (lane == 0) {
        red[4 * wave + 0] = xmin;
        red[4 * wave + 1] = xmax;
        red[4 * wave + 2] = ymin;
        red[4 * wave + 3] = ymax;
    }
    // each slot's 16-byte head: the border pixel repeated (a border pixel
    // reads its taps there, with weights (2048,0) x (2048,0))
    if (tid < 4 * ns) {
        uint32_t bp = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) bp |= (uint32_t)(int)L.border[(4 * (tid & 3) + e) % CC] << (8 * e);
        *reinterpret_cast<uint32_t*>(lds + (tid >> 2) * slot + 4 * (tid & 3)) = bp;
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        xmin = min(xmin, red[4 * w + 0]);
        xmax = max(xmax, red[4 * w + 1]);
        ymin = min(ymin, red[4 * w + 2]);
        ymax = max(ymax, red[4 * w + 3]);
    }
    xmin = __builtin_amdgcn_readfirstlane(xmin);
    xmax = __builtin_amdgcn_readfirstlane(xmax);
    ymin = __builtin_amdgcn_readfirstlane(ymin);
    ymax = __builtin_amdgcn_readfirstlane(ymax);
    const bool any = xmax >= 0;
    const int bx0 = any ? (xmin & ~3) : 0;                         // first staged column (bx0 * CC dword-aligned)
    const int G = any ? ((xmax + 2 - bx0) * CC + 15) >> 4 : 0;     // 16-byte chunks per staged row
    const int R = any ? ymax + 2 - ymin : 0;                       // staged rows ymin .. ymax + 1
    const int Gs = S >> 4;                                         // chunks per LDS row
    const int n_inst = (R * Gs + 63) >> 6;                         // 1 KiB DMA instructions per frame
    const bool staged = any && G <= Gs && R <= rows_max && n_inst <= 4 * kRingMaxIt;  // uniform
    // this wave's DMA instructions per frame: i = wave, wave + 4, ...
    const int n_w = staged && n_inst > wave ? (n_inst - wave + 3) >> 2 : 0;
    uint32_t rw[NP], wxp[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const bool ok = (okm >> j) & 1u;
        const int sx = (int)(sxy[j] & 0xFFFFu), sy = (int)(sxy[j] >> 16);
        rw[j] = (ok ? (uint32_t)(16 + (sy - ymin) * S + (sx - bx0) * CC) : 0u) | (vwa[j] & 0xFFFF0000u);
        const uint32_t v0 = vwa[j] & 0xFFFFu;  // outside: (2048, 0)
        wxp[j] = ok ? (v0 | ((2048u - v0) << 16)) : 2048u;
    }

    // Row spans.  The box's rows near its top and bottom need only part of
    // its width (a rotated tile's source footprint is a parallelogram: ~0.6
    // of its bounding box at 15 degrees).  Thread t < R clips the
    // parallelogram of the tile's corners to the band of source rows whose
    // pixels tap row ymin + t (fy in [r - 1, r + 1), widened by 0.05 px for
    // the float rounding of the reference's coordinates) and records the
    // 16-byte chunks it needs, columns floor(x) .. floor(x) + 1.
    // The table lives in the last slot's data, which no DMA writes before
    // frame f0's barrier.
    uint32_t* spans = reinterpret_cast<uint32_t*>(lds + (ns - 1) * slot + 16);  // after that slot's border head
    if (staged && tid < R) {
        const float X0 = (float)(bx * kFrTileW), X1 = (float)(min(bx * kFrTileW + kFrTileW, L.dst.w) - 1);
        const float Y0 = (float)(by * TH), Y1 = (float)(min(by * TH + TH, L.dst.h) - 1);
        float cx[4], cy[4];
        const float px[4] = {X0, X1, X1, X0}, py[4] = {Y0, Y0, Y1, Y1};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            cx[i] = (M[0] * px[i] + M[1] * py[i]) + M[2];
            cy[i] = (M[3] * px[i] + M[4] * py[i]) + M[5];
        }
        const float r = (float)(ymin + tid), ya = r - 1.05f, yb = r + 1.05f;
        float lo = 3.0e38f, hi = -3.0e38f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int i2 = (i + 1) & 3;
            if (cy[i] >= ya && cy[i] <= yb) { lo = fminf(lo, cx[i]); hi = fmaxf(hi, cx[i]); }
#pragma unroll
            for (int e = 0; e < 2; ++e) {
                const float yl = e ? yb : ya;
                if ((cy[i] - yl) * (cy[i2] - yl) < 0.f) {
                    const float xc = cx[i] + (yl - cy[i]) / (cy[i2] - cy[i]) * (cx[i2] - cx[i]);
                    lo = fminf(lo, xc);
                    hi = fmaxf(hi, xc);
                }
            }
        }
        uint32_t sp = 1u;  // empty: lo = 1 > hi = 0
        if (lo <= hi) {
            const int clo = (int)floorf(fmaxf(lo - 0.05f, -1.0e9f)) - bx0;       // left tap column
            const int chi = (int)floorf(fminf(hi + 0.05f, 1.0e9f)) + 1 - bx0;    // right tap column
            if (chi >= 0 && clo * CC <= 16 * G - 1) {
                const int glo = (max(clo, 0) * CC) >> 4, ghi = min(((chi + 1) * CC - 1) >> 4, G - 1);
                sp = (uint32_t)glo | ((uint32_t)ghi << 16);
            }
        }
        spans[tid] = sp;
    }
    __syncthreads();

    // this lane's DMA source offsets (frame-relative), frame-independent:
    // instruction u of this wave covers the slot's chunks 64 (wave + 4u) + lane.
    // vm: chunks inside their row's span; tailm: those reaching past the
    // plane's last byte (loaded bytewise after the DMA instead)
    uint32_t goff[kRingMaxIt];
    uint32_t vm = 0, tailm = 0;
#pragma unroll
    for (int u = 0; u < kRingMaxIt; ++u) {
        goff[u] = 0;
        if (u < n_w) {
            const int c = 64 * (wave + 4 * u) + lane;
            const int row = (int)(__umul24((uint32_t)c, ginv) >> 20), col = c - row * Gs;  // c / Gs
            if (row < R && col < G) {
                const uint32_t sp = spans[row];
                if ((int)(sp & 0xFFFFu) <= col && col <= (int)(sp >> 16)) {
                    goff[u] = (uint32_t)(ymin + row) * rp + (uint32_t)(bx0 * CC + 16 * col);
                    if ((int64_t)goff[u] + 16 > L.src.plane_bytes) tailm |= 1u << u;
                    else vm |= 1u << u;
                }
            }
        }
    }
    // frame f's box -> slot s: n_w instructions, idle lanes out of range
    // (an out-of-range lane writes zeros to its own 16 bytes of the slot)
    auto dma = [&](int f, int s, bool live) {
        const Rsrc rs = make_rsrc(L.src.base + frame_off(min(f, nfr - 1), L.src), L.src.plane_bytes);
        unsigned char* base = lds + s * slot + 16 + 1024 * wave;
#pragma unroll
        for (int u = 0; u < kRingMaxIt; ++u) {
            if (u < n_w) {
                const int off = (live && ((vm >> u) & 1u)) ? (int)(goff[u] + rs.delta) : (int)0x80000000;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs.r, (lds_void*)(base + 4096 * u), 16, off, 0, 0, kAux);
            }
        }
    };
    // the rare chunks at the plane's end, bytewise (after frame f's DMA landed)
    auto fix_tail = [&](int f, int s) {
        const Rsrc rs = make_rsrc(L.src.base + frame_off(f, L.src), L.src.plane_bytes);
#pragma unroll
        for (int u = 0; u < kRingMaxIt; ++u) {
            if ((tailm >> u) & 1u) {
                uint32_t d[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    uint32_t w = 0;
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        w |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rs.r, (int)(goff[u] + rs.delta) + 4 * q + e,
                                                                           0, 0) << (8 * e);
                    d[q] = w;
                }
                const int c = 64 * (wave + 4 * u) + lane;
                *reinterpret_cast<u32x4*>(lds + s * slot + 16 + 16 * c) = u32x4{d[0], d[1], d[2], d[3]};
            }
        }
    };

    const uint32_t dpitch = (uint32_t)L.dst.row_pitch;
    const bool tile_full = bx * kFrTileW + kFrTileW <= L.dst.w && by * TH + TH <= L.dst.h &&
                           (OUT != kOutSame || dst_al);
    constexpr uint32_t kOob = 0x80000000u;
    // vector-memory stores per sampled frame, every one issued (the wait
    // count).  Full tiles issue only 16-byte (u8) or one-per-row fp32 stores
    // at per-row addresses, which the compiler cannot merge, so the count is
    // exact; edge tiles count 0, i.e. their wait also drains the previous
    // frame's byte stores (conservative: ~9 % of cfg4's tiles).
    const int n_st = !tile_full ? 0 : OUT != kOutSame ? NP : NP / 2;

    auto emit = [&](auto full_c, int fv, int j, uint32_t tlo, uint32_t thi, uint32_t blo, uint32_t bhi) {
        constexpr bool FULL = decltype(full_c)::value;
        const int f = __builtin_amdgcn_readfirstlane(fv);
        const int y = yw + j;
        const bool inside = FULL || (x < L.dst.w && y < L.dst.h);
        unsigned char* dbase = const_cast<unsigned char*>(L.dst.base) + frame_off(f, L.dst);
        const Rsrc drs = make_rsrc(dbase, L.dst.plane_bytes);
        const us2 wx = __builtin_bit_cast(us2, wxp[j]);
        const uint32_t wA = rw[j] >> 16, wB = 8192u - (rw[j] >> 16);
        uint32_t vv[CC];
#pragma unroll
        for (int k = 0; k < CC; ++k) {
            // channel k of the left tap (byte k) and of the right tap (byte CC + k)
            const uint32_t sel = (uint32_t)k | (0x0Cu << 8) | ((uint32_t)(CC + k) << 16) | (0x0Cu << 24);
            const uint32_t top = __builtin_amdgcn_perm(thi, tlo, sel);
            const uint32_t bot = __builtin_amdgcn_perm(bhi, blo, sel);
            const uint32_t ht = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, top), wx, 0u, false);
            const uint32_t hb = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, bot), wx, 0u, false);
            vv[k] = __umul24(ht, wA) + __umul24(hb, wB);  // warp_affine_naive.cpp:50-54, x4
        }
        const uint32_t drow = (uint32_t)y * dpitch + drs.delta;
        if constexpr (OUT == kOutSame) {
            uint32_t own;
            if constexpr (CC == 1) {
                own = vv[0] >> 24;
            } else if constexpr (CC == 2) {
                own = __builtin_amdgcn_perm(vv[1], vv[0], 0x0C0C0703u);
            } else if constexpr (CC == 3) {
                own = __builtin_amdgcn_perm(vv[2], __builtin_amdgcn_perm(vv[1], vv[0], 0x0C0C0703u), 0x0C070100u);
            } else {
                own = __builtin_amdgcn_perm(__builtin_amdgcn_perm(vv[3], vv[2], 0x0C0C0703u),
                                            __builtin_amdgcn_perm(vv[1], vv[0], 0x0C0C0703u), 0x05040100u);
            }
            if constexpr (FULL) {
                const uint32_t word = quad_pack<CC>(own, lane & 3);
                constexpr int kRowB = 64 * CC;
                unsigned char* xw = xch + (j & 1) * kRowB;
                if ((lane & 3) < CC) *reinterpret_cast<uint32_t*>(xw + 4 * ((lane >> 2) * CC + (lane & 3))) = word;
                if (j & 1) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    constexpr int kChunks = kRowB / 16;
                    const int m = lane % (2 * kChunks);
                    const u32x4 v = *reinterpret_cast<const u32x4*>(xch + 16 * m);
                    const uint32_t rowoff = (uint32_t)(y - 1 + (m >= kChunks)) * dpitch + drs.delta;
                    const uint32_t off = lane < 2 * kChunks
                                             ? rowoff + (uint32_t)(bx * kFrTileW * CC + 16 * (m % kChunks))
                                             : kOob;
                    __builtin_amdgcn_raw_buffer_store_b128(v, drs.r, (int)off, 0, VACV_STORE_AUX);
                }
            } else {  // the edges, or a byte-aligned destination: CC byte stores, all issued
                const uint32_t off = inside ? drow + (uint32_t)(x * CC) : kOob;
#pragma unroll
                for (int k = 0; k < CC; ++k)
                    __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(own >> (8 * k)), drs.r,
                                                         (int)(inside ? off + k : kOob), 0, VACV_STORE_AUX);
            }
        } else {
            u32x4 o;
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                const int v = (int)(vv[k] >> 24);
                float fv;
                if (OUT == kOutF32) {
                    fv = (float)v;
                } else {
                    const int img = frame_img(f), pl = f - img * L.src.planes;
                    const ChanNorm cn = chan_norm(L.norm, img, PLANAR ? pl : k);
                    fv = normalize_u8v(cn, v);
                }
                o[k] = __builtin_bit_cast(uint32_t, fv);
            }
            const int off = (int)(inside ? drow + (uint32_t)(x * CC * 4) : kOob);
            if constexpr (CC == 1) {
                __builtin_amdgcn_raw_buffer_store_b32(o[0], drs.r, off, 0, VACV_STORE_AUX);
            } else if constexpr (CC == 2) {
                typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                __builtin_amdgcn_raw_buffer_store_b64(u32x2{o[0], o[1]}, drs.r, off, 0, VACV_STORE_AUX);
            } else if constexpr (CC == 3) {
                typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
                const u32x3 o3 = {o[0], o[1], o[2]};
                __builtin_amdgcn_raw_buffer_store_b96(o3, drs.r, off, 0, VACV_STORE_AUX);
            } else {
                __builtin_amdgcn_raw_buffer_store_b128(o, drs.r, off, 0, VACV_STORE_AUX);
            }
        }
    };

    using full_t = std::integral_constant<bool, true>;
    using edge_t = std::integral_constant<bool, false>;
    if (!any) {
        // uniform: no pixel of the tile taps the source (a rotated warp's
        // corners: 80 of cfg4's 460 tiles) -- every pixel is the border value,
        // with no staging and no per-pixel arithmetic per frame
        auto border_byte = [&](int i) { return (uint32_t)(int)L.border[i % CC]; };
        if constexpr (OUT == kOutSame) {
            if (tile_full) {
                // the 2-row store segments of the byte path, constant: built once
                constexpr int kRowB = 64 * CC, kChunks = kRowB / 16;
                const int m = lane % (2 * kChunks);
                u32x4 v;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    uint32_t w = 0;
#pragma unroll
                    for (int e = 0; e < 4; ++e) w |= border_byte(16 * (m % kChunks) + 4 * q + e) << (8 * e);
                    v[q] = w;
                }
                for (int fv = f0; fv < f1; ++fv) {
                    const int f = __builtin_amdgcn_readfirstlane(fv);
                    const Rsrc drs = make_rsrc(L.dst.base + frame_off(f, L.dst), L.dst.plane_bytes);
#pragma unroll
                    for (int j = 1; j < NP; j += 2) {
                        const uint32_t rowoff = (uint32_t)(yw + j - 1 + (m >= kChunks)) * dpitch + drs.delta;
                        const uint32_t off = lane < 2 * kChunks
                                                 ? rowoff + (uint32_t)(bx * kFrTileW * CC + 16 * (m % kChunks))
                                                 : kOob;
                        __builtin_amdgcn_raw_buffer_store_b128(v, drs.r, (int)off, 0, VACV_STORE_AUX);
                    }
                }
                return;
            }
        }
        // the blend of the border pattern (weights (2048,0) x (2048,0))
        uint32_t bl = 0, bh = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            bl |= border_byte(e) << (8 * e);
            bh |= border_byte(4 + e) << (8 * e);
        }
        for (int f = f0; f < f1; ++f) {
            // opaque per frame: hoisting the 8 blends out of the frame loop
            // kept them all live (103 -> 127 VGPRs for the whole kernel)
            asm volatile("" : "+v"(bl), "+v"(bh));
            if (OUT != kOutSame && tile_full) {  // (byte output took the path above)
                for (int j = 0; j < NP; ++j) emit(full_t(), f, j, bl, bh, bl, bh);
            } else {
                for (int j = 0; j < NP; ++j) emit(edge_t(), f, j, bl, bh, bl, bh);
            }
        }
        return;
    }
    if (!staged) {  // uniform, rare: the box is over the plan -- taps from memory
        for (int f = f0; f < f1; ++f) {
            const unsigned char* sp = L.src.base + frame_off(f, L.src);
            for (int j = 0; j < NP; ++j) {
                uint32_t tl, tr, bl, br;
                direct_taps<CC>(L, sp, x, yw + j, tl, tr, bl, br);
                // as a (lo, hi) byte stream: left tap's CC bytes, then the right tap's
                uint32_t tlo, thi, blo, bhi;
                if constexpr (CC == 4) {
                    tlo = tl; thi = tr; blo = bl; bhi = br;
                } else {
                    const uint64_t t = (uint64_t)tl | ((uint64_t)tr << (8 * CC));
                    const uint64_t b = (uint64_t)bl | ((uint64_t)br << (8 * CC));
                    tlo = (uint32_t)t; thi = (uint32_t)(t >> 32); blo = (uint32_t)b; bhi = (uint32_t)(b >> 32);
                }
                emit(edge_t(), f, j, tlo, thi, blo, bhi);
            }
        }
        return;
    }
    // A tap row's 2 CC bytes start at any byte: read the dwords that cover
    // them (dword-aligned ds_read2_b32 / ds_read_b32 -- an unaligned
    // ds_read_b64 is replayed at 64 cycles) and shift by the byte offset.
    constexpr int kDw = CC == 3 ? 3 : 2;  // dwords covering 2 CC bytes at any byte offset
    auto taps_at = [&](const unsigned char* row, uint32_t sh, uint32_t& lo, uint32_t& hi) {
        const uint32_t* t = reinterpret_cast<const uint32_t*>(row);
        uint32_t d[kDw];
#pragma unroll
        for (int q = 0; q < kDw; ++q) d[q] = t[q];
        if constexpr (CC == 4) {
            lo = d[0];
            hi = d[1];
        } else {
            lo = __builtin_amdgcn_alignbyte(d[1], d[0], sh);
            hi = kDw == 3 ? __builtin_amdgcn_alignbyte(d[kDw - 1], d[1], sh) : 0u;
        }
    };
    auto sample = [&](auto full_c, int f, uint32_t sbase) {
        constexpr int kGrp = OUT == kOutSame ? kRingGrp : 2;
#pragma unroll
        for (int j0 = 0; j0 < NP; j0 += kGrp) {
            uint32_t tp[kGrp][4];
#pragma unroll
            for (int j = 0; j < kGrp; ++j) {
                const uint32_t ra = rw[j0 + j] & 0xFFFFu;
                const unsigned char* a = lds + sbase + (ra & ~3u);
                taps_at(a, ra & 3u, tp[j][0], tp[j][1]);
                taps_at(a + S, ra & 3u, tp[j][2], tp[j][3]);
            }
#pragma unroll
            for (int j = 0; j < kGrp; ++j) emit(full_c, f, j0 + j, tp[j][0], tp[j][1], tp[j][2], tp[j][3]);
        }
    };
    // prologue: frames f0 .. f0 + ns - 2 in flight
    for (int k = 0; k < ns - 1; ++k) dma(f0 + k, k, f0 + k < f1);
    int s = 0;
    for (int f = f0; f < f1; ++f) {
        // this wave's DMA of frame f has landed: later operations still in
        // flight are the DMAs of frames f + 1 .. f + ns - 2 and the stores of
        // the (at most ns - 1) frames sampled since frame f's DMA was issued
        wait_vm((ns - 2) * n_w + min(f - f0, ns - 1) * n_st);
        if (tailm) {
            fix_tail(f, s);
            wait_lgkm();  // its LDS stores land before the barrier (s_barrier does not wait for them)
        }
        __builtin_amdgcn_s_barrier();  // every wave's part of frame f is in; frame f - 1's reads are done
        const int sn = s == 0 ? ns - 1 : s - 1;  // (f + ns - 1) mod ns: the slot frame f - 1 used
        dma(f + ns - 1, sn, f + ns - 1 < f1);
        if (tile_full) sample(full_t(), f, (uint32_t)(s * slot));
        else sample(edge_t(), f, (uint32_t)(s * slot));
        s = s + 1 == ns ? 0 : s + 1;
    }
    wait_vm(0);  // no LDS-DMA may outlive the workgroup's LDS
}

// ---------------------------------------------------------------------------
// warp_exp_kernel (round 5): 3-channel u8 warps.  Two changes against the
// ring kernel, both per workgroup and frame-independent (once per tile):
//
// 1. Compact staging, two frames in flight.  The ring kernel's slots held the
//    box's bounding rectangle (rows_max x G chunks, ~14 KiB at cfg4) although
//    the DMA only fills each row's span of the tile's source parallelogram,
//    so a slot per frame in flight cost the LDS of ~1.6 frames and four
//    workgroups per CU kept only ~36 KiB of HBM reads in flight -- about half
//    of what hides an HBM miss (MI355X_MICROARCH.md: ~72 KiB per CU).  Here a
//    slot holds the spans back to back (row r's chunks glo_r .. ghi_r at
//    chunk RB_r = the prefix of the rows above), ~9 KiB at cfg4, and there
//    are two: frames f + 1 and f + 2 are in flight while f is sampled.
// 2. A 4-byte-pixel image.  Each frame's spans are re-laid once into an LDS
//    image of [b g r x] pixels, again only the spans (16-pixel units of each
//    row, back to back): the re-lay is 3 VALU per 4 source pixels (the first
//    dword as it is, one v_alignbyte / shift for each other); a thread takes
//    4 pixels (a quarter unit) per step, 3 dwords in and one ds_write_b128
//    out, so a wave's writes are 1 KiB contiguous (whole units per lane
//    wrote 64 bytes apart: 4-way LDS bank conflicts, ~290 LDS cycles per
//    tile and frame).  A pixel's taps are then two ds_read2_b32
//    (offsets 0 and 1) at two frame-independent addresses, one per tap row --
//    no per-pixel alignment fix-up (the ring kernel: 6 ds_read_b32 and 4
//    v_alignbyte per pixel); the blend is unchanged (v_perm to the (tl_k,
//    tr_k) u16 pair, v_dot2_u32_u16 per row, 24-bit row multiplies).
//
// The chunk -> row and unit -> row maps are byte tables built once per tile,
// so every lane's DMA source offsets and re-lay offsets are registers.  u8
// output leaves through a 4-row LDS exchange per wave as 12-byte stores (all
// 64 lanes, 192 contiguous bytes per row); fp32 as 16-byte stores per row.
// Per frame: wait for the own DMA of frame f, barrier, re-lay, barrier,
// issue frame f + 2's DMA into the slot just re-laid, sample.
constexpr int kExpQ = 4;         // re-lay quarter units (4 pixels of one box row) per thread and frame, at most
constexpr int kExpUnits = kExpQ * kBlock / 4;  // image units (16 pixels) per tile, at most
constexpr int kExpRows = 128;    // staged rows per tile, at most (the setup tables)
constexpr int kExpTab = 16 + 12 * kExpRows + 64 * 4 * kRingMaxIt + kExpUnits + 16;  // setup tables, bytes
constexpr int kExpGrp = 2;  // pixels whose taps are read before their blends (4: spills at <= 128 VGPRs)
// Output through a per-wave LDS exchange: u8 4 rows -> 12-byte stores (DPP quad
// packing with one dword store per row measured 0.186 vs 0.176 ms), fp32 one
// row -> 16-byte stores (one 12-byte store per pixel: 0.422 vs 0.416 ms).
constexpr int kExpXB(int out) { return out == kOutSame ? 4 * 64 * 4 : 64 * 3 * 4; }  // exchange bytes per wave
// NN: INTER_NEAREST (OpenCV 2.4's warpAffine map, see warp_nearest_kernel in
// k_warp.hip): the same staging, one tap per pixel, no blend.
template <int OUT, int NP, bool NN>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4)))  // <= 128 VGPRs: 4 workgroups per CU, as the LDS plan
warp_exp_kernel(WarpLaunch L, int gx, int gy, int kf, int slot_bytes, int exp_units, int dst_al) {
    constexpr int CC = 3;
    constexpr int TW = kFrTileW;
    constexpr int TH = 4 * NP;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    // [48 B pad][slot 0][slot 1][64 B pad] (the re-lay reads up to 45 B before
    // and 47 B after a row's chunks: bytes of no tapped pixel)
    // [image: 16 B border pixel head, then exp_units x 16 pixels; the setup
    //  tables live here until the first re-lay] [exchange: 4 waves x kXB]
    constexpr int kXB = kExpXB(OUT);
    const uint32_t ebase = 48u + 2u * (uint32_t)slot_bytes + 64u;
    const uint32_t xbase = ebase + 16u + 64u * (uint32_t)max(exp_units, (kExpTab + 63) / 64);
    constexpr int kAux = OUT == kOutSame ? 1 : VACV_LOAD_AUX;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    int* red = reinterpret_cast<int*>(lds + xbase);  // 4 waves x 4 ints, setup only
    unsigned char* xch = lds + xbase + wave * kXB;
    // setup tables (image region): per row span glo | ghi << 16, prefix
    // RB | UP << 16 (chunks, units), first unit | units << 16; chunk -> row and
    // unit -> row bytes; totals
    uint32_t* t_sp = reinterpret_cast<uint32_t*>(lds + ebase + 16);
    uint32_t* t_pre = t_sp + kExpRows;
    uint32_t* t_un = t_pre + kExpRows;
    unsigned char* t_crow = reinterpret_cast<unsigned char*>(t_un + kExpRows);
    unsigned char* t_urow = t_crow + 64 * 4 * kRingMaxIt;
    uint32_t* t_tot = reinterpret_cast<uint32_t*>(t_urow + kExpUnits);
    int* t_min = reinterpret_cast<int*>(t_crow);  // per-row tapped columns (until the chunk map is built)
    int* t_max = t_min + kExpRows;

    const int tiles = gx * gy;
    const int nfr = L.n;
    const int total = tiles * ((nfr + kf - 1) / kf);
    const int per_xcd = (total + 7) / 8;
    const int id = (int)(blockIdx.x % 8) * per_xcd + (int)(blockIdx.x / 8);
    if (id >= total) return;  // uniform
    const int fg = id / tiles, tile = id - fg * tiles;
    const int by = tile / gx, bx = tile - by * gx;
    const int f0 = fg * kf, f1 = min(f0 + kf, nfr);
    const float* M = L.inv;
    const float wlim = (float)(L.src.w - 1), hlim = (float)(L.src.h - 1);
    const int xl = bx * TW + lane;
    const int yw = by * TH + wave * NP;
    auto px_x = [&](int j) { return xl; };      // pixel j's column
    auto px_y = [&](int j) { return yw + j; };  // and row
    const uint32_t rp = (uint32_t)L.src.row_pitch;

    // ---- 1. per-pixel taps, once for every frame (warp_affine_naive.cpp:23-42)
    uint32_t sxy[NP], vwa[NP], okm = 0;
    int xmin = INT_MAX, xmax = INT_MIN, ymin = INT_MAX, ymax = INT_MIN;
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const int x = px_x(j), y = px_y(j);
        const float axm = M[0] * (float)x, aym = M[3] * (float)x;
        bool ok;
        int sx, sy;
        if constexpr (NN) {
            // warpAffine's AB_BITS = 10 fixed point, remap's short map (k_warp.hip)
            const double* Md = L.invd;
            const int X0 = (int)rint((Md[1] * y + Md[2]) * 1024.0) + 512;
            const int Y0 = (int)rint((Md[4] * y + Md[5]) * 1024.0) + 512;
            int X = (int)((uint32_t)X0 + (uint32_t)(int)rint(Md[0] * x * 1024.0)) >> 10;
            int Y = (int)((uint32_t)Y0 + (uint32_t)(int)rint(Md[3] * x * 1024.0)) >> 10;
            X = min(max(X, -32768), 32767);
            Y = min(max(Y, -32768), 32767);
            ok = (x < L.dst.w) & (y < L.dst.h) & ((unsigned)X < (unsigned)L.src.w) & ((unsigned)Y < (unsigned)L.src.h);
            sx = ok ? X : 0;
            sy = ok ? Y : 0;
            vwa[j] = 0;
        } else {
            const float fx = (axm + M[1] * (float)y) + M[2];
            const float fy = (aym + M[4] * (float)y) + M[5];
            ok = (x < L.dst.w) & (y < L.dst.h) & (fx >= 0.f) & (fx < wlim) & (fy >= 0.f) & (fy < hlim);
            sx = ok ? (int)fx : 0;
            sy = ok ? (int)fy : 0;
            const float ax = fx - (float)sx, ay = fy - (float)sy;
            const uint32_t w0 = (uint32_t)(int)((1.f - ay) * 2048.f + 0.5f);
            const uint32_t v0 = (uint32_t)(int)((1.f - ax) * 2048.f + 0.5f);
            vwa[j] = ok ? (v0 | ((4u * w0) << 16)) : (2048u | (8192u << 16));
        }
        sxy[j] = (uint32_t)sx | ((uint32_t)sy << 16);
        okm |= (uint32_t)ok << j;
        if (ok) {
            xmin = min(xmin, sx);
            xmax = max(xmax, sx);
            ymin = min(ymin, sy);
            ymax = max(ymax, sy);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        xmin = min(xmin, __shfl_xor(xmin, o, 64));
        xmax = max(xmax, __shfl_xor(xmax, o, 64));
        ymin = min(ymin, __shfl_xor(ymin, o, 64));
        ymax = max(ymax, __shfl_xor(ymax, o, 64));
    }
    if (lane == 0) {
        red[4 * wave + 0] = xmin;
        red[4 * wave + 1] = xmax;
        red[4 * wave + 2] = ymin;
        red[4 * wave + 3] = ymax;
    }
    // the image's 16-byte head: the border pixel (a pixel outside the source
    // reads its taps there, with weights (2048, 0) x (2048, 0))
    if (tid < 4) {
        uint32_t bp = 0;
#pragma unroll
        for (int e = 0; e < CC; ++e) bp |= (uint32_t)(int)L.border[e] << (8 * e);
        *reinterpret_cast<uint32_t*>(lds + ebase + 4 * tid) = bp;
    }
    if (tid < kExpRows) {
        t_min[tid] = INT_MAX;
        t_max[tid] = -1;
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        xmin = min(xmin, red[4 * w + 0]);
        xmax = max(xmax, red[4 * w + 1]);
        ymin = min(ymin, red[4 * w + 2]);
        ymax = max(ymax, red[4 * w + 3]);
    }
    xmin = __builtin_amdgcn_readfirstlane(xmin);
    xmax = __builtin_amdgcn_readfirstlane(xmax);
    ymin = __builtin_amdgcn_readfirstlane(ymin);
    ymax = __builtin_amdgcn_readfirstlane(ymax);
    const bool any = xmax >= 0;
    const int bx0 = any ? (xmin & ~3) : 0;                         // first staged column (bx0 * CC dword-aligned)
    const int wpx = any ? xmax + 2 - bx0 : 0;                      // pixels of a box row
    const int G = (wpx * CC + 15) >> 4;                            // 16-byte chunks of a box row
    const int R = any ? ymax + 2 - ymin : 0;                       // staged rows ymin .. ymax + 1
    const bool fits = any && R <= kExpRows;                        // uniform

    // ---- 2. row spans: the columns each staged row is tapped at, exactly --
    // an LDS min / max over the tile's pixels (bilinear: columns p, p + 1 of
    // rows r, r + 1; nearest: column p of row r); pixels plo .. phi (relative
    // to bx0), raw chunks glo .. ghi, image units plo/16 .. phi/16
    // Along an output row the taps are monotone in x (an affine map, floored
    // or OpenCV-rounded), so of each run of lanes tapping the same source row
    // only the run's two end lanes can hold its min and max: only they update
    // the table (every lane would serialise 64-way on one address at 0 deg).
    if (fits) {
#pragma unroll
        for (int j = 0; j < NP; ++j) {
            const bool ok = (okm >> j) & 1u;
            const uint32_t key = ok ? (sxy[j] >> 16) : 0xFFFFFFFFu;
            const uint32_t kl = (uint32_t)__shfl_up((int)key, 1, 64), kr = (uint32_t)__shfl_down((int)key, 1, 64);
            if (ok && (lane == 0 || lane == 63 || kl != key || kr != key)) {
                const int p = (int)(sxy[j] & 0xFFFFu) - bx0, r = (int)(sxy[j] >> 16) - ymin;
                atomicMin(&t_min[r], p);
                atomicMax(&t_max[r], NN ? p : p + 1);
                if constexpr (!NN) {
                    atomicMin(&t_min[r + 1], p);
                    atomicMax(&t_max[r + 1], p + 1);
                }
            }
        }
    }
    __syncthreads();
    if (fits && tid < R) {
        const int plo = t_min[tid], phi = t_max[tid];
        uint32_t sp = 0, un = 0, cnt = 0;
        if (plo <= phi) {
            const int glo = (plo * CC) >> 4, ghi = ((phi + 1) * CC - 1) >> 4;
            sp = (uint32_t)glo | ((uint32_t)ghi << 16);
            cnt = (uint32_t)(ghi - glo + 1);
            un = (uint32_t)(plo >> 4) | ((uint32_t)((phi >> 4) - (plo >> 4) + 1) << 16);
        }
        t_sp[tid] = sp;
        t_un[tid] = un;
        t_pre[tid] = cnt | (un & 0xFFFF0000u);  // counts, until the scan
    }
    __syncthreads();
    // prefix over the rows (wave 0, two rows per lane): chunk offsets RB and
    // unit offsets UP, both < 2^16 (packed and added together)
    if (fits && wave == 0) {
        const uint32_t a = lane < R ? t_pre[lane] : 0u, b = lane + 64 < R ? t_pre[lane + 64] : 0u;
        uint32_t ia = a, ib = b;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t va = __shfl_up(ia, o, 64), vb = __shfl_up(ib, o, 64);
            if (lane >= o) { ia += va; ib += vb; }
        }
        const uint32_t ta = __shfl(ia, 63, 64), tb = __shfl(ib, 63, 64);
        if (lane < R) t_pre[lane] = ia - a;
        if (lane + 64 < R) t_pre[lane + 64] = ta + ib - b;
        if (lane == 0) *t_tot = ta + tb;
    }
    __syncthreads();
    // the chunk -> row and unit -> row bytes
    const uint32_t tot = fits ? *t_tot : 0u;
    const int C = (int)(tot & 0xFFFFu), NU = (int)(tot >> 16);
    const int n_inst = (C + 63) >> 6;
    const bool staged = fits && n_inst <= 4 * kRingMaxIt && (n_inst << 10) <= slot_bytes && NU <= exp_units &&
                        NU <= kExpUnits;  // uniform
    if (staged && tid < R) {
        const uint32_t pre = t_pre[tid], un = t_un[tid];
        const int rb = (int)(pre & 0xFFFFu), up = (int)(pre >> 16);
        const int cnt = (tid + 1 < R ? (int)(t_pre[tid + 1] & 0xFFFFu) : C) - rb;
        for (int i = 0; i < cnt; ++i) t_crow[rb + i] = (unsigned char)tid;
        for (int i = 0; i < (int)(un >> 16); ++i) t_urow[up + i] = (unsigned char)tid;
    }
    __syncthreads();
    const int n_w = staged && n_inst > wave ? (n_inst - wave + 3) >> 2 : 0;

    // per pixel, for every frame: the LDS byte addresses of its top and
    // bottom tap pairs in the image (or the border head), the x-weight pair
    // and the row weight
    // (the two addresses as 16-bit halves of one register: LDS offsets are
    // < 64 KiB, and 8 registers fewer keep the kernel at 4 waves per SIMD)
    uint32_t eaTB[NP], wxp[NP], wa[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) {
        const bool ok = staged && ((okm >> j) & 1u);
        eaTB[j] = ebase | (ebase << 16);
        if (ok) {
            const int sx = (int)(sxy[j] & 0xFFFFu), r = (int)(sxy[j] >> 16) - ymin;
            const int p = sx - bx0;
            const uint32_t pt = t_pre[r], pb = t_pre[r + 1];
            const uint32_t ut = t_un[r], ub = t_un[r + 1];
            const uint32_t at = ebase + 4u * (uint32_t)(4 + 16 * ((int)(pt >> 16) - (int)(ut & 0xFFFFu)) + p);
            const uint32_t ab = ebase + 4u * (uint32_t)(4 + 16 * ((int)(pb >> 16) - (int)(ub & 0xFFFFu)) + p);
            eaTB[j] = at | (ab << 16);
        }
        const uint32_t v0 = vwa[j] & 0xFFFFu;
        wxp[j] = ((okm >> j) & 1u) ? (v0 | ((2048u - v0) << 16)) : 2048u;
        wa[j] = vwa[j] >> 16;
    }
    // this lane's DMA source offsets (frame-relative): instruction u of this
    // wave covers slot chunks 64 (wave + 4u) + lane.  vm: chunks to load;
    // tailm: those reaching past the plane's last byte (bytewise after the DMA)
    uint32_t goff[kRingMaxIt];
    uint32_t vm = 0, tailm = 0;
#pragma unroll
    for (int u = 0; u < kRingMaxIt; ++u) {
        goff[u] = 0;
        if (u < n_w) {
            const int c = 64 * (wave + 4 * u) + lane;
            if (c < C) {
                const int r = t_crow[c];
                const int col = (int)(t_sp[r] & 0xFFFFu) + c - (int)(t_pre[r] & 0xFFFFu);
                goff[u] = (uint32_t)(ymin + r) * rp + (uint32_t)(bx0 * CC + 16 * col);
                if ((int64_t)goff[u] + 16 > L.src.plane_bytes) tailm |= 1u << u;
                else vm |= 1u << u;
            }
        }
    }
    // this thread's re-lay quarter units c = tid + 256 q: the raw byte offset
    // of their 4 pixels in a slot (+ 48); their image bytes are 16 + 16 c
    uint32_t rl[kExpQ];
    int n_rl = 0;
#pragma unroll
    for (int q = 0; q < kExpQ; ++q) {
        const int c = tid + kBlock * q;
        rl[q] = 0;
        if (staged && c < 4 * NU) {
            const int r = t_urow[c >> 2];
            const uint32_t pre = t_pre[r];
            const int p = 16 * (int)(t_un[r] & 0xFFFFu) + 4 * (c - 4 * (int)(pre >> 16));  // first pixel
            rl[q] = (uint32_t)(48 + 16 * (int)(pre & 0xFFFFu) + 3 * p - 16 * (int)(t_sp[r] & 0xFFFFu));
            n_rl = q + 1;
        }
    }
    auto dma = [&](int f, int s) {
        const Rsrc rs = make_rsrc(L.src.base + (int64_t)f * L.src.img_pitch, L.src.plane_bytes);
        unsigned char* base = lds + 48 + s * slot_bytes + 1024 * wave;
#pragma unroll
        for (int u = 0; u < kRingMaxIt; ++u) {
            if (u < n_w) {
                const int off = ((vm >> u) & 1u) ? (int)(goff[u] + rs.delta) : (int)0x80000000;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs.r, (lds_void*)(base + 4096 * u), 16, off, 0, 0, kAux);
            }
        }
    };
    auto fix_tail = [&](int f, int s) {
        const Rsrc rs = make_rsrc(L.src.base + (int64_t)f * L.src.img_pitch, L.src.plane_bytes);
#pragma unroll
        for (int u = 0; u < kRingMaxIt; ++u) {
            if ((tailm >> u) & 1u) {
                uint32_t d[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    uint32_t w = 0;
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        w |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rs.r, (int)(goff[u] + rs.delta) + 4 * q + e,
                                                                           0, 0) << (8 * e);
                    d[q] = w;
                }
                const int c = 64 * (wave + 4 * u) + lane;
                *reinterpret_cast<u32x4*>(lds + 48 + s * slot_bytes + 16 * c) = u32x4{d[0], d[1], d[2], d[3]};
            }
        }
    };
    // slot s's raw 3-byte pixels -> the 4-byte image, 4 pixels (12 raw
    // bytes, dword-aligned: 3 p with p a multiple of 4) a quarter unit
    // All of a thread's reads are issued before its first write (one LDS
    // round trip per frame, not one per quarter unit: the per-unit branch
    // serialised them, ~800 of the wave's ~5,800 cycles per frame); a
    // quarter unit past the thread's count reads and rewrites the image's
    // border head (its own bytes, unchanged).
    auto relay = [&](int s) {
        const uint32_t sb = (uint32_t)(s * slot_bytes);
        uint32_t d[kExpQ][3];
#pragma unroll
        for (int q = 0; q < kExpQ; ++q) {
            const uint32_t* p = reinterpret_cast<const uint32_t*>(lds + (q < n_rl ? rl[q] + sb : ebase));
            d[q][0] = p[0];
            d[q][1] = p[1];
            d[q][2] = p[2];
        }
#pragma unroll
        for (int q = 0; q < kExpQ; ++q) {
            if (q < n_rl)
                *reinterpret_cast<u32x4*>(lds + ebase + 16u + 16u * (uint32_t)(tid + kBlock * q)) =
                    u32x4{d[q][0], __builtin_amdgcn_alignbyte(d[q][1], d[q][0], 3),
                          __builtin_amdgcn_alignbyte(d[q][2], d[q][1], 2), d[q][2] >> 8};
        }
    };

    const uint32_t dpitch = (uint32_t)L.dst.row_pitch;
    const bool tile_full = bx * TW + TW <= L.dst.w && by * TH + TH <= L.dst.h && dst_al;
    constexpr uint32_t kOob = 0x80000000u;
    // vector-memory stores per sampled frame (the wait counts; every one is
    // issued): full tiles one 12-byte store per 4 rows (u8) or one 16-byte
    // store per row (fp32); edge tiles count 0, so their waits also drain
    // the stores of the frames before (conservative)
    const int n_st = !tile_full ? 0 : OUT != kOutSame ? NP : NP / 4;

    // one pixel's channels from its 4 taps ([b g r x] each): the sum << 2, the
    // result in bits 24..31 (warp_affine_naive.cpp:50-54)
    auto blend3 = [&](int j, uint32_t tl, uint32_t tr, uint32_t bl, uint32_t br, uint32_t (&vv)[CC]) {
        const us2 wx = __builtin_bit_cast(us2, wxp[j]);
        const uint32_t wA = wa[j], wB = 8192u - wa[j];
#pragma unroll
        for (int k = 0; k < CC; ++k) {
            const uint32_t sel = (uint32_t)k | (0x0Cu << 8) | ((uint32_t)(4 + k) << 16) | (0x0Cu << 24);
            const uint32_t top = __builtin_amdgcn_perm(tr, tl, sel);
            const uint32_t bot = __builtin_amdgcn_perm(br, bl, sel);
            const uint32_t ht = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, top), wx, 0u, false);
            const uint32_t hb = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, bot), wx, 0u, false);
            vv[k] = __umul24(ht, wA) + __umul24(hb, wB);
        }
    };
    ChanNorm cn[CC];
    auto emit = [&](auto full_c, int f, int j, const uint32_t (&vv)[CC]) {
        constexpr bool FULL = decltype(full_c)::value;
        const int x = px_x(j), y = px_y(j);
        const bool inside = FULL || (x < L.dst.w && y < L.dst.h);
        unsigned char* dbase = const_cast<unsigned char*>(L.dst.base) + (int64_t)f * L.dst.img_pitch;
        const Rsrc drs = make_rsrc(dbase, L.dst.plane_bytes);
        if constexpr (OUT == kOutSame) {
            const uint32_t own = __builtin_amdgcn_perm(vv[2], __builtin_amdgcn_perm(vv[1], vv[0], 0x0C0C0703u), 0x0C070100u);
            if constexpr (FULL) {
                *reinterpret_cast<uint32_t*>(xch + 256 * (j & 3) + 4 * lane) = own;
                if ((j & 3) == 3) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    // 4 rows of 64 pixels; a lane stores 4 pixels, 12 bytes
                    const int r = lane >> 4, q = lane & 15;
                    const u32x4 p = *reinterpret_cast<const u32x4*>(xch + 256 * r + 16 * q);
                    typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
                    const u32x3 o = {__builtin_amdgcn_perm(p[1], p[0], 0x04020100u),
                                     __builtin_amdgcn_perm(p[2], p[1], 0x05040201u),
                                     __builtin_amdgcn_perm(p[3], p[2], 0x06050402u)};
                    const uint32_t off = (uint32_t)(y - 3 + r) * dpitch + drs.delta + (uint32_t)(bx * TW * CC + 12 * q);
                    __builtin_amdgcn_raw_buffer_store_b96(o, drs.r, (int)off, 0, VACV_STORE_AUX);
                }
            } else {
                const uint32_t off = (uint32_t)y * dpitch + drs.delta + (uint32_t)(x * CC);
#pragma unroll
                for (int k = 0; k < CC; ++k)
                    __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(own >> (8 * k)), drs.r,
                                                         (int)(inside ? off + k : kOob), 0, VACV_STORE_AUX);
            }
        } else {
            uint32_t o[CC];
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                const int v = (int)(vv[k] >> 24);
                const float fv = OUT == kOutF32 ? (float)v : normalize_u8v(cn[k], v);
                o[k] = __builtin_bit_cast(uint32_t, fv);
            }
            if constexpr (FULL) {
#pragma unroll
                for (int k = 0; k < CC; ++k) *reinterpret_cast<uint32_t*>(xch + 12 * lane + 4 * k) = o[k];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                const u32x4 p = *reinterpret_cast<const u32x4*>(xch + 16 * (lane % (3 * 16)));
                const uint32_t off = lane < 3 * 16 ? (uint32_t)y * dpitch + drs.delta +
                                                         (uint32_t)((x - lane) * CC * 4 + 16 * lane)
                                                   : kOob;
                __builtin_amdgcn_raw_buffer_store_b128(p, drs.r, (int)off, 0, VACV_STORE_AUX);
            } else {
                typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
                const uint32_t off = inside ? (uint32_t)y * dpitch + drs.delta + (uint32_t)(x * CC * 4) : kOob;
                __builtin_amdgcn_raw_buffer_store_b96(u32x3{o[0], o[1], o[2]}, drs.r, (int)off, 0, VACV_STORE_AUX);
            }
        }
    };
    // frame f from the image
    auto sample = [&](auto full_c, int fv) {
        const int f = __builtin_amdgcn_readfirstlane(fv);
        if constexpr (OUT != kOutSame) {
#pragma unroll
            for (int k = 0; k < CC; ++k) cn[k] = chan_norm(L.norm, f, k);
        }
        constexpr int kGrp = kExpGrp;
#pragma unroll
        for (int j0 = 0; j0 < NP; j0 += kGrp) {
            uint32_t tp[kGrp][4];
#pragma unroll
            for (int j = 0; j < kGrp; ++j) {
                const uint32_t e = eaTB[j0 + j];
                const uint32_t* pt = reinterpret_cast<const uint32_t*>(lds + (e & 0xFFFFu));
                const uint32_t* pb = reinterpret_cast<const uint32_t*>(lds + (e >> 16));
                tp[j][0] = pt[0];
                if constexpr (!NN) {
                    tp[j][1] = pt[1];
                    tp[j][2] = pb[0];
                    tp[j][3] = pb[1];
                }
            }
#pragma unroll
            for (int j = 0; j < kGrp; ++j) {
                uint32_t vv[CC];
                if constexpr (NN) {
                    // the tap's channel k in bits 24..31, as the blend leaves it
#pragma unroll
                    for (int q = 0; q < CC; ++q) vv[q] = tp[j][0] << (24 - 8 * q);
                } else {
                    blend3(j0 + j, tp[j][0], tp[j][1], tp[j][2], tp[j][3], vv);
                }
                emit(full_c, f, j0 + j, vv);
            }
        }
    };

    using full_t = std::integral_constant<bool, true>;
    using edge_t = std::integral_constant<bool, false>;
    if (!staged) {
        // no staging: a tile no pixel of which taps the source reads the
        // border head for every pixel (both addresses the head); a box over the
        // plan (never for a planned geometry: the host sized the slots for
        // every tile) takes its taps from memory
        for (int f = f0; f < f1; ++f) {
            if (!any) {
                if (tile_full) sample(full_t(), f);
                else sample(edge_t(), f);
                continue;
            }
            const unsigned char* sp = L.src.base + (int64_t)f * L.src.img_pitch;
            if constexpr (OUT != kOutSame) {
#pragma unroll
                for (int k = 0; k < CC; ++k) cn[k] = chan_norm(L.norm, f, k);
            }
            for (int j = 0; j < NP; ++j) {
                uint32_t vv[CC];
                if constexpr (NN) {
                    uint32_t tl = 0;
#pragma unroll
                    for (int q = 0; q < CC; ++q) tl |= (uint32_t)(int)L.border[q] << (8 * q);
                    if ((okm >> j) & 1u) {
                        const int sx = (int)(sxy[j] & 0xFFFFu), sy = (int)(sxy[j] >> 16);
                        tl = pack_bytes<CC>(sp + (int64_t)sy * L.src.row_pitch + (int64_t)sx * CC);
                    }
#pragma unroll
                    for (int q = 0; q < CC; ++q) vv[q] = tl << (24 - 8 * q);
                } else {
                    uint32_t tl, tr, bl, br;
                    direct_taps<CC>(L, sp, px_x(j), px_y(j), tl, tr, bl, br);
                    blend3(j, tl, tr, bl, br, vv);
                }
                emit(edge_t(), f, j, vv);
            }
        }
        return;
    }
    // prologue: frames f0 and f0 + 1 in flight
    dma(f0, 0);
    if (f0 + 1 < f1) dma(f0 + 1, 1);
    for (int f = f0; f < f1; ++f) {
        const int s = (f - f0) & 1;
        // this wave's DMA of frame f has landed; issued after it and possibly
        // still in flight: frame f + 1's DMA and the stores of the (up to 2)
        // frames sampled since
        wait_vm((f + 1 < f1 ? n_w : 0) + min(f - f0, 2) * n_st);
        if (tailm) {
            fix_tail(f, s);
            wait_lgkm();  // its LDS stores land before the barrier (s_barrier does not wait for them)
        }
        __builtin_amdgcn_s_barrier();  // every wave's part of frame f is in; frame f - 1's image reads are done
        relay(s);
        wait_lgkm();
        __builtin_amdgcn_s_barrier();  // the image holds frame f; slot s is free
        if (f + 2 < f1) dma(f + 2, s);
        if (tile_full) sample(full_t(), f);
        else sample(edge_t(), f);
    }
    wait_vm(0);  // no LDS-DMA may outlive the workgroup's LDS
}

template <typename K>
int64_t frames_resident(K kernel, size_t lds) {
    static std::mutex mu;
    static std::map<std::pair<const void*, size_t>, int64_t> cache;  // (kernel, lds) -> workgroups, device 0 shape
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(reinterpret_cast<const void*>(kernel), lds);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int per_cu = 0, cus = 0, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, lds) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 0;
    const int64_t r = (int64_t)std::max(per_cu, 1) * std::max(cus, 1);
    cache.emplace(key, r);
    return r;
}

template <int OUT, int NP, bool NN = false>
hipError_t launch_exp(const WarpLaunch& L, const WarpFramesPlan& P, hipStream_t s) {
    constexpr int TW = kFrTileW, TH = 4 * NP;
    const int gx = (L.dst.w + TW - 1) / TW, gy = (L.dst.h + TH - 1) / TH;
    auto kern = warp_exp_kernel<OUT, NP, NN>;
    int kf = P.kf;
    if (kf <= 0) {
        const int64_t res = std::max<int64_t>(frames_resident(kern, (size_t)P.lds), 256);
        const int64_t tiles = (int64_t)gx * gy;
        kf = (int)std::max<int64_t>(1, std::min<int64_t>(16, tiles * L.n / (3 * res)));
    }
    const int64_t total = (int64_t)gx * gy * ((L.n + kf - 1) / kf);
    if (total >= 0x7FFFFFF0LL) return hipErrorInvalidValue;
    const int64_t blocks = (total + 7) / 8 * 8;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kBlock), (size_t)P.lds, s, L, gx, gy, kf, P.raw_bytes,
                       P.exp_units, P.dst_al);
    return hipGetLastError();
}

template <int CC, int OUT, int NP, bool PLANAR>
hipError_t launch_frames(const WarpLaunch& L, const WarpFramesPlan& P, hipStream_t s) {
    constexpr int TH = 4 * NP;
    const int gx = (L.dst.w + kFrTileW - 1) / kFrTileW, gy = (L.dst.h + TH - 1) / TH;
    auto kern = warp_ring_kernel<CC, OUT, NP, PLANAR>;
    int kf = P.kf;
    if (kf <= 0) {
        // at most 16 frames per workgroup (the per-tile taps, box and spans
        // amortised over more frames: 720p rot15 8 / 16 / 32 frames 0.183 /
        // 0.175 / 0.185 ms), fewer when that leaves < ~3 rounds of residency
        const int64_t res = std::max<int64_t>(frames_resident(kern, (size_t)P.lds), 256);
        const int64_t tiles = (int64_t)gx * gy;
        kf = (int)std::max<int64_t>(1, std::min<int64_t>(16, tiles * L.n * L.src.planes / (3 * res)));
    }
    const int64_t total = (int64_t)gx * gy * ((L.n * L.src.planes + kf - 1) / kf);
    if (total >= 0x7FFFFFF0LL) return hipErrorInvalidValue;
    const int64_t blocks = (total + 7) / 8 * 8;
    const uint32_t gs = (uint32_t)(P.S / 16), ginv = ((1u << 20) + gs - 1) / gs;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kBlock), (size_t)P.lds, s, L, gx, gy, kf, P.S, P.rows_max,
                       P.ns, P.slot, P.dst_al, ginv);
    return hipGetLastError();
}

template <int CC, int OUT>
hipError_t launch_frames_np(const WarpLaunch& L, const WarpFramesPlan& P, hipStream_t s) {
    if (CC == 1 && L.src.planes > 1)
        return P.th == 16 ? launch_frames<CC, OUT, 4, true>(L, P, s) : launch_frames<CC, OUT, 8, true>(L, P, s);
    return P.th == 16 ? launch_frames<CC, OUT, 4, false>(L, P, s) : launch_frames<CC, OUT, 8, false>(L, P, s);
}

template <int OUT>
hipError_t launch_frames_cc(const WarpLaunch& L, const WarpFramesPlan& P, hipStream_t s) {
    if (P.se > 0) {
        return P.th == 16 ? launch_exp<OUT, 4>(L, P, s) : launch_exp<OUT, 8>(L, P, s);
    }
    switch (L.src.cc) {
        case 1: return launch_frames_np<1, OUT>(L, P, s);
        case 2: return launch_frames_np<2, OUT>(L, P, s);
        case 3: return launch_frames_np<3, OUT>(L, P, s);
        default: return launch_frames_np<4, OUT>(L, P, s);
    }
}

}  // namespace

// The LDS row stride (bytes, a multiple of 16, >= 16 G) with the fewest LDS
// bank conflicts for the tap reads.  A wave's 64 lanes read the taps of 64
// consecutive output pixels of one row; rotated, they fall on several staged
// rows, and the stride decides whether those rows' dwords land on distinct
// banks.  Per tap row a pixel reads the 2 (3 for CC = 3) dwords from byte
// address 16 + row S + col CC rounded down, each a ds_read_b32 (bank = dword
// mod 32 within each half-wave; distinct dwords on one bank serialise).
// Counted on a few sample rows of the output for the 8 strides 16 G ..
// 16 G + 112 (those <= s_max); ties go to the smaller stride.
int ring_stride(const WarpLaunch& L, int G, int s_max) {
    const float* M = L.inv;
    const int CC = L.src.cc;
    int best_s = 16 * G;
    long best_cost = -1;
    for (int k = 0; k < 8; ++k) {
        const int S = 16 * (G + k);
        if (k > 0 && S > s_max) break;
        long cost = 0;
        for (int yi = 1; yi <= 3; ++yi) {
            const int y = L.dst.h * yi / 4;
            for (int xi = 0; xi < 3; ++xi) {
                const int x0 = std::max(0, std::min(L.dst.w - 64, (L.dst.w - 64) * xi / 2));
                for (int half = 0; half < 2; ++half) {
                    long a0[32];
                    for (int l = 0; l < 32; ++l) {
                        const int x = x0 + 32 * half + l;
                        const float fx = (M[0] * (float)x + M[1] * (float)y) + M[2];
                        const float fy = (M[3] * (float)x + M[4] * (float)y) + M[5];
                        long a = 0;  // outside: the slot's border head
                        if (fx >= 0.f && fx < (float)(L.src.w - 1) && fy >= 0.f && fy < (float)(L.src.h - 1))
                            a = 16 + (long)(int)fy * S + (long)(int)fx * CC;
                        a0[l] = a >> 2;
                    }
                    for (int q = 0; q < (CC == 3 ? 3 : 2); ++q) {  // one ds_read_b32 per covering dword
                        int worst = 1;
                        for (int l = 0; l < 32; ++l) {  // distinct dwords on lane l's bank
                            int n = 0;
                            for (int m = 0; m < 32; ++m) {
                                if (((a0[m] - a0[l]) & 31) != 0) continue;
                                bool first = true;
                                for (int t = 0; t < m; ++t) first = first && a0[t] != a0[m];
                                n += first;
                            }
                            worst = std::max(worst, n);
                        }
                        cost += worst;
                    }
                }
            }
        }
        if (best_cost < 0 || cost < best_cost) {
            best_cost = cost;
            best_s = S;
        }
    }
    return best_s;
}

// The LDS layout of one geometry (pointer-independent).  The box bound is the
// tile's coordinate span (|m0|*63 + |m1|*(TH-1) columns, |m3|*63 +
// |m4|*(TH-1) rows) plus floor, the second tap, 4-alignment and slack; the
// kernel re-checks the real box and reads memory if it is larger.  Raw pixel
// rows of G 16-byte chunks; ns slots, each a 16-byte border head and whole
// 1 KiB DMA instructions.  ns (2-4, VACV_TUNE_WARP_SLOTS) defaults to 2:
// occupancy beats depth (720p rot15: 2 / 3 / 4 slots 0.159 / 0.183 / 0.29 ms,
// 5 / 3 / 2 workgroups per CU).
bool ring_layout_th(const WarpLaunch& L, WarpFramesPlan& P, int th) {
    P.th = th;
    const int CC = L.src.cc;
    const double sx = std::fabs(L.inv[0]) * (kFrTileW - 1) + std::fabs(L.inv[1]) * (P.th - 1);
    const double sy = std::fabs(L.inv[3]) * (kFrTileW - 1) + std::fabs(L.inv[4]) * (P.th - 1);
    const int W = (int)std::ceil(sx * (1 + 1e-5) + 1e-3) + 6;  // + floor spread, right tap, 4-alignment
    const int G = (W * CC + 15) / 16;
    P.rows_max = (int)std::ceil(sy * (1 + 1e-5) + 1e-3) + 3;
    const int extra = 64 + (L.out == kOutSame ? 4 * 2 * 64 * CC : 0);
    auto slot_of = [&](int S) { return 16 + (P.rows_max * (S / 16) + 63) / 64 * 1024; };
    if ((P.rows_max * G + 63) / 64 > 4 * kRingMaxIt) return false;
    const int knob = tune(VACV_TUNE_WARP_SLOTS);
    P.ns = knob >= 2 && knob <= 4 ? knob : 2;
    if (P.ns * slot_of(16 * G) + extra > 64 * 1024) return false;
    // strides that keep the same resident workgroups per CU
    const int per_cu = 160 * 1024 / (P.ns * slot_of(16 * G) + extra);
    int s_max = 16 * G;
    for (int S = 16 * G; S <= 16 * (G + 7); S += 16)
        if (160 * 1024 / (P.ns * slot_of(S) + extra) >= per_cu && (P.rows_max * (S / 16) + 63) / 64 <= 4 * kRingMaxIt)
            s_max = S;
    P.S = ring_stride(L, G, s_max);
    P.slot = slot_of(P.S);
    P.lds = P.ns * P.slot + extra;
    return P.lds <= 64 * 1024;
}

// warp_exp_kernel's staging needs, bounded analytically per tile: the most
// span chunks, image units and box rows any tile can need.  A tile's pixels
// map to a parallelogram in the source; clipped to the valid tap region, its
// y extent gives the box rows, and its intersection with each row's band
// (sy in [r - 1, r + 1) bilinear, [r, r + 1) nearest) the row's tapped
// columns.  Every edge is widened by eps = 1/256 pixel, more than the
// kernel's float (and INTER_NEAREST's 1/1024 fixed-point) coordinate error,
// so the bound is never below the kernel's exact per-tile needs; the slots
// and the image are sized from it, so no tile takes the kernel's unstaged
// path.  Round 5 evaluated every pixel's tap twice per tile size tried (15-35
// ms of host time per new matrix at 720p); this is ~1 ms, and against that
// exact count over 300 random affine maps (1,200 cases) it never fell below
// and over-counted cfg4's chunks by < 1 % (551 -> 556, the same 9 DMA
// instructions).
struct ExpNeeds {
    int rows = 0, chunks = 0, units = 0;
};
struct Pt2 {
    double x, y;
};
// a convex polygon clipped to a*x + b*y <= c (Sutherland-Hodgman, one edge)
int clip_poly(const Pt2* in, int n, double a, double b, double c, Pt2* out) {
    int m = 0;
    for (int i = 0; i < n; ++i) {
        const Pt2 p = in[i], q = in[(i + 1) % n];
        const double dp = a * p.x + b * p.y - c, dq = a * q.x + b * q.y - c;
        if (dp <= 0) out[m++] = p;
        if ((dp < 0 && dq > 0) || (dp > 0 && dq < 0)) {
            const double t = dp / (dp - dq);
            out[m++] = {p.x + t * (q.x - p.x), p.y + t * (q.y - p.y)};
        }
    }
    return m;
}
ExpNeeds exp_needs(const WarpLaunch& L, int th, bool nn, int tw = kFrTileW) {
    constexpr int CC = 3;
    double M[6];  // bilinear: the kernel's float map; nearest: OpenCV's fp64 one
    for (int i = 0; i < 6; ++i) M[i] = nn ? L.invd[i] : (double)L.inv[i];
    const double eps = 1.0 / 256, sh = nn ? 0.5 : 0.0;  // nearest: sx = floor(fx + 0.5)
    const double wl = nn ? L.src.w : L.src.w - 1, hl = nn ? L.src.h : L.src.h - 1;
    const int smax = nn ? L.src.w - 1 : L.src.w - 2, ymaxc = nn ? L.src.h - 1 : L.src.h - 2;
    const int gx = (L.dst.w + tw - 1) / tw, gy = (L.dst.h + th - 1) / th;
    ExpNeeds n;
    for (int by = 0; by < gy; ++by)
        for (int bx = 0; bx < gx; ++bx) {
            const int x0 = bx * tw, y0 = by * th, x1 = std::min(x0 + tw, L.dst.w) - 1, y1 = std::min(y0 + th, L.dst.h) - 1;
            auto at = [&](int x, int y) { return Pt2{M[0] * x + M[1] * y + M[2] + sh, M[3] * x + M[4] * y + M[5] + sh}; };
            Pt2 a[12], b[12];
            a[0] = at(x0, y0);
            a[1] = at(x1, y0);
            a[2] = at(x1, y1);
            a[3] = at(x0, y1);
            int k = clip_poly(a, 4, -1, 0, eps, b);  // x >= -eps
            k = clip_poly(b, k, 1, 0, wl + eps, a);  // x <= wl + eps
            k = clip_poly(a, k, 0, -1, eps, b);      // y >= -eps
            k = clip_poly(b, k, 0, 1, hl + eps, a);  // y <= hl + eps
            if (k == 0) continue;
            double lx = 1e30, ly = 1e30, hy = -1e30;
            for (int i = 0; i < k; ++i) {
                lx = std::min(lx, a[i].x);
                ly = std::min(ly, a[i].y);
                hy = std::max(hy, a[i].y);
            }
            const int ylo = std::max((int)std::floor(ly - eps), 0), yhi = std::min((int)std::floor(hy + eps), ymaxc);
            if (yhi < ylo) continue;
            const int xlo = std::max((int)std::floor(lx - eps), 0), bx0 = xlo & ~3, R = yhi + 2 - ylo;
            int chunks = 0, units = 0;
            for (int t = 0; t < R; ++t) {
                const int r = ylo + t;
                Pt2 c[12], d[12];
                int m = clip_poly(a, k, 0, -1, -((nn ? r : r - 1) - eps), c);
                m = clip_poly(c, m, 0, 1, r + 1 + eps, d);
                if (m == 0) continue;
                double qx = 1e30, Qx = -1e30;
                for (int i = 0; i < m; ++i) {
                    qx = std::min(qx, d[i].x);
                    Qx = std::max(Qx, d[i].x);
                }
                const int s0 = std::max((int)std::floor(qx - eps), xlo), s1 = std::min((int)std::floor(Qx + eps), smax);
                if (s1 < s0) continue;
                const int pmin = s0 - bx0, pmax = s1 - bx0 + (nn ? 0 : 1);
                chunks += (((pmax + 1) * CC - 1) >> 4) - ((pmin * CC) >> 4) + 1;
                units += (pmax >> 4) - (pmin >> 4) + 1;
            }
            n.rows = std::max(n.rows, R);
            n.chunks = std::max(n.chunks, chunks);
            n.units = std::max(n.units, units);
        }
    return n;
}

// warp_exp_kernel's LDS: two compact raw slots, the image (at least the setup
// tables), the output exchange; <= 40 KiB keeps 4 workgroups per CU
bool exp_layout_th(const WarpLaunch& L, WarpFramesPlan& P, int th, bool nn = false, int tw = kFrTileW) {
    const ExpNeeds n = exp_needs(L, th, nn, tw);
    const int n_inst = (n.chunks + 63) / 64;
    if (n.rows > kExpRows || n_inst > 4 * kRingMaxIt || n.units > kExpUnits) return false;
    P.th = th;
    P.tw = tw;
    P.se = 1;
    P.raw_bytes = std::max(n_inst, 1) * 1024;
    P.exp_units = n.units;
    P.rows_max = n.rows;
    P.S = 0;
    P.ns = 2;
    P.slot = P.raw_bytes;
    const int xb = 4 * kExpXB(L.out == kOutSame ? kOutSame : kOutF32);
    P.lds = 48 + 2 * P.raw_bytes + 64 + 16 + 64 * std::max(n.units, (kExpTab + 63) / 64) + xb;
    return P.lds <= 64 * 1024;
}

// 32-row tiles (measured faster: 0.171 vs 0.182 ms at 720p rot15) unless
// their box is over the staging budget, then 16.  Interleaved 3-channel u8
// takes warp_exp_kernel where its image fits (VACV_TUNE_WARP_KERNEL = 6:
// the ring kernel instead).
bool frames_layout(const WarpLaunch& L, WarpFramesPlan& P) {
    const int th_knob = tune(VACV_TUNE_WARP_TILE_H);
    P.se = 0;
    P.raw_bytes = 0;
    P.tw = kFrTileW;
    if (L.src.cc == 3 && L.src.planes == 1 && tune(VACV_TUNE_WARP_KERNEL) != 6) {
        WarpFramesPlan Q = P;
        // 32-row tiles (fp32 output too: 0.4155 vs 0.4398 ms normalised at
        // 720p rot15 x128, although its instance spills a few registers)
        const int th0 = 32;
        if (th_knob == 16 || th_knob == 32) {
            if (exp_layout_th(L, Q, th_knob)) { P = Q; return true; }
        } else if (exp_layout_th(L, Q, th0) || exp_layout_th(L, Q, 48 - th0)) {
            P = Q;
            return true;
        }
        P.se = 0;
        P.raw_bytes = 0;
    }
    if (th_knob == 16 || th_knob == 32) return ring_layout_th(L, P, th_knob);
    return ring_layout_th(L, P, 32) || ring_layout_th(L, P, 16);
}

// Host plan: does the frames kernel apply, and with which LDS layout?
// Layouts are cached per geometry (the stride search costs ~0.1 ms of host
// time); the alignment checks are per call.
bool warp_frames_plan(const WarpLaunch& L, WarpFramesPlan& P) {
    const int knob = tune(VACV_TUNE_WARP_KERNEL);
    if (knob >= 0 && knob != 4 && knob != 6) return false;
    if (L.src.esize != 1 || L.border_mode != kBorderConstant) return false;
    if (L.src.planes > 1 && L.src.cc != 1) return false;
    if (L.src.cc < 1 || L.src.cc > 4) return false;
    if (L.src.plane_bytes > kMaxPlaneBytes || L.dst.plane_bytes > kMaxPlaneBytes) return false;
    const auto al4 = [](const PlaneGeom& g) {
        return !(g.row_pitch % 4 || g.img_pitch % 4 || g.plane_pitch % 4 || reinterpret_cast<uintptr_t>(g.base) % 4);
    };
    if (!al4(L.src)) return false;
    if (L.out != kOutSame && !al4(L.dst)) return false;  // float stores
    for (int i = 0; i < 6; ++i)
        if (!std::isfinite(L.inv[i])) return false;
    // everything frames_layout reads: the matrix, the sizes, the tile-height
    // knob, the channel count and whether the output is bytes (the LDS
    // layout of byte output carries the store exchange)
    struct Key {
        float inv[6];
        int sw, sh, dw, dh, th, cc, bytes_out, slots, kernel;
        bool operator<(const Key& o) const { return std::memcmp(this, &o, sizeof(Key)) < 0; }
    };
    Key k;
    std::memset(&k, 0, sizeof(k));
    std::memcpy(k.inv, L.inv, sizeof(k.inv));
    k.sw = L.src.w; k.sh = L.src.h; k.dw = L.dst.w; k.dh = L.dst.h; k.th = tune(VACV_TUNE_WARP_TILE_H);
    k.cc = L.src.cc;
    k.bytes_out = L.out == kOutSame ? 1 : 0;
    k.slots = tune(VACV_TUNE_WARP_SLOTS);
    k.kernel = knob;
    static std::mutex mu;
    static std::map<Key, std::pair<bool, WarpFramesPlan>> cache;
    bool ok;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find(k);
        if (it == cache.end()) {
            WarpFramesPlan Q{};
            const bool r = frames_layout(L, Q);
            if (cache.size() > 256) cache.clear();
            it = cache.emplace(k, std::make_pair(r, Q)).first;
        }
        ok = it->second.first;
        P = it->second.second;
    }
    P.dst_al = al4(L.dst) ? 1 : 0;
    P.kf = tune(VACV_TUNE_WARP_FRAMES);
    return ok;
}

// INTER_NEAREST on warp_exp_kernel: 3-channel u8 NHWC, BORDER_CONSTANT,
// 4-byte aligned destination rows (VACV_TUNE_WARP_KERNEL = 5 keeps the
// gather kernels).  Layouts cached per geometry, as warp_frames_plan.
bool warp_exp_nn_plan(const WarpLaunch& L, WarpFramesPlan& P) {
    if (tune(VACV_TUNE_WARP_KERNEL) == 5) return false;
    if (L.src.esize != 1 || L.src.cc != 3 || L.src.planes != 1 || L.border_mode != kBorderConstant) return false;
    if (L.src.plane_bytes > kMaxPlaneBytes || L.dst.plane_bytes > kMaxPlaneBytes) return false;
    const auto al4 = [](const PlaneGeom& g) {
        return !(g.row_pitch % 4 || g.img_pitch % 4 || g.plane_pitch % 4 || reinterpret_cast<uintptr_t>(g.base) % 4);
    };
    if (!al4(L.src) || !al4(L.dst)) return false;
    for (int i = 0; i < 6; ++i)
        if (!std::isfinite(L.inv[i]) || !std::isfinite(L.invd[i])) return false;
    struct Key {
        double invd[6];
        float inv[6];
        int sw, sh, dw, dh, th, bytes_out;
        bool operator<(const Key& o) const { return std::memcmp(this, &o, sizeof(Key)) < 0; }
    };
    Key k;
    std::memset(&k, 0, sizeof(k));
    std::memcpy(k.invd, L.invd, sizeof(k.invd));
    std::memcpy(k.inv, L.inv, sizeof(k.inv));
    k.sw = L.src.w; k.sh = L.src.h; k.dw = L.dst.w; k.dh = L.dst.h; k.th = tune(VACV_TUNE_WARP_TILE_H);
    k.bytes_out = L.out == kOutSame ? 1 : 0;
    static std::mutex mu;
    static std::map<Key, std::pair<bool, WarpFramesPlan>> cache;
    bool ok;
    {
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find(k);
        if (it == cache.end()) {
            WarpFramesPlan Q{};
            const int th0 = 32;
            const bool r = (k.th == 16 || k.th == 32) ? exp_layout_th(L, Q, k.th, true)
                                                      : exp_layout_th(L, Q, th0, true) || exp_layout_th(L, Q, 48 - th0, true);
            if (cache.size() > 256) cache.clear();
            it = cache.emplace(k, std::make_pair(r, Q)).first;
        }
        ok = it->second.first;
        P = it->second.second;
    }
    P.dst_al = 1;
    P.kf = tune(VACV_TUNE_WARP_FRAMES);
    return ok;
}

hipError_t launch_warp_exp_nn(const WarpLaunch& L, const WarpFramesPlan& P, hipStream_t s) {
    if (L.out == kOutSame) return P.th == 16 ? launch_exp<kOutSame, 4, true>(L, P, s) : launch_exp<kOutSame, 8, true>(L, P, s);
    if (L.out == kOutF32) return P.th == 16 ? launch_exp<kOutF32, 4, true>(L, P, s) : launch_exp<kOutF32, 8, true>(L, P, s);
    return P.th == 16 ? launch_exp<kOutNorm, 4, true>(L, P, s) : launch_exp<kOutNorm, 8, true>(L, P, s);
}

hipError_t launch_warp_frames(const WarpLaunch& L, const WarpFramesPlan& P, hipStream_t s) {
    if (L.out == kOutSame) return launch_frames_cc<kOutSame>(L, P, s);
    if (L.out == kOutF32) return launch_frames_cc<kOutF32>(L, P, s);
    return launch_frames_cc<kOutNorm>(L, P, s);
}

}  // namespace vacv
