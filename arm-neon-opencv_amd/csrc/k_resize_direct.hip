// k_resize_direct.hip -- u8 bilinear resize (all three fixed-point modes)
// with u8 / fp32 / normalised-fp32 output, as per-pixel gathers straight from
// HBM/L2: no LDS staging of source rows, no planner tables, no barriers.
//
// Reference arithmetic (the same as resize_kernel<kLinearFixed>, k_resize.hip):
//   taps  fixed_tap() = resize_naive.cpp:19-45 (REFERENCE), resize_neon.cpp:
//         17-78 (NEON, OPENCV half-even), shared host/device code
//   blend resize_naive.cpp:61-64  (Sum S*wx*wy) >> 22        (REFERENCE)
//         resize_neon.cpp:103-167 int16 rows, (h*w >> 16) + 2 >> 2 (NEON/OPENCV)
//   epilogue u8 -> fp32 and normalize_naive.cpp:74-90 (resize_normalize.cpp:
//         33-107 = resize, convertTo fp32, (x - mean) / (std + 1e-6))
//
// Shape.  Output pixels of one plane are numbered row-major; a wave owns PXL*64
// consecutive pixels -- rows are crossed freely, so every wave is full
// whatever the output width.  Lane l samples pixels p0 + 64q + l: each gather
// instruction reads 64 consecutive output pixels' taps (one contiguous run of
// a source row, ~9 bytes apart at a 3x downscale).  Per pixel and weighted tap
// row ONE unaligned 8-byte buffer load (load_taps, vacv_device.hpp) brings
// both horizontal taps of all CC <= 4 channels.  A row with a zero vertical weight is never read: when no
// output row has two weighted taps (ONE_ROW: the host checks, e.g. an exact
// 3x downscale) a pixel gathers one row only and the lane takes 8 pixels, so
// a CU keeps twice the bytes in flight for the same registers.  Outputs are
// re-assembled in LDS, 256 pixels at a time, and leave as 16-byte
// non-temporal stores: one store instruction writes 1 KiB of contiguous output.
#pragma clang fp contract(off)

#include <cmath>
#include <cstdlib>

#include "vacv_device.hpp"


namespace vacv {
namespace {

constexpr int kGroupPx = 256;  // pixels per LDS exchange round (4 per lane)

// cache policy of the fp32-output stores and tap gathers (aux bits:
// 1 sc0, 2 nt, 16 sc1)
constexpr int kDirectSaux = VACV_STORE_AUX;
constexpr int kDirectLaux = 0;
// resize_cols_kernel's fp32-output gathers at CW = 2 on 3 channels: non-temporal (round 5) -- its
// blocks end on 128-byte lines (CW = 2 / the edge-lane shift), no source line
// is read by two waves, so nothing is gained by keeping lines in L2
// (kbench 0.2092 -> 0.2075 ms, bench kernel 0.2127 / 0.2122 -> 0.2107 / 0.2095)
constexpr int kColsLaux = 2;

// Pixels per lane: 8 when one tap row is gathered and the kernel still fits
// 64 VGPRs (8 waves per SIMD) at 8, else 4 (measured: spills otherwise).
constexpr int direct_pxl(int cc, int out, bool one_row) {
    return one_row && (cc < 4 || out == kOutSame) ? 8 : 4;
}

template <int CC, int OUT, int MODE, bool ONE_ROW>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8)))
resize_direct_kernel(ResizeLaunch L, int blocks_per_plane, int total, int xcd) {
    using TOut = typename std::conditional<(OUT == kOutSame), uint8_t, float>::type;
    // pixels per lane (4-channel fp32 output at 8 would spill under 64 VGPRs)
    constexpr int PXL = direct_pxl(CC, OUT, ONE_ROW);
    constexpr int NR = ONE_ROW ? 1 : 2;                // gathered rows per pixel
    constexpr int kWavePx = 64 * PXL;
    constexpr int kOutPx = CC * (int)sizeof(TOut);    // output bytes per pixel
    // tap gathers: the default cache policy under fp32 output, so a 128-byte
    // source line split between two waves is re-read from L2, not HBM
    // (headline 0.2206 -> 0.2180 ms; sc0 0.2185); non-temporal under byte
    // output, where the default policy measured slower (0.1232 -> 0.1267 ms)
    constexpr int kLoadAux = OUT == kOutSame ? VACV_LOAD_AUX : kDirectLaux;
    constexpr int kStoreAux = OUT == kOutSame ? VACV_STORE_AUX : kDirectSaux;
    __shared__ __attribute__((aligned(16))) unsigned char xch[4][kGroupPx * kOutPx];

    // xcd: workgroup b runs on XCD b % 8; give each XCD one contiguous eighth
    // of the work so source rows shared by neighbouring workgroups (two-tap
    // rows) are fetched into one L2 only
    const int per_xcd = (total + 7) >> 3;
    const int id = xcd ? (int)(blockIdx.x & 7) * per_xcd + (int)(blockIdx.x >> 3) : (int)blockIdx.x;
    if (id >= total) return;  // uniform
    const int pidx = id / blocks_per_plane;  // image * planes + plane
    const int blk = id - pidx * blocks_per_plane;
    const int W = L.dst.w;
    const int P = W * L.dst.h;                            // output pixels per plane
    const int p0 = (blk * 4 + (int)threadIdx.y) * kWavePx;
    if (p0 >= P) return;  // whole wave
    const int npx = min(kWavePx, P - p0);
    const int lane = threadIdx.x;
    const int img = pidx / L.src.planes;
    const int plane = pidx - img * L.src.planes;

    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
    const Rsrc srs = make_rsrc(sp, L.src.plane_bytes);
    const uint32_t slimit = (uint32_t)L.src.plane_bytes + srs.delta;
    const int64_t rp = L.src.row_pitch;
    const uint32_t rp32 = (uint32_t)rp;  // plane_bytes < 2^31 (kMaxPlaneBytes): every row offset fits

    // ---- taps and gathers: every load of the lane issued before any blend ---
    const int y_first = p0 / W;  // wave-uniform
    const int x_first = p0 - y_first * W;
    uint32_t tap[PXL][NR][2];    // the 8 bytes at each gathered tap row
    uint32_t wxp[PXL], wyp[PXL]; // {a0, a1} and {wA, wB} as u16 pairs
    // vertical taps: a wave of an output at least kWavePx wide touches at most
    // two rows, whose taps are computed once (uniform); narrower outputs
    // compute them per pixel
    const bool wide = W >= kWavePx;
    const FixedTap ty0 = tap_of<MODE>(y_first, L.src.h, L.dst.h, L.scale_yf, L.scale_yd);
    const FixedTap ty1 = tap_of<MODE>(min(y_first + 1, L.dst.h - 1), L.src.h, L.dst.h, L.scale_yf, L.scale_yd);
#pragma unroll
    for (int q = 0; q < PXL; ++q) {
        const int d = x_first + q * 64 + lane;  // < W + kWavePx
        const int dy = wide ? (d >= W ? 1 : 0) : d / W;
        const int y = y_first + dy;
        const int x = d - dy * W;
#pragma unroll
        for (int r = 0; r < NR; ++r) tap[q][r][0] = tap[q][r][1] = 0u;
        wxp[q] = wyp[q] = 0u;
        if (q * 64 + lane >= npx) continue;
        const FixedTap tx = tap_of<MODE>(x, L.src.w, W, L.scale_xf, L.scale_xd);
        FixedTap ty;
        if (wide) {
            ty.i = dy ? ty1.i : ty0.i;
            ty.w0 = dy ? ty1.w0 : ty0.w0;
            ty.w1 = dy ? ty1.w1 : ty0.w1;
        } else {
            ty = tap_of<MODE>(y, L.src.h, L.dst.h, L.scale_yf, L.scale_yd);
        }
        if (ONE_ROW && ty.w0 == 0) { ty.i += 1; ty.w0 = ty.w1; ty.w1 = 0; }  // the weighted row as row A
        wxp[q] = (uint32_t)tx.w0 | ((uint32_t)tx.w1 << 16);
        wyp[q] = (uint32_t)ty.w0 | ((uint32_t)ty.w1 << 16);
        const uint32_t oa = (uint32_t)ty.i * rp32 + (uint32_t)(tx.i * CC) + srs.delta;
        const uint32_t ob = oa + rp32;
        if ((ONE_ROW ? oa : ob) + 8u <= slimit) {  // the unaligned 8 bytes in range
            if (ONE_ROW || ty.w0) load_taps<CC, false, kLoadAux>(srs, oa, tap[q][0][0], tap[q][0][1]);
            if (!ONE_ROW && ty.w1) load_taps<CC, false, kLoadAux>(srs, ob, tap[q][NR - 1][0], tap[q][NR - 1][1]);
        } else {
            // the plane's last pixels: an 8-byte load overhanging the end of
            // the buffer would read as zeros, so take the 2*CC bytes singly
            const unsigned char* r0 = sp + (int64_t)ty.i * rp + (int64_t)tx.i * CC;
#pragma unroll
            for (int e = 0; e < 2 * CC; ++e) {
                tap[q][0][e >> 2] |= (ty.w0 ? (uint32_t)r0[e] : 0u) << (8 * (e & 3));
                if (!ONE_ROW) tap[q][NR - 1][e >> 2] |= (ty.w1 ? (uint32_t)r0[rp + e] : 0u) << (8 * (e & 3));
            }
        }
    }

    ChanNorm cn[CC] = {};
    if (OUT == kOutNorm) {
#pragma unroll
        for (int k = 0; k < CC; ++k) cn[k] = chan_norm(L.norm, img, CC == 1 ? plane % L.norm.c_total : k);
    }

    unsigned char* dp = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                        (int64_t)plane * L.dst.plane_pitch;
    const uint32_t out_row = (uint32_t)W * kOutPx;  // dense bytes of one output row
    const uint32_t rowp = (uint32_t)L.dst.row_pitch;
    const bool dense = L.dst.row_pitch == (int64_t)out_row;
    const bool chunked = (reinterpret_cast<uintptr_t>(dp) & 15) == 0 && (L.dst.row_pitch & 15) == 0 &&
                         (dense || (out_row & 15) == 0);  // 16-byte chunks never straddle rows
    const Rsrc rd = make_rsrc(dp, L.dst.plane_bytes);
    TOut* xrow = reinterpret_cast<TOut*>(xch[threadIdx.y]);
    const unsigned char* xs = xch[threadIdx.y];

#pragma unroll
    for (int g = 0; g < PXL / 4; ++g) {
        // ---- blend 256 pixels into the wave's LDS buffer ---------------------
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int q = g * 4 + j;
            const us2 wx = __builtin_bit_cast(us2, wxp[q]);
            const uint32_t wA = wyp[q] & 0xFFFFu, wB = wyp[q] >> 16;
            TOut* o = xrow + (j * 64 + lane) * CC;
#pragma unroll
            for (int k = 0; k < CC; ++k) {
                // tap pair (byte k, byte CC + k) -> u16 lanes {lo, hi} (v_perm_b32)
                const uint32_t sel = (uint32_t)k | (0x0Cu << 8) | ((uint32_t)(CC + k) << 16) | (0x0Cu << 24);
                const uint32_t top = __builtin_amdgcn_perm(tap[q][0][1], tap[q][0][0], sel);
                const uint32_t bot = ONE_ROW ? 0u : __builtin_amdgcn_perm(tap[q][NR - 1][1], tap[q][NR - 1][0], sel);
                const int v = blend_fixed<MODE>(top, bot, wx, wA, wB);
                if (OUT == kOutSame) o[k] = (TOut)v;
                else if (OUT == kOutF32) o[k] = (TOut)(float)v;
                else o[k] = (TOut)normalize_u8v(cn[k], v);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

        // ---- LDS -> HBM: dense byte b of the plane's output lives at row
        // b / out_row, column byte b % out_row ---------------------------------
        const int gp = npx - g * kGroupPx;  // valid pixels of this round (uniform)
        if (gp > 0) {
            // 32-bit offsets: the plane is < 2^31 bytes (kMaxPlaneBytes)
            const uint32_t vbytes = (uint32_t)(min(gp, kGroupPx) * kOutPx);
            const uint32_t b0 = (uint32_t)(p0 + g * kGroupPx) * kOutPx;  // 16-byte aligned (256 | p0)
            if (chunked) {
                for (uint32_t c = lane; c * 16 < vbytes; c += 64) {
                    const uint32_t b = b0 + 16 * c;
                    uint32_t off = b;
                    if (!dense) {
                        const uint32_t r = b / out_row;
                        off = r * rowp + (b - r * out_row);
                    }
                    if (c * 16 + 16 <= vbytes) {
                        const u32x4 v = *reinterpret_cast<const u32x4*>(xs + 16 * c);
                        __builtin_amdgcn_raw_buffer_store_b128(v, rd.r, (int)(off + rd.delta), 0, kStoreAux);
                    } else {
                        for (uint32_t e = c * 16; e < vbytes; ++e) dp[off + (e - c * 16)] = xs[e];
                    }
                }
            } else {
                for (uint32_t e = lane; e < vbytes; e += 64) {
                    const uint32_t b = b0 + e;
                    const uint32_t r = b / out_row;
                    dp[r * rowp + (b - r * out_row)] = xs[e];
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// ---------------------------------------------------------------------------
// resize_cols_kernel: one-tap-row geometries with COLUMN-stationary lanes.  A
// wave owns a block of 64 output columns x 8 output rows; lane l keeps column
// x0 + l for all 8 rows, so its horizontal tap (index, weights) is computed
// once instead of per pixel, and the rows' vertical taps are computed once
// per wave by lanes 0..7 in parallel and broadcast (readlane).  Per pixel
// what is left is one address add, the gather and the blend.  A gather
// instruction still reads one contiguous run of a source row (64 columns),
// and the 8 x 64 results leave through the wave's LDS buffer as 16-byte
// non-temporal stores, 4 rows at a time.  Same arithmetic as above.
constexpr int kColsRows = 8;  // output rows per wave task at 64 columns (a multiple of 8)
// Column blocks of CW x 64 output columns (lane l keeps columns x0 + l,
// x0 + 64 + l, ...) and kColsRows / CW rows, so a task's pixels stay 512.
// CW = 2 at an exact 3x downscale of 3-channel u8: a block's source span is
// 128 x 9 = 1,152 bytes = 9 whole 128-byte lines, so no line is split
// between two blocks (64-column blocks split every other one: PMC read
// 1.067 x the weighted rows) -- the host picks CW (cols_cw).
template <int CC, int OUT, int MODE, bool ONE_ROW, int CW>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(8)))
resize_cols_kernel(ResizeLaunch L, int col_blocks, int row_groups, int tasks, int xcd_groups) {
    constexpr int NR = ONE_ROW ? 1 : 2;           // gathered source rows per output row
    constexpr int ROWS = kColsRows / CW;          // output rows per task
    using TOut = typename std::conditional<(OUT == kOutSame), uint8_t, float>::type;
    constexpr int kOutPx = CC * (int)sizeof(TOut);
    constexpr int kHalf = 4 / CW;                  // rows per LDS exchange round
    constexpr int kRowB = 64 * CW * kOutPx;        // output bytes of one block row
    constexpr int kLoadAux = OUT == kOutSame ? VACV_LOAD_AUX : (CW == 2 && CC == 3 ? kColsLaux : kDirectLaux);
    constexpr int kStoreAux = OUT == kOutSame ? VACV_STORE_AUX : kDirectSaux;
    __shared__ __attribute__((aligned(16))) unsigned char xch[4][kHalf * kRowB];
    const int lane = (int)threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    // (plane, row group, column block), column block fastest.  xcd_groups > 0:
    // XCD-contiguous order -- workgroup b runs on XCD b % 8, and the 8 XCDs
    // take consecutive runs of xcd_groups workgroups (neighbouring column
    // blocks share the 128-byte source lines at their edges, which then come
    // from one L2)
    const int blk = xcd_groups > 0 ? (int)(blockIdx.x % 8) * xcd_groups + (int)(blockIdx.x / 8) : (int)blockIdx.x;
    const int task = blk * 4 + wave;
    if (task >= tasks) return;                     // whole wave
    const int per_plane = col_blocks * row_groups;
    const int pidx = task / per_plane;
    const int rem = task - pidx * per_plane;
    const int rg = rem / col_blocks, cb = rem - rg * col_blocks;
    const int img = pidx / L.src.planes, plane = pidx - img * L.src.planes;
    const int W = L.dst.w, H = L.dst.h;
    const int x0 = cb * 64 * CW, y0 = rg * ROWS;
    const int ncol = min(64 * CW, W - x0);         // uniform
    const int nrow = min(ROWS, H - y0);            // uniform

    const unsigned char* sp = L.src.base + (int64_t)img * L.src.img_pitch + (int64_t)plane * L.src.plane_pitch;
    const Rsrc srs = make_rsrc(sp, L.src.plane_bytes);
    const uint32_t slimit = (uint32_t)L.src.plane_bytes + srs.delta;
    const uint32_t rp = (uint32_t)L.src.row_pitch;

    // the columns' taps (once), the rows' taps (lanes 0..ROWS-1, then broadcast)
    us2 wx[CW];
    uint32_t xoff[CW];
    // CW = 2: the block's last column loads its 8 bytes from 2 bytes earlier
    // (its 6 tap bytes end where the block's source span does), so no gather
    // reaches into the next block's first line
    constexpr bool kTail = CW == 2 && CC == 3;
    const uint32_t tsh = kTail && lane == 63 ? 2u : 0u;
#pragma unroll
    for (int c = 0; c < CW; ++c) {
        const int xc = 64 * c + lane < ncol ? x0 + 64 * c + lane : W - 1;
        const FixedTap tx = tap_of<MODE>(xc, L.src.w, W, L.scale_xf, L.scale_xd);
        wx[c] = __builtin_bit_cast(us2, (uint32_t)tx.w0 | ((uint32_t)tx.w1 << 16));
        xoff[c] = (uint32_t)(tx.i * CC) + srs.delta - (c == CW - 1 ? tsh : 0u);
    }
    uint32_t my_row = 0, my_w = 0;  // lane r < ROWS: row r's first source row offset, weights (w0 | w1 << 16)
    if (lane < ROWS) {
        FixedTap ty = tap_of<MODE>(min(y0 + lane, H - 1), L.src.h, H, L.scale_yf, L.scale_yd);
        if (ONE_ROW && ty.w0 == 0) { ty.i += 1; ty.w0 = ty.w1; ty.w1 = 0; }  // the weighted row
        my_row = (uint32_t)ty.i * rp;
        my_w = (uint32_t)ty.w0 | ((uint32_t)ty.w1 << 16);
    }
    uint32_t tap[ROWS][CW][NR][2];
    // uniform: can any gather of the task reach past the plane's last byte
    // (only tasks holding the plane's last source row)?  If not, the gathers
    // are issued without a per-lane range check (no exec-mask branch per load)
    const uint32_t last_ro = (uint32_t)__builtin_amdgcn_readlane((int)my_row, nrow - 1) + (uint32_t)(NR - 1) * rp;
    const bool safe = __builtin_amdgcn_ballot_w64(last_ro + xoff[CW - 1] + 8u > slimit) == 0;
    auto gather = [&](auto safe_c) {
        constexpr bool SAFE = decltype(safe_c)::value;
#pragma unroll
        for (int r = 0; r < ROWS; ++r) {
            const uint32_t ro = (uint32_t)__builtin_amdgcn_readlane((int)my_row, r);
            const uint32_t wr = (uint32_t)__builtin_amdgcn_readlane((int)my_w, r);
#pragma unroll
            for (int c = 0; c < CW; ++c) {
#pragma unroll
                for (int n = 0; n < NR; ++n) {
                    const uint32_t o = ro + (uint32_t)n * rp + xoff[c];
                    tap[r][c][n][0] = tap[r][c][n][1] = 0u;
                    // a row of zero weight is not read (its product is 0 either way)
                    if (r < nrow && (n == 0 ? (ONE_ROW || (wr & 0xFFFFu)) : (wr >> 16))) {
                        const uint32_t sh = c == CW - 1 ? tsh : 0u;
                        if (SAFE || o + 8u <= slimit) {
                            // (the shifted load's 2 leading bytes are skipped by the blend's selectors)
                            load_taps<CC, false, kLoadAux>(srs, o, tap[r][c][n][0], tap[r][c][n][1]);
                        } else {  // the plane's last pixels: bytewise (an overhanging load reads zeros)
                            const unsigned char* b = sp + (int64_t)(o - srs.delta);
                            // (positions sh .. sh + 2 CC - 1, as the shifted load has them)
#pragma unroll
                            for (int e = 0; e < 2 * CC + (kTail ? 2 : 0); ++e)
                                if (e >= (int)sh && e < (int)sh + 2 * CC)
                                    tap[r][c][n][e >> 2] |= (uint32_t)b[e] << (8 * (e & 3));
                        }
                    }
                }
            }
        }
    };
    if (safe) gather(std::true_type());
    else gather(std::false_type());
    ChanNorm cn[CC] = {};
    if (OUT == kOutNorm) {
#pragma unroll
        for (int k = 0; k < CC; ++k) cn[k] = chan_norm(L.norm, img, CC == 1 ? plane % L.norm.c_total : k);
    }
    unsigned char* dp = const_cast<unsigned char*>(L.dst.base) + (int64_t)img * L.dst.img_pitch +
                        (int64_t)plane * L.dst.plane_pitch;
    const Rsrc rd = make_rsrc(dp, L.dst.plane_bytes);
    const bool full = ncol == 64 * CW;  // 16-byte chunks (the host checked the alignment)
    TOut* xo = reinterpret_cast<TOut*>(xch[wave]);
    const unsigned char* xs = xch[wave];
#pragma unroll
    for (int g = 0; g < ROWS / kHalf; ++g) {
#pragma unroll
        for (int j = 0; j < kHalf; ++j) {
            const int r = g * kHalf + j;
            const uint32_t wr = (uint32_t)__builtin_amdgcn_readlane((int)my_w, r);
            const uint32_t wA = wr & 0xFFFFu, wB = ONE_ROW ? 0u : wr >> 16;
#pragma unroll
            for (int c = 0; c < CW; ++c) {
#pragma unroll
                for (int k = 0; k < CC; ++k) {
                    // the block's last column (kTail, lane 63) finds its bytes 2 later
                    const uint32_t sel = ((uint32_t)k | (0x0Cu << 8) | ((uint32_t)(CC + k) << 16) | (0x0Cu << 24)) +
                                         (kTail && c == CW - 1 ? tsh * 0x00010001u : 0u);
                    const uint32_t top = __builtin_amdgcn_perm(tap[r][c][0][1], tap[r][c][0][0], sel);
                    const uint32_t bot =
                        ONE_ROW ? 0u : __builtin_amdgcn_perm(tap[r][c][NR - 1][1], tap[r][c][NR - 1][0], sel);
                    const int v = blend_fixed<MODE>(top, bot, wx[c], wA, wB);
                    TOut ov;
                    if (OUT == kOutSame) ov = (TOut)v;
                    else if (OUT == kOutF32) ov = (TOut)(float)v;
                    else ov = (TOut)normalize_u8v(cn[k], v);
                    xo[(j * 64 * CW + 64 * c + lane) * CC + k] = ov;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int rows = min(kHalf, nrow - g * kHalf);  // uniform
        if (rows > 0) {
            const uint32_t base = (uint32_t)(y0 + g * kHalf) * (uint32_t)L.dst.row_pitch + (uint32_t)(x0 * kOutPx) +
                                  rd.delta;
            if (full) {
                constexpr int kCpr = kRowB / 16;  // 16-byte chunks per block row
                for (int c = lane; c < rows * kCpr; c += 64) {
                    const int rr = c / kCpr, cc = c - rr * kCpr;
                    __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(xs + 16 * c), rd.r,
                                                           (int)(base + (uint32_t)rr * (uint32_t)L.dst.row_pitch + 16u * cc),
                                                           0, kStoreAux);
                }
            } else {  // the image's last column block: bytes
                const int rb = ncol * kOutPx;
                for (int e = lane; e < rows * rb; e += 64) {
                    const int rr = e / rb, cc = e - rr * rb;
                    __builtin_amdgcn_raw_buffer_store_b8(xs[rr * kRowB + cc], rd.r,
                                                         (int)(base + (uint32_t)rr * (uint32_t)L.dst.row_pitch + cc), 0,
                                                         kStoreAux);
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// CW for a geometry: 2 where a 128-column block's source span is whole
// 128-byte lines and 64-column blocks' spans are not (the column step times
// 64 x CC is an odd number of 64-byte halves: e.g. 3x of 3 channels, 576 B),
// the output has whole 128-column blocks and the source rows are line-aligned
// (VACV_TUNE_RESIZE_TILE_W = 64 forces 1; 128 forces 2 where the step is an
// integer and the output has whole 128-column blocks).
int cols_cw(const ResizeLaunch& L) {
    const int knob = tune(VACV_TUNE_RESIZE_TILE_W);
    if (knob == 64) return 1;
    const double step = (double)L.src.w / L.dst.w;  // source columns per output column
    // the 128-column blocks need an integer step and whole blocks, forced or not
    if (step != std::floor(step) || L.dst.w % 128) return 1;
    if (knob == 128) return 2;
    const int64_t span64 = (int64_t)step * 64 * L.src.cc * L.src.esize;
    const bool lines = L.src.row_pitch % 128 == 0 && (reinterpret_cast<uintptr_t>(L.src.base) & 127) == 0 &&
                       L.src.img_pitch % 128 == 0 && L.src.plane_pitch % 128 == 0;
    return lines && span64 % 128 != 0 && (2 * span64) % 128 == 0 ? 2 : 1;
}

// The column kernel's grid, or false where it does not apply (it needs
// 16-byte aligned block rows in the destination).
bool cols_plan(const ResizeLaunch& L, int out_px, int cw, int& col_blocks, int& row_groups, int64_t& tasks) {
    const uintptr_t dbits = reinterpret_cast<uintptr_t>(L.dst.base) | (uintptr_t)L.dst.row_pitch |
                            (uintptr_t)L.dst.img_pitch | (uintptr_t)L.dst.plane_pitch;
    if ((dbits & 15) || (64 * out_px) % 16) return false;
    col_blocks = (L.dst.w + 64 * cw - 1) / (64 * cw);
    row_groups = (L.dst.h + kColsRows / cw - 1) / (kColsRows / cw);
    tasks = (int64_t)col_blocks * row_groups * L.n * L.src.planes;
    return tasks < 0x7FFFFFF0LL;
}

template <int CC, int OUT, int MODE, bool ONE_ROW>
hipError_t launch_one(const ResizeLaunch& L, hipStream_t s) {
    {
        constexpr int kOutPx = CC * (OUT == kOutSame ? 1 : 4);
        int col_blocks = 0, row_groups = 0;
        int64_t tasks = 0;
        const int cw = cols_cw(L);
        if (cols_plan(L, kOutPx, cw, col_blocks, row_groups, tasks)) {
            const int64_t groups = (tasks + 3) / 4;
            const int xcd = tune_or(VACV_TUNE_DIRECT_XCD, 0) ? (int)((groups + 7) / 8) : 0;
            const int64_t grid = xcd ? (int64_t)xcd * 8 : groups;
            if (cw == 2)
                hipLaunchKernelGGL((resize_cols_kernel<CC, OUT, MODE, ONE_ROW, 2>), dim3((unsigned)grid), dim3(kBlock), 0,
                                   s, L, col_blocks, row_groups, (int)tasks, xcd);
            else
                hipLaunchKernelGGL((resize_cols_kernel<CC, OUT, MODE, ONE_ROW, 1>), dim3((unsigned)grid), dim3(kBlock), 0,
                                   s, L, col_blocks, row_groups, (int)tasks, xcd);
            return hipGetLastError();
        }
    }
    constexpr int kBlockPx = 4 * 64 * direct_pxl(CC, OUT, ONE_ROW);
    const int64_t P = (int64_t)L.dst.w * L.dst.h;
    const int64_t per_plane = (P + kBlockPx - 1) / kBlockPx;
    const int64_t total = per_plane * L.n * L.src.planes;
    if (P >= 0x7FFFFFFF - kBlockPx || total > 0x7FFFFFF0LL) return hipErrorInvalidValue;
    // XCD-contiguous order only where neighbouring workgroups share source
    // rows (two-tap rows); one-tap rows stream fastest in plain address order
    // (measured 0.222 vs 0.233 ms on the headline; VACV_TUNE_DIRECT_XCD overrides)
    const int xcd = tune_or(VACV_TUNE_DIRECT_XCD, ONE_ROW ? 0 : 1) ? 1 : 0;
    const int64_t blocks = xcd ? (total + 7) / 8 * 8 : total;
    hipLaunchKernelGGL((resize_direct_kernel<CC, OUT, MODE, ONE_ROW>), dim3((unsigned)blocks), dim3(64, 4), 0, s,
                       L, (int)per_plane, (int)total, xcd);
    return hipGetLastError();
}

template <int OUT, int MODE, bool ONE_ROW>
hipError_t launch_cc(const ResizeLaunch& L, hipStream_t s) {
    switch (L.src.cc) {
        case 1: return launch_one<1, OUT, MODE, ONE_ROW>(L, s);
        case 2: return launch_one<2, OUT, MODE, ONE_ROW>(L, s);
        case 3: return launch_one<3, OUT, MODE, ONE_ROW>(L, s);
        case 4: return launch_one<4, OUT, MODE, ONE_ROW>(L, s);
        default: return hipErrorInvalidValue;
    }
}

template <int OUT, bool ONE_ROW>
hipError_t launch_mode(const ResizeLaunch& L, hipStream_t s) {
    switch (L.mode) {
        case VACV_LINEAR_REFERENCE: return launch_cc<OUT, VACV_LINEAR_REFERENCE, ONE_ROW>(L, s);
        case VACV_LINEAR_NEON: return launch_cc<OUT, VACV_LINEAR_NEON, ONE_ROW>(L, s);
        default: return launch_cc<OUT, VACV_LINEAR_OPENCV, ONE_ROW>(L, s);
    }
}

template <int OUT>
hipError_t launch_rows(const ResizeLaunch& L, bool one_row, hipStream_t s) {
    return one_row ? launch_mode<OUT, true>(L, s) : launch_mode<OUT, false>(L, s);
}

}  // namespace

bool resize_one_tap_rows(const ResizeLaunch& L) {
    // no output row has two non-zero vertical weights (the kernel's taps, on
    // the host)
    for (int y = 0; y < L.dst.h; ++y) {
        const FixedTap t = fixed_tap(y, L.src.h, L.dst.h, L.scale_yf, L.scale_yd, L.mode);
        if (t.w0 != 0 && t.w1 != 0) return false;
    }
    return true;
}

hipError_t launch_resize_direct(const ResizeLaunch& L, hipStream_t s) {
    if (L.kind != kLinearFixed) return hipErrorInvalidValue;
    const bool one_row = resize_one_tap_rows(L);
    if (L.out == kOutSame) return launch_rows<kOutSame>(L, one_row, s);
    if (L.out == kOutF32) return launch_rows<kOutF32>(L, one_row, s);
    return launch_rows<kOutNorm>(L, one_row, s);
}

}  // namespace vacv
