// k_yuv_resize.hip -- YUV420sp (NV21 / NV12) -> BGR -> u8 bilinear resize
// -> (u8 | fp32 | normalised fp32), NHWC or NCHW, in one pass over HBM.
//
// This is the camera-frame-to-model-input step: the
// reference's callers run it as three or four separate passes,
//   CvtColor::nv_to_bgr_naive        cvt_color.cpp:39-135 (decode)
//   ResizeNaive::resize_naive_inter_linear_u8  resize_naive.cpp:10-68
//   Tensor::change_dtype + NormalizeNaive::normalize_naive_*
//                                    tensor.cpp:459-502, normalize_naive.cpp:74-90
//   Tensor::change_layout (HWC -> CHW)  tensor.cpp:393-457
// each writing a full-size intermediate.  Here every output pixel decodes
// only the (at most) four source pixels its bilinear taps weight, straight
// from the NV21 planes, so the decoded BGR frame never exists: HBM traffic
// is the weighted Y and chroma rows plus the output.
//
// Exactness.  A tap pixel is decoded with the reference's integer formula
// (chroma_terms, vacv_semantics.hpp) to the same u8 BGR triple
// nv_to_bgr_naive writes, and the blend is the u8 resize's fixed point
// (blend_fixed / tap_of, vacv_device.hpp) on those bytes; the result is
// therefore bit-identical to decode -> resize -> convert -> normalize ->
// change_layout.  Rows with a zero vertical weight are never read (they
// contribute exactly 0 in every mode).
//
// Shape.  Output pixels of an image are numbered row-major; wave v of
// workgroup b owns the 256 pixels from p0 = (4b + v)*256 and lane l samples
// p0 + 64j + l (j < 4), so each gather instruction reads one contiguous run
// of a source row.  Per source row a pixel issues two dword gathers: 4 Y
// bytes at the left tap (2 used) and 4 chroma bytes covering both taps' VU
// pairs (clamped so the read never leaves the row).  When no output row
// weights two source rows (ONE_ROW, checked on the host) only one row is
// gathered; otherwise both rows always are (a zero weight multiplies exactly).
// Results are re-assembled in LDS (plane-major for NCHW) and leave as 16-byte
// non-temporal stores, 1 KiB of contiguous output per store instruction.
#pragma clang fp contract(off)

#include <type_traits>

#include "vacv_device.hpp"

namespace vacv {
namespace {

// Pixels per lane: 8 when one source row is gathered per pixel (twice the
// bytes in flight for the same registers), else 4.
constexpr int yuv_pxl(bool one_row) { return one_row ? 8 : 4; }

// Raw gathers of one weighted source row sy for a pixel whose left tap is
// column tx: 4 Y bytes at tx (2 used) and 4 chroma bytes holding the VU
// pairs of columns tx and tx + 1 (one pair when tx is even), read from an
// even column no later than w - 4 so the dword never leaves the row.
// w >= 4 and even, tx <= w - 2.
struct RowTaps {
    uint32_t y, c;   // raw dwords
};

// Where the two taps' VU pairs sit in RowTaps::c: bits 0-1 = byte index of
// the left tap's pair (0 or 2), bits 2-3 = the right tap's (equal when tx is
// even, the next pair when odd).
__device__ __forceinline__ uint32_t chroma_sel(int w, int tx) {
    const int ca = tx & ~1;
    const uint32_t a = (uint32_t)(ca - min(ca, w - 4));
    return a | ((a + 2u * (uint32_t)(tx & 1)) << 2);
}

// yo / co: byte offsets (from the 16-byte aligned base) of the Y row and of
// its chroma row.  Default cache policy, not non-temporal: a 64-pixel gather
// shares its 128-byte lines with the neighbouring wave's, and the chroma row
// serves two Y rows; in L2 they are fetched once (256 x NV21 1080p ->
// 640x360: u8 0.1447 -> 0.1361 ms, CHW fp32 0.1986 -> 0.1950 ms).
constexpr int kYuvAux = 0;
__device__ __forceinline__ void gather_row(const Rsrc& rs, uint32_t yo, uint32_t co, int w, int tx, RowTaps& t) {
    t.y = __builtin_amdgcn_raw_buffer_load_b32(rs.r, (int)(yo + (uint32_t)tx), 0, kYuvAux);
    const int ca = tx & ~1;
    const int c0 = min(ca, w - 4);
    t.c = __builtin_amdgcn_raw_buffer_load_b32(rs.r, (int)(co + (uint32_t)c0), 0, kYuvAux);
}

struct RowOffs {
    uint32_t y0, c0, y1, c1;  // rows i and i + 1 of a vertical tap
};
__device__ __forceinline__ RowOffs row_offs(int i, uint32_t rp, uint32_t uvbase, uint32_t delta) {
    RowOffs o;
    o.y0 = (uint32_t)i * rp + delta;
    o.y1 = o.y0 + rp;
    o.c0 = uvbase + (uint32_t)(i >> 1) * rp + delta;
    o.c1 = uvbase + (uint32_t)((i + 1) >> 1) * rp + delta;
    return o;
}

typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ s16x2 clamp_u8x2(s16x2 v) {
    return __builtin_elementwise_max(__builtin_elementwise_min(v, (s16x2)(short)255), (s16x2)(short)0);
}

// Decode two pixels, cvt_color.cpp:66-88, on packed 16-bit pairs (Y, V, U
// as u16 lanes): every intermediate of the reference's int arithmetic fits in
// int16 (|179(v-128)|, |44(u-128) + 91(v-128)|, |227(u-128)| < 2^15, Y + term
// in [-227, 481]), >> is arithmetic as in the reference, so each lane is
// exact.  Out: B, G, R as u16 pairs.
__device__ __forceinline__ void decode_yuv(s16x2 Y, s16x2 V, s16x2 U, uint32_t& bp, uint32_t& gp, uint32_t& rp) {
    const s16x2 vm = V - (short)128, um = U - (short)128;
    const s16x2 ra = (vm * (short)179) >> (short)7;
    const s16x2 ga = (um * (short)44 + vm * (short)91) >> (short)7;
    const s16x2 ba = (um * (short)227) >> (short)7;
    bp = __builtin_bit_cast(uint32_t, clamp_u8x2(Y + ba));
    gp = __builtin_bit_cast(uint32_t, clamp_u8x2(Y - ga));
    rp = __builtin_bit_cast(uint32_t, clamp_u8x2(Y + ra));
}

// A row's two tap pixels {left, right} decoded -- the layout the blend's
// v_dot2_u32_u16 takes.
__device__ __forceinline__ void decode_row(const RowTaps& t, uint32_t cs, int v_first, uint32_t& bp, uint32_t& gp,
                                           uint32_t& rp, uint32_t ysel = 0x0C010C00u) {
    // v_perm selectors: byte (a + vi) -> lane 0, byte (b + vi) -> lane 1, 0x0C = 0
    const uint32_t base = (cs & 3u) | ((cs >> 2) << 16) | 0x0C000C00u;
    const uint32_t vo = v_first ? 0u : 0x00010001u;  // NV21: V first in a pair
    const s16x2 V = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(0u, t.c, base + vo));
    const s16x2 U = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(0u, t.c, base + (0x00010001u - vo)));
    const s16x2 Y = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(0u, t.y, ysel));  // Y bytes -> u16 lanes
    decode_yuv(Y, V, U, bp, gp, rp);
}

// Output pixels per wave and per LDS exchange round (4 per lane).
constexpr int kGroupPx = 256;

// Waves per SIMD the register budget is set for: the normalised one-row
// kernel needs ~70 VGPRs at 8 pixels per lane (64 would spill).
constexpr int yuv_waves(int out, bool one_row) { return (one_row && out == kOutNorm) ? 6 : 8; }

template <int OUT, int MODE, bool CHW, bool ONE_ROW>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(yuv_waves(OUT, ONE_ROW))))
yuv_resize_kernel(YuvResizeLaunch L) {
    using TOut = typename std::conditional<(OUT == kOutSame), uint8_t, float>::type;
    constexpr int kES = (int)sizeof(TOut);
    constexpr int NR = ONE_ROW ? 1 : 2;
    constexpr int PXL = yuv_pxl(ONE_ROW);
    constexpr int kWavePx = 64 * PXL;
    constexpr int kSpan = kGroupPx * kES * (CHW ? 1 : 3);  // bytes one round writes per plane
    __shared__ __attribute__((aligned(16))) unsigned char xch[4][3 * kGroupPx * kES];

    const int img = blockIdx.y;
    const int P = L.wo * L.ho;
    const int p0 = ((int)blockIdx.x * 4 + (int)threadIdx.y) * kWavePx;
    if (p0 >= P) return;  // whole wave
    const int npx = min(kWavePx, P - p0);
    const int lane = threadIdx.x;

    const unsigned char* sp = L.src + (int64_t)img * L.src_img;
    const Rsrc rs = make_rsrc(sp, L.src_bytes);
    const uint32_t rp = (uint32_t)L.src_row;
    const uint32_t uvbase = (uint32_t)L.h * rp;

    // ---- gathers: lane l takes pixels p0 + 64j + l, so one gather
    // instruction reads a contiguous run of a source row; every load is
    // issued before any decode ------------------------------------------------
    RowTaps t[PXL][NR];
    // wyp = {wA, wB} as u16; ONE_ROW keeps chroma_sel in the (zero) wB half
    uint32_t wxp[PXL], wyp[PXL], csel[ONE_ROW ? 1 : PXL];
    // vertical taps: when the output is at least a wave's pixels wide a wave
    // touches at most two output rows, whose taps are computed once
    const int W = L.wo;
    const int y_first = p0 / W;  // wave-uniform
    const int x_first = p0 - y_first * W;
    const bool wide = W >= kWavePx;
    FixedTap ty0 = tap_of<MODE>(y_first, L.h, L.ho, L.scale_yf, L.scale_yd);
    FixedTap ty1 = tap_of<MODE>(min(y_first + 1, L.ho - 1), L.h, L.ho, L.scale_yf, L.scale_yd);
    if (ONE_ROW && ty0.w0 == 0) { ty0.i += 1; ty0.w0 = ty0.w1; ty0.w1 = 0; }  // the weighted row as row A
    if (ONE_ROW && ty1.w0 == 0) { ty1.i += 1; ty1.w0 = ty1.w1; ty1.w1 = 0; }
    // wave-uniform; readfirstlane keeps them scalar (otherwise LLVM folds
    // the per-pixel select of two products into a per-pixel multiply)
    RowOffs ro0 = row_offs(ty0.i, rp, uvbase, rs.delta);
    RowOffs ro1 = row_offs(ty1.i, rp, uvbase, rs.delta);
    ro0.y0 = __builtin_amdgcn_readfirstlane(ro0.y0);
    ro0.c0 = __builtin_amdgcn_readfirstlane(ro0.c0);
    ro0.y1 = __builtin_amdgcn_readfirstlane(ro0.y1);
    ro0.c1 = __builtin_amdgcn_readfirstlane(ro0.c1);
    ro1.y0 = __builtin_amdgcn_readfirstlane(ro1.y0);
    ro1.c0 = __builtin_amdgcn_readfirstlane(ro1.c0);
    ro1.y1 = __builtin_amdgcn_readfirstlane(ro1.y1);
    ro1.c1 = __builtin_amdgcn_readfirstlane(ro1.c1);
#pragma unroll
    for (int j = 0; j < PXL; ++j) {
#pragma unroll
        for (int r = 0; r < NR; ++r) t[j][r].y = t[j][r].c = 0u;
        wxp[j] = wyp[j] = 0u;
        if (!ONE_ROW) csel[j] = 0u;
        if (j * 64 + lane >= npx) continue;
        const int d = x_first + j * 64 + lane;  // < W + kWavePx
        const int dy = wide ? (d >= W ? 1 : 0) : d / W;
        const int x = wide ? (dy ? d - W : d) : d - dy * W;
        const FixedTap tx = tap_of<MODE>(x, L.w, W, L.scale_xf, L.scale_xd);
        FixedTap ty;
        RowOffs ro;
        if (wide) {
            ty.i = dy ? ty1.i : ty0.i;
            ty.w0 = dy ? ty1.w0 : ty0.w0;
            ty.w1 = dy ? ty1.w1 : ty0.w1;
            ro.y0 = dy ? ro1.y0 : ro0.y0;
            ro.c0 = dy ? ro1.c0 : ro0.c0;
            ro.y1 = dy ? ro1.y1 : ro0.y1;
            ro.c1 = dy ? ro1.c1 : ro0.c1;
        } else {
            ty = tap_of<MODE>(y_first + dy, L.h, L.ho, L.scale_yf, L.scale_yd);
            if (ONE_ROW && ty.w0 == 0) { ty.i += 1; ty.w0 = ty.w1; ty.w1 = 0; }
            ro = row_offs(ty.i, rp, uvbase, rs.delta);
        }
        wxp[j] = (uint32_t)tx.w0 | ((uint32_t)tx.w1 << 16);
        const uint32_t cs = chroma_sel(L.w, tx.i);
        wyp[j] = (uint32_t)ty.w0 | ((ONE_ROW ? cs : (uint32_t)ty.w1) << 16);
        if (!ONE_ROW) csel[j] = cs;
        // both rows of a two-row pixel are always read (rows i, i + 1 exist);
        // a zero weight multiplies them out exactly
        gather_row(rs, ro.y0, ro.c0, L.w, tx.i, t[j][0]);
        if (!ONE_ROW) gather_row(rs, ro.y1, ro.c1, L.w, tx.i, t[j][NR - 1]);
    }

    ChanNorm cn[3] = {};
    if (OUT == kOutNorm) {
#pragma unroll
        for (int k = 0; k < 3; ++k) cn[k] = chan_norm(L.norm, img, k);
    }

    unsigned char* dimg = L.dst + (int64_t)img * L.dst_img;
    const uint32_t out_row = (uint32_t)L.wo * kES * (CHW ? 1 : 3);  // dense bytes of one output row
    const uint32_t rowp = (uint32_t)L.dst_row;
    const bool dense = L.dst_row == (int64_t)out_row;
    TOut* xo = reinterpret_cast<TOut*>(xch[threadIdx.y]);

#pragma unroll
    for (int g = 0; g < PXL / 4; ++g) {
        // ---- decode + blend 256 pixels into the wave's LDS buffer:
        // plane-major for NCHW ([k][256]), pixel-major for NHWC ([256][3]) ---
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int j = g * 4 + jj;
            uint32_t pa[3], pb[3] = {0u, 0u, 0u};  // rows A/B: B, G, R as u16 pairs {left, right}
            const uint32_t cs = ONE_ROW ? wyp[j] >> 16 : csel[j];
            decode_row(t[j][0], cs, L.v_first, pa[0], pa[1], pa[2]);
            if (!ONE_ROW) decode_row(t[j][NR - 1], cs, L.v_first, pb[0], pb[1], pb[2]);
            if (L.rgb) {  // output order R, G, B
                const uint32_t x0 = pa[0], x1 = pb[0];
                pa[0] = pa[2]; pa[2] = x0;
                pb[0] = pb[2]; pb[2] = x1;
            }
            const us2 wx = __builtin_bit_cast(us2, wxp[j]);
            const uint32_t wA = wyp[j] & 0xFFFFu, wB = ONE_ROW ? 0u : wyp[j] >> 16;
            const int q = jj * 64 + lane;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const uint32_t top = pa[k], bot = pb[k];
                const int v = blend_fixed<MODE>(top, bot, wx, wA, wB);
                TOut ov;
                if (OUT == kOutSame) ov = (TOut)v;
                else if (OUT == kOutF32) ov = (TOut)(float)v;
                else ov = (TOut)normalize_u8v(cn[k], v);
                xo[CHW ? k * kGroupPx + q : q * 3 + k] = ov;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

        // ---- LDS -> HBM: dense byte b of a plane's output lives at row
        // b / out_row, column byte b % out_row --------------------------------
        const int gp = npx - g * kGroupPx;  // valid pixels of this round (uniform)
        if (gp > 0) {
            const uint32_t vbytes = (uint32_t)min(gp, kGroupPx) * kES * (CHW ? 1 : 3);
            const uint32_t b0 = (uint32_t)(p0 + g * kGroupPx) * kES * (CHW ? 1 : 3);
#pragma unroll
            for (int k = 0; k < (CHW ? 3 : 1); ++k) {
                unsigned char* dp = dimg + (int64_t)k * L.dst_plane;
                const unsigned char* xs = xch[threadIdx.y] + k * kSpan;
                const bool chunked = (reinterpret_cast<uintptr_t>(dp) & 15) == 0 && (L.dst_row & 15) == 0 &&
                                     (dense || (out_row & 15) == 0);  // 16-byte chunks never straddle rows
                if (chunked) {
                    for (uint32_t c = lane; c * 16 < vbytes; c += 64) {
                        const uint32_t b = b0 + 16 * c;
                        uint32_t off = b;
                        if (!dense) {
                            const uint32_t r = b / out_row;
                            off = r * rowp + (b - r * out_row);
                        }
                        if (c * 16 + 16 <= vbytes) {
                            __builtin_nontemporal_store(*reinterpret_cast<const u32x4*>(xs + 16 * c),
                                                        reinterpret_cast<u32x4*>(dp + off));
                        } else {
                            for (uint32_t e = c * 16; e < vbytes; ++e) dp[off + (e - c * 16)] = xs[e];
                        }
                    }
                } else {
                    for (uint32_t e = lane; e < vbytes; e += 64) {
                        const uint32_t b = b0 + e;
                        const uint32_t r = b / out_row;
                        dp[(int64_t)r * rowp + (b - r * out_row)] = xs[e];
                    }
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// ---------------------------------------------------------------------------
// yuv_cols_kernel (round 5): the same arithmetic with COLUMN-stationary lanes,
// the shape that lifted the u8 resize (resize_cols_kernel, k_resize_direct.hip).
// A wave owns 64 output columns x kYuvRows output rows of one image; lane l
// keeps column x0 + l for all of them, so its horizontal tap (index, weights)
// and chroma byte selector are computed once, not per pixel (yuv_resize_kernel
// numbered pixels row-major and recomputed tap_of, chroma_sel and the row
// select for every one); the rows' vertical taps and source-row offsets are
// computed by lanes 0..kYuvRows-1 in parallel and broadcast as scalars
// (readlane).  Per pixel and weighted row what is left: two dword gathers
// (one contiguous run of a source row per instruction), the packed decode
// and the blend.  Results leave through the wave's LDS buffer, kYuvHalf rows
// at a time, as 16-byte non-temporal stores (plane-major for NCHW).
//
// CW = 2 (round 6): blocks of 128 output columns x kYuvRows / 2 rows (lane l
// keeps columns x0 + l and x0 + 64 + l), chosen where a 128-column block's
// Y and chroma spans are whole 128-byte lines and a 64-column block's are not
// (an odd integer step, e.g. 1080p -> 640x360: 384 bytes = 3 lines per row):
// no line is then split between two blocks, which neighbouring workgroups on
// other XCDs would both fetch from HBM (the headline kernel's CW = 2, k_resize_direct.hip).
//
// POINT (round 6): every output row and column weights one source row and
// column, with 2048 (an odd integer downscale: 1080p -> 640x360 taps rows and
// columns 3d + 1).  The blend then returns the tapped pixel in every mode
// (reference (p*2048*2048) >> 22 = p; NEON / OpenCV ((4p) + 2) >> 2 = p), so
// the output pixel IS the decoded source pixel: one Y byte and one VU pair
// are gathered per output pixel, a lane's pixels are decoded two at a time
// (the packed decode's lanes = two output pixels, not two taps), no blend.
constexpr int kYuvRows = 8;   // output rows per wave task (at CW = 1)
constexpr int kYuvHalf = 4;   // rows per LDS exchange round (at CW = 1)
template <int OUT, int MODE, bool CHW, bool ONE_ROW, int CW, bool POINT = false>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(yuv_waves(OUT, ONE_ROW))))
yuv_cols_kernel(YuvResizeLaunch L, int col_blocks, int row_groups) {
    static_assert(!POINT || ONE_ROW, "POINT gathers one row");
    using TOut = typename std::conditional<(OUT == kOutSame), uint8_t, float>::type;
    constexpr int kES = (int)sizeof(TOut);
    constexpr int NR = ONE_ROW ? 1 : 2;
    constexpr int ROWS = kYuvRows / CW;                       // output rows per task
    constexpr int HALF = kYuvHalf / CW;                       // rows per exchange round
    constexpr int kRowB = 64 * CW * kES * (CHW ? 1 : 3);      // bytes of one block row (per plane)
    constexpr int kPlaneB = HALF * kRowB;                     // one round's bytes per plane
    __shared__ __attribute__((aligned(16))) unsigned char xch[4][3 * kYuvHalf * 64 * kES];
    const int lane = (int)threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
    const int task = (int)blockIdx.x * 4 + wave;              // (row group, column block), column block fastest
    if (task >= col_blocks * row_groups) return;              // whole wave
    const int img = blockIdx.y;
    const int rg = task / col_blocks, cb = task - rg * col_blocks;
    const int W = L.wo, H = L.ho;
    const int x0 = cb * 64 * CW, y0 = rg * ROWS;
    const int ncol = min(64 * CW, W - x0), nrow = min(ROWS, H - y0);  // uniform

    const unsigned char* sp = L.src + (int64_t)img * L.src_img;
    const Rsrc rs = make_rsrc(sp, L.src_bytes);
    const uint32_t rp = (uint32_t)L.src_row;
    const uint32_t uvbase = (uint32_t)L.h * rp;

    // the columns' taps and chroma selectors (once).  The block's last column
    // (lane 63 of its last 64) reads its Y dword (and, at an even tap, its
    // chroma dword) from 2 bytes earlier, its bytes picked by the selectors:
    // so no gather reaches into the next block's first 128-byte line, which
    // neighbouring workgroups -- on other XCDs -- would otherwise both fetch
    // from HBM (PMC: reads 413 -> 372 MB at 256 x NV21 1080p -> 640x360, B_alg 354 MB).
    us2 wx[CW];
    uint32_t cs[CW], ycol[CW], ysel[CW], ccol[CW];
#pragma unroll
    for (int c = 0; c < CW; ++c) {
        const int x = 64 * c + lane < ncol ? x0 + 64 * c + lane : W - 1;
        const FixedTap tx = tap_of<MODE>(x, L.w, W, L.scale_xf, L.scale_xd);
        wx[c] = __builtin_bit_cast(us2, (uint32_t)tx.w0 | ((uint32_t)tx.w1 << 16));
        if constexpr (POINT) {
            // the weighted column and its VU pair (no neighbour is read)
            const int xi = tx.w0 == 0 ? tx.i + 1 : tx.i;
            ycol[c] = (uint32_t)xi;
            ccol[c] = (uint32_t)(xi & ~1);
            continue;
        }
        const bool edge = c == CW - 1 && lane == 63 && tx.i >= 2;
        const int ca = tx.i & ~1, c0 = min(ca, L.w - 4);
        const int c1 = edge && (tx.i & 1) == 0 && c0 == ca ? c0 - 2 : c0;
        const uint32_t ca_rel = (uint32_t)(ca - c1);
        cs[c] = ca_rel | ((ca_rel + 2u * (uint32_t)(tx.i & 1)) << 2);
        ycol[c] = (uint32_t)(edge ? tx.i - 2 : tx.i);
        ysel[c] = edge ? 0x0C030C02u : 0x0C010C00u;
        ccol[c] = (uint32_t)c1;
    }
    // lane r < ROWS: row r's tap -- source Y / chroma row offsets (rows i
    // and i + 1) and weights wA | wB << 16
    uint32_t my_y0 = 0, my_c0 = 0, my_y1 = 0, my_c1 = 0, my_w = 0;
    if (lane < ROWS) {
        FixedTap ty = tap_of<MODE>(min(y0 + lane, H - 1), L.h, H, L.scale_yf, L.scale_yd);
        if (ONE_ROW && ty.w0 == 0) { ty.i += 1; ty.w0 = ty.w1; ty.w1 = 0; }  // the weighted row as row A
        const RowOffs ro = row_offs(ty.i, rp, uvbase, rs.delta);
        my_y0 = ro.y0; my_c0 = ro.c0; my_y1 = ro.y1; my_c1 = ro.c1;
        my_w = (uint32_t)ty.w0 | ((uint32_t)ty.w1 << 16);
    }
    // every gather of the task, issued before any decode
    RowTaps t[ROWS][CW][NR];
#pragma unroll
    for (int r = 0; r < ROWS; ++r) {
        const uint32_t ya = (uint32_t)__builtin_amdgcn_readlane((int)my_y0, r);
        const uint32_t ca = (uint32_t)__builtin_amdgcn_readlane((int)my_c0, r);
        const uint32_t yb = ONE_ROW ? 0u : (uint32_t)__builtin_amdgcn_readlane((int)my_y1, r);
        const uint32_t cb2 = ONE_ROW ? 0u : (uint32_t)__builtin_amdgcn_readlane((int)my_c1, r);
#pragma unroll
        for (int c = 0; c < CW; ++c) {
            if constexpr (POINT) {
                t[r][c][0].y = __builtin_amdgcn_raw_buffer_load_b8(rs.r, (int)(ya + ycol[c]), 0, kYuvAux);
                t[r][c][0].c = __builtin_amdgcn_raw_buffer_load_b16(rs.r, (int)(ca + ccol[c]), 0, kYuvAux);
                continue;
            }
            t[r][c][0].y = __builtin_amdgcn_raw_buffer_load_b32(rs.r, (int)(ya + ycol[c]), 0, kYuvAux);
            t[r][c][0].c = __builtin_amdgcn_raw_buffer_load_b32(rs.r, (int)(ca + ccol[c]), 0, kYuvAux);
            if constexpr (!ONE_ROW) {
                t[r][c][1].y = __builtin_amdgcn_raw_buffer_load_b32(rs.r, (int)(yb + ycol[c]), 0, kYuvAux);
                t[r][c][1].c = __builtin_amdgcn_raw_buffer_load_b32(rs.r, (int)(cb2 + ccol[c]), 0, kYuvAux);
            }
        }
    }
    ChanNorm cn[3] = {};
    if (OUT == kOutNorm) {
#pragma unroll
        for (int k = 0; k < 3; ++k) cn[k] = chan_norm(L.norm, img, k);
    }
    unsigned char* dimg = L.dst + (int64_t)img * L.dst_img;
    const Rsrc rd = make_rsrc(dimg, CHW ? L.dst_plane * 3 : L.dst_img);
    // 16-byte chunks wherever the block row's bytes are whole chunks (the
    // host checked the alignment): every block but a partial last one whose
    // width is not (e.g. 224 = 3.5 blocks: 32 fp32 columns are 8 chunks)
    const int rbytes = ncol * kES * (CHW ? 1 : 3);
    const bool chunks = (rbytes & 15) == 0;  // uniform
    const int cpr = rbytes >> 4;
    TOut* xo = reinterpret_cast<TOut*>(xch[wave]);
    const unsigned char* xs = xch[wave];
#pragma unroll
    for (int g = 0; g < ROWS / HALF; ++g) {
#pragma unroll
        for (int j = 0; j < HALF; ++j) {
            const int r = g * HALF + j;
            if constexpr (POINT) {
                // pixels A, B of the pair: the lane's two columns of row r
                // (CW = 2) or its column in rows r and r + 1
                if (CW == 1 && (j & 1)) continue;
                const RowTaps& ta = t[r][0][0];
                const RowTaps& tb = CW == 2 ? t[r][CW - 1][0] : t[min(r + 1, ROWS - 1)][0][0];
                const uint32_t vsel = L.v_first ? 0x0C040C00u : 0x0C050C01u;
                const s16x2 Y = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(tb.y, ta.y, 0x0C040C00u));
                const s16x2 V = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(tb.c, ta.c, vsel));
                const s16x2 U = __builtin_bit_cast(s16x2, __builtin_amdgcn_perm(tb.c, ta.c, vsel ^ 0x00010001u));
                uint32_t q[3];
                decode_yuv(Y, V, U, q[0], q[1], q[2]);
                if (L.rgb) {  // output order R, G, B
                    const uint32_t q0 = q[0];
                    q[0] = q[2];
                    q[2] = q0;
                }
#pragma unroll
                for (int e = 0; e < 2; ++e) {
                    const int jj = CW == 2 ? j : j + e, cc = CW == 2 ? e : 0;
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        const int v = (int)((q[k] >> (16 * e)) & 0xFFu);
                        TOut ov;
                        if (OUT == kOutSame) ov = (TOut)v;
                        else if (OUT == kOutF32) ov = (TOut)(float)v;
                        else ov = (TOut)normalize_u8v(cn[k], v);
                        const int px = jj * 64 * CW + 64 * cc + lane;
                        xo[CHW ? k * (HALF * 64 * CW) + px : px * 3 + k] = ov;
                    }
                }
                continue;
            }
            const uint32_t wr = (uint32_t)__builtin_amdgcn_readlane((int)my_w, r);
            const uint32_t wA = wr & 0xFFFFu, wB = ONE_ROW ? 0u : wr >> 16;
#pragma unroll
            for (int c = 0; c < CW; ++c) {
                uint32_t pa[3], pb[3] = {0u, 0u, 0u};  // rows A/B: B, G, R as u16 pairs {left, right}
                decode_row(t[r][c][0], cs[c], L.v_first, pa[0], pa[1], pa[2], ysel[c]);
                if (!ONE_ROW) decode_row(t[r][c][NR - 1], cs[c], L.v_first, pb[0], pb[1], pb[2], ysel[c]);
                if (L.rgb) {  // output order R, G, B
                    const uint32_t q0 = pa[0], q1 = pb[0];
                    pa[0] = pa[2]; pa[2] = q0;
                    pb[0] = pb[2]; pb[2] = q1;
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const int v = blend_fixed<MODE>(pa[k], pb[k], wx[c], wA, wB);
                    TOut ov;
                    if (OUT == kOutSame) ov = (TOut)v;
                    else if (OUT == kOutF32) ov = (TOut)(float)v;
                    else ov = (TOut)normalize_u8v(cn[k], v);
                    const int px = j * 64 * CW + 64 * c + lane;  // pixel in the round
                    xo[CHW ? k * (HALF * 64 * CW) + px : px * 3 + k] = ov;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int rows = min(HALF, nrow - g * HALF);  // uniform
        if (rows > 0) {
            const uint32_t base = (uint32_t)(y0 + g * HALF) * (uint32_t)L.dst_row +
                                  (uint32_t)(x0 * kES * (CHW ? 1 : 3)) + rd.delta;
#pragma unroll
            for (int k = 0; k < (CHW ? 3 : 1); ++k) {
                const uint32_t pbase = base + (uint32_t)(k * L.dst_plane);
                const unsigned char* xk = xs + k * kPlaneB;
                if (chunks) {
                    for (int c = lane; c < rows * cpr; c += 64) {
                        const int rr = c / cpr, cc = c - rr * cpr;
                        __builtin_amdgcn_raw_buffer_store_b128(*reinterpret_cast<const u32x4*>(xk + rr * kRowB + 16 * cc),
                                                               rd.r,
                                                               (int)(pbase + (uint32_t)rr * (uint32_t)L.dst_row + 16u * cc),
                                                               0, VACV_STORE_AUX);
                    }
                } else {  // a partial last column block of odd bytes: bytes
                    const int rb = rbytes;
                    for (int e = lane; e < rows * rb; e += 64) {
                        const int rr = e / rb, cc = e - rr * rb;
                        __builtin_amdgcn_raw_buffer_store_b8(xk[rr * kRowB + cc], rd.r,
                                                             (int)(pbase + (uint32_t)rr * (uint32_t)L.dst_row + cc), 0,
                                                             VACV_STORE_AUX);
                    }
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// CW for a geometry (see yuv_cols_kernel): 2 where the column step is an odd
// integer, the output has whole 128-column blocks and the source rows are
// line-aligned (VACV_TUNE_RESIZE_TILE_W = 64 forces 1)
int yuv_cols_cw(const YuvResizeLaunch& L) {
    if (tune(VACV_TUNE_RESIZE_TILE_W) == 64) return 1;
    if (L.w % L.wo || L.wo % 128) return 1;
    const int step = L.w / L.wo;
    const bool lines = L.src_row % 128 == 0 && (reinterpret_cast<uintptr_t>(L.src) & 127) == 0 && L.src_img % 128 == 0;
    return lines && (step & 1) ? 2 : 1;
}

template <int OUT, int MODE, bool CHW, bool ONE_ROW, int CW, bool POINT = false>
hipError_t launch_cols_cw(const YuvResizeLaunch& L, hipStream_t s) {
    const int col_blocks = (L.wo + 64 * CW - 1) / (64 * CW), row_groups = (L.ho + kYuvRows / CW - 1) / (kYuvRows / CW);
    const dim3 grid((unsigned)((col_blocks * row_groups + 3) / 4), (unsigned)L.n);
    hipLaunchKernelGGL((yuv_cols_kernel<OUT, MODE, CHW, ONE_ROW, CW, POINT>), grid, dim3(kBlock), 0, s, L, col_blocks,
                       row_groups);
    return hipGetLastError();
}

// taps: 0 two rows, 1 one row (ONE_ROW), 2 one row and one column (POINT)
template <int OUT, int MODE, bool CHW>
hipError_t launch_cols_t(const YuvResizeLaunch& L, int taps, hipStream_t s) {
    if (yuv_cols_cw(L) == 2) {
        if (taps == 2) return launch_cols_cw<OUT, MODE, CHW, true, 2, true>(L, s);
        return taps ? launch_cols_cw<OUT, MODE, CHW, true, 2>(L, s) : launch_cols_cw<OUT, MODE, CHW, false, 2>(L, s);
    }
    if (taps == 2) return launch_cols_cw<OUT, MODE, CHW, true, 1, true>(L, s);
    return taps ? launch_cols_cw<OUT, MODE, CHW, true, 1>(L, s) : launch_cols_cw<OUT, MODE, CHW, false, 1>(L, s);
}

template <int OUT, int MODE, bool CHW>
hipError_t launch_rows_t(const YuvResizeLaunch& L, bool one_row, dim3 grid, hipStream_t s) {
    if (one_row) hipLaunchKernelGGL((yuv_resize_kernel<OUT, MODE, CHW, true>), grid, dim3(64, 4), 0, s, L);
    else hipLaunchKernelGGL((yuv_resize_kernel<OUT, MODE, CHW, false>), grid, dim3(64, 4), 0, s, L);
    return hipGetLastError();
}

template <int OUT, int MODE>
hipError_t launch_layout_t(const YuvResizeLaunch& L, int taps, dim3 grid, hipStream_t s) {
    const bool one_row = taps > 0;
    // the column kernel needs 16-byte aligned block rows (and plane and image
    // pitches) in the destination; VACV_TUNE_RESIZE_DIRECT = 2 forces the
    // row-major kernel (A/B)
    constexpr int kES = OUT == kOutSame ? 1 : 4;
    const int64_t rowb = 64 * kES * (L.chw ? 1 : 3);
    const uintptr_t bits = reinterpret_cast<uintptr_t>(L.dst) | (uintptr_t)L.dst_row | (uintptr_t)L.dst_img |
                           (uintptr_t)(L.chw ? L.dst_plane : 0);
    const int64_t span = L.chw ? L.dst_plane * 3 : L.dst_img;
    if (!(bits & 15) && rowb % 16 == 0 && tune(VACV_TUNE_RESIZE_DIRECT) != 2 && span < kMaxPlaneBytes &&
        (int64_t)L.wo * L.ho < 0x7FFFFFF0LL / 4)
        return L.chw ? launch_cols_t<OUT, MODE, true>(L, taps, s) : launch_cols_t<OUT, MODE, false>(L, taps, s);
    return L.chw ? launch_rows_t<OUT, MODE, true>(L, one_row, grid, s)
                 : launch_rows_t<OUT, MODE, false>(L, one_row, grid, s);
}

template <int OUT>
hipError_t launch_mode_t(const YuvResizeLaunch& L, int taps, dim3 grid, hipStream_t s) {
    switch (L.mode) {
        case VACV_LINEAR_REFERENCE: return launch_layout_t<OUT, VACV_LINEAR_REFERENCE>(L, taps, grid, s);
        case VACV_LINEAR_NEON: return launch_layout_t<OUT, VACV_LINEAR_NEON>(L, taps, grid, s);
        default: return launch_layout_t<OUT, VACV_LINEAR_OPENCV>(L, taps, grid, s);
    }
}

// every tap of the axis weights one source index, with 2048 (then the blend
// returns that pixel, see yuv_cols_kernel's POINT)
bool point_axis(int n_in, int n_out, float scale_f, double scale_d, int mode) {
    for (int d = 0; d < n_out; ++d) {
        const FixedTap t = fixed_tap(d, n_in, n_out, scale_f, scale_d, mode);
        if (!((t.w0 == 2048 && t.w1 == 0) || (t.w0 == 0 && t.w1 == 2048))) return false;
    }
    return true;
}

}  // namespace

hipError_t launch_yuv_resize(const YuvResizeLaunch& L, hipStream_t s) {
    // the host (vacv_abi.cpp) has checked: w, h even, w >= 4, h >= 2, the
    // image's bytes fit one buffer resource, wo*ho < 2^31 - 2048, n <= 65535
    const int64_t P = (int64_t)L.wo * L.ho;
    // no output row weights two source rows (e.g. an integer downscale >= 2):
    // gather one row per pixel (the taps are the u8 resize's, resize_one_tap_rows)
    bool one_row = true;
    for (int y = 0; y < L.ho && one_row; ++y) {
        const FixedTap t = fixed_tap(y, L.h, L.ho, L.scale_yf, L.scale_yd, L.mode);
        one_row = !(t.w0 != 0 && t.w1 != 0);
    }
    const int64_t block_px = 4 * 64 * yuv_pxl(one_row);
    const dim3 grid((unsigned)((P + block_px - 1) / block_px), (unsigned)L.n);
    const int taps = !one_row                                                       ? 0
                     : tune(VACV_TUNE_RESIZE_DIRECT) != 3 &&
                               point_axis(L.h, L.ho, L.scale_yf, L.scale_yd, L.mode) &&
                               point_axis(L.w, L.wo, L.scale_xf, L.scale_xd, L.mode)
                         ? 2
                         : 1;
    if (L.out == kOutSame) return launch_mode_t<kOutSame>(L, taps, grid, s);
    if (L.out == kOutF32) return launch_mode_t<kOutF32>(L, taps, grid, s);
    return launch_mode_t<kOutNorm>(L, taps, grid, s);
}

}  // namespace vacv
